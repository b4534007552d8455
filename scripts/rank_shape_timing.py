"""Per-stage time of ONE rank's share of the bench step at S ranks, on one GPU
(no communication): what the N-GPU bench line should approach per step, minus
the all-gather / all-reduce time.

    python scripts/rank_shape_timing.py [--shards 1,2,4,8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="an A/B build of the library (make ab)")
    ap.add_argument("--rest", default="0",
                    help="pairs: comma list of PhiEngine.REST_BESIDE settings (1, 0)")
    ap.add_argument("--side", default="0",
                    help="pairs: comma list of PhiEngine.WINDOW_SIDE_STREAM settings (0, 1)")
    ap.add_argument("--fwdz", default="0",
                    help="pairs: comma list of PhiEngine.FWD_ZSPLIT settings (0 = chosen, 1 = none)")
    ap.add_argument("--set", action="append", default=[],
                    help="pairs: NAME=v1,v2 sweeps a PhiEngine split override "
                         "(W_SPLITS, H_SPLITS, REST_SPLITS; 0 = chosen)")
    ap.add_argument("--square", default=None,
                    help="pairs: comma list of PairSplitPlan.FULL_SQUARE settings (0, 1)")
    ap.add_argument("--mode", default="timer",
                    help="comma list: timer (stage events), plain (no events), graph (the step "
                         "captured as one HIP graph and replayed: the launch gaps' bound)")
    ap.add_argument("--xmap", default="1",
                    help="comma list of dsvgd_phi_set_xmap settings (slices mapped to XCDs)")
    ap.add_argument("--layout", default="both", choices=["rows", "pairs", "both"],
                    help="rows: the row-block layout; pairs: the pair-split layout (DESIGN.md 6; "
                         "the partials' exchange left out, their buffers zero)")
    ap.add_argument("--scores", default="gathered",
                    help="comma list: gathered (DistSampler gather_data: the own m particles "
                         "over all Ng data rows, prior x S; the score blocks' all-gather left "
                         "out) | allreduce (all n particles over the rank's Ng / S rows; the "
                         "all-reduce left out)")
    args = ap.parse_args()
    import dsvgd
    if args.lib:
        dsvgd._native.LIB_PATH = os.path.abspath(args.lib)
    from dsvgd.engine import StageTimer
    from bench import synthetic_data
    n, d, Ng = 65536, 256, 16384
    x, t = synthetic_data(Ng, d - 1)
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    runs = []
    overrides = [{}]
    for spec in args.set:
        k, vals = spec.split("=")
        overrides = [dict(o, **{k: int(v)}) for o in overrides for v in vals.split(",")]
    if args.square:
        overrides = [dict(o, FULL_SQUARE=int(v)) for o in overrides for v in args.square.split(",")]
    for S in [int(v) for v in args.shards.split(",")]:
        for lay in (("rows", "pairs") if args.layout == "both" else (args.layout,)):
            if lay == "rows":
                runs.append((S, lay, False, True, 0, {}))
            elif S > 1 and dsvgd.PhiEngine.pair_split_ok(n, d, S):
                for side in args.side.split(","):
                    for rest in args.rest.split(","):
                        for fz in args.fwdz.split(","):
                            for ov in overrides:
                                runs.append((S, lay, bool(int(side)), bool(int(rest)), int(fz),
                                             ov))
    runs = [rn + (sm,) for rn in runs for sm in args.scores.split(",")]
    for S, lay, side, rest, fz, ov, smode in runs:
        for k in ("W_SPLITS", "H_SPLITS", "REST_SPLITS"):
            setattr(dsvgd.PhiEngine, k, ov.get(k) or None)
        from dsvgd.pairsplit import PairSplitPlan
        PairSplitPlan.FULL_SQUARE = (bool(ov["FULL_SQUARE"]) if "FULL_SQUARE" in ov else None)
        dsvgd.PhiEngine.WINDOW_SIDE_STREAM = side
        dsvgd.PhiEngine.REST_BESIDE = rest
        dsvgd.PhiEngine.FWD_ZSPLIT = fz or None
        m, r = n // S, S // 2          # a middle rank (a high one of the pair split)
        per = Ng // S
        gathered = smode == "gathered" and S > 1
        tgt = (dsvgd.targets.LogisticRegression(x, t) if gathered else
               dsvgd.targets.LogisticRegression(x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]))
        eng = dsvgd.PhiEngine(n, d, m=m, row0=r * m, device="cuda:0",
                              pair_split=(r, S) if lay == "pairs" else None)
        if eng.plan is not None:
            for b in eng.recvbuf:
                b.zero_()
        if S > 1:
            # the rank's 1/S of the bracket sample; the other ranks' shares
            # (the all-gather) stand in as a device copy of the whole sample
            full = torch.empty(eng.SAMPLE, device="cuda:0")
            from dsvgd import _native as NN
            eng.pack(X, None)
            NN.call("dsvgd_sample_sqdist", NN.ptr(eng.Y), eng.ldy, n, d, eng.SAMPLE, eng.SEED,
                    NN.ptr(full), NN.stream(0))

            def gather(sample, a, b, full=full):
                sample[:a].copy_(full[:a])
                sample[b:].copy_(full[b:])
            eng.sample_share = (r, S, gather)
        Sx = torch.empty_like(X)
        if gathered:   # the other ranks' score blocks (the all-gather's) stand in
            tgt.score(X, Sx, 1.0, prior_weight=float(S))
        Xo = X[r * m:(r + 1) * m].clone()
        timer = StageTimer()

        def step():
            with torch.cuda.device(0):
                from dsvgd.engine import span
                with span(eng.timer, "scores"):
                    if gathered:              # the own block over every rank's data
                        tgt.score(X[r * m:(r + 1) * m], Sx[r * m:(r + 1) * m], 1.0,
                                  prior_weight=float(S))
                    else:                     # all_scores: every particle on the local data
                        tgt.score(X, Sx)
                eng.pack(X, Sx)
                eng.distances(median=True)
                # the other S-1 ranks' counts approximated by this rank's (x S):
                # keeps the bracket check on its real (candidate) path
                eng.median_bandwidth((lambda v: v.mul_(S)) if S > 1 else None)
                eng.direction(Xo, 1e-6, write_phi=False)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        from dsvgd import _native as NX
        for mode, xv in [(a, b) for a in args.mode.split(",") for b in args.xmap.split(",")]:
          NX.load().dsvgd_phi_set_xmap(int(xv))
          run = step
          if mode == "timer":
              eng.timer = timer
              timer.events.clear()
          else:
              eng.timer = None
          if mode == "graph":
              from dsvgd.engine import StepGraph
              run = StepGraph(step, torch.device("cuda:0"))
              run()
              run()
              torch.cuda.synchronize()
          e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          e0.record()
          for _ in range(args.steps):
              run()
          e1.record()
          torch.cuda.synchronize()
          st = ({k: round(float(np.mean(v)), 3) for k, v in timer.summary().items()}
                if mode == "timer" else {})
          print(json.dumps({"shards": S, "mode": mode, "xmap": int(xv), "layout": lay + ("+side" if side else "")
                          + ("+rest" if lay == "pairs" and eng.plan is not None
                             and eng.rest_beside else ""), "m": m,
                          "fwd_z": getattr(eng, "fwd_z", None),
                          "w_splits": getattr(eng, "w_splits", None),
                          "h_splits": getattr(eng, "h_splits", None),
                          "t_splits": getattr(eng, "t_splits", None),
                          "row0": r * m, "N_local": per,
                          "scores": "gathered" if gathered else "allreduce",
                          "ms_per_step_no_comm": e0.elapsed_time(e1) / args.steps,
                          "sym_layout": bool(eng.sym), "full_square": bool(PairSplitPlan.full_square(S)),
                          "stages_ms": st}), flush=True)
          eng.timer = None
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
