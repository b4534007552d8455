"""The reference's default Gauss-Seidel order (sampler.py:64-68,
distsampler.py:194-200) at the BASELINE shapes: one DistSampler step of
config D (n = 65536, d = 256, logreg, all_scores: the scores frozen for the
sweep) and of config E's shape (d = 1024) through the wide blocked sweep,
next to the per-row path (one phi_row_split launch per particle) timed on a
bounded sample of rows and extrapolated to the whole sweep.

    python scripts/seq_timing.py [--only D,E] [--rows-sample 2048]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="D,E")
    ap.add_argument("--group", default=None,
                    help="comma list of engine.GSW_GROUP values: the blocked sweep alone "
                         "timed for each (blocks per wide pass)")
    ap.add_argument("--inc", default=None,
                    help="comma list of dsvgd_gsw_set_inc values (1: the incremental walk, "
                         "0: the four-wave walk): the blocked sweep alone timed for each")
    ap.add_argument("--ab", default=None,
                    help="NAME=v1,v2: the blocked sweep alone timed for each value of the "
                         "library switch NAME (e.g. dsvgd_gsw_set_corr_lds=1,0); the first "
                         "value is restored after")
    ap.add_argument("--splits", default=None,
                    help="comma list of engine.GSW_SPLITS values (0: chosen): the blocked "
                         "sweep alone timed for each")
    ap.add_argument("--pipe", default=None,
                    help="comma list of engine.GSW_PIPELINE values (1: the pipelined wide "
                         "sweep, 0: block group after group): the blocked sweep alone timed "
                         "for each, the results compared")
    ap.add_argument("--reserve", default=None,
                    help="comma list of engine.GSW_SIDE_RESERVE values (CUs the pipelined "
                         "sweep's side passes leave to the walk): the sweep timed for each")
    ap.add_argument("--graphs", type=int, default=0,
                    help="1: also time DistSampler.make_step as the product runs it at S = 1 "
                         "(captured as one HIP graph on the second call, replayed after)")
    ap.add_argument("--pipe-max-d", type=int, default=None,
                    help="engine.GSW_PIPELINE_MAX_D for the --pipe / --reserve runs")
    ap.add_argument("--rows-sample", type=int, default=2048,
                    help="rows of the per-row path to time (0: skip it)")
    args = ap.parse_args()
    import dsvgd
    from dsvgd.engine import sequential_sweep
    from bench import synthetic_data
    # R: a logreg target whose scores are refreshed after every move (the
    # partition mode's exchange_scores=False; 2048 data rows = config D's
    # N_local at S = 8), scores scaled by N_global / N_local = 8
    shapes = {"D": (65536, 256, 16384), "E": (65536, 1024, 8192), "R": (16384, 256, 2048)}
    if args.pipe_max_d is not None:
        import dsvgd.engine as E
        E.GSW_PIPELINE_MAX_D = args.pipe_max_d
    for name in args.only.split(","):
        n, d, Ng = shapes[name]
        refresh = name == "R"
        x, t = synthetic_data(Ng, d - 1)
        g = torch.Generator(device="cpu").manual_seed(0)
        X = (0.1 * torch.randn(n, d, generator=g)).cuda()
        ds = dsvgd.DistSampler(0, 1, dsvgd.targets.LogisticRegression(x, t), dsvgd.RBF("median"),
                               X, 8 * Ng if refresh else Ng, Ng, exchange_particles=True,
                               exchange_scores=not refresh, include_wasserstein=False,
                               order="sequential")
        tgt = ds._target if refresh else None
        scale = 8.0 if refresh else 1.0
        ds.graphs = False
        ds.make_step(1e-4)                      # warm-up (workspaces, median engine)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ds.make_step(1e-4)
        torch.cuda.synchronize()
        blocked_ms = 1e3 * (time.perf_counter() - t0)
        graph_ms = None
        if args.graphs:
            ds.graphs = True
            ds.make_step(1e-4)                  # eager (graphs start counting here)
            ds.make_step(1e-4)                  # captured
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                ds.make_step(1e-4)              # replayed
            torch.cuda.synchronize()
            graph_ms = 1e3 * (time.perf_counter() - t0) / 2
            ds.graphs = False
        # the per-row kernels over a sample of rows, same scores and bandwidth
        eng = next(iter(ds._engines.values()))
        if refresh:     # the sweep's starting scores (the sampler keeps them internal)
            S0 = torch.empty_like(X)
            tgt.score(X, S0, scale)
        else:
            S0 = ds._scores
        k = min(args.rows_sample, n)
        per_row_ms = None
        if k > 0:
            Xc, Sc = X.clone(), S0.clone()
            sequential_sweep(Xc, Sc, range(0, 64), eng.state, 1e-4, target=tgt, score_scale=scale,
                             blocked=False)   # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sequential_sweep(Xc, Sc, range(64, 64 + k), eng.state, 1e-4, target=tgt,
                             score_scale=scale, blocked=False)
            torch.cuda.synchronize()
            per_row_ms = 1e3 * (time.perf_counter() - t0) * n / k
        # the blocked sweep alone (no median / scores), for the stage split
        Xb, Sb = X.clone(), S0.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
        torch.cuda.synchronize()
        sweep_ms = 1e3 * (time.perf_counter() - t0)
        print(json.dumps({"config": name, "n": n, "d": d, "N_local": Ng,
                          "scores": "refreshed (logreg)" if refresh else "frozen (all_scores)",
                          "order": "sequential",
                          "step_ms_blocked": blocked_ms, "step_ms_graph": graph_ms,
                          "sweep_only_ms_blocked": sweep_ms,
                          "particle_updates_per_s": n / blocked_ms * 1e3,
                          "per_row_ms_extrapolated": per_row_ms, "per_row_sample_rows": k,
                          "speedup_vs_per_row": per_row_ms / sweep_ms if per_row_ms else None}),
              flush=True)
        if args.group:
            import dsvgd.engine as E
            res = {}
            for gv in [int(v) for v in args.group.split(",")] * 2:
                E.GSW_GROUP = gv
                Xb, Sb = X.clone(), S0.clone()
                sequential_sweep(Xb, Sb, range(0, 512), eng.state, 1e-4, target=tgt,
                                 score_scale=scale)     # warm-up (buffers for this group)
                Xb, Sb = X.clone(), S0.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
                torch.cuda.synchronize()
                res.setdefault(gv, []).append(1e3 * (time.perf_counter() - t0))
                res.setdefault("x_%d" % gv, Xb[::4096].cpu())
            ref = res.pop("x_1", None)
            out = {"config": name, "sweep_ms_by_group": {k: v for k, v in res.items()
                                                         if not str(k).startswith("x_")}}
            if ref is not None:
                out["max_abs_diff_vs_group1"] = {k[2:]: float((v - ref).abs().max())
                                                 for k, v in res.items() if str(k).startswith("x_")}
            print(json.dumps(out), flush=True)
            E.GSW_GROUP = None
        if args.pipe:
            import dsvgd.engine as E
            res, xs = {}, {}
            for pv in [int(v) for v in args.pipe.split(",")] * 2:
                E.GSW_PIPELINE = bool(pv)
                Xb, Sb = X.clone(), S0.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
                torch.cuda.synchronize()
                res.setdefault(pv, []).append(1e3 * (time.perf_counter() - t0))
                xs[pv] = Xb
            vals = list(xs.values())
            scale_x = float((vals[0] - X).abs().max())
            print(json.dumps({"config": name, "sweep_ms_by_pipeline": res,
                              "finite": [bool(torch.isfinite(v).all()) for v in vals],
                              "max_abs_diff_between": float((vals[0] - vals[-1]).abs().max()),
                              "max_abs_move": scale_x}), flush=True)
            E.GSW_PIPELINE = True
        if args.reserve:
            import dsvgd.engine as E
            res, xs = {}, {}
            keep = E.GSW_SIDE_RESERVE
            for rv in [int(v) for v in args.reserve.split(",")] * 2:
                E.GSW_SIDE_RESERVE = rv
                Xb, Sb = X.clone(), S0.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
                th = time.perf_counter()        # the host's enqueue time of the sweep
                torch.cuda.synchronize()
                res.setdefault(rv, []).append(1e3 * (time.perf_counter() - t0))
                res.setdefault("host_%d" % rv, []).append(1e3 * (th - t0))
                xs[rv] = Xb
            vals = list(xs.values())
            print(json.dumps({"config": name, "sweep_ms_by_side_reserve": res,
                              "finite": [bool(torch.isfinite(v).all()) for v in vals],
                              "max_abs_diff_between": float((vals[0] - vals[-1]).abs().max())}),
                  flush=True)
            E.GSW_SIDE_RESERVE = keep
        if args.splits:
            import dsvgd.engine as E
            res = {}
            for zv in [int(v) for v in args.splits.split(",")] * 2:
                E.GSW_SPLITS = zv or None
                Xb, Sb = X.clone(), S0.clone()
                sequential_sweep(Xb, Sb, range(0, 512), eng.state, 1e-4, target=tgt,
                                 score_scale=scale)     # warm-up (this split count's buffers)
                Xb, Sb = X.clone(), S0.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
                torch.cuda.synchronize()
                res.setdefault(zv, []).append(1e3 * (time.perf_counter() - t0))
            E.GSW_SPLITS = None
            print(json.dumps({"config": name, "sweep_ms_by_splits": res}), flush=True)
        if args.inc or args.ab:
            from dsvgd import _native as NN
            lib = NN.load()
            sw, vals = ("dsvgd_gsw_set_inc", args.inc) if args.inc else args.ab.split("=")
            vals = [int(u) for u in vals.split(",")]
            res, xs = {}, {}
            for v in vals * 2:
                getattr(lib, sw)(v)
                Xb, Sb = X.clone(), S0.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sequential_sweep(Xb, Sb, range(n), eng.state, 1e-4, target=tgt, score_scale=scale)
                torch.cuda.synchronize()
                res.setdefault(v, []).append(1e3 * (time.perf_counter() - t0))
                xs[v] = Xb
            getattr(lib, sw)(vals[0])
            out = {"config": name, "switch": sw, "sweep_ms_by_value": res}
            ref = xs[vals[-1]]
            out["max_rel_diff_vs_last"] = {
                k: float((v - ref).abs().max() / ref.abs().max()) for k, v in xs.items()}
            print(json.dumps(out), flush=True)
            del xs
        del ds, eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
