"""Time the GPU W2/JKO term (dsvgd.w2.W2Term.grad: cost + auction + gradient)
on random and SVGD-shaped inputs.

    python scripts/w2_timing.py [--big] [--lib A/B library]

SVGD shape: the owned block X (m rows) against previous particles of which
the first m rows are X before a small step (all_particles / all_scores mode
with R = n/m ranks) -- the structure make_step hands to the term.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def case(m, n, d, kind, seed=0):
    import dsvgd
    g = torch.Generator(device="cpu").manual_seed(seed)
    X = torch.randn(m, d, generator=g)
    if kind == "random":
        P = torch.randn(n, d, generator=g)
    else:   # svgd: own rows moved by a small step, other rows other ranks' particles
        P = torch.randn(n, d, generator=g)
        P[:m] = X - 1e-3 * torch.randn(m, d, generator=g)
    X, P = X.cuda(), P.cuda()
    w = dsvgd.w2.W2Term(m, n, d, "cuda:0", warm=False)
    # the cost matrix alone (the form W2Term chose), HIP events over 3 calls
    from dsvgd import _native as N
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(2):
        e0.record()
        for _ in range(3):
            if w.cost == "h2":
                N.call("dsvgd_w2_cost_h2", N.ptr(X), d, m, N.ptr(P), d, n, d, N.ptr(w.C), w.ldc,
                       (N.ptr(w.cws) + 255) // 256 * 256, float(w.TAU), N.ptr(w.cstat),
                       N.stream(X.device))
            else:
                N.call("dsvgd_w2_cost", N.ptr(X), d, m, N.ptr(P), d, n, d, N.ptr(w.C), w.ldc,
                       N.stream(X.device))
        e1.record()
        torch.cuda.synchronize()
    cost_ms = e0.elapsed_time(e1) / 3
    w.grad(X, P, 1.0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    w.grad(X, P, 1.0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    out = {"m": m, "n": n, "d": d, "kind": kind, "ms": round(ms, 3), "rounds": w.rounds,
           "cost_ms": round(cost_ms, 3),
           "us_per_round": round(ms * 1e3 / max(w.rounds, 1), 2)}
    # the next SVGD step: rows and columns both moved by a small step; warm
    # start from this solve's prices vs a cold solve of the same problem
    cold_plan = None
    g2 = torch.Generator(device="cpu").manual_seed(seed + 7)
    X2 = X + 1e-3 * torch.randn(m, d, generator=g2).cuda()
    P2 = P + 1e-3 * torch.randn(n, d, generator=g2).cuda()
    for warm in (False, True):
        ww = dsvgd.w2.W2Term(m, n, d, "cuda:0", warm=warm)
        ww.grad(X, P, 1.0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        G = ww.grad(X2, P2, 1.0).clone()
        torch.cuda.synchronize()
        key = "warm" if warm else "cold"
        out[key + "_next_ms"] = round((time.perf_counter() - t) * 1e3, 3)
        out[key + "_next_rounds"] = ww.rounds
        out[key + "_next_tail_bids_scans"] = ww.tail_stats()
        cost = float(((X2[torch.arange(n, device="cuda") // (n // m)] - P2[ww.assign.long()]) ** 2)
                     .sum())
        out[key + "_next_cost"] = cost
        if cold_plan is None:
            cold_plan = G
        else:
            out["warm_vs_cold_grad_maxdiff"] = float((G - cold_plan).abs().max())
        if TRACE:
            out[key + "_next_profile"] = profile(ww.trace())
        out["cost_form"] = ww.cost
        out["_plan"] = ww.assign.clone()
    return out


def profile(tr):
    """Rounds per epsilon phase, split by how many slots were unassigned when
    they ran (from the 16-round control readbacks)."""
    buckets = (16, 256, 4096, 1 << 62)
    prof, prev = {}, 0
    for rounds, phase, un in tr:
        b = next(k for k in buckets if un < k)
        ph = prof.setdefault(str(phase), {str(k): 0 for k in buckets})
        ph[str(b)] += rounds - prev
        prev = rounds
    return prof


TRACE = False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--warm-sweep", action="store_true",
                    help="warm-start phases 1..5 on two R > 1 shapes")
    ap.add_argument("--lib", default=None, help="an A/B build of the library (make ab)")
    ap.add_argument("--shapes", default=None,
                    help="m x n x d list, e.g. 8192x65536x256,2048x16384x256 (svgd shape)")
    ap.add_argument("--trace", action="store_true",
                    help="rounds per phase by unassigned-slot count")
    ap.add_argument("--theta", default="8",
                    help="comma list of W2Term.THETA settings to sweep on --shapes")
    ap.add_argument("--keep", default="0",
                    help="comma list of W2Term.KEEP settings to sweep on --shapes (1, 0)")
    ap.add_argument("--cost", default="auto",
                    help="comma list of W2Term.COST settings to sweep on --shapes (auto, h2, exact)")
    ap.add_argument("--warm-phases", default=None,
                    help="comma list of warm phase counts to sweep on --shapes (a = adaptive)")
    ap.add_argument("--fuse-first", type=int, default=1,
                    help="R = 1 warm starts: violation + first-round scans in one pass "
                         "(dsvgd_w2_set_fuse_first)")
    args = ap.parse_args()
    from dsvgd import _native
    _native.load().dsvgd_w2_set_fuse_first(args.fuse_first)
    global TRACE
    TRACE = args.trace
    if args.shapes:
        import dsvgd
        shapes = [tuple(int(v) for v in sh.split("x")) + ("svgd",) for sh in args.shapes.split(",")]
        for keep, theta in [(bool(int(k)), float(th)) for k in args.keep.split(",")
                            for th in args.theta.split(",")]:
            dsvgd.w2.W2Term.KEEP = keep
            dsvgd.w2.W2Term.THETA = theta
            for ph in ([None if v == "a" else int(v) for v in args.warm_phases.split(",")]
                       if args.warm_phases else [dsvgd.w2.W2Term.WARM_PHASES]):
                dsvgd.w2.W2Term.WARM_PHASES = ph
                for sh in shapes:
                    plans = {}
                    for cm in args.cost.split(","):
                        dsvgd.w2.W2Term.COST = cm
                        r = case(*sh)
                        r["warm_phases"] = ph
                        r["keep"] = keep
                        r["theta"] = theta
                        r["cost_mode"] = cm
                        plans[cm] = r.pop("_plan")
                        if len(plans) > 1:
                            first = next(iter(plans.values()))
                            r["plan_equal_to_" + next(iter(plans))] = bool(
                                torch.equal(first, plans[cm]))
                        print(json.dumps(r), flush=True)
                    dsvgd.w2.W2Term.COST = "auto"
        return
    if args.lib:
        import dsvgd
        dsvgd._native.LIB_PATH = os.path.abspath(args.lib)
    if args.warm_sweep:
        import dsvgd
        for ph in (1, 2, 3, 4, 5):
            dsvgd.w2.W2Term.WARM_PHASES = ph
            for sh in ((1024, 8192, 16, "svgd"), (2048, 16384, 256, "svgd")):
                r = case(*sh)
                print(json.dumps({"warm_phases": ph, "m": sh[0], "n": sh[1],
                                  "warm_next_ms": r["warm_next_ms"],
                                  "warm_next_rounds": r["warm_next_rounds"],
                                  "cold_next_rounds": r["cold_next_rounds"]}), flush=True)
        return
    shapes = [(256, 256, 16, "random"), (2048, 2048, 64, "random"), (500, 4000, 3, "random"),
              (1024, 8192, 16, "svgd"), (4096, 4096, 256, "svgd"), (2048, 16384, 256, "svgd"),
              (4096, 32768, 64, "svgd")]
    if args.big:
        shapes += [(8192, 65536, 256, "svgd"), (65536, 65536, 256, "svgd")]
    for s in shapes:
        r = case(*s)
        r.pop("_plan", None)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
