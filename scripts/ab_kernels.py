"""Interleaved in-process A/B timing of kernel variants at the headline shape
(cdna_hip_programming.md rule 24: rounds interleaved in ONE process).

    python scripts/ab_kernels.py [--n 65536 --d 256 --rounds 5]

Variants are switched through environment variables the launchers read on
every call (DSVGD_NN_SHAPE=w2 forces the 16-deep NN K-step of the f32 engine;
ENGINE_X3 picks the phi_mm engine).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import dsvgd
    n, d = args.n, args.d
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.randn(n, d, generator=g).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    eng = dsvgd.PhiEngine(n, d, device="cuda:0")
    eng.pack(X, S)
    eng.distances(median=True)
    eng.median_bandwidth()
    # ENGINE_X3: "1" = the bf16-split phi_mm (default), "0" = the f32 MFMA engine
    variants = json.loads(os.environ.get("AB_VARIANTS", "null")) or {
        "phi=x3": {"ENGINE_X3": "1", "RECOMPUTE_D": "1"},
        "phi=f32": {"ENGINE_X3": "0", "RECOMPUTE_D": "1"}}  # f32: the full D layout
    res = {k: [] for k in variants}
    ref = None
    keys = {k for env in variants.values() for k in env}
    for _ in range(args.rounds):
        for name, env in variants.items():
            for k in keys:               # a variant's knobs must not leak into the next
                os.environ.pop(k, None)
            os.environ.update(env)
            eng.x3 = env.get("ENGINE_X3", "1") == "1" and hasattr(eng, "Yx")
            if env.get("RECOMPUTE_D") == "1":  # the variant changes D's layout
                eng.distances(median=True)
                eng.median_bandwidth()
            res[name].append(timed(lambda: eng.direction(write_phi=True)))
            if ref is None:
                ref = eng.phi.clone()
            elif not env.get("NOCHECK"):
                err = float((eng.phi - ref).abs().max() / ref.abs().max())
                assert err < 1e-5, (name, err)
    eng.x3 = hasattr(eng, "Yx")  # the default engines (and D layout) for the timings below
    for k in keys:
        os.environ.pop(k, None)
    flops = 4.0 * n * n * d
    out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
               "tflops": flops / (np.median(v) * 1e-3) / 1e12} for k, v in res.items()}
    out["sqdist_ms"] = timed(lambda: eng.distances(median=False))
    if getattr(eng, "x3_gram", False):
        eng.x3_gram = False
        out["sqdist_f32_ms"] = timed(lambda: eng.distances(median=False))
        out["sqdist_bracket_f32_ms"] = timed(lambda: eng.distances(median=True))
        eng.x3_gram = True
    for k, v in json.loads(os.environ.get("AB_SQ_VARIANTS", "{}")).items():
        os.environ.update(v)
        out["sqdist_ms[%s]" % k] = timed(lambda: eng.distances(median=False))
        out["sqdist_bracket_ms[%s]" % k] = timed(lambda: eng.distances(median=True))
        out["sqdist_select_ms[%s]" % k] = timed(
            lambda: (eng.distances(median=True), eng.median_bandwidth()))
        for key in v:
            os.environ.pop(key, None)
    # logistic-regression scores at the bench shape (N = 16384 rows, p = d - 1)
    xd = torch.randn(16384, d - 1, generator=g) / (d ** 0.5)
    tl = torch.where(torch.randn(16384, generator=g) > 0, 1.0, -1.0)
    tgt = dsvgd.targets.LogisticRegression(xd, tl)
    Sx = torch.empty_like(X)
    out["logreg_score_ms"] = timed(lambda: tgt.score(X, Sx))
    out["sqdist_bracket_ms"] = timed(lambda: eng.distances(median=True))
    out["sqdist_select_ms"] = timed(lambda: (eng.distances(median=True), eng.median_bandwidth()))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
