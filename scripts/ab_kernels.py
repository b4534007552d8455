"""Interleaved in-process A/B timing of the contraction engines at the
headline shape (cdna_hip_programming.md rule 24: rounds interleaved in ONE
process): phi_mm, the distance Gram (+ bracket accounting) and the logreg
scores on FmtH2 / FmtX3 / f32 (PhiEngine(gemm=...), LogisticRegression(gemm=...)).

    python scripts/ab_kernels.py [--n 65536 --d 256 --rounds 5 --engines h2,x3]

Epilogue pricing needs an A/B build of the library (-DDSVGD_SQ_EPI=1|2|3,
see csrc/sqdist.hip), not a switch of the shipped one.
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
    ap.add_argument("--N", type=int, default=16384, help="logreg data rows")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--engines", default="h2,x3")
    args = ap.parse_args()
    import dsvgd
    n, d = args.n, args.d
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    xd = torch.randn(args.N, d - 1, generator=g) / (d ** 0.5)
    tl = torch.where(torch.randn(args.N, generator=g) > 0, 1.0, -1.0)
    engines = args.engines.split(",")
    res = {e: {"phi_mm": [], "distances": [], "scores": []} for e in engines}
    phis = {}
    for _ in range(args.rounds):
        for e in engines:
            eng = dsvgd.PhiEngine(n, d, device="cuda:0", gemm=e)
            tgt = dsvgd.targets.LogisticRegression(xd, tl, gemm=e)
            Sx = torch.empty_like(X)
            res[e]["scores"].append(timed(lambda: tgt.score(X, Sx)))
            eng.pack(X, S)
            res[e]["distances"].append(timed(lambda: eng.distances(median=True)))
            eng.median_bandwidth()
            res[e]["phi_mm"].append(timed(lambda: eng.direction(write_phi=True)))
            phis[e] = eng.phi.clone()
            del eng, tgt
            torch.cuda.empty_cache()
    ref = phis[engines[0]]
    out = {}
    for e in engines:
        out[e] = {k: float(np.median(v)) for k, v in res[e].items()}
        out[e]["phi_vs_%s" % engines[0]] = float((phis[e] - ref).abs().max() / ref.abs().max())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
