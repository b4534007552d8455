"""phi_mm and the distance stage alone at the headline shape on chosen engines / D layouts (for
rocprofv3 counter passes): one distance + median stage, then `--reps`
direction() calls per configuration.

    python scripts/phi_probe.py [--configs h2:sym,h2:full,x3:sym] [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--configs", default="h2:sym,h2:full,x3:sym,x3:full")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=None, help="an A/B build of the library (make ab)")
    ap.add_argument("--dump", default=None,
                    help="save every 256th row of phi per configuration to DUMP_<cfg>.npy")
    args = ap.parse_args()
    import dsvgd
    if args.lib:
        dsvgd._native.LIB_PATH = os.path.abspath(args.lib)
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(args.n, args.d, generator=g)).cuda()
    S = torch.randn(args.n, args.d, generator=g).cuda()
    out = {}
    for cfg in args.configs.split(","):
        gemm, lay = cfg.split(":")
        eng = dsvgd.PhiEngine(args.n, args.d, device="cuda:0", gemm=gemm, sym_layout=lay == "sym")
        eng.pack(X, S)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.distances(median=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.reps):
            eng.distances(median=True)
        e1.record()
        torch.cuda.synchronize()
        dist_ms = e0.elapsed_time(e1) / args.reps
        e0.record()
        for _ in range(args.reps):
            eng.distances(median=False)
        e1.record()
        torch.cuda.synchronize()
        dist_plain_ms = e0.elapsed_time(e1) / args.reps
        eng.distances(median=True)
        eng.median_bandwidth()
        eng.direction(write_phi=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.reps):
            eng.direction(write_phi=True)
        e1.record()
        torch.cuda.synchronize()
        if args.dump:
            import numpy as np
            np.save("%s_%s.npy" % (args.dump, cfg.replace(":", "_")),
                    eng.phi[::256].float().cpu().numpy())
        out[cfg] = {"sym": bool(eng.sym), "phi_ms": e0.elapsed_time(e1) / args.reps,
                    "distances_ms": dist_ms, "distances_no_select_ms": dist_plain_ms}
        print(json.dumps({cfg: out[cfg]}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
