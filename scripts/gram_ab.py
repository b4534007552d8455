"""The S = 1 distance Gram (n = 65536, d = 256, bracketed median accounting)
with an A/B switch of the one-wave-per-SIMD Gram at --on and --off,
alternating, HIP events; D must come out bit-identical.  (profiles/r13ad: the
switches dsvgd_gram_set_adepth and dsvgd_gram_set_packed of two builds since
reverted.)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", required=True, help="an int setter exported by the library")
    ap.add_argument("--on", type=int, default=1)
    ap.add_argument("--off", type=int, default=0)
    args = ap.parse_args()
    import dsvgd
    from dsvgd import _native as N
    lib = N.load()
    n, d = 65536, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    Sx = (0.1 * torch.randn(n, d, generator=g)).cuda()
    eng = dsvgd.PhiEngine(n, d, device="cuda:0")
    eng.pack(X, Sx)
    ref = {}
    for ad in (args.on, args.off):
        getattr(lib, args.switch)(ad)
        eng.distances(median=True)
        eng.median_bandwidth()
        torch.cuda.synchronize()
        ref[ad] = eng.D.clone()
    same_D = bool(torch.equal(ref[args.on], ref[args.off]))
    del ref
    res = {args.on: [], args.off: []}
    for _ in range(4):
        for ad in (args.on, args.off):
            getattr(lib, args.switch)(ad)
            eng.distances(median=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                eng.distances(median=True)
            e1.record()
            torch.cuda.synchronize()
            res[ad].append(e0.elapsed_time(e1) / 5)
    getattr(lib, args.switch)(args.on)
    print(json.dumps({"distances_ms": {str(k): v for k, v in res.items()},
                      "switch": args.switch, "mean_on": float(np.mean(res[args.on][1:])),
                      "mean_off": float(np.mean(res[args.off][1:])),
                      "D_identical": same_D}), flush=True)


if __name__ == "__main__":
    main()
