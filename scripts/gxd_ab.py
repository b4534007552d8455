"""logreg scores at the headline (n = 65536, p = 255, N = 16384, and the S = 8
shard N = 2048), an A/B switch on (1) and off (0), alternating, HIP events:
--switch dsvgd_phi_set_gxd_w1 (G . Xd on phi_w1_kernel<0, 2, false>) or
dsvgd_logreg_set_fused (the fused score kernel)."""
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
    ap.add_argument("--switch", default="dsvgd_phi_set_gxd_w1")
    ap.add_argument("--on", type=int, default=1, help="the switch value compared with --off")
    ap.add_argument("--off", type=int, default=0)
    args = ap.parse_args()
    import dsvgd
    from dsvgd import _native as N
    from bench import synthetic_data
    lib = N.load()
    n, d = 65536, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    out = {}
    for Ng in (16384, 2048):
        x, t = synthetic_data(Ng, d - 1)
        tgt = dsvgd.targets.LogisticRegression(x, t)
        S = {}
        for mode in (1, 0):
            getattr(lib, args.switch)(args.on if mode else args.off)
            Sx = torch.empty_like(X)
            tgt.score(X, Sx)
            S[mode] = Sx
        rel = float((S[1] - S[0]).abs().max() / S[0].abs().max())
        res = {1: [], 0: []}
        for _ in range(3):
            for mode in (1, 0):
                getattr(lib, args.switch)(args.on if mode else args.off)
                Sx = torch.empty_like(X)
                tgt.score(X, Sx)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    tgt.score(X, Sx)
                e1.record()
                torch.cuda.synchronize()
                res[mode].append(e0.elapsed_time(e1) / 5)
        out[Ng] = {"w1_ms": res[1], "nn_ms": res[0], "mean_w1": float(np.mean(res[1])),
                   "mean_nn": float(np.mean(res[0])), "scores_rel_diff": rel}
    getattr(lib, args.switch)(args.off)
    print(json.dumps({"switch": args.switch, "by_N": out}), flush=True)


if __name__ == "__main__":
    main()
