"""phi_mm on the symmetric layout (n = 65536, d = 256): one launch per row
(dsvgd_phi_set_symrow(1), phi_w1 DS 4) against the two-launch hybrid (0),
alternating, HIP events around phi_mm only.

    python scripts/symrow_ab.py [--rounds 4 --steps 4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    args = ap.parse_args()
    import dsvgd
    from dsvgd import _native as N
    from dsvgd.engine import StageTimer
    n, d = args.n, args.d
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    eng = dsvgd.PhiEngine(n, d, device="cuda:0")
    lib = N.load()
    out = {}
    phis = {}
    for mode in (1, 0):
        lib.dsvgd_phi_set_symrow(mode)
        eng.step(X, S, h=None, write_phi=True)
        phis[mode] = eng.phi.clone()
    diff = float((phis[1] - phis[0]).abs().max() / phis[0].abs().max())
    # forms: (symrow, xmap, splits)
    forms = {"rows": (1, 1, eng.splits), "rows_noxmap": (1, 0, eng.splits),
             "rows_z2": (1, 1, 2), "hybrid": (0, 1, eng.splits)}
    base_splits = eng.splits
    for _ in range(args.rounds):
        for mode, (sr, xm, z) in forms.items():
            lib.dsvgd_phi_set_symrow(sr)
            lib.dsvgd_phi_set_xmap(xm)
            eng.splits = z
            eng.step(X, S, h=None, write_phi=False)
            t = StageTimer(only={"phi_mm", "sqdist"})
            eng.timer = t
            for _ in range(args.steps):
                eng.step(X, S, h=None, write_phi=False)
            eng.timer = None
            sm = t.summary()
            out.setdefault(mode, []).append(float(np.mean(sm["phi_mm"])))
    lib.dsvgd_phi_set_symrow(1)
    lib.dsvgd_phi_set_xmap(1)
    eng.splits = base_splits
    print(json.dumps({"n": n, "d": d, "splits": int(base_splits), "sym": bool(eng.sym),
                      "phi_mm_ms": out,
                      "mean": {k: float(np.mean(v)) for k, v in out.items()},
                      "phi_rel_diff_rows_vs_hybrid": diff}), flush=True)


if __name__ == "__main__":
    main()
