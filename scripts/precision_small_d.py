"""phi precision of the Gram/MFMA path vs the explicit-difference (direct)
path at small d, against the fp64 oracle (max-normalised, sampled rows):
where may d <= 64 move to MFMA without losing the 1e-5 tolerance?

    python scripts/precision_small_d.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dist-svgd_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dsvgd  # noqa: E402
from oracle import svgd_oracle as O  # noqa: E402


def phi_err(X, S, mfma):
    n, d = X.shape
    eng = dsvgd.PhiEngine(n, d, device="cuda:0")
    if mfma:
        eng.DIRECT_MAX_D = 0
    eng.step(torch.tensor(X).cuda(), torch.tensor(S).cuda(), h=None)
    torch.cuda.synchronize()
    h = eng.state.read()[1]
    rows = np.sort(np.random.RandomState(1).choice(n, min(n, 256), replace=False))
    ref = O.phi(X, S, h, rows=rows)
    got = eng.phi[torch.as_tensor(rows, device="cuda:0")].cpu().numpy()
    e = float(np.abs(got - ref).max() / np.abs(ref).max())
    return e, h


def main():
    out = {}
    for kind in ("gauss", "gmm"):
        for d in ([1, 2] if kind == "gmm" else [2, 4, 8, 16, 32, 64]):
            for n in (2048, 16384):
                rs = np.random.RandomState(n + d)
                X = rs.randn(n, d).astype(np.float32)
                if kind == "gauss":
                    mu = rs.randn(d).astype(np.float32)
                    lam = rs.uniform(0.5, 2, d).astype(np.float32)
                    S = O.score_gaussian(X, mu, lam).astype(np.float32)
                else:
                    S = O.score_gmm(X).astype(np.float32)
                ed, h = phi_err(X, S, False)
                em, _ = phi_err(X, S, True)
                out["%s_d%d_n%d" % (kind, d, n)] = {"direct": ed, "mfma": em, "h": h}
                print(json.dumps({"%s_d%d_n%d" % (kind, d, n): out["%s_d%d_n%d" % (kind, d, n)]}),
                      flush=True)


if __name__ == "__main__":
    main()
