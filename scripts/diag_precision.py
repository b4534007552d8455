"""Where does the full-size phi error come from?  n=65536, d=256, sampled rows:
compare D, r' = sum_{j!=i} k_ij, K'X, K'S and phi against fp64.

    python scripts/diag_precision.py [n] [A/B library]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dist-svgd_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dsvgd  # noqa: E402
from oracle import svgd_oracle as O  # noqa: E402

n, d = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 256
if len(sys.argv) > 2:
    dsvgd._native.LIB_PATH = os.path.abspath(sys.argv[2])
rs = np.random.RandomState(0)
X = rs.randn(n, d).astype(np.float32)
mu = rs.randn(d).astype(np.float32)
lam = rs.uniform(0.5, 2, d).astype(np.float32)
S = O.score_gaussian(X, mu, lam).astype(np.float32)
eng = dsvgd.PhiEngine(n, d, device="cuda:0")
eng.step(torch.tensor(X).cuda(), torch.tensor(S).cuda(), h=None)
med, h, inv_h = eng.state.read()
rows = np.sort(rs.choice(n, 64, replace=False))
Dd = eng.dense_D()[torch.as_tensor(rows, device="cuda:0")].cpu().numpy().astype(np.float64)
Dr = O.sqdist(X[rows], X)
print("h", h, "inv_h", inv_h, "1/h", 1 / h)
print("D: max abs err", np.abs(Dd - Dr).max(), "max rel", (np.abs(Dd - Dr) / np.maximum(Dr, 1e-30)).max())
K = np.exp(-Dr / h)
for a, i in enumerate(rows):
    K[a, i] = 0.0
Xc = X.astype(np.float64) - X.astype(np.float64).mean(0)
KY = eng.KY.view(eng.splits, n, -1).sum(0)[torch.as_tensor(rows, device="cuda:0")].cpu().numpy()
rsum = eng.rowsum.view(eng.splits, -1).sum(0)[torch.as_tensor(rows, device="cuda:0")].cpu().numpy()
dp = eng.dp
kx_ref, ks_ref, r_ref = K @ Xc, K @ S.astype(np.float64), K.sum(1)
print("r'   rel err", np.abs(rsum - r_ref).max() / np.abs(r_ref).max(), "max r'", np.abs(r_ref).max())
print("K'X  rel err", np.abs(KY[:, :d] - kx_ref).max() / np.abs(kx_ref).max(), "max", np.abs(kx_ref).max())
print("K'S  rel err", np.abs(KY[:, dp:dp + d] - ks_ref).max() / np.abs(ks_ref).max(), "max", np.abs(ks_ref).max())
# what phi error each part alone causes (normalised by max |phi|)
phi_ref = O.phi(X, S, h, rows=rows)
scale = np.abs(phi_ref).max()
g = 2.0 / h
e_r = g * (rsum - r_ref)[:, None] * Xc[rows] / n
e_kx = -g * (KY[:, :d] - kx_ref) / n
e_ks = (KY[:, dp:dp + d] - ks_ref) / n
print("phi err from r'", np.abs(e_r).max() / scale, "from K'X", np.abs(e_kx).max() / scale,
      "from K'S", np.abs(e_ks).max() / scale)
got = eng.phi[torch.as_tensor(rows, device="cuda:0")].cpu().numpy()
print("phi total err", np.abs(got - phi_ref).max() / scale, "max|phi|", scale)
# rowsum accumulated in fp64 from the GPU's own K
Kg = np.exp2(Dd * np.float32(-inv_h * 1.4426950408889634))
for a, i in enumerate(rows):
    Kg[a, i] = 0.0
print("r' from GPU D in fp64 vs fp64 ref", np.abs(Kg.sum(1) - r_ref).max() / np.abs(r_ref).max())
