"""FmtH2's dynamic-range window: an fp16 part keeps 22
significant bits only for entries within 2^-16 of the largest magnitude
sharing its power-of-two scale (a column of phi_mm's B operand [Xc | S], the
whole Xc tensor of the Gram's row image, the whole W of logreg's Z);
smaller ones keep an absolute bound of 2^-38 of that largest.  fp32 has no
such window, so the max-normalised phi error can hide a tail particle next
to a divergent one.  These tests put one outlier particle -- far away, with
scores 2^16 .. 2^30 times the rest, or both -- among n ordinary ones and
check every row in ROW-normalised form,

    max_i |phi_i - phi_i^ref|_2 / |phi_i^ref|_2  <=  1e-5

against the fp64 restatement (and the same for the logreg scores), next to
the exact f32 MFMA engine on the same inputs.  The engine's range guard
(pack's row / column maxima -> dsvgd_h2_scales: an operand whose range
exceeds 2^16 runs that step's contraction on the FmtX3 engine instead) is
what keeps the default engine inside the bound; its decision is checked too.
"""
import numpy as np
import pytest
import torch

from conftest import record_parity
from oracle import svgd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROW_TOL = 1e-5


def dsvgd():
    import dsvgd as m
    return m


def gpu(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def row_err(got, ref):
    num = np.sqrt(((np.asarray(got, np.float64) - ref) ** 2).sum(1))
    den = np.sqrt((ref ** 2).sum(1))
    return num / np.maximum(den, 1e-300)


def _outlier_case(n, d, kind, k, seed=0):
    rs = np.random.RandomState(seed)
    X = (0.3 * rs.randn(n, d)).astype(np.float32)
    S = (-X / 0.09 + rs.randn(n, d)).astype(np.float32)
    j = 17
    if kind in ("far", "far_score"):
        X[j] = X[j] + np.float32(2.0 ** k * 0.3)          # no kernel weight to anyone
    if kind in ("score", "far_score"):
        S[j] = S[j] * np.float32(2.0 ** k)
    return X, S


def _phi(X, S, gemm):
    n, d = X.shape
    eng = dsvgd().PhiEngine(n, d, device=DEV, gemm=gemm)
    Xo = gpu(X).clone()
    eng.step(gpu(X), gpu(S), X_own=Xo, step=0.0, h=None)
    torch.cuda.synchronize()
    return eng.phi.cpu().numpy(), eng.state.read()[1], eng


CASES = [(kind, k) for kind in ("score", "far", "far_score") for k in (16, 20, 24, 30)]


@pytest.mark.parametrize("n,d", [(2048, 64), (4096, 256)])
@pytest.mark.parametrize("kind,k", CASES)
def test_phi_row_normalised_with_outlier(n, d, kind, k):
    X, S = _outlier_case(n, d, kind, k)
    phi_h2, h, eng = _phi(X, S, "h2")
    phi_f32, h32, _ = _phi(X, S, "f32")
    ref = O.phi(X, S, h)
    e_h2, e_f32 = row_err(phi_h2, ref), row_err(phi_f32, O.phi(X, S, h32))
    record_parity(float(e_h2.max()), f32=float(e_f32.max()), kind=kind, k=k,
                  guard=getattr(eng, "range_guard", lambda: None)())
    assert e_h2.max() <= ROW_TOL, (e_h2.max(), int(e_h2.argmax()), e_f32.max())


@pytest.mark.parametrize("k", [18, 24, 30])
def test_logreg_scores_row_normalised_with_outlier(k):
    """One particle's w 2^k times the others' (logreg's W image shares one
    tensor scale): every particle's score row vs fp64, row-normalised."""
    n, N, p = 1024, 4096, 255
    rs = np.random.RandomState(k)
    X = (0.1 * rs.randn(n, p + 1)).astype(np.float32)
    X[5, 1:] *= np.float32(2.0 ** k)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    ref = O.score_logreg(X, xd, t)
    errs = {}
    for gemm in ("h2", "f32"):
        out = torch.zeros(n, p + 1, device=DEV)
        dsvgd().targets.LogisticRegression(xd, t, gemm=gemm).score(gpu(X), out)
        errs[gemm] = row_err(out.cpu().numpy(), ref)
    record_parity(float(errs["h2"].max()), f32=float(errs["f32"].max()), k=k)
    assert errs["h2"].max() <= ROW_TOL, (errs["h2"].max(), int(errs["h2"].argmax()),
                                        errs["f32"].max())
