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
    far = np.float32(2.0 ** k * 0.3)
    if kind in ("far", "far_score"):
        X[j, 0] += far                                   # no kernel weight to anyone
    if kind == "far_pair":                               # two of them, opposite sides
        X[j, 0] += far
        X[j + 1, 0] -= far
    if kind in ("score", "far_score", "far_pair"):
        S[j] = S[j] * np.float32(2.0 ** k)
    return X, S


def _phi(X, S, **kw):
    n, d = X.shape
    eng = dsvgd().PhiEngine(n, d, device=DEV, **kw)
    Xo = gpu(X).clone()
    eng.step(gpu(X), gpu(S), X_own=Xo, step=0.0, h=None)
    torch.cuda.synchronize()
    return eng.phi.cpu().numpy(), eng.state.read()[1], eng


KINDS = ("score", "far", "far_score", "far_pair")
CASES = [(kind, k) for kind in KINDS for k in (16, 20, 24, 30)]


@pytest.mark.parametrize("n,d", [(2048, 64), (4096, 256)])
@pytest.mark.parametrize("kind,k", CASES)
def test_phi_row_normalised_with_outlier(n, d, kind, k):
    """One particle (two for far_pair) 2^k away from the rest and / or with
    scores 2^k larger: every row of phi within 1e-5 of fp64, row-normalised,
    on the default engine (the f32 engine beside it for reference).  Far
    particles exercise the robust centre (dsvgd_colcenter) and the per-row
    scales of the Gram's row image; scores 2^k larger the phi_mm range guard."""
    X, S = _outlier_case(n, d, kind, k)
    phi_h2, h, eng = _phi(X, S)
    phi_f32, h32, _ = _phi(X, S, gemm="f32")
    ref = O.phi(X, S, h)
    e_h2, e_f32 = row_err(phi_h2, ref), row_err(phi_f32, O.phi(X, S, h32))
    guard = eng.range_guard()
    record_parity(float(e_h2.max()), f32=float(e_f32.max()), kind=kind, k=k, guard=guard)
    assert e_h2.max() <= ROW_TOL, (e_h2.max(), int(e_h2.argmax()), e_f32.max())
    assert e_f32.max() <= ROW_TOL, e_f32.max()
    if k >= 20:      # rows spanning > 2^16 in a half of [Xc | S]: the step ran on FmtX3
        assert guard is True
    if kind == "far_pair":
        assert h == pytest.approx(h32, rel=1e-5)


@pytest.mark.parametrize("n,d", [(2048, 64), (4096, 256)])
def test_guard_off_for_ordinary_particles(n, d):
    """The guard stays off on the distributions the other tests use."""
    rs = np.random.RandomState(n)
    X = rs.randn(n, d).astype(np.float32)
    S = (-X + 0.3 * rs.randn(n, d)).astype(np.float32)
    _, _, eng = _phi(X, S)
    assert eng.range_guard() is False


def test_guard_path_is_the_x3_phi_mm():
    """With the guard on, KY and the row sums are bit for bit those of the
    FmtX3 phi_mm on the same D (gram_gemm h2 under both)."""
    X, S = _outlier_case(4096, 256, "far_pair", 20)
    _, _, eng = _phi(X, S)
    _, _, eng3 = _phi(X, S, phi_gemm="x3", gram_gemm="h2")
    assert eng.range_guard() is True and eng3.phi_gemm == "x3"
    torch.testing.assert_close(eng.dense_D(), eng3.dense_D(), rtol=0, atol=0)
    assert torch.equal(eng.KY, eng3.KY) and torch.equal(eng.rowsum, eng3.rowsum)


@pytest.mark.parametrize("k", [18, 24, 30])
def test_logreg_scores_row_normalised_with_outlier(k):
    """One particle's w 2^k times the others' (logreg's W image: one FmtH2
    scale per particle row): every particle's score row vs fp64, row-normalised."""
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


@pytest.mark.parametrize("kind,k", [("score", 20), ("far_score", 24), (None, 0)])
def test_unfused_scales_path_has_the_guard(kind, k):
    """d > 1024: pack writes no column maxima, so the scales come from a pass
    over Y (dsvgd_h2_colscale_guarded), which now carries the same range
    guard as the fused path: an outlier trips it, ordinary
    particles do not, and every row stays within 1e-5 row-normalised."""
    n, d = 1024, 1100
    if kind is None:
        rs = np.random.RandomState(3)
        X = (0.3 * rs.randn(n, d)).astype(np.float32)
        S = (-X / 0.09 + rs.randn(n, d)).astype(np.float32)
    else:
        X, S = _outlier_case(n, d, kind, k)
    phi_h2, h, eng = _phi(X, S)
    assert not eng.fused_scales and eng.phi_gemm == "h2"
    e = row_err(phi_h2, O.phi(X, S, h))
    guard = eng.range_guard()
    record_parity(float(e.max()), kind=str(kind), k=k, guard=guard)
    assert guard is (kind is not None)
    assert e.max() <= ROW_TOL, (e.max(), int(e.argmax()))


def test_guard_falls_back_to_f32_when_no_x3_image_fits():
    """roundup(n,128) * ldy * 6 >= 2^31: no FmtX3 image fits its 32-bit
    offsets, so the range guard hands phi_mm to the exact f32 engine
    (dsvgd_phi_mm_gated) instead of letting FmtH2 run out of its window
    (ADVICE r3).  A 256-row block of n = 45056, d = 4096 with one score row
    2^20 larger: sampled rows within 1e-5 row-normalised of fp64."""
    n, d, m, row0 = 45056, 4096, 256, 4096
    X, S = _outlier_case(n, d, "score", 20, seed=5)
    eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV)
    assert eng.Yx3 is None and eng.phi_gemm == "h2" and not eng.sym
    h = 2.0 * d * 0.09
    Xo = gpu(X[row0:row0 + m]).clone()
    eng.step(gpu(X), gpu(S), X_own=Xo, step=0.0, h=h)
    torch.cuda.synchronize()
    assert eng.range_guard() is True
    rows = np.arange(row0, row0 + m, 4)
    ref = O.phi(X, S, h, rows=rows)
    e = row_err(eng.phi.cpu().numpy()[rows - row0], ref)
    record_parity(float(e.max()))
    assert e.max() <= ROW_TOL, (e.max(), int(e.argmax()))
