"""The bf16-split phi_mm engine (csrc/gemm_x3.hpp) against the exact-fp32 MFMA
engine and the fp64 oracle.

Claim under test: the 3-way bf16 split with the six i + j <= 2 products
carries fp32 GEMM rounding, not bf16's -- so (1) the split reconstructs every
fp32 input to within 2^-24 relative, (2) phi_mm_x3's K.[Xc|S] is as close to
the fp64 product of the same D as the f32 engine's (within 2x + 1e-7; bf16
alone would be ~2^-9 off) and its row sums match the f32 engine's, and (3) phi through it meets the north_star tolerance
(1e-5 max-normalised vs fp64) on the same cases the f32 path is tested on.
"""
import numpy as np
import pytest
import torch

from conftest import record_parity
from oracle import svgd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PHI_TOL = 1e-5
KY_TOL = 5e-6


def dsvgd():
    import dsvgd as m
    return m


def gpu(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def decode_ysplit(Yx, rows, ldy):
    """CPU inverse of dsvgd_ysplit's image: (3, rows, ldy) float64 parts."""
    raw = Yx.cpu().numpy().view(np.uint16).astype(np.uint32) << 16
    v = raw.view(np.float32).astype(np.float64).reshape(rows // 16, 3, ldy, 2, 8)
    sw = (np.arange(ldy) >> 3) & 1
    out = np.empty((3, rows, ldy))
    for c in range(ldy):
        halves = v[:, :, c, :, :]
        if sw[c]:
            halves = halves[:, :, ::-1, :]
        out[:, :, c] = halves.reshape(rows // 16, 3, 16).transpose(1, 0, 2).reshape(3, rows)
    return out


@pytest.mark.parametrize("rows,ldy", [(128, 128), (256, 512), (64, 200)])
def test_ysplit_reconstructs_fp32(rows, ldy):
    from dsvgd import _native as N
    rs = np.random.RandomState(rows + ldy)
    Y = (rs.randn(rows, ldy) * np.exp(rs.uniform(-20, 20, (rows, ldy)))).astype(np.float32)
    Y[0, :8] = 0.0
    lib = N.load()
    Yx = torch.empty(lib.dsvgd_ysplit_bytes(rows, ldy) // 2, dtype=torch.int16, device=DEV)
    N.call("dsvgd_ysplit", N.ptr(gpu(Y)), ldy, rows, N.ptr(Yx), 1, N.stream(torch.device(DEV)))
    torch.cuda.synchronize()
    parts = decode_ysplit(Yx, rows, ldy)
    rec = parts.sum(0)
    Y64 = Y.astype(np.float64)
    err = np.abs(rec - Y64) / np.maximum(np.abs(Y64), 1e-300)
    record_parity(float(err.max()))
    assert err.max() <= 2.0 ** -24
    # each part is at most half an ulp(bf16) of the remainder before it
    assert np.all(np.abs(parts[1]) <= np.abs(Y64) * 2.0 ** -8 + 1e-300)


def _both_engines(monkeypatch, X, S, h, m=None, row0=0):
    """phi and the raw (KY, rowsum) of one step through each engine."""
    out = {}
    for gemm in ("f32", "x3"):
        monkeypatch.setenv("DSVGD_PHI_GEMM", gemm)
        n, d = X.shape
        eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV)
        assert eng.x3 == (gemm == "x3")
        Xo = gpu(X[row0:row0 + eng.m]).clone()
        eng.pack(gpu(X), gpu(S))
        eng.distances(median=h is None)
        if h is None:
            eng.median_bandwidth()
        else:
            eng.fixed_bandwidth(h)
        eng.direction(Xo, 0.0)
        torch.cuda.synchronize()
        KY = eng.KY.view(eng.splits, eng.m, eng.ldy).double().sum(0).cpu().numpy()
        r = eng.rowsum.view(eng.splits, eng.m_pad)[:, :eng.m].double().sum(0).cpu().numpy()
        out[gemm] = (eng.phi.cpu().numpy(), KY, r, eng.state.read()[1])
    # the exact K.[Xc|S] of this D (fp64), diagonal left out like phi_mm
    D = eng.dense_D().double()
    K = torch.exp(-D / out["x3"][3])
    rows = torch.arange(eng.m, device=DEV)
    K[rows, rows + row0] = 0.0
    Y = eng.Y[:n].double()
    out["exact"] = ((K @ Y).cpu().numpy(), K.sum(1).cpu().numpy())
    return out


def _ky_errors(res):
    """max-normalised error of each engine's KY against the fp64 product."""
    KY64 = res["exact"][0]
    scale = np.abs(KY64).max()
    return {g: float(np.abs(res[g][1] - KY64).max() / scale) for g in ("f32", "x3")}


@pytest.mark.parametrize("n,d,h", [(300, 20, 5.0), (1000, 64, None), (2048, 256, None),
                                   (513, 100, 40.0), (4096, 3, None), (1500, 1024, None),
                                   (777, 500, None)])
def test_phi_mm_x3_matches_f32_engine_and_oracle(monkeypatch, n, d, h):
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d).astype(np.float32)
    S = (-X + 0.3 * rs.randn(n, d)).astype(np.float32)
    res = _both_engines(monkeypatch, X, S, h)
    phi32, KY32, r32, h32 = res["f32"]
    phix, KYx, rx, hx = res["x3"]
    assert h32 == hx
    # the split engine is as accurate as the fp32 one (bf16 alone: ~2^-9)
    e = _ky_errors(res)
    record_parity(e["x3"])
    assert e["x3"] <= 2.0 * e["f32"] + 1e-7 and e["x3"] < KY_TOL, e
    e_r = float(np.abs(rx - r32).max() / np.abs(r32).max())
    assert e_r < 1e-6
    ref = O.phi(X, S, hx)
    e_phi = float(np.abs(phix - ref).max() / np.abs(ref).max())
    record_parity(e_phi)
    assert e_phi < PHI_TOL


def test_phi_mm_x3_row_block_split_k(monkeypatch):
    """A DistSampler rank's block (m < n, row0 > 0): diagonal offset, split-K."""
    n, d, m, row0 = 4096, 128, 1024, 2048
    rs = np.random.RandomState(11)
    X = rs.randn(n, d).astype(np.float32)
    S = rs.randn(n, d).astype(np.float32)
    res = _both_engines(monkeypatch, X, S, 30.0, m=m, row0=row0)
    phix = res["x3"][0]
    e = _ky_errors(res)
    assert e["x3"] <= 2.0 * e["f32"] + 1e-7 and e["x3"] < KY_TOL, e
    ref = O.phi(X, S, 30.0, rows=np.arange(row0, row0 + m))
    e = float(np.abs(phix - ref).max() / np.abs(ref).max())
    record_parity(e)
    assert e < PHI_TOL


@pytest.mark.parametrize("n,N,p", [(1000, 3000, 20), (512, 16384, 255), (300, 129, 40),
                                   (600, 2000, 1023), (257, 700, 511)])
def test_logreg_scores_x3_as_accurate_as_f32(monkeypatch, n, N, p):
    """The logreg score GEMMs (Z = W Xd^T on the split NT engine, G Xd on
    the split NN engine without exp) against the fp64 oracle, next to the
    f32 MFMA engines on the same inputs."""
    rs = np.random.RandomState(n + N + p)
    X = (rs.randn(n, p + 1) * 0.5).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    tgt = dsvgd().targets.LogisticRegression(xd, t)
    ref = O.score_logreg(X, xd, t)
    err = {}
    for gemm in ("f32", "x3"):
        monkeypatch.setenv("DSVGD_LOGREG_GEMM", gemm)
        out = torch.zeros(n, p + 1, device=DEV)
        tgt.score(gpu(X), out)
        err[gemm] = float(np.abs(out.cpu().numpy() - ref).max() / np.abs(ref).max())
    record_parity(err["x3"])
    assert err["x3"] <= 2.0 * err["f32"] + 1e-7 and err["x3"] < 1e-5, err


@pytest.mark.parametrize("n,d,m,row0", [(700, 48, None, 0), (5000, 64, None, 0),
                                        (3000, 130, 1000, 1500), (513, 3, None, 0),
                                        (1000, 100, None, 0), (1900, 256, None, 0),
                                        (4500, 128, None, 0), (3000, 130, 1024, 1024),
                                        (2300, 96, 1280, 0), (2600, 64, 512, 2048)])
def test_sqdist_x3_as_accurate_as_f32(monkeypatch, n, d, m, row0):
    """Distances through the split Gram (dsvgd_sqdist_x3) against fp64, next
    to the f32 Gram on the same particles: symmetric, bracketed (n = 5000:
    n^2 >= 2^24) and row-block launches; the median select stays bit-exact
    on the kernel's own D."""
    rs = np.random.RandomState(n + d)
    X = (rs.randn(n, d) * 1.5 + 3.0).astype(np.float32)
    Xc = X.astype(np.float64) - X.astype(np.float64).mean(0)
    mm = n if m is None else m
    ref = ((Xc[row0:row0 + mm, None, :] - Xc[None, :, :]) ** 2).sum(-1) if n * mm <= 4e6 else None
    nrm = (Xc ** 2).sum(1)
    err, med, Dall = {}, {}, {}
    for gemm in ("f32", "x3"):
        monkeypatch.setenv("DSVGD_GRAM_GEMM", gemm)
        eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV)
        assert eng.x3_gram == (gemm == "x3")
        eng.pack(gpu(X))
        eng.distances(median=True)
        eng.median_bandwidth()
        Dm = eng.dense_D().cpu().numpy().astype(np.float64)
        k = (n * mm - 1) // 2
        med[gemm] = eng.state.read()[0]
        # symmetric layout exactly when the split engines take the whole matrix at ldy % 256 == 0
        assert eng.sym == (gemm == "x3" and m is None and d > 2 and eng.ldy % 256 == 0)
        if eng.sym:  # weighted counting over the stored tiles == counting the dense matrix
            for v in (med[gemm], 0.5 * med[gemm]):
                assert eng.count_D(lambda t: t < v) == int((eng.dense_D(padded=True) < v).sum())
        if m is None:
            assert np.float32(med[gemm]).view(np.uint32) == \
                np.float32(np.partition(Dm.ravel(), k)[k]).view(np.uint32)
            assert np.all(np.diag(Dm) == 0.0)
        if ref is not None:
            scale = nrm[row0:row0 + mm, None] + nrm[None, :] + 1e-30
            err[gemm] = float(np.max(np.abs(Dm - ref) / scale))
        Dall[gemm] = Dm
    if ref is not None:
        record_parity(err["x3"])
        assert err["x3"] <= 2.0 * err["f32"] + 1e-7 and err["x3"] < 2e-6, err
    # every entry of the block, incl. the mirrored / square-split ones of a
    # 256-aligned row block, against the f32 Gram's
    scale = nrm[row0:row0 + mm, None] + nrm[None, :] + 1e-30
    e = float(np.max(np.abs(Dall["x3"] - Dall["f32"]) / scale))
    record_parity(e)
    assert e < 4e-6
