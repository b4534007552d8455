"""The split MFMA engines against the exact-fp32 MFMA engine and the fp64
oracle: FmtH2 (two fp16 parts of a power-of-two-scaled operand, three
products; the default) and FmtX3 (three bf16 parts, six products), both in
csrc/gemm_x3.hpp.

Claim under test: a split engine carries fp32 GEMM rounding, not its input
format's -- so (1) its images reconstruct every fp32 input (FmtX3 to 2^-24,
FmtH2 to 2^-22 for entries within 2^-18 of their column's largest), (2)
phi_mm's K.[Xc|S] is as close to the fp64 product of the same D as the f32
engine's (within 2x + 1e-7; bf16 alone would be ~2^-9 off, fp16 ~2^-12) and
its row sums match the f32 engine's, (3) the distances and the logreg scores
likewise, and (4) phi through it meets the north_star tolerance (1e-5
max-normalised vs fp64) on the cases the f32 path is tested on.
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
SPLIT = ["h2", "x3"]


def dsvgd():
    import dsvgd as m
    return m


def gpu(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def decode_ysplit(Yx, rows, ldy):
    """CPU inverse of dsvgd_ysplit's (FmtX3) image: (3, rows, ldy) float64 parts."""
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


def decode_h2(img, kdim, xdim):
    """CPU inverse of an FmtH2 image img[kstep][part][x][16 k] (16-B halves
    swapped on x with bit 3 set): (2, kdim, xdim) float64 parts."""
    v = img.cpu().numpy().view(np.float16).astype(np.float64).reshape(kdim // 16, 2, xdim, 2, 8)
    v = np.where(((np.arange(xdim) >> 3) & 1)[None, None, :, None, None] == 1, v[:, :, :, ::-1, :], v)
    return v.reshape(kdim // 16, 2, xdim, 16).transpose(1, 0, 3, 2).reshape(2, kdim, xdim)


@pytest.mark.parametrize("rows,ldy", [(128, 128), (256, 512), (64, 200)])
def test_ysplit_reconstructs_fp32(rows, ldy):
    from dsvgd import _native as N
    rs = np.random.RandomState(rows + ldy)
    Y = (rs.randn(rows, ldy) * np.exp(rs.uniform(-20, 20, (rows, ldy)))).astype(np.float32)
    Y[0, :8] = 0.0
    lib = N.load()
    Yx = torch.empty(lib.dsvgd_ysplit_bytes(rows, ldy) // 2, dtype=torch.int16, device=DEV)
    N.call("dsvgd_ysplit", N.ptr(gpu(Y)), ldy, rows, N.ptr(Yx), 1, None, N.stream(torch.device(DEV)))
    torch.cuda.synchronize()
    parts = decode_ysplit(Yx, rows, ldy)
    rec = parts.sum(0)
    Y64 = Y.astype(np.float64)
    err = np.abs(rec - Y64) / np.maximum(np.abs(Y64), 1e-300)
    record_parity(float(err.max()))
    assert err.max() <= 2.0 ** -24
    # each part is at most half an ulp(bf16) of the remainder before it
    assert np.all(np.abs(parts[1]) <= np.abs(Y64) * 2.0 ** -8 + 1e-300)


@pytest.mark.parametrize("rows,ldy", [(128, 128), (512, 512), (64, 256)])
def test_h2_images_reconstruct_fp32(rows, ldy):
    """dsvgd_h2_colscale + dsvgd_h2_ysplit / dsvgd_h2_rowsplit: power-of-two
    scales putting each column's (tensor's) largest magnitude in [2^14, 2^15),
    parts that sum back to s v within 2^-22 relative for entries within 2^-16
    of the scale's reference magnitude (2^-22 relative + 2^-38 of it for all),
    zero / inf / NaN columns handled."""
    from dsvgd import _native as N
    lib = N.load()
    s = N.stream(torch.device(DEV))
    rs = np.random.RandomState(rows + ldy)
    colmag = np.exp(rs.uniform(-12, 12, ldy))
    Y = (rs.randn(rows, ldy) * colmag).astype(np.float32)
    Y[:, 3] = 0.0                                   # all-zero column: scale 1
    Yg = gpu(Y)
    ws = torch.empty(lib.dsvgd_h2_colscale_workspace_floats(rows, ldy), device=DEV)
    sc = torch.empty(2 * ldy + 3, device=DEV)
    N.call("dsvgd_h2_colscale", N.ptr(Yg), ldy, rows, ldy, N.ptr(ws), N.ptr(sc), s)
    img = torch.empty(lib.dsvgd_h2_image_bytes(rows, ldy) // 2, dtype=torch.int16, device=DEV)
    N.call("dsvgd_h2_ysplit", N.ptr(Yg), ldy, rows, N.ptr(sc), N.ptr(img), s)
    torch.cuda.synchronize()
    scale = sc.cpu().numpy().astype(np.float64)
    s_c = scale[:ldy]
    mx = np.abs(Y).max(0).astype(np.float64)
    live = mx > 0
    assert np.all(np.log2(s_c) == np.round(np.log2(s_c)))           # powers of two
    assert np.all((s_c * mx)[live] >= 2.0 ** 14) and np.all((s_c * mx)[live] < 2.0 ** 15)
    assert s_c[3] == 1.0 and np.all(scale[ldy:2 * ldy] * s_c == 1.0)
    assert scale[2 * ldy] == s_c[live].min() and scale[2 * ldy + 1] * scale[2 * ldy] == 1.0
    assert scale[2 * ldy + 2] == 0.0      # no range guard on the colscale path
    parts = decode_h2(img, rows, ldy)
    rec = parts.sum(0) / s_c[None, :]
    Y64 = Y.astype(np.float64)
    # the second part is exact to 2^-11 of itself while normal (|s v| >= 2^-3
    # keeps 2^-22 |s v| above fp16's subnormal half-spacing 2^-25)
    big = (np.abs(Y64) >= mx[None, :] * 2.0 ** -16) & (Y64 != 0)
    err = np.abs(rec - Y64)[big] / np.abs(Y64)[big]
    record_parity(float(err.max()))
    assert err.max() <= 2.0 ** -22
    assert np.all(np.abs(rec - Y64) <= 2.0 ** -22 * np.abs(Y64) + 2.0 ** -38 * mx[None, :])
    # the row image of the same tensor with its tensor scale
    t = sc[2 * ldy:2 * ldy + 1]
    img2 = torch.empty(lib.dsvgd_h2_image_bytes(rows + 16, ldy) // 2, dtype=torch.int16, device=DEV)
    N.call("dsvgd_h2_rowsplit", N.ptr(Yg), ldy, rows, ldy, rows + 16, ldy, N.ptr(t),
           N.ptr(img2), s)
    torch.cuda.synchronize()
    rp = decode_h2(img2, ldy, rows + 16)                       # (2, k, row)
    rec2 = rp.sum(0).T / scale[2 * ldy]
    assert np.all(rec2[rows:] == 0.0)
    tb = (np.abs(Y64) >= np.abs(Y64).max() * 2.0 ** -16) & (Y64 != 0)
    assert np.all(np.abs(rec2[:rows] - Y64)[tb] <= 2.0 ** -22 * np.abs(Y64)[tb])
    assert np.all(np.abs(rec2[:rows] - Y64) <= 2.0 ** -22 * np.abs(Y64) + 2.0 ** -38 * np.abs(Y64).max())
    # a non-finite column forces the tensor scale to 1 (inf / NaN propagate)
    Y[5, 7] = np.inf
    N.call("dsvgd_h2_colscale", N.ptr(gpu(Y)), ldy, rows, ldy, N.ptr(ws), N.ptr(sc), s)
    torch.cuda.synchronize()
    assert float(sc[7]) == 1.0 and float(sc[2 * ldy]) == 1.0


def _pow2_scale(m):
    """numpy restatement of pow2_scale (csrc/common.hpp)."""
    m = np.asarray(m, np.float64)
    out = np.ones_like(m)
    ok = (m > 0) & np.isfinite(m)
    e = np.frexp(m[ok])[1]
    out[ok] = np.ldexp(1.0, np.minimum(15 - e, 100))
    return out


@pytest.mark.parametrize("n,d,ldx,special", [(1000, 64, 64, None), (777, 100, 101, "zero"),
                                             (300, 3, 3, "inf"), (2100, 1024, 1024, "nan"),
                                             (129, 250, 252, None), (1000, 64, 64, "range")])
def test_pack_maxima_match_colscale(n, d, ldx, special):
    """dsvgd_pack_h2 (pack + the FmtH2 statistics) then dsvgd_h2_scales:
    Y / norms as the numpy restatement of dsvgd_pack, scales bit-identical to
    dsvgd_h2_colscale's over the same Y -- after pack(X, S), and after pack(X)
    + pack(NULL, S) (the scores arriving after the distance stage); zero and
    non-finite columns; unaligned row strides (element-load path); the per-row
    scales of the X half; the range guard word against its numpy restatement
    (largest |entry| of a half > 2^16 x its smallest nonzero row max)."""
    from dsvgd import _native as N
    lib = N.load()
    s = N.stream(torch.device(DEV))
    rs = np.random.RandomState(n + d)
    X = (rs.randn(n, ldx) * np.exp(rs.uniform(-6, 6, ldx))).astype(np.float32)
    S = (rs.randn(n, ldx) * np.exp(rs.uniform(-6, 6, ldx))).astype(np.float32)
    if special == "zero":
        X[:, 5] = 1.25                                # centred: an all-zero column
        S[:, 9] = 0.0
    elif special == "range":                          # one particle's scores 2^20 x
        X = (rs.randn(n, ldx)).astype(np.float32)
        S = (rs.randn(n, ldx)).astype(np.float32)
        S[11] *= np.float32(2.0 ** 20)
    elif special == "inf":
        S[7, 1] = np.inf
    elif special == "nan":
        X[3, 600] = np.nan
    dp, n_pad = lib.dsvgd_dp(d), lib.dsvgd_pad128(n)
    ldy = lib.dsvgd_ldy(dp)
    rows = n_pad + 128
    nb = lib.dsvgd_pack_blocks(rows)
    Xg, Sg = gpu(X)[:, :d], gpu(S)[:, :d]
    mean = torch.empty(d, device=DEV)
    N.call("dsvgd_colcenter", N.ptr(Xg), ldx, n, d, N.ptr(mean), s)
    ws = torch.empty(lib.dsvgd_h2_colscale_workspace_floats(n_pad, ldy), device=DEV)
    for split_scores in (False, True):
        Y = torch.full((rows, ldy), 7.0, device=DEV)  # every entry must be written
        norms = torch.empty(rows, device=DEV)
        part = torch.full((nb * ldy,), -1, dtype=torch.int32, device=DEV)
        gmax = torch.full((4 * nb,), -1, dtype=torch.int32, device=DEV)
        rsc = torch.full((rows,), -1.0, device=DEV)
        args = (N.ptr(mean), n, d, rows, N.ptr(Y), ldy)
        if split_scores:
            N.call("dsvgd_pack_h2", N.ptr(Xg), ldx, None, d, 1.0, *args, N.ptr(norms),
                   N.ptr(part), N.ptr(gmax), N.ptr(rsc), s)
            N.call("dsvgd_pack_h2", None, d, N.ptr(Sg), ldx, 0.5, *args, None,
                   N.ptr(part), N.ptr(gmax), None, s)
        else:
            N.call("dsvgd_pack_h2", N.ptr(Xg), ldx, N.ptr(Sg), ldx, 0.5, *args, N.ptr(norms),
                   N.ptr(part), N.ptr(gmax), N.ptr(rsc), s)
        got = {}
        for cols in (dp, ldy):
            ref = torch.empty(2 * cols + 3, device=DEV)
            out = torch.empty(2 * cols + 3, device=DEV)
            N.call("dsvgd_h2_colscale", N.ptr(Y), ldy, n_pad, cols, N.ptr(ws), N.ptr(ref), s)
            N.call("dsvgd_h2_scales", N.ptr(part), N.ptr(gmax), nb, ldy, cols, dp, N.ptr(out), s)
            got[cols] = (ref, out)
        torch.cuda.synchronize()
        Yc = Y.cpu().numpy()
        mc = mean.cpu().numpy()
        exp = np.zeros((rows, ldy), np.float32)
        exp[:n, :d] = X[:, :d] - mc[None, :]
        exp[:n, dp:dp + d] = np.float32(0.5) * S[:, :d]
        np.testing.assert_array_equal(Yc, exp)
        nr = (exp[:, :d].astype(np.float64) ** 2).sum(1)
        got_n = norms.cpu().numpy()
        fin = np.isfinite(nr)
        np.testing.assert_allclose(got_n[fin], nr[fin], rtol=1e-5, atol=1e-30)
        assert np.all(got_n[rows - 128:] == 0.0)
        Y64 = np.abs(Yc[:n].astype(np.float64))
        with np.errstate(invalid="ignore"):
            rx, rs_ = Y64[:, :dp].max(1), Y64[:, dp:].max(1)
        np.testing.assert_array_equal(rsc.cpu().numpy()[:n], _pow2_scale(rx).astype(np.float32))
        assert np.all(rsc.cpu().numpy()[n:] == 1.0)

        def wide(r):
            r = r[np.isfinite(r) | np.isnan(r)]
            nz = r[r > 0]
            return bool(nz.size and np.nanmax(r) > 2.0 ** 16 * nz.min())
        for cols, (ref, out) in got.items():
            o = out.cpu().numpy()
            np.testing.assert_array_equal(o[:2 * cols + 2].view(np.uint32),
                                          ref.cpu().numpy()[:2 * cols + 2].view(np.uint32))
            if special in ("inf", "nan"):
                continue
            expect = wide(rx) or (cols > dp and wide(rs_))
            assert o[2 * cols + 2] == (1.0 if expect else 0.0), (cols, o[2 * cols + 2])
            if special == "range":
                assert o[2 * cols + 2] == (1.0 if cols > dp else 0.0)


def _engines(X, S, h, split, m=None, row0=0):
    """phi and the raw (KY, rowsum) of one step through the f32 engine and `split`."""
    out = {}
    for gemm in ("f32", split):
        n, d = X.shape
        # the same (split) Gram under both: phi_mm compared on identical D
        eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV, phi_gemm=gemm, gram_gemm=split)
        assert eng.phi_gemm == gemm
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
        out[gemm] = (eng.phi.cpu().numpy(), KY, r, eng.state.read()[1], eng)
    # the exact K.[Xc|S] of the split engine's own D (fp64), diagonal left out like phi_mm
    eng = out[split][4]
    D = eng.dense_D().double()
    K = torch.exp(-D / out[split][3])
    rows = torch.arange(eng.m, device=DEV)
    K[rows, rows + row0] = 0.0
    Y = eng.Y[:n].double()
    out["exact"] = ((K @ Y).cpu().numpy(), K.sum(1).cpu().numpy())
    return out


def _ky_errors(res, split):
    """max-normalised error of each engine's KY against the fp64 product."""
    KY64 = res["exact"][0]
    scale = np.abs(KY64).max()
    return {g: float(np.abs(res[g][1] - KY64).max() / scale) for g in ("f32", split)}


@pytest.mark.parametrize("split", SPLIT)
@pytest.mark.parametrize("n,d,h", [(300, 20, 5.0), (1000, 64, None), (2048, 256, None),
                                   (513, 100, 40.0), (4096, 3, None), (1500, 1024, None),
                                   (777, 500, None), (700, 1100, None)])
def test_phi_mm_split_matches_f32_engine_and_oracle(split, n, d, h):
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d).astype(np.float32)
    S = (-X + 0.3 * rs.randn(n, d)).astype(np.float32)
    res = _engines(X, S, h, split)
    phix, KYx, rx, hx, _ = res[split]
    assert res["f32"][3] == hx
    e = _ky_errors(res, split)
    record_parity(e[split])
    assert e[split] <= 2.0 * e["f32"] + 1e-7 and e[split] < KY_TOL, e
    e_r = float(np.abs(rx - res["exact"][1]).max() / np.abs(res["exact"][1]).max())
    assert e_r < 1e-6
    ref = O.phi(X, S, hx)
    e_phi = float(np.abs(phix - ref).max() / np.abs(ref).max())
    record_parity(e_phi)
    assert e_phi < PHI_TOL


@pytest.mark.parametrize("split", SPLIT)
def test_phi_mm_split_row_block_split_k(split):
    """A DistSampler rank's block (m < n, row0 > 0): diagonal offset, split-K."""
    n, d, m, row0 = 4096, 128, 1024, 2048
    rs = np.random.RandomState(11)
    X = rs.randn(n, d).astype(np.float32)
    S = rs.randn(n, d).astype(np.float32)
    res = _engines(X, S, 30.0, split, m=m, row0=row0)
    phix = res[split][0]
    e = _ky_errors(res, split)
    assert e[split] <= 2.0 * e["f32"] + 1e-7 and e[split] < KY_TOL, e
    ref = O.phi(X, S, 30.0, rows=np.arange(row0, row0 + m))
    e = float(np.abs(phix - ref).max() / np.abs(ref).max())
    record_parity(e)
    assert e < PHI_TOL


def test_phi_mm_h2_wide_column_range():
    """FmtH2's per-column scales: scores 1e4 x larger than the particles (one
    tensor scale would leave Xc's columns with ~2^-4 of fp16's precision)."""
    n, d = 2048, 64
    rs = np.random.RandomState(12)
    X = (1e-3 * rs.randn(n, d)).astype(np.float32)
    S = (10.0 * rs.randn(n, d)).astype(np.float32)
    res = _engines(X, S, None, "h2")
    e = _ky_errors(res, "h2")
    assert e["h2"] < KY_TOL, e
    ref = O.phi(X, S, res["h2"][3])
    e_phi = float(np.abs(res["h2"][0] - ref).max() / np.abs(ref).max())
    record_parity(e_phi)
    assert e_phi < PHI_TOL


@pytest.mark.parametrize("split", SPLIT)
@pytest.mark.parametrize("n,N,p", [(1000, 3000, 20), (512, 16384, 255), (300, 129, 40),
                                   (600, 2000, 1023), (257, 700, 511), (1000, 1000, 255)])
def test_logreg_scores_split_as_accurate_as_f32(split, n, N, p):
    """The logreg score GEMMs (Z = W Xd^T on the split NT engine, G Xd on the
    split NN engine without exp) against the fp64 oracle, next to the f32 MFMA
    engines on the same inputs."""
    rs = np.random.RandomState(n + N + p)
    X = (rs.randn(n, p + 1) * 0.5).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    ref = O.score_logreg(X, xd, t)
    err = {}
    for gemm in ("f32", split):
        tgt = dsvgd().targets.LogisticRegression(xd, t, gemm=gemm)
        out = torch.zeros(n, p + 1, device=DEV)
        tgt.score(gpu(X), out)
        err[gemm] = float(np.abs(out.cpu().numpy() - ref).max() / np.abs(ref).max())
    record_parity(err[split])
    assert err[split] <= 2.0 * err["f32"] + 1e-7 and err[split] < 1e-5, err


@pytest.mark.parametrize("split", SPLIT)
@pytest.mark.parametrize("n,d,m,row0", [(700, 48, None, 0), (5000, 64, None, 0),
                                        (3000, 130, 1000, 1500), (513, 3, None, 0),
                                        (1000, 100, None, 0), (1900, 256, None, 0),
                                        (4500, 128, None, 0), (3000, 130, 1024, 1024),
                                        (2300, 96, 1280, 0), (2600, 64, 512, 2048)])
def test_sqdist_split_as_accurate_as_f32(split, n, d, m, row0):
    """Distances through the split Gram against fp64, next to the f32 Gram on
    the same particles: symmetric, bracketed (n = 5000: n^2 >= 2^24) and
    row-block launches; the median select stays bit-exact on the kernel's
    own D."""
    rs = np.random.RandomState(n + d)
    X = (rs.randn(n, d) * 1.5 + 3.0).astype(np.float32)
    Xc = X.astype(np.float64) - X.astype(np.float64).mean(0)
    mm = n if m is None else m
    ref = ((Xc[row0:row0 + mm, None, :] - Xc[None, :, :]) ** 2).sum(-1) if n * mm <= 4e6 else None
    nrm = (Xc ** 2).sum(1)
    err, med, Dall = {}, {}, {}
    for gemm in ("f32", split):
        eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV, gram_gemm=gemm)
        assert eng.gram_gemm == gemm
        eng.pack(gpu(X))
        eng.distances(median=True)
        eng.median_bandwidth()
        Dm = eng.dense_D().cpu().numpy().astype(np.float64)
        k = (n * mm - 1) // 2
        med[gemm] = eng.state.read()[0]
        # symmetric layout exactly when the split engines take the whole matrix at ldy % 256 == 0
        assert eng.sym == (gemm != "f32" and m is None and d > 2 and eng.ldy % 256 == 0)
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
        record_parity(err[split])
        assert err[split] <= 2.0 * err["f32"] + 1e-7 and err[split] < 2e-6, err
    # every entry of the block, incl. the mirrored / square-split ones of a
    # 256-aligned row block, against the f32 Gram's
    scale = nrm[row0:row0 + mm, None] + nrm[None, :] + 1e-30
    e = float(np.max(np.abs(Dall[split] - Dall["f32"]) / scale))
    record_parity(e)
    assert e < 4e-6


@pytest.mark.parametrize("n,N", [(1000, 1000), (200, 33), (4096, 8192)])
def test_logreg_scores_general_labels(n, N):
    """Labels that are not +-1 (logreg_prepare folds t into the data:
    t sigma(-t z) xd = sigma(-z') xd' with z' = t z, so the FmtH2 image of G
    holds 2^15 sigma in (0, 2^15) whatever |t| -- unfolded, |t| > 2 overflowed
    fp16), particle and data counts off the tiles, at p = 255, against fp64
    and next to the f32 engine."""
    p = 255
    rs = np.random.RandomState(n + 7 * N)
    X = (rs.randn(n, p + 1) * 0.3).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = rs.uniform(-3.0, 3.0, N).astype(np.float32)
    ref = O.score_logreg(X, xd, t)
    err = {}
    for gemm in ("f32", "h2"):
        out = torch.zeros(n, p + 1, device=DEV)
        dsvgd().targets.LogisticRegression(xd, t, gemm=gemm).score(gpu(X), out)
        err[gemm] = float(np.abs(out.cpu().numpy() - ref).max() / np.abs(ref).max())
    record_parity(err["h2"], f32=err["f32"])
    assert err["h2"] <= 2.0 * err["f32"] + 1e-7 and err["h2"] < 1e-5, err


@pytest.mark.parametrize("n,d,ties", [(65536, 256, False), (1000, 7, False), (4099, 33, True),
                                      (3, 5, True)])
def test_colcenter_is_the_lower_median_of_its_sample(n, d, ties):
    """dsvgd_colcenter: per column the lower median of min(n, 1024) evenly
    spaced rows (row k n / m) -- value-exact against numpy on the same
    sample, ties (repeated values, signed zeros) included."""
    from dsvgd import _native as N
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d).astype(np.float32)
    if ties:
        X = np.round(X * 2.0).astype(np.float32) / 2.0   # few distinct values, zeros of both signs
        X[::3, 0] = -0.0
    Xg = gpu(X)
    mean = torch.full((d,), np.nan, device=DEV)
    N.call("dsvgd_colcenter", N.ptr(Xg), d, n, d, N.ptr(mean), N.stream(0))
    torch.cuda.synchronize()
    m = min(n, 1024)
    rows = (np.arange(m, dtype=np.int64) * n) // m
    want = np.sort(X[rows], axis=0, kind="stable")[(m - 1) // 2]
    got = mean.cpu().numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)


@pytest.mark.parametrize("n,p,off", [(65536, 255, 1), (1000, 100, 1), (300, 64, 0), (17, 1023, 3)])
def test_rowimage_equals_rowscale_then_rowsplit(n, p, off):
    """dsvgd_h2_rowimage (the logreg W image in one pass) gives the same bits
    as dsvgd_h2_rowscale + dsvgd_h2_rowsplit_rows: scales, inverses, image."""
    from dsvgd import _native as N
    lib = N.load()
    rs = np.random.RandomState(n + p)
    ld = off + p + 5
    X = rs.randn(n, ld).astype(np.float32) * np.exp2(rs.randint(-20, 20, size=(n, 1))).astype(np.float32)
    X[min(5, n - 1)] = 0.0      # a zero row: scale 1
    Xg = gpu(X)
    rows_pad = -(-n // 256) * 256
    kpad = -(-p // 32) * 32
    nb = lib.dsvgd_h2_image_bytes(rows_pad, kpad)
    out = []
    for fused in (False, True):
        sc = torch.full((rows_pad,), -1.0, device=DEV)
        inv = torch.full((rows_pad,), -1.0, device=DEV)
        img = torch.full((nb // 2,), 7, dtype=torch.int16, device=DEV)
        A = N.ptr(Xg) + 4 * off
        if fused:
            N.call("dsvgd_h2_rowimage", A, ld, n, p, rows_pad, kpad, N.ptr(sc), N.ptr(inv),
                   N.ptr(img), N.stream(0))
        else:
            N.call("dsvgd_h2_rowscale", A, ld, n, p, rows_pad, N.ptr(sc), N.ptr(inv), N.stream(0))
            N.call("dsvgd_h2_rowsplit_rows", A, ld, n, p, rows_pad, kpad, N.ptr(sc), N.ptr(img),
                   N.stream(0))
        torch.cuda.synchronize()
        out.append((sc.cpu().numpy(), inv.cpu().numpy(), img.cpu().numpy()))
    for a, b in zip(*out):
        assert np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                              b.view(np.uint32) if b.dtype == np.float32 else b)


@pytest.mark.parametrize("n,N,labels", [(512, 16384, "pm1"), (1000, 1000, "pm1"), (4096, 8192, "general"),
                                        (300, 129, "general"), (65536, 2048, "pm1")])
def test_logreg_scores_fused(n, N, labels):
    """The fused FmtH2 score (dsvgd_logreg_set_fused: Z, sigma and G . Xd in
    one kernel, G in registers, the column image K-permuted) at p = 255
    against fp64 and next to the two-GEMM path on the same inputs: particle
    and data counts off the tiles (padding rows on both sides), +-1 and
    general labels."""
    from dsvgd import _native as N_
    p = 255
    rs = np.random.RandomState(n + 3 * N)
    X = (rs.randn(n, p + 1) * 0.4).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = (np.where(rs.randn(N) > 0, 1.0, -1.0) if labels == "pm1"
         else rs.uniform(-3.0, 3.0, N)).astype(np.float32)
    lib = N_.load()
    out = {}
    for fused in (1, 0):
        prev = lib.dsvgd_logreg_set_fused(fused)
        try:
            o = torch.zeros(n, p + 1, device=DEV)
            dsvgd().targets.LogisticRegression(xd, t, gemm="h2").score(gpu(X), o)
            torch.cuda.synchronize()
            out[fused] = o.cpu().numpy()
        finally:
            lib.dsvgd_logreg_set_fused(prev)
    scale = None
    if n * N <= 2 ** 27:
        ref = O.score_logreg(X, xd, t)
        scale = np.abs(ref).max()
        e_f = float(np.abs(out[1] - ref).max() / scale)
        e_2 = float(np.abs(out[0] - ref).max() / scale)
        record_parity(e_f, two_gemm=e_2)
        assert e_f < 1e-5 and e_f <= 2.0 * e_2 + 1e-7, (e_f, e_2)
    d = float(np.abs(out[1] - out[0]).max() / np.abs(out[0]).max())
    assert d < 5e-6, d


@pytest.mark.parametrize("n,N,S,fused", [(512, 16384, 8, 1), (1000, 3000, 4, 1), (300, 700, 2, 0)])
def test_logreg_scores_prior_weight(n, N, S, fused):
    """dsvgd_score_logreg_prior: the prior terms weighted by S -- what the
    reference's all_scores all-reduce of S per-rank logp gradients sums to
    (distsampler.py:160-170) -- against fp64 (data term + S x prior), and
    weight 1 bit-identical to dsvgd_score_logreg_prepared."""
    from dsvgd import _native as N_
    p = 255
    rs = np.random.RandomState(n + N + S)
    X = (rs.randn(n, p + 1) * 0.4).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    lib = N_.load()
    prev = lib.dsvgd_logreg_set_fused(fused)
    try:
        tg = dsvgd().targets.LogisticRegression(xd, t, gemm="h2")
        o1, ow, op = (torch.zeros(n, p + 1, device=DEV) for _ in range(3))
        tg.score(gpu(X), o1)
        tg.score(gpu(X), op, prior_weight=1.0 + 0.0 * S)      # the plain path
        tg.score(gpu(X), ow, prior_weight=float(S))
        torch.cuda.synchronize()
    finally:
        lib.dsvgd_logreg_set_fused(prev)
    np.testing.assert_array_equal(o1.cpu().numpy(), op.cpu().numpy())
    ref = O.score_logreg(X, xd, t)
    prior = O.score_logreg(X, xd[:0], t[:0])              # no data: the prior terms alone
    ref = ref + (S - 1) * prior
    err = float(np.abs(ow.cpu().numpy() - ref).max() / np.abs(ref).max())
    record_parity(err)
    assert err < 1e-5, err
