"""The one-wave-per-SIMD FmtH2 distance Gram (csrc/gram_w1.hpp) through the
engine: the launches it takes (dp % 256 == 0, the none / bracket select modes,
the symmetric layout and row-block rectangles) against the exact f32 Gram on
the same particles, plus the layout invariants the rest of the step relies on
-- exact-zero diagonal, +inf padding, weighted symmetric counting, the
bracket's below / candidate counts and a bit-exact median of the kernel's own
D.  Cases: odd and even 128-tile counts, n off the 128 grid, dp = 256 / 512
(the second one runs K-steps past the epilogue's 16), a 256-aligned row block
(rectangle + mirrored square from the 8-wave kernel) and a 16-aligned one (a
single rectangle)."""
import numpy as np
import pytest
import torch

from conftest import record_parity

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dsvgd():
    import dsvgd as m
    return m


def gpu(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def _block_D(n, d, m, row0, median, X):
    out = {}
    for gemm in ("f32", "h2"):
        eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV, gram_gemm=gemm)
        assert eng.gram_gemm == gemm
        eng.pack(gpu(X))
        if median:
            eng.distances(median=True)
            eng.median_bandwidth()
        else:
            eng.distances(median=False)
        torch.cuda.synchronize()
        out[gemm] = eng
    return out


@pytest.mark.parametrize("n,d,m,row0,median", [
    (4200, 256, None, 0, True),     # symmetric, bracketed, 33 tiles (odd), n off the grid
    (1000, 256, None, 0, False),    # symmetric, no select
    (300, 250, None, 0, False),     # 3 tiles, d off the 256 grid (dp = 256)
    (6000, 512, None, 0, True),     # dp = 512: K-steps 16..31 without epilogue work
    (8192, 256, 4096, 4096, True),  # 256-aligned row block: rectangle + mirrored square
    (8000, 256, 2504, 2496, True),  # 16-aligned row block: one rectangle
    (3000, 256, 1000, 1024, False),  # rectangles left and right of a 256-aligned square
])
def test_gram_w1_matches_f32(n, d, m, row0, median):
    rs = np.random.RandomState(n + d + row0)
    X = (rs.randn(n, d) * 1.5 + 3.0).astype(np.float32)
    eng = _block_D(n, d, m, row0, median, X)
    h2, f32 = eng["h2"], eng["f32"]
    mm = n if m is None else m
    Dh = h2.dense_D(padded=True)
    Df = f32.dense_D(padded=True)
    # padding rows / columns +inf, valid entries finite
    assert bool(torch.isposinf(Dh[mm:, :]).all()) and bool(torch.isposinf(Dh[:, n:]).all())
    D = Dh[:mm, :n].double()
    assert bool(torch.isfinite(D).all())
    # the owned block's diagonal: exactly 0 without the select accounting;
    # with the bracket accounting as computed, a rounding residue of the
    # row's norm (csrc/gram_w1.hpp), below the bracket
    idx = torch.arange(mm, device=DEV)
    Xc = X.astype(np.float64) - X.astype(np.float64).mean(0)
    nrm = torch.as_tensor((Xc ** 2).sum(1), device=DEV)
    diag = D[idx, row0 + idx]
    if median:
        assert bool((diag >= 0).all()) and bool((diag <= 4e-6 * 2 * nrm[row0 + idx]).all())
        if h2.bracketed:
            assert bool((diag < h2.state.bracket()[0]).all())
    else:
        assert bool((diag == 0).all())
    # against the f32 Gram, normalised by the norms of the centred rows
    scale = nrm[row0:row0 + mm, None] + nrm[None, :] + 1e-30
    e = float(((D - Df[:mm, :n].double()).abs() / scale).max())
    record_parity(e)
    assert e < 4e-6, e
    if h2.sym:
        for v in (float(D.median()), 0.5 * float(D.median())):
            assert h2.count_D(lambda t: t < v) == int((Dh < v).sum())
    if median:
        med = h2.state.read()[0]
        if m is None:
            k = (n * n - 1) // 2
            exact = torch.kthvalue(D.flatten().float().cpu(), k + 1).values.item()
            assert np.float32(med).view(np.uint32) == np.float32(exact).view(np.uint32)
        if h2.bracketed:
            lo, hi, below, ncand, fb = h2.state.bracket()
            if m is None and not fb:
                Df32 = D.float()
                assert below == int((Df32 < lo).sum())
                assert ncand == int(((Df32 >= lo) & (Df32 <= hi)).sum())


def test_gram_w1_sharded_counts_sum_to_whole():
    """Two 256-aligned row blocks' bracket counts (below / candidates) add up
    to the whole matrix's: the rectangles (gram_w1) and the mirrored squares
    (8-wave kernel) together cover every entry exactly once."""
    n, d = 8192, 256
    X = np.random.RandomState(11).randn(n, d).astype(np.float32)
    tot = None
    whole = dsvgd().PhiEngine(n, d, device=DEV)
    whole.pack(gpu(X))
    whole.distances(median=True)
    torch.cuda.synchronize()
    lo, hi, below, ncand, _ = whole.state.bracket()
    got = np.zeros(2, np.int64)
    for r in range(2):
        eng = dsvgd().PhiEngine(n, d, m=n // 2, row0=r * n // 2, device=DEV)
        eng.pack(gpu(X))
        eng.distances(median=True)
        from dsvgd import _native as N
        N.call("dsvgd_bracket_totals", eng.state.ptr, N.ptr(eng.cand), N.stream(DEV))
        torch.cuda.synchronize()
        b = eng.state.bracket()
        assert (b[0], b[1]) == (lo, hi)
        got += np.array(b[2:4], np.int64)
    from dsvgd import _native as N
    N.call("dsvgd_bracket_totals", whole.state.ptr, N.ptr(whole.cand), N.stream(DEV))
    torch.cuda.synchronize()
    b = whole.state.bracket()
    assert tuple(got) == (b[2], b[3])


@pytest.mark.parametrize("n,d,m,row0,median", [
    (4200, 256, None, 0, True),     # symmetric, bracketed, ragged n
    (1000, 256, None, 0, False),    # symmetric, no select (the diagonal fix-up)
    (6000, 512, None, 0, True),     # dp = 512: K-steps past the epilogue's 16
    (8192, 256, 4096, 4096, True),  # rectangle + mirrored square
    (8000, 256, 2504, 2496, True),  # 16-aligned row block: one rectangle
    (3000, 256, 1000, 1024, False),  # rectangles either side of the square
    (65536, 256, None, 0, True),    # the headline Gram
])
def test_gram_rs_matches_gram_w1(n, d, m, row0, median):
    """the split-role Gram (gram_rs_kernel: MFMA waves +
    epilogue waves through an LDS hand-off, csrc/gram_rs.hpp) computes the
    same D bits as the one-wave kernel (same fragments, products and order),
    the same bracket counts and the same median; one selected per
    dsvgd_gram_set_rs."""
    from dsvgd import _native as N
    lib = N.load()
    rs = np.random.RandomState(n + d + 7)
    X = gpu((0.1 * rs.randn(n, d)).astype(np.float32))
    out = {}
    prev = lib.dsvgd_gram_set_rs(1)
    try:
        for mode in (1, 0):
            lib.dsvgd_gram_set_rs(mode)
            eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV)
            eng.pack(X)
            if median:
                eng.distances(median=True)
                eng.median_bandwidth()
            else:
                eng.distances(median=False)
            torch.cuda.synchronize()
            # the stored tiles (the symmetric layout's lower ones are never written)
            out[mode] = (eng.dense_D(padded=True).clone(), eng.state.read()[:2] if median else None,
                         eng.state.bracket()[2:4] if median and eng.bracketed else None)
            del eng
            torch.cuda.empty_cache()
    finally:
        lib.dsvgd_gram_set_rs(prev)
    assert torch.equal(out[1][0], out[0][0])
    # (a row block's median needs the other blocks' counts: NaN on both sides)
    assert np.array_equal(np.asarray(out[1][1], np.float64), np.asarray(out[0][1], np.float64),
                          equal_nan=True)
    assert out[1][2] == out[0][2]
