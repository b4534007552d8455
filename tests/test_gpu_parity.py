"""GPU parity tests: the gfx950 kernels (through the C ABI / dsvgd API) against
the CPU oracle and the reference's golden vectors.

Tolerances (north_star): phi within 1e-5 relative per step, max-normalised
(max_i |phi_i - ref_i|_inf / max |ref|_inf); Gauss-Seidel trajectories 1e-4
absolute; the radix-select median is BIT-EXACT against np.partition of the
kernel's own D (integer work), and within 1e-5 of the fp64 oracle median.
"""
import math

import numpy as np
import pytest
import torch

from conftest import record_parity
from oracle import svgd_oracle as O

pytestmark = pytest.mark.gpu
PHI_TOL = 1e-5
TRAJ_TOL = 1e-4
DEV = "cuda:0"


def dsvgd():
    import dsvgd as m
    return m


def rel_err(got, ref):
    """max-normalised error (north_star's per-step phi tolerance form)."""
    e = float(np.abs(np.asarray(got, np.float64) - ref).max() / np.abs(ref).max())
    record_parity(e)
    return e


def abs_err(got, ref):
    e = float(np.abs(np.asarray(got, np.float64) - ref).max())
    record_parity(e)
    return e


def gpu(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32, device=DEV)


def target_for(g):
    T = dsvgd().targets
    tgt = str(g["target"])
    if tgt == "gmm":
        return T.GaussianMixture1D(), O.score_gmm
    if tgt == "gaussian":
        return T.Gaussian(g["mu"], g["lam"]), (lambda X: O.score_gaussian(X, g["mu"], g["lam"]))
    x, t = g["x_train"], g["t_train"]
    return T.LogisticRegression(x, t), (lambda X: O.score_logreg(X, x, t))


def engine_phi(X, S, h):
    """phi of all rows through the MFMA path (fixed h, or median if h is None)."""
    n, d = X.shape
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    Xg, Sg = gpu(X), gpu(S)
    eng.step(Xg, Sg, h=h)
    return eng.phi.cpu().numpy(), eng


# ----------------------------------------------------------- distances --
@pytest.mark.parametrize("n,d", [(1, 1), (2, 3), (129, 37), (300, 64), (513, 256), (1000, 100)])
def test_sqdist_matches_oracle(n, d):
    rs = np.random.RandomState(n + d)
    X = (rs.randn(n, d) * 1.5 + 3.0).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    eng.pack(gpu(X))
    eng.distances(median=True)
    D = eng.dense_D().cpu().numpy().astype(np.float64)
    ref = O.sqdist(X, X)
    nrm = ((X - X.mean(0)) ** 2).sum(1).astype(np.float64)
    scale = nrm[:, None] + nrm[None, :] + 1e-30
    assert np.all(np.diag(D) == 0.0)
    assert np.max(np.abs(D - ref) / scale) < 2e-6
    # padding of the panel buffer is +inf, valid entries finite
    full = eng.dense_D(padded=True).cpu().numpy()
    assert np.all(np.isfinite(full[:n, :n]))
    assert np.all(np.isposinf(full[n:, :])) and np.all(np.isposinf(full[:, n:]))


@pytest.mark.parametrize("n,d", [(1, 1), (2, 1), (3, 2), (200, 5), (1024, 1), (777, 64), (2048, 256)])
def test_median_select_bit_exact(n, d):
    rs = np.random.RandomState(7 * n + d)
    X = rs.randn(n, d).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    eng.pack(gpu(X))
    eng.distances(median=True)
    eng.median_bandwidth()
    med, h, inv_h = eng.state.read()
    D = eng.dense_D().cpu().numpy()
    k = (n * n - 1) // 2
    exact = np.partition(D.ravel(), k)[k]
    assert np.float32(med).view(np.uint32) == np.float32(exact).view(np.uint32)
    if n > 1 and exact > 0:
        assert h == pytest.approx(float(exact) / math.log(n), rel=1e-6)
        h64, med64 = O.median_bandwidth(X)
        assert abs(med - med64) <= 1e-5 * med64
    else:
        assert h == 1.0


def _sample_pairs(n, s, seed):
    """Pair (i, j) of sample p, as csrc/select.hip sample_sqdist_kernel hashes it
    (test restatement of its 64-bit finalizer)."""
    M = (1 << 64) - 1
    out = []
    for p in range(s):
        x = (seed ^ ((0x9e3779b97f4a7c15 * (p + 1)) & M)) & M
        x ^= x >> 33
        x = (x * 0xff51afd7ed558ccd) & M
        x ^= x >> 33
        x = (x * 0xc4ceb9fe1a85ec53) & M
        x ^= x >> 33
        out.append(((x & 0xffffffff) % n, (x >> 32) % n))
    return np.array(out, dtype=np.int64)


@pytest.mark.parametrize("d,ldy", [(256, 512), (61, 64), (61, 67), (5, 5)])
def test_sample_sqdist_pairs(d, ldy):
    """Sampled-pair distances behind the bracket (16-byte path when ldy % 4 == 0,
    generic path otherwise; columns >= d are never read into the sum)."""
    from dsvgd import _native as N
    n, s, seed = 3000, 4099, 0x5EED5EED
    rs = np.random.RandomState(d + ldy)
    Yh = rs.randn(n, ldy).astype(np.float32)
    Y = gpu(Yh)
    out = torch.empty(s, dtype=torch.float32, device=DEV)
    N.call("dsvgd_sample_sqdist", N.ptr(Y), ldy, n, d, s, seed, N.ptr(out), N.stream(DEV))
    torch.cuda.synchronize()
    ij = _sample_pairs(n, s, seed)
    Yd = Yh[:, :d].astype(np.float64)
    ref = ((Yd[ij[:, 0]] - Yd[ij[:, 1]]) ** 2).sum(1)
    got = out.cpu().numpy().astype(np.float64)
    assert np.abs(got - ref).max() <= 1e-5 * ref.max()


@pytest.mark.parametrize("d,s,klo,khi", [(256, 1 << 18, 127000, 135143), (61, 4100, 0, 4099),
                                          (8, 4096, 2047, 2047), (3, 1 << 16, 5, 60000)])
def test_sample_bracket_fused(d, s, klo, khi):
    """dsvgd_sample_bracket (7 launches, shared sweeps, both digits per pick)
    = sample_sqdist + two 3-pass selects + bracket_init: the same sample bits,
    lo / hi = the exact k_lo-th / k_hi-th order statistics, st armed with them."""
    from dsvgd import _native as N
    from dsvgd.engine import SelectState
    n, ldy, seed = 5000, ((d + 3) // 4) * 4, 0x5EED5EED
    rs = np.random.RandomState(d + s)
    Y = gpu(rs.randn(n, ldy).astype(np.float32))
    ref = torch.empty(s, dtype=torch.float32, device=DEV)
    out = torch.full((s,), np.nan, dtype=torch.float32, device=DEV)
    lo, hi, st = SelectState(DEV), SelectState(DEV), SelectState(DEV)
    strm = N.stream(DEV)
    N.call("dsvgd_sample_sqdist", N.ptr(Y), ldy, n, d, s, seed, N.ptr(ref), strm)
    for rep in range(2):                       # the call re-arms itself
        N.call("dsvgd_sample_bracket", N.ptr(Y), ldy, n, d, s, seed, klo, khi, N.ptr(out),
               lo.ptr, hi.ptr, st.ptr, 12345, 1 << 20, strm)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        srt = np.sort(ref.cpu().numpy())
        for state, k in ((lo, klo), (hi, khi)):
            med = state.read()[0]
            assert np.float32(med).view(np.uint32) == srt[k].view(np.uint32), (rep, k)
            assert int(state.hist.abs().sum()) == 0
        blo, bhi, below, ncand, fb = st.bracket()
        assert (blo, bhi, below, ncand, fb) == (float(srt[klo]), float(srt[khi]), 0, 0, 0)


@pytest.mark.parametrize("n,d,force_miss", [(4200, 100, False), (4200, 8, False),
                                             (4200, 100, True)])
def test_bracketed_median_bit_exact(n, d, force_miss):
    """Bracketed select (sample -> [lo, hi] -> candidates): bit-exact median,
    and the exact fallback to the passes over D when the bracket misses."""
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    assert eng.bracketed
    if force_miss:
        eng.k_lo = eng.k_hi = 0          # bracket [min, min] cannot hold the median
    eng.pack(gpu(X))
    eng.distances(median=True)
    eng.median_bandwidth()
    med, h, _ = eng.state.read()
    lo, hi, below, ncand, fallback = eng.state.bracket()
    D = eng.dense_D().cpu().numpy()
    k = (n * n - 1) // 2
    exact = np.partition(D.ravel(), k)[k]
    assert np.float32(med).view(np.uint32) == np.float32(exact).view(np.uint32)
    assert fallback == (1 if force_miss else 0)
    if not force_miss:
        assert lo <= med <= hi
        assert below == int((D < lo).sum()) and ncand == int(((D >= lo) & (D <= hi)).sum())
        assert ncand < 0.05 * n * n


@pytest.mark.parametrize("n", [100, 4200])
def test_median_all_identical_particles(n):
    X = np.ones((n, 4), np.float32)
    eng = dsvgd().PhiEngine(n, 4, device=DEV)
    eng.pack(gpu(X))
    eng.distances(median=True)
    eng.median_bandwidth()
    med, h, _ = eng.state.read()
    assert med == 0.0 and h == 1.0
    if eng.bracketed:                    # every entry in [0, 0]: overflow -> fallback
        assert eng.state.bracket()[4] == 1


def test_fused_histogram_equals_standalone_pass1():
    from dsvgd import _native as N
    n, d = 700, 48
    X = np.random.RandomState(3).randn(n, d).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    eng.pack(gpu(X))
    eng.distances(median=True)
    fused = eng.state.hist.clone()
    st2 = dsvgd().engine.SelectState(DEV)
    s = N.stream(DEV)
    N.call("dsvgd_select_init", st2.ptr, n, -1, s)
    N.call("dsvgd_radix_hist", N.ptr(eng.D), eng.m_pad * eng.n_pad, None, 1, st2.ptr,
           eng.n_pad if eng.sym else 0, s)
    assert torch.equal(fused, st2.hist)
    assert int(fused.sum()) == n * n


# ------------------------------------------------------------------ phi --
@pytest.mark.parametrize("name", ["g1_gmm_n64", "g1_gauss_n128_d8_medh", "g1_gauss_n64_d64_h1",
                                  "g1_logreg_n100"])
def test_phi_matches_reference_golden(golden, name):
    g = golden(name)
    tgt, _ = target_for(g)
    X = g["X"]
    Xg = gpu(X)
    S = torch.empty_like(Xg)
    tgt.score(Xg, S)
    phi, _ = engine_phi(X, S.cpu().numpy(), float(g["h"]))
    assert rel_err(phi, g["phi"]) < PHI_TOL


@pytest.mark.parametrize("n,d,median", [(1000, 1, True), (640, 64, True), (513, 256, False),
                                        (300, 1024, True)])
def test_phi_matches_oracle(n, d, median):
    rs = np.random.RandomState(n)
    X = rs.randn(n, d).astype(np.float32)
    mu = rs.randn(d).astype(np.float32)
    lam = rs.uniform(0.5, 2, d).astype(np.float32)
    S = O.score_gaussian(X, mu, lam).astype(np.float32)
    h = None if median else 2.0 * d
    phi, eng = engine_phi(X, S, h)
    hh = eng.state.read()[1] if median else h
    ref = O.phi(X, S, hh)
    assert rel_err(phi, ref) < PHI_TOL


@pytest.mark.parametrize("n,d", [(640, 64), (3000, 8)])
def test_direct_kernels_up_to_d64(n, d):
    """The explicit-difference kernels (default for d <= 2) stay exact up to
    their d = 64 limit (forced here through the engine: dsvgd_sqdist_direct,
    dsvgd_phi_direct)."""
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d).astype(np.float32)
    S = O.score_gmm(X).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    eng.DIRECT_MAX_D = 64
    eng.step(gpu(X), gpu(S), h=None)
    h = eng.state.read()[1]
    D = eng.dense_D().cpu().numpy().astype(np.float64)
    assert abs_err(D, O.sqdist(X, X)) <= 2e-6 * np.abs(O.sqdist(X, X)).max()
    assert rel_err(eng.phi.cpu().numpy(), O.phi(X, S, h)) < PHI_TOL


@pytest.mark.parametrize("n,d,m,row0,xmap", [(4096, 256, 1024, 1024, 1), (16384, 96, 2048, 14336, 1),
                                             (3000, 40, 1000, 1500, 1), (8192, 256, 2048, 4096, 3),
                                             (8192, 256, 2048, 4096, 0)])
def test_phi_row_block_split_k(n, d, m, row0, xmap):
    """A DistSampler rank's row block (non-symmetric D, split-K phi_mm); at
    d = 256, m = 2048 the slices are mapped to XCDs (xmap mask 3) or not (0)."""
    from dsvgd import _native as N
    prev = N.load().dsvgd_phi_set_xmap(xmap)
    try:
        _phi_row_block(n, d, m, row0)
    finally:
        N.load().dsvgd_phi_set_xmap(prev)


def _phi_row_block(n, d, m, row0):
    rs = np.random.RandomState(m)
    X = rs.randn(n, d).astype(np.float32)
    S = rs.randn(n, d).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, m=m, row0=row0, device=DEV)
    if n >= 4096:
        assert eng.splits > 1
    h = 2.0 * d          # fixed: the median rank is global (needs the hist all-reduce)
    eng.step(gpu(X), gpu(S), h=h)
    sample = np.arange(0, m, max(1, m // 64))
    ref = O.phi(X, S, h, rows=row0 + sample)
    got = eng.phi.cpu().numpy()[sample]
    assert rel_err(got, ref) < PHI_TOL


def test_phi_full_size_sampled_rows():
    """n = 65536, d = 256 (the headline shape): 256 sampled rows vs fp64, and the
    median checked by counting (size-independent property of the select)."""
    n, d = 65536, 256
    rs = np.random.RandomState(0)
    X = rs.randn(n, d).astype(np.float32)
    mu = rs.randn(d).astype(np.float32)
    lam = rs.uniform(0.5, 2, d).astype(np.float32)
    S = O.score_gaussian(X, mu, lam).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    eng.step(gpu(X), gpu(S), h=None)
    med, h, _ = eng.state.read()
    assert eng.sym  # the headline shape runs on the symmetric layout
    below = eng.count_D(lambda t: t < med)
    at_or_below = eng.count_D(lambda t: t <= med)
    k = (n * n - 1) // 2
    assert below <= k < at_or_below
    rows = np.sort(rs.choice(n, 256, replace=False))
    ref = O.phi(X, S, h, rows=rows)
    got = eng.phi[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    assert rel_err(got, ref) < PHI_TOL


@pytest.mark.parametrize("symrow", [1, 0])
@pytest.mark.parametrize("n,d", [(4096, 1024), (8192, 256), (4200, 256)])
def test_phi_symmetric_hybrid_sampled_rows(n, d, symrow):
    """The symmetric layout's phi_mm at split-K >= 2: one launch per row
    (symrow = 1, phi_w1 DS 4: contiguous slices, transposed K-steps first,
    slices mapped to XCDs when 8 | row blocks x slices) or the two-launch
    hybrid (DS 1 + DS 2, interleaved slices): rows from every region of the
    triangle -- first and last row blocks, block edges, the diagonal tiles --
    vs fp64; d = 1024 runs four column blocks per row block (no XCD map),
    n = 4200 a ragged last row block (33 row blocks: the map only with 8
    slices)."""
    from dsvgd import _native as N
    prev = N.load().dsvgd_phi_set_symrow(symrow)
    try:
        _phi_symmetric_rows(n, d)
    finally:
        N.load().dsvgd_phi_set_symrow(prev)


def _phi_symmetric_rows(n, d):
    rs = np.random.RandomState(n + d)
    X = (0.2 * rs.randn(n, d)).astype(np.float32)
    mu = rs.randn(d).astype(np.float32)
    lam = rs.uniform(0.5, 2, d).astype(np.float32)
    S = O.score_gaussian(X, mu, lam).astype(np.float32)
    eng = dsvgd().PhiEngine(n, d, device=DEV)
    assert eng.sym and eng.splits >= 2
    eng.step(gpu(X), gpu(S), h=None)
    h = eng.state.read()[1]
    rows = np.unique(np.concatenate([np.arange(0, 130), np.arange(n - 130, n),
                                     np.arange(127, n, 1024), np.arange(128, n, 1024),
                                     rs.choice(n, 64, replace=False)]))
    ref = O.phi(X, S, h, rows=rows)
    got = eng.phi[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    assert rel_err(got, ref) < PHI_TOL


# --------------------------------------------------------------- scores --
def test_scores_match_oracle():
    T = dsvgd().targets
    rs = np.random.RandomState(5)
    X = rs.randn(1000, 21).astype(np.float32)
    mu, lam = rs.randn(21).astype(np.float32), rs.uniform(0.5, 2, 21).astype(np.float32)
    out = torch.empty(1000, 21, device=DEV)
    T.Gaussian(mu, lam).score(gpu(X), out, 2.0)
    assert rel_err(out.cpu().numpy(), 2.0 * O.score_gaussian(X, mu, lam)) < 1e-6
    T.GaussianMixture1D().score(gpu(X * 3), out)
    assert rel_err(out.cpu().numpy(), O.score_gmm(X * 3)) < 1e-5
    xd, t = rs.randn(777, 20).astype(np.float32), np.sign(rs.randn(777)).astype(np.float32)
    X[:, 0] = rs.uniform(-1, 1, 1000)
    T.LogisticRegression(xd, t).score(gpu(X), out, 0.5)
    assert rel_err(out.cpu().numpy(), 0.5 * O.score_logreg(X, xd, t)) < 1e-5


@pytest.mark.parametrize("n,N,p", [(1, 400, 2), (7, 777, 20), (32, 8192, 255), (33, 100, 5)])
def test_logreg_scores_small_and_gemm_paths(n, N, p):
    """Both logistic-regression score paths (one block per particle for
    n <= 32, N <= 8192; the two-GEMM path otherwise) against the oracle,
    including a single-row view of a bigger particle matrix (the
    Gauss-Seidel refresh)."""
    rs = np.random.RandomState(n + N)
    X = (rs.randn(n + 3, p + 1) * 0.5).astype(np.float32)
    xd = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    tgt = dsvgd().targets.LogisticRegression(xd, t)
    Xg = gpu(X)
    out = torch.zeros(n + 3, p + 1, device=DEV)
    tgt.score(Xg[1:n + 1], out[1:n + 1], 3.0)
    ref = 3.0 * O.score_logreg(X[1:n + 1], xd, t)
    assert rel_err(out[1:n + 1].cpu().numpy(), ref) < 1e-5
    assert float(out[0].abs().max()) == 0.0 and float(out[n + 1:].abs().max()) == 0.0


def test_callable_target_matches_builtin():
    import dsvgd as m
    rs = np.random.RandomState(9)
    mu, lam = rs.randn(6).astype(np.float32), rs.uniform(0.5, 2, 6).astype(np.float32)
    mu_t, lam_t = gpu(mu), gpu(lam)
    tgt = m.targets.resolve_target(lambda x: -0.5 * (lam_t * (x - mu_t) ** 2).sum())
    X = gpu(rs.randn(50, 6))
    a, b = torch.empty_like(X), torch.empty_like(X)
    tgt.score(X, a)
    m.targets.Gaussian(mu, lam).score(X, b)
    assert torch.allclose(a, b, atol=1e-6)


@pytest.mark.parametrize("n,d,ldx", [(6000, 64, 64), (4096, 3, 3), (2048, 70, 72), (9000, 256, 256)])
def test_phi_row_split_matches_oracle(n, d, ldx):
    """Gauss-Seidel rows at large n (dsvgd_phi_row_split: the j range over
    dsvgd_phi_row_blocks workgroups): 24 consecutive row updates against the
    fp64 sequential restatement, and against the one-workgroup row kernel."""
    from dsvgd import _native as N
    from dsvgd.engine import SelectState, sequential_sweep
    lib = N.load()
    assert lib.dsvgd_phi_row_blocks(n, d) > 1
    rs = np.random.RandomState(n + d)
    X0 = (0.5 * rs.randn(n, d)).astype(np.float32)
    S = rs.randn(n, d).astype(np.float32)
    h, step, rows = 0.8 * d, 0.05, list(range(100, 124))
    st = SelectState(DEV)
    N.call("dsvgd_set_bandwidth", st.ptr, h, N.stream(DEV))
    buf = torch.zeros(n, ldx, dtype=torch.float32, device=DEV)
    Xg = buf[:, :d]
    Xg.copy_(gpu(X0))
    Sg = gpu(S)
    sequential_sweep(Xg, Sg, rows, st, step)
    got = Xg.cpu().numpy().astype(np.float64)
    ref = X0.astype(np.float64)
    for i in rows:
        ref[i] += step * O.phi(ref, S, h, rows=[i])[0]
    moved = np.abs(ref[rows] - X0[rows]).max()
    assert rel_err(got[rows] - X0[rows], ref[rows] - X0[rows]) < PHI_TOL * 10, moved
    assert np.array_equal(got[:100], X0[:100]) and np.array_equal(got[124:], X0[124:])
    # the one-workgroup kernel on the same rows
    X1 = gpu(X0)
    for i in rows:
        N.call("dsvgd_phi_row", N.ptr(X1), d, N.ptr(Sg), d, n, d, i, st.ptr, step, None, None,
               N.stream(DEV))
    one = X1.cpu().numpy().astype(np.float64)
    assert np.abs(one[rows] - got[rows]).max() <= 1e-5 * np.abs(got[rows]).max()


@pytest.mark.parametrize("n,d,lo,hi,kind", [(300, 3, 0, 300, "gauss"), (2000, 64, 37, 300, "none"),
                                             (1000, 1, 100, 331, "gmm"), (700, 33, 0, 700, "gauss"),
                                             # the wide sweep (64 < d <= 1024, f32 MFMA wide pass)
                                             (1500, 128, 10, 700, "gauss"),
                                             (1200, 256, 0, 1200, "none"),
                                             # the incremental walk's other shapes
                                             (1100, 256, 5, 1000, "gmm"),
                                             (900, 96, 0, 900, "gauss"),
                                             (800, 700, 50, 400, "gauss"),
                                             (600, 1024, 0, 300, "gmm"),
                                             # the logistic regression's score
                                             # refreshed in the walk (any d)
                                             (4096, 128, 0, 4096, "logreg"),
                                             (1000, 55, 13, 900, "logreg"),
                                             (700, 96, 0, 300, "logreg_big")])
def test_blocked_sweep_matches_oracle(n, d, lo, hi, kind):
    """The blocked Gauss-Seidel sweep (csrc/gs.hip: 64-row blocks, a wide pass
    against all n rows + one workgroup for the in-block order) against the
    fp64 sequential restatement -- blocks cut anywhere in the range, scores
    frozen or refreshed after every move (Gaussian, GMM, the logistic
    regression on N = 1024 data rows or 5000 of them (two LDS chunks) with
    the partition mode's N_global / N_local scale), W2-style extra rows and
    phi_out -- and against the per-row path."""
    from dsvgd import _native as N
    from dsvgd.engine import SelectState, sequential_sweep
    m = dsvgd()
    rs = np.random.RandomState(n + d)
    X0 = (0.7 * rs.randn(n, d)).astype(np.float32)
    mu = rs.randn(d).astype(np.float32)
    lam = rs.uniform(0.5, 2.0, d).astype(np.float32)
    scale, step = 1.0, 0.05
    if kind.startswith("logreg"):
        nd = 5000 if kind == "logreg_big" else 1024
        xd = (0.3 * rs.randn(nd, d - 1) / np.sqrt(d)).astype(np.float32)
        td = np.where(rs.rand(nd) < 0.5, -1.0, 1.0).astype(np.float32)
        X0[:, 0] = (0.3 * rs.randn(n)).astype(np.float32)      # log alpha
        scale, step = 2.0, 0.01
    tgt = {"gauss": lambda: m.targets.Gaussian(mu, lam), "gmm": m.targets.GaussianMixture1D,
           "none": lambda: None, "logreg": lambda: m.targets.LogisticRegression(xd, td),
           "logreg_big": lambda: m.targets.LogisticRegression(xd, td)}[kind]()
    fn = {"gauss": lambda X: O.score_gaussian(X, mu, lam), "gmm": O.score_gmm,
          "none": None, "logreg": lambda X: scale * O.score_logreg(X, xd, td),
          "logreg_big": lambda X: scale * O.score_logreg(X, xd, td)}[kind]
    S0 = (fn(X0) if fn else rs.randn(n, d)).astype(np.float32)
    h = 0.9 * d + 0.5
    rows = range(lo, hi)
    extra = (0.01 * rs.randn(hi - lo, d)).astype(np.float32)
    st = SelectState(DEV)
    N.call("dsvgd_set_bandwidth", st.ptr, h, N.stream(DEV))
    out = {}
    for blocked in (True, False):
        Xg, Sg = gpu(X0), gpu(S0)
        phi = torch.zeros(hi - lo, d, device=DEV)
        sequential_sweep(Xg, Sg, rows, st, step, target=tgt, score_scale=scale, phi_out=phi,
                         extra=gpu(extra), blocked=blocked)
        out[blocked] = (Xg.cpu().numpy().astype(np.float64), Sg.cpu().numpy(), phi.cpu().numpy())
    ref = X0.astype(np.float64)
    S = S0.astype(np.float64)
    ref_phi = np.zeros((hi - lo, d))
    for k, i in enumerate(rows):
        ref_phi[k] = O.phi(ref, S, h, rows=[i])[0] + extra[k]
        ref[i] += step * ref_phi[k]
        if fn:
            S[i] = fn(ref[i:i + 1])[0]
    got, gs, gphi = out[True]
    assert np.array_equal(got[:lo], X0[:lo]) and np.array_equal(got[hi:], X0[hi:])
    e = rel_err(gphi, ref_phi)
    assert e < PHI_TOL, e
    assert abs_err(got, ref) < TRAJ_TOL
    if fn:
        assert np.abs(gs[rows.start:rows.stop] - S[rows.start:rows.stop]).max() <= \
            1e-5 * np.abs(S).max()
    # the per-row kernels on the same sweep (different summation order only)
    assert np.abs(out[False][0] - got).max() <= 1e-5 * max(1.0, np.abs(got).max())


@pytest.mark.parametrize("n,d,lo,hi,kind", [(2000, 256, 0, 2000, "none"), (1500, 200, 31, 1400, "gauss"),
                                             (700, 64 + 32, 0, 700, "gmm"),
                                             # 2 and 4 columns per thread (16 / 32-row blocks)
                                             (700, 512, 3, 650, "gauss"),
                                             (600, 1024, 0, 600, "none"),
                                             (500, 1000, 7, 480, "gmm")])
def test_incremental_walk_matches_four_wave_walk(n, d, lo, hi, kind):
    """The incremental walk (dsvgd_gsw_set_inc(1): each moved row's pair terms
    added to every later row of the block at once) and the four-wave walk
    (per row: distances to the moved rows, then the column loop) move the same
    rows to the same places up to rounding (different summation order),
    with phi_out and extra rows."""
    from dsvgd import _native as N
    from dsvgd.engine import SelectState, sequential_sweep
    m = dsvgd()
    lib = N.load()
    rs = np.random.RandomState(7 * n + d)
    X0 = (0.6 * rs.randn(n, d)).astype(np.float32)
    mu = rs.randn(d).astype(np.float32)
    lam = rs.uniform(0.5, 2.0, d).astype(np.float32)
    tgt = {"gauss": lambda: m.targets.Gaussian(mu, lam), "gmm": m.targets.GaussianMixture1D,
           "none": lambda: None}[kind]()
    S0 = rs.randn(n, d).astype(np.float32) if tgt is None else \
        {"gauss": lambda: O.score_gaussian(X0, mu, lam), "gmm": lambda: O.score_gmm(X0)}[kind]().astype(np.float32)
    st = SelectState(DEV)
    N.call("dsvgd_set_bandwidth", st.ptr, 0.8 * d, N.stream(DEV))
    extra = (0.01 * rs.randn(hi - lo, d)).astype(np.float32)
    out = {}
    prev = lib.dsvgd_gsw_set_inc(1)
    try:
        for inc in (1, 0):
            lib.dsvgd_gsw_set_inc(inc)
            Xg, Sg = gpu(X0), gpu(S0)
            phi = torch.zeros(hi - lo, d, device=DEV)
            sequential_sweep(Xg, Sg, range(lo, hi), st, 0.05, target=tgt, phi_out=phi,
                             extra=gpu(extra))
            torch.cuda.synchronize()
            out[inc] = (Xg.cpu().numpy(), Sg.cpu().numpy(), phi.cpu().numpy())
    finally:
        lib.dsvgd_gsw_set_inc(prev)
    (x1, s1, p1), (x0, s0, p0) = out[1], out[0]
    assert np.array_equal(x1[:lo], X0[:lo]) and np.array_equal(x1[hi:], X0[hi:])
    assert np.abs(p1 - p0).max() <= 1e-5 * np.abs(p0).max()
    assert np.abs(x1 - x0).max() <= 1e-5 * max(1.0, np.abs(x0).max())
    assert np.abs(s1 - s0).max() <= 1e-5 * max(1.0, np.abs(s0).max())


def test_sampler_blocked_sweep_matches_reference(golden, monkeypatch):
    """The reference's own Sampler trajectories (GMM n = 50, Gauss-Seidel) run
    through the blocked sweep (its row threshold lowered to 1)."""
    import dsvgd.engine as E
    monkeypatch.setattr(E, "GS_BLOCK_MIN_ROWS", 1)
    g = golden("g2_sample_gmm_n50")
    torch.manual_seed(int(g["seed"]))
    s = dsvgd().Sampler(1, dsvgd().targets.GaussianMixture1D(), dsvgd().RBF(float(g["h"])))
    df = s.sample(int(g["n"]), int(g["T"]), float(g["eps"]), verbose=False)
    vals = np.stack(df["value"].to_list()).reshape(g["values"].shape)
    assert abs_err(vals, g["values"]) < TRAJ_TOL


# --------------------------------------------------------- samplers ----
@pytest.mark.parametrize("name", ["g2_sample_gauss_n32_d2", "g2_sample_gmm_n50"])
def test_sampler_sequential_matches_reference(golden, name):
    g = golden(name)
    tgt, _ = target_for(g)
    torch.manual_seed(int(g["seed"]))
    s = dsvgd().Sampler(int(g["d"]), tgt, dsvgd().RBF(float(g["h"])))
    df = s.sample(int(g["n"]), int(g["T"]), float(g["eps"]), verbose=False)
    vals = np.stack(df["value"].to_list()).reshape(g["values"].shape)
    np.testing.assert_array_equal(vals[0], g["values"][0])
    assert abs_err(vals, g["values"]) < TRAJ_TOL
    np.testing.assert_array_equal(df["timestep"].to_numpy(), g["timestep"])
    np.testing.assert_array_equal(df["particle"].to_numpy(), g["particle"])


def test_sampler_reference_kernel_callable(golden):
    """A plain reference kernel lambda is accepted (probed to RBF(1))."""
    g = golden("g2_sample_gmm_n50")
    torch.manual_seed(int(g["seed"]))
    s = dsvgd().Sampler(1, dsvgd().targets.GaussianMixture1D(),
                        lambda x, y: torch.exp(-1. * torch.dist(x, y, p=2) ** 2))
    df = s.sample(50, 3, 1.0, verbose=False)
    vals = np.stack(df["value"].to_list()).reshape(g["values"].shape)
    assert abs_err(vals, g["values"]) < TRAJ_TOL


@pytest.mark.parametrize("median", [False, True])
def test_sampler_jacobi_matches_oracle(median):
    mu, lam = np.array([1.0, -0.5, 0.2], np.float32), np.array([1.0, 2.0, 0.5], np.float32)
    torch.manual_seed(4)
    s = dsvgd().Sampler(3, dsvgd().targets.Gaussian(mu, lam),
                        dsvgd().RBF("median" if median else 1.5))
    df = s.sample(200, 5, 0.05, order="jacobi", verbose=False)
    vals = np.stack(df["value"].to_list()).reshape(6, 200, 3)
    ref = O.sampler_jacobi(vals[0], lambda X: O.score_gaussian(X, mu, lam), 1.5, 5, 0.05,
                           median=median)
    assert abs_err(vals, ref) < TRAJ_TOL


def test_gmm_posterior_statistics_jacobi():
    """Jacobi vs reference order: posterior mean/var agree within MC error."""
    torch.manual_seed(42)
    s = dsvgd().Sampler(1, dsvgd().targets.GaussianMixture1D(), dsvgd().RBF(1.0))
    df = s.sample(1024, 300, 1.0, order="jacobi", verbose=False)
    x = np.stack(df[df["timestep"] == 300]["value"].to_list())[:, 0]
    # target: equal mixture of N(-2,1), N(2,1): mean 0, var 5
    assert abs(x.mean()) < 3 * math.sqrt(5.0 / 1024) + 0.05
    assert abs(x.var() - 5.0) < 0.5


@pytest.mark.parametrize("order", ["sequential", "jacobi"])
def test_distsampler_s1_matches_reference(golden, order):
    g = golden("g3_dist_s1_partitions")
    x, t = g["x_train"], g["t_train"]
    parts = torch.tensor(g["init"][0])
    ds = dsvgd().DistSampler(0, 1, dsvgd().targets.LogisticRegression(x, t), dsvgd().RBF(1.0),
                             parts, x.shape[0], x.shape[0], exchange_particles=False,
                             exchange_scores=False, include_wasserstein=False, order=order)
    for step in range(int(g["steps"])):
        ds.make_step(float(g["eps"]), h=10.0)
        got = ds.particles.numpy()
        if order == "sequential":
            assert abs_err(got, g["own"][0][step]) < TRAJ_TOL
    if order == "jacobi":
        fn = lambda X: O.score_logreg(X, x, t)  # noqa: E731
        D = O.DistOracle([g["init"][0]], [fn], x.shape[0], x.shape[0], False, False,
                         sequential=False)
        for _ in range(int(g["steps"])):
            D.step(float(g["eps"]))
        assert abs_err(ds.particles.numpy(), D.own(0)) < TRAJ_TOL
    # the caller's CPU tensor is mutated like the reference's view (a7)
    np.testing.assert_array_equal(parts.numpy(), ds._particles.numpy())


# ----------------------------------------------------- W2 / JKO term --
W2_GOLDEN = ["g5_w2_m8_n8_d2", "g5_w2_m12_n12_d3", "g5_w2_m8_n16_d3", "g5_w2_m6_n24_d5",
             "g5_w2_m16_n32_d4_near", "g5_w2_m24_n24_d3_near"]


def _row_sets(plan, m):
    """The plan as per-row column sets (slots of one row are interchangeable)."""
    return np.sort(np.asarray(plan).reshape(m, -1), axis=1)


def _w2_gpu(X, P, h=1.0):
    X = torch.tensor(np.ascontiguousarray(X, np.float32), device=DEV)
    P = torch.tensor(np.ascontiguousarray(P, np.float32), device=DEV)
    w = dsvgd().w2.W2Term(X.shape[0], P.shape[0], X.shape[1], DEV)
    G = w.grad(X, P, h).cpu().numpy().astype(np.float64)
    return G, w.plan(), w


@pytest.mark.parametrize("name", W2_GOLDEN)
def test_w2_grad_matches_reference_lp(golden, name):
    """GPU auction + gradient == the reference's linprog plan (golden)."""
    g = golden(name)
    G, plan, _ = _w2_gpu(g["X"], g["P"], h=1.0)
    err = abs_err(G, g["grad"]) / max(np.abs(g["grad"]).max(), 1e-30)
    record_parity(err)
    assert err < PHI_TOL, err
    m = g["X"].shape[0]
    np.testing.assert_array_equal(_row_sets(plan, m), _row_sets(O.w2_plan(O.w2_cost(g["X"], g["P"])), m))


@pytest.mark.parametrize("m,n,d,near", [(256, 256, 16, None), (512, 1024, 8, None),
                                        (500, 4000, 3, None), (2048, 2048, 64, None),
                                        (1024, 1024, 32, 0.05), (1024, 4096, 8, 0.01),
                                        (3000, 3000, 2, 0.2), (64, 1024, 8, None),
                                        (32, 1024, 4, None), (512, 4096, 16, "svgd")])
def test_w2_assignment_optimal(m, n, d, near):
    """Plan == scipy's exact assignment on the fp64 costs (random inputs: no
    near-ties at these sizes), and the gradient within PHI_TOL.  R = n/m up to
    32; "svgd": the owned rows' previous copies (all_particles mode) plus
    other ranks' particles."""
    rs = np.random.RandomState(m + n + d)
    X = rs.randn(m, d).astype(np.float32)
    if near is None:
        P = rs.randn(n, d).astype(np.float32)
    elif near == "svgd":
        P = rs.randn(n, d).astype(np.float32)
        P[:m] = X - 1e-3 * rs.randn(m, d).astype(np.float32)
    else:
        P = (np.tile(X, (n // m, 1)) + near * rs.randn(n, d)).astype(np.float32)
    G, plan, w = _w2_gpu(X, P, h=2.5)
    C = O.w2_cost(X, P)
    ref_plan = O.w2_plan(C)
    R = n // m
    rows = np.arange(n) // R
    got_cost, opt_cost = C[rows, plan].sum(), C[rows, ref_plan].sum()
    assert sorted(plan.tolist()) == list(range(n))
    assert got_cost <= opt_cost * (1 + 1e-6) + 1e-9, (got_cost, opt_cost)
    same = float((_row_sets(plan, m) == _row_sets(ref_plan, m)).all(1).mean())
    ref = 2.5 * O.w2_grad(X, P, ref_plan)[0]
    err = abs_err(G, ref) / np.abs(ref).max()
    record_parity(err, rounds=w.rounds, same_plan=same)
    assert same == 1.0, same
    assert err < PHI_TOL, err


@pytest.mark.parametrize("m,n,d", [(512, 4096, 16), (1024, 1024, 32)])
def test_w2_tail_stall_finishes_on_bid_rounds(m, n, d):
    """the phase tail's scan helpers share the device with other
    work; if they do not answer in time the tail turns itself off for the
    solve and the bid rounds finish it.  Forced here (dsvgd_w2_set_tail_debug:
    the helpers exit at once): at least one stall is recorded and the plan is
    still scipy's exact assignment (R = 8 with the price cache, R = 1)."""
    from dsvgd import _native
    lib = _native.load()
    rs = np.random.RandomState(m + n + d + 1)
    X = rs.randn(m, d).astype(np.float32)
    P = rs.randn(n, d).astype(np.float32)
    lib.dsvgd_w2_set_tail_debug(1)
    try:
        G, plan, w = _w2_gpu(X, P, h=2.5)
        stats = w.tail_stats()
    finally:
        lib.dsvgd_w2_set_tail_debug(0)
    assert stats[5] >= 1, stats
    ref_plan = O.w2_plan(O.w2_cost(X, P))
    assert (_row_sets(plan, m) == _row_sets(ref_plan, m)).all()
    ref = 2.5 * O.w2_grad(X, P, ref_plan)[0]
    assert abs_err(G, ref) / np.abs(ref).max() < PHI_TOL


@pytest.mark.parametrize("m,n,d,step", [(512, 4096, 16, 1e-3), (512, 4096, 16, 0.3),
                                        (1024, 1024, 32, 1e-2), (256, 2048, 8, 1e-4)])
def test_w2_warm_start_same_plan(m, n, d, step):
    """The next SVGD step's solve warm-started from this one's prices and
    plan (dsvgd_w2_assign_warm: first epsilon from the old plan's slackness
    violation) == scipy's exact plan of the new problem, for small and large
    steps; fixed-phase warm starts and a cold solve agree with it."""
    rs = np.random.RandomState(m + n + d)
    X = rs.randn(m, d).astype(np.float32)
    P = rs.randn(n, d).astype(np.float32)
    P[:m] = X - 1e-3 * rs.randn(m, d).astype(np.float32)
    X2 = (X + step * rs.randn(m, d)).astype(np.float32)
    P2 = (P + step * rs.randn(n, d)).astype(np.float32)
    ref = O.w2_plan(O.w2_cost(X2, P2))
    W2 = dsvgd().w2.W2Term
    plans = {}
    for mode in (None, 2, 0):
        w = W2(m, n, d, DEV, warm=True)
        old = W2.WARM_PHASES
        W2.WARM_PHASES = mode
        try:
            w.grad(gpu(X), gpu(P), 1.0)
            w.grad(gpu(X2), gpu(P2), 1.0)
        finally:
            W2.WARM_PHASES = old
        plans[mode] = (w.plan(), w.rounds)
    for mode, (plan, rounds) in plans.items():
        np.testing.assert_array_equal(_row_sets(plan, m), _row_sets(ref, m), err_msg=str(mode))
    record_parity(0.0, rounds_adaptive=plans[None][1], rounds_cold=plans[0][1])


@pytest.mark.parametrize("m,d,step,cost,ties", [(1024, 32, 1e-2, "exact", False),
                                                (512, 8, 0.3, "exact", False),
                                                (400, 3, 1e-2, "exact", True),
                                                (2048, 256, 1e-3, "h2", False),
                                                (2048, 64, 1e-3, "h2", True)])
def test_w2_fused_first_round_same_solve(m, d, step, cost, ties):
    """An R = 1 warm start takes the violation and the first round's row
    scans (best value, its column -- the lower on a tie --, second value) in
    one pass over C and bids from them (dsvgd_w2_set_fuse_first): the same
    plan slot for slot, the same round count and bit-identical prices and
    gradient as the violation pass + full-scan bid round, and scipy's plan.
    `ties`: previous particles duplicated in pairs, so rows see equal costs."""
    lib = dsvgd()._native.load()
    rs = np.random.RandomState(m + d + (7 if ties else 0))
    X = rs.randn(m, d).astype(np.float32)
    if ties:
        P = np.repeat(rs.randn(m // 2, d).astype(np.float32), 2, axis=0)
        X2 = X + np.float32(step) * rs.randn(m, d).astype(np.float32)
        P2 = P.copy()
    else:
        P = X - 1e-3 * rs.randn(m, d).astype(np.float32)
        X2 = (X + step * rs.randn(m, d)).astype(np.float32)
        P2 = (P + step * rs.randn(m, d)).astype(np.float32)
    W2 = dsvgd().w2.W2Term
    out = {}
    for fuse in (1, 0):
        old_cost, W2.COST = W2.COST, cost
        try:
            w = W2(m, m, d, DEV, warm=True)
        finally:
            W2.COST = old_cost
        assert w.cost == cost
        prev = lib.dsvgd_w2_set_fuse_first(fuse)
        try:
            w.grad(gpu(X), gpu(P), 1.0)
            G = w.grad(gpu(X2), gpu(P2), 1.0).cpu().numpy()
        finally:
            lib.dsvgd_w2_set_fuse_first(prev)
        price = w.ws[256:256 + 8 * m].cpu().numpy().view(np.float64).copy()
        out[fuse] = (w.plan(), w.rounds, price, G)
    (p1, r1, q1, g1), (p0, r0, q0, g0) = out[1], out[0]
    np.testing.assert_array_equal(p1, p0)
    assert r1 == r0, (r1, r0)
    np.testing.assert_array_equal(q1, q0)
    np.testing.assert_array_equal(g1, g0)
    C = O.w2_cost(X2, P2)
    ref = O.w2_plan(C)
    rows = np.arange(m)
    if ties:  # several optimal plans: the cost must be optimal
        assert C[rows, p1].sum() <= C[rows, ref].sum() * (1 + 1e-6)
    else:
        np.testing.assert_array_equal(p1, ref)
    record_parity(0.0, rounds=r1)


@pytest.mark.parametrize("m,n,d,pad", [(1, 1, 1, 0), (129, 127, 37, 3), (130, 300, 64, 0),
                                       (256, 1024, 256, 1), (77, 515, 5, 2)])
def test_w2_cost_tiles(m, n, d, pad):
    """dsvgd_w2_cost (128 x 128 tiles): C_ij = ||x_i - y_j||^2 from explicit
    fp32 differences, ragged tile edges, row-strided X / Y, ldc > n and a C
    that is not 16-byte aligned (pad) -- vs fp64 within fp32 rounding; the
    padding columns stay untouched."""
    N = dsvgd()._native
    rs = np.random.RandomState(m * 7 + n + d)
    X = rs.randn(m, d + 3).astype(np.float32)
    Y = rs.randn(n, d + 1).astype(np.float32)
    ldc = n + 5
    Xg, Yg = gpu(X), gpu(Y)
    buf = torch.full((m * ldc + pad,), -1.0, device=DEV)
    C = buf[pad:]
    N.call("dsvgd_w2_cost", N.ptr(Xg), d + 3, m, N.ptr(Yg), d + 1, n, d, N.ptr(C), ldc,
           N.stream(torch.device(DEV)))
    got = C.view(m, ldc).cpu().numpy()
    ref = ((X[:, None, :d].astype(np.float64) - Y[None, :, :d]) ** 2).sum(-1)
    np.testing.assert_allclose(got[:, :n], ref, rtol=2e-6 * d, atol=1e-6)
    assert np.all(got[:, n:] == -1.0)
    assert np.all(buf[:pad].cpu().numpy() == -1.0)


def test_w2_degenerate_and_identity():
    """All-equal particles (every cost 0) -> zero gradient; previous ==
    current (S = 1 consecutive steps) -> identity plan, zero gradient."""
    X = np.ones((64, 5), np.float32)
    G, plan, _ = _w2_gpu(X, np.ones((128, 5), np.float32))
    assert np.all(G == 0)
    Y = np.random.RandomState(3).randn(300, 7).astype(np.float32)
    G, plan, _ = _w2_gpu(Y, Y)
    np.testing.assert_array_equal(plan, np.arange(300))
    assert np.all(G == 0)


def test_w2_ties_reach_optimal_cost():
    """Duplicated previous particles make the plan non-unique (the LP may
    return any vertex): the cost must still be optimal."""
    rs = np.random.RandomState(7)
    X = rs.randn(200, 3).astype(np.float32)
    P = np.repeat(rs.randn(100, 3).astype(np.float32), 2, axis=0)
    _, plan, _ = _w2_gpu(X, P)
    C = O.w2_cost(X, P)
    opt = C[np.arange(200), O.w2_plan(C)].sum()
    assert C[np.arange(200), plan].sum() <= opt * (1 + 1e-6)


def test_w2_errors():
    X = torch.zeros((3, 2), device=DEV)
    with pytest.raises(ValueError):
        dsvgd().w2.W2Term(3, 4, 2, DEV)
    w = dsvgd().w2.W2Term(3, 3, 2, DEV)
    bad = torch.full((3, 2), float("nan"), device=DEV)
    with pytest.raises(dsvgd()._native.NativeError):
        w.grad(X, bad, 1.0)


# ---- the W2 cost on the MFMA Gram (dsvgd_w2_cost_h2) --
def _w2_cost(X, P, form):
    """C (m x n) from W2Term's cost form `form` ("h2" / "exact")."""
    N = dsvgd()._native
    W2 = dsvgd().w2.W2Term
    old = W2.COST
    W2.COST = form
    try:
        w = W2(X.shape[0], P.shape[0], X.shape[1], DEV)
    finally:
        W2.COST = old
    Xg, Pg = gpu(X), gpu(P)
    if form == "h2":
        N.call("dsvgd_w2_cost_h2", N.ptr(Xg), X.shape[1], X.shape[0], N.ptr(Pg), P.shape[1],
               P.shape[0], X.shape[1], N.ptr(w.C), w.ldc, (N.ptr(w.cws) + 255) // 256 * 256,
               float(w.TAU), N.ptr(w.cstat), N.stream(torch.device(DEV)))
    else:
        N.call("dsvgd_w2_cost", N.ptr(Xg), X.shape[1], X.shape[0], N.ptr(Pg), P.shape[1],
               P.shape[0], X.shape[1], N.ptr(w.C), w.ldc, N.stream(torch.device(DEV)))
    torch.cuda.synchronize()
    C = w.C[:X.shape[0], :P.shape[0]].cpu().numpy()
    if form == "h2":
        # the largest entry and the finite flag, taken while C was written
        # (what the solve's own pass over C would find; dsvgd_w2_assign_stat)
        st = w.cstat.cpu().numpy().view(np.uint32)
        assert st[0] == C.max().view(np.uint32) and st[1] == 0, (st, C.max())
    return C


@pytest.mark.parametrize("m,n,d,kind", [(300, 900, 37, "random"), (1024, 1024, 256, "svgd"),
                                        (512, 4096, 256, "svgd"), (250, 1000, 700, "random"),
                                        (150, 300, 3, "near"), (2048, 2048, 64, "svgd")])
def test_w2_cost_h2_matches_exact(m, n, d, kind):
    """The Gram-form W2 cost on the split-role MFMA Gram against the
    explicit-difference VALU tiles: every entry within 2e-5 of it (the FmtH2
    bound, ~2^-19 of the entry where the form is kept), and the near pairs
    -- a particle and its own previous position, the entries that decide an
    SVGD plan -- recomputed to the same bits."""
    rs = np.random.RandomState(m + n + d)
    X = rs.randn(m, d).astype(np.float32)
    P = rs.randn(n, d).astype(np.float32)
    if kind == "svgd":
        P[:m] = X - 1e-3 * rs.randn(m, d).astype(np.float32)
    elif kind == "near":
        P = (np.tile(X, (n // m + 1, 1))[:n] + 0.05 * rs.randn(n, d)).astype(np.float32)
    Ch, Ce = _w2_cost(X, P, "h2"), _w2_cost(X, P, "exact")
    assert np.isfinite(Ch).all()
    rel = np.abs(Ch.astype(np.float64) - Ce) / np.maximum(Ce, 1e-30)
    record_parity(float(rel.max()))
    assert rel.max() < 2e-5, rel.max()
    if kind == "svgd":
        idx = np.arange(m)
        np.testing.assert_array_equal(Ch[idx, idx], Ce[idx, idx])


@pytest.mark.parametrize("m,n,d", [(1024, 1024, 256), (300, 900, 37), (2048, 4096, 64)])
def test_w2_cost_h2_line_stores_identical(m, n, d):
    """dsvgd_w2_set_cost_lines: C written as whole 128-byte row lines (two
    slices' values traded between lane pairs) and as half lines -- the same
    bits everywhere, ragged tiles included."""
    lib = dsvgd()._native.load()
    rs = np.random.RandomState(m + n + d + 5)
    X = rs.randn(m, d).astype(np.float32)
    P = rs.randn(n, d).astype(np.float32)
    P[:min(m, n)] = X[:min(m, n)] - 1e-3 * rs.randn(min(m, n), d).astype(np.float32)
    out = {}
    for lines in (1, 0):
        prev = lib.dsvgd_w2_set_cost_lines(lines)
        try:
            out[lines] = _w2_cost(X, P, "h2")
        finally:
            lib.dsvgd_w2_set_cost_lines(prev)
    np.testing.assert_array_equal(out[1], out[0])


@pytest.mark.parametrize("name", W2_GOLDEN)
def test_w2_h2_cost_golden_plans(golden, name):
    """The golden LPs (reference linprog plans, near-tie sets included) on the
    MFMA cost form (forced; W2Term takes it from 2^22 entries by default):
    the same plans and gradients."""
    W2 = dsvgd().w2.W2Term
    old = W2.COST
    W2.COST = "h2"
    try:
        g = golden(name)
        G, plan, w = _w2_gpu(g["X"], g["P"], h=1.0)
        assert w.cost == "h2"
    finally:
        W2.COST = old
    err = abs_err(G, g["grad"]) / max(np.abs(g["grad"]).max(), 1e-30)
    assert err < PHI_TOL, err
    m = g["X"].shape[0]
    np.testing.assert_array_equal(_row_sets(plan, m), _row_sets(O.w2_plan(O.w2_cost(g["X"], g["P"])), m))


@pytest.mark.parametrize("m,n,d,near", [(256, 256, 16, None), (512, 1024, 8, None),
                                        (2048, 2048, 64, None), (1024, 1024, 32, 0.05),
                                        (1024, 4096, 8, 0.01), (512, 4096, 16, "svgd"),
                                        (4096, 4096, 256, "svgd"), (2048, 16384, 256, "svgd")])
def test_w2_h2_cost_same_plan_as_exact(m, n, d, near):
    """Plans on the MFMA cost form == plans on the exact VALU cost form ==
    scipy's assignment (up to 4096 x 4096), R = 1 .. 8, random and
    SVGD-shaped (the owned rows' previous copies among the columns)."""
    rs = np.random.RandomState(m + n + d + 3)
    X = rs.randn(m, d).astype(np.float32)
    if near is None:
        P = rs.randn(n, d).astype(np.float32)
    elif near == "svgd":
        P = rs.randn(n, d).astype(np.float32)
        P[:m] = X - 1e-3 * rs.randn(m, d).astype(np.float32)
    else:
        P = (np.tile(X, (n // m, 1)) + near * rs.randn(n, d)).astype(np.float32)
    W2 = dsvgd().w2.W2Term
    old = W2.COST
    plans = {}
    try:
        for form in ("h2", "exact"):
            W2.COST = form
            G, plan, w = _w2_gpu(X, P, h=2.5)
            assert w.cost == form
            plans[form] = (plan, G)
    finally:
        W2.COST = old
    np.testing.assert_array_equal(_row_sets(plans["h2"][0], m), _row_sets(plans["exact"][0], m))
    # (the same row sets; the slots of a row may hold them in another order, so the
    # gradient's sum over a row's columns may round differently in the last bits)
    Gh, Ge = plans["h2"][1], plans["exact"][1]
    assert np.abs(Gh - Ge).max() <= 1e-6 * np.abs(Ge).max()
    if m * n <= 4096 * 4096 and d <= 64:
        ref_plan = O.w2_plan(O.w2_cost(X, P))
        np.testing.assert_array_equal(_row_sets(plans["h2"][0], m), _row_sets(ref_plan, m))


# ------------------------------------------ DistSampler, 2 ranks, 1 GPU --
def _dist_gpu_worker(rank, S, port, name, order, q, median=False):
    import os
    import sys
    import torch.distributed as dist
    from conftest import GOLDEN, PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    x, t = g["x_train"], g["t_train"]
    per = x.shape[0] // S
    mode = str(g["mode"])
    tgt = m.targets.LogisticRegression(x[rank * per:(rank + 1) * per], t[rank * per:(rank + 1) * per])
    parts = torch.tensor(g["init"][rank], device=DEV)
    w2 = bool(g["w2"]) if "w2" in g else False
    hjko = float(g["hjko"]) if "hjko" in g else 10.0
    ds = m.DistSampler(rank, S, tgt, m.RBF("median" if median else 1.0), parts, per, per * S,
                       exchange_particles=mode in ("all_particles", "all_scores"),
                       exchange_scores=mode == "all_scores", include_wasserstein=w2,
                       order=order)
    out = []
    for _ in range(int(g["steps"])):
        ds.make_step(float(g["eps"]), h=hjko)
        out.append((ds.particles.cpu().numpy(), ds._particles.cpu().numpy(), ds._particle_start_idx))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


DIST_S2 = (["g4_dist_s2_" + m for m in ("partitions", "all_particles", "all_scores")]
           + ["g5_dist_s2_%s_w2" % m for m in ("partitions", "all_particles", "all_scores")])


@pytest.mark.parametrize("name", DIST_S2)
def test_distsampler_two_ranks_match_reference(golden, name):
    """Two ranks share cuda:0 (gloo for the exchange; kernels on the GPU);
    g5_*: include_wasserstein=True, the W2/JKO term from the second step."""
    import torch.multiprocessing as mp
    g = golden(name)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + DIST_S2.index(name)
    ps = [ctx.Process(target=_dist_gpu_worker, args=(r, 2, port, name, "sequential", q))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, out in res:
        for step, (own, full, start) in enumerate(out):
            assert start == int(g["start"][rank][step])
            assert abs_err(own, g["own"][rank][step]) < TRAJ_TOL
            assert abs_err(full, g["full"][rank][step]) < TRAJ_TOL


def _dist_median_worker(rank, S, port, X, d, steps, eps, q):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    mu = np.zeros(d, np.float32)
    lam = np.ones(d, np.float32)
    parts = torch.tensor(X, device=DEV)
    ds = m.DistSampler(rank, S, m.targets.Gaussian(mu, lam), m.RBF("median"), parts,
                       1, 1, exchange_particles=True, exchange_scores=False,
                       include_wasserstein=False, order="jacobi")
    hs = []
    for _ in range(steps):
        ds.make_step(eps)
        eng = next(iter(ds._engines.values()))
        hs.append((eng.bracketed, eng.state.read()[1], eng.state.bracket()[4]))
    q.put((rank, ds.particles.cpu().numpy(), hs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,d,S", [(6000, 16, 2), (6000, 80, 2), (6144, 80, 2),
                                   (8192, 80, 4), (8192, 64, 8)])
def test_distsampler_median_multi_rank_jacobi(n, d, S):
    """Row-sharded D over S ranks sharing cuda:0 (all-reduced counts and
    histograms) vs the oracle's global-median Jacobi step.  Owned blocks of
    >= 2^24 entries take the bracketed select, smaller ones (S = 8 here) the
    all-reduced radix passes.  n = 6144 / 8192: 256-row aligned blocks, whose
    distance pass computes the diagonal square's upper triangle (+ mirror) and
    the rectangles beside it in separate launches (S = 4 / 8: interior ranks
    with rectangles on both sides, the bench's S = 8 geometry scaled down)."""
    import torch.multiprocessing as mp
    steps, eps = 2, 0.05
    X = np.random.RandomState(d).randn(n, d).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_median_worker, args=(r, S, 29830 + d + n % 7 + 10 * S, X, d, steps, eps, q))
          for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ref = np.array(X, np.float64)
    for _ in range(steps):
        ref = ref + eps * O.phi(ref, -ref, O.median_bandwidth(ref)[0])
    got = np.concatenate([r[1] for r in res])
    assert abs_err(got, ref) < TRAJ_TOL
    for _, _, hs in res:
        for bracketed, h, fallback in hs:
            assert bracketed == ((n // S) * n >= (1 << 24))
            assert not bracketed or fallback == 0
    for r in res[1:]:
        assert r[2] == res[0][2]             # identical h on every rank


@pytest.mark.parametrize("name", DIST_S2)
def test_distsampler_two_ranks_jacobi_vs_oracle(golden, name):
    """Jacobi DistSampler over 2 ranks (the all_scores path overlaps the score
    all-reduce with the distance stage) vs the oracle's Jacobi DistSampler."""
    import torch.multiprocessing as mp
    g = golden(name)
    mode = str(g["mode"])
    w2 = bool(g["w2"]) if "w2" in g else False
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29860 + DIST_S2.index(name)
    ps = [ctx.Process(target=_dist_gpu_worker, args=(r, 2, port, name, "jacobi", q))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    x, t = g["x_train"], g["t_train"]
    per = x.shape[0] // 2
    fns = [(lambda X, r=r: O.score_logreg(X, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]))
           for r in range(2)]
    D = O.DistOracle(list(g["init"]), fns, per, 2 * per,
                     exchange_particles=mode != "partitions", exchange_scores=mode == "all_scores",
                     h=1.0, sequential=False, include_wasserstein=w2)
    for step in range(int(g["steps"])):
        D.step(float(g["eps"]), float(g["hjko"]) if "hjko" in g else 10.0)
        for rank, out in res:
            own, full, start = out[step]
            assert start == D.start[rank]
            assert abs_err(own, D.own(rank)) < TRAJ_TOL


# ------------------------------------ logreg: test accuracy after T steps --
def _banana_like(N, p=2, seed=0, w_seed=1, noise_seed=2):
    """Synthetic stand-in for benchmarks.mat 'banana' (an LFS pointer in the
    reference): x ~ N(0, I), t = sign(x.w* + logistic noise)."""
    x = np.random.RandomState(seed).randn(N, p).astype(np.float32)
    w = np.random.RandomState(w_seed).randn(p)
    z = x @ w + np.random.RandomState(noise_seed).logistic(size=N)
    return x, np.where(z > 0, 1.0, -1.0).astype(np.float32)


@pytest.mark.parametrize("order,n,T", [("sequential", 100, 100), ("jacobi", 1024, 100)])
def test_logreg_test_accuracy_after_T_steps(order, n, T):
    """experiments/logreg.py config A (S = 1, partitions, eps = 1e-3, h = 10,
    rank-0 reference init) for T steps: particles vs the oracle, then the
    posterior mean / variance and the posterior-predictive test accuracy of
    logreg_plots.py:42-50 on 4900 held-out points."""
    x, t = _banana_like(400)
    x_test, t_test = _banana_like(4900, seed=10, noise_seed=12)
    X0 = O.ref_init(n, 3, 0)
    ds = dsvgd().DistSampler(0, 1, dsvgd().targets.LogisticRegression(x, t), dsvgd().RBF(1.0),
                             torch.tensor(X0), 400, 400, exchange_particles=False,
                             exchange_scores=False, include_wasserstein=False, order=order)
    for _ in range(T):
        ds.make_step(1e-3, h=10.0)
    got = ds.particles.numpy().astype(np.float64)
    fn = lambda X: O.score_logreg(X, x, t)  # noqa: E731
    D = O.DistOracle([X0], [fn], 400, 400, False, False, sequential=order == "sequential")
    for _ in range(T):
        D.step(1e-3)
    ref = D.own(0)
    err = abs_err(got, ref)
    assert err < 1e-3, err
    # posterior mean / variance of the weights: same algorithm, so far inside MC error
    se = np.sqrt(ref[:, 1:].var(0) / n)
    assert np.all(np.abs(got[:, 1:].mean(0) - ref[:, 1:].mean(0)) < 0.01 * se + 1e-5)
    assert np.all(np.abs(got[:, 1:].var(0) / ref[:, 1:].var(0) - 1) < 1e-3)
    acc_gpu = dsvgd().metrics.test_accuracy(ds._work, x_test, t_test)   # on the GPU
    assert acc_gpu == O.test_accuracy(got, x_test, t_test)
    acc_ref = O.test_accuracy(ref, x_test, t_test)
    record_parity(err, acc_gpu=acc_gpu, acc_oracle=acc_ref)
    assert abs(acc_gpu - acc_ref) <= 0.01
    assert acc_gpu > 0.6        # the posterior predicts (chance is ~0.5)


@pytest.mark.parametrize("n,d,Nt", [(100, 3, 4900), (1000, 256, 3000), (300, 1024, 129),
                                    (4200, 33, 1)])
def test_predictive_prob_and_test_accuracy(n, d, Nt):
    """dsvgd.metrics (dsvgd_logreg_predict) vs the fp64 restatement of
    logreg_plots.py:42-50: ensemble-mean probabilities within 2e-6 absolute;
    the accuracy identical except for test points within 1e-5 of 0.5."""
    rs = np.random.RandomState(n + d)
    P = (rs.randn(n, d) * 0.5).astype(np.float32)
    xt = (rs.randn(Nt, d - 1) / np.sqrt(d)).astype(np.float32)
    tt = np.where(rs.randn(Nt) > 0, 1.0, -1.0).astype(np.float32)
    prob = dsvgd().metrics.predictive_prob(gpu(P), xt).cpu().numpy()
    ref = O.predictive_prob(P, xt)
    assert abs_err(prob, ref) < 2e-6
    acc = dsvgd().metrics.test_accuracy(gpu(P), xt, tt)
    sure = np.abs(ref - 0.5) > 1e-5
    agree = ((ref > 0.5) == (tt > 0))
    lo, hi = agree[sure].sum() / Nt, (agree[sure].sum() + (~sure).sum()) / Nt
    assert lo - 1e-12 <= acc <= hi + 1e-12


@pytest.mark.parametrize("m,d,dp,splits,extra,off", [(1000, 256, 256, 2, False, 0),
                                                       (513, 64, 64, 3, True, 0),
                                                       (300, 36, 64, 1, True, 0),
                                                       (200, 256, 256, 2, False, 1)])
def test_phi_finish_vec_same_bits(m, d, dp, splits, extra, off):
    """dsvgd_phi_set_finish_vec: four columns per thread (16-byte accesses)
    gives the same phi and the same updated X bits as one element per thread
    (the split-K partials summed in slice order, the self term, extra rows);
    off = 1 misaligns X so the call falls back to the scalar kernel."""
    from dsvgd import _native as N
    from dsvgd.engine import SelectState
    dsvgd()
    lib = N.load()
    g = torch.Generator(device="cpu").manual_seed(m + d)
    ldk, ldy, row0 = 2 * dp, 2 * dp, 7
    mp = (m + 127) // 128 * 128
    KY = torch.randn(splits * m * ldk, generator=g).to(DEV)
    rs = torch.rand(splits * mp, generator=g).to(DEV)
    Y = torch.randn((row0 + m) * ldy, generator=g).to(DEV)
    ex = torch.randn(m * d, generator=g).to(DEV) if extra else None
    X0 = torch.randn(m * d + 4, generator=g).to(DEV)
    st = SelectState(DEV)
    N.call("dsvgd_set_bandwidth", st.ptr, 3.7, N.stream(DEV))
    out = {}
    prev = lib.dsvgd_phi_set_finish_vec(1)
    try:
        for vec in (1, 0):
            lib.dsvgd_phi_set_finish_vec(vec)
            phi = torch.empty(m * d, device=DEV)
            X = X0.clone()
            Xv = X[off:off + m * d]
            N.call("dsvgd_phi_finish", N.ptr(KY), ldk, N.ptr(rs), splits, N.ptr(Y), ldy, row0, m,
                   d, dp, st.ptr, 1.0 / 4096, 0.01, N.ptr(ex) if extra else None, d, N.ptr(phi), d,
                   N.ptr(Xv), d, N.stream(DEV))
            torch.cuda.synchronize()
            out[vec] = (phi.cpu(), X.cpu())
    finally:
        lib.dsvgd_phi_set_finish_vec(prev)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert bool(torch.isfinite(out[1][0]).all())
