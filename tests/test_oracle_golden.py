"""Pin the CPU oracle to the reference: every golden vector in tests/golden/
(produced by running the reference itself, see tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import svgd_oracle as O

PHI_TOL = 1e-5      # north_star: 1e-5 relative per step on phi (max-normalised)
TRAJ_TOL = 1e-4     # Gauss-Seidel trajectory, fp64 oracle vs fp32 reference


def score_fn_for(g):
    tgt = str(g["target"])
    if tgt == "gmm":
        return O.score_gmm
    if tgt == "gaussian":
        return lambda X: O.score_gaussian(X, g["mu"], g["lam"])
    if tgt == "logreg":
        return lambda X: O.score_logreg(X, g["x_train"], g["t_train"])
    raise KeyError(tgt)


@pytest.mark.parametrize("name", ["g1_gmm_n64", "g1_gauss_n128_d8_medh", "g1_gauss_n64_d64_h1",
                                  "g1_logreg_n100"])
def test_phi_matches_reference(golden, name):
    g = golden(name)
    X, ref = g["X"], g["phi"]
    got = O.phi(X, score_fn_for(g)(X), float(g["h"]))
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < PHI_TOL, err


def test_median_h_fixture_definition(golden):
    g = golden("g1_gauss_n128_d8_medh")
    h, med = O.median_bandwidth(g["X"])
    assert abs(h - float(g["h"])) <= 1e-12 * h


def test_pairloop_matches_vectorised(golden):
    g = golden("g1_logreg_n100")
    X = g["X"].astype(np.float64)
    fn = score_fn_for(g)
    full = O.phi(X, fn(X), 1.0)
    for i in (0, 17, 99):
        row = O.phi_pairloop_row(i, X, fn, 1.0)
        assert np.abs(row - full[i]).max() <= 1e-12 * np.abs(full).max()


@pytest.mark.parametrize("name", ["g2_sample_gauss_n32_d2", "g2_sample_gmm_n50"])
def test_sampler_trajectory(golden, name):
    g = golden(name)
    n, d, T = int(g["n"]), int(g["d"]), int(g["T"])
    X0 = O.ref_init(n, d, int(g["seed"]))
    np.testing.assert_array_equal(X0, g["values"][0])     # bit-exact reference init
    hist = O.sampler_sequential(X0, score_fn_for(g), float(g["h"]), T, float(g["eps"]))
    assert np.abs(hist - g["values"]).max() < TRAJ_TOL
    # history layout of sampler.py:66,73: rows ordered (timestep, particle)
    np.testing.assert_array_equal(g["timestep"], np.repeat(np.arange(T + 1), n))
    np.testing.assert_array_equal(g["particle"], np.tile(np.arange(n), T + 1))


def _dist_oracle(g, sequential=True):
    S, n = int(g["S"]), int(g["n"])
    mode = str(g["mode"])
    x, t = g["x_train"], g["t_train"]
    per = x.shape[0] // S
    fns = [(lambda X, r=r: O.score_logreg(X, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]))
           for r in range(S)]
    return O.DistOracle(list(g["init"]), fns, per, per * S,
                        exchange_particles=mode in ("all_particles", "all_scores"),
                        exchange_scores=mode == "all_scores", h=1.0, sequential=sequential,
                        include_wasserstein=bool(g["w2"]) if "w2" in g else False)


W2_DIRECT = ["g5_w2_m8_n8_d2", "g5_w2_m12_n12_d3", "g5_w2_m8_n16_d3", "g5_w2_m6_n24_d5",
             "g5_w2_m16_n32_d4_near", "g5_w2_m24_n24_d3_near"]
W2_DIST = ["g5_dist_s2_%s_w2" % m for m in ("partitions", "all_particles", "all_scores")]


@pytest.mark.parametrize("name", W2_DIRECT)
def test_w2_grad_matches_reference_lp(golden, name):
    """The exact-assignment restatement == the reference's linprog plan
    (distsampler.py:103-129), including replicated rows (n = R m)."""
    g = golden(name)
    got, plan = O.w2_grad(g["X"], g["P"])
    ref = g["grad"]
    # HiGHS returns the vertex to its ~1e-9 feasibility tolerance; a different
    # assignment would move a row by |x - y| / n ~ 1e-2
    assert np.abs(got - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())
    n, m = g["P"].shape[0], g["X"].shape[0]
    assert sorted(plan.tolist()) == list(range(n))           # a permutation of the columns
    C = O.w2_cost(g["X"], g["P"])
    assert C.shape == (m, n)


@pytest.mark.parametrize("name", ["g3_dist_s1_partitions"] + [
    "g4_dist_s%d_%s" % (S, m) for S in (2, 4) for m in ("partitions", "all_particles", "all_scores")]
    + W2_DIST)
def test_distsampler_steps(golden, name):
    g = golden(name)
    D = _dist_oracle(g)
    for step in range(int(g["steps"])):
        D.step(float(g["eps"]), float(g["hjko"]) if "hjko" in g else 1.0)
        for r in range(D.S):
            assert D.start[r] == int(g["start"][r][step])
            assert np.abs(D.own(r) - g["own"][r][step]).max() < TRAJ_TOL
            assert np.abs(D.X[r] - g["full"][r][step]).max() < TRAJ_TOL


def test_scores_match_autograd():
    """Closed-form scores == torch autograd of the reference closures."""
    import torch
    from oracle.loop_baseline import logreg_logp, _dlogp
    rs = np.random.RandomState(0)
    x, t = rs.randn(50, 3).astype(np.float32), np.sign(rs.randn(50)).astype(np.float32)
    X = rs.randn(7, 4).astype(np.float32)
    lp = logreg_logp(x, t)
    ref = np.stack([_dlogp(lp, torch.tensor(X[i])).numpy() for i in range(7)])
    got = O.score_logreg(X, x, t)
    assert np.abs(got - ref).max() < 1e-4 * max(1.0, np.abs(ref).max())


def test_sqdist_gram_form_matches_explicit_differences():
    """The fp64 Gram form the oracle takes for large problems (sqdist_gram)
    agrees with the explicit-difference form on the same inputs, including
    particles far from the origin (the centring keeps it well conditioned)."""
    rs = np.random.RandomState(4)
    for n, d, off in ((300, 64, 0.0), (200, 1024, 0.0), (257, 17, 50.0)):
        X = rs.randn(n, d) + off
        rows = rs.choice(n, 40, replace=False)
        a = O.sqdist_gram(X[rows], X)
        b = ((X[rows][:, None, :] - X[None, :, :]) ** 2).sum(-1)
        assert np.abs(a - b).max() <= 1e-11 * b.max()


@pytest.mark.parametrize("S,sequential", [(2, True), (2, False), (4, False)])
def test_replicated_score_gather_equals_redundant_scoring(S, sequential):
    """Replicated data (all_particles, N_local == N_global): gathering the
    owners' block scores is the same step as every rank scoring all n
    particles (distsampler.py:94-99) when every rank holds the same data."""
    rs = np.random.RandomState(S)
    n, p = 16 * S, 3
    x, t = rs.randn(40, p), np.sign(rs.randn(40))
    init = [rs.randn(n, p + 1) * 0.5 for _ in range(S)]
    fns = [lambda X: O.score_logreg(X, x, t)] * S
    a = O.DistOracle(init, fns, 40, 40, True, False, sequential=sequential, replicated=True)
    b = O.DistOracle(init, fns, 40, 40, True, False, sequential=sequential, replicated=False)
    assert a.replicated and not b.replicated
    for _ in range(3):
        a.step(0.05)
        b.step(0.05)
    for r in range(S):
        assert np.abs(a.X[r] - b.X[r]).max() < 1e-12


def _lag_setup(S, n=24, p=3, seed=0, same=False):
    rs = np.random.RandomState(seed)
    x, t = rs.randn(30, p), np.sign(rs.randn(30))
    base = rs.randn(n, p + 1) * 0.5
    init = [base.copy() if same else rs.randn(n, p + 1) * 0.5 for _ in range(S)]
    fns = [(lambda X, r=r: O.score_logreg(X, x[10 * r % 30:], t[10 * r % 30:])) for r in range(S)]
    return init, fns


@pytest.mark.parametrize("lagged", ["local", "updateall"])
def test_lagged_modes_reduce_to_all_particles_s1(lagged):
    """S = 1: nothing travels, the held block is the whole set -> the
    all_particles / partitions step (both orders, fixed and median h)."""
    init, fns = _lag_setup(1)
    for seq in (True, False):
        for h in (1.0, "median"):
            a = O.DistOracle(init, fns, 30, 30, False, False, h=h, sequential=seq, lagged=lagged)
            b = O.DistOracle(init, fns, 30, 30, True, False, h=h, sequential=seq)
            for _ in range(2):
                a.step(0.05)
                b.step(0.05)
            assert np.abs(a.X[0] - b.X[0]).max() < 1e-12


def test_laggedlocal_first_step_is_all_particles_jacobi_step():
    """With identical local copies nothing is stale at step 1: each rank's
    received block moves exactly as in all_particles Jacobi (same data)."""
    S = 4
    init, _ = _lag_setup(S, same=True)
    rs = np.random.RandomState(1)
    x, t = rs.randn(30, 3), np.sign(rs.randn(30))
    fns = [lambda X: O.score_logreg(X, x, t)] * S
    a = O.DistOracle(init, fns, 30, 30, False, False, sequential=False, lagged="local")
    b = O.DistOracle(init, fns, 30, 30, True, False, sequential=False)
    a.step(0.05)
    b.step(0.05)
    for r in range(S):
        assert a.held[r] == (r - 1) % S
        assert np.abs(a.own(r) - b.own(a.held[r])).max() < 1e-12


def test_laggedlocal_block_travel():
    """Blocks go round the ring and land in their home rows: after S steps
    every rank holds its own block again, and a rank's copy of block b is
    the value b had when it last passed through."""
    S = 3
    init, fns = _lag_setup(S)
    a = O.DistOracle(init, fns, 30, 30, False, False, sequential=False, lagged="local")
    for step in range(1, 2 * S + 1):
        a.step(0.05)
        for r in range(S):
            assert a.held[r] == (r - step) % S
    # updateall moves every row of every copy
    u = O.DistOracle(init, fns, 30, 30, False, False, sequential=False, lagged="updateall")
    u.step(0.05)
    for r in range(S):
        assert np.all(np.abs(u.X[r] - init[r]).max(1) > 0)


@pytest.mark.parametrize("n,d,lo,hi,fn", [(200, 5, 0, 200, "gauss"), (150, 3, 17, 140, None),
                                          (90, 7, 5, 90, "gmm"),
                                          # 64-row blocks on the fp64 Gram path (64 n d >= 2^26)
                                          # with the logistic-regression score refreshed
                                          (4096, 256, 1000, 1130, "logreg")])
def test_blocked_sequential_restatement_equals_row_loop(n, d, lo, hi, fn):
    """O.sequential_sweep (blocked, for full-size checks) against the plain
    row-by-row restatement of sampler.py:64-68 (O.phi per row, score refreshed
    after each move): the same sweep to fp64 rounding (the Gram path's
    distances to its cancellation bound)."""
    rs = np.random.RandomState(n)
    X0 = 0.8 * rs.randn(n, d)
    mu, lam = rs.randn(d), rs.uniform(0.5, 2.0, d)
    xd = rs.randn(300, d - 1) / np.sqrt(d)
    td = np.where(rs.rand(300) < 0.5, -1.0, 1.0)
    score = {"gauss": lambda X: O.score_gaussian(X, mu, lam), "gmm": O.score_gmm, None: None,
             "logreg": lambda X: O.score_logreg(X, xd, td)}[fn]
    gram = fn == "logreg"
    if gram:
        X0 *= 0.1 / 0.8
    S0 = score(X0) if score else rs.randn(n, d)
    h, step = 0.8 * d + 0.3, 0.07
    extra = 0.01 * rs.randn(hi - lo, d)
    X, S = X0.copy(), S0.copy()
    ref_phi = np.zeros((hi - lo, d))
    for k, i in enumerate(range(lo, hi)):
        ref_phi[k] = O.phi(X, S, h, rows=[i])[0] + extra[k]
        X[i] += step * ref_phi[k]
        if score:
            S[i] = score(X[i:i + 1])[0]
    Xb, Sb, pb = O.sequential_sweep(X0, S0, h, range(lo, hi), step, score_fn=score, extra=extra,
                                    block=64 if gram else 16)
    tol = 1e-9 if gram else 1e-12
    assert np.abs(Xb - X).max() < tol and np.abs(pb - ref_phi).max() < tol * max(1.0, np.abs(ref_phi).max())
    assert np.abs(Sb - S).max() < 1e-10 * max(1.0, np.abs(S).max())
