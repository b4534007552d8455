"""CPU ORACLE for the SVGD particle update -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (dist-svgd_amd/dsvgd) never imports it and has no CPU compute path.

An independent numpy restatement (fp64 by default) of the reference algorithm
(Sandy4321/dist-svgd, paths relative to that tree):

  * phi on frozen particles ............ dsvgd/sampler.py:35-40, dsvgd/distsampler.py:84-101
      phi_i = 1/n sum_j [ k(x_j,x_i) s_j + grad_{x_j} k(x_j,x_i) ],  k = exp(-|x-y|^2/h)
      grad_{x_j} k(x_j, x_i) = (2/h) (x_i - x_j) k  (autograd of experiments/logreg.py:60-61)
  * Gauss-Seidel sweeps ................ dsvgd/sampler.py:62-74 (in-place row update, :68)
  * DistSampler.make_step .............. dsvgd/distsampler.py:172-205 for S simulated
    ranks: partitions ring shift (:131-150), all_particles all_gather (:152-158),
    all_scores all_reduce (:160-170), N_global/N_local score scaling (:97-99)
  * target scores (closed-form autograd of) experiments/gmm.py:16-21,
    experiments/logreg.py:45-58 and the synthetic Gaussian N(mu, diag(1/lam))
  * median bandwidth (absent from the reference): lower median
    k=(n^2-1)//2 of the full n x n squared-distance matrix, h = median / log n.

Parity pinning: checked against the golden vectors in tests/golden/*.npz, which
tests/golden/make_golden.py produced by running the reference itself.
"""
import math

import numpy as np


# ------------------------------------------------------------------ scores --
def score_gaussian(X, mu, lam):
    X = np.asarray(X, np.float64)
    return -np.asarray(lam, np.float64) * (X - np.asarray(mu, np.float64))


def score_gmm(X):
    """d/dx log(1/3 N(x;-2,1) + 1/3 N(x;2,1)) per coordinate (gmm.py:19-21)."""
    X = np.asarray(X, np.float64)
    a = -0.5 * (X + 2.0) ** 2
    b = -0.5 * (X - 2.0) ** 2
    m = np.maximum(a, b)
    ea, eb = np.exp(a - m), np.exp(b - m)
    return -(ea * (X + 2.0) + eb * (X - 2.0)) / (ea + eb)


def score_logreg(X, x_train, t_train):
    """grad of logreg.py:45-58: x = [log alpha, w]; Gamma(1,1) prior on alpha
    (no log-Jacobian), N(0, I/alpha) prior on w, logistic likelihood."""
    X = np.asarray(X, np.float64)
    xd = np.asarray(x_train, np.float64)
    t = np.asarray(t_train, np.float64).reshape(-1)
    rows = max(1, (1 << 27) // max(1, xd.shape[0]))      # bound the (rows, N) Z block
    if X.shape[0] > rows:
        return np.concatenate([score_logreg(X[s:s + rows], xd, t)
                               for s in range(0, X.shape[0], rows)])
    a = np.exp(X[:, 0])
    W = X[:, 1:]
    p = W.shape[1]
    Z = W @ xd.T                              # (n, N)
    G = t[None, :] * _sigmoid(-t[None, :] * Z)
    S = np.empty_like(X)
    S[:, 0] = -a + 0.5 * p - 0.5 * a * (W * W).sum(1)
    S[:, 1:] = G @ xd - a[:, None] * W
    return S


def _sigmoid(u):
    out = np.empty_like(u)
    pos = u >= 0
    out[pos] = 1.0 / (1.0 + np.exp(-u[pos]))
    e = np.exp(u[~pos])
    out[~pos] = e / (1.0 + e)
    return out


# ------------------------------------------------------------- bandwidth --
GRAM_MIN_WORK = 1 << 31


def sqdist(Xr, X, self_cols=None):
    """||x_i - x_j||^2 from explicit differences (as torch.dist**2 per pair),
    chunked over rows to bound memory.  Large problems (rows * n * d >=
    GRAM_MIN_WORK, e.g. 256 sampled rows of config E: 65536 x 1024) take the
    fp64 Gram form of sqdist_gram instead, which a CPU test pins to this one.
    self_cols[k]: the column of X that row k of Xr is (its distance is exactly
    0; the Gram form would leave fp64 rounding of |x|^2 there)."""
    Xr = np.asarray(Xr, np.float64)
    X = np.asarray(X, np.float64)
    if Xr.shape[0] * X.size >= GRAM_MIN_WORK:
        out = sqdist_gram(Xr, X)
        if self_cols is not None:
            out[np.arange(Xr.shape[0]), np.asarray(self_cols)] = 0.0
        return out
    out = np.empty((Xr.shape[0], X.shape[0]))
    step = max(1, (1 << 24) // max(1, X.size))
    for s in range(0, Xr.shape[0], step):
        out[s:s + step] = ((Xr[s:s + step, None, :] - X[None, :, :]) ** 2).sum(-1)
    return out


def sqdist_gram(Xr, X):
    """fp64 ||a||^2 + ||b||^2 - 2 a.b about the coordinate-wise median of X
    (translation invariant; unlike the mean it stays inside the bulk when
    one particle is far away), clamped at 0; fp64 keeps the cancellation
    error ~1e-16 |x|^2, far below the 1e-5 fp32 tolerances."""
    X = np.asarray(X, np.float64)
    mu = np.median(X, 0)
    A = np.asarray(Xr, np.float64) - mu
    B = X - mu
    out = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2.0 * (A @ B.T)
    np.maximum(out, 0.0, out=out)
    return out


def lower_median(values):
    """k-th smallest, k = (N-1)//2 (== torch.median semantics on a flat tensor)."""
    v = np.asarray(values).ravel()
    k = (v.size - 1) // 2
    return np.partition(v, k)[k]


def median_bandwidth(X):
    """h = lower_median(D) / log(n) over the full n x n matrix (diag included);
    h = 1 when n <= 1 or the median is 0 (all particles coincide)."""
    X = np.asarray(X, np.float64)
    n = X.shape[0]
    med = float(lower_median(sqdist(X, X, self_cols=np.arange(n))))
    if n <= 1 or med <= 0.0:
        return 1.0, med
    return med / math.log(n), med


# ------------------------------------------------------------------- phi --
def phi(X, S, h, rows=None):
    """Jacobi phi for `rows` (default all) against the frozen set X (n x d)."""
    X = np.asarray(X, np.float64)
    S = np.asarray(S, np.float64)
    Xr = X if rows is None else X[rows]
    self_cols = np.arange(X.shape[0]) if rows is None else np.asarray(rows).reshape(-1)
    K = np.exp(-sqdist(Xr, X, self_cols) / h)  # K[i, j] = k(x_j, x_i)
    n = X.shape[0]
    rep = (2.0 / h) * (K.sum(1)[:, None] * Xr - K @ X)
    return (K @ S + rep) / n


def phi_pairloop_row(i, X, score_fn, h):
    """Literal restatement of the per-pair loop (sampler.py:36-40), one row."""
    X = np.asarray(X, np.float64)
    x = X[i]
    total = np.zeros_like(x)
    for xj in X:
        k = math.exp(-float(((xj - x) ** 2).sum()) / h)
        total += k * score_fn(xj[None, :])[0] + (2.0 / h) * (x - xj) * k
    return total / X.shape[0]


# ----------------------------------------------- Sampler (Gauss-Seidel) --
def sampler_sequential(X0, score_fn, h, num_iter, step_size, dtype=np.float64):
    """sampler.py:62-74: returns the history (num_iter+1, n, d); history[l] is
    the particle set at the start of sweep l (== what the reference records
    for every particle right before its own update)."""
    X = np.array(X0, dtype=dtype)
    n = X.shape[0]
    hist = [X.copy()]
    for _ in range(num_iter):
        for i in range(n):
            S = score_fn(X)
            p = phi(X, S, h, rows=[i])[0]
            X[i] = X[i] + step_size * p
        hist.append(X.copy())
    return np.stack(hist)


def sequential_sweep(X, S, h, rows, step, score_fn=None, extra=None, block=64):
    """One Gauss-Seidel sweep over `rows` (sampler.py:64-68: row i moves with
    phi_i of the CURRENT particles, its score refreshed after the move when
    score_fn is given), in place on fp64 copies; returns (X, S, phi rows).

    The same arithmetic as looping O.phi(X, S, h, rows=[i]) row by row (a CPU
    test pins the two), organised in blocks so full-size sweeps finish: a
    block's interactions with every row outside the rows moved before it are
    one matrix product, the in-block terms a short loop."""
    X = np.array(X, np.float64)
    S = np.array(S, np.float64)
    rows = list(rows)
    n = X.shape[0]
    out = np.zeros((len(rows), X.shape[1]))
    for b in range(0, len(rows), block):
        idx = np.array(rows[b:b + block])
        # the block's rows against all n as the block starts (large: the fp64
        # centred Gram, pinned to the explicit differences by a CPU test)
        if len(idx) * X.size >= (1 << 26):
            D = sqdist_gram(X[idx], X)
            D[np.arange(len(idx)), idx] = 0.0
        else:
            D = sqdist(X[idx], X, self_cols=idx)
        K = np.exp(-D / h)
        # terms with block rows moved before i are recomputed below
        for a, i in enumerate(idx):
            K[a, idx[:a]] = 0.0
        xi = X[idx].copy()
        Q = K @ S + (2.0 / h) * (K.sum(1)[:, None] * xi - K @ X)
        for a, i in enumerate(idx):
            moved = idx[:a]
            p = Q[a].copy()
            if len(moved):
                km = np.exp(-((xi[a][None, :] - X[moved]) ** 2).sum(1) / h)
                p += km @ S[moved] + (2.0 / h) * (km.sum() * xi[a] - km @ X[moved])
            p /= n
            if extra is not None:
                p = p + extra[b + a]
            out[b + a] = p
            X[i] = xi[a] + step * p
            if score_fn is not None:
                S[i] = score_fn(X[i:i + 1])[0]
    return X, S, out


def sampler_jacobi(X0, score_fn, h, num_iter, step_size, median=False):
    X = np.array(X0, np.float64)
    hist = [X.copy()]
    for _ in range(num_iter):
        hh = median_bandwidth(X)[0] if median else h
        X = X + step_size * phi(X, score_fn(X), hh)
        hist.append(X.copy())
    return np.stack(hist)


# ----------------------------------------------------- DistSampler (S ranks) --
# ------------------------------------------------------------ W2 / JKO --
def w2_cost(X, P):
    """C[i][j] = ||x_i - p_j||^2 in fp64 from explicit differences, as the
    reference builds `diffs` and `c` (distsampler.py:107-114)."""
    X = np.asarray(X, np.float64)
    P = np.asarray(P, np.float64)
    if X.shape[0] * P.shape[0] * X.shape[1] <= 1 << 26:
        return ((X[:, None, :] - P[None, :, :]) ** 2).sum(-1)
    return np.maximum(sqdist(X, P), 0.0)


def w2_plan(C):
    """Optimal plan of the reference LP (distsampler.py:115-126): minimise
    <P, C> over P >= 0 with row sums 1/m and column sums 1/n.  For n = R m the
    vertices are integral after replicating each row R times (supplies R,
    demands 1, scaled by n), so the LP optimum is an exact assignment of
    n slots (slot s -> row s // R) to n columns, each carrying mass 1/n.
    Returns the column of every slot (scipy's exact Hungarian solver)."""
    from scipy.optimize import linear_sum_assignment
    m, n = C.shape
    assert n % m == 0, "the reference LP is integral here only for n = R m"
    R = n // m
    rows, cols = linear_sum_assignment(np.repeat(C, R, axis=0))
    out = np.empty(n, np.int64)
    out[rows] = cols
    return out


def w2_grad(X, P, plan=None):
    """sum_j P_ij (x_i - p_j) (distsampler.py:128), P_ij = 1/n on the slots of
    row i.  Returns (grad (m, d) fp64, plan)."""
    X = np.asarray(X, np.float64)
    P = np.asarray(P, np.float64)
    m, n = X.shape[0], P.shape[0]
    if plan is None:
        plan = w2_plan(w2_cost(X, P))
    R = n // m
    g = (X[:, None, :] - P[plan].reshape(m, R, -1)).sum(1) / n
    return g, plan


class DistOracle:
    """All S ranks of DistSampler simulated in one process (distsampler.py:9-205).

    `particles[r]` is rank r's (n, d) copy; `score_fns[r](X)` the rank-local
    score grad log p_r (prior + local likelihood).  sequential=True follows the
    reference's in-place Gauss-Seidel order; False is the Jacobi variant.
    include_wasserstein adds the JKO term h_jko * w2_grad(own, previous) to
    every owned row's direction (distsampler.py:190-198) from the second step
    on; previous = all n rows after the sweep when particles are exchanged,
    else the owned block (:202-205).
    """

    def __init__(self, particles, score_fns, N_local, N_global, exchange_particles,
                 exchange_scores, h=1.0, sequential=True, include_wasserstein=False,
                 replicated=False, lagged=None):
        assert not (exchange_scores and not exchange_particles)
        self.S = len(particles)
        n = np.asarray(particles[0]).shape[0]
        self.per = int(n / self.S)
        self.n = self.per * self.S
        self.X = [np.array(p, np.float64)[:self.n].copy() for p in particles]
        self.score_fns = score_fns
        self.N_local, self.N_global = N_local, N_global
        self.xp, self.xs = exchange_particles, exchange_scores
        self.h = h
        self.sequential = sequential
        self.start = [r * self.per for r in range(self.S)]
        self.w2 = include_wasserstein
        self.prev = [None] * self.S
        # replicated data (all_particles, every rank holding the whole data
        # set): each rank scores its owned block, the blocks are gathered --
        # the same numbers as every rank scoring all n (identical score_fns)
        self.replicated = replicated and exchange_particles and not exchange_scores and self.S > 1
        # lagged modes (notes.md:108-114): full local copies, blocks travel
        # round-robin and land in their home rows; "local" moves the held
        # block against the whole copy, "updateall" moves the whole copy.
        # h = "median": the held block's own m x n lower median (updateall:
        # the copy's n x n), / log n
        assert lagged in (None, "local", "updateall")
        assert not (lagged and (exchange_particles or exchange_scores))
        self.lagged = lagged
        self.held = list(range(self.S))

    def own(self, r):
        return self.X[r][self.start[r]:self.start[r] + self.per]

    def _exchange(self):
        S = self.S
        if S <= 1:
            return None
        if self.xp:
            full = np.concatenate([self.own(r) for r in range(S)])
            for r in range(S):
                self.X[r][:] = full
            if self.xs:
                tot = sum(self.score_fns[r](full) for r in range(S))
                return [tot.copy() for _ in range(S)]
            if self.replicated:
                scale = self.N_global / self.N_local
                g = np.concatenate([scale * self.score_fns[r](self.own(r)) for r in range(S)])
                return [g.copy() for _ in range(S)]
            return None
        if self.lagged:
            sent = [(self.held[r], self.own(r).copy()) for r in range(S)]
            for r in range(S):
                b, rows = sent[(r - 1 + S) % S]
                self.held[r] = b
                self.start[r] = b * self.per
                self.X[r][self.start[r]:self.start[r] + self.per] = rows
            return None
        blocks = [self.own(r).copy() for r in range(S)]
        for r in range(S):
            src = (r - 1 + S) % S
            s0 = src * self.per
            self.X[r][s0:s0 + self.per] = blocks[src]
            self.start[r] = s0
        return None

    def step(self, step_size, h_jko=1.0):
        scores = self._exchange()
        if scores is None and self.xs:      # S == 1 with exchange_scores: local scores
            scores = [self.score_fns[r](self.X[r]) for r in range(self.S)]
        for r in range(self.S):
            Xr = self.X[r]
            s0, s1 = self.start[r], self.start[r] + self.per
            lo, hi = (0, self.n) if (self.xp or self.lagged) else (s0, s1)
            if self.lagged == "updateall":
                s0, s1 = 0, self.n
            h = self.h
            if h == "median":     # all_particles: the global n x n (identical copies)
                med = lower_median(sqdist(Xr[lo:hi] if self.xp else Xr[s0:s1], Xr[lo:hi]))
                h = med / math.log(hi - lo) if (hi - lo > 1 and med > 0) else 1.0
            scale = 1.0 if self.xs else self.N_global / self.N_local
            extra = np.zeros((s1 - s0, Xr.shape[1]))
            if self.w2 and self.prev[r] is not None:
                extra = h_jko * w2_grad(Xr[s0:s1], self.prev[r])[0]
            if self.sequential:
                for i in range(s0, s1):
                    Xi = Xr[lo:hi]
                    if self.xs:
                        Sj = scores[r][lo:hi]
                    elif self.replicated:        # gathered blocks frozen, owned rows current
                        Sj = scores[r].copy()
                        Sj[s0:s1] = scale * self.score_fns[r](Xr[s0:s1])
                    else:
                        Sj = scale * self.score_fns[r](Xi)
                    Xr[i] += step_size * (phi(Xi, Sj, h, rows=[i - lo])[0] + extra[i - s0])
            else:
                Xi = Xr[lo:hi].copy()
                Sj = scores[r][lo:hi] if (self.xs or self.replicated) else \
                    scale * self.score_fns[r](Xi)
                Xr[s0:s1] += step_size * (phi(Xi, Sj, h, rows=np.arange(s0 - lo, s1 - lo))
                                          + extra)
            if self.w2:
                self.prev[r] = (Xr if self.xp else Xr[s0:s1]).copy()


# --------------------------------------------------------------- metric --
def predictive_prob(particles, x_test):
    """logreg_plots.py:44-48: mean over particles of expit(x_test . w), w = x[1:]."""
    P = np.asarray(particles, np.float64)
    return _sigmoid(np.asarray(x_test, np.float64) @ P[:, 1:].T).mean(1)


def test_accuracy(particles, x_test, t_test):
    """logreg_plots.py:42-50: posterior-predictive ensemble accuracy."""
    prob = predictive_prob(particles, x_test)
    return float(((prob > 0.5) == (np.asarray(t_test).reshape(-1) > 0)).mean())


def ref_init(n, d, seed):
    """Reference init (sampler.py:58-60): n successive Normal(0,1).sample((d,1))
    draws from torch's global CPU generator (== n successive torch.randn(d,1))."""
    import torch
    torch.manual_seed(seed)
    return torch.cat([torch.randn(d, 1) for _ in range(n)], dim=1).t().contiguous().numpy()
