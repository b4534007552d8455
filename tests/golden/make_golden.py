"""Generate the golden fixtures in tests/golden/*.npz by RUNNING THE REFERENCE.

This script is the only file in the repository that imports the reference
package (`/root/reference/dsvgd`).  It runs in the build container only; the
fixtures it writes are plain numpy arrays (inputs + the reference's outputs),
so nothing of the reference travels to the GPU box.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Targets and kernels below restate the reference experiments' closures:
  * RBF kernel            experiments/logreg.py:60-61, experiments/gmm.py:23-24
                          (optionally with a bandwidth h: exp(-||x-y||^2 / h))
  * GMM log-density       experiments/gmm.py:16-21 (equal 1/3 weights, as coded)
  * logreg log-posterior  experiments/logreg.py:45-58, with the labels held as a
                          float32 torch tensor (the numpy (N,1) * Tensor product
                          at logreg.py:57 raises TypeError on torch 2.10)
  * Gaussian              N(mu, diag(1/lam)), the survey's synthetic target
The golden outputs are the reference's own Sampler._phi_hat (sampler.py:35-40),
Sampler.sample (sampler.py:42-74), DistSampler.make_step
(distsampler.py:172-205, S = 1, 2, 4 under gloo, all three exchange modes) and
DistSampler._wasserstein_grad (distsampler.py:103-129, the W2/JKO LP; called
unbound with self=None -- it reads nothing from self -- and through make_step
with include_wasserstein=True).
"""
import contextlib
import io
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


def _ref():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import dsvgd  # noqa: E402  (reference package, read-only)
    return dsvgd


# ---------------------------------------------------------------- targets ---
def rbf(h=1.0):
    import torch

    def kernel(x, y):
        return torch.exp(-1. * torch.dist(x, y, p=2) ** 2 / h)
    return kernel


def gmm_logp():
    import torch
    from torch.distributions.normal import Normal
    p1, p2 = Normal(-2, 1), Normal(2, 1)

    def logp(x):
        return torch.log(1. / 3. * torch.exp(p1.log_prob(x)) + 1. / 3. * torch.exp(p2.log_prob(x)))
    return logp


def gauss_logp(mu, lam):
    import torch
    mu_t = torch.tensor(mu, dtype=torch.float32)
    lam_t = torch.tensor(lam, dtype=torch.float32)

    def logp(x):
        return -0.5 * (lam_t * (x - mu_t) ** 2).sum()
    return logp


def logreg_logp(x_train, t_train):
    import torch
    from torch.distributions.gamma import Gamma
    from torch.distributions.multivariate_normal import MultivariateNormal
    xt = torch.tensor(x_train, dtype=torch.float32)
    tt = torch.tensor(t_train, dtype=torch.float32).reshape(-1, 1)
    p = xt.shape[1]
    alpha_prior = Gamma(1, 1)

    def w_prior(alpha):
        return MultivariateNormal(torch.zeros(p), torch.eye(p) / alpha)

    def logp(x):
        alpha = torch.exp(x[0])
        w = x[1:].reshape(-1)
        lp = alpha_prior.log_prob(alpha)
        lp += w_prior(alpha).log_prob(w)
        lp += -torch.log(1. + torch.exp(-1. * torch.mv(tt * xt, w))).sum()
        return lp
    return logp


def banana_like(N=400, p=2, seed=0):
    """Synthetic stand-in for benchmarks.mat 'banana' (only an LFS pointer here)."""
    rs = np.random.RandomState(seed)
    x = rs.randn(N, p).astype(np.float32)
    w = np.random.RandomState(seed + 1).randn(p)
    z = x @ w + np.random.RandomState(seed + 2).logistic(size=N)
    t = np.where(z > 0, 1.0, -1.0).astype(np.float32)
    return x, t


def ref_init(n, d, seed):
    """Reference particle init (sampler.py:58-60, logreg.py:63-66)."""
    import torch
    from torch.distributions.normal import Normal
    torch.manual_seed(seed)
    q = Normal(0, 1)
    return torch.cat([q.sample((d, 1)) for _ in range(n)], dim=1).t()


def median_h(X):
    """Survey a18 definition, fp64: lower median of the full n x n squared
    distance matrix (diagonal included) divided by log(n)."""
    X = np.asarray(X, np.float64)
    D = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1).ravel()
    k = (D.size - 1) // 2
    return float(np.partition(D, k)[k] / np.log(X.shape[0]))


# ------------------------------------------------------------------ cases ---
def phi_case(name, X, logp, h, extra):
    dsvgd = _ref()
    import torch
    s = dsvgd.Sampler(X.shape[1], logp, rbf(h))
    Xt = torch.tensor(X, dtype=torch.float32)
    phi = torch.stack([s._phi_hat(Xt[i], Xt) for i in range(Xt.shape[0])]).numpy()
    np.savez(os.path.join(OUT, name + ".npz"), X=X.astype(np.float32), phi=phi,
             h=np.float64(h), **extra)
    print(name, X.shape, "max|phi|", np.abs(phi).max())


def sample_case(name, d, n, T, eps, logp, h, seed, extra):
    dsvgd = _ref()
    import torch
    torch.manual_seed(seed)
    s = dsvgd.Sampler(d, logp, rbf(h))
    with contextlib.redirect_stdout(io.StringIO()):
        df = s.sample(n, T, eps)
    vals = np.stack(df["value"].to_list()).reshape(T + 1, n, d)
    np.savez(os.path.join(OUT, name + ".npz"), values=vals,
             timestep=df["timestep"].to_numpy(), particle=df["particle"].to_numpy(),
             seed=np.int64(seed), n=np.int64(n), d=np.int64(d), T=np.int64(T),
             eps=np.float64(eps), h=np.float64(h), **extra)
    print(name, vals.shape)


def w2_case(name, m, n, d, seed, near=None):
    """_wasserstein_grad(particles (m,d), previous (n,d)) -> (m,d) float64.
    near: previous = particles (tiled n/m times) + near * noise, the shape the
    JKO term sees between consecutive SVGD steps."""
    dsvgd = _ref()
    import torch
    rs = np.random.RandomState(seed)
    X = rs.randn(m, d).astype(np.float32)
    if near is None:
        P = rs.randn(n, d).astype(np.float32)
    else:
        P = (np.tile(X, (n // m, 1)) + near * rs.randn(n, d)).astype(np.float32)
    g = dsvgd.DistSampler._wasserstein_grad(None, torch.tensor(X), torch.tensor(P))
    np.savez(os.path.join(OUT, name + ".npz"), X=X, P=P, grad=np.asarray(g, np.float64))
    print(name, (m, n, d), "max|grad|", np.abs(g).max())


def _dist_worker(rank, S, port, n, steps, eps, hjko, mode, x, t, q, w2=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    dsvgd = _ref()
    N = x.shape[0]
    per = N // S
    logp = logreg_logp(x[rank * per:(rank + 1) * per], t[rank * per:(rank + 1) * per])
    # logreg.py:24 seeds with rank.  .contiguous(): the reference's transposed
    # init tensor makes _exchange_round_robin's torch.empty_like receive buffer
    # non-contiguous, which dist.irecv rejects on torch 2.10 (values unchanged).
    parts = ref_init(n, x.shape[1] + 1, rank).contiguous()
    init = parts.clone().numpy()
    ds = dsvgd.DistSampler(rank, S, logp, rbf(1.0), parts, per, per * S,
                           exchange_particles=mode in ("all_particles", "all_scores"),
                           exchange_scores=mode == "all_scores",
                           include_wasserstein=w2)
    own, full, start = [], [], []
    for _ in range(steps):
        ds.make_step(eps, h=hjko)
        own.append(ds.particles.clone().numpy())
        full.append(ds._particles.clone().numpy())
        start.append(ds._particle_start_idx)
    q.put((rank, init, np.stack(own), np.stack(full), np.array(start)))
    dist.barrier()
    dist.destroy_process_group()


def dist_case(name, S, n, steps, eps, mode, port, w2=False, hjko=10.0):
    import torch.multiprocessing as mp
    x, t = banana_like(N=400)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker,
                         args=(r, S, port, n, steps, eps, hjko, mode, x, t, q, w2))
             for r in range(S)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(S)], key=lambda r: r[0])
    for p in procs:
        p.join()
        assert p.exitcode == 0
    np.savez(os.path.join(OUT, name + ".npz"), S=np.int64(S), n=np.int64(n),
             steps=np.int64(steps), eps=np.float64(eps), mode=np.array(mode),
             w2=np.bool_(w2), hjko=np.float64(hjko),
             x_train=x, t_train=t,
             init=np.stack([r[1] for r in res]), own=np.stack([r[2] for r in res]),
             full=np.stack([r[3] for r in res]), start=np.stack([r[4] for r in res]))
    print(name, "done")


def main(which=None):
    import torch
    torch.set_num_threads(1)
    cases = []
    # G1 -- phi on frozen particles (sampler.py:35-40)
    cases.append(("g1_gmm_n64", lambda: phi_case(
        "g1_gmm_n64", ref_init(64, 1, 42).numpy(), gmm_logp(), 1.0, {"target": np.array("gmm")})))

    def g1_gauss8():
        X = ref_init(128, 8, 7).numpy()
        mu = np.random.RandomState(1).randn(8).astype(np.float32)
        lam = np.random.RandomState(2).uniform(0.5, 2.0, 8).astype(np.float32)
        phi_case("g1_gauss_n128_d8_medh", X, gauss_logp(mu, lam), median_h(X),
                 {"target": np.array("gaussian"), "mu": mu, "lam": lam})
    cases.append(("g1_gauss_n128_d8_medh", g1_gauss8))

    def g1_gauss64():
        X = (0.1 * ref_init(64, 64, 11)).numpy()
        mu = np.random.RandomState(3).randn(64).astype(np.float32)
        lam = np.random.RandomState(4).uniform(0.5, 2.0, 64).astype(np.float32)
        phi_case("g1_gauss_n64_d64_h1", X, gauss_logp(mu, lam), 1.0,
                 {"target": np.array("gaussian"), "mu": mu, "lam": lam})
    cases.append(("g1_gauss_n64_d64_h1", g1_gauss64))

    def g1_logreg():
        x, t = banana_like(N=400)
        X = ref_init(100, 3, 0).numpy()
        phi_case("g1_logreg_n100", X, logreg_logp(x, t), 1.0,
                 {"target": np.array("logreg"), "x_train": x, "t_train": t})
    cases.append(("g1_logreg_n100", g1_logreg))

    # G2 -- Sampler.sample Gauss-Seidel trajectories (sampler.py:42-74)
    def g2_gauss():
        mu = np.array([0.5, -1.0], np.float32)
        lam = np.array([1.0, 2.0], np.float32)
        sample_case("g2_sample_gauss_n32_d2", 2, 32, 3, 0.1, gauss_logp(mu, lam), 1.0, 42,
                    {"target": np.array("gaussian"), "mu": mu, "lam": lam})
    cases.append(("g2_sample_gauss_n32_d2", g2_gauss))
    cases.append(("g2_sample_gmm_n50", lambda: sample_case(
        "g2_sample_gmm_n50", 1, 50, 3, 1.0, gmm_logp(), 1.0, 42, {"target": np.array("gmm")})))

    # G3 / G4 -- DistSampler.make_step (distsampler.py:172-205)
    cases.append(("g3_dist_s1_partitions", lambda: dist_case(
        "g3_dist_s1_partitions", 1, 40, 3, 0.05, "partitions", 29611)))
    port = 29620
    for S, n in ((2, 16), (4, 32)):
        for mode in ("partitions", "all_particles", "all_scores"):
            nm = "g4_dist_s%d_%s" % (S, mode)
            cases.append((nm, (lambda nm=nm, S=S, n=n, mode=mode, port=port:
                               dist_case(nm, S, n, 3, 0.05, mode, port))))
            port += 1
    # G5 -- the W2/JKO term (distsampler.py:103-129, 190-198)
    for nm, m, n, d, seed, near in (("g5_w2_m8_n8_d2", 8, 8, 2, 5, None),
                                    ("g5_w2_m12_n12_d3", 12, 12, 3, 6, None),
                                    ("g5_w2_m8_n16_d3", 8, 16, 3, 7, None),
                                    ("g5_w2_m6_n24_d5", 6, 24, 5, 8, None),
                                    ("g5_w2_m16_n32_d4_near", 16, 32, 4, 9, 0.05),
                                    ("g5_w2_m24_n24_d3_near", 24, 24, 3, 10, 0.02)):
        cases.append((nm, (lambda nm=nm, m=m, n=n, d=d, seed=seed, near=near:
                           w2_case(nm, m, n, d, seed, near))))
    for mode in ("partitions", "all_particles", "all_scores"):
        nm = "g5_dist_s2_%s_w2" % mode
        cases.append((nm, (lambda nm=nm, mode=mode, port=port:
                           dist_case(nm, 2, 16, 3, 0.05, mode, port, w2=True))))
        port += 1
    for nm, fn in cases:
        if which and nm not in which:
            continue
        fn()


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)
