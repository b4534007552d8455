"""CPU BASELINE (test/bench infrastructure only): the reference algorithm's
per-pair autograd loop, restated with torch on the host.

Follows dsvgd/sampler.py:19-40 / dsvgd/distsampler.py:68-101 literally: for
each interacting particle x_j, kernel(x_j, x_i) forward, grad_{x_j} k by
autograd, grad log p(x_j) by autograd, accumulate, scale by 1/n.  Only
bench.py's cpu_baseline leg times it; it is never part of the product path.
"""
import time

import torch


def rbf(h):
    def kernel(x, y):
        return torch.exp(-1. * torch.dist(x, y, p=2) ** 2 / h)
    return kernel


def _dkernel(kernel, x, y):
    _x = x.detach().clone().requires_grad_(True)
    kernel(_x, y.detach()).backward()
    return _x.grad


def _dlogp(logp, x):
    _x = x.detach().clone().requires_grad_(True)
    logp(_x).backward()
    return _x.grad


def phi_hat(particle, particles, logp, kernel):
    total = torch.zeros(particle.size())
    for other in particles:
        total += kernel(other, particle) * _dlogp(logp, other) + _dkernel(kernel, other, particle)
    return (1.0 / particles.shape[0]) * total


def logreg_logp(x_train, t_train):
    """experiments/logreg.py:45-58 restated (labels as a float tensor)."""
    from torch.distributions.gamma import Gamma
    from torch.distributions.multivariate_normal import MultivariateNormal
    xt = torch.as_tensor(x_train, dtype=torch.float32)
    tt = torch.as_tensor(t_train, dtype=torch.float32).reshape(-1, 1)
    p = xt.shape[1]
    alpha_prior = Gamma(1., 1.)
    txt = tt * xt

    def logp(x):
        alpha = torch.exp(x[0])
        w = x[1:].reshape(-1)
        lp = alpha_prior.log_prob(alpha)
        lp = lp + MultivariateNormal(torch.zeros(p), torch.eye(p) / alpha).log_prob(w)
        lp = lp + (-torch.log(1. + torch.exp(-1. * torch.mv(txt, w))).sum())
        return lp
    return logp


def time_particle_updates(X, logp, h, m, budget_s=20.0):
    """Time up to `m` particle updates (each a full n-term pair loop) within a
    wall budget; returns (seconds_per_particle_update, updates_done, pairs_done)."""
    X = torch.as_tensor(X, dtype=torch.float32)
    kernel = rbf(h)
    n = X.shape[0]
    t0 = time.perf_counter()
    done = pairs = 0
    for i in range(m):
        total = torch.zeros(X.shape[1])
        for j in range(n):
            other = X[j]
            total += kernel(other, X[i]) * _dlogp(logp, other) + _dkernel(kernel, other, X[i])
            pairs += 1
            if time.perf_counter() - t0 > budget_s and j < n - 1:
                el = time.perf_counter() - t0
                return el / pairs * n, done, pairs
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    el = time.perf_counter() - t0
    return el / pairs * n, done, pairs
