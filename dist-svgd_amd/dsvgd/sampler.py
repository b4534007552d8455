"""Drop-in `dsvgd.Sampler` (reference: dsvgd/sampler.py:6-74) on MI355X.

Same constructor and `sample(n, num_iter, step_size) -> pandas.DataFrame`
(columns timestep, particle, value; n*(num_iter+1) rows ordered by
(timestep, particle); value = float32 ndarray (d,)), same particle init from
torch's global CPU generator, same "Iteration l" / mean prints.

Extensions (keyword-only, defaults keep the reference behaviour):
  order="sequential"  the reference's in-place Gauss-Seidel sweep
                      (sampler.py:64-68), one gfx950 row kernel per particle;
  order="jacobi"      all particles move together from the frozen set -- the
                      MFMA fast path (sq-distances, radix-select median, fused
                      exp, K.[X|S]) used for throughput;
  device              HIP device (default: current cuda device);
  verbose             the reference's per-iteration prints;
  graphs              capture one iteration as a HIP graph and replay it
                      (built-in targets; default on).
The kernel must be RBF-shaped (see dsvgd.kernels); RBF("median") selects the
median-heuristic bandwidth h = median(D)/log(n), recomputed every iteration.
"""
import pandas as pd
import torch
from torch.distributions.normal import Normal

from . import _native as N
from .engine import PhiEngine, SelectState, StepGraph, sequential_sweep
from .kernels import resolve_kernel
from .targets import BuiltinTarget, resolve_target


class Sampler(object):
    def __init__(self, d, logp, kernel):
        """Initializes a SVGD sampler.

        Params:
            d - dimensionality of each particle
            kernel - kernel function (RBF family; see dsvgd.kernels)
            logp - log density function, or a dsvgd.targets.Target
        """
        self._d = d
        self._logp = logp
        self._kernel = kernel
        self._target = resolve_target(logp)
        self._rbf = resolve_kernel(kernel, d)

    def sample(self, n, num_iter, step_size, *, order="sequential", device=None, verbose=True,
               graphs=True):
        """Generate samples using SVGD (sampler.py:42-74)."""
        if order not in ("sequential", "jacobi"):
            raise ValueError("order must be 'sequential' or 'jacobi'")
        dev = N.require_gpu(device if device is not None else "cuda")
        q = Normal(0, 1)
        make_sample = lambda: q.sample((self._d, 1))  # noqa: E731  (sampler.py:58-60)
        particles = torch.cat([make_sample() for _ in range(n)], dim=1).t()
        X = torch.empty(n, self._d, dtype=torch.float32, device=dev)
        X.copy_(particles)
        d = self._d
        hist = torch.empty(num_iter + 1, n, d, dtype=torch.float32, device=dev)
        S = torch.empty(n, d, dtype=torch.float32, device=dev)
        median = self._rbf.median
        engine = PhiEngine(n, d, device=dev) if (order == "jacobi" or median) else None
        state = engine.state if engine is not None else SelectState(dev)
        if not median:
            N.call("dsvgd_set_bandwidth", state.ptr, float(self._rbf.h), N.stream(dev))
        target = self._target

        def iteration():
            target.score(X, S)
            if order == "jacobi":
                engine.step(X, S, X_own=X, step=step_size, h=None if median else self._rbf.h,
                            write_phi=False)
            else:
                if median:
                    engine.pack(X)
                    engine.distances(median=True)
                    engine.median_bandwidth()
                sequential_sweep(X, S, range(n), state, step_size, target=target)

        # built-in targets are pure kernel launches: capture the iteration
        # once and replay it (user callables run eagerly)
        step = StepGraph(iteration, dev, enabled=graphs and isinstance(target, BuiltinTarget))
        for l in range(num_iter):
            if verbose:
                print('Iteration {}'.format(l))
            hist[l].copy_(X)
            step()
            if verbose:
                print(X.mean(dim=0).cpu())
        hist[num_iter].copy_(X)
        vals = hist.cpu().numpy().reshape(-1, d)
        steps = torch.arange(num_iter + 1).repeat_interleave(n).numpy()
        ids = torch.arange(n).repeat(num_iter + 1).numpy()
        return pd.DataFrame({"timestep": steps, "particle": ids, "value": list(vals)})
