"""Target densities: batched scores grad log p(X) for all particles at once.

The reference differentiates a per-particle Python `logp(x) -> 0-d tensor`
with autograd, once per interacting pair (dsvgd/sampler.py:28-33,
dsvgd/distsampler.py:77-82).  Here a target computes the scores of ALL n
particles in one batched device call:

* built-in targets run hand-written gfx950 kernels (libdsvgd_hip.so):
  :class:`Gaussian`, :class:`GaussianMixture1D` (experiments/gmm.py:16-21),
  :class:`LogisticRegression` (experiments/logreg.py:45-58, two MFMA GEMMs);
* any other `logp` callable is wrapped by :class:`CallableTarget`, which runs
  the user's own torch code under ``torch.func.vmap(torch.func.grad(logp))``
  on the particles' device (user code, not a dsvgd compute path).

Every target is also a reference-compatible callable ``target(x) -> log p(x)``
so it can be handed to the reference implementation unchanged.
"""
import math

import torch

from . import _native as N


def _host_bytes(t):
    """The bytes of a tensor's values wherever it lives (a target built from
    device tensors digests the same as one built from host tensors)."""
    return t.detach().cpu().contiguous().numpy().tobytes()


class Target(object):
    def score(self, X, out, scale=1.0):
        """out[:] = scale * grad log p(X) for X (n, d) on the device."""
        raise NotImplementedError

    def __call__(self, x):
        return self.logp(x)


class BuiltinTarget(Target):
    """Targets whose score is a libdsvgd_hip kernel sequence (graph-capturable)."""


class Gaussian(BuiltinTarget):
    """N(mu, diag(1/lam)): log p = -1/2 sum_c lam_c (x_c - mu_c)^2 (+ const)."""

    def __init__(self, mu, lam):
        self.mu = torch.as_tensor(mu, dtype=torch.float32).reshape(-1)
        self.lam = torch.as_tensor(lam, dtype=torch.float32).reshape(-1)
        self._dev = {}

    def logp(self, x):
        mu, lam = self.mu.to(x.device), self.lam.to(x.device)
        return -0.5 * (lam * (x - mu) ** 2).sum()

    def _params(self, dev):
        if dev not in self._dev:
            self._dev[dev] = (self.mu.to(dev).contiguous(), self.lam.to(dev).contiguous())
        return self._dev[dev]

    def fingerprint(self):
        import hashlib
        return hashlib.sha1(b"gauss" + _host_bytes(self.mu) + _host_bytes(self.lam)).hexdigest()

    def score(self, X, out, scale=1.0):
        n, d = X.shape
        assert d == self.mu.numel(), "Gaussian target has d=%d" % self.mu.numel()
        mu, lam = self._params(X.device)
        N.call("dsvgd_score_gaussian", N.ptr(X), N.ld(X), n, d, N.ptr(mu), N.ptr(lam),
               float(scale), N.ptr(out), N.ld(out), N.stream(X.device))


class GaussianMixture1D(BuiltinTarget):
    """log(1/3 N(x; -2, 1) + 1/3 N(x; 2, 1)) per coordinate (experiments/gmm.py:16-21;
    the code uses equal 1/3 weights although its comment says 1/3, 2/3)."""

    def logp(self, x):
        a = -0.5 * (x + 2.0) ** 2
        b = -0.5 * (x - 2.0) ** 2
        return (torch.logaddexp(a, b) + math.log(1.0 / 3.0) - 0.5 * math.log(2 * math.pi)).sum()

    def fingerprint(self):
        return "gmm1d"

    def score(self, X, out, scale=1.0):
        n, d = X.shape
        N.call("dsvgd_score_gmm", N.ptr(X), N.ld(X), n, d, float(scale), N.ptr(out),
               N.ld(out), N.stream(X.device))


class LogisticRegression(BuiltinTarget):
    """Bayesian logistic regression of experiments/logreg.py:45-58.

    x = [log alpha, w] (d = 1 + p); alpha ~ Gamma(1, 1) (no log-Jacobian, as in
    the reference), w ~ N(0, I/alpha), labels t in {-1, +1}.
    """

    ENGINES = {"h2": 0, "x3": 1, "f32": 2}   # dsvgd_score_logreg_engine
    SMALL_ROWS = 32      # one-block-per-particle path (no workspace), csrc/logreg.hip

    def __init__(self, x_train, t_train, gemm="h2"):
        self.x = torch.as_tensor(x_train, dtype=torch.float32)
        self.t = torch.as_tensor(t_train, dtype=torch.float32).reshape(-1)
        assert self.x.shape[0] == self.t.shape[0]
        if gemm not in self.ENGINES:
            raise ValueError("gemm must be one of %s" % sorted(self.ENGINES))
        self.gemm = gemm
        self._dev = {}
        self._ws = {}             # workspace key -> buffer, least recently used first
        self._prepared = {}       # workspace key -> engine whose data image it holds
        self._pinned = set()      # keys a captured HIP graph holds (never evicted)

    @property
    def N(self):
        return self.x.shape[0]

    def logp(self, x):
        from torch.distributions.gamma import Gamma
        from torch.distributions.multivariate_normal import MultivariateNormal
        xt, tt = self.x.to(x.device), self.t.to(x.device)
        p = xt.shape[1]
        alpha = torch.exp(x[0])
        w = x[1:].reshape(-1)
        lp = Gamma(torch.tensor(1., device=x.device), torch.tensor(1., device=x.device)).log_prob(alpha)
        lp = lp + MultivariateNormal(torch.zeros(p, device=x.device),
                                     torch.eye(p, device=x.device) / alpha).log_prob(w)
        lp = lp + (-torch.log(1. + torch.exp(-1. * torch.mv(tt[:, None] * xt, w))).sum())
        return lp

    def _params(self, dev):
        if dev not in self._dev:
            self._dev[dev] = (self.x.to(dev).contiguous(), self.t.to(dev).contiguous())
        return self._dev[dev]

    def _params_aligned(self, dev):
        """(data with 16-byte rows -- ld = roundup(p, 4), zero pad -- labels)
        on dev: the Gauss-Seidel walk's one-pass score refresh
        (dsvgd_gsw_block_sweep, score_kind 3) reads the rows as dwordx4."""
        key = ("aligned", dev)
        if key not in self._dev:
            xd, t = self._params(dev)
            p = xd.shape[1]
            pa = -(-p // 4) * 4
            buf = torch.zeros(xd.shape[0], pa, dtype=torch.float32, device=dev)
            buf[:, :p] = xd
            self._dev[key] = (buf, t)
        return self._dev[key]

    def fingerprint(self):
        """Digest of the data (DistSampler: ranks whose targets agree on it
        hold the same data, so their scores of a particle are the same)."""
        import hashlib
        h = hashlib.sha1(b"logreg")
        h.update(_host_bytes(self.x))
        h.update(_host_bytes(self.t))
        return h.hexdigest()

    MAX_WORKSPACES = 4   # unpinned score workspaces kept (least recently used evicted)

    def _workspace(self, key, n, d, dev):
        ws = self._ws.pop(key, None)
        if ws is None:
            nbytes = N.load().dsvgd_logreg_workspace_bytes(n, self.N, d - 1) if key[1] else 256
            ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
        self._ws[key] = ws                     # most recently used last
        if torch.cuda.is_current_stream_capturing():
            self._pinned.add(key)              # a graph now holds its address
        free = [k for k in self._ws if k not in self._pinned and k != key]
        for k in free[:max(0, len(free) + 1 - self.MAX_WORKSPACES)]:
            del self._ws[k]
            self._prepared.pop(k, None)
        return ws

    def score(self, X, out, scale=1.0, prior_weight=1.0):
        """out = scale * grad log p(X); prior_weight != 1 weighs the prior
        terms (DistSampler's gathered-data all_scores: the prior of S ranks'
        logp, distsampler.py:160-170), on the prepared path only."""
        n, d = X.shape
        assert d == self.x.shape[1] + 1, "logreg target has d = 1 + p = %d" % (self.x.shape[1] + 1)
        xd, t = self._params(X.device)
        # one workspace per (device, n): the ones a captured HIP graph
        # (engine.StepGraph) holds are pinned and never freed behind it
        # (release() frees them explicitly); of the others the
        # MAX_WORKSPACES most recently used stay.  The few-particle path
        # (the Gauss-Seidel refreshes) needs none.
        small = n <= self.SMALL_ROWS and (d - 1 <= 32 or self.N <= 8192)   # logreg.hip's test
        key = (X.device, 0 if small else n)
        ws = self._workspace(key, n, d, X.device)
        base = ws.data_ptr()
        aligned = (base + 255) // 256 * 256
        eng = self.ENGINES[self.gemm]
        s = N.stream(X.device)
        if small:
            if prior_weight != 1.0:
                raise ValueError("prior_weight needs more than %d particles" % self.SMALL_ROWS)
            N.call("dsvgd_score_logreg_engine", N.ptr(X), N.ld(X), n, d, N.ptr(xd), N.ld(xd),
                   N.ptr(t), self.N, float(scale), N.ptr(out), N.ld(out), aligned, eng, s)
            return
        if self._prepared.get(key) != eng:
            # the data-only half of the workspace (padded data, its scales
            # and split images) once per workspace; every later step reuses it
            N.call("dsvgd_logreg_prepare", N.ptr(xd), N.ld(xd), N.ptr(t), self.N, n, d, aligned,
                   eng, s)
            self._prepared[key] = eng
            if not torch.cuda.is_current_stream_capturing():
                # later calls may come on other streams (the DistSampler side stream)
                torch.cuda.current_stream(X.device).synchronize()
        if prior_weight != 1.0:
            N.call("dsvgd_score_logreg_prior", N.ptr(X), N.ld(X), n, d, self.N, float(scale),
                   float(prior_weight), N.ptr(out), N.ld(out), aligned, eng, s)
            return
        N.call("dsvgd_score_logreg_prepared", N.ptr(X), N.ld(X), n, d, self.N, float(scale),
               N.ptr(out), N.ld(out), aligned, eng, s)

    def release(self):
        """Free the score workspaces (no graph that captured them may replay after)."""
        self._ws.clear()
        self._prepared.clear()
        self._pinned.clear()


class CallableTarget(Target):
    """Any reference-style `logp(x[d]) -> 0-d tensor`, batched with torch.func.

    The callable must accept tensors on the particles' device; dsvgd does not
    move user code or data to the host.
    """

    def __init__(self, logp, chunk=65536):
        self._logp = logp
        self.chunk = chunk
        self._vg = None

    def logp(self, x):
        return self._logp(x)

    def score(self, X, out, scale=1.0):
        if self._vg is None:
            self._vg = torch.func.vmap(torch.func.grad(self._logp))
        try:
            for s in range(0, X.shape[0], self.chunk):
                g = self._vg(X[s:s + self.chunk])
                out[s:s + self.chunk].copy_(g.reshape(out[s:s + self.chunk].shape)).mul_(scale)
        except RuntimeError as e:
            if "device" in str(e) or "vmap" in str(e).lower() or "batch" in str(e).lower():
                self._score_loop(X, out, scale, e)
            else:
                raise

    def _score_loop(self, X, out, scale, why):
        """Per-particle autograd on the device (callables vmap cannot batch)."""
        for j in range(X.shape[0]):
            x = X[j].detach().clone().requires_grad_(True)
            try:
                lp = self._logp(x)
            except RuntimeError as e:
                raise RuntimeError(
                    "logp could not be evaluated on %s tensors (%s); dsvgd runs scores on the "
                    "particles' device -- use a dsvgd.targets class or a device-agnostic logp"
                    % (X.device, e)) from why
            (g,) = torch.autograd.grad(lp, x)
            out[j] = scale * g


def resolve_target(logp):
    if isinstance(logp, Target):
        return logp
    if not callable(logp):
        raise ValueError("logp must be callable")
    return CallableTarget(logp)
