"""Device engine: buffers + the kernel sequence of one SVGD step on MI355X.

One engine serves an owned row block [row0, row0+m) of an interacting set of n
particles (the whole set for Sampler; the DistSampler rank's block otherwise).
Per Jacobi step, all stream-ordered on the current HIP stream, no host sync:

  colmean -> pack          Y = [X - mean | scale*S] (n_pad+128, ldy), norms
  select_init -> sqdist    D = ||y_i||^2+||y_j||^2-2 y_i.y_j on MFMA (panel layout)
                           + radix histogram of key digit 1 (bits 31..21)
  [allreduce hist] pick1 -> hist2 -> [allreduce] pick2 -> hist3 -> [allreduce] pick3
                           exact lower median of the n^2 distances -> h (median mode)
  phi_mm                   [K Xc | K S], rowsum K, K = exp(-D/h) fused (MFMA)
  phi_finish               phi = (KS + 2/h (r x - K X)) / n ; X_own += step * phi

The hist all-reduce hook is where a DistSampler with a row-sharded D makes the
median global (RCCL all_reduce of 2048 int64 counts per pass).
"""
import ctypes

import torch

from . import _native as N

NBINS = 2048


class _SelectState(ctypes.Structure):
    _fields_ = [("hist", ctypes.c_uint64 * NBINS), ("k", ctypes.c_uint64),
                ("n_total", ctypes.c_uint64), ("prefix", ctypes.c_uint32),
                ("passes_done", ctypes.c_uint32), ("median", ctypes.c_float),
                ("h", ctypes.c_float), ("inv_h", ctypes.c_float), ("pad_", ctypes.c_float)]


_OFF_MEDIAN = _SelectState.median.offset
_OFF_PREFIX = _SelectState.prefix.offset


class SelectState(object):
    """Device-resident dsvgd_select_state (histogram first: all-reducible)."""

    def __init__(self, device):
        nbytes = N.load().dsvgd_select_state_bytes()
        assert nbytes == ctypes.sizeof(_SelectState), "dsvgd_select_state layout mismatch"
        self.buf = torch.zeros(nbytes // 8, dtype=torch.int64, device=device)
        self.device = device

    @property
    def ptr(self):
        return self.buf.data_ptr()

    @property
    def hist(self):
        return self.buf[:NBINS]

    def read(self):
        """(median, h, inv_h) -- synchronises with the device."""
        raw = self.buf.view(torch.uint8)[_OFF_MEDIAN:_OFF_MEDIAN + 12].view(torch.float32).cpu()
        return float(raw[0]), float(raw[1]), float(raw[2])

    def prefix(self):
        return int(self.buf.view(torch.uint8)[_OFF_PREFIX:_OFF_PREFIX + 4].view(torch.int32).cpu()[0])


class StageTimer(object):
    """Optional per-stage HIP-event timing on the current stream (bench only).
    `with timer("name"):` records an event pair; `summary()` syncs and returns
    {stage: [ms, ...]}.  A None timer costs nothing."""

    def __init__(self):
        self.events = {}

    def __call__(self, name):
        return _Span(self, name)

    def summary(self):
        torch.cuda.synchronize()
        return {k: [a.elapsed_time(b) for a, b in v] for k, v in self.events.items()}


class _Span(object):
    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record()

    def __exit__(self, *exc):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.timer.events.setdefault(self.name, []).append((self.e0, e1))


class _Null(object):
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL = _Null()


def span(timer, name):
    return _NULL if timer is None else timer(name)


class PhiEngine(object):
    timer = None

    def __init__(self, n, d, m=None, row0=0, device=None):
        dev = N.require_gpu(device if device is not None else "cuda")
        lib = N.load()
        m = n if m is None else m
        assert 0 < m and 0 <= row0 and row0 + m <= n
        self.n, self.d, self.m, self.row0, self.device = n, d, m, row0, dev
        self.n_pad = lib.dsvgd_pad128(n)
        self.m_pad = lib.dsvgd_pad128(m)
        self.dp = lib.dsvgd_dp(d)
        self.ldy = lib.dsvgd_ldy(self.dp)
        f32 = dict(dtype=torch.float32, device=dev)
        rows = self.n_pad + 128
        self.Y = torch.zeros(rows, self.ldy, **f32)
        self.norms = torch.zeros(rows, **f32)
        self.D = torch.empty(self.m_pad * self.n_pad, **f32)
        self.splits = lib.dsvgd_phi_splits(m, n, self.ldy)
        self.KY = torch.empty(self.splits * m, self.ldy, **f32)
        self.rowsum = torch.empty(self.splits * self.m_pad, **f32)
        self.mean = torch.empty(d, **f32)
        self.mean_ws = torch.empty(max(1, lib.dsvgd_colmean_workspace_floats(n, d)), **f32)
        self.phi = torch.empty(m, d, **f32)
        self.state = SelectState(dev)

    # ------------------------------------------------------------ stages --
    def pack(self, X, S=None, score_scale=1.0):
        """X, S: (n, d) device tensors (row stride may exceed d)."""
        assert X.shape == (self.n, self.d)
        s = N.stream(self.device)
        with span(self.timer, "pack"):
            self._pack(X, S, score_scale, s)

    def _pack(self, X, S, score_scale, s):
        N.call("dsvgd_colmean", N.ptr(X), N.ld(X), self.n, self.d, N.ptr(self.mean_ws),
               N.ptr(self.mean), s)
        lds = N.ld(S) if S is not None else self.d
        if S is not None:
            assert S.shape == (self.n, self.d)
        N.call("dsvgd_pack", N.ptr(X), N.ld(X), N.ptr(S), lds, float(score_scale),
               N.ptr(self.mean), self.n, self.d, self.Y.shape[0], N.ptr(self.Y), self.ldy,
               N.ptr(self.norms), s)

    def distances(self, histogram=True):
        s = N.stream(self.device)
        st = None
        if histogram:
            N.call("dsvgd_select_init", self.state.ptr, self.n, s)
            st = self.state.ptr
        with span(self.timer, "sqdist"):
            N.call("dsvgd_sqdist", N.ptr(self.Y), self.ldy, N.ptr(self.norms), self.row0, self.m,
                   self.n, self.d, N.ptr(self.D), self.n_pad, st, s)

    def median_bandwidth(self, allreduce=None):
        """Radix select over D (after distances(histogram=True))."""
        s = N.stream(self.device)
        for p in (1, 2, 3):
            if p > 1:
                with span(self.timer, "radix_hist"):
                    N.call("dsvgd_radix_hist", N.ptr(self.D), self.n_pad, self.m, self.n, p,
                           self.state.ptr, s)
            if allreduce is not None:
                with span(self.timer, "hist_allreduce"):
                    allreduce(self.state.hist)
            N.call("dsvgd_radix_pick", self.state.ptr, p, s)

    def fixed_bandwidth(self, h):
        N.call("dsvgd_set_bandwidth", self.state.ptr, float(h), N.stream(self.device))

    DIRECT_MAX_D = 64

    def direction(self, X_own=None, step=0.0, write_phi=True, inv_n=None):
        """phi for the owned rows; optionally X_own += step * phi (in place).
        d <= 64: pairwise VALU form (dsvgd_phi_direct); else K.[Xc|S] on MFMA."""
        s = N.stream(self.device)
        if X_own is not None:
            assert X_own.shape == (self.m, self.d)
        inv_n = 1.0 / self.n if inv_n is None else inv_n
        phi = N.ptr(self.phi) if write_phi else None
        xo = N.ptr(X_own)
        ldx = N.ld(X_own) if X_own is not None else self.d
        if self.d <= self.DIRECT_MAX_D:
            with span(self.timer, "phi_direct"):
                N.call("dsvgd_phi_direct", N.ptr(self.D), self.n_pad, N.ptr(self.Y), self.ldy,
                       self.row0, self.m, self.n, self.d, self.state.ptr, float(inv_n),
                       float(step), phi, self.d, xo, ldx, s)
            return
        with span(self.timer, "phi_mm"):
            N.call("dsvgd_phi_mm", N.ptr(self.D), self.n_pad, N.ptr(self.Y), self.ldy, self.m,
                   self.n, self.state.ptr, self.splits, N.ptr(self.KY), self.ldy,
                   N.ptr(self.rowsum), s)
        N.call("dsvgd_phi_finish", N.ptr(self.KY), self.ldy, N.ptr(self.rowsum), self.splits,
               N.ptr(self.Y), self.ldy, self.row0, self.m, self.d, self.dp, self.state.ptr,
               float(inv_n), float(step), phi, self.d, xo, ldx, s)

    # ------------------------------------------------------------ helpers --
    def step(self, X, S, X_own=None, step=0.0, h=None, score_scale=1.0, allreduce=None,
             write_phi=True):
        """One Jacobi step: h=None -> median bandwidth, else fixed h."""
        self.pack(X, S, score_scale)
        median = h is None
        self.distances(histogram=median)
        if median:
            self.median_bandwidth(allreduce)
        else:
            self.fixed_bandwidth(h)
        self.direction(X_own, step, write_phi)

    def dense_D(self):
        """D as a dense (m, n) tensor (tests/inspection; un-does the panel layout)."""
        mp, np_ = self.m_pad, self.n_pad
        Dd = self.D.view(mp // 128, np_ // 16, 128, 16).permute(0, 2, 1, 3).reshape(mp, np_)
        return Dd[:self.m, :self.n]


def sequential_sweep(X, S, rows, h_state, step, target=None, score_scale=1.0, phi_out=None):
    """Gauss-Seidel sweep in the reference order over `rows` of the interacting
    set X (n, d): for each i, phi_i from the CURRENT X (earlier rows already
    moved), X[i] += step * phi_i, then (if `target`) S[i] is recomputed for the
    moved particle, which is what re-running _dlogp per pair amounts to
    (dsvgd/sampler.py:64-68, dsvgd/distsampler.py:194-200)."""
    n, d = X.shape
    s = N.stream(X.device)
    for k, i in enumerate(rows):
        N.call("dsvgd_phi_row", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), n, d, int(i),
               h_state.ptr, float(step), N.ptr(phi_out[k]) if phi_out is not None else None, s)
        if target is not None:
            target.score(X[i:i + 1], S[i:i + 1], score_scale)
