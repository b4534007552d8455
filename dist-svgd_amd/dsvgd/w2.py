"""The W2 / JKO term of DistSampler.make_step on the GPU
(reference dsvgd/distsampler.py:103-129, applied at :190-198).

    G = h * sum_j P_ij (x_i - y_j)

with P the optimal plan of the reference LP (uniform marginals 1/m, 1/n).
For n = R m the plan is an assignment of n slots to n columns (include/dsvgd.h,
dsvgd_w2_*): cost tiles (dsvgd_w2_cost) -> epsilon-scaling auction
(dsvgd_w2_assign) -> dsvgd_w2_grad, all on device.  G is handed to the phi
epilogue as `extra`, so the update is x_i += step * (phi_i + G_i) as at
distsampler.py:196-200.
"""
import ctypes

import torch

from . import _native as N


class W2Term(object):
    """Buffers for one (m, n, d) shape: cost C (m x n fp32), auction workspace,
    slot assignment (n int32) and G (m x d)."""

    MAX_ROUNDS = 1 << 18
    # warm start from the previous step's prices and plan: None = adaptive
    # (the first epsilon from the old plan's slackness violation under the
    # new costs, dsvgd_w2_assign_warm); k > 0 = k fixed phases above the
    # final eps; 0 = cold every step.  The first call on a workspace is cold.
    WARM_PHASES = None
    # a new epsilon phase (and the warm start's first) keeps the slots whose
    # column still meets eps-CS (dsvgd_w2_set_keep); False: all re-bid.  Off:
    # at m = 8192, n = 65536 the warm solve took 1.81 s with it against 79 ms
    # without, the cold one 3.95 vs 4.04 s (profiles/r11g/w2.log)
    KEEP = False
    THETA = 8.0   # eps divisor between phases (dsvgd_w2_set_theta)
    # the cost matrix: "h2" on the split-role MFMA Gram with the near pairs
    # recomputed exactly (dsvgd_w2_cost_h2), "exact" the explicit-difference
    # VALU tiles (dsvgd_w2_cost), "auto" h2 from H2_MIN_ENTRIES entries on
    # (smaller plans: the VALU tiles take microseconds) for 2 < d <= 1024
    COST = "auto"
    H2_MIN_ENTRIES = 1 << 22
    # an entry is recomputed from explicit differences when its Gram form is
    # below TAU (|x_i - c|^2 + |y_j - c|^2): there the form's error bound
    # (~2^-21 of that sum) exceeds 2^-19 of the entry
    TAU = 0.25

    def __init__(self, m, n, d, device, warm=True):
        if n % m:
            raise ValueError("W2 term needs n to be a multiple of m (n = R m)")
        self.m, self.n, self.d = m, n, d
        self.device = torch.device(device)
        lib = N.load()
        mode = self.COST
        if mode == "auto":
            mode = "h2" if (m * n >= self.H2_MIN_ENTRIES and 2 < d <= 1024) else "exact"
        self.cost = mode
        if mode == "h2":
            # whole 128-row x 256-column tiles are written (padding included)
            self.ldc = -(-n // 256) * 256
            self.C = torch.empty((-(-m // 128) * 128, self.ldc), dtype=torch.float32,
                                 device=self.device)
            nb = int(lib.dsvgd_w2_cost_h2_workspace_bytes(m, n, d))
            self.cws = torch.empty(nb + 256, dtype=torch.uint8, device=self.device)
            # C's largest entry and finiteness, taken while the cost kernel
            # writes C (the solve then skips its own pass over C for them)
            self.cstat = torch.zeros(2, dtype=torch.int32, device=self.device)
        else:
            self.ldc = n
            self.C = torch.empty((m, n), dtype=torch.float32, device=self.device)
        nbytes = int(N.load().dsvgd_w2_workspace_bytes(m, n))
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.assign = torch.empty(n, dtype=torch.int32, device=self.device)
        self.G = torch.empty((m, d), dtype=torch.float32, device=self.device)
        self.rounds = 0
        self.warm = warm
        self._solved = False

    def grad(self, X, Y, h):
        """G (m, d) = h * W2 gradient of the owned rows X (m, d) against the
        previous particles Y (n, d).  Blocks until the auction has converged."""
        assert X.shape == (self.m, self.d) and Y.shape == (self.n, self.d)
        s = N.stream(self.device)
        if self.cost == "h2":
            ws = N.ptr(self.cws)
            ws = (ws + 255) // 256 * 256
            N.call("dsvgd_w2_cost_h2", N.ptr(X), N.ld(X), self.m, N.ptr(Y), N.ld(Y), self.n,
                   self.d, N.ptr(self.C), self.ldc, ws, float(self.TAU), N.ptr(self.cstat), s)
        else:
            N.call("dsvgd_w2_cost", N.ptr(X), N.ld(X), self.m, N.ptr(Y), N.ld(Y), self.n, self.d,
                   N.ptr(self.C), self.ldc, s)
        rounds = ctypes.c_int64(0)
        N.load().dsvgd_w2_set_keep(int(bool(self.KEEP)))    # returns the old setting
        N.load().dsvgd_w2_set_theta(float(self.THETA))
        if self.cost == "h2":
            warm_start = self.warm and self._solved and self.WARM_PHASES is None
            warm = (self.WARM_PHASES or 0) if (self.warm and self._solved) else 0
            N.call("dsvgd_w2_assign_stat", N.ptr(self.C), self.ldc, self.m, self.n,
                   N.ptr(self.ws), self.MAX_ROUNDS, 0 if warm_start else warm,
                   N.ptr(self.assign) if warm_start else None, N.ptr(self.assign),
                   ctypes.addressof(rounds), N.ptr(self.cstat), s)
        elif self.warm and self._solved and self.WARM_PHASES is None:
            # prev and out may alias: the plan is only written after the solve
            N.call("dsvgd_w2_assign_warm", N.ptr(self.C), self.ldc, self.m, self.n,
                   N.ptr(self.ws), self.MAX_ROUNDS, N.ptr(self.assign), N.ptr(self.assign),
                   ctypes.addressof(rounds), s)
        else:
            warm = (self.WARM_PHASES or 0) if (self.warm and self._solved) else 0
            N.call("dsvgd_w2_assign", N.ptr(self.C), self.ldc, self.m, self.n, N.ptr(self.ws),
                   self.MAX_ROUNDS, warm, N.ptr(self.assign), ctypes.addressof(rounds), s)
        self.rounds = int(rounds.value)
        self._solved = True
        N.call("dsvgd_w2_grad", N.ptr(X), N.ld(X), self.m, N.ptr(Y), N.ld(Y), self.n, self.d,
               N.ptr(self.assign), float(h), N.ptr(self.G), self.d, s)
        return self.G

    def tail_stats(self):
        """The last solve's phase tails: (bids, full row scans, us in the
        cached bids, us in the scans, us in the resolves, tails that stalled
        on their helpers and handed the phase back to the bid rounds)."""
        buf = (ctypes.c_int64 * 6)()
        N.load().dsvgd_w2_tail_stats(buf)
        return tuple(int(v) for v in buf)

    def trace(self):
        """The last solve's progress: (rounds, phase, unassigned) every 16 rounds."""
        k = int(N.load().dsvgd_w2_trace(None, 0))
        buf = (ctypes.c_int64 * (3 * k))()
        N.load().dsvgd_w2_trace(buf, k)
        return [tuple(buf[3 * e:3 * e + 3]) for e in range(k)]

    def plan(self):
        """The last slot -> column assignment as a host int64 array."""
        return self.assign.cpu().numpy().astype("int64")
