"""Device engine: buffers + the kernel sequence of one SVGD step on MI355X.

One engine serves an owned row block [row0, row0+m) of an interacting set of n
particles (the whole set for Sampler; the DistSampler rank's block otherwise).
Per Jacobi step, all stream-ordered on the current HIP stream, no host sync:

  colcenter -> pack        Y = [X - c | scale*S] (n_pad+128, ldy), norms (c: robust centre)
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
import math

import torch

from . import _native as N

NBINS = 2048


class _SelectState(ctypes.Structure):
    """Mirror of dsvgd_select_state (include/dsvgd.h)."""
    _fields_ = [("hist", ctypes.c_uint64 * NBINS), ("k", ctypes.c_uint64),
                ("n_total", ctypes.c_uint64), ("prefix", ctypes.c_uint32),
                ("passes_done", ctypes.c_uint32), ("median", ctypes.c_float),
                ("h", ctypes.c_float), ("inv_h", ctypes.c_float), ("fallback", ctypes.c_uint32),
                ("below_total", ctypes.c_uint64), ("ncand_total", ctypes.c_uint64),
                ("overflow", ctypes.c_uint64), ("lo", ctypes.c_float), ("hi", ctypes.c_float),
                ("cand_cap", ctypes.c_uint64), ("nslots", ctypes.c_uint64),
                ("slot_cap", ctypes.c_uint64)]

SEL_NONE, SEL_HIST, SEL_BRACKET = 0, 1, 2


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

    @property
    def totals(self):
        """int64[3] view of (below_total, ncand_total, overflow) -- all-reduced
        between dsvgd_bracket_totals and dsvgd_bracket_check."""
        o = _SelectState.below_total.offset // 8
        return self.buf[o:o + 3]

    def bracket(self):
        """(lo, hi, below_total, ncand_total, fallback) -- synchronises."""
        raw = self.buf.cpu()
        u8 = raw.view(torch.uint8)
        lo, hi = u8[_SelectState.lo.offset:_SelectState.lo.offset + 8].view(torch.float32).tolist()
        fb = int(u8[_SelectState.fallback.offset:_SelectState.fallback.offset + 4]
                 .view(torch.int32)[0])
        o = _SelectState.below_total.offset // 8
        b, c = raw[o:o + 2].tolist()
        return lo, hi, b, c, fb

    def read(self):
        """(median, h, inv_h) -- synchronises with the device."""
        raw = self.buf.view(torch.uint8)[_OFF_MEDIAN:_OFF_MEDIAN + 12].view(torch.float32).cpu()
        return float(raw[0]), float(raw[1]), float(raw[2])

    def prefix(self):
        return int(self.buf.view(torch.uint8)[_OFF_PREFIX:_OFF_PREFIX + 4].view(torch.int32).cpu()[0])


class StageTimer(object):
    """Optional per-stage HIP-event timing on the current stream (bench only).
    `with timer("name"):` records an event pair; `summary()` syncs and returns
    {stage: [ms, ...]}.  A None timer costs nothing; `only` (a set of stage
    names) times those stages alone -- every event pair is a pair of stream
    markers the GPU waits on (≈ 10 µs each between kernels, profiles/r13j)."""

    def __init__(self, only=None):
        self.events = {}
        self.only = None if only is None else frozenset(only)

    def __call__(self, name):
        if self.only is not None and name not in self.only:
            return _NULL
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
    # median select: bracketed (sample -> [lo, hi] -> candidates) when the
    # owned block has at least this many entries, plain radix passes over D below
    BRACKET_MIN_ENTRIES = 1 << 24
    SAMPLE = 1 << 18            # sampled pairs that fix the bracket
    SIGMAS = 6.0                # bracket half-width in sample-rank standard deviations
    SEED = 0x5EED5EED

    # pair split: run the own window on a second stream beside the transposed
    # partials (the batched forward launch holds 192 of the 256 CUs)
    WINDOW_SIDE_STREAM = False
    # pair split: the transposed partials left beside the batched forward
    # launch (the antipodal half) on a second stream next to it without
    # split-K when both fit the 256 CUs together (S = 8: 192 + 32 or 64).
    # Off: measured slower, partials 0.98-1.00 vs 0.78 ms at S = 8 in one
    # process (profiles/r11m/rank_rest.log)
    REST_BESIDE = False
    # pair split: the batched forward launch's K range (each block's m rows
    # of D) split into this many slices so that its workgroups fill whole
    # waves of the 256 CUs (None: chosen -- S = 8 at the headline: 3 x 64
    # workgroups x 4 = three full waves instead of 192 of 256), the slices
    # summed in order into the messages (dsvgd_phi_partial_reduce_blocks)
    FWD_ZSPLIT = None
    # pair split, A/B overrides of the other products' split-K factors (None:
    # chosen -- dsvgd_phi_splits for the window and the row half, the
    # fill-the-CUs rule for the other transposed partials)
    W_SPLITS = None
    H_SPLITS = None
    REST_SPLITS = None

    GEMMS = ("h2", "x3", "f32")
    DEFAULT_GEMM = "h2"

    def __init__(self, n, d, m=None, row0=0, device=None, local_median=False, gemm=None,
                 phi_gemm=None, gram_gemm=None, sym_layout=True, pair_split=None):
        """local_median: the median bandwidth is the lower median of the owned
        block's own m x n entries (k = (m n - 1) // 2, h = median / log n) --
        a rank-local bandwidth (the lagged DistSampler modes) -- instead of the
        n x n matrix's (whose rank k needs every row block's counts).

        gemm: the MFMA engine of the two contractions (phi_gemm / gram_gemm
        override it per contraction; None: DEFAULT_GEMM): "h2" the fp16 two-part split (default,
        include/dsvgd.h FmtH2), "x3" the bf16 three-part split, "f32" the exact
        f32 MFMA (precision reference).  sym_layout=False keeps the full D
        layout where the symmetric one would apply (layout experiments).

        pair_split=(rank, S): the owned block is rank's row block of S and
        the S ranks split the symmetric matrix by block pairs
        (dsvgd.pairsplit): distances() computes this rank's
        parts only, direction(p2p=...) exchanges the transposed partials.
        Needs the same scores on every rank, the FmtH2 engines, m = n / S a
        multiple of 256 (of 512 for even S), roundup(d, 32) a multiple of 256 and a bracketed
        (or fixed) bandwidth -- PhiEngine.pair_split_ok says whether it applies."""
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
        self._check_memory(dev)
        rows = self.n_pad + 128
        self.Y = torch.zeros(rows, self.ldy, **f32)
        self.norms = torch.zeros(rows, **f32)
        self.D = torch.empty(self.m_pad * self.n_pad, **f32)
        self.splits = lib.dsvgd_phi_splits(m, n, self.ldy)
        gemm = gemm or self.DEFAULT_GEMM
        phi_gemm = phi_gemm or gemm
        gram_gemm = gram_gemm or gemm
        if phi_gemm not in self.GEMMS or gram_gemm not in self.GEMMS:
            raise ValueError("gemm must be one of %s" % (self.GEMMS,))
        # the split engines address their images with 32-bit offsets: beyond
        # that, the exact f32 engine (include/dsvgd.h)
        bpe = {"h2": 4, "x3": 6}
        if phi_gemm != "f32" and self.n_pad * self.ldy * bpe[phi_gemm] >= (1 << 31):
            phi_gemm = "f32"
        self.gram_rows = self.n_pad + 256   # Yg image rows (include/dsvgd.h, dsvgd_sqdist_x3)
        if gram_gemm != "f32" and self.dp * self.gram_rows * bpe[gram_gemm] >= (1 << 31):
            gram_gemm = "f32"
        self.phi_gemm, self.gram_gemm, self.sym_layout = phi_gemm, gram_gemm, sym_layout
        if phi_gemm == "x3":
            nb = lib.dsvgd_ysplit_bytes(self.n_pad, self.ldy)
            self.Yx = torch.empty(nb // 2, dtype=torch.int16, device=dev)
        elif phi_gemm == "h2":
            nb = lib.dsvgd_h2_image_bytes(self.n_pad, self.ldy)
            self.Yx = torch.empty(nb // 2, dtype=torch.int16, device=dev)
        if gram_gemm == "x3":
            nb = lib.dsvgd_rowsplit_bytes(self.gram_rows, self.dp)
            self.Yg = torch.empty(nb // 2, dtype=torch.int16, device=dev)
        elif gram_gemm == "h2":
            nb = lib.dsvgd_h2_image_bytes(self.gram_rows, self.dp)
            self.Yg = torch.empty(nb // 2, dtype=torch.int16, device=dev)
        if gram_gemm == "h2":
            # per-row FmtH2 scales of Y's X half: the Gram's row image
            self.rsc = torch.ones(rows, **f32)
        if phi_gemm == "h2":
            # FmtH2 column scales of all of Y for phi_mm's B image
            # (dsvgd_h2_colscale layout: [s_c | 1/s_c | t | 1/t | range guard])
            self.yscale = torch.empty(2 * self.ldy + 3, **f32)
            # the range guard's fallback: phi_mm on the FmtX3 image (when its
            # 32-bit offsets allow; include/dsvgd.h FmtH2)
            self.m16_fb = self.ldy % 256 == 0
            if self.n_pad * self.ldy * 6 < (1 << 31):
                nb = lib.dsvgd_ysplit_bytes(self.n_pad, self.ldy)
                self.Yx3 = torch.empty(nb // 2, dtype=torch.int16, device=dev)
            else:
                # no FmtX3 image fits its 32-bit offsets: the guard's fallback
                # is the exact f32 phi_mm (dsvgd_phi_mm_gated), which reads the
                # full D layout only
                self.Yx3 = None
                self.sym_layout = False
        # d <= 1024: pack writes the column maxima the scales come from
        # (dsvgd_pack_h2 / dsvgd_h2_scales); wider, a separate pass over Y
        self.fused_scales = ("h2" in (phi_gemm, gram_gemm) and self.ldy <= lib.dsvgd_pack_max_ldy()
                             and d > self.DIRECT_MAX_D)
        if self.fused_scales:
            self.colmax_nb = lib.dsvgd_pack_blocks(rows)
            i32 = dict(dtype=torch.int32, device=dev)
            self.colmax = torch.zeros(self.colmax_nb * self.ldy, **i32)
            self.gmax = torch.zeros(4 * self.colmax_nb, **i32)
        elif "h2" in (phi_gemm, gram_gemm):
            self.scale_ws = torch.empty(
                max(1, lib.dsvgd_h2_colscale_workspace_floats(self.n_pad, self.ldy)), **f32)
        if self.sym and phi_gemm == "h2":
            # the one-launch form (phi_w1 DS 4) walks longer slices
            self.splits = int(lib.dsvgd_phi_splits_sym(n, self.ldy))
        self.KY = torch.empty(self.splits * m, self.ldy, **f32)
        self.rowsum = torch.empty(self.splits * self.m_pad, **f32)
        self.mean = torch.empty(d, **f32)    # the packing centre (dsvgd_colcenter)
        self.phi = torch.empty(m, d, **f32)
        self.state = SelectState(dev)
        self.plan = None
        if pair_split is not None:
            self._init_pair_split(*pair_split)
        self.k_rank = (m * n - 1) // 2 if (local_median and m < n) else -1
        self.bracketed = m * n >= self.BRACKET_MIN_ENTRIES and self.k_rank < 0
        if self.bracketed:
            s = self.SAMPLE
            half = 0.5 * s
            dk = self.SIGMAS * math.sqrt(s) / 2.0
            self.k_lo = max(0, int(math.floor(half - dk)))
            self.k_hi = min(s - 1, int(math.ceil(half + dk)))
            self.sample = torch.empty(s, **f32)
            self.st_lo, self.st_hi = SelectState(dev), SelectState(dev)
            # one fixed-capacity slot per distance-launch wave (include/dsvgd.h);
            # 1/16 of the entries leaves ~5x headroom over the ~1.2 % in bracket
            self.cand_cap = max(1 << 22, (m * n) // 16)
            self.cand = torch.empty(self.cand_cap, **f32)

    def set_row0(self, row0):
        """Move the owned block to rows [row0, row0 + m) of the same
        interacting set (no buffer depends on it; the symmetric layout is
        only used for row0 == 0 == n - m)."""
        assert 0 <= row0 and row0 + self.m <= self.n
        if row0 != self.row0:
            assert self.m < self.n, "the whole matrix has no other row block"
            self.row0 = row0

    def _check_memory(self, dev):
        """D is materialised (m_pad x n_pad fp32, no recompute path), so one
        engine's footprint grows as m n: refuse up front, with the sizes, what
        would otherwise be an allocator OOM halfway through the buffers."""
        d_bytes = 4 * self.m_pad * self.n_pad
        cand = 4 * max(1 << 22, (self.m * self.n) // 16) if self.m * self.n >= self.BRACKET_MIN_ENTRIES else 0
        splits = N.load().dsvgd_phi_splits(self.m, self.n, self.ldy)
        # Y, its FmtH2 image, the FmtX3 fallback image (1.5 Y) and the Gram's
        # row image, rounded up; the split-K partials
        other = 4 * ((self.n_pad + 128) * self.ldy * 4 + splits * self.m * self.ldy)
        need = d_bytes + cand + other
        free, _ = torch.cuda.mem_get_info(dev)
        # the caching allocator's reserved-but-unused blocks are free to torch too
        free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        if need > free:
            raise MemoryError(
                "PhiEngine(n=%d, d=%d, m=%d) needs %.1f GiB of device memory (D is %d x %d "
                "fp32 = %.1f GiB) but %.1f GiB are free; shard the rows over more ranks "
                "(DistSampler, m = n / num_shards) or reduce n"
                % (self.n, self.d, self.m, need / 2**30, self.m_pad, self.n_pad,
                   d_bytes / 2**30, free / 2**30))

    # ------------------------------------------------------------ stages --
    def pack(self, X, S=None, score_scale=1.0):
        """X, S: (n, d) device tensors (row stride may exceed d).  S=None packs
        the X half only and leaves Y's S half as it was (pack_scores fills it
        before direction(); the distances read only the X half)."""
        assert X.shape == (self.n, self.d)
        s = N.stream(self.device)
        with span(self.timer, "pack"):
            self._pack(X, S, score_scale, s)

    def pack_scores(self, S, score_scale=1.0):
        """Write only the S half of Y (the X half from an earlier pack(X))."""
        assert S.shape == (self.n, self.d)
        s = N.stream(self.device)
        with span(self.timer, "pack"):
            N.call("dsvgd_pack_h2", None, self.d, N.ptr(S), N.ld(S), float(score_scale), None,
                   self.n, self.d, self.Y.shape[0], N.ptr(self.Y), self.ldy, None,
                   *self._maxima(), None, s)

    def _maxima(self):
        if self.fused_scales:
            return N.ptr(self.colmax), N.ptr(self.gmax)
        return None, None

    def _scales(self, cols, out, s):
        """FmtH2 column scales of Y's first `cols` columns into `out`."""
        if self.fused_scales:
            N.call("dsvgd_h2_scales", N.ptr(self.colmax), N.ptr(self.gmax), self.colmax_nb,
                   self.ldy, cols, self.dp, N.ptr(out), s)
        else:   # d > 1024: a pass over Y, with the range guard of its halves
            N.call("dsvgd_h2_colscale_guarded", N.ptr(self.Y), self.ldy, self.n_pad, cols,
                   min(self.dp, cols), N.ptr(self.scale_ws), N.ptr(out), s)

    def _pack(self, X, S, score_scale, s):
        N.call("dsvgd_colcenter", N.ptr(X), N.ld(X), self.n, self.d, N.ptr(self.mean), s)
        lds = N.ld(S) if S is not None else self.d
        if S is not None:
            assert S.shape == (self.n, self.d)
        rsc = self.rsc if (self.gram_gemm == "h2" and self.fused_scales) else None
        N.call("dsvgd_pack_h2", N.ptr(X), N.ld(X), N.ptr(S), lds, float(score_scale),
               N.ptr(self.mean), self.n, self.d, self.Y.shape[0], N.ptr(self.Y), self.ldy,
               N.ptr(self.norms), *self._maxima(), N.ptr(rsc), s)

    def distances(self, median=False):
        """D for the owned rows.  median=True also does the select's first
        stage: the fused digit-1 histogram, or (bracketed) the sample bracket +
        the below-count / candidate compaction."""
        s = N.stream(self.device)
        st, cand, mode = None, None, SEL_NONE
        if median and self.bracketed:
            with span(self.timer, "bracket"):
                self._bracket(s)
            st, cand, mode = self.state.ptr, N.ptr(self.cand), SEL_BRACKET
        elif median:
            N.call("dsvgd_select_init", self.state.ptr, self.n, self.k_rank, s)
            st, mode = self.state.ptr, SEL_HIST
        if self.plan is not None:
            with span(self.timer, "rowsplit"):
                N.call("dsvgd_h2_rowsplit_rows", N.ptr(self.Y), self.ldy, self.n_pad, self.dp,
                       self.gram_rows, self.dp, N.ptr(self.rsc), N.ptr(self.Yg), s)
            with span(self.timer, "sqdist"):
                self._gram_parts(self._gparts, mode, st, cand, s)
            return
        if self.gram_gemm == "h2" and self.d > self.DIRECT_MAX_D:
            with span(self.timer, "rowsplit"):
                if not self.fused_scales:   # (pack wrote them otherwise)
                    N.call("dsvgd_h2_rowscale", N.ptr(self.Y), self.ldy, self.n_pad, self.dp,
                           self.rsc.numel(), N.ptr(self.rsc), None, s)
                N.call("dsvgd_h2_rowsplit_rows", N.ptr(self.Y), self.ldy, self.n_pad, self.dp,
                       self.gram_rows, self.dp, N.ptr(self.rsc), N.ptr(self.Yg), s)
            with span(self.timer, "sqdist"):
                N.call("dsvgd_sqdist_h2", N.ptr(self.Yg), N.ptr(self.norms), self.row0, self.m,
                       self.n, self.d, N.ptr(self.D), self.n_pad, mode, st, cand, int(self.sym),
                       N.ptr(self.rsc), s)
            return
        if self.gram_gemm == "x3" and self.d > self.DIRECT_MAX_D:
            with span(self.timer, "rowsplit"):
                # the 256-tile Gram runs 16x16x32 MFMAs on an unswizzled image
                N.call("dsvgd_rowsplit", N.ptr(self.Y), self.ldy, self.n_pad, self.dp,
                       self.gram_rows, self.dp, N.ptr(self.Yg), 0, s)
            with span(self.timer, "sqdist"):
                N.call("dsvgd_sqdist_x3", N.ptr(self.Yg), N.ptr(self.norms), self.row0, self.m,
                       self.n, self.d, N.ptr(self.D), self.n_pad, mode, st, cand, int(self.sym), s)
            return
        with span(self.timer, "sqdist"):
            fn = "dsvgd_sqdist_direct" if self.d <= self.DIRECT_MAX_D else "dsvgd_sqdist"
            N.call(fn, N.ptr(self.Y), self.ldy, N.ptr(self.norms), self.row0, self.m,
                   self.n, self.d, N.ptr(self.D), self.n_pad, mode, st, cand, s)

    # (rank, S, gather): the S ranks that share this interacting set (same Y)
    # each compute 1/S of the bracket sample and gather(sample, start, end)
    # all-gathers the shares in place (DistSampler, particles exchanged)
    sample_share = None

    def _bracket(self, s):
        if self.sample_share is not None and self.SAMPLE % self.sample_share[1] == 0:
            rank, S, gather = self.sample_share
            per = self.SAMPLE // S
            N.call("dsvgd_sample_sqdist_range", N.ptr(self.Y), self.ldy, self.n, self.d,
                   self.SAMPLE, self.SEED, rank * per, (rank + 1) * per, N.ptr(self.sample), s)
            gather(self.sample, rank * per, (rank + 1) * per)
            N.call("dsvgd_sample_bracket_select", N.ptr(self.sample), self.SAMPLE, self.k_lo,
                   self.k_hi, self.st_lo.ptr, self.st_hi.ptr, self.state.ptr, self.n,
                   self.cand_cap, s)
            return
        N.call("dsvgd_sample_bracket", N.ptr(self.Y), self.ldy, self.n, self.d, self.SAMPLE,
               self.SEED, self.k_lo, self.k_hi, N.ptr(self.sample), self.st_lo.ptr,
               self.st_hi.ptr, self.state.ptr, self.n, self.cand_cap, s)

    def median_bandwidth(self, allreduce=None):
        """Exact radix select (after distances(median=True)); `allreduce` sums
        an int64 device tensor over the ranks that share the n x n matrix."""
        s = N.stream(self.device)
        count = self.m_pad * self.n_pad
        cand = None
        if self.bracketed:
            N.call("dsvgd_bracket_totals", self.state.ptr, N.ptr(self.cand), s)
            if allreduce is not None:
                allreduce(self.state.totals)
            N.call("dsvgd_bracket_check", self.state.ptr, s)
            cand = N.ptr(self.cand)
        for p in (1, 2, 3):
            if p > 1 or self.bracketed:
                with span(self.timer, "radix_hist"):
                    if self.plan is not None:   # the fallback over D weighs the rank's tiles
                        N.call("dsvgd_radix_hist_wmap", N.ptr(self.D), self.m_pad, self.n_pad,
                               cand, p, self.state.ptr, N.ptr(self.wmap), s)
                    else:
                        N.call("dsvgd_radix_hist", N.ptr(self.D), count, cand, p,
                               self.state.ptr, self.n_pad if self.sym else 0, s)
            if allreduce is not None:
                with span(self.timer, "hist_allreduce"):
                    allreduce(self.state.hist)
            N.call("dsvgd_radix_pick", self.state.ptr, p, s)

    def fixed_bandwidth(self, h):
        N.call("dsvgd_set_bandwidth", self.state.ptr, float(h), N.stream(self.device))

    # d <= 2: explicit-difference distances and pairwise phi (the Gram /
    # K.X form cancels past the 1e-5 tolerance at d = 1); d >= 3: MFMA (as
    # or more accurate there, scripts/precision_small_d.py).  Must match the
    # library's default (kDirectDefaultD in csrc/sqdist.hip).
    DIRECT_MAX_D = 2

    @property
    def x3(self):
        """phi_mm runs on a split engine (h2 or x3), not the f32 MFMA."""
        return self.phi_gemm != "f32"

    @property
    def x3_gram(self):
        """the Gram runs on a split engine (h2 or x3), not the f32 MFMA."""
        return self.gram_gemm != "f32"

    @property
    def m16(self):
        """phi_mm's x3 engine on v_mfma_f32_16x16x32_bf16 (ldy % 256 == 0)."""
        return self.phi_gemm == "x3" and self.ldy % 256 == 0

    @property
    def sym(self):
        """D is in the symmetric layout (upper-triangle tiles only, written by
        dsvgd_sqdist_{h2,x3} layout 1 and read transposed by dsvgd_phi_mm_{h2,x3}
        and dsvgd_radix_hist): the whole n x n matrix on the split engines,
        with ldy % 256 == 0."""
        return (self.m == self.n and self.row0 == 0 and self.d > self.DIRECT_MAX_D
                and self.x3 and self.x3_gram and self.ldy % 256 == 0 and self.sym_layout)

    def direction(self, X_own=None, step=0.0, write_phi=True, inv_n=None, extra=None, p2p=None):
        """phi for the owned rows (+ `extra`, e.g. the h * W2 gradient rows);
        optionally X_own += step * phi (in place).
        d <= DIRECT_MAX_D: pairwise VALU form (dsvgd_phi_direct); else K.[Xc|S] on MFMA.
        Pair split: p2p(sends, recvs) posts the partials' exchange
        ([(tensor, rank)] each) and returns a callable that joins it."""
        s = N.stream(self.device)
        if self.plan is not None:
            self._direction_pair_split(X_own, step, write_phi, inv_n, extra, p2p, s)
            return
        if X_own is not None:
            assert X_own.shape == (self.m, self.d)
        if extra is not None:
            assert extra.shape == (self.m, self.d) and extra.dtype == torch.float32
        ex, lde = (N.ptr(extra), N.ld(extra)) if extra is not None else (None, self.d)
        inv_n = 1.0 / self.n if inv_n is None else inv_n
        phi = N.ptr(self.phi) if write_phi else None
        xo = N.ptr(X_own)
        ldx = N.ld(X_own) if X_own is not None else self.d
        if self.d <= self.DIRECT_MAX_D:
            with span(self.timer, "phi_direct"):
                # KY (the MFMA path's split-K buffer) doubles as the split-J scratch
                N.call("dsvgd_phi_direct", N.ptr(self.D), self.n_pad, N.ptr(self.Y), self.ldy,
                       self.row0, self.m, self.n, self.d, self.state.ptr, float(inv_n),
                       float(step), ex, lde, phi, self.d, xo, ldx, N.ptr(self.KY),
                       self.KY.numel(), s)
            return
        if self.sym and self.phi_gemm == "h2":
            # the slices were sized for the symmetric phi_mm form in force at
            # construction (dsvgd_phi_splits_sym: longer slices for the
            # one-launch form only); if the form was switched since
            # (dsvgd_phi_set_symrow), re-size them for the current one
            want = int(N.load().dsvgd_phi_splits_sym(self.n, self.ldy))
            if want != self.splits:
                self.splits = want
                self.KY = torch.empty(want * self.m, self.ldy, dtype=torch.float32,
                                      device=self.device)
                self.rowsum = torch.empty(want * self.m_pad, dtype=torch.float32,
                                          device=self.device)
        if self.phi_gemm == "h2":
            # the range guard word of the scales: phi_mm_h2 runs while it
            # reads 0; otherwise the FmtX3 image and phi_mm_x3 behind it do,
            # or (no FmtX3 image fits) the exact f32 phi_mm (all stay on the
            # stream -- no host round trip)
            guard = N.ptr(self.yscale) + 4 * (2 * self.ldy + 2)
            with span(self.timer, "ysplit"):
                self._scales(self.ldy, self.yscale, s)
                N.call("dsvgd_h2_ysplit", N.ptr(self.Y), self.ldy, self.n_pad,
                       N.ptr(self.yscale), N.ptr(self.Yx), s)
            with span(self.timer, "phi_mm"):
                N.call("dsvgd_phi_mm_h2", N.ptr(self.D), self.n_pad, N.ptr(self.Yx), self.ldy,
                       self.row0, self.m, self.n, self.state.ptr, self.splits, N.ptr(self.KY),
                       self.ldy, N.ptr(self.rowsum), int(self.sym),
                       N.ptr(self.yscale) + 4 * self.ldy, guard, s)
            if self.Yx3 is None:
                with span(self.timer, "phi_guard"):
                    N.call("dsvgd_phi_mm_gated", N.ptr(self.D), self.n_pad, N.ptr(self.Y),
                           self.ldy, self.row0, self.m, self.n, self.state.ptr, self.splits,
                           N.ptr(self.KY), self.ldy, N.ptr(self.rowsum), guard, s)
            else:
                with span(self.timer, "phi_guard"):
                    N.call("dsvgd_ysplit", N.ptr(self.Y), self.ldy, self.n_pad, N.ptr(self.Yx3),
                           0 if self.m16_fb else 1, guard, s)
                    N.call("dsvgd_phi_mm_x3", N.ptr(self.D), self.n_pad, N.ptr(self.Yx3),
                           self.ldy, self.row0, self.m, self.n, self.state.ptr, self.splits,
                           N.ptr(self.KY), self.ldy, N.ptr(self.rowsum), int(self.sym),
                           int(self.m16_fb), guard, s)
        elif self.x3:
            m16 = self.m16
            with span(self.timer, "ysplit"):
                N.call("dsvgd_ysplit", N.ptr(self.Y), self.ldy, self.n_pad, N.ptr(self.Yx),
                       0 if m16 else 1, None, s)
            with span(self.timer, "phi_mm"):
                N.call("dsvgd_phi_mm_x3", N.ptr(self.D), self.n_pad, N.ptr(self.Yx), self.ldy,
                       self.row0, self.m, self.n, self.state.ptr, self.splits, N.ptr(self.KY),
                       self.ldy, N.ptr(self.rowsum), int(self.sym), int(m16), None, s)
        else:
            with span(self.timer, "phi_mm"):
                N.call("dsvgd_phi_mm", N.ptr(self.D), self.n_pad, N.ptr(self.Y), self.ldy,
                       self.row0, self.m, self.n, self.state.ptr, self.splits, N.ptr(self.KY),
                       self.ldy, N.ptr(self.rowsum), s)
        N.call("dsvgd_phi_finish", N.ptr(self.KY), self.ldy, N.ptr(self.rowsum), self.splits,
               N.ptr(self.Y), self.ldy, self.row0, self.m, self.d, self.dp, self.state.ptr,
               float(inv_n), float(step), ex, lde, phi, self.d, xo, ldx, s)

    # ---------------------------------------------------- pair split --
    @classmethod
    def pair_split_ok(cls, n, d, S, gemm=None, median=True):
        """Whether PhiEngine(n, d, m=n/S, pair_split=(r, S)) applies."""
        lib = N.load()
        m = n // S
        dp = lib.dsvgd_dp(d)
        ldy = lib.dsvgd_ldy(dp)
        n_pad = lib.dsvgd_pad128(n)
        from .pairsplit import PairSplitPlan
        return (S >= 2 and m * S == n and PairSplitPlan.aligned(S, m) and dp % 256 == 0
                and ldy % 512 == 0
                and (gemm or cls.DEFAULT_GEMM) == "h2" and d > cls.DIRECT_MAX_D
                and n_pad * ldy * 6 < (1 << 31) and dp * (n_pad + 256) * 4 < (1 << 31)
                and (not median or m * n >= cls.BRACKET_MIN_ENTRIES)
                and ldy <= lib.dsvgd_pack_max_ldy())

    def _init_pair_split(self, rank, S):
        from .pairsplit import PairSplitPlan
        lib = N.load()
        if not (self.m * S == self.n and self.row0 == rank * self.m and self.phi_gemm == "h2"
                and self.gram_gemm == "h2" and self.fused_scales and self.Yx3 is not None
                and self.ldy % 512 == 0 and self.dp % 256 == 0
                and PairSplitPlan.aligned(S, self.m)):
            raise ValueError("pair_split needs m = n / S = the rank's block, the FmtH2 engines, "
                             "m % 256 == 0 (m % 512 == 0 for even S) and "
                             "roundup(d, 32) % 256 == 0")
        P = self.plan = PairSplitPlan(rank, S, self.m)
        self._side = None   # WINDOW_SIDE_STREAM's stream
        dev, f32 = self.device, dict(dtype=torch.float32, device=self.device)

        def gparts(lst):
            arr = (N.GramPart * len(lst))()
            for a, q in zip(arr, lst):
                a.row_off, a.rows, a.col0, a.cols = q["row_off"], q["rows"], q["col0"], q["cols"]
                a.kind, a.weight2 = q["kind"], q["weight2"]
            return arr
        self._gparts = gparts(P.gram_parts)
        self._fbparts = gparts(P.fallback_parts)
        self.wmap = torch.tensor(P.tile_weights(), dtype=torch.uint8, device=dev).reshape(-1)
        # rows of the FmtH2 B image the rank's products read (16-row K-steps;
        # the image's byte offset of row r is 4 r ldy, like Y's)
        self._yx_rows = P.image_rows()
        ldy = self.ldy
        # own direct product over the window: split-K slices into KY (the
        # fallback's whole-row phi_mm uses self.splits slices of the same KY)
        wlen = P.window[1]
        self.w_splits = self.W_SPLITS or self.window_split(self.m, wlen, ldy)
        need = max(self.w_splits, self.splits)
        if self.KY.shape[0] < need * self.m:
            self.KY = torch.empty(need * self.m, ldy, **f32)
            self.rowsum = torch.empty(need * self.m_pad, **f32)
        # the high rank's row half: its own slices
        if P.row_half:
            ro, nr, c0, nc = P.row_half
            self.h_splits = self.H_SPLITS or int(lib.dsvgd_phi_splits(nr, nc, ldy))
            self.KYh = torch.empty(self.h_splits * nr, ldy, **f32)
            self.rsh = torch.empty(self.h_splits * lib.dsvgd_pad128(nr), **f32)

        # partials: one message per peer = [mo x ldy | roundup128(mo)] floats
        def msg(rows):
            return torch.empty(rows * ldy + lib.dsvgd_pad128(rows), **f32)
        # the forward blocks' partials in ONE launch without split-K when
        # they fill most of the CUs (S >= 8: 3 x 64 workgroups of 512
        # K-steps), written straight into one contiguous message buffer
        nf = len(P.forward)
        self.fwd_msg = self.m * ldy + lib.dsvgd_pad128(self.m)
        self.fwd_batched = nf > 0 and nf * (self.m // 128) * (ldy // 512) >= 192
        self.send_fwd = torch.empty(max(1, nf) * self.fwd_msg, **f32) if self.fwd_batched else None
        self.fwd_z = 1
        if self.fwd_batched:
            wg = nf * (self.m // 128) * (ldy // 512)
            self.fwd_z = self.FWD_ZSPLIT or self.fill_split(wg, self.m)
        self.fwd_tmp = (torch.empty(self.fwd_z * nf * self.fwd_msg, **f32)
                        if self.fwd_z > 1 else None)
        self.t_splits = []
        smax = 0
        for k, q in enumerate(P.sends):
            blocks = (ldy // 512) * (q["mo"] // 128)
            z = 1
            while blocks * z < 256 and q["krows"] // (2 * z) >= 1024:
                z *= 2
            if self.REST_SPLITS and k >= (nf if self.fwd_batched else 0):
                z = self.REST_SPLITS
            self.t_splits.append(z)
            smax = max(smax, z * q["mo"]) if z > 1 else smax
        fwd_wg = nf * (self.m // 128) * (ldy // 512) if self.fwd_batched else 0
        rest_wg = [(ldy // 512) * (q["mo"] // 128) for q in P.sends[nf:]]
        self.rest_beside = bool(self.REST_BESIDE and self.fwd_batched and rest_wg
                                and fwd_wg + sum(rest_wg) <= 256)
        if self.rest_beside:
            for k in range(nf, len(P.sends)):
                self.t_splits[k] = 1
        self._tside = None
        self.sendbuf = [msg(q["mo"]) for q in P.sends]
        if self.fwd_batched:   # the forward messages as views of the one buffer
            for k in range(nf):
                self.sendbuf[k] = self.send_fwd[k * self.fwd_msg:(k + 1) * self.fwd_msg]
        self.recvbuf = [msg(q["rows"]) for q in P.recvs]
        mo_max = max([q["mo"] for q in P.sends] + [128])
        self.tP = torch.empty(max(smax, 1), ldy, **f32)
        self.tRS = torch.empty(max(t for t in self.t_splits) * lib.dsvgd_pad128(mo_max), **f32)
        parts = []
        if P.row_half:
            ro, nr, _, _ = P.row_half
            parts.append((N.ptr(self.KYh), N.ptr(self.rsh), ldy, ro, nr, self.h_splits))
        for q, buf in zip(P.recvs, self.recvbuf):
            parts.append((N.ptr(buf), N.ptr(buf) + 4 * q["rows"] * ldy, ldy, q["row_off"],
                          q["rows"], 1))
        arr = (N.PhiPart * len(parts))()
        for a, q in zip(arr, parts):
            a.ky, a.rs, a.ldk, a.row_off, a.rows, a.splits = q
        self._phiparts = arr

    @staticmethod
    def window_split(m, wlen, ldy, cus=256, max_chain=16384):
        """The own window's split-K factor: the smallest power of two whose
        workgroups (m/128 row blocks x ldy/512 column blocks each) cover the
        CUs once, with at most max_chain columns per slice (phi_splits'
        precision bound) -- one wave of long slices rather than
        dsvgd_phi_splits' two: half the slices to write and re-read in
        phi_finish_parts (S = 8: 3.19 vs 3.25 ms, profiles/r13k)."""
        wg = (m // 128) * max(1, ldy // 512)
        z = 1
        while (wg * z < cus or -(-wlen // z) > max_chain) and z < 64 and wlen // (2 * z) >= 1024:
            z *= 2
        return z

    @staticmethod
    def fill_split(wg, rows, cus=256, min_rows=1024):
        """The split-K factor z (a power of two, rows / z >= min_rows) whose
        wg * z workgroups -- one per CU at a time -- fill whole waves of the
        CUs best (ties: the smallest z)."""
        best, best_eff = 1, 0.0
        z = 1
        while z <= 16 and rows // z >= min_rows and rows % (16 * z) == 0:
            w = wg * z
            eff = w / (cus * -(-w // cus))
            if eff > best_eff + 1e-9:
                best, best_eff = z, eff
            z *= 2
        return best

    def _gram_parts(self, arr, mode, st, cand, s, gate=None):
        N.call("dsvgd_sqdist_h2_parts", N.ptr(self.Yg), N.ptr(self.norms), self.row0, self.m,
               self.n, self.d, N.ptr(self.D), self.n_pad, mode, st, cand, ctypes.addressof(arr),
               len(arr), gate, N.ptr(self.rsc), s)

    def _direction_pair_split(self, X_own, step, write_phi, inv_n, extra, p2p, s):
        """phi of the owned rows in the pair-split layout: the transposed
        partials of the blocks this rank holds for others (sent as soon as
        they are reduced), the own window (and row half) while they travel,
        then phi_finish over the own slices + the partials received.  The
        FmtH2 range guard (device word) instead runs the FmtX3 phi_mm over
        the whole row block, after the Gram of the parts this rank does not
        hold (gated launches: no host round trip)."""
        P, ldy, lib = self.plan, self.ldy, N.load()
        guard = N.ptr(self.yscale) + 4 * (2 * ldy + 2)
        colinv = N.ptr(self.yscale) + 4 * ldy
        with span(self.timer, "ysplit"):
            self._scales(ldy, self.yscale, s)
            # only the rows the rank's products read: its window, the high
            # rank's antipodal block (the row half's columns); the transposed
            # partials read the own rows, inside the window.  (The guard's
            # fallback reads the FmtX3 image, made from Y.)
            for r0, nr in self._yx_rows:
                N.call("dsvgd_h2_ysplit", N.ptr(self.Y) + 4 * r0 * ldy, ldy, nr,
                       N.ptr(self.yscale), N.ptr(self.Yx) + 4 * r0 * ldy, s)
        fork = torch.cuda.current_stream(self.device).record_event() \
            if self.WINDOW_SIDE_STREAM else None
        with span(self.timer, "phi_partials"):
            nf = len(P.forward) if self.fwd_batched else 0
            if nf and self.fwd_z > 1:
                N.call("dsvgd_phi_h2_transposed_blocks_split", N.ptr(self.D), self.n_pad,
                       N.ptr(self.Yx), ldy, self.row0, self.m, (P.rank + 1) % P.S, P.S, nf,
                       self.fwd_z, self.n, self.state.ptr, N.ptr(self.fwd_tmp), ldy,
                       self.fwd_msg, colinv, guard, 0, s)
                N.call("dsvgd_phi_partial_reduce_blocks", N.ptr(self.fwd_tmp), ldy, self.fwd_msg,
                       self.fwd_z, nf, self.m, ldy, N.ptr(self.send_fwd), ldy, self.fwd_msg, s)
            elif nf:
                N.call("dsvgd_phi_h2_transposed_blocks", N.ptr(self.D), self.n_pad,
                       N.ptr(self.Yx), ldy, self.row0, self.m, (P.rank + 1) % P.S, P.S, nf,
                       self.n, self.state.ptr, N.ptr(self.send_fwd), ldy, self.fwd_msg, colinv,
                       guard, 0, s)
            beside = bool(nf) and self.rest_beside
            main = torch.cuda.current_stream(self.device)
            if beside:
                if self._tside is None:
                    self._tside = torch.cuda.Stream(device=self.device)
                self._tside.wait_stream(main)     # behind ysplit only
            with torch.cuda.stream(self._tside if beside else main):
                sr = N.stream(self.device)
                for q, z, buf in list(zip(P.sends, self.t_splits, self.sendbuf))[nf:]:
                    Dq = N.ptr(self.D) + 4 * q["row_off"] * self.n_pad
                    mo = q["mo"]
                    rs_out = N.ptr(buf) + 4 * mo * ldy
                    if z == 1:
                        N.call("dsvgd_phi_h2_transposed", Dq, self.n_pad, N.ptr(self.Yx), ldy,
                               self.row0 + q["row_off"], q["krows"], q["col0"], mo, self.n,
                               self.state.ptr, 1, N.ptr(buf), ldy, rs_out, colinv, guard, 0, sr)
                    else:
                        N.call("dsvgd_phi_h2_transposed", Dq, self.n_pad, N.ptr(self.Yx), ldy,
                               self.row0 + q["row_off"], q["krows"], q["col0"], mo, self.n,
                               self.state.ptr, z, N.ptr(self.tP), ldy, N.ptr(self.tRS), colinv,
                               guard, 0, sr)
                        N.call("dsvgd_phi_partial_reduce", N.ptr(self.tP), ldy, N.ptr(self.tRS),
                               z, mo, ldy, N.ptr(buf), ldy, rs_out, sr)
            if beside:
                main.wait_stream(self._tside)     # every partial before the exchange
        join = None
        if p2p is not None:
            with span(self.timer, "partials_post"):
                join = p2p([(b, q["dest"]) for q, b in zip(P.sends, self.sendbuf)],
                           [(b, q["src"]) for q, b in zip(P.recvs, self.recvbuf)])
        # the own window: after the partials on this stream, or (the A/B
        # option) on a second stream that waited only for ysplit
        main = torch.cuda.current_stream(self.device)
        side = self.WINDOW_SIDE_STREAM
        if side:
            if self._side is None:
                self._side = torch.cuda.Stream(device=self.device)
            self._side.wait_event(fork)
        with torch.cuda.stream(self._side if side else main):
            sw = N.stream(self.device)
            with span(self.timer, "phi_mm"):
                w0, wl = P.window
                N.call("dsvgd_phi_h2_window", N.ptr(self.D), self.n_pad, N.ptr(self.Yx), ldy,
                       self.row0, self.m, self.n, w0, wl, self.state.ptr, self.w_splits,
                       N.ptr(self.KY), ldy, N.ptr(self.rowsum), colinv, guard, 0, sw)
                if P.row_half:
                    ro, nr, c0, nc = P.row_half
                    N.call("dsvgd_phi_h2_window", N.ptr(self.D) + 4 * ro * self.n_pad,
                           self.n_pad, N.ptr(self.Yx), ldy, self.row0 + ro, nr, self.n, c0, nc,
                           self.state.ptr, self.h_splits, N.ptr(self.KYh), ldy, N.ptr(self.rsh),
                           colinv, guard, 0, sw)
        if side:
            main.wait_stream(self._side)   # KY / rowsum, and D free for the next Gram
        with span(self.timer, "phi_guard"):
            # the range guard's fallback: the rest of the row block's D, then
            # the FmtX3 phi_mm over all of it (gated: nothing while the guard is 0)
            self._gram_parts(self._fbparts, SEL_NONE, None, None, s, gate=guard)
            N.call("dsvgd_ysplit", N.ptr(self.Y), ldy, self.n_pad, N.ptr(self.Yx3),
                   0 if self.m16_fb else 1, guard, s)
            N.call("dsvgd_phi_mm_x3", N.ptr(self.D), self.n_pad, N.ptr(self.Yx3), ldy, self.row0,
                   self.m, self.n, self.state.ptr, self.splits, N.ptr(self.KY), ldy,
                   N.ptr(self.rowsum), 0, int(self.m16_fb), guard, s)
        if join is not None:
            with span(self.timer, "partials_wait"):
                join()
        if extra is not None:
            assert extra.shape == (self.m, self.d) and extra.dtype == torch.float32
        ex, lde = (N.ptr(extra), N.ld(extra)) if extra is not None else (None, self.d)
        inv_n = 1.0 / self.n if inv_n is None else inv_n
        phi = N.ptr(self.phi) if write_phi else None
        xo = N.ptr(X_own)
        ldx = N.ld(X_own) if X_own is not None else self.d
        N.call("dsvgd_phi_finish_parts", N.ptr(self.KY), ldy, N.ptr(self.rowsum), self.w_splits,
               N.ptr(self.Y), ldy, self.row0, self.m, self.d, self.dp, self.state.ptr,
               float(inv_n), float(step), ex, lde, phi, self.d, xo, ldx,
               ctypes.addressof(self._phiparts), len(self._phiparts), guard, self.splits, s)

    def range_guard(self):
        """The last phi_mm's FmtH2 range guard (True: it ran on the fallback
        -- the FmtX3 engine, or the exact f32 one where no FmtX3 image fits;
        None: not the h2 engine) -- synchronises."""
        if self.phi_gemm != "h2" or self.d <= self.DIRECT_MAX_D:
            return None
        return bool(float(self.yscale[2 * self.ldy + 2]) != 0.0)

    # ------------------------------------------------------------ helpers --
    def step(self, X, S, X_own=None, step=0.0, h=None, score_scale=1.0, allreduce=None,
             write_phi=True, extra=None):
        """One Jacobi step: h=None -> median bandwidth, else fixed h."""
        self.pack(X, S, score_scale)
        median = h is None
        self.distances(median=median)
        if median:
            self.median_bandwidth(allreduce)
        else:
            self.fixed_bandwidth(h)
        self.direction(X_own, step, write_phi, extra=extra)

    def dense_D(self, padded=False):
        """D as a dense (m, n) tensor (tests/inspection; un-does the panel
        layout, and in the symmetric layout fills the unwritten lower tiles
        from the stored upper ones).  padded: the whole (m_pad, n_pad) buffer."""
        mp, np_ = self.m_pad, self.n_pad
        Dd = self.D.view(mp // 128, np_ // 16, 128, 16).permute(0, 2, 1, 3).reshape(mp, np_)
        if self.sym:
            Dd = Dd.clone()
            for I in range(1, np_ // 128):
                Dd[I * 128:(I + 1) * 128, :I * 128] = Dd[:I * 128, I * 128:(I + 1) * 128].t()
        return Dd if padded else Dd[:self.m, :self.n]

    def count_D(self, pred):
        """Entries of the full n_pad x n_pad D matching pred (a tensor -> bool
        tensor function), counted without densifying: in the symmetric layout
        an off-diagonal stored tile stands for its transpose too."""
        if not self.sym:
            return int(pred(self.D).sum())
        T = self.n_pad // 128
        c = torch.stack([pred(self.D.view(T, T, 128 * 128)[I]).sum(-1) for I in range(T)])
        w = torch.triu(torch.full((T, T), 2, dtype=c.dtype, device=c.device), 1)
        w += torch.eye(T, dtype=c.dtype, device=c.device)
        return int((c * w).sum())


class StepGraph(object):
    """One SVGD iteration captured as a HIP graph and replayed.

    Every libdsvgd_hip call only enqueues kernels on the current stream (no
    allocation, no host synchronisation), so a whole iteration -- scores, the
    median select, and for the reference's Gauss-Seidel order the n row
    kernels plus n per-particle score refreshes -- is capturable.  The first
    call runs eagerly (workspaces get allocated), the second captures
    (torch.cuda.CUDAGraph = hipGraph on ROCm) and every call replays; at
    small n the eager loop is launch-bound (two host launches per particle),
    the replay is not.  `fn` must keep its device buffers fixed across calls.
    """

    def __init__(self, fn, device, enabled=True):
        self.fn, self.device, self.enabled = fn, device, enabled
        self.graph = None
        self.calls = 0

    def __call__(self):
        self.calls += 1
        if not self.enabled or self.calls == 1:
            self.fn()
            return
        if self.graph is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.device(self.device), torch.cuda.graph(g):
                self.fn()
            self.graph = g
        self.graph.replay()


_ROW_PARTIALS = {}   # (device, blocks, d) -> partial sums of dsvgd_phi_row_split (kept: graphs)


_GS_PARTIALS = {}    # (device, nsplit, d) -> split-J partials of dsvgd_gs_block_part (kept: graphs)
GS_BLOCK_MIN_ROWS = 128   # shorter sweeps keep the per-row kernels


def _gs_score_kind(target):
    """The blocked sweeps refresh the built-in targets' scores themselves:
    dsvgd_gs_block_sweep's / dsvgd_gsw_block_sweep's score_kind (3, the
    logistic regression: the wide sweep only), or None (per-row path)."""
    from .targets import Gaussian, GaussianMixture1D, LogisticRegression
    if target is None:
        return 0
    if isinstance(target, Gaussian):
        return 1
    if isinstance(target, GaussianMixture1D):
        return 2
    if isinstance(target, LogisticRegression):
        return 3
    return None


def sequential_sweep(X, S, rows, h_state, step, target=None, score_scale=1.0, phi_out=None,
                     extra=None, blocked=True):
    """Gauss-Seidel sweep in the reference order over `rows` of the interacting
    set X (n, d): for each i, phi_i from the CURRENT X (earlier rows already
    moved), X[i] += step * (phi_i + extra[k]), then (if `target`) S[i] is
    recomputed for the moved particle, which is what re-running _dlogp per
    pair amounts to (dsvgd/sampler.py:64-68, dsvgd/distsampler.py:194-200).
    extra: optional (len(rows), d) contiguous rows (the h * W2 gradient).

    Blocked form (contiguous rows, frozen scores or a built-in target): a
    block of rows at a time, one wide pass for the block against all n rows
    and one workgroup for the in-block order (csrc/gs.hip) -- the same sweep;
    d <= 64 with an elementwise target on the VALU form, 64 < d <= 1024 (and
    the logistic regression at any d <= 1024, its score refreshed in the
    walk) on the wide one; otherwise one row kernel (+ one score refresh) per
    row."""
    n, d = X.shape
    s = N.stream(X.device)
    if extra is not None:
        assert extra.is_contiguous() and extra.shape == (len(rows), d)
    kind = _gs_score_kind(target)
    rows = range(rows.start, rows.stop) if isinstance(rows, range) else rows
    contiguous = isinstance(rows, range) and rows.step == 1
    if (blocked and kind is not None and contiguous and len(rows) >= GS_BLOCK_MIN_ROWS
            and X.is_contiguous() and S.is_contiguous()):
        if d <= 64 and kind != 3:
            _blocked_sweep(X, S, rows, h_state, step, kind, target, score_scale, phi_out, extra, s)
            return
        if d <= GSW_MAX_D:
            _blocked_sweep_wide(X, S, rows, h_state, step, kind, target, score_scale, phi_out,
                                extra, s)
            return
    blocks = int(N.load().dsvgd_phi_row_blocks(n, d))
    part = None
    if blocks > 1:
        # the j range of each row over `blocks` workgroups (csrc/phi.hip)
        key = (X.device, blocks, d)
        part = _ROW_PARTIALS.get(key)
        if part is None:
            part = _ROW_PARTIALS[key] = torch.empty(blocks * d, dtype=torch.float32,
                                                    device=X.device)
    for k, i in enumerate(rows):
        ex = N.ptr(extra[k]) if extra is not None else None
        po = N.ptr(phi_out[k]) if phi_out is not None else None
        if part is None:
            N.call("dsvgd_phi_row", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), n, d, int(i),
                   h_state.ptr, float(step), ex, po, s)
        else:
            N.call("dsvgd_phi_row_split", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), n, d, int(i),
                   h_state.ptr, float(step), ex, po, N.ptr(part), blocks, s)
        if target is not None:
            target.score(X[i:i + 1], S[i:i + 1], score_scale)


GSW_MAX_D = 1024       # the wide blocked sweep (csrc/gs.hip gsw_sweep_kernel)
GSW_GEMM = "split"     # its wide pass: "split" (FmtH2 Gram + FmtX3 phi_mm) or "f32"


class _WideSweep(object):
    """Buffers of the wide blocked sweep for (device, n, d): Y = [X - c | S]
    and norms (kept current as rows move), the split engines' images of Y
    (the Gram's per-row-scaled FmtH2 row image, phi_mm's FmtX3 image; the
    rows a block moves are re-split after its walk), the block's D panel
    row, the split-K partials of its wide pass and their sums."""

    def __init__(self, dev, n, d, gemm, kind):
        lib = N.load()
        f32 = dict(dtype=torch.float32, device=dev)
        self.n, self.d = n, d
        self.n_pad = lib.dsvgd_pad128(n)
        self.dp = lib.dsvgd_dp(d)
        self.ldy = lib.dsvgd_ldy(self.dp)
        # rows per block: the walk keeps x' and w (and, refreshed, s') in LDS
        self.B = int(lib.dsvgd_gsw_block_rows(d, kind))
        # blocks per wide pass (GSW_GROUP): the group's rows in one pass, the
        # earlier blocks' moved rows added after each walk (dsvgd_gsw_group_corr)
        # (None: about 128 rows per pass -- config D 2 x 64 rows, config E
        # 8 x 16: 160 / 487 ms against 162.9 / 811 at 4 x 64 / 2 x 16,
        # profiles/r13ak, r13ap, r13aq)
        grp = GSW_GROUP if GSW_GROUP else max(1, 128 // self.B)
        self.G = max(1, min(grp, 256 // self.B))
        self.GB = self.G * self.B
        gpad = -(-self.GB // 128) * 128
        self.Y = torch.zeros(self.n_pad + 128, self.ldy, **f32)
        self.norms = torch.zeros(self.n_pad + 128, **f32)
        self.mean = torch.empty(d, **f32)
        self.D = torch.empty(gpad * self.n_pad, **f32)
        split = gemm == "split"
        # phi_mm on FmtX3 (no scales: moved rows cannot leave a scale's window)
        self.phi_x3 = split and self.n_pad * self.ldy * 6 < (1 << 31)
        if self.phi_x3:
            self.m16 = self.ldy % 256 == 0
            self.Yx3 = torch.empty(lib.dsvgd_ysplit_bytes(self.n_pad, self.ldy) // 2,
                                   dtype=torch.int16, device=dev)
        # the Gram on FmtH2 row images with per-row scales (the one-wave Gram
        # needs roundup(d, 32) % 256 == 0; otherwise the exact f32 engine)
        self.gram_rows = self.n_pad + 256
        self.gram_h2 = (split and self.dp % 256 == 0
                        and self.dp * self.gram_rows * 4 < (1 << 31))
        if self.gram_h2:
            self.rsc = torch.ones(self.n_pad + 128, **f32)
            self.Yg = torch.empty(lib.dsvgd_h2_image_bytes(self.gram_rows, self.dp) // 2,
                                  dtype=torch.int16, device=dev)
        # split-K slices of the group's wide pass: ldy / 512 column blocks x
        # 128-row tiles per slice, so ~256 blocks fill the CUs
        cb = max(1, self.ldy // 512) * (gpad // 128)
        z = max(1, 256 // cb) if not GSW_SPLITS else GSW_SPLITS
        while z > 1 and self.n_pad // z < 128:
            z //= 2
        self.splits = z
        self.KY = torch.empty(z * self.GB, self.ldy, **f32)
        self.rowsum = torch.empty(z * gpad, **f32)
        self.Q = torch.empty(self.GB, self.ldy, **f32)
        self.Qr = torch.empty(gpad, **f32)
        # the pipelined sweep (GSW_PIPELINE): group g + 1's sums beside group
        # g's, the norms snapshot its wide pass reads, its stream
        self.Q2 = torch.empty(self.GB, self.ldy, **f32)
        self.Qr2 = torch.empty(gpad, **f32)
        self.norms_s = torch.empty_like(self.norms)
        self.side = None

    def images(self, r0, nr, s):
        """(Re)split rows [r0, r0 + nr) of Y into the engines' images (the
        whole image, padding rows zeroed, when nr = n_pad)."""
        if self.gram_h2:
            rb = 4 * r0
            N.call("dsvgd_h2_rowscale", N.ptr(self.Y) + rb * self.ldy, self.ldy, nr, self.dp, nr,
                   N.ptr(self.rsc) + rb, None, s)
            if nr == self.n_pad:
                N.call("dsvgd_h2_rowsplit_rows", N.ptr(self.Y), self.ldy, self.n_pad, self.dp,
                       self.gram_rows, self.dp, N.ptr(self.rsc), N.ptr(self.Yg), s)
            else:
                N.call("dsvgd_h2_rowsplit_rows_range", N.ptr(self.Y), self.ldy, self.n_pad,
                       self.dp, self.gram_rows, self.dp, N.ptr(self.rsc), N.ptr(self.Yg), r0, nr,
                       s)
        if self.phi_x3:
            k0, k1 = r0 // 16, -(-(r0 + nr) // 16)    # whole 16-row K-steps
            N.call("dsvgd_ysplit", N.ptr(self.Y) + 4 * 16 * k0 * self.ldy, self.ldy,
                   16 * (k1 - k0), N.ptr(self.Yx3) + 2 * 3 * 16 * k0 * self.ldy,
                   0 if self.m16 else 1, None, s)


_WIDE = {}
# the pipelined wide sweep (round 6): group g + 1's wide pass on a second
# stream while group g walks, group g's columns left out of it and added at
# their moved positions by dsvgd_gsw_group_corr before g + 1 walks
# (d <= GSW_PIPELINE_MAX_D: config D sweep 136.4 vs 155.3 ms; at config E,
# d = 1024, the extra whole-group corrections cost more than the overlap
# saves, 536 vs 488 ms -- profiles/r14h)
GSW_PIPELINE = True
GSW_PIPELINE_MAX_D = 256
# CUs the side stream's passes leave free (dsvgd_set_cu_reserve, and the
# phi_mm split-K slices cut by as many) so the walk -- one workgroup with
# most of a CU's LDS -- starts beside them instead of after them
GSW_SIDE_RESERVE = 8
GSW_PIPE_SPIN_NS = 0   # tests: hold the walk's stream this long after each pass is posted
# blocks per wide pass of the wide Gauss-Seidel sweep (1: block after block;
# config D sweep 278.7 / 253.0 / 256.2 ms at 1 / 2 / 4, profiles/r13u; None:
# as many blocks as make about 128 rows)
GSW_GROUP = None
# split-K slices of a group's wide pass (None: ~256 blocks; an A/B override)
GSW_SPLITS = None


def _blocked_sweep_wide(X, S, rows, h_state, step, kind, target, score_scale, phi_out, extra, s):
    """The reference's Gauss-Seidel sweep for 64 < d <= 1024, B rows at a
    time: the block's interactions with every row not moved before it in the
    block on the MFMA engines (the Gram, dsvgd_gs_mask, phi_mm over split-K
    slices, dsvgd_phi_partial_reduce), then one workgroup walks the B rows in
    order (dsvgd_gsw_block_sweep) and the moved rows are re-split into the
    engines' images -- the same terms as the per-row path, in blocked order."""
    n, d = X.shape
    key = (X.device, n, d, GSW_GEMM, kind != 0, GSW_GROUP, GSW_SPLITS)
    W = _WIDE.get(key)
    if W is None:
        _WIDE.clear()
        W = _WIDE[key] = _WideSweep(X.device, n, d, GSW_GEMM, kind)
    sk, mu, lam, xd, td = kind, None, None, None, None
    if sk == 1:
        mu, lam = target._params(X.device)
    elif sk == 3:    # the rank's data (16-byte rows) and labels
        xd, td = target._params_aligned(X.device)
    N.call("dsvgd_colcenter", N.ptr(X), N.ld(X), n, d, N.ptr(W.mean), s)
    N.call("dsvgd_pack", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), 1.0, N.ptr(W.mean), n, d,
           W.Y.shape[0], N.ptr(W.Y), W.ldy, N.ptr(W.norms), s)
    W.images(0, W.n_pad, s)
    B, GB = W.B, W.GB
    groups = [(g0, min(GB, rows.stop - g0)) for g0 in range(rows.start, rows.stop, GB)]
    if GSW_PIPELINE and d <= GSW_PIPELINE_MAX_D and len(groups) >= 2:
        _pipelined_sweep_wide(W, X, S, groups, n, d, h_state, step, sk, mu, lam, xd, td,
                              score_scale, phi_out, extra, rows.start, s)
        return
    for g0 in range(rows.start, rows.stop, GB):
        gn = min(GB, rows.stop - g0)
        # the group's wide pass: every row against every row not moved before
        # it, the group's own earlier pairs masked (the walks add the block's
        # own, dsvgd_gsw_group_corr the earlier blocks' at their moved rows)
        if W.gram_h2:
            N.call("dsvgd_sqdist_h2", N.ptr(W.Yg), N.ptr(W.norms), g0, gn, n, d, N.ptr(W.D),
                   W.n_pad, 0, None, None, 0, N.ptr(W.rsc), s)
        else:
            N.call("dsvgd_sqdist", N.ptr(W.Y), W.ldy, N.ptr(W.norms), g0, gn, n, d, N.ptr(W.D),
                   W.n_pad, 0, None, None, s)
        N.call("dsvgd_gs_mask", N.ptr(W.D), W.n_pad, g0, gn, s)
        if W.phi_x3:
            N.call("dsvgd_phi_mm_x3", N.ptr(W.D), W.n_pad, N.ptr(W.Yx3), W.ldy, g0, gn, n,
                   h_state.ptr, W.splits, N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), 0, int(W.m16),
                   None, s)
        else:
            N.call("dsvgd_phi_mm", N.ptr(W.D), W.n_pad, N.ptr(W.Y), W.ldy, g0, gn, n,
                   h_state.ptr, W.splits, N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), s)
        N.call("dsvgd_phi_partial_reduce", N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), W.splits, gn,
               2 * W.dp, N.ptr(W.Q), W.ldy, N.ptr(W.Qr), s)
        for b0 in range(g0, g0 + gn, B):
            nb = min(B, g0 + gn - b0)
            k0, q0 = b0 - rows.start, b0 - g0
            ex = N.ptr(extra[k0:k0 + nb]) if extra is not None else None
            po = N.ptr(phi_out[k0:k0 + nb]) if phi_out is not None else None
            N.call("dsvgd_gsw_block_sweep", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), N.ptr(W.Y),
                   W.ldy, N.ptr(W.norms), N.ptr(W.mean), n, d, b0, nb, h_state.ptr, float(step),
                   N.ptr(W.Q) + 4 * q0 * W.ldy, W.ldy, N.ptr(W.Qr) + 4 * q0, ex, d, po,
                   N.ld(phi_out) if phi_out is not None else d, sk, N.ptr(mu), N.ptr(lam),
                   float(score_scale), N.ptr(xd), N.ld(xd) if xd is not None else d, N.ptr(td),
                   td.numel() if td is not None else 0, s)
            r1 = b0 + nb
            if r1 < g0 + gn:   # the group's later rows gain this block at its moved rows
                N.call("dsvgd_gsw_group_corr", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S),
                       N.ptr(W.mean), n, d, r1, g0 + gn - r1, b0, nb, h_state.ptr,
                       N.ptr(W.Q) + 4 * (r1 - g0) * W.ldy, W.ldy, N.ptr(W.Qr) + 4 * (r1 - g0), s)
        # the group's moved rows into the images once, after its last walk:
        # only the next groups' wide passes read them (the walks read Y, the
        # correction X and S)
        W.images(g0, gn, s)


def _gsw_pass(W, g0, gn, n, d, h_state, norms, Q, Qr, s, exclude=None, splits=None):
    """The wide pass of the group's rows [g0, g0 + gn) against every row not
    moved before them in the group (and, pipelined, not in the `exclude` =
    (p0, pn) group walking beside it): Q = [K Xc | K S], Qr = K 1."""
    z = splits or W.splits
    if W.gram_h2:
        N.call("dsvgd_sqdist_h2", N.ptr(W.Yg), N.ptr(norms), g0, gn, n, d, N.ptr(W.D),
               W.n_pad, 0, None, None, 0, N.ptr(W.rsc), s)
    else:
        N.call("dsvgd_sqdist", N.ptr(W.Y), W.ldy, N.ptr(norms), g0, gn, n, d, N.ptr(W.D),
               W.n_pad, 0, None, None, s)
    N.call("dsvgd_gs_mask", N.ptr(W.D), W.n_pad, g0, gn, s)
    if exclude is not None:
        N.call("dsvgd_gs_mask_cols", N.ptr(W.D), W.n_pad, gn, exclude[0], exclude[1], s)
    if W.phi_x3:
        N.call("dsvgd_phi_mm_x3", N.ptr(W.D), W.n_pad, N.ptr(W.Yx3), W.ldy, g0, gn, n,
               h_state.ptr, z, N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), 0, int(W.m16),
               None, s)
    else:
        N.call("dsvgd_phi_mm", N.ptr(W.D), W.n_pad, N.ptr(W.Y), W.ldy, g0, gn, n,
               h_state.ptr, z, N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), s)
    N.call("dsvgd_phi_partial_reduce", N.ptr(W.KY), W.ldy, N.ptr(W.rowsum), z, gn,
           2 * W.dp, N.ptr(Q), W.ldy, N.ptr(Qr), s)


def _pipelined_sweep_wide(W, X, S, groups, n, d, h_state, step, sk, mu, lam, xd, td,
                          score_scale, phi_out, extra, r_start, s):
    """The wide blocked sweep with group g + 1's wide pass on a second stream
    beside group g's walk.  What the two streams share, and why it is safe:

      * the side stream alone writes D, KY, rowsum (its passes in order) and
        the sums Qs[(g + 1) % 2]; the walk of g reads Qs[g % 2];
      * the pass of g + 1 reads the images (Yg, rsc, Yx3) and a SNAPSHOT of
        the norms (norms_s), both refreshed on the side stream after the walk
        of g - 1 (an event), behind the pass of g: the walk of g rewrites
        Y / norms / X rows of group g, which the pass of g + 1 masks;
      * the images of g are re-split on the side stream after the walk of g
        and after the pass of g + 1 (stream order), before the pass of g + 2;
        nothing on the walk's stream reads the images;
      * before g + 1 walks, its sums gain group g's rows at their moved
        positions (dsvgd_gsw_group_corr, block by block, on the walk's stream).

    So the walk's stream runs only the walks and the corrections.  The same
    terms as the block-after-block sweep, in another order
    (tests/test_gpu_configs.py: against the fp64 restatement, the overlap
    forced)."""
    dev = X.device
    main = torch.cuda.current_stream(dev)
    if W.side is None:
        W.side = torch.cuda.Stream(device=dev)
    side = W.side
    B = W.B
    Qs = ((W.Q, W.Qr), (W.Q2, W.Qr2))
    done = [None] * len(groups)

    lib = N.load()
    zs = max(1, W.splits - GSW_SIDE_RESERVE) if W.splits > 2 * GSW_SIDE_RESERVE else W.splits

    def post(k):
        g0, gn = groups[k]
        prev = lib.dsvgd_set_cu_reserve(GSW_SIDE_RESERVE)
        try:
            with torch.cuda.stream(side):
                _gsw_pass(W, g0, gn, n, d, h_state, W.norms_s, *Qs[k % 2], side.cuda_stream,
                          exclude=groups[k - 1] if k > 0 else None, splits=zs)
                done[k] = side.record_event()
        finally:
            lib.dsvgd_set_cu_reserve(prev)

    side.wait_stream(main)              # Y, its images, the norms of the sweep's start
    with torch.cuda.stream(side):
        W.norms_s.copy_(W.norms)
    post(0)
    for k, (g0, gn) in enumerate(groups):
        Q, Qr = Qs[k % 2]
        main.wait_event(done[k])
        if k > 0:   # the previous group's moved rows, left out of this pass
            p0, pn = groups[k - 1]
            # (one launch for up to 128 of them, in row order)
            step_rows = 128
            for b0 in range(p0, p0 + pn, step_rows):
                nb = min(step_rows, p0 + pn - b0)
                N.call("dsvgd_gsw_group_corr", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S),
                       N.ptr(W.mean), n, d, g0, gn, b0, nb, h_state.ptr, N.ptr(Q), W.ldy,
                       N.ptr(Qr), s)
        if k + 1 < len(groups):
            post(k + 1)
            if GSW_PIPE_SPIN_NS:
                N.call("dsvgd_debug_spin", int(GSW_PIPE_SPIN_NS), s)
        for b0 in range(g0, g0 + gn, B):
            nb = min(B, g0 + gn - b0)
            k0, q0 = b0 - r_start, b0 - g0
            ex = N.ptr(extra[k0:k0 + nb]) if extra is not None else None
            po = N.ptr(phi_out[k0:k0 + nb]) if phi_out is not None else None
            N.call("dsvgd_gsw_block_sweep", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), N.ptr(W.Y),
                   W.ldy, N.ptr(W.norms), N.ptr(W.mean), n, d, b0, nb, h_state.ptr, float(step),
                   N.ptr(Q) + 4 * q0 * W.ldy, W.ldy, N.ptr(Qr) + 4 * q0, ex, d, po,
                   N.ld(phi_out) if phi_out is not None else d, sk, N.ptr(mu), N.ptr(lam),
                   float(score_scale), N.ptr(xd), N.ld(xd) if xd is not None else d, N.ptr(td),
                   td.numel() if td is not None else 0, s)
            r1 = b0 + nb
            if r1 < g0 + gn:
                N.call("dsvgd_gsw_group_corr", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S),
                       N.ptr(W.mean), n, d, r1, g0 + gn - r1, b0, nb, h_state.ptr,
                       N.ptr(Q) + 4 * (r1 - g0) * W.ldy, W.ldy, N.ptr(Qr) + 4 * (r1 - g0), s)
        if k + 2 < len(groups):
            # for the passes of g + 2 on: this group's images and the norms,
            # on the side stream after this walk (and after the pass of g + 1)
            side.wait_event(main.record_event())
            with torch.cuda.stream(side):
                W.images(g0, gn, side.cuda_stream)
                W.norms_s.copy_(W.norms)
    main.wait_stream(side)


def _blocked_sweep(X, S, rows, h_state, step, kind, target, score_scale, phi_out, extra, s):
    n, d = X.shape
    lib = N.load()
    B = int(lib.dsvgd_gs_block_rows())
    nsplit = int(lib.dsvgd_gs_splits(n))
    key = (X.device, nsplit, d)
    part = _GS_PARTIALS.get(key)
    if part is None:
        part = _GS_PARTIALS[key] = torch.empty(nsplit * B * d, dtype=torch.float32,
                                               device=X.device)
    sk, mu, lam = kind, None, None
    if sk == 1:   # the Gaussian target's parameters on this device
        mu, lam = target._params(X.device)
    for b0 in range(rows.start, rows.stop, B):
        nb = min(B, rows.stop - b0)
        k0 = b0 - rows.start
        N.call("dsvgd_gs_block_part", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), n, d, b0, nb,
               h_state.ptr, N.ptr(part), nsplit, s)
        ex = N.ptr(extra[k0:k0 + nb]) if extra is not None else None
        po = N.ptr(phi_out[k0:k0 + nb]) if phi_out is not None else None
        N.call("dsvgd_gs_block_sweep", N.ptr(X), N.ld(X), N.ptr(S), N.ld(S), n, d, b0, nb,
               h_state.ptr, float(step), N.ptr(part), nsplit, ex, d, po,
               N.ld(phi_out) if phi_out is not None else d, sk, N.ptr(mu), N.ptr(lam),
               float(score_scale), s)
