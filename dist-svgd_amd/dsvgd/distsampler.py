"""Drop-in `dsvgd.DistSampler` (reference: dsvgd/distsampler.py:8-205) on MI355X.

Constructor, `particles` property (owned row-block view; setter asserts the
shape, distsampler.py:53-62), `make_step(step_size, h=1.0) -> None` and the
three exchange modes keep the reference semantics:

  partitions     (exchange_particles=False): ring shift of the owned block to
                 rank+1, receive into rank-1's rows, which become the owned rows
                 from then on (distsampler.py:131-150); interactions and the
                 median are local to the block; score = N_global/N_local *
                 grad log p_local (:97-99).
  all_particles  all-gather of the owned blocks; owned rows interact with all n;
                 score = N_global/N_local * grad log p_local.
  all_scores     all-gather, then the local-data scores of ALL n particles are
                 all-reduced (SUM) and frozen for the step (:160-170); like the
                 reference the prior is summed S times.

Device model: one process per GPU; the process group (nccl = RCCL) must be
initialised before make_step when num_shards > 1.  A device `particles`
tensor is updated in place (the reference mutates the caller's tensor, a7);
a CPU tensor (or a device tensor that is not row-major fp32, e.g. the
reference's `torch.cat(...).t()` view) is staged through a contiguous device
copy and mirrored back after every make_step.

Extensions (keyword-only): order="sequential" (reference in-place
Gauss-Seidel over the owned rows) | "jacobi" (MFMA fast path); device; group.
include_wasserstein (the reference default) adds the W2/JKO term from the
second step on (distsampler.py:103-129, 190-198): the reference's LP is solved
exactly as an assignment on the GPU (dsvgd.w2), and h * grad is added to every
owned row's direction before the update.  previous particles = all n rows
after the step when particles are exchanged, else the owned block (:202-205).

Replicated data (all_particles, every rank holding the same data set): every
rank's scores of a particle are the same numbers, so each rank scores only
its owned block and the blocks are all-gathered (north_star's "all-gather of
particles and scores") instead of every rank scoring all
n particles (distsampler.py:94-99).  `replicated=None` (default) turns this
on only where it is provably the reference's result: N_local == N_global and
built-in targets whose data digests (`fingerprint()`) agree on every rank,
checked once at the first step; a plain `logp` callable (which may close over
rank-specific data, as logreg.py:68's `logp(rank, x)` can) keeps the
redundant per-rank scoring.  `replicated=True` forces it, False disables it.

Gathered data (all_scores with the built-in LogisticRegression target,
`gather_data=None` = auto): the reference sums every rank's local-data score
of ALL n particles with an all-reduce (distsampler.py:160-170), i.e. score_i
= grad of the likelihood over all ranks' data + S x the prior (each rank's
logp carries the prior once).  Here the ranks' data are all-gathered once (at
the first step) and each rank scores only its OWN block over all of them with
the prior weighted S (dsvgd_score_logreg_prior), and the score blocks are
all-gathered -- north_star's "RCCL all-gather of particles and scores": the
same scores to fp32 rounding, 1/S of the per-particle score work, an
all-gather instead of an all-reduce (half the bytes), and the own block's
scores need only the own rows, so they run while the particle all-gather is
in flight (Jacobi: the gather on the side stream).  On when every rank's
target is a LogisticRegression, m > LogisticRegression.SMALL_ROWS and the
gathered data fit GATHER_DATA_MAX_BYTES; gather_data=False keeps the
all-reduce, True requires the mode (ValueError where it cannot apply).

Lagged modes (keyword `lagged`; the reference's notes.md:108-114, which
describe them and time them at :134-135 but ship no code):

  lagged="local"      ("laggedlocal") every rank keeps a full local copy of
                      the n particles.  Blocks travel round-robin as in
                      partitions (the held block goes to rank+1, rank-1's
                      arrives), but a received block is written to its home
                      rows, so the copy holds "the most recent copy of x_i
                      received" and stale rows elsewhere.  The held block
                      interacts with all n rows of the copy; scores are the
                      local-data ones scaled by N_global/N_local; a median
                      bandwidth is the lower median of the held block's own
                      m x n distances (no collective).
  lagged="updateall"  ("laggedlocal-updateall") the same exchange, but every
                      rank moves all n rows of its copy each step (phi of the
                      whole copy), the received block having overwritten its
                      rows first.

Both require exchange_particles=False, exchange_scores=False (nothing but
the travelling block is communicated) and include_wasserstein=False.

Deviation: exchange_scores with num_shards == 1 uses the local scores (the
reference reads an uninitialised buffer there).
"""
import warnings

import torch

from . import _native as N
from . import exchange
from .engine import PhiEngine, SelectState, StepGraph, sequential_sweep, span
from .kernels import resolve_kernel
from .targets import BuiltinTarget, LogisticRegression, resolve_target
from .w2 import W2Term


class DistSampler(object):
    timer = None   # optional engine.StageTimer (bench instrumentation)
    keep_phi = False  # Jacobi: also write phi of the owned rows to the engine's `phi` (tests)
    graphs = True  # S = 1, no W2, built-in target: replay each step as a HIP graph
    W2_WARN_ENTRIES = 1 << 24  # R > 1 plans this large warn at construction
    GATHER_DATA_MAX_BYTES = 1 << 30  # gathered-data all_scores: all ranks' data, per rank

    def __init__(self, rank, num_shards, logp, kernel, particles,
                 N_local, N_global,
                 exchange_particles=True, exchange_scores=True, include_wasserstein=True,
                 *, order="sequential", device=None, group=None, replicated=None,
                 lagged=None, gather_data=None):
        """Initializes a distributed SVGD sampler (distsampler.py:9-51)."""
        assert not (exchange_scores and not exchange_particles), \
            "must exchange particles to also exchange scores"
        if order not in ("sequential", "jacobi"):
            raise ValueError("order must be 'sequential' or 'jacobi'")
        if lagged not in (None, "local", "updateall"):
            raise ValueError("lagged must be None, 'local' or 'updateall'")
        if lagged and (exchange_particles or exchange_scores or include_wasserstein):
            raise ValueError("lagged modes travel blocks round-robin: they need "
                             "exchange_particles=False, exchange_scores=False, "
                             "include_wasserstein=False")
        self._lagged = lagged
        self._rank = rank
        self._num_shards = num_shards
        self._logp = logp
        self._kernel = kernel
        self._N_local = N_local
        self._N_global = N_global
        self._d = particles.shape[1]
        self._exchange_particles = exchange_particles
        self._exchange_scores = exchange_scores
        self._include_wasserstein = include_wasserstein
        self._order = order
        self._group = group
        self._target = resolve_target(logp)
        # score all-gather: particles exchanged, scores not all-reduced, S > 1
        eligible = exchange_particles and not exchange_scores and num_shards > 1
        if not eligible or replicated is False:
            self._replicated = False
        elif replicated:
            self._replicated = True
        else:   # decided at the first step (needs the process group)
            self._replicated = None if (N_local == N_global and
                                        hasattr(self._target, "fingerprint")) else False
        self._rbf = resolve_kernel(kernel, self._d)
        # gathered-data all_scores: decided at the first step (needs the group)
        if gather_data not in (None, True, False):
            raise ValueError("gather_data must be None, True or False")
        self._gdata = False if (gather_data is False or not exchange_scores
                                or num_shards == 1) else gather_data
        if gather_data and not (exchange_scores and num_shards > 1):
            raise ValueError("gather_data=True needs exchange_scores=True and num_shards > 1")
        self._gtarget = None

        # NOTE: drops particles if not divisible by num_shards (as the reference)
        self._particles_per_shard = int(particles.shape[0] / self._num_shards)
        self._num_particles = self._particles_per_shard * self._num_shards
        self._particles = particles[:self._num_particles]
        row_major = (self._particles.dtype == torch.float32 and self._particles.dim() == 2
                     and self._particles.stride(1) == 1)
        if particles.is_cuda and row_major:
            self._device = N.require_gpu(particles.device)
            self._work = self._particles          # updated in place
        elif particles.is_cuda:                   # e.g. the reference's cat(...).t() view
            self._device = N.require_gpu(particles.device)
            self._work = self._particles.to(torch.float32).contiguous()
        else:
            self._device = N.require_gpu(device if device is not None else "cuda")
            self._work = torch.empty(self._particles.shape, dtype=torch.float32,
                                     device=self._device)
            self._work.copy_(self._particles)
        self._scores = None
        if exchange_scores:
            self._scores = torch.empty(self._work.shape, dtype=torch.float32, device=self._device)

        (start, end) = self._particle_idx_range(rank)
        self._held = rank        # lagged modes: index of the block this rank holds
        self._particle_start_idx = start
        self._particle_end_idx = end
        self._previous_particles = None
        self._engines = {}
        self._state = None
        self._w2 = None
        self._side = None        # score all-reduce stream (Jacobi, S > 1)
        self._sbuf = None
        self._graph = None
        self._graph_key = None
        self._group_checked = False
        self._warn_w2_cost()

    def _warn_w2_cost(self):
        """The W2 term is the reference default, but with particles exchanged
        (R = n / m = num_shards > 1) the first step's exact assignment is a
        cold auction (1.75 s at 8192 x 65536; later steps
        start warm from the previous plan, 55 ms): say so once, at construction,
        instead of letting the first make_step stall for seconds."""
        m = self._particles_per_shard
        n = self._num_particles if self._exchange_particles else m
        if self._include_wasserstein and n > m and m * n >= self.W2_WARN_ENTRIES:
            warnings.warn(
                "DistSampler: include_wasserstein=True with R = n/m = %d > 1 and an "
                "%d x %d plan: the exact W2 assignment of the first step takes seconds "
                "at this size (m=8192, n=65536 on one MI355X: ~1.8 s cold, then ~55 ms per "
                "step warm-started from the previous plan); "
                "pass include_wasserstein=False for throughput" % (n // m, m, n),
                RuntimeWarning, stacklevel=3)

    # ---------------------------------------------------- reference API --
    @property
    def particles(self):
        "Returns particles currently being updated on this sampler"
        return self._particles[self._particle_start_idx:self._particle_end_idx, :]

    @particles.setter
    def particles(self, value):
        "Sets value of particles currently being updated on this sampler"
        assert value.shape == self.particles.shape
        s, e = self._particle_start_idx, self._particle_end_idx
        self._particles[s:e, :] = value
        if self._work is not self._particles:
            self._work[s:e, :] = value.to(self._device)

    def _particle_idx_range(self, rank):
        assert rank >= 0 and rank < self._num_shards
        return (self._particles_per_shard * rank, self._particles_per_shard * (rank + 1))

    # -------------------------------------------------------- exchange --
    def _exchange_round_robin(self):
        "Exchanges single particle partitions round robin (distsampler.py:131-150)."
        s, e = self._particle_start_idx, self._particle_end_idx
        send = self._work[s:e].clone()
        src = (self._rank - 1 + self._num_shards) % self._num_shards
        start, end = self._particle_idx_range(src)
        recv = torch.empty_like(send)
        exchange.ring_shift(send, recv, self._rank, self._num_shards, self._group)
        self._work[start:end] = recv
        self._particle_start_idx = start
        self._particle_end_idx = end

    def _exchange_lagged(self):
        """laggedlocal exchange (notes.md:110-112): the held block goes to
        rank+1, rank-1's held block arrives and is written to ITS home rows of
        the local copy, and is the block held (and moved) from now on."""
        S = self._num_shards
        s, e = self._particle_start_idx, self._particle_end_idx
        send = self._work[s:e].clone()
        self._held = (self._held - 1 + S) % S
        start, end = self._particle_idx_range(self._held)
        recv = torch.empty_like(send)
        exchange.ring_shift(send, recv, self._rank, S, self._group)
        self._work[start:end] = recv
        self._particle_start_idx = start
        self._particle_end_idx = end

    def _exchange_all_particles(self):
        "Gathers all particles to all shards (distsampler.py:152-158)."
        s, e = self._particle_start_idx, self._particle_end_idx
        if exchange.all_gather_in_place(self._work, s, e, self._group):
            return
        out = torch.empty_like(self._work)
        exchange.all_gather_blocks(self._work[s:e], out, self._group)
        self._work.copy_(out)

    def _local_scores(self, X, out, scale=1.0):
        self._target.score(X, out, scale)

    def _exchange_all_scores(self):
        "Sum of every shard's local-data scores of all particles (distsampler.py:160-170)."
        self._local_scores(self._work, self._scores)
        exchange.all_reduce_sum(self._scores, self._group)

    def _gather_scores(self, Si):
        """Owned blocks of Si -> every rank (replicated data; like the particle
        all-gather, in place on RCCL)."""
        s, e = self._particle_start_idx, self._particle_end_idx
        if exchange.all_gather_in_place(Si, s, e, self._group):
            return
        out = torch.empty_like(Si)
        exchange.all_gather_blocks(Si[s:e], out, self._group)
        Si.copy_(out)

    def _score_buffer(self, shape):
        if self._sbuf is None or tuple(self._sbuf.shape) != tuple(shape):
            self._sbuf = torch.empty(shape, dtype=torch.float32, device=self._device)
        return self._sbuf

    def _wasserstein_grad(self, particles, previous_particles, h):
        """h * W2 gradient (distsampler.py:103-129 times h, :198) of the owned
        rows against the previous particles, on the GPU (dsvgd.w2)."""
        key = (particles.shape[0], previous_particles.shape[0], self._d)
        if self._w2 is None or (self._w2.m, self._w2.n, self._w2.d) != key:
            self._w2 = W2Term(*key, device=self._device)
        return self._w2.grad(particles, previous_particles, h)

    def _check_group(self):
        """The shard rank / count are ranks of `group` (all_gather order and
        the ring's peers): refuse a mismatch before any collective."""
        import torch.distributed as dist
        size, rank = dist.get_world_size(self._group), dist.get_rank(self._group)
        if size != self._num_shards or rank != self._rank:
            raise ValueError("DistSampler(rank=%d, num_shards=%d) but this process is rank %d "
                             "of a %d-rank group: pass the group rank and size"
                             % (self._rank, self._num_shards, rank, size))
        self._group_checked = True

    def _resolve_replicated(self):
        """replicated=None: on iff every rank's target has the same data
        digest (one all_gather_object of a short string, first step only)."""
        import torch.distributed as dist
        fps = [None] * self._num_shards
        with torch.cuda.device(self._device):     # nccl stages the objects on the current device
            dist.all_gather_object(fps, self._target.fingerprint(), group=self._group)
        self._replicated = all(f == fps[0] for f in fps)

    def _resolve_gather_data(self):
        """gather_data=None/True, first step: every rank's (x, t) gathered
        once when every rank's target is a LogisticRegression (one
        all_gather_object; all ranks decide alike from the same gathered
        list); the gathered target scores the own block, prior weighted S."""
        import torch.distributed as dist
        m = self._particles_per_shard
        tg = self._target
        ok = (type(tg) is LogisticRegression and m > LogisticRegression.SMALL_ROWS
              and not self._lagged and self._exchange_particles)
        mine = (bool(ok), tg.x.cpu() if ok else None, tg.t.cpu() if ok else None,
                tg.gemm if ok else None)
        parts = [None] * self._num_shards
        with torch.cuda.device(self._device):     # nccl stages the objects on the current device
            dist.all_gather_object(parts, mine, group=self._group)
        every = all(q[0] for q in parts) and len({q[3] for q in parts}) == 1
        if every:
            x = torch.cat([q[1] for q in parts])
            t = torch.cat([q[2] for q in parts])
            every = (x.numel() + t.numel()) * 4 <= self.GATHER_DATA_MAX_BYTES
        if not every:
            if self._gdata:
                raise ValueError("gather_data=True: every rank needs a LogisticRegression "
                                 "target (same engine), more than %d particles per rank and "
                                 "at most GATHER_DATA_MAX_BYTES of data in all"
                                 % LogisticRegression.SMALL_ROWS)
            self._gdata = False
            return
        self._gtarget = LogisticRegression(x, t, gemm=parts[0][3])
        self._gdata = True

    def _gathered_scores(self, X, Si, jacobi):
        """Gathered-data all_scores: the own block's scores over every
        rank's data (prior x S) while the particle all-gather runs (Jacobi:
        on the side stream), then the score blocks all-gathered (Jacobi: on
        the side stream, joined before pack_scores)."""
        S = self._num_shards
        s, e = self._particle_start_idx, self._particle_end_idx
        main = torch.cuda.current_stream(self._device)
        side = main
        if jacobi:
            if self._side is None:
                self._side = torch.cuda.Stream(device=self._device)
            side = self._side
            side.wait_stream(main)             # the own rows' last update
        with torch.cuda.stream(side):
            with span(self.timer, "allgather_x"):
                self._exchange_all_particles()
        with span(self.timer, "scores"):   # own rows only: beside the gather
            self._gtarget.score(X[s:e], Si[s:e], 1.0, prior_weight=float(S))
        if side is not main:
            main.wait_stream(side)             # the gathered particles
            side.wait_stream(main)             # the own scores
        with torch.cuda.stream(side):
            with span(self.timer, "allgather_scores"):
                self._gather_scores(Si)
        return side

    # ------------------------------------------------------------ step --
    pair_split = True   # Jacobi with identical scores on every rank: the block-pair layout

    def _use_pair_split(self, n_int, m):
        """The pair-split layout (dsvgd.pairsplit) applies when
        every rank moves its own block with the same scores of all n
        particles (all_scores, or replicated data) in the Jacobi order."""
        S = self._num_shards
        return (self.pair_split and S > 1 and self._order == "jacobi" and self._exchange_particles
                and (self._exchange_scores or self._replicated) and not self._lagged
                and n_int == S * m and PhiEngine.pair_split_ok(n_int, self._d, S,
                                                               median=self._rbf.median))

    _routes_ok = None    # the pair split's point-to-point routes, checked once
    _probe_corrupt = False   # tests: this rank's probe sees a wrong payload

    def _pair_split_routes(self, m):
        """The pair split exchanges transposed partials point to point; before
        its first step, every rank checks the plan's routes on the live
        backend with a tagged probe through the same post / join path
        (exchange.probe_p2p, ADVICE r4: that path had never run on a
        multi-rank RCCL group).  A failed probe keeps the row-block layout on
        every rank (the verdict is shared), with a warning."""
        if self._routes_ok is None:
            from .pairsplit import PairSplitPlan
            P = PairSplitPlan(self._rank, self._num_shards, m)
            self._routes_ok = exchange.probe_p2p([q["dest"] for q in P.sends],
                                                 [q["src"] for q in P.recvs], self._rank,
                                                 self._device, self._group,
                                                 _corrupt=self._probe_corrupt)
            if not self._routes_ok:
                warnings.warn("DistSampler: the pair-split layout's point-to-point probe "
                              "failed on this process group; using the row-block layout",
                              RuntimeWarning, stacklevel=4)
        return self._routes_ok

    # the pair split's first step, checked against the row-block layout:
    # max |phi_pair - phi_rows| / max |phi_rows| over every rank's owned rows
    # (None until that step ran; inf when the routes or the check failed)
    pair_split_check = None
    PAIR_SPLIT_CHECK_TOL = 1e-5    # north_star's per-step phi tolerance
    _check_corrupt = False         # tests: spoil this rank's pair-split phi before the check

    def _check_pair_split(self, eng, run, X_own, step):
        """the pair split's first step is checked against the
        row-block layout on the live backend.  The row-block engine computes
        phi of the owned rows without moving them, then the pair split runs
        its real step (partials posted point to point, kernels in flight,
        joined, finished with the update); the two phis are compared on every
        rank and the verdict (MAX of the errors) is shared.  Above the
        tolerance -- a mis-routed or stale partial, on any rank -- the owned
        rows are reset and moved by the row-block phi, and every rank keeps
        the row-block layout from then on, with a warning."""
        rows_eng = PhiEngine(eng.n, self._d, m=eng.m, row0=eng.row0, device=self._device)
        rows_eng.timer = self.timer
        rows_eng.sample_share = eng.sample_share
        run(rows_eng, 0.0, True, move=False)   # the row-block phi; particles unmoved
        X0 = X_own.clone()
        run(eng, step, True)              # the pair split's step
        ref = rows_eng.phi
        if self._check_corrupt:            # tests: a partial gone wrong on this rank
            eng.phi[0, 0] += 1e3 * float(ref.abs().max())
        err = ((eng.phi - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).double()
        err = float(exchange.all_reduce_max(err.reshape(1), self._group)[0])
        self.pair_split_check = err
        if not err <= self.PAIR_SPLIT_CHECK_TOL:     # (a NaN fails too)
            X_own.copy_(X0)
            X_own.add_(ref, alpha=step)
            self._routes_ok = False
            self._engines = {(eng.n, eng.m, False, False): rows_eng}
            warnings.warn("DistSampler: the pair-split layout's first step differs from the "
                          "row-block layout's by %.3g of max|phi| on this process group; using "
                          "the row-block layout" % err, RuntimeWarning, stacklevel=4)

    def _engine(self, n_int, m, row0):
        """One engine per (interacting set, owned rows, median kind, layout);
        the owned rows' offset row0 is set per step (lagged modes rotate it)."""
        local = self._lagged == "local"
        ps = self._use_pair_split(n_int, m) and self._pair_split_routes(m)
        key = (n_int, m, local, ps)
        if key not in self._engines:
            self._engines.clear()      # the old D is freed before the new one is allocated
            self._engines[key] = PhiEngine(
                n_int, self._d, m=m, row0=row0, device=self._device, local_median=local,
                pair_split=(self._rank, self._num_shards) if ps else None)
        eng = self._engines[key]
        eng.set_row0(row0)
        eng.timer = self.timer
        if self._exchange_particles and self._num_shards > 1 and not self._lagged:
            # every rank packs the same particles: 1/S of the bracket sample each
            eng.sample_share = (self._rank, self._num_shards, self._gather_sample)
        return eng

    def _gather_sample(self, sample, start, end):
        if exchange.all_gather_in_place(sample, start, end, self._group):
            return
        out = torch.empty_like(sample)
        exchange.all_gather_blocks(sample[start:end], out, self._group)
        sample.copy_(out)

    def _compute(self, step_size, h):
        """Scores, bandwidth, W2 term and the particle update of one step
        (distsampler.py:190-200), after the exchange."""
        S = self._num_shards
        jacobi = self._order == "jacobi"
        s, e = self._particle_start_idx, self._particle_end_idx
        X = self._work
        if self._exchange_particles or self._lagged:
            Xi, lo = X, 0
        else:
            Xi, lo = X[s:e], s
        n_int = Xi.shape[0]
        # the rows this step moves: the owned / held block, or (updateall) all
        us, ue = (0, n_int) if self._lagged == "updateall" else (s, e)
        scale = 1.0 if self._exchange_scores else self._N_global / self._N_local
        Si = self._scores if self._exchange_scores else self._score_buffer(Xi.shape)
        median = self._rbf.median
        share = self._exchange_particles and S > 1
        hook = (lambda t: exchange.all_reduce_sum(t, self._group)) if share else None

        # scores: all n particles' local-data scores, all-reduced over the
        # shards (all_scores, distsampler.py:160-170), else the interacting
        # set's scaled local scores (:94-99).  Jacobi: the all-reduce runs on a
        # side stream, concurrent with the distance / median stage (which
        # needs X only).  The score kernels themselves stay on the main
        # stream: run beside the distance kernel they only time-slice the CUs
        # (measured: no gain), both being MFMA-bound.
        main = torch.cuda.current_stream(self._device)
        side = main
        if self._gdata:
            side = self._gathered_scores(X, Si, jacobi)
        else:
            with span(self.timer, "scores"):
                if self._exchange_scores:
                    self._local_scores(X, Si)
                elif self._replicated:                 # owned block only, gathered below
                    self._local_scores(X[s:e], Si[s:e], scale)
                else:
                    self._local_scores(Xi, Si, scale)
        if (self._exchange_scores or self._replicated) and S > 1 and not self._gdata:
            if jacobi:
                if self._side is None:
                    self._side = torch.cuda.Stream(device=self._device)
                side = self._side
                side.wait_stream(main)
            with torch.cuda.stream(side):
                if self._exchange_scores:
                    with span(self.timer, "allreduce_scores"):
                        exchange.all_reduce_sum(Si, self._group)
                else:
                    with span(self.timer, "allgather_scores"):
                        self._gather_scores(Si)

        w2g = None
        if self._include_wasserstein and self._previous_particles is not None:
            with span(self.timer, "w2"):
                w2g = self._wasserstein_grad(X[s:e], self._previous_particles, h)

        if jacobi:
            eng = self._engine(n_int, ue - us, us - lo)

            def run(e, step, write_phi, move=True):
                e.pack(Xi)                         # X half only: the scores are in flight
                e.distances(median=median)
                if median:
                    e.median_bandwidth(hook)
                else:
                    e.fixed_bandwidth(self._rbf.h)
                if side is not main:
                    main.wait_stream(side)
                e.pack_scores(Si)                  # Si already carries the score scale
                p2p = None
                if e.plan is not None:
                    p2p = lambda sends, recvs: exchange.exchange_p2p_async(sends, recvs,
                                                                           self._group)
                e.direction(X[us:ue] if move else None, step, write_phi=write_phi, extra=w2g,
                            p2p=p2p)

            if eng.plan is not None and self.pair_split_check is None:
                self._check_pair_split(eng, run, X[us:ue], step_size)
            else:
                run(eng, step_size, self.keep_phi)
        else:
            if median:
                eng = self._engine(n_int, ue - us, us - lo)
                eng.pack(Xi)
                eng.distances(median=True)
                eng.median_bandwidth(hook)
                state = eng.state
            else:
                if self._state is None:
                    self._state = SelectState(self._device)
                state = self._state
                N.call("dsvgd_set_bandwidth", state.ptr, float(self._rbf.h),
                       N.stream(self._device))
            tgt = None if self._exchange_scores else self._target
            sequential_sweep(Xi, Si, range(us - lo, ue - lo), state, step_size, target=tgt,
                             score_scale=scale, extra=w2g)


    def make_step(self, step_size, h=1.0):
        """Performs one step of SVGD (distsampler.py:172-205).

        Params:
            step_size - step size
            h - discretization size for the JKO (W2) term
        """
        S = self._num_shards
        if S > 1 and not self._group_checked:
            self._check_group()
        if self._replicated is None:
            self._resolve_replicated()
        if self._gdata is None or (self._gdata and self._gtarget is None):
            self._resolve_gather_data()
        if S > 1:
            if self._gdata:
                pass                       # in _compute, beside the own block's scores
            elif self._exchange_particles:
                with span(self.timer, "allgather_x"):
                    self._exchange_all_particles()
            elif self._lagged:
                with span(self.timer, "ring_shift"):
                    self._exchange_lagged()
            else:
                with span(self.timer, "ring_shift"):
                    self._exchange_round_robin()

        # S = 1 without the W2 term is pure kernel launches: one HIP graph
        # per step size, replayed (dsvgd.engine.StepGraph)
        if (S == 1 and self.graphs and not self._include_wasserstein and self.timer is None
                and isinstance(self._target, BuiltinTarget)):
            key = float(step_size)
            if self._graph is None or self._graph_key != key:
                self._graph = StepGraph(lambda: self._compute(step_size, h), self._device)
                self._graph_key = key
            self._graph()
        else:
            self._compute(step_size, h)

        s, e = self._particle_start_idx, self._particle_end_idx
        X = self._work
        if self._include_wasserstein:
            src = X if self._exchange_particles else X[s:e]
            self._previous_particles = src.clone()
        if self._work is not self._particles:
            self._particles.copy_(self._work)
