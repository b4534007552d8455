"""DistSampler paths beyond the reference's three golden modes, with S ranks
sharing cuda:0 over gloo (kernels on the GPU, exchange through host copies):

  * replicated data (all_particles with N_local == N_global): each rank
    scores its owned block and the score blocks are all-gathered (north_star
    "all-gather of particles and scores") -- identical
    to every rank scoring all n particles (reference distsampler.py:94-99),
    and to the oracle;
  * the `particles` setter (distsampler.py:58-62) on a device tensor and on
    the CPU-mirrored path.
"""
import numpy as np
import pytest
import torch

from conftest import record_parity
from oracle import svgd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TRAJ_TOL = 1e-4


def dsvgd():
    import dsvgd as m
    return m


def _data(seed=3, N=300, p=15, n=512):
    rs = np.random.RandomState(seed)
    x = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    init = (0.5 * rs.randn(n, p + 1)).astype(np.float32)
    return x, t, init


def _worker(rank, S, port, cfg, q):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    x, t, init = _data(**cfg.get("data", {}))
    out = {}
    for replicated in cfg["variants"]:
        tgt = m.targets.LogisticRegression(x, t)           # every rank: the whole data set
        parts = torch.tensor(init, device=DEV)
        ds = m.DistSampler(rank, S, tgt, m.RBF(cfg.get("h", 1.0)), parts, x.shape[0], x.shape[0],
                           exchange_particles=True, exchange_scores=False,
                           include_wasserstein=False, order=cfg["order"], replicated=replicated)
        assert ds._replicated == bool(replicated)
        traj = []
        for _ in range(cfg["steps"]):
            ds.make_step(cfg["eps"])
            traj.append(ds.particles.cpu().numpy())
        out[replicated] = (traj, ds._work.cpu().numpy())
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _run(S, port, cfg):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, S, port, cfg, q)) for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("S,order", [(2, "jacobi"), (4, "jacobi"), (2, "sequential")])
def test_replicated_scores_allgather(S, order):
    """Owned-block scores + all-gather == redundant all-n scoring, bit for bit,
    and == the oracle's DistSampler (all_particles, replicated data)."""
    steps, eps = 3, 0.05
    cfg = {"variants": [True, False], "order": order, "steps": steps, "eps": eps,
           "data": {"n": 512 if order == "jacobi" else 128}}   # > 32 owned rows: GEMM score path
    res = _run(S, 29900 + 10 * S + (order == "sequential"), cfg)
    x, t, init = _data(**cfg["data"])
    fn = lambda X: O.score_logreg(X, x, t)  # noqa: E731
    D = O.DistOracle([init] * S, [fn] * S, x.shape[0], x.shape[0], True, False,
                     sequential=order == "sequential", replicated=True)
    for step in range(steps):
        D.step(eps)
        for rank, out in res:
            gathered, redundant = out[True][0][step], out[False][0][step]
            np.testing.assert_array_equal(gathered, redundant)
            err = float(np.abs(gathered - D.own(rank)).max())
            record_parity(err)
            assert err < TRAJ_TOL, err


def _auto_worker(rank, S, port, q):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    x, t, init = _data(n=256)
    xr, tr, _ = _data(seed=40 + rank, n=256)          # rank-specific data, same N
    out = {}
    for case, tgt in (("same", m.targets.LogisticRegression(x, t)),
                      ("differ", m.targets.LogisticRegression(xr, tr))):
        ds = m.DistSampler(rank, S, tgt, m.RBF(1.0), torch.tensor(init, device=DEV), x.shape[0],
                           x.shape[0], exchange_particles=True, exchange_scores=False,
                           include_wasserstein=False, order="jacobi")
        assert ds._replicated is None            # decided at the first step
        traj = []
        for _ in range(2):
            ds.make_step(0.05)
            traj.append(ds.particles.cpu().numpy())
        out[case] = (ds._replicated, traj)
    lp = m.targets.LogisticRegression(xr, tr).logp   # a plain callable: never assumed replicated
    ds = m.DistSampler(rank, S, lp, m.RBF(1.0), torch.tensor(init, device=DEV), x.shape[0],
                       x.shape[0], exchange_particles=True, exchange_scores=False,
                       include_wasserstein=False, order="jacobi")
    out["callable"] = ds._replicated
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_default_needs_identical_data():
    """replicated=None (default) all-gathers owned-block scores
    only when every rank's built-in target digests the same data; ranks with
    rank-specific data of the same size (N_local == N_global) keep scoring
    every particle with their own logp, as the reference does -- both
    against the oracle; a plain callable is never assumed replicated."""
    S = 2
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_auto_worker, args=(r, S, 29940, q)) for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    x, t, init = _data(n=256)
    same = lambda X: O.score_logreg(X, x, t)  # noqa: E731
    own = [(lambda X, r=r: O.score_logreg(X, *_data(seed=40 + r, n=256)[:2])) for r in range(S)]
    for case, fns, rep in (("same", [same] * S, True), ("differ", own, False)):
        D = O.DistOracle([init] * S, fns, x.shape[0], x.shape[0], True, False, sequential=False,
                         replicated=rep)
        for step in range(2):
            D.step(0.05)
            for rank, out in res:
                flag, traj = out[case]
                assert flag is rep, (case, flag)
                err = float(np.abs(traj[step] - D.own(rank)).max())
                record_parity(err)
                assert err < TRAJ_TOL, (case, step, rank, err)
    for rank, out in res:
        assert out["callable"] is False


def test_logreg_workspaces_bounded():
    """scoring many particle counts keeps at most MAX_WORKSPACES
    unpinned workspaces (least recently used evicted) and the scores stay
    right after an eviction."""
    m = dsvgd()
    x, t, _ = _data()
    tgt = m.targets.LogisticRegression(x, t)
    ref = {}
    for n2 in (40, 48, 64, 96, 128, 192, 40):
        X2 = torch.tensor(0.1 * np.random.RandomState(n2).randn(n2, x.shape[1] + 1),
                          dtype=torch.float32, device=DEV)
        S2 = torch.empty_like(X2)
        tgt.score(X2, S2)
        assert len(tgt._ws) <= tgt.MAX_WORKSPACES
        got = S2.cpu().numpy()
        want = O.score_logreg(X2.cpu().numpy().astype(np.float64), x, t)
        assert np.abs(got - want).max() <= 1e-5 * np.abs(want).max()
        if n2 in ref:
            np.testing.assert_array_equal(got, ref[n2])
        ref[n2] = got


@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_particles_setter(where):
    """distsampler.py:58-62: the setter asserts the shape and writes the owned
    rows -- of the caller's device tensor, or of the CPU tensor and its device
    mirror -- and the next step starts from them."""
    x, t, init = _data(n=64)
    parts = torch.tensor(init, device=DEV if where == "cuda" else "cpu")
    ds = dsvgd().DistSampler(0, 1, dsvgd().targets.LogisticRegression(x, t), dsvgd().RBF(1.0),
                             parts, x.shape[0], x.shape[0], exchange_particles=False,
                             exchange_scores=False, include_wasserstein=False, order="jacobi")
    new = torch.tensor(0.3 * np.random.RandomState(1).randn(64, init.shape[1]).astype(np.float32))
    with pytest.raises(AssertionError):
        ds.particles = new[:10]
    ds.particles = new.to(parts.device)
    np.testing.assert_array_equal(parts.cpu().numpy(), new.numpy())     # caller's tensor
    np.testing.assert_array_equal(ds._work.cpu().numpy(), new.numpy())  # device copy
    ds.make_step(1e-2, h=10.0)
    fn = lambda X: O.score_logreg(X, x, t)  # noqa: E731
    D = O.DistOracle([new.numpy()], [fn], x.shape[0], x.shape[0], False, False, sequential=False)
    D.step(1e-2)
    assert np.abs(ds.particles.cpu().numpy() - D.own(0)).max() < TRAJ_TOL


# ------------------------------------------------ laggedlocal (notes.md:108-114) --
def _lag_worker(rank, S, port, cfg, q):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    x, t, inits = _lag_data(S, cfg["n"])
    per = x.shape[0] // S
    tgt = m.targets.LogisticRegression(x[rank * per:(rank + 1) * per], t[rank * per:(rank + 1) * per])
    parts = torch.tensor(inits[rank], device=DEV)
    ds = m.DistSampler(rank, S, tgt, m.RBF(cfg["h"]), parts, per, per * S,
                       exchange_particles=False, exchange_scores=False, include_wasserstein=False,
                       order=cfg["order"], lagged=cfg["lagged"])
    out = []
    for _ in range(cfg["steps"]):
        ds.make_step(cfg["eps"])
        out.append((ds.particles.cpu().numpy(), ds._work.cpu().numpy(), ds._particle_start_idx))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _lag_data(S, n, N=240, p=7):
    rs = np.random.RandomState(11)
    x = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    inits = [(0.5 * np.random.RandomState(r).randn(n, p + 1)).astype(np.float32) for r in range(S)]
    return x, t, inits


LAG_CASES = [(2, "local", "jacobi", 1.0), (4, "local", "jacobi", "median"),
             (2, "local", "sequential", 1.0), (2, "updateall", "jacobi", "median"),
             (4, "updateall", "jacobi", 1.0), (2, "updateall", "sequential", 1.0)]


@pytest.mark.parametrize("S,lagged,order,h", LAG_CASES)
def test_lagged_modes_match_oracle(S, lagged, order, h):
    """laggedlocal / laggedlocal-updateall over S ranks sharing cuda:0 vs the
    oracle's restatement (per-rank local copies, round-robin blocks landing
    in their home rows, rank-local median): held block, its start index and
    every rank's whole local copy after each step."""
    steps, eps = 2 * S, 0.05
    n = 64 if order == "jacobi" else 16
    cfg = {"n": n, "lagged": lagged, "order": order, "h": h, "steps": steps, "eps": eps}
    res = _run_lag(S, 29950 + LAG_CASES.index((S, lagged, order, h)), cfg)
    x, t, inits = _lag_data(S, n)
    per = x.shape[0] // S
    fns = [(lambda X, r=r: O.score_logreg(X, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]))
           for r in range(S)]
    D = O.DistOracle(inits, fns, per, per * S, False, False, h=h,
                     sequential=order == "sequential", lagged=lagged)
    for step in range(steps):
        D.step(eps)
        for rank, out in res:
            own, full, start = out[step]
            assert start == D.start[rank] == ((rank - step - 1) % S) * (n // S)
            err = max(float(np.abs(own - D.own(rank)).max()), float(np.abs(full - D.X[rank]).max()))
            record_parity(err)
            assert err < TRAJ_TOL, (step, rank, err)


def _run_lag(S, port, cfg):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_lag_worker, args=(r, S, port, cfg, q)) for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_lagged_mode_arguments():
    x, t, inits = _lag_data(1, 8)
    tgt = dsvgd().targets.LogisticRegression(x, t)
    for kw in (dict(exchange_particles=True, exchange_scores=False),
               dict(exchange_particles=False, exchange_scores=False, include_wasserstein=True)):
        kw.setdefault("include_wasserstein", False)
        with pytest.raises(ValueError):
            dsvgd().DistSampler(0, 1, tgt, dsvgd().RBF(1.0), torch.tensor(inits[0], device=DEV),
                                240, 240, lagged="local", **kw)
    with pytest.raises(ValueError):
        dsvgd().DistSampler(0, 1, tgt, dsvgd().RBF(1.0), torch.tensor(inits[0], device=DEV), 240,
                            240, False, False, False, lagged="sometimes")


def test_w2_cost_warning_at_scale():
    """include_wasserstein=True (reference default) with R = n/m > 1 on a plan
    of >= 2^24 entries warns at construction; R = 1 and
    small plans stay silent."""
    import warnings
    m = dsvgd()
    x, t, _ = _data()
    tgt = m.targets.LogisticRegression(x, t)
    parts = torch.zeros(8192, 16, device=DEV)
    with pytest.warns(RuntimeWarning, match="include_wasserstein"):
        m.DistSampler(0, 4, tgt, m.RBF(1.0), parts, 300, 300, True, False, True)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        m.DistSampler(0, 4, tgt, m.RBF(1.0), parts, 300, 300, False, False, True)   # R = 1
        m.DistSampler(0, 4, tgt, m.RBF(1.0), parts[:512], 300, 300, True, False, True)
        m.DistSampler(0, 4, tgt, m.RBF(1.0), parts, 300, 300, True, False, False)


def test_engine_refuses_oversized_d():
    """D is materialised (m_pad x n_pad fp32): an engine whose D cannot fit
    raises MemoryError naming the sizes before allocating."""
    m = dsvgd()
    with pytest.raises(MemoryError, match="shard the rows"):
        m.engine.PhiEngine(1 << 20, 64)
    e = m.engine.PhiEngine(1 << 20, 64, m=1024, row0=0)      # 4 GiB row block fits
    assert e.D.numel() == 1024 * (1 << 20)


def test_graph_replay_keeps_score_workspace():
    """A captured step (S = 1, built-in target: DistSampler.graphs) holds the
    logreg workspace address; scoring the same target at four other particle
    counts between replays must not free or move it (workspaces
    are never evicted).  Trajectory == a sampler whose target scored nothing else."""
    m = dsvgd()
    x, t, init = _data(n=256)
    runs = []
    for extra in (False, True):
        tgt = m.targets.LogisticRegression(x, t)
        ds = m.DistSampler(0, 1, tgt, m.RBF("median"), torch.tensor(init, device=DEV),
                           x.shape[0], x.shape[0], exchange_particles=False,
                           exchange_scores=False, include_wasserstein=False, order="jacobi")
        traj = []
        for step in range(4):
            ds.make_step(1e-2)
            traj.append(ds.particles.cpu().numpy())
            if extra:
                for n2 in (48, 96, 192, 384):
                    X2 = torch.tensor(0.1 * np.random.RandomState(n2).randn(n2, init.shape[1]),
                                      dtype=torch.float32, device=DEV)
                    S2 = torch.empty_like(X2)
                    tgt.score(X2, S2)
        assert ds._graph is not None and ds._graph.graph is not None   # replays ran
        runs.append(np.stack(traj))
    np.testing.assert_array_equal(runs[0], runs[1])


def _nccl_worker(rank, S, port, mode, order, q):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=S, device_id=dev)
    x, t, init = _data(n=512)
    per = x.shape[0] // S
    tgt = m.targets.LogisticRegression(x[rank * per:(rank + 1) * per], t[rank * per:(rank + 1) * per])
    ep, es = {"partitions": (False, False), "all_particles": (True, False),
              "all_scores": (True, True)}[mode]
    ds = m.DistSampler(rank, S, tgt, m.RBF(1.0), torch.tensor(init, device=dev), per, x.shape[0],
                       exchange_particles=ep, exchange_scores=es, include_wasserstein=False,
                       order=order)
    traj = []
    for _ in range(3):
        ds.make_step(0.05)
        traj.append(ds.particles.cpu().numpy())
    q.put((rank, traj))
    dist.barrier()
    dist.destroy_process_group()


def _nccl_world1_worker(port, q):
    """Every device-collective branch of dsvgd.exchange on RCCL with one rank:
    the calls, aliasing, stream use and dtypes are the S > 1 ones; with one
    rank each collective's result is known exactly."""
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    from dsvgd import exchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert not exchange._is_gloo()
    out = {}
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(1024, 48, generator=g).to(dev)
    X0 = X.clone()
    # in-place all-gather: the rank's block aliases its slot of the output
    out["inplace_taken"] = exchange.all_gather_in_place(X, 0, X.shape[0])
    out["inplace_equal"] = bool(torch.equal(X, X0))
    # out-of-place all-gather into a separate buffer
    o = torch.full_like(X, float("nan"))
    exchange.all_gather_blocks(X[:256], o[:256])
    out["gather_equal"] = bool(torch.equal(o[:256], X0[:256]))
    # ring shift through batch_isend_irecv (rank 0 sends to and receives from itself)
    r = torch.full((256, 48), float("nan"), device=dev)
    exchange.ring_shift(X[256:512].contiguous(), r, 0, 1)
    out["ring_equal"] = bool(torch.equal(r, X0[256:512]))
    # the all_scores all-reduce on a side stream, joined back like DistSampler._compute
    side = torch.cuda.Stream(device=dev)
    S = X * 3.0
    S0 = S.clone()
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        exchange.all_reduce_sum(S)
    main.wait_stream(side)
    out["allreduce_equal"] = bool(torch.equal(S, S0))
    # the pair split's partial exchange (exchange_p2p_async, verdict r4 next
    # #2): several sends and receives posted on the process group's stream
    # right behind the kernels that write the send buffers, unrelated kernels
    # enqueued on the compute stream before the join, the received buffers
    # read on the compute stream after it; twice, reusing the buffers as a
    # DistSampler step does
    src = [torch.randn(rows, 96, generator=g).to(dev) for rows in (256, 128, 384, 64)]
    sends = [torch.empty_like(t) for t in src]
    recvs = [torch.full_like(t, float("nan")) for t in src]
    ok = []
    for it in range(2):
        for t, a in zip(sends, src):
            torch.mul(a, float(it + 2), out=t)       # written just before the post
        join = exchange.exchange_p2p_async([(t, 0) for t in sends], [(t, 0) for t in recvs])
        busy = torch.randn(2048, 2048, device=dev)
        for _ in range(4):
            busy = torch.mm(busy, busy) * 1e-3
        join()
        sums = torch.stack([(r - a * float(it + 2)).abs().sum() for r, a in zip(recvs, src)])
        ok.append(float(sums.sum().item()) == 0.0)
        for r in recvs:
            r.fill_(float("nan"))
    out["p2p_async_equal"] = all(ok)
    # the route probe DistSampler runs before its first pair-split step
    out["probe_ok"] = exchange.probe_p2p([0, 0], [0, 0], 0, dev)
    # the median's histogram all-reduce hook (int64 bins, bracket counts) on a
    # row-block engine: the same bandwidth as without the hook
    # (radix passes over D; the bracketed select, n * n >= 2^24; one rank
    # holds the whole matrix, so its order statistic exists without peers)
    out["median_h"] = []
    for n in (2048, 4096):
        Xm = (0.3 * torch.randn(n, 32, generator=g)).to(dev)
        hs = []
        for hook in (None, lambda t: exchange.all_reduce_sum(t)):
            eng = m.PhiEngine(n, 32, device=dev)
            eng.pack(Xm)
            eng.distances(median=True)
            eng.median_bandwidth(hook)
            torch.cuda.synchronize()
            hs.append(eng.state.read()[1])
        out["median_h"].append(hs)
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()
    q.put(out)


def test_rccl_world1_exchange_primitives():
    """One GPU: the RCCL branches of dsvgd.exchange (in-place
    all_gather_into_tensor, batch_isend_irecv ring shift, the side-stream
    all-reduce, the median hook's int64 all-reduces) run on hardware -- the
    S > 1 call sites (reference distsampler.py:136,143,156,170) with results
    known exactly at one rank."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(29650, q))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    assert p.exitcode == 0
    for k in ("inplace_taken", "inplace_equal", "gather_equal", "ring_equal", "allreduce_equal",
              "p2p_async_equal", "probe_ok"):
        assert out[k], k
    for a, b in out["median_h"]:
        assert a == b and np.isfinite(a) and a > 0, out["median_h"]


def _nccl_pair_split_worker(port, q):
    """Both ranks of an S = 2 pair-split plan as two engines in ONE process
    on a one-rank RCCL group: every message of the plan goes rank 0 -> rank 0
    through exchange_p2p_async (batch_isend_irecv on the process group's
    stream), matched in the plan's order, so the real direction() path runs
    on RCCL -- partials computed and posted, the own window's kernels
    enqueued between the post and the join, the received partials summed by
    phi_finish_parts after it."""
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import dsvgd as m
    from dsvgd import exchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    S, mm, d = 2, 2048, 256
    n = S * mm
    h = 2.0 * d * 0.01 / 8.0
    eps = 1e-3
    rs = np.random.RandomState(41)
    X0 = (0.1 * rs.randn(n, d)).astype(np.float32)
    S0 = rs.randn(n, d).astype(np.float32)
    X = torch.tensor(X0, device=dev)
    Sc = torch.tensor(S0, device=dev)
    engs = [m.PhiEngine(n, d, m=mm, row0=r * mm, device=dev, pair_split=(r, S)) for r in range(S)]
    own = [X[r * mm:(r + 1) * mm].clone() for r in range(S)]
    for e in engs:
        assert e.plan is not None
        for b in e.recvbuf:
            b.fill_(float("nan"))
        e.pack(X, Sc)
        e.distances(median=False)
        e.fixed_bandwidth(h)
    # rank 1's partials first (its exchange captured, not run) ...
    captured = {}

    def capture(sends, recvs):
        captured["sends"] = sends
        return lambda: None
    engs[1].direction(own[1].clone(), 0.0, write_phi=True, p2p=capture)
    # ... then rank 0's real step: its sends to rank 1 land in rank 1's
    # receive buffers, rank 1's sends to rank 0 in rank 0's, each pair of
    # (send, receive) posted in the plan's order on the one RCCL rank
    posted = {}

    def self_peered(sends, recvs):
        P0, P1 = engs[0].plan, engs[1].plan
        to0 = [t for t, dst in captured["sends"] if dst == 0]
        from0 = [b for b, q_ in zip(engs[1].recvbuf, P1.recvs) if q_["src"] == 0]
        out0 = [t for t, dst in sends if dst == 1]
        in0 = [t for t, src in recvs if src == 1]
        assert len(to0) == len(in0) and len(out0) == len(from0)
        sl = [(t, 0) for t in to0] + [(t, 0) for t in out0]
        rl = [(t, 0) for t in in0] + [(t, 0) for t in from0]
        assert all(a.numel() == b.numel() for (a, _), (b, _) in zip(sl, rl))
        posted["messages"] = len(sl)
        return exchange.exchange_p2p_async(sl, rl)
    engs[0].direction(own[0], eps, write_phi=True, p2p=self_peered)
    # rank 1 finishes with the partials rank 0 sent it (no exchange of its own)
    engs[1].direction(own[1], eps, write_phi=True, p2p=None)
    torch.cuda.synchronize()
    out = {"messages": posted.get("messages", 0),
           "phi": [e.phi.cpu().numpy() for e in engs], "X1": [o.cpu().numpy() for o in own],
           "h": [e.state.read()[1] for e in engs], "X0": X0, "S0": S0, "eps": eps}
    dist.barrier()
    dist.destroy_process_group()
    q.put(out)


def test_rccl_world1_pair_split_direction():
    """the pair split's real direction() path with
    exchange_p2p_async on RCCL (both ranks of an S = 2 plan in one process,
    every message self-peered on a one-rank group; the own window's kernels
    run between the post and the join): phi of both row blocks and their
    update against the fp64 oracle (1e-5 max-normalised)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_pair_split_worker, args=(29652, q))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    assert p.exitcode == 0
    assert out["messages"] == 2
    X0, S0, eps = out["X0"].astype(np.float64), out["S0"].astype(np.float64), out["eps"]
    h = out["h"][0]
    assert out["h"][1] == h
    mm = X0.shape[0] // 2
    for r in range(2):
        rows = np.arange(r * mm, (r + 1) * mm)
        ref = O.phi(X0, S0, h, rows=rows)
        e = np.abs(out["phi"][r] - ref).max() / np.abs(ref).max()
        assert e < 1e-5, (r, e)
        X1 = out["X1"][r].astype(np.float64)
        tol = eps * 1e-5 * np.abs(ref).max() + 2 * np.spacing(np.abs(X1).astype(np.float32)).max()
        assert np.abs(X1 - (X0[rows] + eps * ref)).max() <= tol


@pytest.mark.parametrize("S", [2, 4, 8])
@pytest.mark.parametrize("mode", ["partitions", "all_particles", "all_scores"])
@pytest.mark.parametrize("order", ["jacobi", "sequential"])
def test_rccl_ranks_match_oracle(S, mode, order):
    """The device collectives (in-place all_gather_into_tensor, batch_isend_irecv
    ring shift, the all_scores all-reduce on a side stream beside the
    histogram all-reduces) on S GPUs over RCCL, one process per GPU, against
    DistOracle -- every S the box has GPUs for."""
    if torch.cuda.device_count() < S:
        pytest.skip("RCCL at S=%d needs %d GPUs" % (S, S))
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = (29600 + 8 * [2, 4, 8].index(S) + 2 * ["partitions", "all_particles", "all_scores"].index(mode)
            + (order == "jacobi"))
    ps = [ctx.Process(target=_nccl_worker, args=(r, S, port, mode, order, q)) for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    x, t, init = _data(n=512)
    per = x.shape[0] // S
    fns = [lambda X, r=r: O.score_logreg(X, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per])
           for r in range(S)]
    ep, es = {"partitions": (False, False), "all_particles": (True, False),
              "all_scores": (True, True)}[mode]
    D = O.DistOracle([init] * S, fns, per, x.shape[0], ep, es, sequential=order == "sequential")
    for step in range(3):
        D.step(0.05)
        for rank, traj in res:
            err = float(np.abs(traj[step] - D.own(rank)).max())
            record_parity(err)
            assert err < TRAJ_TOL, (step, rank, err)


def test_target_fingerprint_of_device_tensors():
    """A target built from device tensors digests like one built from host
    arrays (DistSampler's replicated-data check calls fingerprint() at the
    first step)."""
    x, t, _ = _data()
    T = dsvgd().targets
    host = T.LogisticRegression(x, t).fingerprint()
    dev = T.LogisticRegression(torch.tensor(x, device=DEV), torch.tensor(t, device=DEV))
    assert dev.fingerprint() == host
    g = T.Gaussian(torch.zeros(3, device=DEV), torch.ones(3, device=DEV))
    assert g.fingerprint() == T.Gaussian(np.zeros(3), np.ones(3)).fingerprint()


@pytest.mark.parametrize("load", ["torch", "scores"])
def test_side_stream_work_beside_the_step(load):
    """DistSampler overlaps the score all-reduce (a side stream) with the
    distance / median stage (distsampler.py _compute, reference :160-170):
    the step's kernels must give the same bits with other work running on
    another stream.  One engine step (Gram + bracketed median + phi_mm) alone,
    then again while a side stream runs torch GEMMs / elementwise kernels or
    the logreg score kernels on other buffers -- phi and h bit-identical."""
    m = dsvgd()
    n, d = 16384, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    X = (0.1 * torch.randn(n, d, generator=g)).to(DEV)
    S = torch.randn(n, d, generator=g).to(DEV)
    eng = m.PhiEngine(n, d, device=DEV)
    side = torch.cuda.Stream(device=DEV)
    A = torch.randn(4096, 4096, device=DEV)
    if load == "scores":
        x, t, _ = _data(N=4096, p=d - 1, n=8)
        tgt = m.targets.LogisticRegression(x, t)
        Xs = (0.1 * torch.randn(n, d, generator=g)).to(DEV)
        Ss = torch.empty_like(Xs)

    def step():
        eng.pack(X, S)
        eng.distances(median=True)
        eng.median_bandwidth()
        eng.direction(write_phi=True)

    step()
    torch.cuda.synchronize()
    ref_phi, ref_h = eng.phi.clone(), eng.state.read()[1]
    for rep in range(3):
        side.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(side):
            for _ in range(6):
                if load == "torch":
                    B = A @ A
                    B.mul_(1e-3).add_(1.0)
                else:
                    tgt.score(Xs, Ss)
        step()
        torch.cuda.current_stream(DEV).wait_stream(side)
        torch.cuda.synchronize()
        assert eng.state.read()[1] == ref_h, rep
        assert torch.equal(eng.phi, ref_phi), (rep, float((eng.phi - ref_phi).abs().max()))
