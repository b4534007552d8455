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
           "data": {"n": 512 if order == "jacobi" else 64}}
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
    for rank, out in res[1:]:   # every rank holds the same gathered particle set
        np.testing.assert_array_equal(out[True][1], res[0][1][True][1])


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
