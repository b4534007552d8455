"""The pair-split layout of DistSampler (dsvgd/pairsplit.py; the
reference semantics it shards: dsvgd/distsampler.py:84-101 over the particles
all-gathered at :152-158, with the scores all-reduced at :160-170 or
replicated).  S gloo ranks share cuda:0; each rank computes only its share of
the block pairs of the n x n matrix, sends the transposed partials of the
blocks it holds for other ranks and sums those it receives.

Checked against the fp64 oracle on every rank's sampled rows: the scores,
phi (1e-5 max-normalised, north_star) and the update, the median bandwidth
(every rank agrees; fp64 distances of all n^2 pairs bracket it), at S = 2,
3, 4 with a median and with a fixed bandwidth; plus a step whose FmtH2
range guard trips (one particle 2^20 away), which runs the FmtX3 phi_mm over
the whole row block after the Gram of the parts the rank does not hold.
"""
import math

import numpy as np
import pytest
import torch

from conftest import record_parity
from oracle import svgd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PHI_TOL = 1e-5


def _inputs(n, d, N, seed):
    rs = np.random.RandomState(seed)
    x = (rs.randn(N, d - 1) / np.sqrt(d - 1)).astype(np.float32)
    t = np.where(rs.randn(N) > 0, 1.0, -1.0).astype(np.float32)
    X0 = (0.1 * rs.randn(n, d)).astype(np.float32)
    return x, t, X0


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
    n, d, N, eps = cfg["n"], cfg["d"], cfg["N"], cfg["eps"]
    x, t, X0 = _inputs(n, d, N, cfg["seed"])
    if cfg.get("far"):
        X0[cfg["far"], 1:] += np.float32(2.0 ** 20 * 0.1)
    per = N // S
    if cfg["mode"] == "all_scores":
        tgt = m.targets.LogisticRegression(x[rank * per:(rank + 1) * per],
                                           t[rank * per:(rank + 1) * per])
        ds = m.DistSampler(rank, S, tgt, m.RBF(cfg["h"]), torch.tensor(X0, device=DEV), per,
                           per * S, exchange_particles=True, exchange_scores=True,
                           include_wasserstein=False, order="jacobi")
    else:   # replicated data: every rank holds all N rows, scores its block, all-gathers
        tgt = m.targets.LogisticRegression(x, t)
        ds = m.DistSampler(rank, S, tgt, m.RBF(cfg["h"]), torch.tensor(X0, device=DEV), N, N,
                           exchange_particles=True, exchange_scores=False,
                           include_wasserstein=False, order="jacobi")
    ds.keep_phi = True
    ds._probe_corrupt = cfg.get("probe_corrupt") == rank
    ds._check_corrupt = cfg.get("check_corrupt") == rank
    ds.make_step(eps)
    torch.cuda.synchronize()
    eng = next(iter(ds._engines.values()))
    rows = np.sort(np.random.RandomState(60 + rank).choice(n // S, cfg["nrows"], replace=False))
    if cfg.get("far") is not None and rank == cfg["far"] // (n // S):
        rows = np.unique(np.concatenate([rows, [cfg["far"] % (n // S)]]))
    ridx = torch.as_tensor(rows, device=DEV)
    s0 = ds._particle_start_idx
    Si = ds._scores if cfg["mode"] == "all_scores" else ds._sbuf
    out = {"rows": s0 + rows, "h": eng.state.read()[1], "median": eng.state.read()[0],
           "plan": eng.plan is not None, "guard": eng.range_guard(),
           "check": ds.pair_split_check, "engines": len(ds._engines),
           "scores": Si[torch.as_tensor(s0 + rows, device=DEV)].cpu().numpy(),
           "phi": eng.phi[ridx].cpu().numpy(), "X1": ds.particles[ridx].cpu().numpy()}
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
    res = sorted([q.get(timeout=600) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    return res


def _check(S, cfg, res):
    n, d, N, eps = cfg["n"], cfg["d"], cfg["N"], cfg["eps"]
    x, t, X0 = _inputs(n, d, N, cfg["seed"])
    if cfg.get("far"):
        X0[cfg["far"], 1:] += np.float32(2.0 ** 20 * 0.1)
    X0 = X0.astype(np.float64)
    if cfg["mode"] == "all_scores":
        per = N // S
        S_ref = sum(O.score_logreg(X0, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per])
                    for r in range(S))
    else:
        S_ref = O.score_logreg(X0, x, t)
    h, med = res[0][1]["h"], res[0][1]["median"]
    want = cfg.get("expect_plan", True)
    assert all(o["plan"] == want for _, o in res), "pair-split layout engaged: %s, expected %s" % (
        [o["plan"] for _, o in res], want)
    assert all(o["engines"] == 1 for _, o in res)
    checks = [o["check"] for _, o in res]
    if cfg.get("check_corrupt") is not None:      # the first step's check caught it everywhere
        assert all(c is not None and c > PHI_TOL for c in checks), checks
    elif want:                                    # the first step's check passed everywhere
        assert all(c is not None and c <= PHI_TOL for c in checks), checks
    else:                                         # declined or the probe failed: never checked
        assert all(c is None for c in checks), checks
    assert all(o["h"] == h for _, o in res)
    if cfg["h"] == "median":
        assert all(o["median"] == med for _, o in res)
        k = (n * n - 1) // 2
        D64 = O.sqdist(X0, X0, self_cols=np.arange(n))
        assert (D64 < med * (1 - 1e-5)).sum() <= k < (D64 <= med * (1 + 1e-5)).sum()
        assert h == pytest.approx(med / math.log(n), rel=1e-6)
    else:
        assert h == pytest.approx(cfg["h"], rel=1e-7)
    worst = 0.0
    for rank, o in res:
        rows = o["rows"]
        if cfg.get("far") is not None:
            assert o["guard"] is True
        else:
            assert o["guard"] is False
        e_s = float(np.abs(o["scores"] - S_ref[rows]).max() / np.abs(S_ref[rows]).max())
        ref = O.phi(X0, S_ref, h, rows=rows)
        if cfg.get("far") is not None:   # row-normalised: the outlier's own row is far larger
            num = np.sqrt(((o["phi"].astype(np.float64) - ref) ** 2).sum(1))
            e_p = float((num / np.sqrt((ref ** 2).sum(1))).max())
        else:
            e_p = float(np.abs(o["phi"] - ref).max() / np.abs(ref).max())
        worst = max(worst, e_s, e_p)
        assert e_s < PHI_TOL, (rank, e_s)
        assert e_p < PHI_TOL, (rank, e_p)
        X1 = o["X1"].astype(np.float64)
        tol = eps * PHI_TOL * np.abs(ref).max(1, keepdims=True) + \
            2 * np.spacing(np.abs(X1).astype(np.float32))
        assert (np.abs(X1 - (X0[rows] + eps * ref)) <= tol).all()
    record_parity(worst, S=S, mode=cfg["mode"], h=str(cfg["h"]))


@pytest.mark.parametrize("S,m", [(2, 4096), (3, 4096), (4, 2048)])
def test_pair_split_all_scores_median(S, m):
    """all_scores (the bench's mode) with the median bandwidth at S = 2, 3, 4."""
    cfg = dict(n=S * m, d=256, N=2048, eps=1e-3, seed=S, h="median", mode="all_scores",
               nrows=64)
    _check(S, cfg, _run(S, 29810 + S, cfg))


@pytest.mark.parametrize("S", [2, 4])
def test_pair_split_replicated_fixed_h(S):
    """Replicated data (all_particles, N_local == N_global: score blocks
    all-gathered), fixed bandwidth, d = 512."""
    cfg = dict(n=S * 2048, d=512, N=1024, eps=1e-3, seed=10 + S, h=2.0 * 512 * 0.01 / 8.0,
               mode="replicated", nrows=48)
    _check(S, cfg, _run(S, 29820 + S, cfg))


def test_pair_split_range_guard_fallback():
    """One particle 2^20 away: the FmtH2 range guard trips on every rank (the
    X half spans > 2^16), each rank computes the rest of its row block's D
    and phi_mm runs on the FmtX3 engine over the whole row block; phi rows
    within 1e-5 row-normalised, the outlier's row among them."""
    S, m = 2, 4096
    cfg = dict(n=S * m, d=256, N=2048, eps=1e-3, seed=7, h="median", mode="all_scores",
               nrows=48, far=5000)
    _check(S, cfg, _run(S, 29830, cfg))


def test_pair_split_declined_for_unaligned_half_block():
    """even S with m = 256 (mod 512) -- the antipodal
    half-block m/2 is not a 256-aligned Gram part -- must keep the row-block
    layout (the plan is declined up front) and still match the oracle."""
    S, m = 2, 2304
    cfg = dict(n=S * m, d=256, N=1024, eps=1e-3, seed=21, h=2.0 * 256 * 0.01 / 8.0,
               mode="all_scores", nrows=48, expect_plan=False)
    _check(S, cfg, _run(S, 29835, cfg))


def test_xcd_slice_maps_give_identical_bits():
    """The XCD slice maps (dsvgd_phi_set_xmap bits: 2 the window / row-half
    DS 0 launches, 4 the batched forward partials) only change which block
    runs which (row block, slice): one S = 8 rank's pair-split step at the
    headline size (m = 8192: the forward partials batched and K-split) gives
    the same bits -- its own rows' KY slices, row sums and every send
    buffer -- with every map on and off."""
    import dsvgd as m
    from dsvgd import _native as N
    n, d, S, r = 65536, 256, 8, 4
    mm = n // S
    rs = np.random.RandomState(7)
    X = torch.tensor((0.1 * rs.randn(n, d)).astype(np.float32), device=DEV)
    Sx = torch.tensor(rs.randn(n, d).astype(np.float32), device=DEV)
    lib = N.load()
    out = {}
    for mask in (7, 0):
        prev = lib.dsvgd_phi_set_xmap(mask)
        try:
            eng = m.PhiEngine(n, d, m=mm, row0=r * mm, device=DEV, pair_split=(r, S))
            assert eng.plan is not None and eng.fwd_batched and eng.fwd_z > 1
            for b in eng.recvbuf:
                b.zero_()
            eng.step(X, Sx, X_own=X[r * mm:(r + 1) * mm].clone(), h=2.0 * d, write_phi=True)
            torch.cuda.synchronize()
            out[mask] = ([eng.phi.clone()] + [b.clone() for b in eng.sendbuf])
            del eng
            torch.cuda.empty_cache()
        finally:
            lib.dsvgd_phi_set_xmap(prev)
    for a, b in zip(out[7], out[0]):
        assert torch.equal(a, b)


def test_pair_split_failed_route_probe_keeps_row_blocks():
    """one rank's route probe sees a wrong payload (the received
    buffer spoiled before the comparison): every rank keeps the row-block
    layout from the first step on, and the step still matches the oracle."""
    S, m = 2, 4096     # m * n >= 2^24: the bracketed median, so the layout applies
    cfg = dict(n=S * m, d=256, N=1024, eps=1e-3, seed=31, h="median", mode="all_scores",
               nrows=48, expect_plan=False, probe_corrupt=1)
    _check(S, cfg, _run(S, 29837, cfg))


def test_pair_split_first_step_check_falls_back():
    """the pair split's first step is checked against the
    row-block layout on every rank (DistSampler._check_pair_split).  With one
    rank's pair-split phi spoiled the shared verdict fails on both ranks, the
    owned rows are moved by the row-block phi instead (the update matches the
    oracle) and the row-block engine is the only one kept."""
    S, m = 2, 4096     # m * n >= 2^24: the bracketed median, so the layout applies
    cfg = dict(n=S * m, d=256, N=1024, eps=1e-3, seed=33, h="median", mode="all_scores",
               nrows=48, expect_plan=False, check_corrupt=0)
    _check(S, cfg, _run(S, 29839, cfg))
