"""bench.py contract: the roofline traffic comes from the phi_mm launches of the
committed PMC summary, and the multi-rank path (barrier, max-over-ranks time,
one JSON line from rank 0) runs under torch.distributed.run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_pmc_traffic_picks_phi_mm():
    """The quoted traffic is phi_mm's: on the symmetric layout phi_w1<4> (one
    launch per row), or with the two-launch form the sum of phi_w1<1>
    (transposed K-steps) and phi_w1<2> (the rest) of the same step -- never a
    logreg launch -- and nothing when a launch of the pair is missing."""
    import bench
    summ = os.path.join(ROOT, "profiles", "latest_summary.json")
    if not os.path.exists(summ):
        pytest.skip("no committed PMC summary")
    with open(summ) as f:
        ks = json.load(f)["kernels"]
    w1 = "_ZN5dsvgd13phi_w1_kernelILi1E"
    w2 = "_ZN5dsvgd13phi_w1_kernelILi2E"

    def per_launch(prefix):
        hit = [v["hbm_bytes_per_launch"] for k, v in ks.items()
               if k.startswith(prefix) and "hbm_bytes_per_launch" in v]
        return hit[0] if hit else None

    a, b = per_launch(w1), per_launch(w2)
    both, src = bench.pmc_traffic([w1, w2])
    if a is None or b is None:
        assert both is None   # a launch of the pair missing: nothing quoted
    else:
        assert both == a + b
        assert src == os.path.join("profiles", "latest_summary.json")
    assert bench.pmc_traffic(["no-such-kernel"]) == (None, None)
    w4 = "_ZN5dsvgd13phi_w1_kernelILi4E"   # the one-launch form (default since round 5)
    c = per_launch(w4)
    assert bench.pmc_traffic([w4])[0] == c
    lr = [k for k in ks if "logreg" in k and "hbm_bytes_per_launch" in ks[k]]
    if lr and a is not None:
        assert all(not k.startswith(w1) for k in lr)


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launches_its_own_ranks(n):
    """`python bench.py --gpus N` with no launcher starts N ranks itself
    (VERDICT r2 next #1): every rank joins one process group of N, rank 0
    prints the one line.  --launch-check stops before any GPU work, so this
    runs on the CPU."""
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--backend", "gloo", "--launch-check"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and sorted(out["ranks"]) == list(range(n))


def test_bench_rejects_world_size_mismatch():
    """A launcher that starts fewer ranks than --gpus asks for is an error,
    not a silent one-GPU measurement."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29771", "bench.py", "--gpus", "4",
           "--backend", "gloo", "--launch-check"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_gloo():
    """`python bench.py --gpus 2` (the driver's form) measures two ranks."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--particles", "4096", "--dim", "64", "--data-rows", "1024", "--backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["process_group"]["world_size_seen"] == 2
    # all_scores with the logreg target: the own block's scores over the
    # gathered data, the score blocks all-gathered (DistSampler gather_data)
    assert "allgather_x" in out["stages_ms"] and "allgather_scores" in out["stages_ms"]
    assert out["multi_gpu"]["scores_gathered_data"] == [True, True]
    assert "hist_allreduce" in out["stages_ms"]


@pytest.mark.gpu
def test_bench_two_ranks_gloo():
    """2 ranks sharing cuda:0, gloo exchange: the N>1 timing/reporting path,
    at a shape where the pair-split layout applies (d = 256, m = 4096), with
    the self-describing multi-GPU keys: the layout each
    rank ran, the route probe, the first-step check, per-rank exchange times."""
    env = _env()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29763", "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--particles", "8192", "--dim", "256",
           "--data-rows", "1024", "--backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2
    assert out["config"]["particles_per_gpu"] == 4096
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert abs(out["value"] - 8192 * 2 / (out["ms_per_step"] * 2e-3)) < 1e-6 * out["value"]
    mg = out["multi_gpu"]
    assert mg["world_size"] == 2 and mg["backend"] == "gloo"
    assert mg["pair_split_engaged"] == [True, True] and mg["route_probe_ok"] == [True, True]
    assert mg["pair_split_first_step_check"] <= mg["pair_split_check_tol"] == 1e-5
    assert mg["scores_gathered_data"] == [True, True]
    assert len(mg["exchange_ms_per_rank"]) == 2
    for ex in mg["exchange_ms_per_rank"]:
        for k in ("allgather_x", "allgather_scores", "hist_allreduce", "partials_wait"):
            assert k in ex and ex[k] >= 0.0
    assert out["roofline"]["traffic"] is None   # N=1 PMC summary is not quoted at N>1
    assert "cpu_baseline" not in out
