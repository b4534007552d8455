"""bench.py -- SVGD particle-updates/s at n=65536, d=256 (BASELINE.json metric).

Workload (BASELINE.json configs[3]): dist-logreg via
DistSampler, exchange=all_scores (all-gather of particles + the scores of all
n particles over all N data rows: at N > 1 by default each rank scores its own
block over the once-gathered data and the score blocks are all-gathered --
DistSampler gather_data, the same sums as the reference's all-reduce of the
shard-local scores), median-heuristic bandwidth, Jacobi
order, n = 65536 particles of d = 256 (p = 255 weights), N_global = 16384
synthetic data rows sharded N/S, the n particles sharded n/S per GPU.
One step = exchange + scores + median (exact radix select over n^2 distances)
+ phi (K.[X|S] on MFMA) + x += eps*phi for all n particles.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, RCCL)

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment
launches its N ranks itself (a torch.distributed.run child on 127.0.0.1,
started before this process touches the GPU; like the reference harness's
one-Process-per-rank launch, experiments/logreg.py:126-140) and relays rank
0's line.  Every rank checks that the process group has exactly --gpus ranks.

Prints ONE JSON line (rank 0).  value = n*K / max-over-ranks wall time of the K
timed steps (whole job).  roofline: the dominant kernel (phi_mm, the fused
exp + K.[Xc|S] MFMA GEMM) -- algorithmic 4*m*n*d flop per launch / its mean
HIP-event duration, against the ceiling of the engine it runs on: the
fp32-accurate fp16-split engine FmtH2 (2516 TF fp16 dense / 3 products = 839
TF of fp32 products; csrc/gemm_x3.hpp), the bf16-split FmtX3 (/ 6 = 419 TF) or
the 157.3 TF fp32 MFMA peak (--gemm x3 / f32).  cpu_baseline: the
reference algorithm's per-pair autograd loop (oracle/loop_baseline.py, a port)
timed on this host on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "dist-svgd_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, spec
# phi_mm runs on v_mfma_f32_32x32x16_bf16 (1024 flop/clk/SIMD x 1024 SIMDs x
# 2.4 GHz = 2516 TF dense) with six split products per fp32 product
# (csrc/gemm_x3.hpp): the fp32-equivalent ceiling of that engine
PEAK_BF16_MFMA_TFLOPS = 2516.6     # = the fp16 MFMA rate (same cycles)
SPLIT_PRODUCTS = {"h2": 3, "x3": 6}
PEAK_X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / SPLIT_PRODUCTS["x3"]


def engine_peak(gemm):
    """fp32-product ceiling of an engine (TFLOP/s) and its basis."""
    if gemm == "f32":
        return PEAK_FP32_MFMA_TFLOPS, "f32 MFMA (v_mfma_f32_32x32x2_f32)"
    k = SPLIT_PRODUCTS[gemm]
    return (PEAK_BF16_MFMA_TFLOPS / k,
            "%s dense MFMA %.1f TF / %d split products" % ("fp16" if gemm == "h2" else "bf16",
                                                          PEAK_BF16_MFMA_TFLOPS, k))
PEAK_HBM_GBS = 8000.0
# what the chip sustains on bare back-to-back v_mfma_f32_32x32x16_f16 with
# random operands, one wave per SIMD on every CU (the clock it holds under
# that load): scripts/mfma_shape_probe.hip, profiles/r9b/mfma_probe.log
SUSTAINED_F16_MFMA_TFLOPS = 1724.0


def synthetic_data(N, p, seed=0):
    rs = np.random.RandomState(seed)
    x = rs.randn(N, p).astype(np.float32) / np.sqrt(p)
    w = np.random.RandomState(seed + 1).randn(p)
    z = x @ w + np.random.RandomState(seed + 2).logistic(size=N)
    t = np.where(z > 0, 1.0, -1.0).astype(np.float32)
    return x, t


def cpu_baseline(n, d, x_local, t_local, budget_s):
    """Reference-algorithm per-pair loop (port) on a bounded sample."""
    from oracle import loop_baseline as L
    from oracle import cpu_vectorized as V
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(1)
    rs = np.random.RandomState(1)
    X = rs.randn(n, d).astype(np.float32) * 0.1
    logp = L.logreg_logp(x_local, t_local)
    sec_per_update, updates, pairs = L.time_particle_updates(X, logp, h=float(d), m=1,
                                                             budget_s=budget_s)
    out = {"value": 1.0 / sec_per_update, "unit": "particle-updates/s", "cores": 1,
           "kind": "port",
           "sample": "reference per-pair autograd loop (kernel, grad kernel, grad logp per pair; "
                     "oracle/loop_baseline.py), %d pair terms of one n=%d particle update timed, "
                     "extrapolated x n; logreg target N_local=%d" % (pairs, n, x_local.shape[0])}
    # vectorised torch-CPU restatement on all host cores (extra, for scale)
    nt = min(cores, 64)
    torch.set_num_threads(nt)
    S = rs.randn(n, d).astype(np.float32)
    spu, rows = V.time_rows(X, S, float(d), rows=4096, chunk=512, budget_s=budget_s / 2)
    out["vectorized_value"] = 1.0 / spu
    out["vectorized_cores"] = nt
    out["vectorized_sample"] = "torch-CPU fp32 phi for %d rows against all n=%d (oracle/cpu_vectorized.py)" % (rows, n)
    out["host_cores_available"] = cores
    return out


def pmc_traffic(kernel_prefixes):
    """HBM bytes per phi_mm from the committed rocprofv3 --pmc summary
    (FETCH_SIZE x2 [gfx950 half-count] + WRITE_SIZE, separate passes;
    scripts/pmc_summary.py): the sum over the launches phi_mm makes (one
    kernel, or on the symmetric layout phi_w1<1>'s transposed part + phi_w1<2>'s
    plain part) -- None unless every one of them is in the summary."""
    path = os.path.join(ROOT, "profiles", "latest_summary.json")
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    total = 0.0
    for prefix in kernel_prefixes:
        hit = [v["hbm_bytes_per_launch"] for name, v in ks.items()
               if name.startswith(prefix) and "hbm_bytes_per_launch" in v]
        if not hit:
            return None, None
        total += hit[0]
    return total, os.path.relpath(path, ROOT)


def pmc_mfma(prefix):
    """MFMA-busy (SQ_VALU_MFMA_BUSY_CYCLES over the kernel's cycles x 1024
    SIMDs) and the clock under load of the first kernel named `prefix` in the
    committed PMC summary (scripts/pmc_summary.py "mfma" pass), or None."""
    path = os.path.join(ROOT, "profiles", "latest_summary.json")
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for name, v in ks.items():
        if name.startswith(prefix) and "mfma_busy" in v:
            return {"mfma_busy": v["mfma_busy"], "clock_ghz": v.get("clock_ghz"),
                    "kernel": name, "source": os.path.relpath(path, ROOT)}
    return None


def passes(eng, stages, m, n, d, n_local, score_gemm):
    """The other passes of the step, each against its own bound (north_star:
    MFMA rate for the contractions, HBM GB/s for the distance and select
    passes; the RBF exp is fused into phi_mm's A staging, no pass of its own).
    The distance pass is credited the D entries its layout writes (upper
    256-tiles only in the symmetric layout), 2d flop and 4 bytes each (the m*n
    figure without symmetry credit rides along); the select passes the
    candidate floats they read (bracketed) or D (radix passes over D)."""
    out = {}
    t = stages.get("sqdist")
    if t:
        if eng.sym:
            tiles = -(-eng.n_pad // 256)
            d_bytes = 4.0 * 256 * 256 * tiles * (tiles + 1) / 2
        else:
            d_bytes = 4.0 * m * eng.n_pad
        # computed work: the tiles the layout writes, 2d flop per entry
        tf = 2.0 * d * (d_bytes / 4.0) / (t * 1e-3) / 1e12
        peak = engine_peak(eng.gram_gemm)[0]
        out["distances"] = {"ms": t, "bound": "mfma", "tflops": tf, "frac_mfma": tf / peak,
                            "tflops_no_symmetry_credit": 2.0 * m * n * d / (t * 1e-3) / 1e12,
                            "d_bytes_written": d_bytes,
                            "write_gbs": d_bytes / (t * 1e-3) / 1e9,
                            "frac_hbm": d_bytes / (t * 1e-3) / 1e9 / PEAK_HBM_GBS,
                            "pmc": pmc_mfma("_ZN5dsvgd14gram_rs_kernelILi2ELb1E") or
                            pmc_mfma("_ZN5dsvgd14gram_w1_kernelILi2ELb1E")}
    t = stages.get("radix_hist")
    if t:
        if eng.bracketed:
            _, _, _, ncand, fb = eng.state.bracket()
            nbytes = 4.0 * ncand if not fb else 4.0 * m * eng.n_pad
            # stages average per launch: the bracketed select runs 3 candidate passes
            out["select"] = {"ms_per_pass": t, "passes": 3, "candidates": int(ncand),
                             "fallback": int(fb), "bytes_per_pass": nbytes,
                             "read_gbs": nbytes / (t * 1e-3) / 1e9}
        else:
            nbytes = 4.0 * m * eng.n_pad
            out["select"] = {"ms_per_pass": t, "passes": 2, "bytes_per_pass": nbytes,
                             "read_gbs": nbytes / (t * 1e-3) / 1e9}
    t = stages.get("scores")
    if t:
        tf = 4.0 * n * n_local * (d - 1) / (t * 1e-3) / 1e12
        peak = engine_peak(score_gemm)[0]
        out["scores"] = {"ms": t, "bound": "mfma", "tflops": tf, "frac_mfma": tf / peak,
                         "pmc": pmc_mfma("_ZN5dsvgd19logreg_fused_kernel")}
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def kfd_gpu_count():
    """GPUs the KFD topology lists (nodes with a nonzero gpu_id), read from
    sysfs: no HIP runtime call, so the launching parent never initialises the
    GPU stack before it starts the ranks.  None when the topology is unreadable."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(base)
    except OSError:
        return None
    count = 0
    for nd in nodes:
        try:
            with open(os.path.join(base, nd, "gpu_id")) as f:
                count += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis is not None:
        count = min(count, len([v for v in vis.split(",") if v.strip() != ""]))
    return count


def launch_ranks(args, argv):
    """--gpus N > 1 without a launcher: run N ranks as a torch.distributed.run
    child (one process per GPU, rendezvous on 127.0.0.1) and pass its output
    through.  This process never touches the HIP runtime (GPUs are counted from
    the KFD sysfs topology), so the ranks own their devices; exits with the
    child's code."""
    import subprocess
    if args.backend == "nccl":
        have = kfd_gpu_count()
        if have is not None and have < args.gpus:
            print("bench.py: --gpus %d but only %d GPU(s) visible" % (args.gpus, have),
                  file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:           # streamed: rank 0's JSON line and progress
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def gather_max(d, world, backend, dev):
    """{name: value} -> {name: max over ranks} (stage times at N > 1)."""
    if world == 1:
        return d
    objs = [None] * world
    dist.all_gather_object(objs, d)
    keys = sorted(set().union(*[o.keys() for o in objs]))
    return {k: max(o.get(k, 0.0) for o in objs) for k in keys}


EXCHANGE_STAGES = ("allgather_x", "allreduce_scores", "allgather_scores", "hist_allreduce",
                   "partials_post", "partials_wait")


def multi_gpu_report(sampler, eng, local_stages, world):
    """N > 1: what ran, per rank -- whether the
    pair-split layout engaged, its route probe's verdict and
    its first-step check against the row-block layout (DistSampler), and
    each rank's mean HIP-event time per step of every exchange stage (the
    particle all-gather, the score all-reduce or, with gathered data, the
    score all-gather, the median's histogram
    all-reduces, the pair split's partials post / join wait)."""
    mine = {"rank": dist.get_rank(),
            "pair_split": eng.plan is not None,
            "gathered_data": bool(sampler._gdata),
            "route_probe_ok": sampler._routes_ok,
            "exchange_ms": {k: local_stages[k] for k in EXCHANGE_STAGES if k in local_stages}}
    ranks = [None] * world
    dist.all_gather_object(ranks, mine)
    ranks.sort(key=lambda r: r["rank"])
    return {"backend": dist.get_backend(),
            "world_size": dist.get_world_size(),
            "pair_split_engaged": [r["pair_split"] for r in ranks],
            # all_scores as the own block's scores over every rank's data,
            # all-gathered (DistSampler gather_data); False: the all-reduce
            "scores_gathered_data": [r["gathered_data"] for r in ranks],
            "route_probe_ok": [r["route_probe_ok"] for r in ranks],
            "pair_split_first_step_check": sampler.pair_split_check,
            "pair_split_check_tol": sampler.PAIR_SPLIT_CHECK_TOL,
            "exchange_ms_per_rank": [r["exchange_ms"] for r in ranks]}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    # (no option that abbreviates torchrun's own: --n would clash with --nnodes)
    ap.add_argument("--particles", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--data-rows", type=int, default=16384, help="global data rows")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--breakdown", type=int, default=3,
                    help="extra steps after the timed region with every stage's HIP events")
    ap.add_argument("--gemm", default="h2", choices=["h2", "x3", "f32"],
                    help="MFMA engine of the contractions (h2: fp16 split, the default)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: CPU-staged rehearsal of the multi-rank path (e.g. 2 ranks on 1 GPU)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher self-test: ranks form the (gloo) group and report, no GPU work")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        if world > 1:
            dist.init_process_group("gloo")
        seen = dist.get_world_size() if world > 1 else 1
        ranks = [None] * seen
        if world > 1:
            dist.all_gather_object(ranks, rank)
        if rank == 0:
            print(json.dumps({"n_gpus": seen, "ranks": ranks if world > 1 else [0],
                              "gpus_requested": args.gpus}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0 if seen == args.gpus else 3
    if args.backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            print("bench.py: process group has %d ranks but --gpus %d"
                  % (dist.get_world_size(), args.gpus), file=sys.stderr)
            return 3
    elif args.gpus != 1:
        print("bench.py: --gpus %d but WORLD_SIZE=1" % args.gpus, file=sys.stderr)
        return 3

    import dsvgd
    from dsvgd.engine import StageTimer

    n, d, Ng = args.particles, args.dim, args.data_rows
    p = d - 1
    per_data = Ng // world
    x, t = synthetic_data(Ng, p)
    xl, tl = x[rank * per_data:(rank + 1) * per_data], t[rank * per_data:(rank + 1) * per_data]
    gen = torch.Generator(device="cpu").manual_seed(0)
    parts = (0.1 * torch.randn(n, d, generator=gen)).to(dev)
    dsvgd.PhiEngine.DEFAULT_GEMM = args.gemm
    sampler = dsvgd.DistSampler(rank, world, dsvgd.targets.LogisticRegression(xl, tl, gemm=args.gemm),
                                dsvgd.RBF("median"), parts, per_data, per_data * world,
                                exchange_particles=True, exchange_scores=True,
                                include_wasserstein=False, order="jacobi")
    eps = 1e-4

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        sampler.make_step(eps)
    torch.cuda.synchronize()
    # phi_mm's HIP events ride along the timed steps (same stream as its
    # kernels); every other stage's pair of stream markers would stall the
    # queue between kernels (≈ 10 µs each, profiles/r13j), so the per-stage
    # breakdown is timed on --breakdown extra steps after the timed region
    timer = StageTimer(only={"phi_mm"})
    sampler.timer = timer
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sampler.make_step(eps)
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    sampler.timer = None
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64,
                          device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ev = timer.summary().get("phi_mm") or [float("nan")]
    phi_timed = gather_max({"phi_mm": float(np.mean(ev))}, world, args.backend, dev)
    full = StageTimer()
    sampler.timer = full
    for _ in range(args.breakdown):
        sampler.make_step(eps)
    sampler.timer = None
    local_stages = {k: float(np.mean(v)) for k, v in full.summary().items()}
    # N > 1: each stage's mean HIP-event time, max over ranks (the exchange
    # stages allgather_x / allreduce_scores / hist_allreduce included)
    stages = gather_max(local_stages, world, args.backend, dev)
    assert bool(torch.isfinite(sampler._work).all()), "non-finite particles"

    m = n // world
    phi_ms = phi_timed["phi_mm"]     # the timed region's own launches
    eng = sampler._engines[next(iter(sampler._engines))]
    gemm = eng.phi_gemm
    peak, peak_basis = engine_peak(gemm)
    # the committed PMC summary is an N=1 profile: only quoted for the N=1 run
    # phi_mm is the NN tile with the fused exp (<TN, DMA, EXP=true, ..., Fmt>);
    # the logreg G.Xd launch is the same tile with EXP=false
    from dsvgd import _native as NL
    symrow = NL.load().dsvgd_phi_set_symrow(1)       # read the form back (set returns it)
    NL.load().dsvgd_phi_set_symrow(symrow)
    knames = {"h2": ((["_ZN5dsvgd13phi_w1_kernelILi4E"] if symrow else
                      ["_ZN5dsvgd13phi_w1_kernelILi1E", "_ZN5dsvgd13phi_w1_kernelILi2E"])
                     if eng.sym else ["_ZN5dsvgd13phi_w1_kernelILi0E"]),
              "x3": ["void dsvgd::nn_x3_kernel<4, true, true, true, 2, dsvgd::FmtX3,"],
              "f32": ["void dsvgd::nn_kernel<4, true,"]}[gemm]
    traffic, traffic_src = pmc_traffic(knames) if world == 1 else (None, None)
    flops = 4.0 * m * n * d
    achieved = flops / (phi_ms * 1e-3) / 1e12
    out = {
        "metric": "SVGD particle-updates/sec (n=65536,d=256) at 1/2/4/8 GPUs + % MFMA/HBM roofline",
        "value": n * args.steps / el,
        "unit": "particle-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        # what the contractions run on: fp32 operands split into 16-bit parts
        # whose products the MFMA accumulates exactly in fp32
        "mfma_operands": {"h2": "f16 x2 parts (3 products), fp32 accumulate",
                          "x3": "bf16 x3 parts (6 products), fp32 accumulate",
                          "f32": "f32"}[args.gemm],
        "data": "synthetic (logreg data N(0,1/p), labels from a random w + logistic noise; "
                "particles 0.1*N(0,1))",
        "config": {"workload": "dist-logreg DistSampler all_scores, Jacobi, median bandwidth",
                   "n": n, "d": d, "N_global": Ng, "parallelism": "dp%d" % world,
                   "particles_per_gpu": m},
        "roofline": {"bound": "mfma",
                     "kernel": {"h2": (("phi_mm (phi_w1_kernel<4>: one launch, each row block's "
                                        "split-K slices walking contiguous K ranges, its transposed "
                                        "K-steps first, slices mapped to XCDs; one wave per SIMD, FmtH2"
                                        if symrow else
                                        "phi_mm (phi_w1_kernel<1> on each row block's "
                                        "transposed K-steps + phi_w1_kernel<2> on the rest: one wave "
                                        "per SIMD, FmtH2") if eng.sym
                                       else "phi_mm (phi_w1_kernel<0>: one wave per SIMD, FmtH2") +
                                      ": fp32-accurate 2-part fp16 split, 3 fp16 MFMA products "
                                      "per fp32 product; D layout %s)" % ("symmetric" if eng.sym
                                                                          else "full"),
                                "x3": "phi_mm (nn_x3_kernel<4, FmtX3>: fp32-accurate 3-part bf16 "
                                      "split, 6 bf16 MFMA products per fp32 product)",
                                "f32": "phi_mm (nn_kernel<4,true>: f32 MFMA)"}[gemm],
                     "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "peak_basis": peak_basis,
                     "frac": achieved / peak, "frac_of_f32_mfma_peak": achieved / PEAK_FP32_MFMA_TFLOPS,
                     "frac_of_sustained_mfma": (achieved / (SUSTAINED_F16_MFMA_TFLOPS / SPLIT_PRODUCTS[gemm])
                                                if gemm in SPLIT_PRODUCTS else None),
                     "sustained_basis": "bare fp16 32x32x16 MFMA loop under DVFS, 1724 TF "
                                        "(profiles/r9b/mfma_probe.log) / split products",
                     "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "algorithmic_bytes": 4.0 * m * n + 4.0 * (n + 128) * 512,
                     "flop_per_launch": flops, "avg_launch_ms": phi_ms,
                     # the committed N = 1 PMC pass of the same kernel (None at N > 1)
                     "pmc": pmc_mfma(knames[0]) if world == 1 else None},
        "stages_ms": stages,
        "stages_basis": "mean HIP-event time per step over %d steps after the timed region "
                        "(phi_mm in roofline: the timed steps' own)" % args.breakdown,
        "passes": passes(eng, stages, m, n, d, per_data, args.gemm),
        "gemm": gemm,
        "step_6n2d_f32_mfma_frac": (6.0 * m * n * d) / (el / args.steps) / 1e12 / PEAK_FP32_MFMA_TFLOPS,
        "phi_splits": int(eng.splits),
        "process_group": {"backend": args.backend if world > 1 else None,
                          "world_size_seen": dist.get_world_size() if world > 1 else 1,
                          "stages": "mean per step, max over ranks" if world > 1 else "mean per step"},
    }
    if world > 1:
        out["multi_gpu"] = multi_gpu_report(sampler, eng, local_stages, world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, d, xl, tl, args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
