"""Per-stage timings of one Jacobi DistSampler step (S = 1, median bandwidth)
at BASELINE.json's other configurations, with the achieved rate of each
stage against its roofline (HBM GB/s for the distance / select / exp passes,
MFMA TF/s for the contractions).

    python scripts/configs_bench.py [--only B,C,E] [--steps 5] [--order sequential]

--order sequential times the reference's default Gauss-Seidel order (one
phi_row launch + one score refresh per particle, host-driven) instead of the
Jacobi fast path; only the whole-step time is reported then.

  B  experiments/gmm.py target, n = 1024, d = 1          (direct VALU kernels)
  C  Gaussian N(mu, diag(1/lam)), n = 16384, d = 64       (MFMA, short K)
  D  dist-logreg headline, n = 65536, d = 256, N = 16384  (the bench.py workload)
  E  BNN-like logreg, n = 65536, d = 1024, N = 8192       (one GPU's share x 8)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_TF, PEAK_GBS = 157.3, 8000.0
PEAK_X3_TF = 2516.6 / 6   # split engine: bf16 dense / six products per fp32 product


def logreg_data(N, p, seed=0):
    rs = np.random.RandomState(seed)
    x = (rs.randn(N, p) / np.sqrt(p)).astype(np.float32)
    w = np.random.RandomState(seed + 1).randn(p)
    t = np.where(x @ w + np.random.RandomState(seed + 2).logistic(size=N) > 0, 1.0, -1.0)
    return x, t.astype(np.float32)


def config(name):
    import dsvgd
    T = dsvgd.targets
    rs = np.random.RandomState(1)
    if name == "B":
        return 1024, 1, T.GaussianMixture1D(), 1.0, 1
    if name == "C":
        d = 64
        return 16384, d, T.Gaussian(rs.randn(d), rs.uniform(0.5, 2, d)), 1.0, 1
    if name == "D":
        x, t = logreg_data(16384, 255)
        return 65536, 256, T.LogisticRegression(x, t), 0.1, 16384
    x, t = logreg_data(8192, 1023)
    return 65536, 1024, T.LogisticRegression(x, t), 0.1, 8192


def run(name, steps, order="jacobi"):
    import dsvgd
    from dsvgd.engine import StageTimer
    n, d, tgt, scale, N = config(name)
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (scale * torch.randn(n, d, generator=g)).cuda()
    ds = dsvgd.DistSampler(0, 1, tgt, dsvgd.RBF("median"), X, N, N, exchange_particles=False,
                           exchange_scores=False, include_wasserstein=False, order=order)
    for _ in range(2 if order == "jacobi" else 1):
        ds.make_step(1e-4)
    torch.cuda.synchronize()
    timer = StageTimer()
    ds.timer = timer
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        ds.make_step(1e-4)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    st = {k: float(np.mean(v)) for k, v in timer.summary().items()}
    if order != "jacobi":
        # the same sweeps as replays of the captured HIP graph (S = 1, built-in
        # target: one graph node per row kernel and per score refresh)
        ds.timer = None
        ds.make_step(1e-4)                   # eager call that captures the graph next
        ds.make_step(1e-4)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(steps):
            ds.make_step(1e-4)
        e1.record()
        torch.cuda.synchronize()
        ms_graph = e0.elapsed_time(e1) / steps
        return {"n": n, "d": d, "order": order, "ms_per_step": ms,
                "particle_updates_per_s": n / ms * 1e3, "graph_ms_per_step": ms_graph,
                "graph_particle_updates_per_s": n / ms_graph * 1e3, "stages_ms": st}
    # the same steps as replays of the captured HIP graph (no per-stage events)
    ds.timer = None
    e0.record()
    for _ in range(steps):
        ds.make_step(1e-4)
    e1.record()
    torch.cuda.synchronize()
    ms_graph = e0.elapsed_time(e1) / steps
    eng = next(iter(ds._engines.values()))
    m = n
    out = {"n": n, "d": d, "ms_per_step": ms, "particle_updates_per_s": n / ms * 1e3,
           "graph_ms_per_step": ms_graph, "graph_particle_updates_per_s": n / ms_graph * 1e3,
           "stages_ms": st, "bracketed_select": bool(eng.bracketed)}
    rates = {}
    if "phi_mm" in st:
        rates["sqdist_TFs_on_sym_flops"] = (n * n * eng.dp) / (st["sqdist"] * 1e-3) / 1e12
        rates["sqdist_GBs_written"] = 4.0 * m * n / (st["sqdist"] * 1e-3) / 1e9
        rates["phi_mm_TFs"] = 4.0 * m * n * d / (st["phi_mm"] * 1e-3) / 1e12
        rates["phi_mm_frac_of_f32_peak"] = rates["phi_mm_TFs"] / PEAK_TF
        if getattr(eng, "x3", False):
            rates["phi_mm_frac_of_x3_peak"] = rates["phi_mm_TFs"] / PEAK_X3_TF
        rates["phi_mm_GBs_D_read"] = 4.0 * m * n / (st["phi_mm"] * 1e-3) / 1e9
    else:
        # distance pass: 4 B written per entry (the kernel's HBM traffic);
        # phi_direct: D read once (4 B per entry) + the exp of every entry
        rates["sqdist_GBs_written"] = 4.0 * m * n / (st["sqdist"] * 1e-3) / 1e9
        rates["phi_direct_GBs_D_read"] = 4.0 * m * n / (st["phi_direct"] * 1e-3) / 1e9
        rates["phi_direct_VALU_TFs"] = 3.0 * m * n * d / (st["phi_direct"] * 1e-3) / 1e12
    if "radix_hist" in st:
        rates["select_ms_after_distances"] = st.get("radix_hist", 0) * 3 + st.get("bracket", 0)
    if isinstance(tgt, dsvgd.targets.LogisticRegression):
        rates["scores_TFs"] = 4.0 * n * N * (d - 1) / (st["scores"] * 1e-3) / 1e12
    out["rates"] = rates
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="B,C,D,E")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--order", default="jacobi", choices=["jacobi", "sequential"])
    ap.add_argument("--lib", default=None, help="an A/B build of the library (make ab)")
    args = ap.parse_args()
    if args.lib:
        import dsvgd
        dsvgd._native.LIB_PATH = os.path.abspath(args.lib)
    res = {}
    for c in args.only.split(","):
        res[c] = run(c, args.steps, args.order)
        print(json.dumps({c: res[c]}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
