"""notes.md's timing configuration on the GPU harness: distributed logistic
regression, 50 particles, 500 iterations, step 3e-3 (reference: 2007 s at
world size 1 ... 59 s at 8; 8-laggedlocal 226 s, 8-laggedlocal-updateall
2771 s -- notes.md:120-135, CPU/tcp).  Synthetic banana-like data
(benchmarks.mat is a git-LFS pointer).  S > 1: S ranks share cuda:0 over
gloo (this box has one GPU), the slowest rank's wall time is reported.

    python scripts/notes_timing.py [--order sequential|jacobi] [--niter 500]
                                   [--nproc 8 --exchange laggedlocal]
"""
import argparse
import importlib.util
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

REFERENCE_S = {("partitions", 1): 2007.11, ("partitions", 2): 538.59, ("partitions", 4): 157.17,
               ("partitions", 8): 59.353, ("laggedlocal", 8): 226.24,
               ("laggedlocal-updateall", 8): 2770.66}


def _harness():
    spec = importlib.util.spec_from_file_location(
        "lr", os.path.join(ROOT, "dist-svgd_amd", "experiments", "logreg.py"))
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    return H


def _rank(rank, S, port, args, d, q):
    import torch.distributed as dist
    H = _harness()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    t = {}
    H.run(rank, S, 'banana', 42, args.nparticles, args.niter, 3e-3, args.exchange, False, d,
          None, args.order, 'cuda:0', timings=t)
    dist.barrier()
    dist.destroy_process_group()
    q.put(t["wall_s"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="sequential")
    ap.add_argument("--niter", type=int, default=500)
    ap.add_argument("--nparticles", type=int, default=50)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--exchange", default="partitions")
    args = ap.parse_args()
    H = _harness()
    with tempfile.TemporaryDirectory() as d:
        if args.nproc == 1:
            t = {}
            H.run(0, 1, 'banana', 42, args.nparticles, args.niter, 3e-3, args.exchange, False, d,
                  None, args.order, 'cuda:0', timings=t)
            wall = t["wall_s"]
        else:
            import torch.multiprocessing as mp
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            ps = [ctx.Process(target=_rank, args=(r, args.nproc, 29700 + args.nproc, args, d, q))
                  for r in range(args.nproc)]
            for p in ps:
                p.start()
            wall = max(q.get(timeout=1200) for _ in ps)
            for p in ps:
                p.join(60)
        df = H.load_results(d)
        x, tr, xt, tt = H.synthetic_banana()
        acc = H.test_accuracy_curve(df[df.timestep == args.niter], x, tr, xt, tt)
    out = {"config": "notes.md timing: n=%d, T=%d, eps=3e-3, S=%d, %s, %s"
                      % (args.nparticles, args.niter, args.nproc, args.exchange, args.order),
           "wall_s": wall,
           "reference_wall_s_notes_md": REFERENCE_S.get((args.exchange, args.nproc)),
           "ranks_share_one_gpu": args.nproc > 1,
           "final_test_acc": float(acc['dsvgd'].iloc[0]),
           "sklearn_test_acc": float(acc['sklearn logreg'].iloc[0])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
