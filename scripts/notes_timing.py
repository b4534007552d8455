"""notes.md's timing configuration on the GPU harness: distributed logistic
regression, 50 particles, 500 iterations, step 3e-3 (reference: 2007 s at
world size 1 ... 59 s at 8, notes.md 'Timing results', CPU/tcp).  Synthetic
banana-like data (benchmarks.mat is a git-LFS pointer).

    python scripts/notes_timing.py [--order sequential|jacobi] [--niter 500]
"""
import argparse
import importlib.util
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="sequential")
    ap.add_argument("--niter", type=int, default=500)
    ap.add_argument("--nparticles", type=int, default=50)
    args = ap.parse_args()
    spec = importlib.util.spec_from_file_location(
        "lr", os.path.join(ROOT, "dist-svgd_amd", "experiments", "logreg.py"))
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        t = {}
        H.run(0, 1, 'banana', 42, args.nparticles, args.niter, 3e-3, 'partitions', False, d, None,
              args.order, 'cuda:0', timings=t)
        df = H.load_results(d)
        x, tr, xt, tt = H.synthetic_banana()
        acc = H.test_accuracy_curve(df[df.timestep == args.niter], x, tr, xt, tt)
        out = {"config": "notes.md timing: n=%d, T=%d, eps=3e-3, S=1, partitions, %s"
                         % (args.nparticles, args.niter, args.order),
               "wall_s": t["wall_s"], "reference_wall_s_notes_md": 2007.11,
               "final_test_acc": float(acc['dsvgd'].iloc[0]),
               "sklearn_test_acc": float(acc['sklearn logreg'].iloc[0])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
