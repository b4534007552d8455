"""2 ranks (gloo) share cuda:0: row-sharded engine with the all-reduced median."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dist-svgd_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def worker(rank, S, port, X, q):
    import torch.distributed as dist
    import dsvgd
    from dsvgd import exchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=S)
    n, d = X.shape
    m = n // S
    Xg = torch.tensor(X, device="cuda:0")
    Sg = -Xg
    eng = dsvgd.PhiEngine(n, d, m=m, row0=rank * m, device="cuda:0")
    eng.pack(Xg, Sg)
    eng.distances(median=True)
    pre = eng.state.bracket()
    eng.median_bandwidth(lambda t: exchange.all_reduce_sum(t))
    eng.direction(write_phi=True)
    q.put((rank, eng.state.read(), pre, eng.state.bracket(), eng.bracketed, eng.phi.cpu().numpy(),
           eng.dense_D().cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    from oracle import svgd_oracle as O
    n, d, S = int(sys.argv[1]), int(sys.argv[2]), 2
    X = np.random.RandomState(d).randn(n, d).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, S, 29900, X, q)) for r in range(S)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(S)], key=lambda r: r[0])
    for p in ps:
        p.join()
    h64, med64 = O.median_bandwidth(X)
    Dall = np.concatenate([r[6] for r in res])
    k = (n * n - 1) // 2
    exact = np.partition(Dall.ravel(), k)[k]
    print("oracle med", med64, "h", h64, "| exact med of GPU D", exact)
    for r in res:
        print("rank", r[0], "state(med,h,inv_h)", r[1], "bracket pre", r[2], "post", r[3], "bracketed", r[4])
    h = res[0][1][1]
    phi = np.concatenate([r[5] for r in res])
    ref = O.phi(X, -X, h)
    print("phi err (GPU h)", np.abs(phi - ref).max() / np.abs(ref).max(), "max|phi|", np.abs(ref).max())
    ref2 = O.phi(X, -X, h64)
    print("phi err (oracle h)", np.abs(phi - ref2).max() / np.abs(ref2).max())


if __name__ == "__main__":
    main()
