"""Distributed Bayesian logistic regression with dsvgd on MI355X -- the
reference's experiment harness (experiments/logreg.py:23-92, results reader
and test-accuracy curve of experiments/logreg_plots.py:19-67,94-112) on the
gfx950 sampler.

    python experiments/logreg.py --nproc 1 --nparticles 50 --niter 500 --stepsize 3e-3
    torchrun --nproc-per-node 8 experiments/logreg.py --nparticles 65536 ...

Same CLI options, per-shard result pickles (`shard-{rank}.pkl`, columns
timestep / value, one row per owned particle per timestep, written right
before every update and after the last, logreg.py:74-92) in the same
directory naming (get_results_dir, logreg_plots.py:19-22), same particle
init (`manual_seed(rank)` then n x Normal(0,1).sample((d,1)), logreg.py:24,63-66),
same RBF kernel exp(-|x-y|^2) (h = 1, logreg.py:60-61) and JKO step h = 10
(logreg.py:77).  Differences, all outside the sampler:

* data: `benchmarks.mat` is read when present (--data-dir; the reference
  ships it as a git-LFS pointer only); otherwise a synthetic "banana-like"
  set with the same structure (p = 2, 400 train / 4900 test rows,
  t = sign(x.w* + logistic noise)) -- SURVEY.md 8(d) config A;
* ranks: one process per GPU (torchrun, or --nproc processes spawned here),
  `nccl` (RCCL) when every rank has its own GPU, else `gloo` with ranks
  sharing the GPUs;
* plots: visdom is not available; `make_plots` writes the test-accuracy
  curve (dsvgd ensemble vs an sklearn logistic regression, logreg_plots.py:25-67)
  to `test_acc.csv` in the results directory, computed on the GPU
  (dsvgd.metrics, the posterior-predictive mean of logreg_plots.py:42-50).
"""
import os
import shutil
import sys
import time

import click
import numpy as np
import pandas as pd
import torch
import torch.distributed as dist
from torch.distributions.normal import Normal

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import dsvgd  # noqa: E402

RESULTS_DIR = os.environ.get("DSVGD_RESULTS_DIR", os.path.join(os.getcwd(), "results"))
DATASETS = ['banana', 'diabetis', 'german', 'image', 'splice', 'titanic', 'waveform']


# notes.md:108-114,134-135 (described and timed there, no code in the reference)
LAGGED = {'laggedlocal': 'local', 'laggedlocal-updateall': 'updateall'}


def get_results_dir(dataset_name, fold, nproc, nparticles, stepsize, exchange, wasserstein,
                    results_dir=None):
    """logreg_plots.py:19-22 (same subdirectory name)."""
    subdir = 'logreg_{}_{}-nshards={}-nparticles={}-exchange={}-wasserstein={}-stepsize={:.0e}'.format(
        dataset_name, fold, nproc, nparticles, exchange, wasserstein, stepsize)
    return os.path.join(results_dir or RESULTS_DIR, subdir)


def synthetic_banana(N_train=400, N_test=4900, p=2, seed=0):
    """Stand-in with the banana split's structure."""
    def make(N, s):
        x = np.random.RandomState(s).randn(N, p).astype(np.float32)
        w = np.random.RandomState(seed + 1).randn(p)
        z = x @ w + np.random.RandomState(s + 2).logistic(size=N)
        return x, np.where(z > 0, 1.0, -1.0).reshape(-1, 1)
    x_train, t_train = make(N_train, seed)
    x_test, t_test = make(N_test, seed + 10)
    return x_train, t_train, x_test, t_test


def load_dataset(dataset_name, fold, data_dir=None):
    """(x_train, t_train, x_test, t_test) of benchmarks.mat split `fold`
    (logreg.py:29-35, logreg_plots.py:27-34), or the synthetic stand-in."""
    path = os.path.join(data_dir, 'benchmarks.mat') if data_dir else None
    if path and os.path.isfile(path) and os.path.getsize(path) > 4096:
        from scipy.io import loadmat
        dataset = loadmat(path)[dataset_name][0, 0]
        x_train = dataset[0][dataset[2] - 1][fold].astype(np.float32)
        t_train = dataset[1][dataset[2] - 1][fold]
        x_test = dataset[0][dataset[3] - 1][fold]
        t_test = dataset[1][dataset[3] - 1][fold]
        return x_train, t_train, x_test, t_test
    return synthetic_banana()


def run(rank, num_shards, dataset_name, fold, nparticles, niter, stepsize, exchange, wasserstein,
        results_dir, data_dir=None, order="sequential", device=None, timings=None):
    """One rank of the experiment (logreg.py:23-92)."""
    torch.manual_seed(rank)
    dev = torch.device(device) if device is not None else torch.device(
        "cuda", rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    x_train, t_train, _, _ = load_dataset(dataset_name, fold, data_dir)
    samples_per_shard = int(x_train.shape[0] / num_shards)
    s, e = samples_per_shard * rank, samples_per_shard * (rank + 1)
    target = dsvgd.targets.LogisticRegression(x_train[s:e], np.asarray(t_train[s:e], np.float32))
    d = 1 + x_train.shape[1]

    q = Normal(0, 1)
    make_sample = lambda: q.sample((d, 1))  # noqa: E731
    particles = torch.cat([make_sample() for _ in range(nparticles)], dim=1).t()
    particles = particles.to(dev)

    sampler = dsvgd.DistSampler(rank, num_shards, target, dsvgd.RBF(1.0), particles,
                                samples_per_shard, samples_per_shard * num_shards,
                                exchange_particles=exchange in ['all_particles', 'all_scores'],
                                exchange_scores=exchange == 'all_scores',
                                include_wasserstein=wasserstein, order=order,
                                lagged=LAGGED.get(exchange))
    m = sampler.particles.shape[0]
    hist = torch.empty(niter + 1, m, d, dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for l in range(niter):
        if rank == 0:
            print('Iteration {}'.format(l))
        hist[l].copy_(sampler.particles)       # right before the update (logreg.py:81-83)
        sampler.make_step(stepsize, h=10.0)
    hist[niter].copy_(sampler.particles)       # after the last update (logreg.py:88-89)
    torch.cuda.synchronize(dev)
    if timings is not None:
        timings["wall_s"] = time.perf_counter() - t0
    vals = hist.cpu().numpy().reshape(-1, d)
    steps = np.repeat(np.arange(niter + 1), m)
    pd.DataFrame({'timestep': steps, 'value': list(vals)}).to_pickle(
        os.path.join(results_dir, 'shard-{}.pkl'.format(rank)))


def load_results(results_dir):
    """All shards' rows (logreg_plots.py:107)."""
    from glob import glob
    files = sorted(glob(os.path.join(results_dir, 'shard-*.pkl')))
    if not files:
        raise FileNotFoundError("no shard-*.pkl in %s" % results_dir)
    return pd.concat(map(pd.read_pickle, files))


def test_accuracy_curve(df, x_train, t_train, x_test, t_test, device="cuda"):
    """Per timestep: the dsvgd posterior-predictive test accuracy (on the GPU)
    and the sklearn logistic-regression baseline (logreg_plots.py:25-58)."""
    from sklearn.linear_model import LogisticRegression
    baseline = (LogisticRegression().fit(x_train, np.asarray(t_train).reshape(-1))
                .score(x_test, np.asarray(t_test).reshape(-1)))
    rows = []
    for t, g in df.groupby('timestep'):
        P = torch.as_tensor(np.stack(g['value'].values), dtype=torch.float32, device=device)
        rows.append({'timestep': int(t),
                     'dsvgd': dsvgd.metrics.test_accuracy(P, x_test, t_test),
                     'sklearn logreg': baseline})
    return pd.DataFrame(rows)


def make_plots(dataset, fold, nproc, nparticles, stepsize, exchange, wasserstein,
               results_dir=None, data_dir=None):
    rdir = get_results_dir(dataset, fold, nproc, nparticles, stepsize, exchange, wasserstein,
                           results_dir)
    df = load_results(rdir)
    x_train, t_train, x_test, t_test = load_dataset(dataset, fold, data_dir)
    acc = test_accuracy_curve(df, x_train, t_train, x_test, t_test)
    acc.to_csv(os.path.join(rdir, 'test_acc.csv'), index=False)
    return acc


def _init_distributed(rank, nproc, port, args):
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ['MASTER_PORT'] = str(port)
    backend = 'nccl' if torch.cuda.device_count() >= nproc else 'gloo'
    kw = {}
    if backend == 'nccl':
        kw['device_id'] = torch.device('cuda', rank)
    dist.init_process_group(backend, rank=rank, world_size=nproc, **kw)
    try:
        run(rank, nproc, *args)
    finally:
        dist.destroy_process_group()


@click.command()
@click.option('--dataset', type=click.Choice(DATASETS), default='banana')
@click.option('--fold', type=int, default=42)
@click.option('--nproc', type=click.IntRange(0, 32), default=1)
@click.option('--nparticles', type=int, default=10)
@click.option('--niter', type=int, default=100)
@click.option('--stepsize', type=float, default=1e-3)
@click.option('--exchange', type=click.Choice(['partitions', 'all_particles', 'all_scores']
                                               + sorted(LAGGED)),
              default='partitions')
@click.option('--wasserstein/--no-wasserstein', default=False)
@click.option('--master_addr', default='127.0.0.1', type=str)
@click.option('--master_port', default=29500, type=int)
@click.option('--plots/--no-plots', default=True)
@click.option('--order', type=click.Choice(['sequential', 'jacobi']), default='sequential',
              help='sequential = the reference Gauss-Seidel sweep; jacobi = the MFMA fast path')
@click.option('--results-dir', default=None, help='default: $DSVGD_RESULTS_DIR or ./results')
@click.option('--data-dir', default=None, help='directory holding benchmarks.mat')
def cli(dataset, fold, nproc, nparticles, niter, stepsize, exchange, wasserstein, master_addr,
        master_port, plots, order, results_dir, data_dir):
    """logreg.py:96-140: clean the results directory, run the ranks, plot."""
    world = int(os.environ.get('WORLD_SIZE', '0'))
    if world > 0:            # launched by torchrun: this process is one rank
        rank = int(os.environ['RANK'])
        nproc = world
    rdir = get_results_dir(dataset, fold, nproc, nparticles, stepsize, exchange, wasserstein,
                           results_dir)
    if world == 0 or rank == 0:
        if os.path.isdir(rdir):
            shutil.rmtree(rdir)
        os.makedirs(rdir)
    args = (dataset, fold, nparticles, niter, stepsize, exchange, wasserstein, rdir, data_dir,
            order)
    if world > 0:
        local = int(os.environ.get('LOCAL_RANK', rank))
        backend = 'nccl' if torch.cuda.device_count() >= world else 'gloo'
        kw = {'device_id': torch.device('cuda', local)} if backend == 'nccl' else {}
        dist.init_process_group(backend, **kw)
        dist.barrier()
        run(rank, world, *args, device='cuda:%d' % (local % torch.cuda.device_count()))
        dist.barrier()
        dist.destroy_process_group()
        if rank != 0:
            return
    elif nproc == 1:
        run(0, 1, *args)
    else:
        os.environ['MASTER_ADDR'] = master_addr
        torch.multiprocessing.spawn(_init_distributed, args=(nproc, master_port, args),
                                    nprocs=nproc, join=True)
    if plots:
        acc = make_plots(dataset, fold, nproc, nparticles, stepsize, exchange, wasserstein,
                         results_dir, data_dir)
        print(acc.tail(1).to_string(index=False))


if __name__ == "__main__":
    cli()
