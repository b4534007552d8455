"""The logreg experiment harness (dist-svgd_amd/experiments/logreg.py; §8 f2/f3):
result-directory naming and shard-pickle schema of the reference
(experiments/logreg.py:74-92, logreg_plots.py:19-22,107) on CPU; on the GPU a
short run whose shard pickles and per-timestep test accuracy match the CPU
oracle (Gauss-Seidel, partitions, S = 1)."""
import importlib.util
import os

import numpy as np
import pandas as pd
import pytest
import torch

from conftest import PKG, record_parity
from oracle import svgd_oracle as O


def harness():
    spec = importlib.util.spec_from_file_location(
        "dsvgd_logreg_experiment", os.path.join(PKG, "experiments", "logreg.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_results_dir_naming_matches_reference():
    H = harness()
    got = H.get_results_dir('banana', 42, 8, 50, 3e-3, 'all_scores', False, results_dir='/r')
    assert got == ('/r/logreg_banana_42-nshards=8-nparticles=50-exchange=all_scores-'
                   'wasserstein=False-stepsize=3e-03')


def test_synthetic_dataset_and_loader_fallback(tmp_path):
    H = harness()
    x, t, xt, tt = H.load_dataset('banana', 42, str(tmp_path))   # no benchmarks.mat there
    assert x.shape == (400, 2) and xt.shape == (4900, 2)
    assert t.shape == (400, 1) and set(np.unique(t)) <= {-1.0, 1.0}
    # a git-LFS pointer file is not a dataset either
    (tmp_path / 'benchmarks.mat').write_text('version https://git-lfs.github.com/spec/v1\n')
    x2 = H.load_dataset('banana', 42, str(tmp_path))[0]
    assert np.array_equal(x, x2)


def test_load_results_concatenates_shards(tmp_path):
    H = harness()
    for r in range(2):
        pd.DataFrame({'timestep': [0, 0, 1, 1],
                      'value': [np.full(3, r, np.float32)] * 4}).to_pickle(
            str(tmp_path / ('shard-%d.pkl' % r)))
    df = H.load_results(str(tmp_path))
    assert list(df.columns) == ['timestep', 'value'] and len(df) == 8
    assert sorted(df.groupby('timestep').size().tolist()) == [4, 4]


def test_cli_help():
    from click.testing import CliRunner
    res = CliRunner().invoke(harness().cli, ['--help'])
    assert res.exit_code == 0
    for opt in ('--nparticles', '--niter', '--stepsize', '--exchange', '--wasserstein', '--order'):
        assert opt in res.output


@pytest.mark.gpu
def test_harness_run_matches_oracle(tmp_path):
    """n = 50, T = 20, eps = 3e-3 (notes.md timing configuration, shortened):
    every timestep's particles in shard-0.pkl vs the oracle's Gauss-Seidel
    trajectory, and the GPU test-accuracy curve vs the fp64 restatement."""
    H = harness()
    n, T, eps = 50, 20, 3e-3
    rdir = str(tmp_path)
    H.run(0, 1, 'banana', 42, n, T, eps, 'partitions', False, rdir, None, 'sequential', 'cuda:0')
    df = H.load_results(rdir)
    assert list(df.columns) == ['timestep', 'value'] and len(df) == n * (T + 1)
    x, t, xt, tt = H.synthetic_banana()
    X0 = O.ref_init(n, 3, 0)
    fn = lambda X: O.score_logreg(X, x, t.reshape(-1))  # noqa: E731
    D = O.DistOracle([X0], [fn], 400, 400, False, False, sequential=True)
    traj = [X0.astype(np.float64)]
    for _ in range(T):
        D.step(eps, 10.0)
        traj.append(D.own(0).copy())
    worst = 0.0
    for step, g in df.groupby('timestep'):
        got = np.stack(g['value'].values).astype(np.float64)
        worst = max(worst, float(np.abs(got - traj[step]).max()))
    record_parity(worst)
    assert worst < 1e-4
    acc = H.test_accuracy_curve(df, x, t, xt, tt)
    ref = [O.test_accuracy(traj[s], xt, tt) for s in range(T + 1)]
    assert np.abs(acc['dsvgd'].values - np.array(ref)).max() <= 1.0 / len(tt) + 1e-12
    assert 0.5 < acc['sklearn logreg'].iloc[0] <= 1.0
