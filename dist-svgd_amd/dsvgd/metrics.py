"""Posterior-predictive test accuracy of the logistic-regression experiment
(reference: experiments/logreg_plots.py:42-50, `_test_acc`), on the GPU.

    acc = mean_q[ (mean_j sigma(xt_q . w_j) > 0.5) == (t_q > 0) ]

over the particles x_j = [log alpha, w_j] (no bias; alpha unused, as the
reference).  The ensemble mean runs in `dsvgd_logreg_predict` (NT MFMA tiles
+ a fixed-order reduction over particle blocks); the reference evaluates it
in fp64 with numpy, this in fp32, so a test point whose mean probability is
within ~1e-6 of 0.5 may land on the other side.
"""
import torch

from . import _native as N


def _device_f32(a, dev):
    t = torch.as_tensor(a)
    if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
        t = t.to(device=dev, dtype=torch.float32).contiguous()
    return t


def predictive_prob(particles, x_test):
    """(Nt,) device tensor: mean over particles of sigma(x_test . w)."""
    X = particles
    dev = N.require_gpu(X.device if X.is_cuda else "cuda")
    X = _device_f32(X, dev)
    n, d = X.shape
    xt = _device_f32(x_test, dev).reshape(-1, d - 1)
    Nt = xt.shape[0]
    nbytes = N.load().dsvgd_logreg_predict_workspace_bytes(n, Nt, d - 1)
    ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
    aligned = (ws.data_ptr() + 255) // 256 * 256
    prob = torch.empty(Nt, dtype=torch.float32, device=dev)
    N.call("dsvgd_logreg_predict", N.ptr(X), N.ld(X), n, d, N.ptr(xt), N.ld(xt), Nt,
           N.ptr(prob), aligned, N.stream(dev))
    return prob


def test_accuracy(particles, x_test, t_test):
    """Fraction of test points whose ensemble-mean probability > 0.5 agrees
    with t_test > 0 (logreg_plots.py:42-50)."""
    prob = predictive_prob(particles, x_test)
    t = _device_f32(t_test, prob.device).reshape(-1)
    return int(((prob > 0.5) == (t > 0)).sum()) / prob.numel()
