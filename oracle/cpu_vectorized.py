"""CPU BASELINE (bench infrastructure only): vectorised torch-CPU restatement
of one Jacobi SVGD phi (the survey's "vectorised torch-CPU" baseline,
BASELINE.md section 2), chunked over rows so the n x n kernel matrix is never
materialised whole.  Timed by bench.py's cpu_baseline leg; never shipped."""
import time

import torch


def phi_rows(X, S, h, r0, r1):
    """phi for rows [r0, r1) of X (n, d) fp32 against all n (fixed h)."""
    Xr = X[r0:r1]
    D = torch.cdist(Xr, X) ** 2
    K = torch.exp(-D / h)
    rep = (2.0 / h) * (K.sum(1, keepdim=True) * Xr - K @ X)
    return (K @ S + rep) / X.shape[0]


def time_rows(X, S, h, rows=2048, chunk=1024, budget_s=10.0):
    """Seconds per particle update, timed on up to `rows` rows."""
    X = torch.as_tensor(X, dtype=torch.float32)
    S = torch.as_tensor(S, dtype=torch.float32)
    t0 = time.perf_counter()
    done = 0
    while done < rows and time.perf_counter() - t0 < budget_s:
        phi_rows(X, S, h, done, min(done + chunk, X.shape[0]))
        done = min(done + chunk, X.shape[0])
    return (time.perf_counter() - t0) / done, done
