"""Accuracy / speed probe of the block-Jacobi eigensolver (gpr_syev_apply, csrc/eigen.hip).

For each matrix: eigenvalue error max|lam - eigvalsh| / (n eps ||A||_2), orthogonality of the
applied transform ||C^T C - I||_max with B = I (C = P^T), outer sweeps and wall time.
Run one process per environment variant (GPR_EIG_* are read once per process):
    python tools/eig_probe.py            (GPR_EIG_INNER etc. from the environment)
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
sys.path.insert(0, ROOT)

import gpr_amd as G  # noqa: E402
from oracle import gpr_oracle as O  # noqa: E402


def run(ctx, A, label):
    n = A.shape[0]
    dA, dB = ctx.colmajor(A), ctx.colmajor(np.eye(n))
    lam = ctx.empty(n)
    sw = ctypes.c_int(-1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ctx.sync()
    t0 = time.perf_counter()
    rc = G._lib.lib.gpr_syev_apply(ctx.h, P(dA), n, n, P(dB), n, n, P(lam), ctypes.byref(sw))
    ctx.sync()
    dt = time.perf_counter() - t0
    if rc:
        print(f"{label:28s} n={n:5d} rc={rc} {G._lib.lib.gpr_last_error(ctx.h)}")
        return
    lm, C = ctx.host(lam), ctx.host(dB)
    ref = np.linalg.eigvalsh(A)
    nrm = np.abs(ref).max()
    eps = np.finfo(float).eps
    e_lam = np.abs(np.sort(lm) - ref).max() / (n * eps * nrm)
    e_orth = np.abs(C.T @ C - np.eye(n)).max() / eps
    resid = np.abs(C.T @ np.diag(lm) @ C - A).max() / (nrm * eps)
    print(f"{label:28s} n={n:5d} sweeps={sw.value:3d} {dt * 1e3:9.1f} ms  "
          f"eig err {e_lam:7.2f} n eps|A|  orth {e_orth:8.1f} eps  resid {resid:8.1f} eps|A|")


def main():
    ctx = G.Context(0)
    env = {k: v for k, v in os.environ.items() if k.startswith("GPR_EIG")}
    print("env", env)
    for n in (64, 129, 300, 511, 1100):
        rng = np.random.default_rng(n)
        X = rng.standard_normal((n, n))
        run(ctx, (X + X.T) / 2, "random symmetric")
    for dim, n in ((2, 150), (4, 1100), (1, 300)):
        rng = np.random.default_rng(dim * n)
        x = rng.random((dim, n))
        K = O.kernel([O.SE], O.default_hp([O.SE], dim, length=2.0), x)
        run(ctx, K, f"SE kernel d={dim}")
    n = 2048
    X = np.random.default_rng(5).standard_normal((n, n))
    run(ctx, (X + X.T) / 2, "random symmetric")


if __name__ == "__main__":
    main()
