"""ctypes wrapper of oracle/_build/libkbuild_cpu.so (threaded C K-assembly restatement).

TEST INFRASTRUCTURE ONLY: used by tests/ and by bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import gpr_oracle as O

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libkbuild_cpu.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(_LIB)
        D = ctypes.POINTER(ctypes.c_double)
        _lib.kbuild_cpu.argtypes = [ctypes.c_int, ctypes.c_int, D, ctypes.c_int, D, ctypes.c_int,
                                    D, D, ctypes.c_int, ctypes.c_double, ctypes.c_double, D]
        _lib.kbuild_cpu.restype = None
        I = ctypes.POINTER(ctypes.c_int)
        _lib.mll_grad_cpu.argtypes = [ctypes.c_int, ctypes.c_int, D, ctypes.c_int, I, D, D, D,
                                      ctypes.c_double, D, D, D, D, D]
        _lib.mll_grad_cpu.restype = None
    return _lib


def kbuild_cpu(kinds, hp, x, xp=None, eps=O.EPS_DEFAULT) -> np.ndarray:
    """Same result as oracle.gpr_oracle.kernel(kinds, hp, x, xp, eps), OpenMP-threaded."""
    lib = _load()
    d, n = x.shape
    hps = O.split_hp(kinds, np.asarray(hp, dtype=np.float64), d)
    se = [h for k, h in zip(kinds, hps) if k == O.SE]
    wn = [h for k, h in zip(kinds, hps) if k == O.WN]
    sig = np.array([h[0] for h in se], dtype=np.float64)
    ls = np.ascontiguousarray(np.stack([h[1:] for h in se]), dtype=np.float64)
    xc = np.ascontiguousarray(x.T)  # column-major d x n
    m = n if xp is None else xp.shape[1]
    K = np.empty((m, n), dtype=np.float64)  # row-major (m, n) == column-major n x m
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    xpc = None if xp is None else np.ascontiguousarray(xp.T)
    lib.kbuild_cpu(d, n, P(xc), m, None if xp is None else P(xpc), len(se), P(sig), P(ls),
                   1 if (wn and xp is None) else 0, float(wn[0][0] ** 2) if wn else 0.0, eps,
                   P(K))
    return K.T


def part_kernels_cpu(kinds, hp, x, eps=O.EPS_DEFAULT):
    """kernels!(kerns, covar, hp, x) (src/compose_covar.jl:80-107): one n x n matrix per SE
    part (eps on its diagonal), stacked (nse, n, n) -- each column-major n x n."""
    d = x.shape[0]
    hps = O.split_hp(kinds, np.asarray(hp, dtype=np.float64), d)
    se = [h for k, h in zip(kinds, hps) if k == O.SE]
    out = np.empty((len(se), x.shape[1], x.shape[1]))
    for p, h in enumerate(se):
        out[p] = kbuild_cpu([O.SE], h, x, None, eps).T  # (transpose of a symmetric matrix)
    return out


def mll_grad_cpu(kinds, hp, x, alpha, Kinv, Kp=None, eps=O.EPS_DEFAULT) -> np.ndarray:
    """grad!(dL, MLL, md, tc) (src/cost.jl:119-126) by the threaded C restatement of the
    reference's per-component loop (oracle/mll_grad_cpu.c: materialise dK_i, dgemv, Frobenius
    dot, for each of the D components).  Kp: the per-part matrices (part_kernels_cpu), built
    here if not given.  Same values as O.mll_grad's loop (tests/test_oracle.py)."""
    lib = _load()
    d, n = x.shape
    hp = np.asarray(hp, dtype=np.float64)
    hps = O.split_hp(kinds, hp, d)
    se = [h for k, h in zip(kinds, hps) if k == O.SE]
    wn = [h for k, h in zip(kinds, hps) if k == O.WN]
    if Kp is None:
        Kp = part_kernels_cpu(kinds, hp, x, eps)
    Kp = np.ascontiguousarray(Kp)
    sig = np.array([h[0] for h in se], dtype=np.float64)
    ls = np.ascontiguousarray(np.stack([h[1:] for h in se]), dtype=np.float64)
    pk = (ctypes.c_int * len(kinds))(*[1 if k == O.SE else 2 for k in kinds])
    xc = np.ascontiguousarray(x.T)
    al = np.ascontiguousarray(alpha, dtype=np.float64)
    Ki = np.asfortranarray(Kinv)
    dK = np.empty((n, n))
    tt = np.empty(n)
    g = np.empty(len(hp))
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    lib.mll_grad_cpu(d, n, P(xc), len(kinds), pk, P(Kp), P(sig), P(ls),
                     float(wn[0][0]) if wn else 0.0, P(al), P(Ki), P(dK), P(tt), P(g))
    return g


def fit_upper_inplace(kinds, hp, x, y, eps=O.EPS_DEFAULT, backend="scipy"):
    """update_cache!(pc, md) (src/predict.jl:29-34) at sizes where the NumPy restatement's
    temporaries do not fit in host memory (N = 32768: K alone is 8.6 GB): K by the threaded C
    restatement above, dpotrf('U') in place on it (LAPACK, like cholesky!(Hermitian(K)) --
    the strict lower triangle keeps K), wt = K^{-1} y by the oracle's own cho_solve_upper.
    Returns (U buffer, wt).  tests/test_oracle.py checks it against O.chol_upper /
    O.cho_solve_upper at small N.

    backend "scipy": LAPACK dpotrf of SciPy's bundled OpenBLAS.  backend "mkl": the
    dpotrf of torch's CPU build (MKL LAPACK; torch is host plumbing here).  SciPy's
    scipy-openblas 0.3.28 returns info = 16545 for the positive definite C3 matrix
    (SE+SE+WN, N = 32768; N = 24576 factors fine), so the full-size fixtures use "mkl" and
    verify every result by residuals (tests/golden/make_fullsize.py)."""
    import scipy.linalg as sla

    K = kbuild_cpu(kinds, hp, x, None, eps)         # Fortran-ordered n x n
    if backend == "mkl":
        import torch

        U, info = torch.linalg.cholesky_ex(torch.from_numpy(K.T), upper=True)  # K symmetric
        info = int(info)
        U = U.numpy()  # row-major: U[i, j] = U_ij, strict lower triangle zero
        del K
    else:
        U, info = sla.lapack.dpotrf(K, lower=0, clean=0, overwrite_a=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dpotrf info={info}")
    return U, O.cho_solve_upper(U, y)
