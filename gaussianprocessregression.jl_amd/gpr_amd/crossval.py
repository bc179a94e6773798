"""Cross-validation, mirroring src/crossval.jl and the M-estimator
losses of src/loss_grad.jl:5-30: ``kfoldcv``, ``cv_batch``, ``cv_step``, ``cv_step_`` with the
costs ``MSE``, ``ChiSq`` and ``Mahalanobis``.

Every fold runs on the device in ONE C call (``gpr_cv_batch``): gather the fold's training
and test points from the resident (x, y), fit (K, POTRF, wt), full-covariance posterior at
the test points (the TRSM + SYRK of predict!), and the loss -- for Mahalanobis a second
POTRF of Sigma_p and a forward sweep.  Only the fold losses come back to the host.

Indices are 0-based (Python), where the reference's ``cvset`` holds 1-based Julia indices.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import core as C
from ._lib import GPR_COST_CHISQ, GPR_COST_MAHALANOBIS, GPR_COST_MSE, lib


class MSE:
    """loss(::MSE, y, yp, Sigma_p) = sum((y - yp)^2) / length(y) (src/loss_grad.jl:12-15)."""
    COST = GPR_COST_MSE


class ChiSq:
    """loss(::ChiSq, y, yp, Sigma_p) = sum((y - yp)^2 / Sigma_p[i, i]) (src/loss_grad.jl:17-23)."""
    COST = GPR_COST_CHISQ


class Mahalanobis:
    """loss(::Mahalanobis, y, yp, Sigma_p) = ||L^{-1}(y - yp)||^2 with Sigma_p = L L^T
    (src/loss_grad.jl:25-30)."""
    COST = GPR_COST_MAHALANOBIS


def _cost_code(cost) -> int:
    code = getattr(cost, "COST", None)
    if code is None:
        raise TypeError(f"no cross-validation loss for {cost!r} (MSE, ChiSq, Mahalanobis)")
    return code


def kfoldcv(n: int, k: int, nb: Optional[int] = None, rng=None):
    """kfoldcv(n, k, nb = div(n, k)) (src/crossval.jl:1-11): shuffle 0..n-1; fold i tests the
    k shuffled indices at positions [i k, (i+1) k) and trains on all the others, in shuffled
    order.  Returns (trn, tst), lists of int arrays."""
    nb = n // k if nb is None else nb
    rng = rng if rng is not None else np.random.default_rng()
    nsh = rng.permutation(n)
    trn, tst = [], []
    for i in range(nb):
        keep = np.ones(n, dtype=bool)
        keep[i * k:(i + 1) * k] = False
        tst.append(nsh[i * k:(i + 1) * k].copy())
        trn.append(nsh[keep])
    return trn, tst


def _fold_matrix(folds: Sequence, what: str) -> np.ndarray:
    a = np.asarray([np.asarray(f, dtype=np.int64) for f in folds])
    if a.ndim != 2:
        raise ValueError(f"all {what} folds must have the same length")
    return np.ascontiguousarray(a, dtype=np.int32)


def _cv(md: C.GPRModel, cost, dx, dy, n: int, trn: np.ndarray, tst: np.ndarray,
        eps: float) -> np.ndarray:
    ctx = md.ctx
    kinds, nk = C._kinds_arr(md.covar)
    hpa, hpp = C._hp_arr(md.params)
    nfold, ntrn = trn.shape
    ntst = tst.shape[1]
    if tst.shape[0] != nfold:
        raise ValueError("trn and tst must hold the same number of folds")
    lss = np.zeros(nfold)
    ip = ctypes.POINTER(ctypes.c_int)
    rc = lib.gpr_cv_batch(ctx.h, kinds, nk, hpp, md.d, C._ptr(dx), n, C._ptr(dy),
                          trn.ctypes.data_as(ip), ntrn, tst.ctypes.data_as(ip), ntst, nfold,
                          _cost_code(cost), eps,
                          lss.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc > 0:
        raise C.PosDefException(rc)
    ctx.check(rc, "gpr_cv_batch")
    return lss


def cv_batch(md: C.GPRModel, cost, x, y, cvset, eps: float = C.EPS_DEFAULT) -> np.ndarray:
    """cv_batch(md, cost, x, y, (trn, tst)) (src/crossval.jl:13-35): for every fold, a model
    with md's kernel and hyperparameters fitted on x[:, trn[i]], y[trn[i]] predicts
    x[:, tst[i]] with the full covariance; returns the fold losses."""
    x = np.asarray(x, dtype=np.float64)
    x = x[None, :] if x.ndim == 1 else x
    y = np.asarray(y, dtype=np.float64)
    if y.ndim != 1 or x.shape[1] != y.shape[0]:
        raise ValueError("x and y size mismatch.")
    if x.shape[0] != md.d:
        raise ValueError("x dimension does not match the model")
    trn, tst = cvset
    return _cv(md, cost, md.ctx.colmajor(x), md.ctx.colmajor(y), y.shape[0],
               _fold_matrix(trn, "trn"), _fold_matrix(tst, "tst"), eps)


def cv_step(md: C.GPRModel, cost, xtr, ytr, xtst, ytst, eps: float = C.EPS_DEFAULT) -> float:
    """cv_step(md, cost, xtr, ytr, xtst, ytst) (src/crossval.jl:37-44)."""
    xtr, xtst = (np.asarray(a, dtype=np.float64) for a in (xtr, xtst))
    xtr = xtr[None, :] if xtr.ndim == 1 else xtr
    xtst = xtst[None, :] if xtst.ndim == 1 else xtst
    ntr, nts = xtr.shape[1], xtst.shape[1]
    x = np.concatenate([xtr, xtst], axis=1)
    y = np.concatenate([np.asarray(ytr, dtype=np.float64), np.asarray(ytst, dtype=np.float64)])
    cvset = ([np.arange(ntr)], [np.arange(ntr, ntr + nts)])
    return float(cv_batch(md, cost, x, y, cvset, eps)[0])


def cv_step_(cost, mdt: C.GPRModel, xtst, ytst, pc=None, yp=None, Sigma=None,
             eps: float = C.EPS_DEFAULT) -> float:
    """cv_step!(cost, mdt, xtst, ytst, pc, yp, Sigma_p) (src/crossval.jl:46-51): fit mdt,
    predict xtst with the full covariance, loss.  The predict cache and the yp / Sigma_p
    buffers live inside the device call (pc, yp, Sigma are accepted for signature parity)."""
    return cv_step(mdt, cost, mdt.x, C.get_sample(mdt), xtst, ytst, eps)
