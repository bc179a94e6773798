"""Generate the full-size oracle fixtures (BASELINE.json configs C2-C5) for the GPU parity tests.

Test infrastructure: run ONCE in the build container (8 CPUs, ~64 GB), never on the GPU box:

    python tests/golden/make_fullsize.py            # all configs, ~10-15 min
    python tests/golden/make_fullsize.py C2 C4      # a subset

Inputs are exactly the benches' seeded synthetic data (bench.py, bench_mll.py,
bench_split.py): x = U[0,1)^(d x N) from default_rng(0), test points from default_rng(1), split
grid xe / xq from default_rng(2) / default_rng(3), y = sin(sum_k x_k)^2, hp sigma = 1,
l = 3 sqrt(8/d), sigma_n = 0.1.  The GPU tests regenerate the inputs from the same seeds (cheap)
and check the recorded input checksums, so only compact outputs are stored (< 1 MB total).

What computes the expected values (all in oracle/, each function citing the reference):
  C2  O.predict (the NumPy restatement itself; N = 8192 fits in memory).
  C3  fit by oracle.cpu_kbuild.fit_upper_inplace (C K-build restatement + LAPACK dpotrf in place
      + O.cho_solve_upper: the NumPy K-build's temporaries at N = 32768 exceed host memory; the
      lean fit is pinned to O.chol_upper/O.cho_solve_upper by tests/test_oracle.py), then
      O.predict_from_factor (the restated predict!, src/predict.jl:36-101).
  C4  O.mll and O.kernel_grad + O.mll_grad_parts (src/cost.jl:83-126, src/loss_grad.jl:39-52,
      src/deriv_covar.jl:20-32) per component, both terms kept so the test can scale its
      tolerance to the cancellation in -0.5 (a'dKa - <K^-1, dK>).
  C5  fit as C3, then O.split_predict_from_factor (src/split_predict.jl:5-53) with the default
      var_range 1:3; the mean is stored on every 32nd grid row.
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np
import scipy.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gpr_oracle as O  # noqa: E402
from oracle.cpu_kbuild import fit_upper_inplace, kbuild_cpu  # noqa: E402

SE, WN = O.SE, O.WN

CONFIGS = {
    # name: kinds, N, d, np (or the split grid)
    "C2": dict(kinds=[SE], n=8192, d=8, np=8192),
    "C3": dict(kinds=[SE, SE, WN], n=32768, d=8, np=8192),
    "C4": dict(kinds=[SE, WN], n=16384, d=16),
    "C5": dict(kinds=[SE, WN], n=32768, d=8, ne=1024, nq=1024, var_range=(1, 3), row_step=32),
}


def inputs(cfg):
    """The benches' seeded inputs for one config (shared with the GPU tests)."""
    d, n = cfg["d"], cfg["n"]
    x = np.random.default_rng(0).random((d, n))
    y = np.sin(x.sum(0)) ** 2
    out = dict(x=x, y=y, hp=O.default_hp(cfg["kinds"], d))
    if "np" in cfg:
        out["xp"] = np.random.default_rng(1).random((d, cfg["np"]))
    if "ne" in cfg:
        out["xe"] = np.random.default_rng(2).random((d, cfg["ne"]))
        out["xq"] = np.random.default_rng(3).random((d, cfg["nq"]))
    return out


def checksum(arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def fixture_path(name: str) -> str:
    return os.path.join(HERE, f"fullsize_{name}.npz")


def make_c2(cfg, inp):
    mu, var = O.predict(cfg["kinds"], inp["hp"], inp["x"], inp["y"], inp["xp"], diagonal_var=True)
    K = O.kernel(cfg["kinds"], inp["hp"], inp["x"])
    U = O.chol_upper(K)
    alpha = O.cho_solve_upper(U, inp["y"])
    return dict(mu=mu, var=var, alpha=alpha, min_diag_U2=np.min(np.diag(U)) ** 2,
                mll=O.mll_value(U, inp["y"], alpha))


def verify_fit(kinds, hp, x, y, U, wt, rng):
    """Independent residual checks of a large fit with torch's CPU (MKL) BLAS: the solve
    residual ||K wt - y|| and the factor's backward error on sampled columns."""
    import torch

    K = torch.from_numpy(kbuild_cpu(kinds, hp, x).T)
    Ut = torch.from_numpy(U)
    w = torch.from_numpy(wt)
    r = float(torch.linalg.norm(K @ w - torch.from_numpy(y)))
    scale = float(torch.linalg.norm(K)) * float(torch.linalg.norm(w)) + float(np.linalg.norm(y))
    cols = torch.from_numpy(np.sort(rng.choice(len(y), 96, replace=False)))
    Ucols = torch.triu(Ut)[:, cols]
    be = float((torch.triu(Ut).T @ Ucols - K[:, cols]).abs().max())
    print(f"  verify fit: solve residual {r / scale:.2e}, factor backward error {be:.2e}")
    assert r / scale < 1e-13 and be < 1e-12


def verify_posterior(kinds, hp, x, U, wt, xp, mu, var, rng, nsample=64):
    """mu_j = k_j' wt and var_j = prior - ||U^{-T} k_j||^2 at sampled test points, with the
    triangular solve done by torch's CPU (MKL) instead of SciPy's OpenBLAS."""
    import torch

    js = np.sort(rng.choice(xp.shape[1], nsample, replace=False))
    k = O.kernel(kinds, hp, x, xp[:, js])                       # N x nsample
    v = torch.linalg.solve_triangular(torch.from_numpy(U).T, torch.from_numpy(k), upper=False)
    var_s = O.diag_prior(kinds, hp, x.shape[0]) - (v * v).sum(0).numpy()
    mu_s = k.T @ wt
    em = np.abs(mu_s - mu[js]).max() / np.abs(mu[js]).max()
    ev = np.abs(var_s - var[js]).max()
    print(f"  verify posterior at {nsample} points: mean {em:.2e} (rel), variance {ev:.2e} (abs)")
    assert em < 1e-11 and ev < 1e-11


def make_c3(cfg, inp):
    kinds, hp, x, y = cfg["kinds"], inp["hp"], inp["x"], inp["y"]
    U, wt = fit_upper_inplace(kinds, hp, x, y, backend="mkl")
    mu, var = O.predict_from_factor(kinds, hp, x, U, wt, inp["xp"], diagonal_var=True)
    rng = np.random.default_rng(99)
    verify_posterior(kinds, hp, x, U, wt, inp["xp"], mu, var, rng)
    verify_fit(kinds, hp, x, y, U, wt, rng)
    dU = np.diag(U).copy()
    # loss(MLL, kchol, y, alpha) (src/loss_grad.jl:39-41) as O.mll_value, from diag(U) alone
    mll = 0.5 * (float(np.dot(y, wt)) + 2.0 * float(np.sum(np.log(dU))) + len(dU) * O.LOG2PI)
    return dict(mu=mu, var=var, alpha=wt, min_diag_U2=dU.min() ** 2, mll=mll)


def make_c4(cfg, inp):
    kinds, hp, x, y = cfg["kinds"], inp["hp"], inp["x"], inp["y"]
    K = O.kernel(kinds, hp, x)
    U = O.chol_upper(K)
    del K
    alpha = O.cho_solve_upper(U, y)
    mll = O.mll_value(U, y, alpha)
    # K^{-1} = ldiv!(kchol, I) (src/cost.jl:90-92); LAPACK dpotri gives the same matrix without
    # the N x N identity and second triangular solve's temporaries
    Kinv, info = sla.lapack.dpotri(U, lower=0)
    assert info == 0
    Kinv = np.triu(Kinv) + np.triu(Kinv, 1).T
    dmin = np.min(np.diag(U)) ** 2
    del U
    D = len(hp)
    p1, p2 = np.empty(D), np.empty(D)
    for i in range(1, D + 1):
        t = time.time()
        p1[i - 1], p2[i - 1] = O.mll_grad_parts(O.kernel_grad(kinds, i, hp, x), alpha, Kinv)
        print(f"  C4 grad component {i}/{D}: {time.time() - t:.1f} s", flush=True)
    grad = -0.5 * (p1 - p2)
    return dict(mll=mll, grad=grad, grad_p1=p1, grad_p2=p2, alpha=alpha, min_diag_U2=dmin)


def make_c5(cfg, inp):
    kinds, hp, x, y = cfg["kinds"], inp["hp"], inp["x"], inp["y"]
    U, wt = fit_upper_inplace(kinds, hp, x, y, backend="mkl")
    rows = np.arange(0, cfg["ne"], cfg["row_step"])
    mu_rows, var = O.split_predict_from_factor(kinds, hp, x, U, wt, inp["xe"], inp["xq"],
                                               var_range=cfg["var_range"], mean_rows=rows)
    lo, hi = cfg["var_range"]
    nq = cfg["nq"]
    # the split identity (test/test_split_kernel.jl:29-31): the split mean / variance equal the
    # direct posterior at the grid points x_eq = xe_e + xq_q, checked on sampled points
    rng = np.random.default_rng(98)
    e_s = np.r_[rows[rng.choice(len(rows), 4, replace=False)]]
    pts = (inp["xe"][:, e_s, None] + inp["xq"][:, None, :]).reshape(x.shape[0], -1)
    mu_d = O.kernel(kinds, hp, pts, x) @ wt
    idx = np.searchsorted(rows, e_s)
    em = np.abs(mu_d.reshape(len(e_s), nq) - mu_rows[idx]).max() / np.abs(mu_rows).max()
    print(f"  verify split mean vs direct posterior on 4 rows: {em:.2e} (rel)")
    assert em < 1e-9
    # grid row e, column q -> variance index (e - 1) nq + q (q fastest within e)
    ev_pts = (inp["xe"][:, lo - 1:hi, None] + inp["xq"][:, None, :]).reshape(x.shape[0], -1)
    js = np.sort(rng.choice(ev_pts.shape[1], 48, replace=False))
    import torch
    k = O.kernel(kinds, hp, x, ev_pts[:, js])
    v = torch.linalg.solve_triangular(torch.from_numpy(U).T, torch.from_numpy(k), upper=False)
    var_s = O.diag_prior(kinds, hp, x.shape[0]) - (v * v).sum(0).numpy()
    evv = np.abs(var_s - var[(lo - 1) * nq:hi * nq][js]).max()
    print(f"  verify split variance vs direct posterior at 48 points: {evv:.2e} (abs)")
    assert evv < 1e-9
    verify_fit(kinds, hp, x, y, U, wt, rng)
    return dict(mu_rows=mu_rows, rows=rows, var_head=var[(lo - 1) * nq:hi * nq], alpha=wt,
                min_diag_U2=np.min(np.diag(U)) ** 2)


MAKERS = {"C2": make_c2, "C3": make_c3, "C4": make_c4, "C5": make_c5}


def main(names):
    for name in names:
        cfg = CONFIGS[name]
        inp = inputs(cfg)
        t = time.time()
        out = MAKERS[name](cfg, inp)
        keys = [k for k in ("x", "y", "xp", "xe", "xq") if k in inp]
        out["input_sha256"] = checksum([inp[k] for k in keys])
        out["hp"] = inp["hp"]
        np.savez_compressed(fixture_path(name), **out)
        print(f"{name}: {time.time() - t:.1f} s -> {fixture_path(name)} "
              f"({os.path.getsize(fixture_path(name)) / 1e3:.0f} kB)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS))
