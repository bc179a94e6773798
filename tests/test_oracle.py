"""CPU: pin the oracle against every known-answer / identity test of the reference suite.

The reference (Julia) cannot run here and ships no golden data, so these are the
anchors: closed forms, algebraic identities, finite differences and a 50-digit mpmath
recomputation.  File:line of the reference test each one restates is in its docstring.
"""
import math

import mpmath
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import gpr_oracle as O

SE, WN = O.SE, O.WN


@pytest.mark.parametrize("n", [10, 20, 100])
def test_mll_closed_form_diagonal(n):
    """test/test_loss.jl:1-11."""
    rng = np.random.default_rng(n)
    x, y = rng.random(n) + 0.05, rng.random(n)
    K = np.diag(x)
    U = O.chol_upper(K)
    wt = O.cho_solve_upper(U, y)
    MLE = 0.5 * (np.dot(y, y / x) + np.sum(np.log(x)) + n * math.log(2 * math.pi))
    assert O.mll_value(U, y, wt) == pytest.approx(MLE, rel=1e-14)


@pytest.mark.parametrize("n,dim", [(10, 2), (20, 5), (100, 2)])
def test_grad_identity_dK_equals_K(n, dim):
    """test/test_loss.jl:32: grad(ll, kchol, K, y, inv(K), y) = -0.5 (tr(y y' K) - n)."""
    rng = np.random.default_rng(n * dim)
    x = rng.random((dim, n))
    y = np.sum(np.sin(x), axis=0)
    hp = rng.random(dim + 1) + 0.5
    K = O.kernel([SE], hp, x) + 1e-3 * np.eye(n)
    Kinv = np.linalg.inv(K)
    g = O.mll_grad_term(K, y, Kinv)
    assert g == pytest.approx(-0.5 * (np.trace(np.outer(y, y) @ K) - n), rel=1e-5)


@pytest.mark.parametrize("n,dim", [(10, 2), (20, 5), (100, 2), (100, 5)])
def test_cache_contents_and_fd_grads(n, dim):
    """test/test_loss.jl:22-56: loss identity, cache (U, alpha, K^-1) vs fresh
    cholesky / inv, per-hp gradient vs forward FD (eps 1e-6, rtol 1e-3)."""
    rng = np.random.default_rng(7 * n + dim)
    x = rng.random((dim, n))
    y = np.sum(np.sin(x), axis=0)
    kinds = [SE, WN]
    hp = rng.random(dim + 2) + 0.3
    K = O.kernel(kinds, hp, x)
    U = O.chol_upper(K)
    np.testing.assert_allclose(U.T @ U, K, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(O.cho_solve_upper(U, y), np.linalg.solve(K, y), rtol=1e-8)
    np.testing.assert_allclose(O.kinv_from_upper(U), np.linalg.inv(K), rtol=1e-8, atol=1e-10)
    g = O.mll_grad(kinds, hp, x, y)
    for i in range(len(hp)):
        hpe = hp.copy()
        hpe[i] += 1e-6
        fd = (O.mll(kinds, hpe, x, y) - O.mll(kinds, hp, x, y)) / 1e-6
        assert g[i] == pytest.approx(fd, rel=1e-3, abs=1e-6)


def test_kernel_grad_fd_and_compose_mapping():
    """test/test_covariance.jl:3-9,84-105."""
    rng = np.random.default_rng(1)
    dim, n = 2, 100
    x = rng.random((dim, n))
    hp = rng.random(dim + 1)
    for i in range(1, dim + 2):
        hpe = hp.copy()
        hpe[i - 1] += 1e-7
        fd = (O.kernel([SE], hpe, x) - O.kernel([SE], hp, x)) / 1e-7
        np.testing.assert_allclose(O.kernel_grad([SE], i, hp, x), fd, atol=1e-3)
    kinds = [SE, WN, SE]
    hp = rng.random(2 * dim + 3)
    hps = O.split_hp(kinds, hp, dim)
    for i in range(1, 4):
        np.testing.assert_allclose(O.kernel_grad(kinds, i, hp, x), O.kernel_grad([SE], i, hps[0], x))
    assert O.kernel_grad(kinds, 4, hp, x) == ("I", 2 * hps[1][0])
    for i in range(5, 8):
        np.testing.assert_allclose(O.kernel_grad(kinds, i, hp, x),
                                   O.kernel_grad([SE], i - 4, hps[2], x))


def test_compose_identities():
    """test/test_covariance.jl:34-81."""
    rng = np.random.default_rng(2)
    dim, n = 3, 50
    x, xp = rng.random((dim, n)), rng.random((dim, 2 * n))
    hps = rng.random(dim + 2)
    np.testing.assert_allclose(O.kernel([SE, WN], hps, x),
                               O.kernel([SE], hps[:-1], x) + hps[-1] ** 2 * np.eye(n))
    np.testing.assert_allclose(O.kernel([SE, WN], hps, x, xp), O.kernel([SE], hps[:-1], x, xp))
    hps = rng.random(dim + 2)
    np.testing.assert_allclose(O.kernel([WN, SE], hps, x),
                               O.kernel([SE], hps[1:], x) + hps[0] ** 2 * np.eye(n))
    hps = rng.random(2 * dim + 3)
    np.testing.assert_allclose(
        O.kernel([SE, WN, SE], hps, x),
        O.kernel([SE], hps[:dim + 1], x) + O.kernel([SE], hps[dim + 2:], x) + hps[dim + 1] ** 2 * np.eye(n))


def test_same_object_kernel_forms():
    """src/compose_covar.jl:47-77, src/covariance.jl:49-58: the 5-arg kernel! with x === xp
    adds eps once per SE part and NO noise; the 4-arg form adds the noise too; a different
    object (even with equal values) gets neither."""
    rng = np.random.default_rng(21)
    dim, n = 3, 40
    x = rng.random((dim, n))
    for kinds in ([SE, WN], [SE, SE, WN], [WN, SE], [SE, WN, SE], [SE, SE]):
        hp = rng.random(sum(O.dim_hp(k, dim) for k in kinds))
        hps = O.split_hp(kinds, hp, dim)
        se_sum = sum(O.se_kernel(h, x, x, True) for k, h in zip(kinds, hps) if k == SE)
        noise = sum(h[0] ** 2 for k, h in zip(kinds, hps) if k == WN)
        np.testing.assert_array_equal(O.kernel(kinds, hp, x, x), se_sum)
        np.testing.assert_allclose(O.kernel(kinds, hp, x), se_sum + noise * np.eye(n), rtol=1e-15)
        cross = O.kernel(kinds, hp, x, x.copy())
        nse = kinds.count(SE)
        np.testing.assert_allclose(np.diag(O.kernel(kinds, hp, x, x)) - np.diag(cross),
                                   nse * O.EPS_DEFAULT, rtol=1e-6)


@pytest.mark.parametrize("n", [100, 200, 500])
@pytest.mark.parametrize("npred", [100, 200, 500])
@pytest.mark.parametrize("dim", [1, 2, 5])
def test_interpolation_random_hp_verbatim(n, npred, dim):
    """test/test_models.jl:1-31 verbatim: x = rand(dim, n), y = sin(sum x)^2, and
    GPRModel(cov, x, y) draws hp = rand(D) (src/models.jl:32-37).  predict_mean(md2, x) with
    the model's OWN x takes the same-object branch (eps per SE part on Kxp), so mu = y up to
    the solve's backward error even for the ill-conditioned random hp."""
    rng = np.random.default_rng(1000 * n + 10 * npred + dim)
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    hp2 = rng.random(2 * (dim + 1))
    mu, S = O.predict([SE, SE], hp2, x, y, x)
    assert np.linalg.norm(mu - y) <= 1e-7 * max(np.linalg.norm(mu), np.linalg.norm(y))
    assert np.abs(S).max() <= 1e-7
    hp3 = rng.random(dim + 2)
    hp3[-1] = 1e-5
    mu3, S3 = O.predict([SE, WN], hp3, x, y, x)
    assert np.linalg.norm(mu3 - y) <= 1e-3 * max(np.linalg.norm(mu3), np.linalg.norm(y))
    assert np.abs(S3).max() <= 1e-3


def test_interpolation_and_diag_vs_full():
    """test/test_models.jl:34-48."""
    rng = np.random.default_rng(3)
    dim, n, npred = 2, 200, 100
    x, xp = rng.random((dim, n)), rng.random((dim, npred))
    y = np.sin(x.sum(0)) ** 2
    hp = rng.random(dim + 2) + 0.5
    _, Sf = O.predict([SE, WN], hp, x, y, xp)
    _, Sd = O.predict([SE, WN], hp, x, y, xp, diagonal_var=True)
    np.testing.assert_allclose(np.diag(Sf), Sd, atol=1e-5)


def test_split_identities():
    """test/test_split_kernel.jl:10-44: Cmap layout, distance identity, split kernel."""
    rng = np.random.default_rng(4)
    dim, n = 3, 26
    x, xe, xq = rng.random((dim, n)), rng.random((dim, n + 100)), rng.random((dim, n - 10))
    ne, nq = xe.shape[1], xq.shape[1]
    pts = O.cmap_points(xe, xq)
    for e, q in [(0, 0), (ne - 1, 0), (3, nq - 1)]:
        np.testing.assert_allclose(pts[:, e + q * ne], xe[:, e] + xq[:, q])
    DA = O.split_distance_a(xe, xq)
    DB = O.distance_euclid(xe, x)
    DC = O.split_distance_c(x, xq)
    D = O.distance_euclid(pts, x)
    full = DA[:, :, None] + DB[:, None, :] + DC.T[None, :, :]
    np.testing.assert_allclose(D, full.reshape(ne * nq, n, order="F"), rtol=1e-10, atol=1e-12)
    kinds = [SE, SE, WN]
    hp = rng.random(2 * dim + 3)
    A, B, C = O.split_factors(kinds, hp, x, xe, xq)
    KK = O.kernel(kinds, hp, pts, x)
    Ks = np.einsum("eqk,esk,sqk->eqs", A, B, C).reshape(ne * nq, n, order="F")
    np.testing.assert_allclose(Ks, KK, rtol=1e-10)


@pytest.mark.parametrize("kinds", [[SE], [SE, WN], [SE, SE], [SE, SE, WN]])
def test_split_predict_identities(kinds):
    """test/test_split_kernel.jl:49-77."""
    rng = np.random.default_rng(len(kinds))
    dim, n, e, q = 2, 200, 20, 30
    x, xe, xq = rng.random((dim, n)), rng.random((dim, e)), rng.random((dim, q))
    y = np.sin(x.sum(0)) ** 2
    hp = rng.random(sum(O.dim_hp(k, dim) for k in kinds)) * 0.5 + 0.5
    yps, varps = O.split_predict(kinds, hp, x, y, xe, xq)
    yp, _ = O.predict(kinds, hp, x, y, O.cmap_points(xe, xq), diagonal_var=True)
    np.testing.assert_allclose(yps.reshape(-1, order="F"), yp, rtol=1e-7, atol=1e-9)
    _, varpt = O.predict(kinds, hp, x, y, O.cmap_points(xq, xe), diagonal_var=True)
    np.testing.assert_allclose(varps[:3 * q], varpt[:3 * q], rtol=1e-5)
    assert not np.allclose(varps[:3 * q + 1], varpt[:3 * q + 1], rtol=1e-5)


def test_mpmath_bounds_oracle_error():
    """50-digit recomputation of K, alpha and the MLL at N=24 bounds the oracle's rounding."""
    mpmath.mp.dps = 50
    rng = np.random.default_rng(5)
    dim, n = 2, 24
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    kinds = [SE, WN]
    hp = np.array([1.0, 2.0, 1.5, 0.3])
    Kmp = mpmath.matrix(n, n)
    for a in range(n):
        for b in range(n):
            D = sum((mpmath.mpf(hp[1 + k]) * x[k, a] - mpmath.mpf(hp[1 + k]) * x[k, b]) ** 2
                    for k in range(dim))
            v = mpmath.mpf(hp[0]) ** 2 * mpmath.exp(-D)
            if a == b:
                v += mpmath.mpf(1e-8) + mpmath.mpf(hp[3]) ** 2
            Kmp[a, b] = v
    ymp = mpmath.matrix([mpmath.mpf(v) for v in y])
    amp = mpmath.lu_solve(Kmp, ymp)
    Lmp = mpmath.cholesky(Kmp)
    logdet = 2 * sum(mpmath.log(Lmp[i, i]) for i in range(n))
    mll_mp = 0.5 * (sum(ymp[i] * amp[i] for i in range(n)) + logdet + n * mpmath.log(2 * mpmath.pi))
    K = O.kernel(kinds, hp, x)
    np.testing.assert_allclose(K, np.array(Kmp.tolist(), dtype=float), rtol=1e-14)
    U = O.chol_upper(K)
    alpha = O.cho_solve_upper(U, y)
    np.testing.assert_allclose(alpha, np.array([float(v) for v in amp]), rtol=1e-11)
    assert O.mll_value(U, y, alpha) == pytest.approx(float(mll_mp), rel=1e-13)


def test_fit_upper_inplace_matches_oracle():
    """oracle/cpu_kbuild.fit_upper_inplace (the lean fit behind the full-size fixtures,
    tests/golden/make_fullsize.py) against the NumPy restatement."""
    from oracle.cpu_kbuild import fit_upper_inplace
    for kinds, backend in (([SE], "scipy"), ([SE, SE, WN], "scipy"), ([SE, SE, WN], "mkl")):
        x, y, xp = O.synthetic(8, 512, 64)
        hp = O.default_hp(kinds, 8)
        U, wt = fit_upper_inplace(kinds, hp, x, y, backend=backend)
        U_o = O.chol_upper(O.kernel(kinds, hp, x))
        np.testing.assert_allclose(np.triu(U), U_o, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(wt, O.cho_solve_upper(U_o, y), rtol=1e-10)
        mu, var = O.predict_from_factor(kinds, hp, x, U, wt, xp, diagonal_var=True)
        mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
        np.testing.assert_allclose(mu, mu_o, rtol=1e-12)
        np.testing.assert_allclose(var, var_o, rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("kinds", [[SE, WN], [SE, SE, WN], [SE]])
def test_mll_grad_cpu_matches_oracle(kinds):
    """oracle/mll_grad_cpu.c (the C4 CPU baseline's restatement of the reference's gradient
    loop: materialise dK_i, dgemv, Frobenius dot per component, src/cost.jl:119-126) equals the
    NumPy restatement's grad(MLL, ...) terms component by component."""
    from oracle.cpu_kbuild import mll_grad_cpu
    dim, n = 5, 300
    x, y, _ = O.synthetic(dim, n, 4)
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.1)
    K = O.kernel(kinds, hp, x)
    U = O.chol_upper(K)
    alpha = O.cho_solve_upper(U, y)
    Kinv = O.kinv_from_upper(U)
    g = mll_grad_cpu(kinds, hp, x, alpha, Kinv)
    g_o = np.array([O.mll_grad_term(O.kernel_grad(kinds, i, hp, x), alpha, Kinv)
                    for i in range(1, len(hp) + 1)])
    scale = np.array([abs(float(np.dot(d @ alpha, alpha))) + abs(float(np.sum(Kinv * d)))
                      if not isinstance(d, tuple) else abs(g_o[i]) + 1.0
                      for i, d in enumerate(O.kernel_grad(kinds, j, hp, x)
                                            for j in range(1, len(hp) + 1))])
    assert np.all(np.abs(g - g_o) <= 1e-10 * scale), (g - g_o) / scale
