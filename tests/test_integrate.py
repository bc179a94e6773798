"""Bayesian quadrature (src/integrate.jl), restating test/test_integrate.jl.

CPU part: the scalar integrals and the antiderivative vector of the oracle against numerical
quadrature (test/test_integrate.jl:3-35; the reference uses QuadGK, here SciPy's adaptive
quad), and the host mirror's scalar functions.  GPU part: the device antiderivative and
integrate(md, a, b) against the oracle (rtol 1e-12 / 1e-8), and the integral of the posterior
mean against a tensor Gauss-Legendre rule over the device's predict_mean (rtol 1e-7).
sample_noise: the oracle's eigen path (test/test_integrate.jl:47-111 restated on it) against
the device's shifted factorisations, and the reference's own sample-noise tests (:113-152).
"""
import numpy as np
import pytest
import scipy.linalg as sla
from scipy import integrate as sint

from oracle import gpr_oracle as O

G = pytest.importorskip("gpr_amd")


def test_gauss_and_erf_integrals_vs_quadrature():
    """test/test_integrate.jl:3-20 (100 random cases; erf integral atol 1e-5)."""
    rng = np.random.default_rng(0)
    for _ in range(100):
        xs, w = 3.0 * rng.random(), 3.0 * rng.random() + 1e-3
        a, b = -3.0 + 6 * rng.random(), -3.0 + 6 * rng.random()
        q = sint.quad(lambda x: np.exp(-w ** 2 * (x - xs) ** 2), a, b, epsrel=1e-10)[0]
        assert O.gauss_integ(xs, w, a, b) == pytest.approx(q, rel=1e-8, abs=1e-12)
        assert G.gauss_integ(xs, w, a, b) == pytest.approx(float(O.gauss_integ(xs, w, a, b)),
                                                           rel=1e-13, abs=1e-15)
        q2 = sint.quad(lambda x: float(O.gauss_integ(x, w, a, b)), a, b, epsrel=1e-10)[0]
        assert O.erf_integ(w, a, b) == pytest.approx(q2, abs=1e-5)
        assert G.erf_integ(w, a, b) == pytest.approx(float(O.erf_integ(w, a, b)), rel=1e-13,
                                                     abs=1e-15)


@pytest.mark.parametrize("dim,n", [(2, 100), (3, 300), (5, 500)])
def test_antideriv_oracle_identity(dim, n):
    """test/test_integrate.jl:22-35: antideriv = sigma^2 prod_i gauss_integ(x_i, l_i, a_i, b_i)."""
    rng = np.random.default_rng(dim * n)
    xs = rng.random((dim, n))
    hp = 5.0 * rng.random(dim + 1) + 0.05
    a = -2 + 4 * rng.random(dim)
    b = a + 2.0 * rng.random(dim)
    integ = hp[0] ** 2 * np.prod(O.gauss_integ(xs, hp[1:, None], a[:, None], b[:, None]), axis=0)
    np.testing.assert_allclose(O.antideriv_se(xs, hp, a, b), integ, rtol=1e-12, atol=1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n", [(1, 64), (2, 300), (5, 500), (8, 1000)])
def test_antideriv_device_vs_oracle(dim, n):
    rng = np.random.default_rng(7 + dim)
    xs = rng.random((dim, n))
    hp = 5.0 * rng.random(dim + 1) + 0.05
    a = -2 + 4 * rng.random(dim)
    b = a + 2.0 * rng.random(dim)
    k1 = G.antideriv(G.SquaredExp(), xs, hp, a, b)
    np.testing.assert_allclose(k1, O.antideriv_se(xs, hp, a, b), rtol=1e-12, atol=1e-300)
    assert G.antideriv2(G.SquaredExp(), hp, a, b) == pytest.approx(O.antideriv2_se(hp, a, b),
                                                                     rel=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dim,n", [("SE", 2, 200), ("SE+WN", 3, 700), ("SE+WN", 2, 1500)])
def test_integrate_vs_oracle(name, dim, n):
    kinds = [O.SE] if name == "SE" else [O.SE, O.WN]
    cov = G.SquaredExp() if name == "SE" else G.SquaredExp() + G.WhiteNoise()
    x, y, _ = O.synthetic(dim, n, 0, seed_train=n)
    hp = O.default_hp(kinds, dim, length=1.5, noise=0.05)
    Y = np.stack([y, np.cos(x.sum(0))], axis=1)
    md = G.GPRModel(cov, hp, x, Y)
    a, b = np.full(dim, 0.1), np.full(dim, 0.8)
    I, v = G.integrate(md, a, b)
    Io, vo = O.integrate(kinds, hp, x, Y, a, b)
    np.testing.assert_allclose(I, Io, rtol=1e-8, atol=1e-12)
    assert v[0] == pytest.approx(vo, rel=1e-8, abs=1e-10 * O.antideriv2_se(hp, a, b))
    with pytest.raises(TypeError):  # the reference has no scalar-noise variance method
        G.integrate(md, a, b, sample_noise=1e-5)


@pytest.mark.gpu
def test_integral_of_posterior_mean_vs_gauss_legendre():
    """The quadrature of the device's posterior mean over [a, b]^2 (40-point tensor
    Gauss-Legendre rule) equals integrate's Iout: the k1 weights integrate the same mean."""
    kinds, dim, n = [O.SE, O.WN], 2, 400
    x, y, _ = O.synthetic(dim, n, 0, seed_train=3)
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    a, b = np.array([0.2, 0.1]), np.array([0.9, 0.7])
    I, _ = G.integrate(md, a, b)
    t, w = np.polynomial.legendre.leggauss(40)
    g0 = 0.5 * (b[0] - a[0]) * t + 0.5 * (a[0] + b[0])
    g1 = 0.5 * (b[1] - a[1]) * t + 0.5 * (a[1] + b[1])
    X0, X1 = np.meshgrid(g0, g1, indexing="ij")
    W = np.outer(w, w).ravel() * 0.25 * (b[0] - a[0]) * (b[1] - a[1])
    mu = G.predict_mean(md, np.stack([X0.ravel(), X1.ravel()]))
    assert float(W @ mu) == pytest.approx(I[0], rel=1e-7)


@pytest.mark.parametrize("n", [100, 200])
def test_inverse_diagonal_update_oracle(n):
    """test/test_integrate.jl:47-111 on the oracle's eigen path (scalar and vector noise).
    The reference shifts L L' by 1e-7; at cond ~1e11 the "exact" solve it compares against is
    itself good to ~1e-5 only, so the shift here is 1e-4."""
    rng = np.random.default_rng(n)
    L = np.tril(rng.random((n, n)))
    A = L @ L.T + 1e-4 * np.eye(n)
    lam, P = np.linalg.eigh(A)
    y = rng.random(n)
    e = 1e-5
    ex = np.linalg.solve(A + e * np.eye(n), y)
    np.testing.assert_allclose(O.inverse_diagonal_update(lam, P, e, y), ex, rtol=1e-6)
    assert O.inverse_diagonal_update2(lam, P, e, y) == pytest.approx(y @ ex, rel=1e-6)
    ne = 40
    ev = 1e-5 * rng.random(ne)
    Y = rng.random((n, ne))
    exv = np.stack([np.linalg.solve(A + ev[i] * np.eye(n), Y[:, i]) for i in range(ne)], axis=1)
    np.testing.assert_allclose(O.inverse_diagonal_update(lam, P, ev, Y), exv, rtol=1e-5)
    q = np.array([y @ np.linalg.solve(A + ev[i] * np.eye(n), y) for i in range(ne)])
    np.testing.assert_allclose(O.inverse_diagonal_update2(lam, P, ev, y), q, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("quad", ["auto", "1", "3"])
@pytest.mark.parametrize("name,dim,n,ne", [("SE", 2, 150, 7), ("SE+WN", 3, 300, 12),
                                           ("SE", 4, 1100, 5)])
def test_integrate_sample_noise_vs_oracle(name, dim, n, ne, quad, knobs):
    """Positive shifts: the default picks the per-column factorisations at these ne (fewer
    columns than one reduction costs); GPR_QUAD_EIGEN=1 forces the tridiagonal reduction +
    per-column tridiagonal solves, 3 the reference's full eigendecomposition (reduction +
    divide and conquer) + diagonal updates."""
    if quad != "auto":
        knobs("GPR_QUAD_EIGEN", int(quad))
    kinds = [O.SE] if name == "SE" else [O.SE, O.WN]
    cov = G.SquaredExp() if name == "SE" else G.SquaredExp() + G.WhiteNoise()
    rng = np.random.default_rng(dim + n)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    md = G.GPRModel(cov, hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    noise = 1e-3 * (1.0 + rng.random(ne))
    I, v = G.integrate(md, a, b, sample_noise=noise)
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I, Io, rtol=1e-8)
    np.testing.assert_allclose(v, vo, rtol=1e-7, atol=1e-12 * O.antideriv2_se(hp, a, b))


@pytest.mark.gpu
@pytest.mark.parametrize("quad", ["1", "3"])
@pytest.mark.parametrize("n,ne", [(1, 3), (2, 1), (3, 4), (4, 2), (17, 5), (129, 1)])
def test_integrate_sample_noise_small_sizes(n, ne, quad, knobs):
    """The eigen routes at the smallest sizes: n = 1, 2 (nothing to reduce: T = K), 3 (one
    reflector), 4, 17, 129, one column and a few, positive and negative shifts -- against the
    oracle's eigen path."""
    knobs("GPR_QUAD_EIGEN", int(quad))
    dim = 2
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(10 * n + ne)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    hp = O.default_hp(kinds, dim, length=1.5, noise=0.2)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    lam = np.linalg.eigvalsh(O.kernel(kinds, hp, x))
    noise = np.r_[1e-3, -0.5 * lam.min(), 0.3][:ne] if ne <= 3 else np.r_[1e-3 * (1.0 + rng.random(ne - 1)), -0.5 * lam.min()]
    I, v = G.integrate(md, a, b, sample_noise=noise)
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I, Io, rtol=1e-9, atol=1e-14)
    np.testing.assert_allclose(v, vo, rtol=1e-8, atol=1e-12 * O.antideriv2_se(hp, a, b))


@pytest.mark.gpu
def test_integrate_sample_noise_negative(knobs):
    """Negative sample noise, as the reference's eigen path takes it (src/integrate.jl:71-100:
    K = P Lambda P' once, (Lambda + noise_j)^-1 per column, never a factorisation): a shift
    that keeps K + noise I positive definite and one that makes it negative definite both
    match the oracle's eigen path -- no PosDefException.  With GPR_QUAD_EIGEN=0 (per-column
    factorisations, the fallback when rocSOLVER cannot be loaded) the second raises."""
    dim, n = 3, 200
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(5)
    x = rng.random((dim, n))
    Y = rng.random((n, 2))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)   # lambda_min(K) >= 0.05^2
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    lam = np.linalg.eigvalsh(O.kernel(kinds, hp, x))
    noise = np.array([-0.5 * lam.min(), 0.0])
    I, v = G.integrate(md, a, b, sample_noise=noise)
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I, Io, rtol=1e-7)
    np.testing.assert_allclose(v, vo, rtol=1e-6, atol=1e-10 * O.antideriv2_se(hp, a, b))
    neg = np.array([1e-3, -1.5 * lam.max()])   # K + noise I negative definite, well away from 0
    I, v = G.integrate(md, a, b, sample_noise=neg)
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, neg)
    np.testing.assert_allclose(I, Io, rtol=1e-8)
    np.testing.assert_allclose(v, vo, rtol=1e-8)
    knobs("GPR_QUAD_EIGEN", 0)
    with pytest.raises(G.PosDefException):
        G.integrate(md, a, b, sample_noise=neg)


@pytest.mark.gpu
@pytest.mark.parametrize("quad", ["auto", "1"])
def test_integrate_sample_noise_negative_large(quad, knobs):
    """n = 8192 (beyond the LDS-bound reduction of round 5): a positive shift, a negative one
    that keeps K + s I positive definite (lambda_min(K) >= sigma_n^2) and one below -lambda_max
    (negative definite, as the reference's eigen path allows).  The default tries the per-column
    factorisations (3 columns), meets the indefinite shift and hands the call to the tridiagonal
    reduction (its global-vector variant) -- no PosDefException and no block Jacobi; knob 1 takes
    the reduction directly.  Expected values by a dense LU solve of K + s I (the same function
    k1' (K + s I)^{-1} y the reference's eigen path evaluates)."""
    if quad != "auto":
        knobs("GPR_QUAD_EIGEN", int(quad))
    dim, n = 4, 8192
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(8192)
    x = rng.random((dim, n))
    Y = rng.random((n, 3))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    K = O.kernel(kinds, hp, x)
    lmax = np.abs(K).sum(0).max()
    noise = np.array([1e-3, -0.5 * hp[-1] ** 2, -1.5 * lmax])
    I, v = G.integrate(md, a, b, sample_noise=noise)
    k1 = O.antideriv_se(x, hp, a, b)
    k2 = O.antideriv2_se(hp, a, b)
    for j, s in enumerate(noise):
        sol = np.linalg.solve(K + s * np.eye(n), np.c_[Y[:, j], k1])
        np.testing.assert_allclose(I[j], k1 @ sol[:, 0], rtol=1e-7)
        np.testing.assert_allclose(v[j], k2 - k1 @ sol[:, 1], rtol=1e-6, atol=1e-10 * k2)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,k", [(1, 100, 100), (2, 200, 300), (4, 300, 200)])
def test_integrate_zero_noise_reference(dim, n, k):
    """test/test_integrate.jl:113-126 (random hp as GPRModel(SquaredExp(), x, y))."""
    rng = np.random.default_rng(100 * dim + k)
    x = rng.random((dim, n))
    y = rng.random((n, k))
    md = G.GPRModel(G.SquaredExp(), None, x, y, rng=rng)
    a, b = np.zeros(dim), np.ones(dim)
    mu, s = G.integrate(md, a, b, sample_noise=None)
    mu0, s0 = G.integrate(md, a, b, sample_noise=np.zeros(k))
    np.testing.assert_allclose(mu, mu0, rtol=1e-5)
    assert s[0] == pytest.approx(s0[1], rel=1e-4)
    np.testing.assert_allclose(s0[1:], 0.0, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n,ne", [(1, 100, 100), (3, 200, 300), (4, 300, 100)])
def test_integrate_inverse_perturbation_reference(dim, n, ne):
    """test/test_integrate.jl:128-152: column i against cholesky(K + noise_i I)."""
    rng = np.random.default_rng(7 * dim + ne)
    x = rng.random((dim, n))
    y = rng.random((n, ne))
    md = G.GPRModel(G.SquaredExp(), None, x, y, rng=rng)
    noise = 1e-5 * rng.random(ne)
    a, b = np.zeros(dim), np.ones(dim)
    mu, S = G.integrate(md, a, b, sample_noise=noise)
    K = O.kernel([O.SE], md.params, x)
    k1 = O.antideriv_se(x, md.params, a, b)
    k2 = O.antideriv2_se(md.params, a, b)
    mu_ex, S_ex = np.zeros(ne), np.zeros(ne)
    for i in range(ne):
        U = O.chol_upper(K + noise[i] * np.eye(n))
        mu_ex[i] = O.cho_solve_upper(U, y[:, i]) @ k1
        t = sla.solve_triangular(U, k1, trans="T", lower=False)
        S_ex[i] = k2 - t @ t
    # the reference's `≈ rtol = 1e-5` on arrays is normwise (Julia isapprox); elementwise, S =
    # k2 - t.t cancels k2 down to ~1e-8, so each entry also carries an absolute floor of 64 eps k2
    np.testing.assert_allclose(mu, mu_ex, rtol=1e-5)
    assert np.linalg.norm(S - S_ex) <= 1e-5 * max(np.linalg.norm(S), np.linalg.norm(S_ex))
    np.testing.assert_allclose(S, S_ex, rtol=1e-5, atol=64 * np.finfo(float).eps * k2)


@pytest.mark.gpu
def test_integrate_auto_falls_back_to_eigen_when_not_posdef(knobs):
    """Nonnegative shifts on a singular K (every point the same, no jitter: K = sigma^2 1 1^T,
    the second pivot exactly 0): the default's per-column factorisation fails and hands the
    call to the eigensolver -- no PosDefException, the eigensolver's own result bit for bit."""
    dim, n, ne = 2, 256, 4
    rng = np.random.default_rng(21)
    x = np.full((dim, n), 0.3)
    Y = rng.random((n, ne))
    hp = O.default_hp([O.SE], dim, length=2.0)
    md = G.GPRModel(G.SquaredExp(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    noise = np.zeros(ne)
    I, v = G.integrate(md, a, b, sample_noise=noise, eps=0.0)
    knobs("GPR_QUAD_EIGEN", 1)
    I1, v1 = G.integrate(md, a, b, sample_noise=noise, eps=0.0)
    np.testing.assert_array_equal(I, I1)
    np.testing.assert_array_equal(v, v1)
    knobs("GPR_QUAD_EIGEN", 0)
    with pytest.raises(G.PosDefException):
        G.integrate(md, a, b, sample_noise=noise, eps=0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("n,ne", [(300, 9), (1040, 6)])
def test_integrate_batched_columns_chunking_and_sequential(n, ne, knobs):
    """The default's batched launch (every K + s_j I factored and solved in one tile-DAG
    launch) is the same computation per column whatever the batch: a 1-column memory budget
    (GPR_QUAD_BATCH_GB, one launch per column) gives bit for bit the same result; the
    sequential per-column path (GPR_QUAD_SEQ) and the oracle agree to rounding."""
    dim = 3
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(n + ne)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    noise = 1e-3 * (1.0 + rng.random(ne))
    I, v = G.integrate(md, a, b, sample_noise=noise)
    knobs("GPR_QUAD_BATCH_GB", 1e-9)
    I1, v1 = G.integrate(md, a, b, sample_noise=noise)
    np.testing.assert_array_equal(I, I1)
    np.testing.assert_array_equal(v, v1)
    knobs("GPR_QUAD_BATCH_GB", 16.0)
    knobs("GPR_QUAD_SEQ", 1)
    Is, vs = G.integrate(md, a, b, sample_noise=noise)
    np.testing.assert_allclose(Is, I, rtol=1e-9)
    np.testing.assert_allclose(vs, v, rtol=1e-8, atol=1e-12 * O.antideriv2_se(hp, a, b))
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I, Io, rtol=1e-8)
    np.testing.assert_allclose(v, vo, rtol=1e-7, atol=1e-12 * O.antideriv2_se(hp, a, b))


@pytest.mark.gpu
def test_integrate_tridiagonal_solves_in_chunks():
    """The per-column tridiagonal solves in launches of 7 and 1 columns (test build's
    GPR_TRD_QCHUNK) give bit for bit the one-launch result (tests/fault_scenarios.py
    trd_quad_chunks, in a child process on libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("trd_quad_chunks")
