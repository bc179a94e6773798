"""Bayesian quadrature (src/integrate.jl), restating test/test_integrate.jl.

CPU part: the scalar integrals and the antiderivative vector of the oracle against numerical
quadrature (test/test_integrate.jl:3-35; the reference uses QuadGK, here SciPy's adaptive
quad), and the host mirror's scalar functions.  GPU part: the device antiderivative and
integrate(md, a, b) against the oracle (rtol 1e-12 / 1e-8), and the integral of the posterior
mean against a tensor Gauss-Legendre rule over the device's predict_mean (rtol 1e-7).
"""
import numpy as np
import pytest
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
    with pytest.raises(NotImplementedError):
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
