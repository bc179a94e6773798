"""Host-side logic of the model updater (src/update_model.jl:52-100), restating
test/test_update.jl:1-46: finite-difference Hessian, BFGS inverse-Hessian update and the
quasi-Newton quadratic minimiser.  Pure NumPy on both sides (no device call), so it runs in the
CPU suite; tolerances are the reference test's (eps = 1e-4)."""
import numpy as np
import pytest

G = pytest.importorskip("gpr_amd")


def _spd(rng, dim):
    L = np.tril(rng.random((dim, dim)))
    return L @ L.T + 1e-7 * np.eye(dim)


@pytest.mark.parametrize("dim", [2, 5, 13, 30])
def test_hessian_fd_and_bfgs_quad(dim):
    """test/test_update.jl:1-23 (the reference loops dim = 2:30)."""
    rng = np.random.default_rng(dim)
    J = rng.random(dim)
    H = _spd(rng, dim)
    x0 = rng.random(dim)
    jac = lambda x: J + H @ x  # noqa: E731
    xma = -np.linalg.solve(H, J)
    eps = 1e-4
    assert np.all(np.linalg.eigvalsh(H) > 0)
    Hfd = G.hessian_fd(jac, rng.random(dim))
    assert np.abs(Hfd - H).max() <= eps                      # `≈ H atol = eps`
    xm, Jm, Hm, iters = G.bfgs_quad(x0, jac(x0), 1.0, jac, eps=eps, max_iter=100000)
    assert iters < 100000
    assert np.linalg.norm(xm - xma) <= 10 * eps * max(np.linalg.norm(xm), np.linalg.norm(xma))
    assert np.linalg.norm(Jm) < eps


@pytest.mark.parametrize("dim", [2, 7, 30])
def test_bfgs_hessian_update(dim):
    """test/test_update.jl:25-46: symmetry, positive definiteness, rho = 0 identity, and the
    closed form for Bi = I."""
    rng = np.random.default_rng(100 + dim)
    B = _spd(rng, dim)
    s, t = rng.random(dim), rng.random(dim)
    p = 1.0 / np.dot(s, t)
    Bs = G.bfgs_hessian(B, s, t)
    assert np.array_equal(Bs, Bs.T)
    assert np.all(np.linalg.eigvalsh(Bs) > 0)
    assert np.allclose(G.bfgs_hessian(B, s, t, 0.0), B, rtol=1e-12, atol=1e-12)
    st, ts, ss = np.outer(s, t), np.outer(t, s), np.outer(s, s)
    ref = (np.eye(dim) - p * (st + ts)) + (p ** 2 * np.dot(t, t) + p) * ss
    assert np.allclose(G.bfgs_hessian(1.0, s, t), ref, rtol=1e-10, atol=1e-12)


def test_init_params_and_options():
    """init_params (src/train.jl:1-7): ones for the marginal likelihood."""
    class _Md:  # only .params is read
        params = np.zeros(7)
    assert np.array_equal(G.init_params(G.MarginalLikelihood(), _Md()), np.ones(7))
    o = G.Options(g_tol=1e-2, iterations=200)
    assert o.g_tol == 1e-2 and o.iterations == 200
    assert G.NewtonTrustRegion().order == 2 and G.ConjugateGradient().order == 1
