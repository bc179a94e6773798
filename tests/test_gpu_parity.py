"""GPU parity: libgpr_hip.so (through the C ABI, via gpr_amd) vs the CPU oracle.

Each test restates one of the reference's own tests (file:line cited) and/or compares the
HIP result with the oracle on identical seeded inputs.  Tolerances (fp64):
  kernel matrices   rtol 1e-13 (pure elementwise arithmetic + exp)
  factor / inverse  normwise 1e-11 (well-conditioned inputs)
  posterior, MLL    rtol 1e-8 (BASELINE north_star) -- observed errors are far smaller
"""
import ctypes

import numpy as np
import pytest
import scipy.linalg as sla

from oracle import gpr_oracle as O

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gpr_amd")

SE, WN = O.SE, O.WN
KSETS = {
    "SE": [SE],
    "SE+WN": [SE, WN],
    "SE+SE": [SE, SE],
    "SE+SE+WN": [SE, SE, WN],
    "WN+SE": [WN, SE],
    "SE+WN+SE": [SE, WN, SE],
}


def cov_of(kinds):
    parts = [G.SquaredExp() if k == SE else G.WhiteNoise() for k in kinds]
    c = parts[0]
    for p in parts[1:]:
        c = c + p
    return c


def rand_hp(kinds, d, rng, lo=0.3, hi=2.0):
    return rng.uniform(lo, hi, sum(O.dim_hp(k, d) for k in kinds))


def julia_approx(a, b, rtol=None, atol=0.0):
    """Julia's isapprox on arrays (the reference tests' `≈`): normwise,
    norm(a-b) <= max(atol, rtol*max(norm(a), norm(b))), rtol defaults to sqrt(eps)."""
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    if rtol is None:
        rtol = 0.0 if atol > 0 else np.sqrt(np.finfo(float).eps)
    return np.linalg.norm(a - b) <= max(atol, rtol * max(np.linalg.norm(a), np.linalg.norm(b)))


def relnorm(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


# ---------------------------------------------------------------------------------------
# a2/a3 kernel matrices  (test/test_covariance.jl:11-82)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", list(KSETS))
@pytest.mark.parametrize("n,d", [(1, 1), (63, 2), (64, 3), (65, 5), (200, 7), (300, 8), (130, 16),
                                 (97, 20)])
def test_kernel_matrix(name, n, d):
    kinds = KSETS[name]
    rng = np.random.default_rng(n * 31 + d)
    x = rng.random((d, n))
    xp = rng.random((d, 2 * n))
    hp = rand_hp(kinds, d, rng)
    cov = cov_of(kinds)
    K = G.kernel(cov, hp, x)
    Ko = O.kernel(kinds, hp, x)
    np.testing.assert_allclose(K, Ko, rtol=1e-13, atol=1e-15)
    assert np.array_equal(K, K.T), "symmetric K must be bitwise symmetric (mirror of upper)"
    Kx = G.kernel(cov, hp, x, xp)
    np.testing.assert_allclose(Kx, O.kernel(kinds, hp, x, xp), rtol=1e-13, atol=1e-15)
    assert Kx.shape == (n, 2 * n)


@pytest.mark.parametrize("n,d", [(1, 3), (130, 2), (300, 8), (1000, 5), (2049, 8), (257, 17)])
def test_kernel_matrix_ragged_tiles(n, d):
    """The symmetric Gram K-assembly with ragged last tiles: same values as the oracle, K bitwise
    symmetric, composed parts + noise."""
    rng = np.random.default_rng(n + d)
    x = rng.random((d, n))
    for kinds in ([SE], [SE, SE, WN]):
        hp = rand_hp(kinds, d, rng)
        K = G.kernel(cov_of(kinds), hp, x)
        np.testing.assert_allclose(K, O.kernel(kinds, hp, x), rtol=1e-13, atol=1e-15)
        assert np.array_equal(K, K.T)


def test_kernel_structure_isposdef():
    """test/test_covariance.jl:27-32: issymmetric, isposdef, shapes."""
    rng = np.random.default_rng(5)
    for n in (100, 200, 300):
        for dim in range(1, 8):
            x = rng.random((dim, n))
            hp = rng.random(dim + 1)
            K = G.kernel(G.SquaredExp(), hp, x)
            assert np.array_equal(K, K.T)
            np.linalg.cholesky(K + 0.0)  # raises if not PD (eps jitter keeps it PD)


def test_compose_identities():
    """test/test_covariance.jl:34-81 restated against the HIP kernels."""
    rng = np.random.default_rng(11)
    dim, n = 3, 120
    x, xp = rng.random((dim, n)), rng.random((dim, 2 * n))
    SEk, WNk = G.SquaredExp(), G.WhiteNoise()
    hps = rng.random(dim + 2)
    np.testing.assert_allclose(G.kernel(SEk + WNk, hps, x),
                               G.kernel(SEk, hps[:-1], x) + hps[-1] ** 2 * np.eye(n), rtol=1e-14)
    np.testing.assert_allclose(G.kernel(SEk + WNk, hps, x, xp), G.kernel(SEk, hps[:-1], x, xp),
                               rtol=1e-14)
    hps = rng.random(2 * dim + 2)
    np.testing.assert_allclose(G.kernel(SEk + SEk, hps, x),
                               G.kernel(SEk, hps[:dim + 1], x) + G.kernel(SEk, hps[dim + 1:], x),
                               rtol=1e-14)
    hps = rng.random(2 * dim + 3)
    np.testing.assert_allclose(
        G.kernel(SEk + WNk + SEk, hps, x),
        G.kernel(SEk, hps[:dim + 1], x) + G.kernel(SEk, hps[dim + 2:], x) + hps[dim + 1] ** 2 * np.eye(n),
        rtol=1e-14)


def test_kernels_per_part_and_caches():
    """kernels(K, hp, x) (src/compose_covar.jl:80-107): one matrix per part, 1x1 zero for
    WhiteNoise; cache constructors and predict_mean! from an updated GPRPredictCache."""
    rng = np.random.default_rng(12)
    dim, n, m = 3, 150, 40
    x, xp = rng.random((dim, n)), rng.random((dim, m))
    SEk, WNk = G.SquaredExp(), G.WhiteNoise()
    hps = rng.uniform(0.5, 2.0, 2 * dim + 3)
    Ks = G.kernels(SEk + WNk + SEk, hps, x)
    assert len(Ks) == 3 and Ks[1].shape == (1, 1) and Ks[1][0, 0] == 0.0
    np.testing.assert_allclose(Ks[0], O.kernel([SE], hps[:dim + 1], x), rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(Ks[2], O.kernel([SE], hps[dim + 2:], x), rtol=1e-13, atol=1e-15)
    assert len(G.kernels(SEk, hps[:dim + 1], x)) == 1
    parts, ph = G.rm_noise(SEk + WNk + SEk, ["a", "b", "c"])
    assert len(parts) == 2 and ph == ["a", "c"]
    assert G.loss_cache(G.MarginalLikelihood()) is G.MllLossCache
    assert G.loss_grad_cache(G.MarginalLikelihood()) is G.MllGradCache
    y = np.sin(x.sum(0)) ** 2
    md = G.GPRModel(SEk + WNk, hps[:dim + 2], x, y)
    assert G.predict_cache(md, xp) is G.GPRPredictCache
    pc = G.predict_cache(md, xp)(md, m)
    G.update_predict_cache_(pc, md)
    mu = md.ctx.empty(m)
    G.predict_mean_(mu, md, xp, pc)
    mu_o, _ = O.predict([SE, WN], hps[:dim + 2], x, y, xp, diagonal_var=True)
    np.testing.assert_allclose(md.ctx.host(mu), mu_o, rtol=1e-8, atol=1e-12)
    md2 = G.similar(md, hps[:dim + 2], xp, np.cos(xp.sum(0)))
    assert md2.n == m and md2.covar is md.covar


# ---------------------------------------------------------------------------------------
# a4 dK/dtheta  (test/test_covariance.jl:3-9,84-105)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["SE", "SE+WN+SE"])
def test_kernel_grad(name):
    kinds = KSETS[name]
    rng = np.random.default_rng(3)
    dim, n = 2, 100
    x = rng.random((dim, n))
    hp = rand_hp(kinds, dim, rng)
    cov = cov_of(kinds)
    for i in range(1, len(hp) + 1):
        g = G.grad(cov, i, hp, x)
        go = O.kernel_grad(kinds, i, hp, x)
        if isinstance(go, tuple):
            assert isinstance(g, G.UniformScaling) and g.lam == pytest.approx(go[1])
            continue
        np.testing.assert_allclose(g, go, rtol=1e-12, atol=1e-14)
        # forward FD, eps 1e-7, atol 1e-3 (test/test_covariance.jl:3-9,85)
        hpe = hp.copy()
        hpe[i - 1] += 1e-7
        fd = (G.kernel(cov, hpe, x) - G.kernel(cov, hp, x)) / 1e-7
        np.testing.assert_allclose(g, fd, atol=1e-3)


# ---------------------------------------------------------------------------------------
# a5 POTRF (dpotrf 'U', in place, lower untouched)
# ---------------------------------------------------------------------------------------
def _spd(n, d=4, seed=0, noise=0.3):
    rng = np.random.default_rng(seed)
    x = rng.random((d, n))
    return O.kernel([SE, WN], np.r_[1.0, [1.5] * d, noise], x)


def _dev_potrf(ctx, A, nb=None):
    dA = ctx.colmajor(A)
    n = A.shape[0]
    info = ctypes.c_int(-7)
    rc = G._lib.lib.gpr_potrf_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n, ctypes.byref(info))
    assert rc >= 0, G._lib.lib.gpr_last_error(ctx.h)
    return dA, info.value


@pytest.mark.parametrize("n", [1, 50, 64, 127, 128, 129, 300, 700])
@pytest.mark.parametrize("nb", [128, 64])
def test_potrf_upper(n, nb):
    ctx = G.Context(0, nb=nb)
    A = _spd(n, seed=n)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    R = ctx.host(dA)
    U = sla.cholesky(A, lower=False)
    assert relnorm(np.triu(R), U) < 1e-12
    # strict lower triangle untouched, bit for bit (test/test_loss.jl:46)
    assert np.array_equal(np.tril(R, -1), np.tril(A, -1))


def _blocked_env(monkeypatch):
    """The blocked two-level factorisation alone (per-block panels + lookahead stream; its
    measured-slower panel variants were removed in round 5)."""
    monkeypatch.setenv("GPR_DAG", "0")
    monkeypatch.setenv("GPR_DAG_TAIL", "0")


@pytest.mark.parametrize("n,nb2", [(300, 256), (1000, 256), (1300, 512), (2600, 1024), (1024, 1024),
                                   (1025, 1024), (777, 2048), (3000, 384)])
def test_potrf_outer_panels(n, nb2, monkeypatch):
    """Two-level factorisation across outer-panel boundaries, ragged last panels and tiles."""
    _blocked_env(monkeypatch)
    ctx = G.Context(0)
    assert G._lib.lib.gpr_set_outer_block(ctx.h, nb2) == 0
    A = _spd(n, seed=n + nb2)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    R = ctx.host(dA)
    U = sla.cholesky(A, lower=False)
    assert relnorm(np.triu(R), U) < 1e-12
    assert np.array_equal(np.tril(R, -1), np.tril(A, -1))
    # the factor's block inverses / square inverses feed the solves
    B = np.random.default_rng(3).random((n, 3))
    dB = ctx.colmajor(B)
    assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                      ctypes.c_void_p(dB.data_ptr()), 3, n) == 0
    assert relnorm(ctx.host(dB), O.cho_solve_upper(U, B)) < 1e-11


@pytest.mark.parametrize("j", [0, 255, 256, 700, 1299])
def test_potrf_not_posdef_info_later_panels(j, monkeypatch):
    _blocked_env(monkeypatch)
    ctx = G.Context(0)
    assert G._lib.lib.gpr_set_outer_block(ctx.h, 256) == 0
    A = _spd(1300, seed=2)
    A[j, j] = -1.0
    _, info = _dev_potrf(ctx, A)
    _, info_ref = sla.lapack.dpotrf(A, lower=0)
    assert info == info_ref == j + 1


@pytest.mark.parametrize("n", [16, 128, 144, 256, 400, 1040, 2064, 4112, 1, 50, 129, 333, 1031])
def test_potrf_dag(n, monkeypatch):
    """Persistent tile-DAG factorisation (dag.hip, GPR_DAG=1): one launch, tiles handed
    between workgroups by progress counters; ragged last tile (n % 128 != 0), upper factor,
    lower triangle untouched, block inverses usable by the solves.  n % 16 != 0 goes through
    the padded copy [[A, 0], [0, I]]."""
    monkeypatch.setenv("GPR_DAG", "1")
    ctx = G.Context(0)
    A = _spd(n, seed=n + 7)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    R = ctx.host(dA)
    U = sla.cholesky(A, lower=False)
    assert relnorm(np.triu(R), U) < 1e-12
    assert np.array_equal(np.tril(R, -1), np.tril(A, -1))
    B = np.random.default_rng(4).random((n, 2))
    dB = ctx.colmajor(B)
    assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                      ctypes.c_void_p(dB.data_ptr()), 2, n) == 0
    assert relnorm(ctx.host(dB), O.cho_solve_upper(U, B)) < 1e-11


@pytest.mark.parametrize("n,lda,off", [(1040, 1056, 0), (1040, 1043, 0), (1024, 1048, 8),
                                       (2048, 2176, 128), (1000, 1024, 0)])
def test_potrf_dag_leading_dim(n, lda, off, monkeypatch):
    """The tile-DAG on a block of a larger column-major buffer: lda > n (a multiple of 16:
    taken directly; 1043: through the padded copy), the block starting `off` doubles into
    the buffer (8: a base 64 B off the 128-B alignment -> padded copy).  U in the block's upper
    triangle, its lower triangle and everything outside the block untouched."""
    monkeypatch.setenv("GPR_DAG", "1")
    ctx = G.Context(0)
    A = _spd(n, seed=n + lda)
    rows = off + lda
    buf = np.random.default_rng(1).random((rows, n + 1))  # column-major rows x (n + 1)
    buf[off:off + n, :n] = A
    dbuf = ctx.colmajor(buf)  # column c at c * rows
    base = dbuf.data_ptr() + 8 * off
    info = ctypes.c_int(-7)
    # the block's columns are `rows` apart: pass lda = rows
    rc = G._lib.lib.gpr_potrf_upper(ctx.h, ctypes.c_void_p(base), n, rows, ctypes.byref(info))
    assert rc == 0 and info.value == 0, G._lib.lib.gpr_last_error(ctx.h)
    out = ctx.host(dbuf)
    R = out[off:off + n, :n]
    assert relnorm(np.triu(R), sla.cholesky(A, lower=False)) < 1e-12
    assert np.array_equal(np.tril(R, -1), np.tril(A, -1))
    mask = np.ones_like(buf, dtype=bool)
    mask[off:off + n, :n] = False
    assert np.array_equal(out[mask], buf[mask])


@pytest.mark.parametrize("n,nb2,tail", [(3008, 256, 1024), (2064, 512, 1600), (1040, 256, 1040),
                                         (4096, 1024, 2048)])
def test_potrf_dag_tail(n, nb2, tail, monkeypatch):
    """Blocked factorisation that hands its last <= tail columns to the tile-DAG (GPR_DAG_TAIL):
    one SYRK applies the last blocked panel to the whole trailing matrix, then the DAG factors
    it with global block indices (solves read its W_i slots)."""
    monkeypatch.setenv("GPR_DAG", "0")
    monkeypatch.setenv("GPR_DAG_TAIL", str(tail))
    ctx = G.Context(0)
    assert G._lib.lib.gpr_set_outer_block(ctx.h, nb2) == 0
    A = _spd(n, seed=n + nb2)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    R = ctx.host(dA)
    U = sla.cholesky(A, lower=False)
    assert relnorm(np.triu(R), U) < 1e-12
    assert np.array_equal(np.tril(R, -1), np.tril(A, -1))
    B = np.random.default_rng(5).random((n, 3))
    dB = ctx.colmajor(B)
    assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                      ctypes.c_void_p(dB.data_ptr()), 3, n) == 0
    assert relnorm(ctx.host(dB), O.cho_solve_upper(U, B)) < 1e-11


@pytest.mark.parametrize("j", [3, 300, 2000, 2999])
def test_potrf_dag_tail_not_posdef_info(j, monkeypatch):
    monkeypatch.setenv("GPR_DAG", "0")
    monkeypatch.setenv("GPR_DAG_TAIL", "1024")
    ctx = G.Context(0)
    assert G._lib.lib.gpr_set_outer_block(ctx.h, 256) == 0
    A = _spd(3008, seed=3)
    A[j, j] = -1.0
    _, info = _dev_potrf(ctx, A)
    _, info_ref = sla.lapack.dpotrf(A, lower=0)
    assert info == info_ref == j + 1


@pytest.mark.parametrize("j", [0, 5, 127, 128, 200, 1000, 1039])
def test_potrf_dag_not_posdef_info(j, monkeypatch):
    monkeypatch.setenv("GPR_DAG", "1")
    ctx = G.Context(0)
    A = _spd(1040, seed=2)
    A[j, j] = -1.0
    _, info = _dev_potrf(ctx, A)
    _, info_ref = sla.lapack.dpotrf(A, lower=0)
    assert info == info_ref == j + 1


@pytest.mark.parametrize("gram", ["1", "0"])
def test_fit_kinv_dag_not_posdef_info(gram, monkeypatch):
    """A non-PD K under the tile-DAG with Z and gram tasks: info = the failing minor's order,
    the launch drains (the remaining tasks skip), and the context factors the next matrix."""
    monkeypatch.setenv("GPR_DAG_GRAM", gram)
    kinds = KSETS["SE+WN"]
    dim, n = 4, 1024
    x, y, _ = O.synthetic(dim, n, 0, seed_train=3)
    ctx = G.Context(0)
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, Kinv, alpha = ctx.empty(n, n), ctx.empty(n, n), ctx.empty(n)
    karr = (ctypes.c_int * 2)(1, 2)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    hp = O.default_hp(kinds, dim, noise=0.1)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    # eps = -0.012 on the diagonal: the minor of order 625 fails (mid launch, tile row 4 of 8)
    for eps, ok in ((-0.012, False), (1e-8, True)):
        info = ctypes.c_int(-1)
        rc = G._lib.lib.gpr_fit_kinv(ctx.h, karr, 2, hpp, dim, P(dx), n, P(dy), 1, n, eps, P(K), n,
                                     P(alpha), P(Kinv), n, ctypes.byref(info))
        Ko = O.kernel(kinds, hp, x, None, eps=eps)
        if ok:
            assert rc == 0 and info.value == 0
            Uo = sla.cholesky(Ko, lower=False)
            assert relnorm(ctx.host(Kinv), O.kinv_from_upper(Uo)) < 1e-10
        else:
            _, info_ref = sla.lapack.dpotrf(Ko, lower=0)
            assert info_ref == 625 and rc == info.value == info_ref


@pytest.mark.parametrize("j", [0, 5, 127, 128, 200])
def test_potrf_not_posdef_info(j):
    """Non-PD input: info = order of the failing leading minor (dpotrf / PosDefException)."""
    ctx = G.Context(0)
    A = _spd(260, seed=1)
    A[j, j] = -1.0
    _, info = _dev_potrf(ctx, A)
    _, info_ref = sla.lapack.dpotrf(A, lower=0)
    assert info == info_ref == j + 1


def test_posdef_exception_from_model():
    rng = np.random.default_rng(2)
    x = rng.random((2, 50))
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), np.r_[1.0, 1.0, 1.0, 0.1], x, x[0])
    md.params[0] = float("nan")
    with pytest.raises(G.PosDefException):
        G.loss(G.MarginalLikelihood(), md.params, md)


# ---------------------------------------------------------------------------------------
# a6/a7 solves, K^{-1}
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,nrhs", [(300, 1), (257, 3), (129, 20), (1, 1), (128, 2), (1000, 1),
                                    (3001, 5), (4096, 2)])
def test_potrs(n, nrhs):
    ctx = G.Context(0)
    A = _spd(n, seed=7)
    dA, info = _dev_potrf(ctx, A)
    B = np.random.default_rng(1).random((n, nrhs))
    dB = ctx.colmajor(B)
    rc = G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                   ctypes.c_void_p(dB.data_ptr()), nrhs, n)
    assert rc == 0
    X = ctx.host(dB)
    Xo = O.cho_solve_upper(sla.cholesky(A, lower=False), B)
    assert relnorm(X, Xo) < 1e-11


def test_potrs_repeated_sweeps_identical():
    """The single-launch sweeps hand blocks between workgroups through flags: repeated calls
    must give bit-identical results (any stale hand-off would show up as a difference)."""
    n = 2500
    ctx = G.Context(0)
    A = _spd(n, seed=11)
    dA, info = _dev_potrf(ctx, A)
    B = np.random.default_rng(2).random((n, 2))
    outs = []
    for _ in range(5):
        dB = ctx.colmajor(B)
        assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                          ctypes.c_void_p(dB.data_ptr()), 2, n) == 0
        outs.append(ctx.host(dB))
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])
    Xo = O.cho_solve_upper(sla.cholesky(A, lower=False), B)
    assert relnorm(outs[0], Xo) < 1e-11


def test_potrs_sweeps_under_uneven_load():
    """MI355X guide: test every inter-workgroup hand-off under UNEVEN load with L1-warm
    consumers.  The sweeps (sc1 hand-off vector + counter) run on one context while a second
    context keeps the GPU busy with a factorisation (uneven CU occupancy, other XCDs' L2s
    dirty); every result must be bit-identical to an idle-GPU run."""
    n = 4100
    ctx = G.Context(0)
    A = _spd(n, seed=21)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    B = np.random.default_rng(4).random((n, 3))
    dB = ctx.colmajor(B)
    assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                      ctypes.c_void_p(dB.data_ptr()), 3, n) == 0
    ref = ctx.host(dB)
    Xo = O.cho_solve_upper(sla.cholesky(A, lower=False), B)
    assert relnorm(ref, Xo) < 1e-11
    import torch
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        M1 = torch.rand(6144, 6144, dtype=torch.float64, device="cuda")
    side.synchronize()
    for it in range(6):
        # background FP64 GEMMs on another stream, not synchronised with the solves
        with torch.cuda.stream(side):
            for _ in range(4):
                M1 = (M1 @ M1) * (1.0 / 6144)
        for _ in range(3):
            dB = ctx.colmajor(B)
            assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                              ctypes.c_void_p(dB.data_ptr()), 3, n) == 0
            assert np.array_equal(ctx.host(dB), ref), f"iteration {it}: hand-off result differs"
    side.synchronize()


@pytest.mark.parametrize("n", [100, 300, 513, 256, 1040])
@pytest.mark.parametrize("dag_solve", ["0", "1"])
def test_potri_and_trsm(n, dag_solve, monkeypatch):
    """K^{-1} and B <- U^{-T} B from a factor; dag_solve=1: the solve-only tile-DAG (every
    tile of U final, only B's tiles are tasks; lower-triangular B for K^{-1}'s Z = U^{-T})."""
    monkeypatch.setenv("GPR_DAG_SOLVE", dag_solve)
    ctx = G.Context(0)
    A = _spd(n, seed=9)
    dA, info = _dev_potrf(ctx, A)
    dK = ctx.empty(n, n)
    rc = G._lib.lib.gpr_potri_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                   ctypes.c_void_p(dK.data_ptr()), n)
    assert rc == 0
    Kinv = ctx.host(dK)
    assert relnorm(Kinv, np.linalg.inv(A)) < 1e-11
    assert np.array_equal(Kinv, Kinv.T)
    # trsm: B <- U^{-T} B (>= 128 columns at n % 16 == 0: the solve-only tile-DAG)
    U = sla.cholesky(A, lower=False)
    for nr in (37, 300, 260):  # (260: a 4-column last tile)
        B = np.random.default_rng(2).random((n, nr))
        dB = ctx.colmajor(B)
        rc = G._lib.lib.gpr_trsm_upper_trans(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                            ctypes.c_void_p(dB.data_ptr()), nr, n)
        assert rc == 0
        assert relnorm(ctx.host(dB), sla.solve_triangular(U, B, trans="T")) < 1e-11


def test_dag_wait_timeout_drains_and_context_recovers():
    """Every tile-DAG dependency wait is bounded; forced to expire (the test build's
    GPR_DAG_SPIN_LIMIT=1), the launch drains, the call reports the timeout, and the same
    context is correct afterwards (tests/fault_scenarios.py dag_timeout, in a child process on
    libgpr_hip_testing.so -- the release library has no fault injection)."""
    from conftest import run_fault_scenario
    run_fault_scenario("dag_timeout")


# ---------------------------------------------------------------------------------------
# a8/a9 MLL value and gradient  (test/test_loss.jl)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [10, 20, 100])
def test_mll_closed_form_diagonal(n):
    """test/test_loss.jl:1-11: K = Diagonal(x) -> MLL = 0.5(sum y^2/x + sum log x + n log 2pi)."""
    ctx = G.Context(0)
    rng = np.random.default_rng(n)
    xv, y = rng.random(n) + 0.1, rng.random(n)
    MLE = 0.5 * (np.dot(y, y / xv) + np.sum(np.log(xv)) + n * np.log(2 * np.pi))
    dA, info = _dev_potrf(ctx, np.diag(xv))
    dy = ctx.colmajor(y)
    da = ctx.colmajor(y.copy())
    assert G._lib.lib.gpr_potrs_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                                      ctypes.c_void_p(da.data_ptr()), 1, n) == 0
    out = ctypes.c_double()
    assert G._lib.lib.gpr_mll(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,
                              ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(da.data_ptr()),
                              ctypes.byref(out)) == 0
    assert out.value == pytest.approx(MLE, rel=1e-13)


@pytest.mark.parametrize("n,dim", [(10, 2), (20, 5), (100, 2), (100, 5), (333, 3)])
def test_mll_and_grad(n, dim):
    """test/test_loss.jl:22-56: loss, cache contents, per-hp grads vs FD (rtol 1e-3) and
    vs the oracle (rtol 1e-8 relative to the gradient scale)."""
    rng = np.random.default_rng(n + dim)
    x = rng.random((dim, n))
    y = np.sum(np.sin(x), axis=0)
    kinds = [SE, WN]
    hp = np.r_[1.0, rng.uniform(0.5, 2.0, dim), 0.3]
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    L = G.loss(G.MarginalLikelihood(), hp, md)
    assert L == pytest.approx(O.mll(kinds, hp, x, y), rel=1e-10)
    tc = G.MllGradCache(md)
    G.update_cache_(tc, hp, md)
    ctx = md.ctx
    U = sla.cholesky(O.kernel(kinds, hp, x), lower=False)
    assert relnorm(np.triu(ctx.host(tc.kchol_base)), U) < 1e-11
    np.testing.assert_allclose(ctx.host(tc.alpha), O.cho_solve_upper(U, y), rtol=1e-9, atol=1e-12)
    assert relnorm(ctx.host(tc.Kinv), O.kinv_from_upper(U)) < 1e-10
    g = G.grad(G.MarginalLikelihood(), hp, md)
    go = O.mll_grad(kinds, hp, x, y)
    scale = np.max(np.abs(go)) + 1.0
    np.testing.assert_allclose(g, go, rtol=1e-8, atol=1e-8 * scale)
    for i in range(len(hp)):
        hpe = hp.copy()
        hpe[i] += 1e-6
        fd = (O.mll(kinds, hpe, x, y) - O.mll(kinds, hp, x, y)) / 1e-6
        assert g[i] == pytest.approx(fd, rel=1e-3, abs=1e-5)


def test_mll_2d_y_train_axis():
    """test/test_loss.jl:58-97: 2-D y with a train_axis column."""
    rng = np.random.default_rng(4)
    dim, n, ne = 3, 80, 5
    x = rng.random((dim, n))
    y = np.stack([rng.random() * np.sum(np.sin(x), axis=0) for _ in range(ne)], axis=1)
    ta = 3
    hp = np.r_[1.0, [1.2] * dim, 0.2]
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y, train_axis=ta)
    L = G.loss(G.MarginalLikelihood(), hp, md)
    assert L == pytest.approx(O.mll([SE, WN], hp, x, y[:, ta - 1]), rel=1e-10)
    g = G.grad(G.MarginalLikelihood(), hp, md)
    go = O.mll_grad([SE, WN], hp, x, y, train_axis=ta)
    np.testing.assert_allclose(g, go, rtol=1e-8, atol=1e-8 * (1 + np.abs(go).max()))


def test_log_loss_grad_and_composed():
    rng = np.random.default_rng(8)
    dim, n = 4, 150
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    kinds = [SE, SE, WN]
    hp = np.r_[1.0, [2.0] * dim, 0.5, [0.7] * dim, 0.1]
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    tc = G.MllGradCache(md)
    Gv = np.zeros(len(hp))
    F = G.log_loss_grad_(G.MarginalLikelihood(), 0.0, Gv, np.log(hp), md, tc)
    assert F == pytest.approx(O.mll(kinds, hp, x, y), rel=1e-10)
    go = O.mll_grad(kinds, hp, x, y, log_scale=True)
    np.testing.assert_allclose(Gv, go, rtol=1e-8, atol=1e-8 * (1 + np.abs(go).max()))
    assert isinstance(G.islog(G.MarginalLikelihood(), md), G.LogScale)


# ---------------------------------------------------------------------------------------
# a10/a11 posterior  (test/test_models.jl)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["SE", "SE+WN", "SE+SE", "SE+SE+WN"])
@pytest.mark.parametrize("n,npred,dim", [(100, 100, 1), (200, 500, 2), (500, 200, 5), (333, 77, 8),
                                         (1024, 300, 4)])
def test_predict_vs_oracle(name, n, npred, dim):
    kinds = KSETS[name]
    x, y, xp = O.synthetic(dim, n, npred, seed_train=n, seed_test=npred)
    hp = O.default_hp(kinds, dim, noise=0.05)
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    mu, var = G.predict(md, xp, diagonal_var=True)
    mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    # variances are differences of O(prior) terms: absolute tolerance 1e-8 x prior
    vtol = 1e-8 * O.diag_prior(kinds, hp, dim)
    np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=vtol)
    mu2, S = G.predict(md, xp, diagonal_var=False)
    _, S_o = O.predict(kinds, hp, x, y, xp, diagonal_var=False)
    np.testing.assert_allclose(mu2, mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(S, S_o, rtol=1e-8, atol=vtol)
    np.testing.assert_allclose(G.predict_mean(md, xp), mu_o, rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("n", [100, 200, 500])
@pytest.mark.parametrize("npred", [100, 200, 500])
@pytest.mark.parametrize("dim", [1, 2, 5])
def test_predict_interpolation_random_hp(n, npred, dim):
    """test/test_models.jl:1-31 verbatim: GPRModel(cov, x, y) draws hp = rand(D)
    (src/models.jl:32-37, here seeded), then predict_mean(md2, x) ≈ y rtol 1e-7 and
    predict(md2, x)'s full Sigma ≈ 0 atol 1e-7 with x the model's OWN input: the same-object
    branch of kernel!(Kxp, covar, hp, xp, md.x) (src/predict.jl:37,43) puts eps per SE part
    on Kxp, so Kxp equals K and mu = y up to the solve's backward error for any hp."""
    rng = np.random.default_rng(1000 * n + 10 * npred + dim)
    x = rng.random((dim, n))
    xp = rng.random((dim, npred))
    y = np.sin(x.sum(0)) ** 2
    md2 = G.GPRModel(G.SquaredExp() + G.SquaredExp(), None, x, y, rng=rng)
    assert julia_approx(G.predict_mean(md2, x), y, rtol=1e-7)
    mu2, S = G.predict(md2, x)
    assert julia_approx(mu2, y, rtol=1e-7)
    assert np.abs(S).max() <= 1e-7
    _, Sd = G.predict(md2, x, diagonal_var=True)
    assert np.abs(Sd).max() <= 1e-7
    md3 = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), None, x, y, rng=rng)
    md3.params[-1] = 1e-5
    assert julia_approx(G.predict_mean(md3, x), y, rtol=1e-3)
    _, S3 = G.predict(md3, x)
    assert np.abs(S3).max() <= 1e-3
    # the same-object rule is exactly the oracle's (xp is x), for mean and both variances
    for md, kinds in ((md2, [SE, SE]), (md3, [SE, WN])):
        mu_o, S_o = O.predict(kinds, md.params, x, y, x)
        mu_d, S_d = G.predict(md, x)
        scale = np.linalg.norm(y)
        assert np.linalg.norm(mu_d - mu_o) <= 1e-7 * scale
        assert np.abs(S_d - S_o).max() <= 1e-7
    # a different object with equal values is a cross kernel (no eps): predict(md, copy(x))
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), np.r_[1.0, [3.0] * dim, 0.1], x, y)
    mu_c = G.predict_mean(md, x.copy())
    mu_o = O.predict([SE, WN], md.params, x, y, x.copy(), diagonal_var=True)[0]
    np.testing.assert_allclose(mu_c, mu_o, rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("name", ["SE", "SE+WN", "SE+SE+WN", "WN+SE"])
@pytest.mark.parametrize("diag", [True, False])
def test_predict_same_object_vs_oracle(name, diag):
    """predict(md, md.x) with well-conditioned hp against the oracle's same-object rule, on the
    fused tile-DAG path (n a multiple of 16) and the padded one."""
    kinds = KSETS[name]
    for n, dim in ((256, 3), (250, 2)):
        x, y, _ = O.synthetic(dim, n, 0, seed_train=n)
        hp = O.default_hp(kinds, dim)
        md = G.GPRModel(cov_of(kinds), hp, x, y)
        mu, S = G.predict(md, md.x, diagonal_var=diag)
        mu_o, S_o = O.predict(kinds, hp, x, y, x, diagonal_var=diag)
        vtol = 1e-8 * O.diag_prior(kinds, hp, dim)
        np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(S, S_o, rtol=1e-8, atol=vtol)
        if WN in kinds:  # mu = y - sigma_n^2 alpha exactly (Kxp = K - sigma_n^2 I)
            alpha = O.cho_solve_upper(O.chol_upper(O.kernel(kinds, hp, x)), y)
            sn = O.split_hp(kinds, hp, dim)[kinds.index(WN)][0]
            np.testing.assert_allclose(mu, y - sn ** 2 * alpha, rtol=1e-8, atol=1e-10)


def test_kernel_same_object_forms():
    """gpr_kernel's `same` argument: GPR_SELF = 4-arg kernel!(K, cov, hp, x) (eps + noise),
    GPR_SAME_OBJECT = 5-arg with x === xp (eps per SE part, no noise; src/compose_covar.jl:47-61),
    and an invalid value is rejected."""
    rng = np.random.default_rng(31)
    dim, n = 4, 160
    x = rng.random((dim, n))
    for name in ("SE", "SE+WN", "SE+SE+WN", "WN+SE", "SE+WN+SE"):
        kinds = KSETS[name]
        hp = rand_hp(kinds, dim, rng)
        cov = cov_of(kinds)
        np.testing.assert_allclose(G.kernel(cov, hp, x, x), O.kernel(kinds, hp, x, x),
                                   rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(G.kernel(cov, hp, x), O.kernel(kinds, hp, x),
                                   rtol=1e-13, atol=1e-15)
    ctx = G.default_context()
    dx = ctx.colmajor(x)
    K = ctx.empty(n, n)
    kinds_c = (ctypes.c_int * 1)(1)
    hp = np.r_[1.0, [1.0] * dim]
    rc = G._lib.lib.gpr_kernel(ctx.h, kinds_c, 1, hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                               dim, ctypes.c_void_p(dx.data_ptr()), n, None, n, 3, 1e-8,
                               ctypes.c_void_p(K.data_ptr()), n)
    assert rc == -1  # GPR_E_ARG


def test_predict_multi_output_y():
    rng = np.random.default_rng(21)
    dim, n, ne, npred = 3, 150, 4, 60
    x, xp = rng.random((dim, n)), rng.random((dim, npred))
    y = np.stack([np.sin(x.sum(0) * (k + 1)) for k in range(ne)], axis=1)
    kinds = [SE, WN]
    hp = O.default_hp(kinds, dim)
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    mu = G.predict_mean(md, xp)
    K = O.kernel(kinds, hp, x)
    U = O.chol_upper(K)
    mu_o = O.kernel(kinds, hp, xp, x) @ O.cho_solve_upper(U, y)
    np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)


# ---------------------------------------------------------------------------------------
# a12-a15 split kernel  (test/test_split_kernel.jl)
# ---------------------------------------------------------------------------------------
def test_split_factors_and_identity():
    rng = np.random.default_rng(13)
    for dim, n in [(2, 100), (3, 26), (5, 200)]:
        x, xe, xq = rng.random((dim, n)), rng.random((dim, n + 17)), rng.random((dim, n - 9))
        kinds = [SE, WN, SE]
        hp = rng.random(2 * dim + 3)
        cm = G.Cmap("+", xe, xq)
        Ao, Bo, Co = O.split_factors(kinds, hp, x, xe, xq)
        for part in (0, 1):
            A, B, C = G.split_factors(cov_of(kinds), hp, x, cm, part)
            np.testing.assert_allclose(A, Ao[:, :, part], rtol=1e-13)
            np.testing.assert_allclose(B, Bo[:, :, part], rtol=1e-13)
            np.testing.assert_allclose(C, Co[:, :, part], rtol=1e-13)
        # SplitCovar identity KK[idx, s] = sum_k A B C  (test/test_split_kernel.jl:36-44)
        KK = O.kernel(kinds, hp, cm.points(), x)
        ne, nq = xe.shape[1], xq.shape[1]
        Ksplit = np.einsum("eqk,esk,sqk->eqs", Ao, Bo, Co).reshape(ne * nq, n, order="F")
        np.testing.assert_allclose(Ksplit, KK, rtol=1e-10)


@pytest.mark.parametrize("name", ["SE", "SE+WN", "SE+SE", "SE+SE+WN"])
@pytest.mark.parametrize("dim,n,e,q", [(1, 100, 10, 10), (2, 200, 20, 30), (5, 500, 50, 10)])
def test_split_predict_reference_identities(name, dim, n, e, q):
    """test/test_split_kernel.jl:49-77 with the reference's random hp: split mean == direct
    mean on xeq[:, :]; the first 3q variance entries equal the direct variance on
    Cmap(+, xq, xe) (e-major layout), entry 3q+1 does not (var_range = 1:3)."""
    kinds = KSETS[name]
    rng = np.random.default_rng(dim * 1000 + n + e + q)
    x, xe, xq = rng.random((dim, n)), rng.random((dim, e)), rng.random((dim, q))
    y = np.sin(x.sum(0)) ** 2
    hp = rng.random(sum(O.dim_hp(k, dim) for k in kinds)) * 0.5 + 0.5
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    yps, varps = G.predict(md, cm, diagonal_var=True)
    yp, _ = G.predict(md, cm.points(), diagonal_var=True)
    assert julia_approx(yps.reshape(-1, order="F"), yp)
    xpt = G.Cmap("+", xq, xe).points()
    _, varpt = G.predict(md, xpt, diagonal_var=True)
    assert julia_approx(varps[:3 * q], varpt[:3 * q], rtol=1e-5)
    assert not julia_approx(varps[:3 * q + 1], varpt[:3 * q + 1], rtol=1e-5)


@pytest.mark.parametrize("name", ["SE", "SE+WN", "SE+SE", "SE+SE+WN"])
@pytest.mark.parametrize("dim,n,e,q", [(4, 200, 20, 30), (5, 500, 50, 10), (8, 640, 33, 17)])
def test_split_predict_vs_oracle(name, dim, n, e, q):
    """Split mean/var vs the oracle at rtol 1e-8 on well-posed hp (SURVEY 8d defaults)."""
    kinds = KSETS[name]
    rng = np.random.default_rng(dim * 7 + n + e + q)
    x, xe, xq = rng.random((dim, n)), 0.5 * rng.random((dim, e)), 0.5 * rng.random((dim, q))
    y = np.sin(x.sum(0)) ** 2
    hp = O.default_hp(kinds, dim, noise=0.05)
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    yps, varps = G.predict(md, cm, diagonal_var=True)
    mu_o, var_o = O.split_predict(kinds, hp, x, y, xe, xq)
    np.testing.assert_allclose(yps, mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(varps, var_o, rtol=1e-8, atol=1e-8 * O.diag_prior(kinds, hp, dim))


def test_split_predict_full_var_range_and_rows():
    """var_range = all rows equals the direct diagonal variance; a row-range call writes only
    its rows (the multi-GPU shard contract)."""
    rng = np.random.default_rng(99)
    dim, n, e, q = 3, 300, 12, 40
    x, xe, xq = rng.random((dim, n)), rng.random((dim, e)), rng.random((dim, q))
    y = np.sin(x.sum(0)) ** 2
    kinds = [SE, WN]
    hp = O.default_hp(kinds, dim)
    md = G.GPRModel(cov_of(kinds), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    mu, var = G.predict(md, cm, diagonal_var=True, var_range=(1, e))
    mu_o, var_o = O.split_predict(kinds, hp, x, y, xe, xq, var_range=(1, e))
    np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=1e-8 * O.diag_prior(kinds, hp, dim))
    # shard rows [4, 9)
    ctx = md.ctx
    pc = G.GPRSplitPredictCache(md, e, q, (1, e))
    from gpr_amd.core import _update_predict_cache, pc_adapter, split_predict_
    _update_predict_cache(pc_adapter(pc), md)
    dmu, dvar = ctx.zeros(q, e), ctx.zeros(e * q)
    split_predict_(md, cm, pc, dmu, dvar, 4, 9)
    m2, v2 = ctx.host(dmu), ctx.host(dvar)
    np.testing.assert_allclose(m2[4:9], mu_o[4:9], rtol=1e-8, atol=1e-10)
    assert np.all(m2[:4] == 0) and np.all(m2[9:] == 0)
    np.testing.assert_allclose(v2[4 * q:9 * q], var_o[4 * q:9 * q], rtol=1e-8, atol=1e-8 * O.diag_prior(kinds, hp, dim))
    assert np.all(v2[:4 * q] == 0) and np.all(v2[9 * q:] == 0)


# ---------------------------------------------------------------------------------------
# a5/a6/a10/a11 fused: predict from scratch with the solve inside the factorisation
# ---------------------------------------------------------------------------------------
def _fit_predict_dev(ctx, kinds, hp, x, y, xp, mode, nb2=None):
    if nb2:
        assert G._lib.lib.gpr_set_outer_block(ctx.h, nb2) == 0
    d, n = x.shape
    m = xp.shape[1]
    y2 = y if y.ndim == 2 else y[:, None]
    nrhs = y2.shape[1]
    dx, dy, dxp = ctx.colmajor(x), ctx.colmajor(y2), ctx.colmajor(xp)
    K = ctx.empty(n, n)
    alpha = ctx.empty(nrhs, n)
    mu = ctx.empty(nrhs, m)
    var = ctx.empty(m) if mode == G.GPR_PREDICT_DIAG else ctx.empty(m, m)
    karr = (ctypes.c_int * len(kinds))(*[1 if k == SE else 2 for k in kinds])
    hpa = np.asarray(hp, dtype=np.float64)
    info = ctypes.c_int(-1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = G._lib.lib.gpr_fit_predict(ctx.h, karr, len(kinds),
                                    hpa.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), d, P(dx),
                                    n, P(dy), nrhs, n, 1e-8, P(K), n, P(alpha), P(dxp), m, mode,
                                    P(mu), P(var), m, None, ctypes.byref(info))
    assert rc == 0 and info.value == 0, G._lib.lib.gpr_last_error(ctx.h)
    return ctx.host(K), ctx.host(alpha), ctx.host(mu), ctx.host(var)


def test_fused_rhs_dropped_by_block_sizes(monkeypatch):
    """The blocked factorisation takes fused right-hand sides only for outer blocks up to
    2048; with a 4096 outer block (GPR_DAG=0) it factors alone and the callers solve after
    it: fit_predict, fit (y inside) and fit_kinv (Z and K^{-1}) stay exact."""
    monkeypatch.setenv("GPR_DAG", "0")
    monkeypatch.setenv("GPR_DAG_TAIL", "0")
    monkeypatch.setenv("GPR_FUSE_Y", "1")
    kinds = KSETS["SE+WN"]
    dim, n, m = 4, 4352, 100
    x, y, xp = O.synthetic(dim, n, m, seed_train=7, seed_test=8)
    hp = O.default_hp(kinds, dim, noise=0.1)
    ctx = G.Context(0)
    _, alpha, mu, var = _fit_predict_dev(ctx, kinds, hp, x, y, xp, G.GPR_PREDICT_DIAG, 4096)
    U = sla.cholesky(O.kernel(kinds, hp, x), lower=False)
    mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    np.testing.assert_allclose(mu.ravel(), mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=1e-8 * O.diag_prior(kinds, hp, dim))
    np.testing.assert_allclose(alpha.ravel(), O.cho_solve_upper(U, y), rtol=1e-8,
                               atol=1e-10 * np.abs(O.cho_solve_upper(U, y)).max())
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, Kinv, a2 = ctx.empty(n, n), ctx.empty(n, n), ctx.empty(n)
    karr = (ctypes.c_int * 2)(1, 2)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    info = ctypes.c_int(-1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert G._lib.lib.gpr_fit(ctx.h, karr, 2, hpp, dim, P(dx), n, P(dy), 1, n, 1e-8, P(K), n,
                              P(a2), ctypes.byref(info)) == 0 and info.value == 0
    np.testing.assert_allclose(ctx.host(a2), O.cho_solve_upper(U, y), rtol=1e-8,
                               atol=1e-10 * np.abs(O.cho_solve_upper(U, y)).max())
    assert G._lib.lib.gpr_fit_kinv(ctx.h, karr, 2, hpp, dim, P(dx), n, P(dy), 1, n, 1e-8, P(K),
                                   n, P(a2), P(Kinv), n, ctypes.byref(info)) == 0
    assert info.value == 0
    Ki = ctx.host(Kinv)
    assert np.array_equal(Ki, Ki.T) and relnorm(Ki, O.kinv_from_upper(U)) < 1e-10


@pytest.mark.parametrize("fused", ["1", "2", "0"])
@pytest.mark.parametrize("name,n,npred,dim,nb2", [
    ("SE+WN", 300, 77, 3, None), ("SE+SE+WN", 1300, 200, 8, 256), ("SE+WN", 1025, 64, 2, 1024),
    ("SE+WN", 2600, 500, 5, 1024), ("SE+SE", 700, 1000, 4, 512)])
def test_fit_predict_fused_vs_oracle(name, n, npred, dim, nb2, fused, monkeypatch):
    """gpr_fit_predict = predict(md, xp; diagonal_var) from scratch (src/predict.jl:14-71):
    U in the upper triangle (lower keeps K), alpha, mean and variance vs the oracle, across
    outer-panel boundaries (the solve rides inside the factorisation) and ragged panels;
    fused=0 is the unfused reference order (gpr_fit + gpr_predict)."""
    monkeypatch.setenv("GPR_FUSED_RHS", fused)
    if fused != "0":  # the right-hand sides inside the BLOCKED factorisation
        monkeypatch.setenv("GPR_DAG", "0")
        monkeypatch.setenv("GPR_DAG_TAIL", "0")
    kinds = KSETS[name]
    x, y, xp = O.synthetic(dim, n, npred, seed_train=n, seed_test=npred)
    hp = O.default_hp(kinds, dim, noise=0.05)
    ctx = G.Context(0)
    Kd, alpha, mu, var = _fit_predict_dev(ctx, kinds, hp, x, y, xp, G.GPR_PREDICT_DIAG, nb2)
    K = O.kernel(kinds, hp, x)
    U = sla.cholesky(K, lower=False)
    # the lower triangle keeps K; the upper holds the factor of exactly that K
    np.testing.assert_allclose(np.tril(Kd, -1), np.tril(K, -1), rtol=1e-13, atol=1e-15)
    Kdev = np.tril(Kd) + np.tril(Kd, -1).T
    np.fill_diagonal(Kdev, np.diag(K))
    assert relnorm(np.triu(Kd), sla.cholesky(Kdev, lower=False)) < 1e-11
    np.testing.assert_allclose(alpha.ravel(), O.cho_solve_upper(U, y), rtol=1e-8,
                               atol=1e-10 * np.abs(O.cho_solve_upper(U, y)).max())
    mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    vtol = 1e-8 * O.diag_prior(kinds, hp, dim)
    np.testing.assert_allclose(mu.ravel(), mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=vtol)
    if n <= 1300:
        _, _, mu2, S = _fit_predict_dev(ctx, kinds, hp, x, y, xp, G.GPR_PREDICT_FULL, nb2)
        _, S_o = O.predict(kinds, hp, x, y, xp, diagonal_var=False)
        np.testing.assert_allclose(mu2.ravel(), mu_o, rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(S, S_o, rtol=1e-8, atol=vtol)


@pytest.mark.parametrize("name,n,npred,dim", [("SE+WN", 1040, 200, 3), ("SE+SE+WN", 2048, 300, 8),
                                               ("SE+WN", 4112, 130, 4), ("SE", 256, 77, 8),
                                               ("SE+WN", 1001, 150, 5), ("SE+SE", 333, 64, 3),
                                               ("SE+SE+WN", 2048, 256, 8), ("SE+WN", 1040, 140, 3)])
def test_fit_predict_dag_vs_oracle(name, n, npred, dim, monkeypatch):
    """gpr_fit_predict with the tile-DAG (GPR_DAG=1): V = U^{-T} [K(x, xp) | y] solved by
    right-hand-side tile tasks of the same persistent launch as the factorisation (np + 1 =
    131, 257, 141: a last column tile of 3, 1, 13 columns)."""
    monkeypatch.setenv("GPR_FUSED_RHS", "2")
    monkeypatch.setenv("GPR_DAG", "1")
    kinds = KSETS[name]
    x, y, xp = O.synthetic(dim, n, npred, seed_train=n, seed_test=npred)
    hp = O.default_hp(kinds, dim, noise=0.05)
    ctx = G.Context(0)
    Kd, alpha, mu, var = _fit_predict_dev(ctx, kinds, hp, x, y, xp, G.GPR_PREDICT_DIAG, None)
    K = O.kernel(kinds, hp, x)
    U = sla.cholesky(K, lower=False)
    np.testing.assert_allclose(np.tril(Kd, -1), np.tril(K, -1), rtol=1e-13, atol=1e-15)
    Kdev = np.tril(Kd) + np.tril(Kd, -1).T
    np.fill_diagonal(Kdev, np.diag(K))
    assert relnorm(np.triu(Kd), sla.cholesky(Kdev, lower=False)) < 1e-11
    np.testing.assert_allclose(alpha.ravel(), O.cho_solve_upper(U, y), rtol=1e-8,
                               atol=1e-10 * np.abs(O.cho_solve_upper(U, y)).max())
    mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    vtol = 1e-8 * O.diag_prior(kinds, hp, dim)
    np.testing.assert_allclose(mu.ravel(), mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=vtol)
    _, _, mu2, S = _fit_predict_dev(ctx, kinds, hp, x, y, xp, G.GPR_PREDICT_FULL, None)
    _, S_o = O.predict(kinds, hp, x, y, xp, diagonal_var=False)
    np.testing.assert_allclose(mu2.ravel(), mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(S, S_o, rtol=1e-8, atol=vtol)


def test_fit_predict_multi_output_and_reuse():
    """Multi-column y (md.y N x ne, src/predict.jl:32 solves against all columns); the factor
    and square inverses left by the fused call serve later solves on the same context."""
    kinds = KSETS["SE+WN"]
    dim, n, m = 4, 1100, 150
    x, _, xp = O.synthetic(dim, n, m, seed_train=5, seed_test=6)
    Y = np.stack([np.sin(x.sum(0)), np.cos(x[0]) + x[1]], axis=1)
    hp = O.default_hp(kinds, dim, noise=0.05)
    ctx = G.Context(0)
    assert G._lib.lib.gpr_set_outer_block(ctx.h, 512) == 0
    Kd, alpha, mu, var = _fit_predict_dev(ctx, kinds, hp, x, Y, xp, G.GPR_PREDICT_DIAG)
    K = O.kernel(kinds, hp, x)
    U = sla.cholesky(K, lower=False)
    Kxp = O.kernel(kinds, hp, xp, x)
    for c in range(2):
        a_o = O.cho_solve_upper(U, Y[:, c])
        np.testing.assert_allclose(alpha[:, c], a_o, rtol=1e-8, atol=1e-10 * np.abs(a_o).max())
        np.testing.assert_allclose(mu[:, c], Kxp @ a_o, rtol=1e-8, atol=1e-10)
    # reuse: a TRSM against the fused factor on the same context
    B = np.random.default_rng(1).random((n, 5))
    dB = ctx.colmajor(B)
    dK = ctx.colmajor(Kd)
    assert G._lib.lib.gpr_trsm_upper_trans(ctx.h, ctypes.c_void_p(dK.data_ptr()), n, n,
                                           ctypes.c_void_p(dB.data_ptr()), 5, n) == 0
    assert relnorm(ctx.host(dB), sla.solve_triangular(U, B, trans="T")) < 1e-11


@pytest.mark.parametrize("fuse", ["2", "1", "0"])
@pytest.mark.parametrize("n,nb2", [(300, None), (1300, 256), (2100, 1024), (777, 512), (1040, None),
                                   (2048, None), (4096, None), (16, None), (144, None),
                                   (2064, None)])
def test_fit_kinv(n, nb2, fuse, monkeypatch):
    """gpr_fit_kinv = update_cache!(::MllGradCache) (src/cost.jl:83-111): U, alpha and the
    dense K^{-1}, with Z = U^{-T} solved inside the factorisation and K^{-1} = Z^T Z
    accumulated there (fuse=2: gram tile tasks of the tile-DAG launch at n % 16 == 0 --
    1040 with a short last row block, 2048, 4096 -- else panel by panel in the blocked
    factorisation), Z alone inside (fuse=1), or both after it."""
    monkeypatch.setenv("GPR_FUSE_KINV", fuse)
    kinds = KSETS["SE+WN"]
    dim = 4
    x, y, _ = O.synthetic(dim, n, 0, seed_train=n)
    hp = O.default_hp(kinds, dim, noise=0.1)
    ctx = G.Context(0)
    if nb2:
        assert G._lib.lib.gpr_set_outer_block(ctx.h, nb2) == 0
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, Kinv, alpha = ctx.empty(n, n), ctx.empty(n, n), ctx.empty(n)
    karr = (ctypes.c_int * 2)(1, 2)
    info = ctypes.c_int(-1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = G._lib.lib.gpr_fit_kinv(ctx.h, karr, 2, hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 dim, P(dx), n, P(dy), 1, n, 1e-8, P(K), n, P(alpha), P(Kinv), n,
                                 ctypes.byref(info))
    assert rc == 0 and info.value == 0
    Ko = O.kernel(kinds, hp, x)
    Uo = sla.cholesky(Ko, lower=False)
    Kd = ctx.host(K)
    assert relnorm(np.triu(Kd), Uo) < 1e-11
    np.testing.assert_allclose(ctx.host(alpha), O.cho_solve_upper(Uo, y), rtol=1e-9, atol=1e-12)
    Ki = ctx.host(Kinv)
    assert np.array_equal(Ki, Ki.T)
    assert relnorm(Ki, O.kinv_from_upper(Uo)) < 1e-10


# ---------------------------------------------------------------------------------------
# Upper-only K assembly for a factorisation + the tile-DAG's lower mirror (round 4): the fit
# buffer must still end as the reference's cholesky!(Hermitian(K)) leaves it -- upper U,
# strict lower K (test/test_loss.jl:46 compares whole cache buffers) -- and equal,
# bit for bit, the full symmetric build (gpr_kernel) factored by gpr_potrf_upper.
# ---------------------------------------------------------------------------------------
def _P(t):
    return ctypes.c_void_p(t.data_ptr())


def _karr(kinds):
    return (ctypes.c_int * len(kinds))(*[1 if k == SE else 2 for k in kinds])


def _ref_buffer(ctx, kinds, hp, x, eps=1e-8):
    """gpr_kernel (full symmetric K, GPR_SELF) + gpr_potrf_upper on a second buffer."""
    d, n = x.shape
    dx = ctx.colmajor(x)
    K = ctx.empty(n, n)
    karr = _karr(kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    assert G._lib.lib.gpr_kernel(ctx.h, karr, len(kinds), hpp, d, _P(dx), n, None, n, 1, eps,
                                 _P(K), n) == 0
    Kfull = ctx.host(K).copy()
    info = ctypes.c_int(-7)
    assert G._lib.lib.gpr_potrf_upper(ctx.h, _P(K), n, n, ctypes.byref(info)) >= 0
    return ctx.host(K), Kfull, info.value


@pytest.mark.parametrize("name", ["SE", "SE+WN", "SE+SE+WN", "SE+SE"])
@pytest.mark.parametrize("n,dim", [(128, 3), (144, 8), (1040, 8), (2064, 5), (4096, 8), (1024, 16)])
@pytest.mark.parametrize("call", ["fit", "fit_predict", "fit_kinv"])
def test_fit_buffer_upper_build_dag_mirror(name, n, dim, call):
    kinds = KSETS[name]
    rng = np.random.default_rng(n + dim)
    hp = O.default_hp(kinds, dim, noise=0.1)
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    ctx = G.Context(0)
    Rref, Kfull, info_ref = _ref_buffer(ctx, kinds, hp, x)
    assert info_ref == 0
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, alpha = ctx.empty(n, n), ctx.empty(n)
    karr = _karr(kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    info = ctypes.c_int(-7)
    lib = G._lib.lib
    if call == "fit":
        rc = lib.gpr_fit(ctx.h, karr, len(kinds), hpp, dim, _P(dx), n, _P(dy), 1, n, 1e-8, _P(K), n,
                         _P(alpha), ctypes.byref(info))
    elif call == "fit_predict":
        m = 37
        xp = rng.random((dim, m))
        dxp = ctx.colmajor(xp)
        mu, var, W = ctx.empty(m), ctx.empty(m), ctx.empty(m + 1, n)
        rc = lib.gpr_fit_predict(ctx.h, karr, len(kinds), hpp, dim, _P(dx), n, _P(dy), 1, n, 1e-8,
                                 _P(K), n, _P(alpha), _P(dxp), m, 1, _P(mu), _P(var), m, _P(W),
                                 ctypes.byref(info))
    else:
        Kinv = ctx.empty(n, n)
        rc = lib.gpr_fit_kinv(ctx.h, karr, len(kinds), hpp, dim, _P(dx), n, _P(dy), 1, n, 1e-8, _P(K),
                              n, _P(alpha), _P(Kinv), n, ctypes.byref(info))
    assert rc == 0 and info.value == 0, lib.gpr_last_error(ctx.h)
    R = ctx.host(K)
    assert np.array_equal(R, Rref)                       # the whole buffer, bit for bit
    assert np.array_equal(np.tril(R, -1), np.tril(Kfull, -1))
    Ko = O.kernel(kinds, hp, x, None)
    np.testing.assert_allclose(np.tril(R, -1), np.tril(Ko, -1), rtol=1e-13, atol=1e-300)
    assert relnorm(np.triu(R), sla.cholesky(Ko, lower=False)) < 1e-11


@pytest.mark.parametrize("env", [("GPR_DAG_GRAM", "0"), ("GPR_KBUILD_UPPER", "0")])
def test_fit_buffer_upper_build_other_paths(env, monkeypatch):
    """The upper-only build with a factorisation the DAG does not take as one launch
    (gpr_fit_kinv with GPR_DAG_GRAM=0: the blocked path, which mirrors the strict lower first)
    and with the upper-only build switched off: the same buffer as the full build."""
    monkeypatch.setenv(*env)
    kinds = KSETS["SE+WN"]
    dim, n = 6, 1536
    rng = np.random.default_rng(3)
    hp = O.default_hp(kinds, dim, noise=0.1)
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    ctx = G.Context(0)
    Rref, Kfull, _ = _ref_buffer(ctx, kinds, hp, x)
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, alpha, Kinv = ctx.empty(n, n), ctx.empty(n), ctx.empty(n, n)
    karr = _karr(kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    info = ctypes.c_int(-7)
    rc = G._lib.lib.gpr_fit_kinv(ctx.h, karr, 2, hpp, dim, _P(dx), n, _P(dy), 1, n, 1e-8, _P(K), n,
                                 _P(alpha), _P(Kinv), n, ctypes.byref(info))
    assert rc == 0 and info.value == 0
    R = ctx.host(K)
    assert np.array_equal(np.tril(R, -1), np.tril(Kfull, -1))
    assert relnorm(np.triu(R), np.triu(Rref)) < 1e-12


@pytest.mark.parametrize("eps,fails_at", [(-0.012, 625), (-1.1, 1)])
def test_fit_buffer_not_posdef_keeps_lower_k(eps, fails_at):
    """A failing pivot (info > 0): the tasks after it skip their arithmetic, but the strict lower
    triangle still ends as K everywhere (dpotrf leaves it untouched), as with the full build."""
    kinds = KSETS["SE+WN"]
    dim, n = 4, 1024
    x, y, _ = O.synthetic(dim, n, 0, seed_train=3)
    hp = O.default_hp(kinds, dim, noise=0.1)
    ctx = G.Context(0)
    Ko = O.kernel(kinds, hp, x, None, eps=eps)
    _, info_ref = sla.lapack.dpotrf(Ko, lower=0)
    assert info_ref == fails_at
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    K, alpha = ctx.empty(n, n), ctx.empty(n)
    karr = _karr(kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    info = ctypes.c_int(-7)
    rc = G._lib.lib.gpr_fit(ctx.h, karr, 2, hpp, dim, _P(dx), n, _P(dy), 1, n, eps, _P(K), n,
                            _P(alpha), ctypes.byref(info))
    assert rc == info.value == fails_at
    _, Kfull, _ = _ref_buffer(ctx, kinds, hp, x, eps=eps)
    assert np.array_equal(np.tril(ctx.host(K), -1), np.tril(Kfull, -1))


@pytest.mark.parametrize("n,dim", [(1040, 8), (2064, 5), (4096, 8), (4100, 3), (4099, 3)])
def test_kbuild_colstore_bitwise(n, dim, knobs):
    """GPR_KBUILD_COLSTORE (single-part upper builds of the fits: interior items staged through
    LDS and stored as 1-KB column segments) changes only the store shape: the fit's buffer
    (upper U, strict lower K) is bit for bit that of the MFMA-layout stores (and gpr_kernel's
    full symmetric K, which keeps the MFMA layout, is unchanged by the knob), including the ragged and diagonal items that keep the old path (n = 4100: odd
    leading dimension -> the 16-B path declines)."""
    kinds = KSETS["SE"]
    rng = np.random.default_rng(n * dim)
    hp = O.default_hp(kinds, dim)
    x = rng.random((dim, n))
    y = np.sin(x.sum(0)) ** 2
    ctx = G.core.default_context()
    dx, dy = ctx.colmajor(x), ctx.colmajor(y)
    karr = _karr(kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    lib = G._lib.lib
    out = {}
    for cs in (0, 1):
        knobs("GPR_KBUILD_COLSTORE", cs)
        K, alpha = ctx.empty(n, n), ctx.empty(n)
        info = ctypes.c_int(-7)
        assert lib.gpr_fit(ctx.h, karr, 1, hpp, dim, _P(dx), n, _P(dy), 1, n, 1e-8, _P(K), n,
                           _P(alpha), ctypes.byref(info)) == 0 and info.value == 0
        Kf = ctx.empty(n, n)
        assert lib.gpr_kernel(ctx.h, karr, 1, hpp, dim, _P(dx), n, None, n, 1, 1e-8, _P(Kf), n) == 0
        out[cs] = (ctx.host(K).copy(), ctx.host(alpha).copy(), ctx.host(Kf).copy())
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    np.testing.assert_allclose(out[1][2], O.kernel(kinds, hp, x), rtol=1e-13, atol=1e-300)
