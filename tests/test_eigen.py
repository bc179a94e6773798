"""The hand-written symmetric eigensolver behind the sample_noise quadrature -- the reference's
LAPACK.syevr! (src/integrate.jl:71-80), whose consumer (inverse_diagonal_update!, :81-104) only
ever needs lambda and P^T B: the tridiagonal reduction (csrc/tridiag.hip, dsytrd) followed by
divide and conquer on T (csrc/dstedc.hip, dstedc), block Jacobi (csrc/eigen.hip) beyond their
size bounds.

gpr_syev_apply returns lambda and P^T B, never P; the checks are therefore on what is
basis-independent:
  * eigenvalues vs numpy.linalg.eigvalsh (sorted), |diff| <= 4 n eps ||A||_2 (backward
    stability's bound, which LAPACK's own answer shares)
  * column norms of B preserved: ||P^T b|| = ||b|| (P orthogonal), rtol 1e-13
  * the quantity the quadrature uses: (P^T B)^T diag(1/(lambda + s)) (P^T B) =
    B^T (A + s I)^{-1} B, relative 1e-10 x cond(A + s I) for several shifts s (negative ones
    included: the reference's eigen path takes any shift)
on random symmetric matrices (ragged sizes, 1 to 1100) and on the reference's own SE kernel
matrices (ill-conditioned, clustered spectra).  The oracle here is numpy's LAPACK.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import gpr_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gpr_amd")


def _syev(ctx, A, B):
    n = A.shape[0]
    m = B.shape[1]
    dA, dB = ctx.colmajor(A), ctx.colmajor(B)
    lam = ctx.empty(max(n, 1))
    sw = ctypes.c_int(-1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = G._lib.lib.gpr_syev_apply(ctx.h, P(dA), n, max(n, 1), P(dB), m, max(n, 1), P(lam),
                                   ctypes.byref(sw))
    assert rc == 0, G._lib.lib.gpr_last_error(ctx.h)
    return ctx.host(lam)[:n], ctx.host(dB), sw.value


def _check(A, lam, C, B, shifts):
    n = A.shape[0]
    nrm = np.linalg.norm(A, 2)
    ref = np.linalg.eigvalsh(A)
    eps = np.finfo(float).eps
    assert np.max(np.abs(np.sort(lam) - ref)) <= 4 * n * eps * max(nrm, 1e-300) + 1e-300
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-13)
    for s in shifts:
        M = A + s * np.eye(n)
        want = B.T @ np.linalg.solve(M, B)
        got = C.T @ (C / (lam + s)[:, None])
        ev = np.abs(ref + s)
        cond = ev.max() / ev.min()
        np.testing.assert_allclose(got, want, rtol=1e-10 * cond, atol=1e-10 * cond * np.abs(want).max())


@pytest.mark.parametrize("n", [1, 2, 5, 31, 64, 65, 100, 129, 300, 511, 1100])
def test_syev_random_symmetric(n):
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    B = rng.standard_normal((n, 3))
    ctx = G.Context(0)
    lam, C, sweeps = _syev(ctx, A, B)
    assert 0 <= sweeps < 60
    ref = np.linalg.eigvalsh(A)
    gap = np.min(np.abs(ref))
    _check(A, lam, C, B, [s for s in (0.0, 0.5, -0.7) if np.min(np.abs(ref + s)) > 1e-3 * max(gap, 1e-3)])


@pytest.mark.parametrize("kinds,dim,n,length", [([O.SE], 2, 150, 2.0), ([O.SE, O.WN], 3, 300, 2.0),
                                               ([O.SE], 4, 1100, 2.0), ([O.SE], 1, 100, 1.0)])
def test_syev_se_kernel_matrices(kinds, dim, n, length):
    """The reference's matrices: K of SquaredExp (+ WhiteNoise) on U[0,1) points -- PSD, a
    spectrum decaying to the 1e-8 jitter plateau (clusters of nearly equal eigenvalues)."""
    rng = np.random.default_rng(dim * n)
    x = rng.random((dim, n))
    hp = O.default_hp(kinds, dim, length=length, noise=0.05)
    K = O.kernel(kinds, hp, x)
    B = np.c_[rng.random((n, 2)), O.antideriv_se(x, hp, np.zeros(dim), np.ones(dim))]
    ctx = G.Context(0)
    lam, C, _ = _syev(ctx, K, B)
    lmin = np.linalg.eigvalsh(K).min()
    _check(K, lam, C, B, [1e-3, 1e-5, -0.5 * lmin if lmin > 1e-6 else 1e-2])


def _perm_of(lam, C, d, B):
    """(lam, rows of C) is (d, rows of B) in some order, exactly."""
    used = set()
    for i in range(len(lam)):
        hit = [j for j in range(len(d)) if j not in used and d[j] == lam[i]
               and np.array_equal(B[j], C[i])]
        assert hit, f"eigenpair {i} ({lam[i]}) is not one of the inputs"
        used.add(hit[0])


def test_syev_diagonal_and_zero():
    """Already diagonal (no reflector, every z deflated: exact, in some order), the zero
    matrix, and a 2 x 2 block."""
    ctx = G.Context(0)
    d = np.array([3.0, -1.0, 2.0, 0.0, 7.5])
    B = np.arange(10.0).reshape(5, 2)
    lam, C, sweeps = _syev(ctx, np.diag(d), B)
    _perm_of(lam, C, d, B)
    lam, C, _ = _syev(ctx, np.zeros((70, 70)), np.ones((70, 1)))
    assert np.array_equal(lam, np.zeros(70)) and np.array_equal(C, np.ones((70, 1)))
    A = np.array([[2.0, 1.0], [1.0, 2.0]])
    lam, C, _ = _syev(ctx, A, np.eye(2))
    np.testing.assert_allclose(np.sort(lam), [1.0, 3.0], rtol=1e-15)
    np.testing.assert_allclose(np.abs(C), np.sqrt(0.5), rtol=1e-15)


@pytest.mark.parametrize("quad", ["1", "3", "4", "auto"])
def test_integrate_noise_native_routes_vs_oracle(quad, knobs):
    """The hand-written routes (GPR_QUAD_EIGEN=1 tridiagonal solves, 3 divide and conquer, 4
    block Jacobi) and the default (here the batched factorisations: every shift above
    -lambda_min) against the oracle's eigen path.  The release library has no rocSOLVER
    comparator: route 2 is refused with GPR_E_ARG (it lives in libgpr_hip_testing.so, checked
    by test_integrate_noise_rocsolver_comparator_test_build)."""
    if quad != "auto":
        knobs("GPR_QUAD_EIGEN", int(quad))
    dim, n, ne = 3, 600, 6
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(9)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y)
    a, b = np.zeros(dim), np.ones(dim)
    noise = np.r_[1e-3 * (1.0 + rng.random(ne - 1)), -1e-3]
    I, v = G.integrate(md, a, b, sample_noise=noise)
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I, Io, rtol=1e-8)
    np.testing.assert_allclose(v, vo, rtol=1e-7, atol=1e-12 * O.antideriv2_se(hp, a, b))
    if os.path.basename(G._lib.LIB_PATH) == "libgpr_hip.so":  # (the release build)
        knobs("GPR_QUAD_EIGEN", 2)
        with pytest.raises(G.GprError, match="test build"):
            G.integrate(md, a, b, sample_noise=noise)


def test_integrate_noise_rocsolver_comparator_test_build():
    """rocSOLVER's dsyevd as a comparator (GPR_QUAD_EIGEN=2, compiled into the test build only):
    the same integrals as the hand-written route 1 and the oracle (tests/fault_scenarios.py
    quad_rocsolver, child process on libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("quad_rocsolver")


@pytest.mark.parametrize("n,mult", [(64, 8), (300, 50), (1000, 333), (2049, 700)])
def test_syev_clustered_spectrum(n, mult):
    """Eigenvalues repeated exactly `mult` times (plus a few singles): the divide-and-conquer's
    close-pair deflation (Givens rotations) on every merge; eigenvalues and P^T B as always."""
    rng = np.random.default_rng(n + mult)
    Qm, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = np.repeat(np.arange(1.0, n // mult + 2), mult)[:n]
    ev[-3:] = [50.0, -7.0, 1e-3]
    A = (Qm * ev) @ Qm.T
    A = (A + A.T) / 2
    B = rng.standard_normal((n, 4))
    ctx = G.Context(0)
    lam, C, _ = _syev(ctx, A, B)
    _check(A, lam, C, B, [0.5, -0.25])


@pytest.mark.parametrize("n", [4096])
def test_syev_se_kernel_large(n):
    """An SE kernel matrix at the quadrature's largest measured size (d = 4, l = 2)."""
    rng = np.random.default_rng(n)
    x = rng.random((4, n))
    hp = np.r_[1.0, [2.0] * 4]
    K = O.kernel([O.SE], hp, x)
    B = np.c_[rng.random((n, 2)), O.antideriv_se(x, hp, np.zeros(4), np.ones(4))]
    ctx = G.Context(0)
    lam, C, _ = _syev(ctx, K, B)
    _check(K, lam, C, B, [1e-3, 1e-5])


# ---- the tridiagonal reduction (gpr_sytrd_apply: dsytrd, syevr's first stage) -------------
def _sytrd(ctx, A, B):
    n = A.shape[0]
    m = 0 if B is None else B.shape[1]
    dA = ctx.colmajor(A)
    dB = ctx.colmajor(B) if m else None
    dd, de = ctx.empty(max(n, 1)), ctx.empty(max(n - 1, 1))
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    rc = G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, max(n, 1), P(dB), m, max(n, 1), P(dd), P(de))
    assert rc == 0, G._lib.lib.gpr_last_error(ctx.h)
    d = ctx.host(dd)[:n]
    e = ctx.host(de)[:max(n - 1, 0)]
    return d, e, (ctx.host(dB) if m else None)


def _tri(d, e):
    return np.diag(d) + np.diag(e, 1) + np.diag(e, -1)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 17, 64, 65, 129, 257, 300, 1100, 5500])
def test_sytrd_random_symmetric(n):
    """Q^T A Q = T and Q^T Q = I to rounding (Q^T from B = I), T's eigenvalues are A's.
    (5500: the deferred-update variant, with B = I past the fused width -- the back-transform
    by reflector blocks over the V it leaves.)"""
    rng = np.random.default_rng(100 + n)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    ctx = G.Context(0)
    d, e, Qt = _sytrd(ctx, A, np.eye(n))
    T = _tri(d, e)
    eps = np.finfo(float).eps
    nrm = max(np.linalg.norm(A, 2), 1e-300)
    assert np.linalg.norm(Qt @ Qt.T - np.eye(n)) <= 20 * n * eps
    assert np.linalg.norm(Qt @ A @ Qt.T - T) <= 20 * n * eps * nrm
    assert np.max(np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A))) <= 4 * n * eps * nrm


@pytest.mark.parametrize("kinds,dim,n", [([O.SE], 2, 150), ([O.SE, O.WN], 3, 300), ([O.SE], 4, 1100),
                                         ([O.SE], 3, 2048), ([O.SE, O.WN], 8, 4096)])
def test_sytrd_se_kernel_matrices_quadratic_form(kinds, dim, n):
    """The reference's matrices (spectrum decaying to the 1e-8 jitter plateau): the quantity the
    quadrature uses, B^T (K + s I)^{-1} B = (Q^T B)^T (T + s I)^{-1} (Q^T B), for positive and
    negative shifts, relative 1e-10 x cond(K + s I); column norms of Q^T B preserved."""
    import scipy.linalg as sla
    rng = np.random.default_rng(dim * n)
    x = rng.random((dim, n))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    K = O.kernel(kinds, hp, x)
    B = np.c_[rng.random((n, 2)), O.antideriv_se(x, hp, np.zeros(dim), np.ones(dim))]
    ctx = G.Context(0)
    d, e, C = _sytrd(ctx, K, B)
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-13)
    lam = np.linalg.eigvalsh(K)
    for s in (1e-3, 1e-5, -0.5 * lam.min() if lam.min() > 1e-6 else 1e-2):
        want = B.T @ np.linalg.solve(K + s * np.eye(n), B)
        got = C.T @ sla.solve_banded((1, 1), np.vstack([np.r_[0.0, e], d + s, np.r_[e, 0.0]]), C)
        ev = np.abs(lam + s)
        cond = ev.max() / ev.min()
        np.testing.assert_allclose(got, want, rtol=1e-10 * cond,
                                   atol=1e-10 * cond * np.abs(want).max())


@pytest.mark.parametrize("n,m", [(300, 1500), (1030, 1025), (2049, 1100)])
def test_sytrd_wide_rhs_blocked_matches_fused(n, m):
    """Q^T B for m > 1024 (64-reflector blocks after the launch, the [G | W] products split over
    row slices) against Q^T B for the same A formed inside the launch (B = I, or B's columns in
    pieces of <= 1024): the two paths agree to rounding, and column norms are preserved."""
    rng = np.random.default_rng(n + m)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    B = rng.standard_normal((n, m))
    ctx = G.Context(0)
    d, e, C = _sytrd(ctx, A, B)
    pieces = [_sytrd(ctx, A, B[:, c:c + 1000])[2] for c in range(0, m, 1000)]
    d2, e2, _ = _sytrd(ctx, A, None)
    assert np.array_equal(d, d2) and np.array_equal(e, e2)
    np.testing.assert_allclose(C, np.hstack(pieces), rtol=0, atol=1e-12 * np.abs(B).max() * np.sqrt(n))
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-13)


def test_sytrd_diagonal_and_zero():
    """Nothing to reduce: T = A and Q = I exactly (every tau = 0)."""
    ctx = G.Context(0)
    dg = np.array([3.0, -1.0, 2.0, 0.0, 7.5, 1.0])
    d, e, C = _sytrd(ctx, np.diag(dg), np.eye(6))
    assert np.array_equal(d, dg) and np.array_equal(e, np.zeros(5)) and np.array_equal(C, np.eye(6))
    d, e, _ = _sytrd(ctx, np.zeros((70, 70)), None)
    assert not d.any() and not e.any()


def test_sytrd_handoff_timeout_drains_and_context_recovers():
    """The reduction's hand-off polls are bounded; with one partial sum never published (the
    test build's GPR_TRD_FAIL_STEP), every workgroup gives up, the call reports the time-out,
    and the same context reduces correctly afterwards (tests/fault_scenarios.py trd_timeout, in
    a child process on libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("trd_timeout")


def test_sytrd_deferred_updates_small_n():
    """The deferred-update reduction (n >= 5376 by default) forced at n = 100 .. 4100 in the test
    build, with every panel but the last 64 steps deferred: eigenvalues, Q^T B norms and a
    shifted quadratic form against numpy, once under late-wave injection, and a hand-off
    time-out inside a deferred panel (tests/fault_scenarios.py trd_df_small)."""
    from conftest import run_fault_scenario
    run_fault_scenario("trd_df_small", timeout=600)


@pytest.mark.parametrize("n", [3000, 5500])
def test_sytrd_fused_vs_blocked_back_transform(n):
    """Q^T B two ways from the same reduction: B of 1000 columns is transformed inside the
    launch (at P = 256 workgroups: four columns per workgroup, one wave each), B of 1100 columns
    afterwards by 64-reflector blocks on the MFMA GEMM.  The same d and e bit for bit, and the
    first 1000 columns of Q^T B agree to rounding (LDS variant at 3000, deferred-update at
    5500)."""
    rng = np.random.default_rng(n + 1)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    B = rng.standard_normal((n, 1100))
    ctx = G.Context(0)
    d1, e1, C1 = _sytrd(ctx, A, B[:, :1000])
    d2, e2, C2 = _sytrd(ctx, A, B)
    assert np.array_equal(d1, d2) and np.array_equal(e1, e2)
    scale = np.linalg.norm(B[:, :1000], axis=0)
    assert np.max(np.abs(C1 - C2[:, :1000]) / scale) <= 50 * np.sqrt(n) * np.finfo(float).eps
    np.testing.assert_allclose(np.linalg.norm(C2, axis=0), np.linalg.norm(B, axis=0), rtol=1e-12)


def test_sytrd_global_vector_fallback():
    """The per-step global-vector reduction, kept for grids the deferred-update variant does not
    cover, forced in the test build at n = 6200 on a known spectrum
    (tests/fault_scenarios.py trd_gv_fallback)."""
    from conftest import run_fault_scenario
    run_fault_scenario("trd_gv_fallback", timeout=600)


@pytest.mark.parametrize("n", [4100, 6144, 8192, 8200, 16384])
def test_syev_large_known_spectrum(n):
    """Large sizes with a known spectrum: n = 4100, the LDS variant's reduction; 6144 and up its
    deferred-update variant (DF) with the merge sort in LDS; 8200, the top merge sorted in global
    memory; 16384, both bounds (DF's largest LDS footprint: 64 columns per workgroup).
    A = H3 H2 H1 diag(ev) H1 H2 H3 with Householder H_k, so the
    eigenvalues are ev exactly; eigenvalues within 4 n eps ||A||, column norms of P^T B
    preserved, and the quadratic form B^T (A + s I)^{-1} B from the eigenpairs against the same
    form from the known factors."""
    rng = np.random.default_rng(n)
    ev = np.sort(rng.standard_normal(n)) * 3.0
    ev[::97] = ev[0]  # a few exact repeats: deflation on the top merges
    ev = np.sort(ev)
    A = np.diag(ev)
    vs = [rng.standard_normal(n) for _ in range(3)]
    for v in vs:  # A <- H A H, H = I - 2 v v^T / v^T v
        v = v / np.linalg.norm(v)
        Av = A @ v
        A = A - 2.0 * np.outer(v, Av) - 2.0 * np.outer(Av, v) + 4.0 * (v @ Av) * np.outer(v, v)
    A = (A + A.T) / 2
    B = rng.standard_normal((n, 3))
    ctx = G.Context(0)
    lam, C, _ = _syev(ctx, A, B)
    eps = np.finfo(float).eps
    nrm = np.abs(ev).max()
    assert np.max(np.abs(np.sort(lam) - ev)) <= 4 * n * eps * nrm
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-12)
    # B^T (A + s I)^{-1} B = (H B)^T (D + s I)^{-1} (H B) with H = H1 H2 H3 applied to B
    HB = B.copy()
    for v in reversed(vs):
        v = v / np.linalg.norm(v)
        HB = HB - 2.0 * np.outer(v, v @ HB)
    s = 0.37
    want = HB.T @ (HB / (ev + s)[:, None])
    got = C.T @ (C / (lam + s)[:, None])
    cond = np.abs(ev + s).max() / np.abs(ev + s).min()
    np.testing.assert_allclose(got, want, rtol=1e-10 * cond, atol=1e-10 * cond * np.abs(want).max())


def test_sytrd_and_syev_beyond_bound():
    """One past the reduction's bound (n = 16385) the reduction reports GPR_E_UNSUP before it
    reads A (a 1-element buffer suffices); the eigendecomposition takes block Jacobi there."""
    ctx = G.Context(0)
    n = 16385
    dA, dd, de = ctx.empty(1), ctx.empty(1), ctx.empty(1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, None, 0, n, P(dd), P(de)) == -4


def test_sytrd_se_kernel_quadratic_form_global_vectors():
    """The quadrature's quantity at n = 8192 (the reduction's global-vector variant) on the
    reference's SE + WN kernel, d = 8: B^T (K + s I)^{-1} B = (Q^T B)^T (T + s I)^{-1} (Q^T B)
    for a positive shift, a negative one keeping K + s I definite (lambda_min >= sigma_n^2) and
    one below -lambda_max (negative definite); the condition number from the bounds
    sigma_n^2 <= lambda <= ||K||_1 (no O(n^3) eigensolve on the host)."""
    import scipy.linalg as sla
    n, dim = 8192, 8
    rng = np.random.default_rng(8192)
    x = rng.random((dim, n))
    kinds = [O.SE, O.WN]
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    K = O.kernel(kinds, hp, x)
    B = np.c_[rng.random((n, 2)), O.antideriv_se(x, hp, np.zeros(dim), np.ones(dim))]
    ctx = G.Context(0)
    d, e, C = _sytrd(ctx, K, B)
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-12)
    lmax = np.abs(K).sum(0).max()
    lmin = hp[-1] ** 2
    for s in (1e-3, -0.5 * lmin, -1.5 * lmax):
        want = B.T @ np.linalg.solve(K + s * np.eye(n), B)
        got = C.T @ sla.solve_banded((1, 1), np.vstack([np.r_[0.0, e], d + s, np.r_[e, 0.0]]), C)
        lo = lmin + s if s > -lmin else abs(s) - lmax
        cond = (lmax + abs(s)) / lo
        np.testing.assert_allclose(got, want, rtol=1e-10 * cond,
                                   atol=1e-10 * cond * np.abs(want).max())


def test_sytrd_cooperative_beside_concurrent_kernel():
    """The reduction's launch is cooperative (every workgroup resident, or refused up front):
    with a long matrix product running on another stream of the same device the reduction
    still completes and gives the same d, e and Q^T B as alone (the caller would fall back,
    not spin, if the runtime could not make every workgroup resident)."""
    import torch
    n = 2048
    rng = np.random.default_rng(77)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    B = rng.standard_normal((n, 3))
    ctx = G.Context(0)
    d0, e0, C0 = _sytrd(ctx, A, B)
    side = torch.cuda.Stream()
    M = torch.randn(6144, 6144, dtype=torch.float64, device="cuda")
    with torch.cuda.stream(side):
        for _ in range(6):
            M = (M @ M) * 1e-3
    d, e, C = _sytrd(ctx, A, B)
    side.synchronize()
    assert torch.isfinite(M).all()
    assert np.array_equal(d, d0) and np.array_equal(e, e0) and np.array_equal(C, C0)


@pytest.mark.parametrize("n,m", [(300, 4), (700, 1100)])
def test_syev_and_sytrd_padded_leading_dimensions(n, m):
    """lda > n and ldb > n (a sub-block of larger buffers, as Julia views pass them): the same
    eigenvalues and P^T B as the packed call, and the padding rows of B untouched."""
    rng = np.random.default_rng(n + m)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    B = rng.standard_normal((n, m))
    ctx = G.Context(0)
    lam0, C0, _ = _syev(ctx, A, B)
    lda, ldb = n + 5, n + 3
    Ap = np.full((lda, n), 7.0)
    Ap[:n] = A
    Bp = np.full((ldb, m), -3.0)
    Bp[:n] = B
    dA, dB = ctx.colmajor(Ap), ctx.colmajor(Bp)
    lam = ctx.empty(n)
    sw = ctypes.c_int(0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert G._lib.lib.gpr_syev_apply(ctx.h, P(dA), n, lda, P(dB), m, ldb, P(lam), ctypes.byref(sw)) == 0
    Cp = ctx.host(dB)
    np.testing.assert_array_equal(ctx.host(lam)[:n], lam0)
    np.testing.assert_array_equal(Cp[:n], C0)
    assert (Cp[n:] == -3.0).all()
    dB2 = ctx.colmajor(Bp)
    dd, de = ctx.empty(n), ctx.empty(n)
    assert G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, lda, P(dB2), m, ldb, P(dd), P(de)) == 0
    d0, e0, Q0 = _sytrd(ctx, A, B)
    np.testing.assert_array_equal(ctx.host(dd)[:n], d0)
    np.testing.assert_array_equal(ctx.host(de)[:n - 1], e0)
    np.testing.assert_array_equal(ctx.host(dB2)[:n], Q0)
    assert (ctx.host(dB2)[n:] == -3.0).all()


def test_eigen_suite_under_injected_delays():
    """This file's tests once more, in a child process on the test build libgpr_hip_testing.so
    with late-wave injection in the reduction and the divide and conquer (GPR_TRD_DELAY /
    GPR_DC_DELAY: one wave in three sleeps before each read that follows another wave's LDS or
    global write, and before each hand-off poll -- DESIGN.md section 7's audit lists every such
    slot and what orders it).  The schedule that exposed round 5's dlarfg alpha race (a wave
    reading alpha after thread 0 had replaced it) is forced here on every step, so a missing
    barrier or flag gives wrong results deterministically instead of one run in three."""
    import os
    import subprocess
    import sys
    from conftest import ROOT, TESTING_LIB
    env = dict(os.environ, GPR_HIP_LIB=TESTING_LIB, GPR_TRD_DELAY="1", GPR_DC_DELAY="1")
    for k in ("GPR_TRD_FAIL_STEP", "GPR_TRD_SPIN_LIMIT", "GPR_TRD_QCHUNK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_eigen.py"),
                        "-k", "not injected_delays and not timeout and not rocsolver"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout
