"""Fault-injection scenarios for the GPU suite, run in a CHILD process against the test build
of the library, libgpr_hip_testing.so (GPR_HIP_LIB; Makefile target $(TOUT), -DGPR_TESTING).
The release libgpr_hip.so has no fault injection at all, so an inherited environment can
never make it time out or drop a chunk on purpose; these scenarios need the switches the test
build reads at call time: GPR_DAG_SPIN_LIMIT (every tile-DAG dependency wait gives up at once),
GPR_MGPU_GATE_LIMIT (a streamed broadcast chunk's gate gives up), GPR_MGPU_FAIL_UNPACK (a
receiver's unpack of chunk k fails), GPR_TRD_FAIL_STEP / GPR_TRD_SPIN_LIMIT (a tridiagonal
reduction hand-off that never completes), GPR_TRD_DF / GPR_TRD_DF_TAIL (the deferred-update
reduction at small n), GPR_TRD_QCHUNK (the quadrature's tridiagonal solves
in launches of a few columns), GPR_MGPU_SELF_BCAST (a one-device handle broadcasting to itself)
and the rocSOLVER eigen comparator (GPR_QUAD_EIGEN=2).

    python tests/fault_scenarios.py <scenario> [args...]   -> prints "OK" on success

Each scenario checks that the fault is reported as an error (no hang, no wrong answer) and
that the same context / handle gives correct results afterwards.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gaussianprocessregression.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import gpr_oracle as O  # noqa: E402  (the checker)


def dag_timeout():
    """Every tile-DAG dependency wait is bounded (dag.hip dag_wait); GPR_DAG_SPIN_LIMIT=1
    forces the bound to expire.  The launch must drain (no hang), the call must return
    GPR_E_HIP with the timeout message -- the factorisation (gpr_fit_predict) and a solve-only
    launch (gpr_potri_upper's Z) alike -- and the SAME context must give correct results once
    the bound is back: the info flag a timed-out launch leaves behind must not make the next
    solve-only launch skip its tasks."""
    import gpr_amd as G
    from test_gpu_parity import _dev_potrf, _spd, cov_of, relnorm
    os.environ.pop("GPR_DAG_SPIN_LIMIT", None)
    ctx = G.Context(0)
    ctx.set_knob("GPR_DAG_SOLVE", 1)  # the solve-only tile-DAG at this size
    n = 1024
    A = _spd(n, seed=3)
    dA, info = _dev_potrf(ctx, A)
    assert info == 0
    dK = ctx.empty(n, n)
    potri = lambda: G._lib.lib.gpr_potri_upper(ctx.h, ctypes.c_void_p(dA.data_ptr()), n, n,  # noqa: E731
                                               ctypes.c_void_p(dK.data_ptr()), n)
    x, y, xp = O.synthetic(4, 1024, 200, seed_train=5)
    kinds = [O.SE, O.WN]
    hp = O.default_hp(kinds, 4)
    md = G.GPRModel(cov_of(kinds), hp, x, y, ctx=ctx)
    os.environ["GPR_DAG_SPIN_LIMIT"] = "1"
    for _ in range(2):  # (twice: a drained launch leaves the context usable for the next one)
        try:
            G.predict(md, xp, diagonal_var=True)
            raise AssertionError("no timeout reported")
        except G.GprError as e:
            assert "timed out" in str(e), e
        assert potri() == -2
        assert b"timed out" in G._lib.lib.gpr_last_error(ctx.h)
    del os.environ["GPR_DAG_SPIN_LIMIT"]
    # the factor in dA is intact (the timed-out launches were solves / other buffers); the
    # solve-only launch right after a timed-out one on the same cached factor
    assert potri() == 0
    assert relnorm(ctx.host(dK), np.linalg.inv(A)) < 1e-11
    mu, var = G.predict(md, xp, diagonal_var=True)
    mu_o, var_o = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=1e-8 * O.diag_prior(kinds, hp, 4))


def trd_timeout():
    """The tridiagonal reduction's hand-off polls are bounded (tridiag.hip): with one workgroup's
    partial sum of step 5 never published (GPR_TRD_FAIL_STEP, test build), every workgroup must
    give up -- the launch drains, gpr_sytrd_apply returns GPR_E_HIP "timed out" -- and the SAME
    context must then reduce correctly (the exchange buffers are re-initialised per call)."""
    import gpr_amd as G
    ctx = G.Context(0)
    n = 700
    rng = np.random.default_rng(7)
    X = rng.standard_normal((n, n))
    A = (X + X.T) / 2
    dA = ctx.colmajor(A)
    dd, de = ctx.empty(n), ctx.empty(n)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    call = lambda: G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, None, 0, n, P(dd), P(de))  # noqa: E731
    os.environ["GPR_TRD_FAIL_STEP"] = "5"
    os.environ["GPR_TRD_SPIN_LIMIT"] = "4096"
    for _ in range(2):
        assert call() == -2
        assert b"timed out" in G._lib.lib.gpr_last_error(ctx.h)
    del os.environ["GPR_TRD_FAIL_STEP"], os.environ["GPR_TRD_SPIN_LIMIT"]
    assert call() == 0
    d, e = ctx.host(dd)[:n], ctx.host(de)[:n - 1]
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    nrm = np.linalg.norm(A, 2)
    assert np.max(np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A))) <= 4 * n * np.finfo(float).eps * nrm


def trd_df_small():
    """The large-n reduction's deferred-update variant (tridiag.hip sytrd_df_kernel: panels of
    16 steps whose later columns are only read and corrected, flushed at each panel's start)
    forced at small n in the test build (GPR_TRD_DF=2, GPR_TRD_DF_TAIL=64: every panel but the
    last 64 steps deferred), so its panel / flush / tail boundaries, odd n and grids of 13-256
    workgroups run in seconds: eigenvalues of T within 4 n eps ||A|| of numpy's, ||Q^T B||
    preserved and B^T (A + s I)^{-1} B through T against numpy; once more with late-wave
    injection (GPR_TRD_DELAY=1); and a hand-off that never completes times out cleanly."""
    import scipy.linalg as sla
    import gpr_amd as G
    ctx = G.Context(0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    os.environ["GPR_TRD_DF"] = "2"
    os.environ["GPR_TRD_DF_TAIL"] = "64"
    eps = np.finfo(float).eps
    for n, delay in ((100, 0), (701, 0), (2051, 0), (4100, 0), (701, 1)):
        os.environ["GPR_TRD_DELAY"] = str(delay)
        rng = np.random.default_rng(n)
        X = rng.standard_normal((n, n))
        A = (X + X.T) / 2
        B = rng.standard_normal((n, 3))
        dA, dB = ctx.colmajor(A), ctx.colmajor(B)
        dd, de = ctx.empty(n), ctx.empty(n)
        assert G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, P(dB), 3, n, P(dd), P(de)) == 0, \
            G._lib.lib.gpr_last_error(ctx.h)
        d, e, C = ctx.host(dd)[:n], ctx.host(de)[:n - 1], ctx.host(dB)[:n]
        T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
        nrm = np.linalg.norm(A, 2)
        lam = np.linalg.eigvalsh(A)
        err = np.max(np.abs(np.linalg.eigvalsh(T) - lam))
        assert err <= 4 * n * eps * nrm, (n, delay, err)
        np.testing.assert_allclose(np.linalg.norm(C, axis=0), np.linalg.norm(B, axis=0), rtol=1e-12)
        s = 0.5 * nrm + 0.1  # (A + s I: indefinite, away from singular)
        want = B.T @ np.linalg.solve(A + s * np.eye(n), B)
        got = C.T @ sla.solve_banded((1, 1), np.vstack([np.r_[0.0, e], d + s, np.r_[e, 0.0]]), C)
        cond = np.max(np.abs(lam + s)) / np.min(np.abs(lam + s))
        np.testing.assert_allclose(got, want, rtol=1e-11 * cond, atol=1e-11 * cond * np.abs(want).max())
    os.environ["GPR_TRD_DELAY"] = "0"
    # a partial sum of step 21 (a deferred panel's 6th step) never published: every workgroup
    # gives up, the call reports it, and the same context reduces correctly afterwards
    n = 701
    A = np.random.default_rng(5).standard_normal((n, n))
    A = (A + A.T) / 2
    dA, dd, de = ctx.colmajor(A), ctx.empty(n), ctx.empty(n)
    call = lambda: G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, None, 0, n, P(dd), P(de))  # noqa: E731
    os.environ["GPR_TRD_FAIL_STEP"] = "21"
    os.environ["GPR_TRD_SPIN_LIMIT"] = "4096"
    assert call() == -2 and b"timed out" in G._lib.lib.gpr_last_error(ctx.h)
    del os.environ["GPR_TRD_FAIL_STEP"], os.environ["GPR_TRD_SPIN_LIMIT"]
    assert call() == 0
    T = np.diag(ctx.host(dd)[:n]) + np.diag(ctx.host(de)[:n - 1], 1) + np.diag(ctx.host(de)[:n - 1], -1)
    assert np.max(np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A))) <= 4 * n * eps * np.linalg.norm(A, 2)


def trd_gv_fallback():
    """The per-step global-vector reduction (sytrd_kernel<.., GV = true>), the fallback above
    n = 6144 for grids the deferred-update variant does not cover, forced with GPR_TRD_DF=0 at
    n = 6200 on a known spectrum (A = H3 H2 H1 diag(ev) H1 H2 H3): T's eigenvalues within
    4 n eps ||A|| of ev, ||Q^T B|| preserved."""
    import scipy.linalg as sla
    import gpr_amd as G
    ctx = G.Context(0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    n = 6200
    rng = np.random.default_rng(n)
    ev = np.sort(rng.standard_normal(n)) * 3.0
    A = np.diag(ev)
    for _ in range(3):
        v = rng.standard_normal(n)
        v /= np.linalg.norm(v)
        Av = A @ v
        A = A - 2.0 * np.outer(v, Av) - 2.0 * np.outer(Av, v) + 4.0 * (v @ Av) * np.outer(v, v)
    A = (A + A.T) / 2
    B = rng.standard_normal((n, 3))
    os.environ["GPR_TRD_DF"] = "0"
    dA, dB = ctx.colmajor(A), ctx.colmajor(B)
    dd, de = ctx.empty(n), ctx.empty(n)
    assert G._lib.lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, P(dB), 3, n, P(dd), P(de)) == 0, \
        G._lib.lib.gpr_last_error(ctx.h)
    del os.environ["GPR_TRD_DF"]
    lam = sla.eigvalsh_tridiagonal(ctx.host(dd)[:n], ctx.host(de)[:n - 1])
    assert np.max(np.abs(lam - ev)) <= 4 * n * np.finfo(float).eps * np.abs(ev).max()
    np.testing.assert_allclose(np.linalg.norm(ctx.host(dB)[:n], axis=0), np.linalg.norm(B, axis=0),
                               rtol=1e-12)


def trd_quad_chunks():
    """The quadrature's per-column tridiagonal solves run in launches of at most
    quad_tridiag_chunk(n, ny) columns (scratch bound); GPR_TRD_QCHUNK (test build) forces 7-
    and 1-column launches: the results are bit for bit those of one launch."""
    import gpr_amd as G
    dim, n, ne = 3, 400, 30
    rng = np.random.default_rng(11)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    kinds = [O.SE, O.WN]
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    ctx = G.Context(0)
    ctx.set_knob("GPR_QUAD_EIGEN", 1)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y, ctx=ctx)
    a, b = np.zeros(dim), np.ones(dim)
    noise = np.r_[1e-3 * (1.0 + rng.random(ne - 1)), -1e-3]
    os.environ.pop("GPR_TRD_QCHUNK", None)
    I0, v0 = G.integrate(md, a, b, sample_noise=noise)
    for ch in ("7", "1"):
        os.environ["GPR_TRD_QCHUNK"] = ch
        I, v = G.integrate(md, a, b, sample_noise=noise)
        assert np.array_equal(I, I0) and np.array_equal(v, v0), ch
    del os.environ["GPR_TRD_QCHUNK"]
    Io, vo = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I0, Io, rtol=1e-8)


def quad_rocsolver():
    """GPR_QUAD_EIGEN=2 (rocSOLVER dsyevd, test build only) against route 1 and the oracle."""
    import gpr_amd as G
    dim, n, ne = 3, 600, 6
    kinds = [O.SE, O.WN]
    rng = np.random.default_rng(9)
    x = rng.random((dim, n))
    Y = rng.random((n, ne))
    hp = O.default_hp(kinds, dim, length=2.0, noise=0.05)
    ctx = G.Context(0)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, Y, ctx=ctx)
    a, b = np.zeros(dim), np.ones(dim)
    noise = np.r_[1e-3 * (1.0 + rng.random(ne - 1)), -1e-3]
    ctx.set_knob("GPR_QUAD_EIGEN", 1)
    I, v = G.integrate(md, a, b, sample_noise=noise)
    ctx.set_knob("GPR_QUAD_EIGEN", 2)
    I2, v2 = G.integrate(md, a, b, sample_noise=noise)
    np.testing.assert_allclose(I2, I, rtol=1e-8)
    np.testing.assert_allclose(v2, v, rtol=1e-7, atol=1e-12 * O.antideriv2_se(hp, a, b))
    Io, _ = O.integrate_noise(kinds, hp, x, Y, a, b, noise)
    np.testing.assert_allclose(I2, Io, rtol=1e-8)


def mgpu_self_bcast(ns, stream, chunks):
    """The broadcast path of gpr_split_predict_mgpu on the one-GPU box (GPR_MGPU_SELF_BCAST,
    test build only): device 0 factors with the hook armed (8 CUs left free), packs each chunk of
    tile rows as soon as the tile-DAG's progress counters show it final, runs the 1-rank RCCL
    broadcast of the chunk, unpacks it into a second buffer as a receiver does and predicts from
    that copy with rebuilt block inverses; the result equals the single-device split predict up
    to the rebuilt inverses' rounding (rtol 1e-12) -- a chunk packed before its rows were final
    would differ at O(1).  The schedule knobs go through gpr_mgpu_set_knob."""
    import gpr_amd as G
    import gpr_amd.distributed as gd
    from test_distributed import _problem
    os.environ["GPR_MGPU_SELF_BCAST"] = "1"
    kinds, hp, x, y, xe, xq = _problem(ne=9, nq=33, ns=int(ns), d=5, seed=12)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    mg = gd.MultiGPU([0])
    try:
        mg.set_knob("GPR_MGPU_STREAM", int(stream))
        mg.set_knob("GPR_MGPU_CHUNKS", int(chunks))
        assert mg.get_knob("GPR_MGPU_STREAM") == int(stream)
        assert mg.get_knob("GPR_MGPU_CHUNKS") == int(chunks)
        assert mg.get_knob("GPR_MGPU_SELF_BCAST") == 1
        for _ in range(2):  # (the second call re-uses every buffer)
            mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=(1, 9), fit="broadcast")
    finally:
        mg.close()
    mu1, var1 = G.predict(md, cm, diagonal_var=True, var_range=(1, 9))
    np.testing.assert_allclose(mu, mu1, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(var, var1, rtol=1e-12, atol=1e-14)


def _mgpu_case(seed):
    import gpr_amd as G
    import gpr_amd.distributed as gd
    from test_distributed import _problem
    os.environ["GPR_MGPU_SELF_BCAST"] = "1"
    kinds, hp, x, y, xe, xq = _problem(ne=7, nq=9, ns=4096, d=5, seed=seed)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    return G, gd, md, cm


def _check_vs_single(G, md, cm, mu, var):
    mu1, var1 = G.predict(md, cm, diagonal_var=True, var_range=(1, 7))
    np.testing.assert_allclose(mu, mu1, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(var, var1, rtol=1e-12, atol=1e-14)


def mgpu_gate_timeout():
    """A streamed chunk whose gate gives up (GPR_MGPU_GATE_LIMIT=0: every gate at its first
    poll) is reported as an error after every stream drained -- no hang -- and the next call on
    the same handle, with the default limit, is correct."""
    os.environ["GPR_MGPU_STREAM"] = "1"
    G, gd, md, cm = _mgpu_case(13)
    mg = gd.MultiGPU([0])
    try:
        os.environ["GPR_MGPU_GATE_LIMIT"] = "0"
        try:
            gd.split_predict_mgpu(md, cm, mg, var_range=(1, 7), fit="broadcast")
            raise AssertionError("no gate timeout reported")
        except G.GprError as e:
            assert "gate timed out" in str(e), e
        del os.environ["GPR_MGPU_GATE_LIMIT"]
        mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=(1, 7), fit="broadcast")
    finally:
        mg.close()
    _check_vs_single(G, md, cm, mu, var)


def mgpu_unpack_failure(stream, chunk):
    """A receiver whose unpack of one chunk fails (GPR_MGPU_FAIL_UNPACK=k) keeps receiving
    every remaining chunk and wt -- the sender posts them all -- and reports the error once the
    protocol is complete: the call returns an error instead of hanging, and the next call on the
    same handle is correct."""
    os.environ["GPR_MGPU_STREAM"] = stream
    os.environ["GPR_MGPU_CHUNKS"] = "5"
    G, gd, md, cm = _mgpu_case(14)
    mg = gd.MultiGPU([0])
    try:
        os.environ["GPR_MGPU_FAIL_UNPACK"] = chunk
        try:
            gd.split_predict_mgpu(md, cm, mg, var_range=(1, 7), fit="broadcast")
            raise AssertionError("no unpack failure reported")
        except G.GprError as e:
            assert f"unpack of chunk {chunk} failed" in str(e), e
        del os.environ["GPR_MGPU_FAIL_UNPACK"]
        mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=(1, 7), fit="broadcast")
    finally:
        mg.close()
    _check_vs_single(G, md, cm, mu, var)


if __name__ == "__main__":
    globals()[sys.argv[1]](*sys.argv[2:])
    print("OK", flush=True)
