"""Time the tridiagonal reduction (gpr_sytrd_apply) and the sample_noise quadrature by method
(GPR_QUAD_EIGEN: 0 batched per-column factorisations, 1 tridiagonal reduction + shifted solves,
2 rocSOLVER dsyevd comparator, 4 block Jacobi) on SE kernel matrices (d = 4, l = 2 as
tools/eig_vs_rocsolver.py).  Best of 3 after a warm-up.  Not a test and not the product path."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))

import gpr_amd as G  # noqa: E402
from gpr_amd import core  # noqa: E402


def best(f, reps=3):
    f()
    t = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t = min(t, time.perf_counter() - t0)
    return t * 1e3


def main():
    sizes = [int(s) for s in (sys.argv[1].split(",") if len(sys.argv) > 1 else "512,1100,2048,4096".split(","))]
    arg = sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3,4"
    methods = [] if arg == "none" else [int(s) for s in arg.split(",")]
    ctx = core.default_context()
    lib = G._lib.lib
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for n in sizes:
        rng = np.random.default_rng(n)
        x = rng.random((4, n))
        hp = np.r_[1.0, [2.0] * 4]
        from oracle import gpr_oracle as O  # (input only)
        K = O.kernel([O.SE], hp, x)
        dK, dB = ctx.colmajor(K), ctx.colmajor(rng.random((n, 3)))
        dd, de = ctx.empty(n), ctx.empty(n)

        def trd():
            assert lib.gpr_sytrd_apply(ctx.h, P(dK), n, n, P(dB), 3, n, P(dd), P(de)) == 0, \
                lib.gpr_last_error(ctx.h)
            ctx.sync()
        print(f"sytrd n={n:5d} (m=3): {best(trd):8.2f} ms", flush=True)
        if os.environ.get("TRD_PROBE_CPU"):  # the reference's own CPU step: LAPACK syevr
            import scipy.linalg as sla
            from threadpoolctl import threadpool_limits
            thr = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
            with threadpool_limits(thr):
                tc = best(lambda: sla.eigh(K, driver="evr", overwrite_a=False, check_finite=False), reps=2)
            print(f"cpu   n={n:5d} LAPACK dsyevr (values + vectors, {thr} threads): {tc:8.2f} ms", flush=True)
        dlam = ctx.empty(n)
        for mm in (3, n):
            dB0 = ctx.colmajor(np.eye(n) if mm == n else rng.random((n, mm)))
            dBw = ctx.empty(mm, n)
            sw = ctypes.c_int(0)

            def syev():
                dBw.copy_(dB0)
                assert lib.gpr_syev_apply(ctx.h, P(dK), n, n, P(dBw), mm, n, P(dlam),
                                          ctypes.byref(sw)) == 0, lib.gpr_last_error(ctx.h)
                ctx.sync()
            print(f"syev  n={n:5d} (m={mm}): {best(syev):8.2f} ms  (tridiagonal + divide and conquer)",
                  flush=True)
        for ne in (8, 128):
            y = rng.random((n, ne))
            md = G.GPRModel(G.SquaredExp(), hp, x, y)
            noise = 1e-4 * (1.0 + rng.random(ne))
            a, b = np.zeros(4), np.ones(4)
            ref = None
            for m in methods:
                if m == 4 and n > 2048:
                    continue  # (block Jacobi: seconds)
                ctx.set_knob("GPR_QUAD_EIGEN", m)
                out = {}

                def q():
                    out["r"] = G.integrate(md, a, b, sample_noise=noise)
                t = best(q)
                r = np.r_[out["r"][0], out["r"][1]]
                diff = "" if ref is None else f"  max rel diff vs method {methods[0]} {np.max(np.abs(r - ref) / np.abs(ref)):.1e}"
                ref = r if ref is None else ref
                print(f"  quad n={n:5d} ne={ne:4d} GPR_QUAD_EIGEN={m}: {t:9.2f} ms{diff}", flush=True)
            ctx.set_knob("GPR_QUAD_EIGEN", -1)


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
