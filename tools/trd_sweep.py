"""Tridiagonal reduction time by columns per workgroup (test build: GPR_TRD_COLS), best of 3,
with B = n x 3 (the quadrature's shape).  GPR_HIP_LIB must name libgpr_hip_testing.so."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
sys.path.insert(0, ROOT)
import gpr_amd as G  # noqa: E402
from gpr_amd import core  # noqa: E402
from oracle import gpr_oracle as O  # noqa: E402


def main():
    lib = G._lib.lib
    ctx = core.default_context()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "512,1100,2048,4096").split(",")]
    colss = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "4,8,16,32").split(",")]
    for n in sizes:
        x = np.random.default_rng(n).random((4, n))
        K = O.kernel([O.SE], np.r_[1.0, [2.0] * 4], x)
        dK, dB = ctx.colmajor(K), ctx.colmajor(np.ones((n, 3)))
        dd, de = ctx.empty(n), ctx.empty(n)
        line = f"n={n:5d}:"
        for cols in colss:
            os.environ["GPR_TRD_COLS"] = str(cols)
            best = 1e30
            for _ in range(4):
                t0 = time.perf_counter()
                assert lib.gpr_sytrd_apply(ctx.h, P(dK), n, n, P(dB), 3, n, P(dd), P(de)) == 0, \
                    lib.gpr_last_error(ctx.h)
                ctx.sync()
                best = min(best, time.perf_counter() - t0)
            line += f"  cols={cols}: {best * 1e3:7.2f} ms"
        print(line, flush=True)


if __name__ == "__main__":
    main()
