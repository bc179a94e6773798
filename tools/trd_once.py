"""Two calls of the tridiagonal reduction (gpr_sytrd_apply, m = 3) on an SE kernel matrix of
size n (d = 4, l = 2, as tools/tridiag_probe.py) -- a short program for rocprofv3 counter
passes over sytrd_df_kernel / sytrd_kernel.  Not a test and not the product path.

    python tools/trd_once.py 8192
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
sys.path.insert(0, ROOT)
import gpr_amd as G  # noqa: E402
from gpr_amd import core  # noqa: E402
from oracle import gpr_oracle as O  # noqa: E402  (the input matrix only)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    ctx = core.default_context()
    lib = G._lib.lib
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rng = np.random.default_rng(n)
    K = O.kernel([O.SE], np.r_[1.0, [2.0] * 4], rng.random((4, n)))
    dK, dB = ctx.colmajor(K), ctx.colmajor(rng.random((n, 3)))
    dd, de = ctx.empty(n), ctx.empty(n)
    for _ in range(2):
        assert lib.gpr_sytrd_apply(ctx.h, P(dK), n, n, P(dB), 3, n, P(dd), P(de)) == 0
    ctx.sync()
    print("ok", n, flush=True)


if __name__ == "__main__":
    main()
