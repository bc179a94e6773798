"""Per-workgroup pass times of the tridiagonal reduction (test build libgpr_hip_testing.so,
GPR_HIP_LIB): at steps o, o + 64, o + 128, ... (o: GPR_TRD_WGOFF, default 0) every workgroup's pass duration and pass-end time
relative to the earliest, summarised per XCD (workgroup w runs on XCD w mod 8)."""
import ctypes
import os
import sys

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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    x = np.random.default_rng(n).random((4, n))
    K = O.kernel([O.SE], np.r_[1.0, [2.0] * 4], x)
    dK = ctx.colmajor(K)
    dd, de = ctx.empty(n), ctx.empty(n)
    for _ in range(2):
        assert lib.gpr_sytrd_apply(ctx.h, P(dK), n, n, None, 0, n, P(dd), P(de)) == 0
    ctx.sync()
    tr = np.zeros((6144 // 64, 256, 2), dtype=np.int64)
    assert lib.gpr_testing_trd_wg_trace(tr.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong))) == 0
    nwg = min(256, (n + 15) // 16) if n > 1536 else min(256, (n + 7) // 8)
    xcc = np.zeros(256, dtype=np.int32)
    have_xcc = hasattr(lib, "gpr_testing_trd_xcc") and \
        lib.gpr_testing_trd_xcc(xcc.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == 0
    if have_xcc:
        print("XCC of workgroups 0..15:", " ".join(str(v) for v in xcc[:16]), flush=True)
    for s in range(0, min((n - 2) // 64, 6144 // 64)):  # (steps stamped: below TRD_MAXN)
        st = tr[s, :nwg].astype(np.float64) * 0.01  # us
        dur = st[:, 1] - st[:, 0]
        end = st[:, 1] - st[:, 1].min()
        start = st[:, 0] - st[:, 0].min()
        byx = [end[x::8].mean() for x in range(8)]
        if s % 4 == 0:
            print(f"step {64 * s:5d}: pass {dur.mean():6.2f} us (min {dur.min():6.2f} max {dur.max():6.2f}); "
                  f"start spread {start.max():5.2f}; end spread {end.max():6.2f} us; "
                  f"mean end by XCD " + " ".join(f"{v:5.2f}" for v in byx), flush=True)
            if have_xcc:
                byid = [end[:nwg][xcc[:nwg] == x].mean() if (xcc[:nwg] == x).any() else float("nan")
                        for x in range(8)]
                print("      mean end by XCC_ID " + " ".join(f"{v:5.2f}" for v in byid), flush=True)
            slow = np.argsort(-dur)[:6]
            print("      slowest: " + " ".join(f"w{w}:{dur[w]:.1f}" for w in slow) +
                  f"  (median {np.median(dur):.1f})", flush=True)


if __name__ == "__main__":
    main()
