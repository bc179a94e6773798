"""Phase profile of the tridiagonal reduction (test build libgpr_hip_testing.so, GPR_HIP_LIB):
per step, workgroups 0 and P-1: pass, publish + arrive, wait for the last arrival, exchange
loads + w_j, column update + reflector.  Averages in microseconds over the steps, by quarter."""
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
    for n in [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "1100,4096").split(",")]:
        x = np.random.default_rng(n).random((4, n))
        K = O.kernel([O.SE], np.r_[1.0, [2.0] * 4], x)
        dK = ctx.colmajor(K)
        dd, de = ctx.empty(n), ctx.empty(n)
        for _ in range(2):
            assert lib.gpr_sytrd_apply(ctx.h, P(dK), n, n, None, 0, n, P(dd), P(de)) == 0
        ctx.sync()
        ns = min(n, 6144)  # (TRD_MAXN: the steps the kernel stamps)
        tr = np.zeros((2, ns, 6), dtype=np.int64)
        assert lib.gpr_testing_trd_trace(tr.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ns) == 0
        st = min(n - 2, ns)
        for k, who in enumerate(("wg 0", "wg P-1")):
            t = tr[k, :st].astype(np.float64) * 0.01  # 100 MHz -> us
            ph = np.diff(t, axis=1)  # pass, publish, wait, exchange, reflector
            nxt = t[1:, 0] - t[:-1, 5]
            total = (t[-1, 5] - t[0, 0])
            print(f"n={n} {who}: total {total / 1e3:.2f} ms over {st} steps ({total / st:.2f} us/step)")
            t2 = None
            if hasattr(lib, "gpr_testing_trd_trace2"):  # (DF: the exchange phase split)
                tr2 = np.zeros((2, ns, 2), dtype=np.int64)
                if lib.gpr_testing_trd_trace2(tr2.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ns) == 0:
                    t2 = tr2[k, :st].astype(np.float64) * 0.01
            for q in range(4):
                a, b = q * st // 4, (q + 1) * st // 4
                m = ph[a:b].mean(axis=0)
                print(f"   steps {a:5d}-{b:5d}: pass {m[0]:6.2f}  publish {m[1]:5.2f}  wait {m[2]:6.2f}  "
                      f"exchange {m[3]:5.2f}  reflector {m[4]:5.2f}  gap {nxt[a:min(b, st - 1)].mean():5.2f}")
                if t2 is not None and t2[a:b].min() > 0:
                    c1 = (t2[a:b, 0] - t[a:b, 4]).mean()
                    c2 = (t2[a:b, 1] - t2[a:b, 0]).mean()
                    c3 = (t[a:b, 5] - t2[a:b, 1]).mean()
                    print(f"      (reflector = row chunks {c1:5.2f} + norm, dlarfg {c2:5.2f} + partials {c3:5.2f})")


if __name__ == "__main__":
    main()
