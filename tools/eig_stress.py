"""Diagnostic (not a test): repeat the n = 6144 known-spectrum case of
tests/test_eigen.py::test_syev_largest_size_known_spectrum and report, per repetition, the
reduction's error (eigvalsh of the device T against ev) and gpr_syev_apply's."""
import ctypes
import os
import sys

import numpy as np
import scipy.linalg as sla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
import gpr_amd as G  # noqa: E402


def case(n):
    rng = np.random.default_rng(6144)
    ev = np.sort(rng.standard_normal(n)) * 3.0
    ev[::97] = ev[0]
    ev = np.sort(ev)
    A = np.diag(ev)
    vs = [rng.standard_normal(n) for _ in range(3)]
    for v in vs:
        v = v / np.linalg.norm(v)
        Av = A @ v
        A = A - 2.0 * np.outer(v, Av) - 2.0 * np.outer(Av, v) + 4.0 * (v @ Av) * np.outer(v, v)
    A = (A + A.T) / 2
    B = rng.standard_normal((n, 3))
    return A, ev, B


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6144
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    A, ev, B = case(n)
    ctx = G.Context(0)
    lib = G._lib.lib
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    dA = ctx.colmajor(A)
    ref_d = ref_e = None
    for it in range(reps):
        dd, de = ctx.empty(n), ctx.empty(n)
        dB = ctx.colmajor(B)
        assert lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, P(dB), 3, n, P(dd), P(de)) == 0
        d, e = ctx.host(dd)[:n], ctx.host(de)[:n - 1]
        same = "" if ref_d is None else f" T bitwise same as rep 0: {np.array_equal(d, ref_d) and np.array_equal(e, ref_e)}"
        if ref_d is None:
            ref_d, ref_e = d.copy(), e.copy()
        et = sla.eigvalsh_tridiagonal(d, e)
        lam = ctx.empty(n)
        dB2 = ctx.colmajor(B)
        sw = ctypes.c_int(0)
        assert lib.gpr_syev_apply(ctx.h, P(dA), n, n, P(dB2), 3, n, P(lam), ctypes.byref(sw)) == 0
        lh = np.sort(ctx.host(lam)[:n])
        # D&C alone on the reference T (host -> device): isolates the second stage
        print(f"rep {it}: |eig(T)-ev| {np.abs(et - ev).max():.2e}  |syev-ev| {np.abs(lh - ev).max():.2e}{same}",
              flush=True)


if __name__ == "__main__":
    main()
