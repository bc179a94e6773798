"""Diagnostic (not a test): which stage loses accuracy on A = H3 H2 H1 diag(ev) H1 H2 H3 with
repeated eigenvalues -- the reduction (eigvalsh(T) vs ev) or divide and conquer (syev vs ev)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
import gpr_amd as G  # noqa: E402


def build(n, seed, rep_every):
    rng = np.random.default_rng(seed)
    ev = np.sort(rng.standard_normal(n)) * 3.0
    if rep_every:
        ev[::rep_every] = ev[0]
    ev = np.sort(ev)
    A = np.diag(ev)
    for _ in range(3):
        v = rng.standard_normal(n)
        v /= np.linalg.norm(v)
        Av = A @ v
        A = A - 2.0 * np.outer(v, Av) - 2.0 * np.outer(Av, v) + 4.0 * (v @ Av) * np.outer(v, v)
    return (A + A.T) / 2, ev


def main():
    ctx = G.Context(0)
    lib = G._lib.lib
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for n in [int(s) for s in sys.argv[1].split(",")]:
        for rep in (0, 97):
            A, ev = build(n, n, rep)
            dA = ctx.colmajor(A)
            dd, de = ctx.empty(n), ctx.empty(n)
            assert lib.gpr_sytrd_apply(ctx.h, P(dA), n, n, None, 0, n, P(dd), P(de)) == 0
            d, e = ctx.host(dd)[:n], ctx.host(de)[:n - 1]
            import scipy.linalg as sla
            et = sla.eigvalsh_tridiagonal(d, e)
            lam = ctx.empty(n)
            dB = ctx.colmajor(np.ones((n, 1)))
            sw = ctypes.c_int(0)
            assert lib.gpr_syev_apply(ctx.h, P(dA), n, n, P(dB), 1, n, P(lam), ctypes.byref(sw)) == 0
            lh = np.sort(ctx.host(lam)[:n])
            # D&C alone on the device's T: compare to eigvalsh_tridiagonal of the same T
            print(f"n={n} rep={rep}: |eig(T)-ev| {np.abs(et - ev).max():.2e}  |syev-ev| {np.abs(lh - ev).max():.2e}  "
                  f"|syev-eig(T)| {np.abs(lh - et).max():.2e}  min|e| {np.abs(e).min():.1e} #|e|<1e-12 {(np.abs(e) < 1e-12).sum()}",
                  flush=True)


if __name__ == "__main__":
    main()
