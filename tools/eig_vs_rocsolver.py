"""Time the sample_noise quadrature (gpr_integrate_noise: one eigendecomposition of K, then
(lambda + noise_j)^-1 per column) with the native block-Jacobi eigensolver (default) against
the rocSOLVER dsyevd comparator (GPR_QUAD_EIGEN=2) and the per-column factorisations
(GPR_QUAD_EIGEN=0) and the default choice between them (unset: "auto").  One process per mode:
    GPR_QUAD_EIGEN=2 python tools/eig_vs_rocsolver.py
Prints one line per size: best of 3 after a warm-up, and the result's max relative difference
to the default path's saved output (when present).  Not a test and not the product path.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))

import gpr_amd as G  # noqa: E402


def main():
    mode = os.environ.get("GPR_QUAD_EIGEN", "auto")
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    for n, ne in ((512, 64), (1100, 100), (2048, 128), (4096, 128)):
        rng = np.random.default_rng(n)
        x = rng.random((4, n))
        y = rng.random((n, ne))
        md = G.GPRModel(G.SquaredExp(), np.r_[1.0, [2.0] * 4], x, y)
        noise = 1e-4 * (1.0 + rng.random(ne))
        a, b = np.zeros(4), np.ones(4)
        G.integrate(md, a, b, sample_noise=noise)
        best = 1e30
        for _ in range(3):
            t0 = time.perf_counter()
            mu, S = G.integrate(md, a, b, sample_noise=noise)
            best = min(best, time.perf_counter() - t0)
        ref = os.path.join(out_dir, f"eigq_{n}.npy")
        diff = ""
        if mode == "1":
            np.save(ref, np.r_[mu, S])
        elif os.path.exists(ref):
            r = np.load(ref)
            got = np.r_[mu, S]
            diff = f"  max rel diff vs native {np.max(np.abs(got - r) / np.abs(r)):.2e}"
        print(f"GPR_QUAD_EIGEN={mode}{' SEQ' if os.environ.get('GPR_QUAD_SEQ') else ''} n={n:5d} ne={ne:4d}: {best * 1e3:9.1f} ms{diff}", flush=True)


if __name__ == "__main__":
    main()
