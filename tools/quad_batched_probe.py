"""The sample_noise quadrature's batched per-column factorisations (GPR_QUAD_EIGEN=0) at one
size, three timed calls after a warm-up (for a kernel trace).  Not a test."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
import gpr_amd as G  # noqa: E402
from gpr_amd import core  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ne = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    ctx = core.default_context()
    ctx.set_knob("GPR_QUAD_EIGEN", 0)
    rng = np.random.default_rng(n)
    x = rng.random((4, n))
    y = rng.random((n, ne))
    hp = np.r_[1.0, [2.0] * 4]
    md = G.GPRModel(G.SquaredExp(), hp, x, y)
    noise = 1e-4 * (1.0 + rng.random(ne))
    a, b = np.zeros(4), np.ones(4)
    G.integrate(md, a, b, sample_noise=noise)
    for _ in range(3):
        t0 = time.perf_counter()
        G.integrate(md, a, b, sample_noise=noise)
        print(f"n={n} ne={ne}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
