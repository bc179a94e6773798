"""Cross-validation timing (gpr_cv_batch, src/crossval.jl:13-35): every fold's factorisation
in one batched tile-DAG launch (default, GPR_CV_BATCH=1) against the per-fold path over
child contexts (GPR_CV_BATCH=0), and the two results' largest relative difference.  Not a test.
    python tools/bench_cv.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))

import gpr_amd as G  # noqa: E402
from gpr_amd import crossval as CV  # noqa: E402


def timed(f, reps=3):
    f()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        out = f()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main():
    for n, k, d in ((1000, 100, 4), (2000, 200, 8), (4096, 256, 8), (8192, 512, 8)):
        rng = np.random.default_rng(n)
        x = rng.random((d, n))
        y = np.sin(x.sum(0)) ** 2
        hp = np.r_[1.0, [3.0 * np.sqrt(8.0 / d)] * d, 0.1]
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
        cvset = CV.kfoldcv(n, k, rng=np.random.default_rng(1))
        for cost in (CV.MSE(), CV.Mahalanobis()):
            os.environ["GPR_CV_BATCH"] = "1"
            tb, lb = timed(lambda: CV.cv_batch(md, cost, x, y, cvset))
            os.environ["GPR_CV_BATCH"] = "0"
            ts, ls = timed(lambda: CV.cv_batch(md, cost, x, y, cvset))
            os.environ.pop("GPR_CV_BATCH", None)
            rel = np.max(np.abs(lb - ls) / np.abs(ls))
            print(f"n={n:5d} folds={n // k:3d} ntrn={n - k:5d} ntst={k:4d} {type(cost).__name__:11s}: "
                  f"batched {tb * 1e3:8.1f} ms  per-fold {ts * 1e3:8.1f} ms  max rel diff {rel:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
