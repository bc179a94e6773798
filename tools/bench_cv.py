"""Time cv_batch (src/crossval.jl:13-35) on the device: k-fold cross-validation of an SE+WN
model, Mahalanobis loss (the heaviest: fit + full-covariance posterior + a second POTRF per
fold).  Prints one JSON line per (n, k): folds/s and ms per fold.

  python tools/bench_cv.py [--sizes 2048:64,8192:819,16384:1638] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpr_amd as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2048:64,8192:819,16384:1638")
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cost", default="Mahalanobis")
    a = ap.parse_args()
    cost = {"MSE": G.MSE, "ChiSq": G.ChiSq, "Mahalanobis": G.Mahalanobis}[a.cost]()
    for spec in a.sizes.split(","):
        n, k = (int(v) for v in spec.split(":"))
        rng = np.random.default_rng(0)
        x = rng.random((a.d, n))
        y = np.sin(x.sum(axis=0)) ** 2
        hp = np.array([1.0] + [3.0] * a.d + [0.1])
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
        cvset = G.kfoldcv(n, k, rng=np.random.default_rng(1))
        G.cv_batch(md, cost, x, y, cvset)  # warm-up (allocations, code objects)
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lss = G.cv_batch(md, cost, x, y, cvset)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        nf = len(cvset[0])
        print(json.dumps({"bench": "cv_batch", "cost": a.cost, "n": n, "k": k, "d": a.d,
                          "folds": nf, "ntrn": n - k, "s": round(t, 4),
                          "ms_per_fold": round(1e3 * t / nf, 3),
                          "folds_per_s": round(nf / t, 2),
                          "mean_loss": float(np.mean(lss))}), flush=True)


if __name__ == "__main__":
    main()
