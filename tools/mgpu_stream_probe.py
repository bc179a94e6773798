"""The streamed broadcast of gpr_split_predict_mgpu on ONE GPU (GPR_MGPU_SELF_BCAST=1: device 0
is root and receiver, the RCCL broadcast is a 1-rank no-op, so this times the fit plus the
pack / unpack pipeline, not xGMI).  Mean-only rows (no variance rows), so the call is the fit
plus the U hand-off.  Per mode: median ms of `reps` calls after a warm-up.

  python tools/mgpu_stream_probe.py [ns] [reps] [mode-index ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gaussianprocessregression.jl_amd"))
import numpy as np  # noqa: E402

import gpr_amd as G  # noqa: E402
from gpr_amd import distributed as gd  # noqa: E402


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    d, ne, nq = 8, 64, 64
    rng = np.random.default_rng(0)
    x = rng.random((d, ns))
    y = np.sin(x.sum(0)) ** 2
    xe, xq = 0.5 * rng.random((d, ne)), 0.5 * rng.random((d, nq))
    hp = np.r_[1.0, np.full(d, 2.0), 0.1]
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    mg = gd.MultiGPU([0])
    modes = [("replicate (fit only, no hand-off)", {"GPR_MGPU_SELF_BCAST": "0"}, "replicate"),
             ("broadcast after the fit", {"GPR_MGPU_SELF_BCAST": "1", "GPR_MGPU_STREAM": "0"}, "broadcast"),
             ("broadcast streamed beside the fit", {"GPR_MGPU_SELF_BCAST": "1", "GPR_MGPU_STREAM": "1"}, "broadcast")]
    if len(sys.argv) > 3:  # a subset of the modes (e.g. one, under a kernel trace)
        modes = [modes[int(k)] for k in sys.argv[3:]]
    out = {"ns": ns, "ne": ne, "nq": nq, "reps": reps, "ms": {}}
    try:
        ref = None
        for name, env, fit in modes:
            os.environ.update(env)
            mu, _ = gd.split_predict_mgpu(md, cm, mg, var_range=None, fit=fit)  # warm-up
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                mu, _ = gd.split_predict_mgpu(md, cm, mg, var_range=None, fit=fit)
                ts.append((time.perf_counter() - t0) * 1e3)
            ref = mu if ref is None else ref
            out["ms"][name] = round(float(np.median(ts)), 2)
            out.setdefault("max_rel_diff_vs_first", {})[name] = float(
                np.max(np.abs(mu - ref)) / np.max(np.abs(ref)))
            print(name, out["ms"][name], "ms", flush=True)
    finally:
        mg.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
