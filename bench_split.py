"""C5 benchmark: split-kernel block prediction sharded over GPUs (BASELINE
config 5).  Secondary to bench.py (the driver's headline line); same launch conventions:

  python bench_split.py [--steps K --warmup W]                           # 1 GPU
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench_split.py --gpus N                            # N GPUs (RCCL)

Workload (synthetic, seeded): ns = 32768 training points, d = 8, SE+WN, test grid
x_{e,q} = xe_e + xq_q with ne = nq = 1024 (1,048,576 test points).  One step = the whole
job: fit on rank 0 (K, POTRF, wt; or on every rank with --fit replicate), broadcast of
U (8N^2 bytes) and wt over RCCL, each rank's grid rows (mean for all of them, diagonal
variance for its share of the first --var-rows rows), all_gather to every rank in the
reference layouts.  Scaling is strong (fixed total work).  value = test points per second
for the whole job.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench_launch import spawn_ranks  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ns", type=int, default=32768)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--ne", type=int, default=1024)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--var-rows", type=int, default=32,
                    help="variance for grid rows 1..var_rows (the reference's var_range; "
                         "SURVEY 8d: default 1:3 for parity, full 1:ne = 1024 for throughput)")
    ap.add_argument("--fit", default="broadcast", choices=["broadcast", "replicate"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-ns", type=int, default=4096,
                    help="bounded CPU sample: the oracle's C5 job at this ns (same grid), each "
                         "stage extrapolated to --ns by its complexity")
    return ap.parse_args()


def cpu_baseline(a, hp, xe, xq):
    """The CPU oracle (test infrastructure; this leg only) on a bounded sample of the C5 job:
    predict(md, Cmap(+, xe, xq); diagonal_var=true) in the reference's order (src/predict.jl:
    29-34 fit, src/split_predict.jl:5-53 split factors, mean, variance rows) at ns = a.cpu_ns on
    the same 1024 x 1024 grid and variance rows, median of 3 after a warm-up; stages scaled to
    ns = a.ns by their complexity (K ns^2, dpotrf ns^3, split factors + mean ns, variance
    rows ns^2).
    Threads: OMP_NUM_THREADS for OpenBLAS, reported by threadpoolctl."""
    from threadpoolctl import threadpool_info, threadpool_limits

    sys.path.insert(0, ROOT)
    from oracle import gpr_oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    ns, d = a.cpu_ns, a.d
    kinds = [O.SE, O.WN]
    x = np.random.default_rng(0).random((d, ns))
    y = np.sin(x.sum(0)) ** 2
    vr = (1, a.var_rows) if a.var_rows > 0 else None

    def run():
        t0 = time.perf_counter()
        K = O.kernel(kinds, hp, x)
        tk = time.perf_counter()
        U = O.chol_upper(K)
        wt = O.cho_solve_upper(U, y)
        t1 = time.perf_counter()
        mu, _ = O.split_predict_from_factor(kinds, hp, x, U, wt, xe, xq, var_range=None)
        t2 = time.perf_counter()
        _, var = O.split_predict_from_factor(kinds, hp, x, U, wt, xe, xq, var_range=vr,
                                             mean_rows=[0])
        t3 = time.perf_counter()
        assert np.isfinite(mu).all() and np.isfinite(var).all()
        return np.array([tk - t0, t1 - tk, t2 - t1, t3 - t2])

    with threadpool_limits(limits=threads):
        blas = [{"lib": i.get("internal_api"), "version": i.get("version"),
                 "threads": i.get("num_threads")}
                for i in threadpool_info() if i.get("user_api") == "blas"
                and "scipy.libs" in i.get("filepath", "")]
        run()
        reps = [run() for _ in range(3)]
    t = np.median(np.stack(reps), axis=0)
    r = a.ns / ns
    scale = np.array([r ** 2, r ** 3, r, r ** 2])
    t_job = float(np.sum(t * scale))
    return {
        "value": a.ne * a.nq / t_job, "unit": "test points/s", "cores": threads, "kind": "port",
        "blas": blas,
        "measured_config": {"ns": ns, "ne": a.ne, "nq": a.nq, "var_rows": a.var_rows,
                            "stage_s": [round(v, 4) for v in t.tolist()]},
        "sample": (f"oracle (NumPy/SciPy OpenBLAS, {threads} threads) C5 job at ns={ns}, "
                   f"{a.ne}x{a.nq} grid, {a.var_rows} variance rows (median of 3 after 1 "
                   f"warm-up): stages [kernel, dpotrf + dpotrs, split factors + mean, variance rows] = "
                   f"{[round(v, 4) for v in t.tolist()]} s; extrapolated to ns={a.ns} by ns^2 / "
                   f"ns^3 / ns / ns^2 -> {t_job:.2f} s per job"),
    }


def _safe(f, *args):
    try:
        return f(*args)
    except Exception as ex:  # never let the baseline leg kill the bench line
        return {"value": None, "error": repr(ex)}


def main():
    a = parse()
    code = spawn_ranks(a.gpus)  # --gpus N: N fresh rank processes (bench_launch.py)
    if code is not None:
        sys.exit(code)
    # RCCL prints its banner and warnings to STDOUT from C: everything but the one JSON line
    # goes to stderr (fd 1 points there; the line is written to the saved descriptor)
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    import gpr_amd as G
    from gpr_amd.distributed import split_predict_distributed

    ctx = G.Context(local)
    d = a.d
    x = np.random.default_rng(0).random((d, a.ns))
    y = np.sin(x.sum(0)) ** 2
    xe = np.random.default_rng(2).random((d, a.ne))
    xq = np.random.default_rng(3).random((d, a.nq))
    hp = np.r_[1.0, [3.0 * math.sqrt(8.0 / d)] * d, 0.1]
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y, ctx=ctx)
    cm = G.Cmap("+", xe, xq)
    vr = (1, a.var_rows) if a.var_rows > 0 else None

    def step():
        return split_predict_distributed(md, cm, var_range=vr, fit=a.fit)

    import ctypes
    from gpr_amd import _lib
    lib = _lib.lib
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    # per-launch HIP-event timing on the context's stream: timing class 7 = the solve-only
    # tile-DAG launches (V = U^{-T} Kxq of the variance rows, nq ns^2 flops per grid row),
    # class 6 = the fit's factorisation launch (not the timed quantity here)
    lib.gpr_timing_reset(ctx.h)
    lib.gpr_timing_enable(ctx.h, 1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        mu, var = step()
    torch.cuda.synchronize()
    dist.barrier()
    dt = (time.perf_counter() - t0) / a.steps
    lib.gpr_timing_enable(ctx.h, 0)
    cls = {}
    for c, nm in ((6, "dag_fit"), (7, "dag_solve")):
        ms, ln, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        lib.gpr_timing_get(ctx.h, c, ctypes.byref(ms), ctypes.byref(ln), ctypes.byref(fl))
        cls[nm] = (ms.value, ln.value, fl.value)
    tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    npts = a.ne * a.nq
    mean_flops = 2.0 * a.ne * a.ns * a.nq
    var_flops = float(a.nq) * a.ns * a.ns * (a.var_rows if vr else 0)
    if rank == 0:
        line = json.dumps({
            "metric": "split-predict test points/s (C5: mean + diagonal var rows)",
            "value": npts / dt,
            "unit": "test points/s (whole job)",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (x, xe, xq ~ U[0,1) seeded, y = sin(sum x)^2)",
            "config": {"workload": f"C5 split predict SE+WN ns={a.ns} d={d} ne={a.ne} nq={a.nq} "
                                   f"var_rows={a.var_rows} fit={a.fit}",
                       "parallelism": f"e-row shards x{world}, RCCL broadcast + all_gather"},
            "algorithmic_tflop_per_step": (mean_flops + var_flops) / 1e12,
            # the variance solve (rank 0's solve-only tile-DAG launches, HIP events on the
            # stream they run on): nq ns^2 flops per grid row, against the FP64 matrix peak
            "var_solve": ({"kernel": "potrf_dag_kernel (solve-only launches)", "bound": "mfma",
                           "launches": cls["dag_solve"][1],
                           "avg_launch_ms": cls["dag_solve"][0] / cls["dag_solve"][1],
                           "flops_per_launch": cls["dag_solve"][2] / cls["dag_solve"][1],
                           "achieved_TFLOPs": cls["dag_solve"][2] / cls["dag_solve"][0] / 1e9,
                           "peak_TFLOPs": 78.6,
                           "frac": cls["dag_solve"][2] / cls["dag_solve"][0] / 1e9 / 78.6,
                           "ms_per_step": cls["dag_solve"][0] / a.steps}
                          if cls["dag_solve"][1] else None),
            "fit_dag_ms_per_step": cls["dag_fit"][0] / a.steps,
            "results_finite": bool(np.isfinite(mu).all() and np.isfinite(var).all()),
            "cpu_baseline": None if (a.no_cpu_baseline or world > 1) else _safe(cpu_baseline, a, hp, xe, xq),
        })
        os.write(json_fd, (line + "\n").encode())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
