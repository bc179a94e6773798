#!/usr/bin/env python3
"""bench.py -- GP fit + posterior on MI355X through libgpr_hip.so (BASELINE.json metric).

Workload (BASELINE config 3, the config the headline metric is quoted on): composed kernel
SquaredExp + SquaredExp + WhiteNoise (the parity-pinned stand-in for "SE + periodic": the
reference has no periodic kernel), N = 32768 training points, d = 8, fp64.
One step = one GP job on each GPU, the reference's predict(md, xp; diagonal_var=true) from
scratch (src/predict.jl:14-71: update_cache! = K, cholesky!, ldiv! against y; then predict!)
as ONE call, gpr_fit_predict:
    K-assembly (N x N) and cross kernel K(x, xp) (N x np, np = 8192 test points); ONE
    persistent tile-DAG launch factors K in place (upper Cholesky) and solves
    U^T [V | z] = [K(x, xp) | y] as right-hand-side tile tasks; mean = V^T z, diagonal
    variance = prior - ||V_j||^2, alpha = U^{-1} z (backward sweep).
(GPR_DAG=0: the blocked two-stream factorisation, then POTRS and the posterior TRSM.)
Synthetic data: x ~ U[0,1)^(d x N) seed 0 (+rank), y = sin(sum x)^2, test points
seed 1 (+rank); hp sigma = 1, l = 3 sqrt(8/d), sigma_n = 0.1.  All inputs are resident in
HBM before the timed region.

Multi-GPU: the fit does not shard (no distributed Cholesky) -- every rank runs its
own job ("replicas", weak scaling, no data-path collective); value = jobs/s over all ranks.
`--gpus N` alone starts N ranks (bench_launch.py: a GPU-free parent forks N fresh processes
with RANK / LOCAL_RANK / WORLD_SIZE set); under torch.distributed.run WORLD_SIZE must equal
--gpus or the run exits 2.
Beside it, key `split_predict`: BASELINE config 5 (split-kernel block prediction, 1M test points)
SHARDED over all ranks with the RCCL broadcast of U / wt and an all_gather of the shards
(strong scaling; `--no-split` skips it).

Extra fields: K-build GB/s (bytes written / t: the fit's upper-only build writes ~4 N^2 bytes,
the tile-DAG the strict lower half) and POTRF TFLOP/s ((N^3/3) / t) at N = 32768, stage
times, and `roofline` for the dominant kernel -- potrf_dag_kernel, the persistent tile-DAG
launch that factors K and solves U^T [V | z] = [K(x, xp) | y] (N^3/3 + N^2 (np + 1) flops),
or, with GPR_DAG=0, the pipelined FP64 MFMA GEMM of the blocked path -- measured with HIP
events on the stream it runs on over one instrumented step; `cpu_baseline` = the CPU oracle
(threaded C K-build + OpenBLAS LAPACK) timed on the C3 job itself (N = 32768, np = 8192,
median of 3 after a warm-up; --cpu-n / --cpu-np shrink it, and the stages are then scaled by
their complexity to the job).

Output: rank 0 prints the ONE JSON line on stdout as soon as the headline, its instrumented
step and the CPU baseline are measured -- BEFORE the C5 leg, so a failure or hang inside the
leg (RCCL across ranks) cannot cost the headline.  The C5 leg's own JSON object follows on
stderr (key `split_predict`), and a watchdog ends the process if the leg outlives
--split-timeout seconds.
"""
from __future__ import annotations

import argparse
import ctypes
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

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK = 78.6      # TFLOP/s, FP64 matrix spec (measured 77.7 in tools/probe)
# the pipelined FP64 GEMM: two compiled variants of one kernel (beta != 0 preloads C, `z`
# starts from zero); timing class 5 counts every launch of both
DOMINANT_KERNELS = ("gemm_tn_pipe8_kernel", "gemm_tn_pipe8z_kernel")
# the one-launch tile-DAG factorisation + posterior solve (dag.hip), the default since round 2
DAG_KERNEL = "potrf_dag_kernel"
PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")


def pmc_traffic(kernels, n, npred, largest=False):
    """HBM bytes per launch (dispatch-weighted over `kernels`) from the newest committed PMC summary
    (profiles/rNN_pmc_summary.json, written by tools/profile_round.sh from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench command, FETCH_SIZE
    doubled per the gfx950 16-B/lane correction).  None when no summary matches."""
    try:
        files = sorted(f for f in os.listdir(PROFILES) if f.endswith("_pmc_summary.json"))
    except OSError:
        return None
    for f in reversed(files):
        try:
            with open(os.path.join(PROFILES, f)) as fh:
                js = json.load(fh)
        except (OSError, ValueError):
            continue
        if js.get("config", {}).get("N") != n or js.get("config", {}).get("np") != npred:
            continue
        ks = [js.get("kernels", {}).get(k) for k in kernels]
        if not all(ks):
            continue
        if largest:  # the job's launch of a kernel also launched with less work per call
            if all("traffic_bytes_max_launch" in k for k in ks):
                return max(k["traffic_bytes_max_launch"] for k in ks), f"profiles/{f}"
            continue
        w = [k.get("trace", {}).get("calls") or k.get("dispatches_fetch_pass") or 1 for k in ks]
        return (sum(wi * k["traffic_bytes_per_launch"] for wi, k in zip(w, ks)) / sum(w),
                f"profiles/{f}")
    return None, None


def pmc_mfma(kernel, n, npred):
    """MFMA-pipe utilisation of the kernel's largest launch from the newest committed PMC
    summary with an MFMA pass (tools/profile_round.sh: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE
    / 8 XCDs x 256 CUs x 4 SIMDs), the effective clock, and the summary file).  None if none."""
    try:
        files = sorted(f for f in os.listdir(PROFILES) if f.endswith("_pmc_summary.json"))
    except OSError:
        return None
    for f in reversed(files):
        try:
            with open(os.path.join(PROFILES, f)) as fh:
                js = json.load(fh)
        except (OSError, ValueError):
            continue
        if js.get("config", {}).get("N") != n or js.get("config", {}).get("np") != npred:
            continue
        m = js.get("kernels", {}).get(kernel, {}).get("mfma_largest_launch")
        if m and "mfma_busy_per_cu_cycle" in m:
            return {"busy_frac": m["mfma_busy_per_cu_cycle"] / 4.0,
                    "clock_GHz": m.get("clock_GHz"), "source": f"profiles/{f}"}
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--np", type=int, default=8192, dest="npred")
    ap.add_argument("--kernel", default="SE+SE+WN")
    ap.add_argument("--nb", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-se-ard", action="store_true",
                    help="skip the SE-ARD K-build line (two extra gpr_fit calls: the profile "
                         "runs skip it so the kernel trace holds only the C3 step's DAG launches)")
    ap.add_argument("--cpu-n", type=int, default=None, help="CPU baseline N (default --n)")
    ap.add_argument("--cpu-np", type=int, default=None, help="CPU baseline np (default --np)")
    ap.add_argument("--no-split", action="store_true",
                    help="skip the C5 split-predict leg (extra key `split_predict`)")
    ap.add_argument("--split-steps", type=int, default=2)
    ap.add_argument("--no-split-full", dest="split_full", action="store_false",
                    help="skip the C5 leg's full-range variant (var_range = 1:ne, SURVEY 8d's "
                         "throughput configuration: ~17 s per step on one GPU, 1 warm-up + 1 step)")
    ap.add_argument("--split-timeout", type=float, default=420.0,
                    help="watchdog: end the process (exit 3, headline already printed) if the "
                         "C5 leg runs longer than this many seconds")
    # rehearsal of the multi-rank path on fewer GPUs than ranks (ranks share devices by
    # LOCAL_RANK modulo the device count): gloo carries the collectives (RCCL refuses two
    # ranks on one device); the driver's runs use the default nccl (= RCCL), one rank per GPU
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    a = ap.parse_args()
    a.cpu_n = a.cpu_n or a.n
    a.cpu_np = a.cpu_np or a.npred
    return a


def config_label(a):
    """Which BASELINE.json config the run's workload is (C2: SE-ARD N=8192 d=8; C3: the
    composed kernel at N=32768 d=8); anything else is labelled `custom`."""
    if (a.kernel, a.n, a.d) == ("SE", 8192, 8):
        return "C2"
    if (a.kernel, a.n, a.d) == ("SE+SE+WN", 32768, 8):
        return "C3"
    return "custom"


def kinds_of(name):
    return [1 if k == "SE" else 2 for k in name.split("+")]


def _timing(lib, ctx, c):
    """(ms, launches, flops-or-bytes) of the context's timing class c."""
    ms, ln, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
    lib.gpr_timing_get(ctx.h, c, ctypes.byref(ms), ctypes.byref(ln), ctypes.byref(fl))
    return ms.value, ln.value, fl.value


def default_hp(kinds, d, noise=0.1):
    hp = []
    for k in kinds:
        hp += [1.0] + [3.0 * math.sqrt(8.0 / d)] * d if k == 1 else [noise]
    return np.array(hp, dtype=np.float64)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(a, kinds, hp):
    """Time the CPU oracle (test infrastructure, bench's cpu_baseline leg only): the reference's
    call order (K-build, dpotrf, dpotrs, K(x, xp), mean, dtrsm, row norms) on the C3 job itself,
    N = a.cpu_n, np = a.cpu_np (default the full 32768 / 8192: ~15 s per run on the GPU box's
    16 EPYC threads), median of 3 runs after one warm-up.  If SciPy's OpenBLAS dpotrf refuses
    the matrix (scipy-openblas 0.3.28 returns info = 16545 for the positive definite C3 matrix
    at N = 32768 on the build container's Xeon, not on the GPU box's EPYC -- DESIGN.md), the
    job is timed at half the size and each stage scaled by its complexity (N^2, N^3, N^2,
    np N^2), and the line says so.  Threads: the box's CPU share (OMP_NUM_THREADS, 16 on the
    GPU box) for both the OpenMP K-build and OpenBLAS, set explicitly and reported as measured
    by threadpoolctl."""
    import scipy.linalg as sla

    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    try:
        return _cpu_baseline_at(a, kinds, hp, a.cpu_n, a.cpu_np, threads)
    except sla.LinAlgError as ex:
        out = _cpu_baseline_at(a, kinds, hp, a.cpu_n // 2, a.cpu_np // 2, threads)
        out["fallback"] = f"N={a.cpu_n}: {ex!r}; timed at N={a.cpu_n // 2} and extrapolated"
        return out


def _cpu_baseline_at(a, kinds, hp, n, m, threads):
    import scipy.linalg as sla
    from threadpoolctl import threadpool_info, threadpool_limits

    from oracle import gpr_oracle as O
    from oracle.cpu_kbuild import kbuild_cpu

    d = a.d
    x = np.random.default_rng(0).random((d, n))
    y = np.sin(x.sum(0)) ** 2
    xp = np.random.default_rng(1).random((d, m))
    okinds = [O.SE if k == 1 else O.WN for k in kinds]

    def run():
        t0 = time.perf_counter()
        K = kbuild_cpu(okinds, hp, x)
        t1 = time.perf_counter()
        U = sla.cholesky(K, lower=False, overwrite_a=True, check_finite=False)
        t2 = time.perf_counter()
        alpha = O.cho_solve_upper(U, y)
        t3 = time.perf_counter()
        Kpx = kbuild_cpu(okinds, hp, x, xp)
        mu = Kpx.T @ alpha
        V = sla.solve_triangular(U, Kpx, trans="T", lower=False, check_finite=False,
                                 overwrite_b=True)
        var = O.diag_prior(okinds, hp, d) - np.einsum("ij,ij->j", V, V)
        t4 = time.perf_counter()
        assert np.isfinite(mu).all() and np.isfinite(var).all()
        return np.array([t1 - t0, t2 - t1, t3 - t2, t4 - t3])

    with threadpool_limits(limits=threads):
        blas = [{"lib": i.get("internal_api"), "version": i.get("version"),
                 "threads": i.get("num_threads")}
                for i in threadpool_info() if i.get("user_api") == "blas"
                and "scipy.libs" in i.get("filepath", "")]  # SciPy's own OpenBLAS (LAPACK)
        run()  # warm-up
        reps = [run() for _ in range(3)]
    t = np.median(np.stack(reps), axis=0)
    N, NP = a.n, a.npred
    scale = np.array([(N / n) ** 2, (N / n) ** 3, (N / n) ** 2, (NP / m) * (N / n) ** 2])
    t_job = float(np.sum(t * scale))
    return {
        "value": 1.0 / t_job,
        "unit": "GP jobs/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": _cpu_model(),
        "blas": blas,
        "measured_config": {"N": n, "np": m, "d": d, "kernel": a.kernel,
                            "stage_s": [round(v, 4) for v in t.tolist()],
                            "job_s": round(float(np.sum(t)), 4)},
        "sample": (f"oracle (C OpenMP K-build + OpenBLAS dpotrf/dpotrs/dtrsm via SciPy, "
                   f"{threads} threads) on the C3 job at N={n}, np={m} (median of 3 after 1 "
                   f"warm-up): stages [kbuild, potrf, potrs, posterior] = "
                   f"{[round(v, 4) for v in t.tolist()]} s"
                   + ("" if (n, m) == (N, NP) else
                      f"; extrapolated to N={N}, np={NP} by N^2 / N^3 / N^2 / np*N^2")
                   + f" -> {t_job:.2f} s per job"),
    }


def store_ceiling(lib, ctx, K, n):
    """Pure-store ceilings of the fit's upper-only K build (bench instrumentation,
    csrc/probe/store_ceiling.hip): the MFMA-layout shape (persistent grid, 4 columns x 128 B
    per store instruction), the same items one wave each, 1-KB column chunks in column order one
    per wave, the items with 1-KB column stores (persistent; 16-column strips; one item per
    wave -- the single-part build's own shape since round 6) -- best of 3 after a warm-up each,
    on the bench's K buffer."""
    path = os.path.join(ROOT, "gaussianprocessregression.jl_amd", "gpr_amd", "libgpr_store_probe.so")
    if not os.path.exists(path):
        return None
    pl = ctypes.CDLL(path)
    pl.gpr_probe_upper_store.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double)]
    stream = lib.gpr_ctx_stream(ctx.h)
    out = {}
    for pat, name in ((0, "kernel_pattern"), (1, "item_per_wave"), (2, "chunk1k_column_order"),
                      (3, "items_1k_column_stores"), (4, "items16_1k_column_stores"),
                      (5, "items_1k_column_stores_item_per_wave")):
        ms, nb = ctypes.c_double(), ctypes.c_double()
        rc = pl.gpr_probe_upper_store(stream, n, ctypes.c_void_p(K.data_ptr()), pat, 3,
                                      ctypes.byref(ms), ctypes.byref(nb))
        if rc != 0:
            return {"error": f"gpr_probe_upper_store pattern {pat} rc {rc}"}
        out[name] = {"ms": ms.value, "GBps": nb.value / (ms.value * 1e-3) / 1e9}
        out["bytes"] = nb.value
    out["best_GBps"] = max(v["GBps"] for k, v in out.items() if isinstance(v, dict))
    out["best_hbm_frac"] = out["best_GBps"] / HBM_PEAK_GBS
    return out


class _StdoutToStderr:
    """RCCL prints its banner and warnings to STDOUT from C; the driver reads ONE JSON line
    there.  Point file descriptor 1 at stderr while communicators are created and used, and
    flush C stdio before restoring it."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        try:
            ctypes.CDLL(None).fflush(None)
        except OSError:
            pass
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def split_leg(a, world, rank, local):
    """BASELINE config 5 beside the headline: split-kernel block prediction (ns = 32768, d = 8,
    SE+WN, 1024 x 1024 test grid, variance for the first 32 grid rows) sharded over all ranks
    -- rank 0 fits and broadcasts U (packed upper triangle) and wt over RCCL, every rank takes
    an even share of the variance rows and of the mean-only rows, the shards are all-gathered (gpr_amd/distributed.py; bench_split.py is the standalone
    form).  Strong scaling: fixed total work.  Timed like the headline (warm-up, barrier,
    max over ranks).  With more than one rank the fit="replicate" variant is timed too."""
    import gpr_amd as G
    from gpr_amd.distributed import split_predict_distributed

    ns, d, ne, nq, vr = 32768, 8, 1024, 1024, 32
    x = np.random.default_rng(0).random((d, ns))
    y = np.sin(x.sum(0)) ** 2
    xe = np.random.default_rng(2).random((d, ne))
    xq = np.random.default_rng(3).random((d, nq))
    hp = np.r_[1.0, [3.0 * math.sqrt(8.0 / d)] * d, 0.1]
    err = None
    try:
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y, ctx=G.Context(local))
        cm = G.Cmap("+", xe, xq)
    except Exception as e:  # noqa: BLE001 -- every rank abandons the leg together
        err = e
    bad = torch.tensor([0 if err is None else 1], dtype=torch.int64,
                       device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if int(bad.item()):
        raise err if err is not None else RuntimeError("C5 leg: set-up failed on another rank")
    flops = 2.0 * ne * ns * nq + float(nq) * ns * ns * vr
    coll = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()

    def timed(fit, rows=vr, steps=a.split_steps):
        step = lambda: split_predict_distributed(md, cm, var_range=(1, rows), fit=fit)  # noqa: E731
        step()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            mu, var = step()
        torch.cuda.synchronize()
        dist.barrier()
        dt = (time.perf_counter() - t0) / steps
        tt = torch.tensor([dt], dtype=torch.float64,
                          device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item()), bool(np.isfinite(mu).all() and np.isfinite(var).all())

    dt, ok = timed("broadcast")
    out = {"metric": "split-predict test points/s (C5)", "value": ne * nq / dt,
           "unit": "test points/s (whole job)", "ms_per_step": dt * 1e3, "n_gpus": world,
           "steps": a.split_steps, "scaling": "strong",
           "workload": f"C5 split predict SE+WN ns={ns} d={d} ne={ne} nq={nq} var_rows={vr} "
                       f"fit=broadcast, cost-balanced e-row shards x{world}, {coll} broadcast "
                       "of U's packed upper triangle + all_gather",
           "algorithmic_TFLOPs": flops / dt / 1e12, "results_finite": ok}
    if world > 1:  # every rank refits instead of receiving U (no N^2 exchange)
        dt_r, ok_r = timed("replicate")
        out["replicate"] = {"value": ne * nq / dt_r, "ms_per_step": dt_r * 1e3,
                            "results_finite": ok_r}
    if a.split_full:  # SURVEY 8d's throughput configuration: variance for every grid row
        dt_f, ok_f = timed("broadcast", rows=ne, steps=1)
        flops_f = 2.0 * ne * ns * nq + float(nq) * ns * ns * ne
        out["full_var_range"] = {"value": ne * nq / dt_f, "ms_per_step": dt_f * 1e3, "steps": 1,
                                 "var_rows": ne, "algorithmic_TFLOPs": flops_f / dt_f / 1e12,
                                 "results_finite": ok_f}
    return out


def main():
    a = parse()
    # --gpus N without a launcher: this process only forks N ranks and never touches the GPU;
    # under a launcher WORLD_SIZE must equal --gpus (bench_launch.py)
    code = spawn_ranks(a.gpus)
    if code is not None:
        sys.exit(code)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if a.dist_backend == "gloo":  # rehearsal: ranks share the devices there are
        local %= max(ndev, 1)
    elif local >= ndev:
        sys.exit(f"bench.py: LOCAL_RANK={local} but only {ndev} HIP device(s) are visible "
                 "(one rank per GPU under RCCL; --dist-backend gloo rehearses more ranks)")
    if world > 1:
        torch.cuda.set_device(local)
        with _StdoutToStderr():
            if a.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
            dist.barrier()  # communicator set up here, banner and all
    import gpr_amd as G
    from gpr_amd import _lib

    lib = _lib.lib
    ctx = G.Context(local, nb=a.nb)
    N, d, NP = a.n, a.d, a.npred
    kinds = kinds_of(a.kernel)
    hp = default_hp(kinds, d)
    karr = (ctypes.c_int * len(kinds))(*kinds)
    hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))

    x = np.random.default_rng(0 + rank).random((d, N))
    y = np.sin(x.sum(0)) ** 2
    xp = np.random.default_rng(1 + rank).random((d, NP))
    dx, dy, dxp = ctx.colmajor(x), ctx.colmajor(y), ctx.colmajor(xp)
    K = ctx.empty(N, N)
    alpha = ctx.empty(N)
    mu = ctx.empty(NP)
    var = ctx.empty(NP)
    work = ctx.empty(NP + 1, N)   # [K(x, xp) | y], column-major N x (np + 1)
    info = ctypes.c_int(0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def fit_predict():
        rc = lib.gpr_fit_predict(ctx.h, karr, len(kinds), hpp, d, P(dx), N, P(dy), 1, N, 1e-8,
                                 P(K), N, P(alpha), P(dxp), NP, 1, P(mu), P(var), NP, P(work),
                                 ctypes.byref(info))
        if rc != 0:
            raise RuntimeError(f"gpr_fit_predict rc={rc} info={info.value}: "
                               f"{lib.gpr_last_error(ctx.h)}")

    def posterior():
        ctx.check(lib.gpr_predict(ctx.h, karr, len(kinds), hpp, d, P(dx), N, P(K), N, P(alpha), 1,
                                  P(dxp), NP, 1, 1e-8, P(mu), P(var), NP, P(work)), "gpr_predict")

    def step():
        fit_predict()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    ctx.sync()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    dt = (t1 - t0) / a.steps
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ok = bool(torch.isfinite(mu).all().item() and torch.isfinite(var).all().item())

    # ---- instrumented steps (HIP events on the context stream) --------------------------
    # (a) the unfused reference order (gpr_kernel, gpr_potrf_upper, gpr_potrs_upper,
    #     gpr_predict) for a per-stage breakdown; (b) the fused step with kernel-level timing
    #     classes (K-build bandwidth, pipelined-GEMM roofline).
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    stg = {}
    with torch.cuda.stream(ctx.stream):
        e = [ev() for _ in range(5)]
        e[0].record(ctx.stream)
        kinds_k = (ctypes.c_int * len(kinds))(*kinds)
        ctx.check(lib.gpr_kernel(ctx.h, kinds_k, len(kinds), hpp, d, P(dx), N, None, N, 1, 1e-8,
                                 P(K), N), "gpr_kernel")
        e[1].record(ctx.stream)
        ctx.check(lib.gpr_potrf_upper(ctx.h, P(K), N, N, ctypes.byref(info)), "potrf")
        e[2].record(ctx.stream)
        alpha.copy_(dy)
        ctx.check(lib.gpr_potrs_upper(ctx.h, P(K), N, N, P(alpha), 1, N), "potrs")
        e[3].record(ctx.stream)
        posterior()
        e[4].record(ctx.stream)
        ctx.sync()
        f0, f1 = ev(), ev()
        lib.gpr_timing_reset(ctx.h)
        lib.gpr_timing_enable(ctx.h, 1)
        f0.record(ctx.stream)
        fit_predict()
        f1.record(ctx.stream)
        ctx.sync()
        lib.gpr_timing_enable(ctx.h, 0)
    fused_ms = f0.elapsed_time(f1)
    cls_get = lambda c: _timing(lib, ctx, c)  # noqa: E731
    cls = {nm: cls_get(c) for c, nm in
           enumerate(["kbuild", "syrk", "panel", "trsm_gemm", "other", "gemm_pipe", "dag"])}
    # the SE-ARD kernel (BASELINE configs[1]'s) at this size: the fit's upper-only K build
    # (gpr_fit, timing class 0), second of two runs -- the north_star's K-assembly target names
    # N = 32768, d = 8 without a kernel; the headline kbuild_* fields stay the C3 kernel's
    kse = kinds_of("SE")
    hse = default_hp(kse, d)
    kse_a = (ctypes.c_int * 1)(*kse)
    hse_p = hse.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    kb_se = None
    if a.kernel != "SE" and not a.no_se_ard:
        for _ in range(2):
            lib.gpr_timing_reset(ctx.h)
            lib.gpr_timing_enable(ctx.h, 1)
            rc = lib.gpr_fit(ctx.h, kse_a, 1, hse_p, d, P(dx), N, P(dy), 1, N, 1e-8, P(K), N,
                             P(alpha), ctypes.byref(info))
            ctx.sync()
            lib.gpr_timing_enable(ctx.h, 0)
            if rc < 0:  # (rc > 0, K not positive definite, still timed the build)
                break
            kb_se = cls_get(0)
    ceiling = store_ceiling(lib, ctx, K, N) if not a.no_se_ard else None
    names = ["kbuild", "potrf", "potrs", "posterior"]
    for i, nm in enumerate(names):
        stg[nm] = e[i].elapsed_time(e[i + 1])
    unfused_ms = sum(stg.values())
    # K-assembly of the fit (timing class 0 of the fused step): its "flops" slot carries the
    # bytes it writes -- the upper-only build writes the upper triangle and the 128 x 128
    # diagonal blocks (~4 N^2 + 512 N bytes; the tile-DAG writes the other half), the full
    # symmetric build 8 N^2 -- so the rate is honest for whichever ran
    kb_ms, _, kb_bytes = cls["kbuild"]
    kbuild_gbs = kb_bytes / (kb_ms * 1e-3) / 1e9
    potrf_tf = (N ** 3 / 3.0) / (stg["potrf"] * 1e-3) / 1e12
    # dominant kernel: the persistent tile-DAG launch (factorisation + the posterior solve of
    # [K(x, xp) | y], timing class 6) when it ran, else the pipelined GEMM of the blocked path
    # (timing class 5); each timed per launch with HIP events on the stream it runs on
    if cls["dag"][1] > 0:
        dominant = (DAG_KERNEL,)
        g_ms, g_launch, g_fl = cls["dag"]
    else:
        dominant = DOMINANT_KERNELS
        g_ms, g_launch, g_fl = cls["gemm_pipe"]
    achieved = g_fl / (g_ms * 1e-3) / 1e12 if g_ms > 0 else 0.0
    # the DAG kernel also runs alone (factorisation only) in the stage breakdown: its traffic
    # per JOB launch is the largest of the profiled launches
    traffic, traffic_src = pmc_traffic(dominant, N, NP, largest=dominant == (DAG_KERNEL,))

    out = None
    if rank == 0:
        out = {
            "metric": "GP-fit+predict wall-time and K-build GB/s + POTRF TFLOP/s at N=32768",
            "value": world / dt,
            "unit": "GP jobs/s (fit N=%d + posterior mean/var np=%d, per GPU)" % (N, NP),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (x~U[0,1)^(d x N) seeded, y=sin(sum x)^2)",
            "config": {"workload": f"{config_label(a)} fit+posterior: {a.kernel}, N={N}, d={d}, "
                                   f"np={NP}",
                       "N": N, "d": d, "np": NP, "kernel": a.kernel, "nb": a.nb,
                       "parallelism": f"replicas x{world}"},
            "kbuild_GBps": kbuild_gbs,
            "kbuild_hbm_frac": kbuild_gbs / HBM_PEAK_GBS,
            "kbuild_ms": kb_ms,
            "kbuild_bytes": kb_bytes,
            # the standalone full symmetric K (gpr_kernel, 8 N^2 bytes) of the unfused stages
            "kbuild_full_GBps": 8.0 * N * N / (stg["kbuild"] * 1e-3) / 1e9,
            "kbuild_se_ard": None if kb_se is None else {
                "kernel": "SE-ARD", "ms": kb_se[0], "bytes": kb_se[2],
                "GBps": kb_se[2] / (kb_se[0] * 1e-3) / 1e9,
                "hbm_frac": kb_se[2] / (kb_se[0] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "note": "the fit's upper-only K build for SE-ARD (configs[1]'s kernel) at this "
                        "N and d, timed inside gpr_fit; not the headline kernel",
                "frac_of_store_ceiling": (None if not ceiling else
                                          kb_se[2] / (kb_se[0] * 1e-3) / 1e9 / ceiling["best_GBps"])},
            # the same bytes written with no arithmetic, same box and process (pure-store kernels of
            # libgpr_store_probe.so): the store rate any upper-only K build is bounded by
            "kbuild_store_ceiling": ceiling,
            "potrf_TFLOPs": potrf_tf,
            "potrf_mfma_frac": potrf_tf / FP64_MFMA_PEAK,
            "stage_ms_unfused": stg,
            "unfused_job_ms": unfused_ms,
            "instrumented_step_ms": fused_ms,
            "syrk_TFLOPs": cls["syrk"][2] / (cls["syrk"][0] * 1e-3) / 1e12 if cls["syrk"][0] else None,
            # the persistent tile-DAG launch (whole factorisation at N <= 16384, else the tail)
            "dag_ms": cls["dag"][0], "dag_launches": cls["dag"][1],
            "dag_TFLOPs": cls["dag"][2] / (cls["dag"][0] * 1e-3) / 1e12 if cls["dag"][0] else None,
            "roofline": {
                "kernel": " + ".join(dominant),
                "bound": "mfma",
                "achieved": achieved,
                "peak": FP64_MFMA_PEAK,
                "unit": "TFLOP/s",
                "frac": achieved / FP64_MFMA_PEAK,
                "traffic": traffic,
                # HBM bytes per launch: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE of the
                # kernel's largest launch, from separate rocprofv3 --pmc passes of this command
                # (tools/profile_round.sh), read from the newest committed summary -- not
                # measured inside this run
                "traffic_source": (f"{traffic_src} (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE "
                                   "passes of this bench command; not measured in this run)"
                                   if traffic_src else None),
                "launches": g_launch,
                "avg_launch_us": g_ms * 1e3 / max(g_launch, 1),
                "flops_per_launch": g_fl / max(g_launch, 1),
                # rocprof MFMA counters of the same kernel (committed profile of this command)
                "pmc_mfma": pmc_mfma(dominant[0], N, NP),
            },
            "results_finite": ok,
            "dist_backend": a.dist_backend if world > 1 else None,
            "physical_gpus": ndev,
        }
        if world > 1 and a.dist_backend == "gloo":
            out["rehearsal"] = (f"{world} ranks sharing {ndev} device(s) over gloo: plumbing "
                                "check, not scaling data")
    if rank == 0:
        if not a.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = cpu_baseline(a, kinds, hp)
            except Exception as ex:  # never let the baseline leg kill the bench line
                out["cpu_baseline"] = {"value": None, "error": repr(ex)}
        else:
            out["cpu_baseline"] = None
        out["split_predict"] = ("skipped (--no-split)" if a.no_split else
                                "C5 leg runs after this line; its JSON object is on stderr")
        # the ONE stdout line, before the C5 leg: nothing in the leg can cost the headline
        print(json.dumps(out), flush=True)
    if not a.no_split:
        import threading

        def _watchdog():  # a leg stuck in a collective: end the process, line already out
            print(json.dumps({"split_predict": {"value": None, "error":
                                                f"timed out after {a.split_timeout:.0f} s"}}),
                  file=sys.stderr, flush=True)
            os._exit(3)  # (non-zero: a hung collective must not read as success)

        wd = threading.Timer(a.split_timeout, _watchdog)
        wd.daemon = True
        wd.start()
        try:
            with _StdoutToStderr():
                if not dist.is_initialized():  # one rank: a 1-process RCCL group for C5
                    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                    os.environ.setdefault("MASTER_PORT", "29541")
                    dist.init_process_group("nccl", rank=0, world_size=1,
                                            device_id=torch.device("cuda", local))
                split = split_leg(a, dist.get_world_size(), rank, local)
        except Exception as ex:  # (reported, never raised: the headline is already out)
            # (split_predict_distributed exchanges a status before each data collective, so a
            # failure raises on every rank at the same point and no rank is left blocked)
            split = {"value": None, "error": repr(ex)}
        wd.cancel()
        if rank == 0:
            print(json.dumps({"split_predict": split}), file=sys.stderr, flush=True)
    if dist.is_initialized():
        with _StdoutToStderr():
            dist.barrier()
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
