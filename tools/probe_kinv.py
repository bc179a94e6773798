"""C4's gpr_fit_kinv split by timing class (kbuild / syrk / panel / trsm_gemm / other /
gemm_pipe / dag): where the 80 ms go.  Usage: python tools/probe_kinv.py [N] [d]"""
import ctypes
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
import gpr_amd as G  # noqa: E402
from gpr_amd._lib import lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
ctx = G.Context(0)
kinds = (ctypes.c_int * 2)(1, 2)  # GPR_SE, GPR_WN
hp = np.r_[1.0, [3.0 * math.sqrt(8.0 / d)] * d, 0.1]
hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
x = np.random.default_rng(0).random((d, N))
y = np.sin(x.sum(0)) ** 2
dx, dy = ctx.colmajor(x), ctx.colmajor(y)
K, Kinv, alpha = ctx.empty(N, N), ctx.empty(N, N), ctx.empty(N)
info = ctypes.c_int(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
names = ["kbuild", "syrk", "panel", "trsm_gemm", "other", "gemm_pipe", "dag"]
for rep in range(3):
    lib.gpr_timing_reset(ctx.h)
    lib.gpr_timing_enable(ctx.h, 1 if rep == 2 else 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(ctx.stream):
        e0.record(ctx.stream)
        ctx.check(lib.gpr_fit_kinv(ctx.h, kinds, 2, hpp, d, P(dx), N, P(dy), 1, N, 1e-8, P(K), N,
                                   P(alpha), P(Kinv), N, ctypes.byref(info)), "fit_kinv")
        e1.record(ctx.stream)
    ctx.sync()
    print(f"rep {rep}: fit_kinv {e0.elapsed_time(e1):.2f} ms info={info.value}")
lib.gpr_timing_enable(ctx.h, 0)
for c, nm in enumerate(names):
    ms, ln, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
    lib.gpr_timing_get(ctx.h, c, ctypes.byref(ms), ctypes.byref(ln), ctypes.byref(fl))
    if ln.value:
        tf = fl.value / (ms.value * 1e-3) / 1e12 if ms.value else 0
        print(f"  {nm:10s} {ms.value:8.2f} ms  {ln.value:5d} launches  {tf:6.1f} TF/s")
