"""A/B of the fused MLL gradient pass at C4 (SE+WN, N = 16384, d = 16): the Gram form (default)
against the difference form (GPR_KBUILD_EXACT=1, set here on the context after the factor),
best of 5 after a warm-up, HIP events on the context stream.  Not a test."""
import ctypes
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussianprocessregression.jl_amd"))
import gpr_amd as G  # noqa: E402

N, d = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, 16
ctx = G.Context(0)
lib = G._lib.lib
hp = np.r_[1.0, [3.0 * math.sqrt(8.0 / d)] * d, 0.1]
karr = (ctypes.c_int * 2)(1, 2)
hpp = hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
x = np.random.default_rng(0).random((d, N))
y = np.sin(x.sum(0)) ** 2
dx, dy = ctx.colmajor(x), ctx.colmajor(y)
K, Kinv, alpha = ctx.empty(N, N), ctx.empty(N, N), ctx.empty(N)
info = ctypes.c_int(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
ctx.check(lib.gpr_fit_kinv(ctx.h, karr, 2, hpp, d, P(dx), N, P(dy), 1, N, 1e-8, P(K), N, P(alpha),
                           P(Kinv), N, ctypes.byref(info)), "fit_kinv")
g = np.zeros(len(hp))
gp = g.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
res = {}
for exact in (0, 1, 0, 1):
    ctx.set_knob("GPR_KBUILD_EXACT", exact)
    best = 1e30
    with torch.cuda.stream(ctx.stream):
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ctx.stream)
            ctx.check(lib.gpr_mll_grad(ctx.h, karr, 2, hpp, d, P(dx), N, P(Kinv), N, P(alpha), 1e-8, 1, gp),
                      "grad")
            e1.record(ctx.stream)
            ctx.sync()
            if r:
                best = min(best, e0.elapsed_time(e1))
    res.setdefault(exact, []).append((best, g.copy()))
    print(f"{'difference' if exact else 'gram      '} form: {best:.3f} ms", flush=True)
ga, gb = res[0][0][1], res[1][0][1]
print("max |gram - difference| / max|g|:", float(np.max(np.abs(ga - gb)) / np.max(np.abs(gb))))
