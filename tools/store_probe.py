"""Pure-store ceilings of the upper-only K build (csrc/probe/store_ceiling.hip), all patterns, N
from argv (default 32768), three rounds -- the box's store-rate spread.  Not a test."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pl = ctypes.CDLL(os.path.join(ROOT, "gaussianprocessregression.jl_amd", "gpr_amd", "libgpr_store_probe.so"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
K = torch.empty(n, n, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
names = ["kernel_pattern", "item_per_wave", "chunk1k_column_order", "items_1k_column_stores",
         "items16_1k_column_stores", "items_1k_column_stores_item_per_wave"]
for rnd in range(3):
    for pat, nm in enumerate(names):
        ms, nb = ctypes.c_double(), ctypes.c_double()
        rc = pl.gpr_probe_upper_store(ctypes.c_void_p(s.cuda_stream), n, ctypes.c_void_p(K.data_ptr()),
                                      pat, 3, ctypes.byref(ms), ctypes.byref(nb))
        print(f"round {rnd} {nm:26s} rc={rc} {ms.value:.3f} ms {nb.value / ms.value / 1e6:.0f} GB/s", flush=True)
