#!/bin/bash
# diag kernel v1 vs v2: POTRF timings (N = 32768, 16384, 4096), in-kernel stamps.
set -e
cd "$(dirname "$0")/.."
for n in 4096 32768 16384; do
  for v in v2 v1; do
    if [ $v = v1 ]; then export GPR_DIAG_V1=1; else unset GPR_DIAG_V1; fi
    timeout -k 10 60 tools/gemm_bench $n 768 2 2>&1 | sed "s/^/$v N=$n: /"
  done
done
