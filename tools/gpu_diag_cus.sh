#!/bin/bash
# POTRF with CUs reserved for the diag kernel (GPR_DIAG_CUS), N = 32768 and 16384.
set -e
cd "$(dirname "$0")/.."
for n in 32768 16384; do
  for c in 0 1 2 8; do
    echo "== N=$n diag_cus=$c"
    GPR_DIAG_CUS=$c timeout -k 10 60 tools/gemm_bench $n 768 2 2>&1 | grep -v "sb0\|last diag"
  done
done
