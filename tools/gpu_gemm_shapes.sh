#!/bin/bash
# Posterior-update GEMM shapes (M x 8192 x 1024, strided P and C) across tile-order settings.
set -e
cd "$(dirname "$0")/.."
for args in "8192 1024 3 30720 32768 32768" "8192 1024 3 30720 1024 30720" "8192 1024 3 16384 32768 32768" "8192 8192 1" "30720 1024 3 8192 1024 8192"; do
  for env in "" "GPR_GEMM_XCD=0" "GPR_GEMM_GROUP=4" "GPR_GEMM_GROUP=16"; do
    env $env timeout -k 10 60 tools/gemm_bench $args 2>&1 | tail -1 | sed "s/^/[$env] /"
  done
done
