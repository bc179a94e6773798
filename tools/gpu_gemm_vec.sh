#!/bin/bash
# A/B of the GEMM variants: pipelined 1-WG/CU (GPR_GEMM_PIPE=1), pipelined 2-WG/CU
# (GPR_GEMM_PIPE=2), register-staged 2-WG/CU (GPR_GEMM_NOPIPE=1).
set -e
cd "$(dirname "$0")/.."
for args in "8192 8192 1" "16384 768 1" "32768 768 0" "16384 768 0" "4096 4096 1" "16384 1536 0"; do
  for m in 1 2; do
    GPR_GEMM_PIPE=$m timeout -k 10 60 tools/gemm_bench $args 2>&1 | tail -1 | sed "s/^/pipe$m: /"
  done
  GPR_GEMM_NOPIPE=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | tail -1 | sed 's/^/nopipe: /'
done
for nb2 in 768 1024 1536; do
  GPR_NB2=$nb2 timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep -i "potrf" | tail -1 | sed "s/^/nb2=$nb2 /"
done
