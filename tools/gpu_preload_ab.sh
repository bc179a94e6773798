#!/bin/bash
# A/B of the C preload in the pipelined GEMM (GPR_GEMM_NOPRELOAD=1 disables it).
set -e
cd "$(dirname "$0")/.."
for args in "8192 8192 1" "16384 1024 0" "32768 1024 0" "16384 128 0" "32768 128 1" "8192 128 1"; do
  timeout -k 10 60 tools/gemm_bench $args 2>&1 | tail -1 | sed "s/^/pre:   /"
  GPR_GEMM_NOPRELOAD=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | tail -1 | sed "s/^/nopre: /"
done
timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep -i "potrf N" | sed "s/^/pre:   /"
GPR_GEMM_NOPRELOAD=1 timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep -i "potrf N" | sed "s/^/nopre: /"
