#!/bin/bash
# GEMM correctness (sampled naive check) for the pipelined / register-staged kernels.
set -e
cd "$(dirname "$0")/.."
for args in "4096 1024 0" "4096 1024 1" "4000 128 1" "4000 128 0" "8192 128 1"; do
  GEMM_VERIFY=1 GPR_GEMM_PIPE=1 GPR_GEMM_NOPRELOAD=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | grep verify | sed "s/^/pipe16: /"
  GEMM_VERIFY=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | grep verify | sed "s/^/pre:    /"
  GEMM_VERIFY=1 GPR_GEMM_NOPRELOAD=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | grep verify | sed "s/^/nopre:  /"
  GEMM_VERIFY=1 GPR_GEMM_NOPIPE=1 timeout -k 10 60 tools/gemm_bench $args 2>&1 | grep verify | sed "s/^/nopipe: /"
done
timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep "potrf N" | sed "s/^/pre:    /"
GPR_GEMM_NOPRELOAD=1 timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep "potrf N" | sed "s/^/nopre:  /"
