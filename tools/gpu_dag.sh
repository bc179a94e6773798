#!/bin/bash
# Tile-DAG factorisation: parity tests, then standalone timings against the blocked path
# (whole-matrix DAG, and blocked with the DAG tail hand-off).
# usage: tools/gpu_dag.sh "N1 N2 ..." "TAIL1 TAIL2 ..."
cd $(dirname "$0")/..
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dag" --timeout 120 --timeout-method thread > gpurun_out/dag_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dag_tests.log; [ $rc -ne 0 ] && exit $rc
for N in ${1:-8192 16384 32768}; do
  timeout -k 10 60 tools/gemm_bench $N 0 2 2>&1 | grep "potrf N" | sed "s/^/blocked /"
  GPR_DAG=1 timeout -k 10 60 tools/gemm_bench $N 0 2 2>&1 | grep "potrf N" | sed "s/^/dag     /"
  for T in ${2:-}; do
    GPR_DAG_TAIL=$T timeout -k 10 60 tools/gemm_bench $N 0 2 2>&1 | grep "potrf N" | sed "s/^/tail$T /"
  done
done
