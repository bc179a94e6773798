#!/bin/bash
# POTRF N=32768 stage breakdown across outer-panel widths (GPR_NB2).
set -e
cd "$(dirname "$0")/.."
for nb2 in 768 1024 1536 2048; do
  echo "== nb2=$nb2"
  GPR_NB2=$nb2 timeout -k 10 60 tools/gemm_bench 32768 768 2 2>&1 | grep -v "stamps\|sb0"
done
