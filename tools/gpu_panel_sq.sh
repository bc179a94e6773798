#!/bin/bash
# POTRF N=32768: square-panel path (default) vs per-block panel path, across nb2.
set -e
cd "$(dirname "$0")/.."
for nb2 in 768 1024 1536 2048; do
  for sq in 1 0; do
    GPR_PANEL_SQ=$sq GPR_NB2=$nb2 timeout -k 10 120 tools/gemm_bench 32768 768 2 2>&1 | grep -i "potrf" | tail -1 | sed "s/^/sq=$sq nb2=$nb2 /"
  done
done
