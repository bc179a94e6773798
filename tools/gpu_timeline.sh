#!/bin/bash
# Kernel traces of standalone factorisations (tools/gemm_bench N 0 2) for potrf_timeline.py.
# usage: tools/gpu_timeline.sh tag N [N ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for N in "$@"; do
  OUT=$ROOT/gpurun_out/tl_${TAG}_$N
  rm -rf $OUT && mkdir -p $OUT
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- \
    $ROOT/tools/gemm_bench $N 0 2 > $OUT/out.txt 2> $OUT/err.txt
  cat $OUT/out.txt
  python3 $ROOT/tools/potrf_timeline.py $(find $OUT -name '*kernel_trace.csv' | head -1) > $OUT/timeline.txt
  head -30 $OUT/timeline.txt
done
