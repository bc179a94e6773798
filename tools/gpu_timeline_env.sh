#!/bin/bash
# Kernel trace of one standalone factorisation under an environment setting, for
# potrf_timeline.py.   usage: tools/gpu_timeline_env.sh tag N VAR=value [VAR=value ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; N=$2; shift 2
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/tl_${TAG}_$N
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- \
  $ROOT/tools/gemm_bench $N 0 2 > $OUT/out.txt 2> $OUT/err.txt
python3 $ROOT/tools/potrf_timeline.py $(find $OUT -name '*kernel_trace.csv' | head -1) > $OUT/timeline.txt
head -12 $OUT/timeline.txt
