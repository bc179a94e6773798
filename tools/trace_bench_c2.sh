#!/bin/bash
# Kernel trace of the C2 bench step (bench.py --n 8192 --np 8192 --kernel SE) for timeline analysis.
# usage: tools/trace_bench_c2.sh tag [VAR=value ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
OUT=$ROOT/gpurun_out/trace_c2_$TAG
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- \
  python3 $ROOT/bench.py --n 8192 --np 8192 --kernel SE --steps 2 --warmup 1 --no-cpu-baseline > $OUT/out.json 2> $OUT/err.txt
echo trace done
