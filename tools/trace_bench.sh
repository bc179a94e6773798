#!/bin/bash
# Kernel trace of one short bench run (for timeline analysis with tools/trace_window.py).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/trace_${1:-x}
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- \
  python3 $ROOT/${2:-bench.py} --steps 1 --warmup 1 ${3:---no-cpu-baseline} > $OUT/out.json 2> $OUT/err.txt
echo trace done
