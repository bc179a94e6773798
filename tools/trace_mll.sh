#!/bin/bash
# Kernel trace of bench_mll.py (C4) for timeline analysis.   usage: tools/trace_mll.sh tag
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/trace_mll_${1:-x}
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- \
  python3 $ROOT/bench_mll.py --steps 1 --warmup 1 > $OUT/out.json 2> $OUT/err.txt
echo trace done
