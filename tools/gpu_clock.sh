#!/bin/bash
# Clock under load: a pure back-to-back FP64 MFMA kernel (~300 ms launches) against the DAG
# job launch, same box, GRBM_GUI_ACTIVE / duration from one --pmc pass each
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/clock
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $ROOT/tools/probe/mfma_f64_peak 70 1 > $OUT/peak.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/peak -o p -- $ROOT/tools/probe/mfma_f64_peak 70 1 > $OUT/peak_pmc.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/dag -o p -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-split > $OUT/dag.json 2> $OUT/dag.err || exit 1
echo clock done
