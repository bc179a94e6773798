#!/bin/bash
# Does the DAG's HBM operand stream cost clock?  The DAG's accumulation loop in isolation
# (tools/probe/accum_probe config 0: 128 x 128 tiles, 4 waves, four 16-deep LDS-DMA stages),
# once with its operands held in L2 (mode 2: K wrapped at 1024 rows, 2 MB of operands) and once
# streamed from HBM as the DAG streams them (mode 1: a row's shared panel + a private column
# panel per workgroup, 4.3 GB of operands, ~4.5 TB/s).  Effective clock = GRBM_GUI_ACTIVE /
# 8 XCDs / dispatch duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024
# SIMDs), one --pmc pass each (+ kernel trace for the durations).
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/clock_stream
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for mode in 2 1 2 1; do
  timeout -k 10 120 $ROOT/tools/probe/accum_probe 65536 20 0 $mode >> $OUT/probe.txt 2>&1 || exit 1
done
for mode in 2 1; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_m$mode -o p -- $ROOT/tools/probe/accum_probe 65536 20 0 $mode > $OUT/pmc_m$mode.txt 2>&1 || exit 1
done
echo clock_stream done
