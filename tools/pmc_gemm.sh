#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the GEMM microbench and on
# the library DGEMM, to compare MFMA busy fraction, LDS conflicts and waits.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/pmc_gemm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/own$i -o p -- $ROOT/tools/gemm_bench 8192 8192 1 > /dev/null 2>&1
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/lib$i -o p -- python3 $ROOT/tools/dgemm_ref.py > /dev/null 2>&1
done
echo done
