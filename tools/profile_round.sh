#!/bin/bash
# Round profile of the default bench command: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes, then one pass of MFMA-busy counters; summaries land in
# gpurun_out/prof_<round>/ and are copied into profiles/ by the caller.
# The C5 split leg is skipped (--no-split) so every potrf_dag_kernel launch in the trace is
# one of the C3 step's own.   Usage: tools/profile_round.sh r01
set -e
R=${1:-r01}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$R
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $ROOT/bench.py --no-cpu-baseline --no-split --no-se-ard > $OUT/bench_traced.json 2> $OUT/trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- \
  python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-split --no-se-ard > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- \
  python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-split --no-se-ard > $OUT/bench_write.json 2> $OUT/write.err
# MFMA busy cycles vs the shader clock (GRBM_GUI_ACTIVE, summed over the 8 XCDs); the F64
# MFMA instruction counter joins the pass when this ROCm lists it
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
MF="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"
for c in SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64; do
  if grep -qw "$c" $OUT/avail.txt; then MF="$MF $c"; fi
done
echo "mfma pass: $MF" > $OUT/mfma_pass.txt
timeout -k 10 600 rocprofv3 --pmc $MF --output-format csv -d $OUT/mfma -o p -- \
  python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-split --no-se-ard > $OUT/bench_mfma.json 2> $OUT/mfma.err \
  || echo "mfma pass failed (see $OUT/mfma.err)" >> $OUT/mfma_pass.txt
python3 $ROOT/tools/pmc_summary.py $OUT 32768 8192 > $OUT/pmc_summary.json
echo profile done
