#!/bin/bash
# Round profile of the default bench command: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes; summaries land in gpurun_out/prof_<round>/ and are
# copied into profiles/ by the caller.   Usage: tools/profile_round.sh r01
set -e
R=${1:-r01}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$R
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $ROOT/bench.py --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- \
  python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- \
  python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/write.err
python3 $ROOT/tools/pmc_summary.py $OUT 32768 8192 > $OUT/pmc_summary.json
echo profile done
