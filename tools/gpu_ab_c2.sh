#!/bin/bash
# Same-box A/B of the in-tree library against tools/abl/libgpr_base.so (GPR_HIP_LIB) on C2
# (SE, N = 8192, np = 8192: job ms and the POTRF stage alone), alternating, after the parity
# file on the in-tree library.  Usage: tools/gpu_ab_c2.sh [reps] [c3 reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/ab_c2.txt; : > $out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_c2_tests.log 2>&1 || { tail -20 gpurun_out/ab_c2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_c2_tests.log)" >> $out
R=${1:-3}
for r in $(seq $R); do
  for v in base new; do
    if [ $v = base ]; then export GPR_HIP_LIB=$PWD/tools/abl/libgpr_base.so; else unset GPR_HIP_LIB; fi
    timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-split --no-cpu-baseline --steps 5 > gpurun_out/ab_c2.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_c2.json'));print('$v C2', round(d['ms_per_step'],3), 'ms potrf', round(d['stage_ms_unfused']['potrf'],3))" >> $out
  done
done
for r in $(seq ${2:-1}); do
  for v in base new; do
    if [ $v = base ]; then export GPR_HIP_LIB=$PWD/tools/abl/libgpr_base.so; else unset GPR_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/ab_c3.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_c3.json'));print('$v C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))" >> $out
  done
done
cat $out
