#!/bin/bash
# Same-box A/B of the in-tree library against tools/ab/libgpr_base.so (GPR_HIP_LIB), C3 and C4,
# alternating.  Usage: tools/gpu_ab_lib.sh [reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/ab_lib.txt; : > $out
R=${1:-2}
for r in $(seq $R); do
  for v in base new; do
    if [ $v = base ]; then export GPR_HIP_LIB=$PWD/tools/ab/libgpr_base.so; else unset GPR_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/ab_c3.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_c3.json'));print('$v C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))" >> $out
    timeout -k 10 200 python bench_mll.py > gpurun_out/ab_c4.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_c4.json'));print('$v C4', round(d['ms_per_step'],2), 'ms')" >> $out
  done
done
