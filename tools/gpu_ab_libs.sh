#!/bin/bash
# Same-box A/B of two prebuilt libraries (GPR_HIP_LIB), C3 (DAG launch) alternating.
# Usage: tools/gpu_ab_libs.sh LIB_A LIB_B [reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/ab_libs.txt; : > $out
R=${3:-3}
for r in $(seq $R); do
  for lib in "$1" "$2"; do
    GPR_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/abl.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abl.json'));print('$lib C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))" >> $out
  done
done
