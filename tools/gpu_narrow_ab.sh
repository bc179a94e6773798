#!/bin/bash
# A/B of the narrow right-hand-side tile path on one box (GPR_DAG_NARROW=0/1), C3 and C2
cd $(dirname "$0")/..
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    GPR_DAG_NARROW=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/c3_nar$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c3_nar$v.json'));print('C3 narrow=$v', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2), 'TF', round(d['dag_TFLOPs'],2))"
  done
done
for v in 0 1; do
  GPR_DAG_NARROW=$v timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split --steps 10 --warmup 2 > gpurun_out/c2_nar$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c2_nar$v.json'));print('C2 narrow=$v', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))"
done
