#!/bin/bash
# C5 (1 GPU): the variance right-hand sides through the blocked TRSM vs the solve-only DAG
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/split_ab.txt; : > $out
for r in 1 2; do
  for v in 0 1; do
    GPR_DAG_SOLVE=$v timeout -k 10 200 python bench_split.py > gpurun_out/split_ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/split_ab.json'));print('dag_solve=$v', round(d['ms_per_step'],1))" >> $out
  done
done
