#!/bin/bash
# auto solve-only DAG: potri / trsm parity, C4 unfused potri stage and C5, auto vs off
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/solve_auto.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "potri or trsm or split or fullsize or kinv" --timeout 200 --timeout-method thread > gpurun_out/solve_auto_tests.log 2>&1
rc=$?; tail -1 gpurun_out/solve_auto_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for v in 0 -1; do
  GPR_DAG_SOLVE=$v timeout -k 10 200 python bench_mll.py > gpurun_out/sa_mll.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sa_mll.json'));print('dag_solve=$v C4', round(d['ms_per_step'],2), 'potri stage', round(d['stage_ms_unfused']['potri'],2))" >> $out
  GPR_DAG_SOLVE=$v timeout -k 10 200 python bench_split.py > gpurun_out/sa_split.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sa_split.json'));print('dag_solve=$v C5', round(d['ms_per_step'],1))" >> $out
done
