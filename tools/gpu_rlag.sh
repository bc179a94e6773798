#!/bin/bash
# right-hand-side row lag (GPR_DAG_RLAG) for C2 / C3, alternating settings
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/rlag.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_predict_dag" --timeout 120 --timeout-method thread > gpurun_out/rlag_tests.log 2>&1
rc=$?; tail -1 gpurun_out/rlag_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for l in 0 1 2 4; do
    GPR_DAG_RLAG=$l timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split --steps 10 --warmup 2 > gpurun_out/rl.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/rl.json'));print('rlag=$l C2', round(d['ms_per_step'],2), 'dag', round(d['dag_ms'],2))" >> $out
  done
done
for l in 0 2; do
  GPR_DAG_RLAG=$l timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/rl3.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/rl3.json'));print('rlag=$l C3', round(d['ms_per_step'],2), 'dag', round(d['dag_ms'],2))" >> $out
done
