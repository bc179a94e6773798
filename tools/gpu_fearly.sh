#!/bin/bash
# early diagonal tasks (GPR_DAG_FEARLY): parity subset with it on, then C2 / C3 / C4 A/B
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/fearly.txt; : > $out
GPR_DAG_FEARLY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "dag or fit_kinv or fit_predict or potri or trsm or c3 or c4" --timeout 200 --timeout-method thread > gpurun_out/fearly_tests.log 2>&1
rc=$?; tail -1 gpurun_out/fearly_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 1; do
    GPR_DAG_FEARLY=$v timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split --steps 10 --warmup 2 > gpurun_out/fe.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/fe.json'));print('fearly=$v C2', round(d['ms_per_step'],2), 'dag', round(d['dag_ms'],2))" >> $out
    GPR_DAG_FEARLY=$v timeout -k 10 200 python bench_mll.py > gpurun_out/fe4.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/fe4.json'));print('fearly=$v C4', round(d['ms_per_step'],2))" >> $out
    GPR_DAG_FEARLY=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/fe3.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/fe3.json'));print('fearly=$v C3', round(d['ms_per_step'],2), 'dag', round(d['dag_ms'],2))" >> $out
  done
done
