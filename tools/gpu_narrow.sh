#!/bin/bash
# Narrow right-hand-side tiles in the tile-DAG: parity subset, then C3 and C2 benches
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dag or potri or fit_kinv or fit_predict" --timeout 120 --timeout-method thread > gpurun_out/narrow_tests.log 2>&1
rc=$?; tail -2 gpurun_out/narrow_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/c3_narrow$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3_narrow$r.json'));print('C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2), 'TF', round(d['dag_TFLOPs'],2))"
done
timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split --steps 10 --warmup 2 > gpurun_out/c2_narrow.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/c2_narrow.json'));print('C2', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))"
