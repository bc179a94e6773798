#!/bin/bash
# Tile-DAG in the benches: parity subset, then C2 (fit+predict, N = 8192) without / with the
# DAG, C3 with the tail hand-off.
cd $(dirname "$0")/..
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dag" --timeout 120 --timeout-method thread > gpurun_out/dag_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dag_tests.log; [ $rc -ne 0 ] && exit $rc
C2="--n 8192 --np 8192 --kernel SE --no-cpu-baseline --steps 10 --warmup 2"
for v in 0 1; do
  GPR_DAG=$v timeout -k 10 120 python bench.py $C2 > gpurun_out/c2_dag$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c2_dag$v.json'));print('C2 dag=$v', round(d['ms_per_step'],2), 'ms', {k:round(v,2) for k,v in d['stage_ms_unfused'].items()})"
done
for t in 0 12288 16384; do
  GPR_DAG_TAIL=$t timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/c3_tail$t.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3_tail$t.json'));print('C3 tail=$t', round(d['ms_per_step'],2), 'ms', {k:round(v,2) for k,v in d['stage_ms_unfused'].items()})"
done
