#!/bin/bash
# Same-box comparison of several prebuilt libraries (GPR_HIP_LIB): DAG parity subset per
# library, then C3 rounds in rotation.  Usage: tools/gpu_ab_multi.sh reps lib1 lib2 ...
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/ab_multi.txt; : > $out
R=$1; shift
for lib in "$@"; do
  GPR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "potrf_dag or fit_predict_dag" --timeout 60 --timeout-method thread > gpurun_out/abm_tests.log 2>&1 || { echo "$lib tests FAILED" >> $out; exit 1; }
  echo "$lib $(tail -1 gpurun_out/abm_tests.log)" >> $out
done
for r in $(seq $R); do
  for lib in "$@"; do
    GPR_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/abm.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abm.json'));print('$lib C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2))" >> $out
  done
done
