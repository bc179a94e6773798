#!/bin/bash
# fused MLL gradient kernel rewrite: parity subset, then C4 A/B against tools/ab/libgpr_cur.so
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/grad_ab.txt; : > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -q -k "mll or grad or loss or c4 or train or kinv" --timeout 200 --timeout-method thread > gpurun_out/grad_tests.log 2>&1
rc=$?; tail -1 gpurun_out/grad_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in cur new; do
    if [ $lib = cur ]; then export GPR_HIP_LIB=$PWD/tools/ab/libgpr_cur.so; else unset GPR_HIP_LIB; fi
    timeout -k 10 200 python bench_mll.py > gpurun_out/ga.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ga.json'));print('$lib C4', round(d['ms_per_step'],2), 'grad stage', round(d['stage_ms_unfused']['mll+grad'],3))" >> $out
  done
done
