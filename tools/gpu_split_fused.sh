#!/bin/bash
# split predict with the fit fused: parity subset, then C5 (1 GPU) standalone and bench leg
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/split_fused.txt; : > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_fullsize.py -x -q -m gpu -k "split or fit_predict or fullsize" --timeout 200 --timeout-method thread > gpurun_out/split_fused_tests.log 2>&1
rc=$?; tail -1 gpurun_out/split_fused_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench_split.py > gpurun_out/sf_split.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sf_split.json'));print('C5 bench_split', round(d['ms_per_step'],1))" >> $out
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sf_bench.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/sf_bench.json'));print('C3', round(d['ms_per_step'],1), 'C5 leg', round(d['split_predict']['ms_per_step'],1))" >> $out
