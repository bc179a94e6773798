#!/bin/bash
# split fit + variance fused vs not (GPR_SPLIT_FUSE), at 4 and 32 variance rows (1 GPU)
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/split_fuse_ab.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "split" --timeout 200 --timeout-method thread > gpurun_out/sfab_tests.log 2>&1
rc=$?; tail -1 gpurun_out/sfab_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for vr in 4 8 32; do
  for f in 0 1; do
    GPR_SPLIT_FUSE=$f timeout -k 10 200 python bench_split.py --var-rows $vr > gpurun_out/sfab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/sfab.json'));print('var_rows=$vr fuse=$f', round(d['ms_per_step'],1))" >> $out
  done
done
