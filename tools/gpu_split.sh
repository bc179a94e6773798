#!/bin/bash
# C5 split predict: parity subset (single-process and the RCCL-group tests), then the
# bench_split line and the bench's C5 leg
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -x -q -m gpu -k "split" --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; tail -2 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_split.py > gpurun_out/split_b.json 2> gpurun_out/split_b.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/split_b.json'));print('bench_split', round(d['ms_per_step'],1), 'ms', d['value'])"
