#!/bin/bash
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "fit_predict or c3 or predict" --timeout 200 --timeout-method thread > gpurun_out/colfuse_tests.log 2>&1
rc=$?; tail -1 gpurun_out/colfuse_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_multi.sh 3 tools/ab/libgpr_base.so tools/ab/libgpr_new.so
