#!/bin/bash
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_kinv or potri or dag or mll or fit_predict" --timeout 120 --timeout-method thread > gpurun_out/gram2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gram2_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh 2
