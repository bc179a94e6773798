#!/bin/bash
# DAG accumulate-loop scheduling change: parity subset, then same-box A/B against
# tools/ab/libgpr_base.so (C3 and C4, alternating, 3 rounds)
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dag or fit_kinv or fit_predict or potri" --timeout 120 --timeout-method thread > gpurun_out/sched_tests.log 2>&1
rc=$?; tail -1 gpurun_out/sched_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh 3
