#!/bin/bash
# Z = U^{-T} inside the tile-DAG (GPR_FUSE_KINV=1) with the lower right-hand-side rows lagged
# behind A's rows by GPR_DAG_ZLAG; the default split (fuse 0) for reference
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/zlag.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_kinv or potri" --timeout 120 --timeout-method thread > gpurun_out/zlag_tests.log 2>&1
rc=$?; tail -1 gpurun_out/zlag_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
echo "fuse=0" >> $out
timeout -k 10 120 python tools/probe_kinv.py 2>/dev/null | grep -v amdgpu >> $out || exit 1
for l in 0 1 2 4 8; do
  echo "fuse=1 zlag=$l" >> $out
  GPR_FUSE_KINV=1 GPR_DAG_ZLAG=$l timeout -k 10 120 python tools/probe_kinv.py 2>/dev/null | grep -v amdgpu >> $out || exit 1
done
