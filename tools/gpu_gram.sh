#!/bin/bash
# K^{-1} = Z^T Z as gram tile tasks of the tile-DAG launch: parity subset, then the C4 split
# by timing class for the DAG gram (default), Z-only-in-DAG (fuse 1), blocked fuse 2 (no DAG
# gram), and the C4 bench line
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/gram.txt; : > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_kinv or potri or dag or mll or fit_predict" --timeout 120 --timeout-method thread > gpurun_out/gram_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gram_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
echo "default (DAG gram)" >> $out
timeout -k 10 120 python tools/probe_kinv.py 2>/dev/null | grep -v amdgpu >> $out || exit 1
echo "fuse=1" >> $out
GPR_FUSE_KINV=1 timeout -k 10 120 python tools/probe_kinv.py 2>/dev/null | grep -v amdgpu >> $out || exit 1
echo "fuse=0" >> $out
GPR_FUSE_KINV=0 timeout -k 10 120 python tools/probe_kinv.py 2>/dev/null | grep -v amdgpu >> $out || exit 1
timeout -k 10 200 python bench_mll.py > gpurun_out/gram_mll.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/gram_mll.json'));print('C4', round(d['ms_per_step'],2), 'ms')" >> $out
timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 --warmup 1 > gpurun_out/gram_c3.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/gram_c3.json'));print('C3', round(d['ms_per_step'],2), 'ms dag', round(d['dag_ms'],2), 'TF', round(d['dag_TFLOPs'],2))" >> $out
