#!/bin/bash
# pipelined-GEMM barrier scheduling: GEMM/TRSM/blocked parity with the new library, then the
# blocked C3 (GPR_DAG=0) and the default bench's unfused posterior stage, both libraries
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/gemm_sb.txt; : > $out
GPR_HIP_LIB=$PWD/tools/ab/libgpr_gemmsb.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "gemm or potrf or trsm or potri or predict or split" --timeout 120 --timeout-method thread > gpurun_out/gemm_sb_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gemm_sb_tests.log >> $out; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in libgpr_cur libgpr_gemmsb; do
    GPR_DAG=0 GPR_HIP_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 2 --warmup 1 > gpurun_out/gsb.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/gsb.json'));print('$lib DAG=0 C3', round(d['ms_per_step'],2), 'potrf', round(d['stage_ms_unfused']['potrf'],2), 'posterior', round(d['stage_ms_unfused']['posterior'],2))" >> $out
  done
done
