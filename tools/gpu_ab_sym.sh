cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sym_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sym_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then GB=tools/ab/gemm_bench_base; export GPR_HIP_LIB=$PWD/tools/ab/libgpr_base.so; else GB=tools/gemm_bench; unset GPR_HIP_LIB; fi
    echo "== r$r $v potrf 8192: $(GPR_DAG=1 timeout -k 10 60 $GB 8192 0 2 2>&1 | grep 'potrf N' | tail -1)"
    timeout -k 10 120 python bench.py --n 8192 --kernel SE --np 8192 --no-split --no-cpu-baseline --steps 5 > gpurun_out/ab_c2.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_c2.json'));print('== r$r $v C2 job', round(d['ms_per_step'],3), 'ms potrf stage', round(d['stage_ms_unfused']['potrf'],3))"
  done
done
bash tools/gpu_ab_lib.sh 2 && cat gpurun_out/ab_lib.txt
