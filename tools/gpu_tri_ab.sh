set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/tri_ab.txt; : > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread -k "potrf or fit or c2 or c3 or c4 or kinv or predict or trsm or solve" > gpurun_out/t_tri.log 2>&1 || { tail -30 gpurun_out/t_tri.log; exit 1; }
tail -1 gpurun_out/t_tri.log >> $O
for r in 1 2; do
  for v in _old ""; do
    echo "== r$r$v potrf 8192: $(timeout -k 10 60 tools/gemm_bench$v 8192 0 2 | grep 'potrf N' | tail -1)" >> $O || exit 1
    echo "== r$r$v dag_probe 8192: $(timeout -k 10 60 tools/probe/dag_probe$v 8192 | tail -1)" >> $O || exit 1
  done
done
bash tools/gpu_ab_lib.sh 2 && cat gpurun_out/ab_lib.txt >> $O
cat $O
