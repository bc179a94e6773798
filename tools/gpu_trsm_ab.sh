#!/bin/bash
# Tile-DAG off-diagonal tiles: U_ii^T X = B solved per tile (GPR_DAG_TRSM=1, default) against
# X = W_i^T B with W_i on the chain (=0).  Parity first, then same-box A/B rounds: POTRF alone
# (gemm_bench), the phase profile (dag_probe), C2 / C3 / C4 jobs.  usage: tools/gpu_trsm_ab.sh [reps]
cd $(dirname "$0")/..
set -o pipefail
R=${1:-2}
O=gpurun_out/trsm_ab.txt
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_trsm.log 2>&1 || { tail -30 gpurun_out/t_trsm.log; exit 1; }
tail -1 gpurun_out/t_trsm.log > $O
for r in $(seq $R); do
  for v in 0 1; do
    for n in 8192 16384; do
      echo "== r$r TRSM=$v potrf N=$n: $(GPR_DAG_TRSM=$v timeout -k 10 60 tools/gemm_bench $n 0 2 2>&1 | grep 'potrf N')" >> $O || exit 1
    done
    echo "== r$r TRSM=$v dag_probe 8192: $(GPR_DAG_TRSM=$v timeout -k 10 60 tools/probe/dag_probe 8192 | tail -1)" >> $O || exit 1
    echo "== r$r TRSM=$v C2: $(GPR_DAG_TRSM=$v timeout -k 10 120 python bench.py --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split --steps 5 2>/dev/null | tail -1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(round(j["ms_per_step"],2), "ms/job dag", round(j.get("dag_ms") or 0,2))')" >> $O || exit 1
    echo "== r$r TRSM=$v C3: $(GPR_DAG_TRSM=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-split --steps 3 2>/dev/null | tail -1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(round(j["ms_per_step"],2), "ms/job dag", round(j.get("dag_ms") or 0,2), "TF", round(j["roofline"]["achieved"],2))')" >> $O || exit 1
    echo "== r$r TRSM=$v C4: $(GPR_DAG_TRSM=$v timeout -k 10 200 python bench_mll.py --steps 3 2>/dev/null | tail -1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(round(j["ms_per_step"],2), "ms/eval")')" >> $O || exit 1
  done
done
cat $O
