# tile-DAG ticket-order knobs on one box: C2 job with GPR_DAG_FEARLY 0/1 and GPR_DAG_RLAG 0/2,
# C4 evaluation with GPR_DAG_ZLAG 2/4 (tools/dag_sim.py predicted FEARLY +2 % at C2, ZLAG=4 +1 % at C4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/dag_knobs_r04k.txt; : > $out
for rep in 1 2; do
for v in "GPR_DAG_FEARLY=0" "GPR_DAG_FEARLY=1" "GPR_DAG_RLAG=2" "GPR_DAG_FEARLY=1 GPR_DAG_RLAG=2"; do
  r=$(env $v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split 2>/dev/null) || exit 1
  echo "C2 $v: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.3f ms  dag %.1f TF/s" % (d["ms_per_step"], d["dag_TFLOPs"]))')" >> $out
done
for v in "GPR_DAG_ZLAG=2" "GPR_DAG_ZLAG=4"; do
  r=$(env $v timeout -k 10 120 python bench_mll.py --steps 5 --warmup 2 2>/dev/null) || exit 1
  echo "C4 $v: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.3f ms" % d["ms_per_step"])')" >> $out
done
done
cat $out
