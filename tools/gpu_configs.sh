#!/bin/bash
# smoke() + the bench line at C2 (SE, N = 8192, np = 8192) and C1 (SE, N = 512, d = 2, np = 128),
# outputs under gpurun_out/ (usage: tools/gpu_configs.sh rNN)
set -o pipefail
R=${1:-r03}
cd $(dirname "$0")/..
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$R.txt 2>&1 || { tail -20 gpurun_out/smoke_$R.txt; exit 1; }
timeout -k 10 200 python bench.py --n 8192 --np 8192 --kernel SE --no-split --no-cpu-baseline --steps 5 > gpurun_out/bench_c2_$R.json 2> gpurun_out/bench_c2_$R.err || exit 1
timeout -k 10 120 python bench.py --n 512 --d 2 --np 128 --kernel SE --no-split --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_c1_$R.json 2> gpurun_out/bench_c1_$R.err || exit 1
tail -1 gpurun_out/smoke_$R.txt
for c in c2 c1; do
  python -c "
import json, sys
j = json.loads(open('gpurun_out/bench_${c}_$R.json').read().strip().splitlines()[-1])
print('$c', round(j['ms_per_step'], 3), 'ms/job; potrf', round(j['potrf_TFLOPs'], 2), 'TF/s; dag', j.get('dag_TFLOPs'), 'TF/s; kbuild', round(j['kbuild_GBps']), 'GB/s')"
done
