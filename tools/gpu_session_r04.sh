#!/bin/bash
# Round-4 session: full GPU parity suite, default bench (with CPU baseline and both C5 legs),
# C4 / C5-full benches, the round profile (kernel trace + FETCH / WRITE / MFMA pmc passes).
# Usage: tools/gpu_session_r04.sh rNN
set -o pipefail
R=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -ra --timeout 300 --timeout-method thread > gpurun_out/tests_$R.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err && \
timeout -k 10 300 python bench_mll.py > gpurun_out/bench_mll_$R.json 2> gpurun_out/bench_mll_$R.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --n 8192 --np 8192 --kernel SE --no-cpu-baseline --no-split > gpurun_out/bench_c2_$R.json 2> gpurun_out/bench_c2_$R.err && \
{ for m in 1 2 0; do GPR_QUAD_EIGEN=$m timeout -k 10 240 python tools/eig_vs_rocsolver.py || exit 1; done; } > gpurun_out/eig_vs_rocsolver_$R.txt 2>&1 && \
bash tools/profile_round.sh $R
rc=$?
echo "session rc=$rc"
tail -3 gpurun_out/tests_$R.log; cat gpurun_out/bench_$R.json; grep split_predict gpurun_out/bench_$R.err; grep -v amdgpu.ids gpurun_out/eig_vs_rocsolver_$R.txt
exit $rc
