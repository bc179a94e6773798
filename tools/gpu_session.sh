#!/bin/bash
# One GPU call: gpu parity tests, default bench (with CPU baseline), C4/C5 benches, round profile.
# Usage: tools/gpu_session.sh rNN   (each step time-limited; stops at the first failure)
set -o pipefail
R=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -ra --timeout 300 --timeout-method thread > gpurun_out/tests_$R.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err && \
timeout -k 10 300 python bench_mll.py > gpurun_out/bench_mll_$R.json 2> gpurun_out/bench_mll_$R.err && \
timeout -k 10 300 python bench_split.py > gpurun_out/bench_split_$R.json 2> gpurun_out/bench_split_$R.err && \
bash tools/profile_round.sh $R
rc=$?
echo "session rc=$rc"
tail -3 gpurun_out/tests_$R.log; cat gpurun_out/bench_$R.json
exit $rc
