#!/bin/bash
# Round-5 session, in two gpurun calls:
#   tools/gpu_session_r05.sh tests rNN  -- full GPU parity suite + smoke()
#   tools/gpu_session_r05.sh bench rNN  -- default bench (CPU baseline, C5 legs), C4, C2, C5 full,
#                                          the eigensolver timings, the round profile
set -o pipefail
PH=${1:-tests}
R=${2:-r05}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$PH" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -ra --timeout 300 --timeout-method thread > gpurun_out/tests_$R.log 2>&1 && \
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$R.txt 2>&1
  rc=$?
  tail -3 gpurun_out/tests_$R.log; tail -2 gpurun_out/smoke_$R.txt
  exit $rc
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err && \
timeout -k 10 300 python bench_mll.py > gpurun_out/bench_mll_$R.json 2> gpurun_out/bench_mll_$R.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --n 8192 --np 8192 --kernel SE --no-split > gpurun_out/bench_c2_$R.json 2> gpurun_out/bench_c2_$R.err && \
timeout -k 10 300 python bench_split.py > gpurun_out/bench_split_$R.json 2> gpurun_out/bench_split_$R.err && \
TRD_PROBE_CPU=1 timeout -k 10 400 python -u tools/tridiag_probe.py > gpurun_out/eig_speed_$R.txt 2>&1 && \
bash tools/profile_round.sh $R
rc=$?
echo "session rc=$rc"
cat gpurun_out/bench_$R.json; grep split_predict gpurun_out/bench_$R.err
exit $rc
