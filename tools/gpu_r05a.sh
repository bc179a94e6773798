# round 5: the GPU suite after the knob cleanup (release vs testing library), smoke, and the
# C4 / C5 benches with their new CPU baselines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r05a.log 2>&1; rc=$?; tail -15 gpurun_out/tests_r05a.log
[ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench_mll.py --steps 3 > gpurun_out/bench_mll_r05a.json 2> gpurun_out/bench_mll_r05a.err || exit $?
cat gpurun_out/bench_mll_r05a.json
timeout -k 10 300 python bench_split.py --steps 2 > gpurun_out/bench_split_r05a.json 2> gpurun_out/bench_split_r05a.err || exit $?
cat gpurun_out/bench_split_r05a.json
