# End-of-round check on one box: the whole -m gpu suite in one process, then smoke() and the
# default bench line (both into gpurun_out/final6/).  Usage: bash tools/gpu_r06_final.sh [tests|bench]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final6
O=gpurun_out/final6
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 1080 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
else
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
fi
echo done
