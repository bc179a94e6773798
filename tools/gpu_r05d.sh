set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_r05d.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/tests_r05d.log | tail -60; tail -5 gpurun_out/tests_r05d.log
exit $rc
