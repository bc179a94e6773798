# round 5: tridiagonal reduction -- parity tests, then timings against rocSOLVER / Jacobi
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_r05b.log 2>&1; rc=$?; tail -25 gpurun_out/tests_r05b.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/tridiag_probe.py > gpurun_out/tridiag_probe_r05b.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tridiag_probe_r05b.txt; exit $rc
