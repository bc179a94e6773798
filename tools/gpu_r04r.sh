# batched quadrature chunking test + batched cross-validation: timings and the GPU suites
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_cv.py > gpurun_out/bench_cv_r04r.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench_cv_r04r.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r04r.log 2>&1; rc=$?; tail -12 gpurun_out/tests_r04r.log
exit $rc
