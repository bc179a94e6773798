# batched per-column quadrature (one tile-DAG launch for all K + s_j I): timings against the
# eigensolver, rocSOLVER and the sequential per-column path; eigen + integrate tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
{ GPR_QUAD_EIGEN=1 timeout -k 10 240 python tools/eig_vs_rocsolver.py && \
  GPR_QUAD_EIGEN=2 timeout -k 10 240 python tools/eig_vs_rocsolver.py && \
  GPR_QUAD_EIGEN=0 GPR_QUAD_SEQ=1 timeout -k 10 240 python tools/eig_vs_rocsolver.py && \
  GPR_QUAD_EIGEN=0 timeout -k 10 240 python tools/eig_vs_rocsolver.py && \
  timeout -k 10 240 python tools/eig_vs_rocsolver.py; } > gpurun_out/eig_vs_rocsolver_r04p.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/eig_vs_rocsolver_r04p.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_r04p.log 2>&1; rc=$?; tail -5 gpurun_out/tests_r04p.log
exit $rc
