# shift-floor eigensolver + auto quadrature path: probe, quadrature timings, eigen/integrate tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
{ for m in 1 2 0 auto; do if [ $m = auto ]; then timeout -k 10 240 python tools/eig_vs_rocsolver.py || exit 1; else GPR_QUAD_EIGEN=$m timeout -k 10 240 python tools/eig_vs_rocsolver.py || exit 1; fi; done; } > gpurun_out/eig_vs_rocsolver_r04j.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/eig_vs_rocsolver_r04j.txt
timeout -k 10 300 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_r04j.log 2>&1; rc=$?; tail -5 gpurun_out/tests_r04j.log
exit $rc
