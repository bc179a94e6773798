# eigensolver with the converged-pair early exit: probe (speed/accuracy), quadrature timing vs
# rocSOLVER / per-column, eigen + integrate tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 240 python tools/eig_probe.py > gpurun_out/eig_probe_r04i.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/eig_probe_r04i.txt
{ for m in 1 2 0; do GPR_QUAD_EIGEN=$m timeout -k 10 240 python tools/eig_vs_rocsolver.py || exit 1; done; } > gpurun_out/eig_vs_rocsolver_r04i.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/eig_vs_rocsolver_r04i.txt
timeout -k 10 300 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_r04i.log 2>&1; rc=$?; tail -3 gpurun_out/tests_r04i.log
exit $rc
