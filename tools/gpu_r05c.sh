set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_r05c.log 2>&1; rc=$?; tail -25 gpurun_out/tests_r05c.log
[ $rc = 0 ] || exit $rc
GPR_HIP_LIB=$PWD/gaussianprocessregression.jl_amd/gpr_amd/libgpr_hip_testing.so timeout -k 10 200 python tools/trd_trace.py 1100,4096 > gpurun_out/trd_trace_c.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/trd_trace_c.txt
timeout -k 10 400 python tools/tridiag_probe.py 512,1100,2048,4096 0,1,2 > gpurun_out/tridiag_probe_r05c.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tridiag_probe_r05c.txt; exit $rc
