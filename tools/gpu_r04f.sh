set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "GPR_EIG_REORTH=0" "GPR_EIG_REORTH=1" "GPR_EIG_REORTH=1 GPR_EIG_INNER=2" "GPR_EIG_REORTH=1 GPR_EIG_INNER=1"; do
  echo "== $v"; env $v timeout -k 10 240 python tools/eig_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/eig_probe_r04f.txt 2>&1
echo "probe rc=$?"; cat gpurun_out/eig_probe_r04f.txt
timeout -k 10 500 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/tests_r04f.log 2>&1
echo "tests rc=$?"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/tests_r04f.log | tail -40
KB_FULLPAT=1 timeout -k 10 120 ./tools/kbuild_bench > gpurun_out/kb_fullpat.txt 2>&1; echo "fullpat rc=$?"; grep fullpat gpurun_out/kb_fullpat.txt
