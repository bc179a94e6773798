# eigensolver: two-pass vs merged subproblem update (bitwise the same), VALU vs MFMA transform,
# then the kernel breakdown of the default under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "GPR_EIG_SUBK=1 GPR_EIG_TMFMA=1 GPR_EIG_SKIPI=1"; do
  echo "== $v"; env $v timeout -k 10 240 python tools/eig_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/eig_subk_r04h.txt 2>&1
echo "probe rc=$?"; cat gpurun_out/eig_subk_r04h.txt
GPR_EIG_SUBK=1 GPR_EIG_TMFMA=1 GPR_EIG_SKIPI=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eig -o eig -- python3 tools/eig_probe.py > gpurun_out/eig_prof_run.txt 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/prof_eig -name '*kernel_stats.csv'); echo "$f"; cut -d, -f1-8 $f > gpurun_out/eig_kstats.txt; cat gpurun_out/eig_kstats.txt
[ $rc = 0 ] && GPR_EIG_SUBK=1 GPR_EIG_TMFMA=1 GPR_EIG_SKIPI=1 timeout -k 10 300 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_r04h.log 2>&1; rc=$?; tail -3 gpurun_out/tests_r04h.log
exit $rc
