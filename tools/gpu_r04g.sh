# K-build item geometry A/B (16x128 default vs 32x256 / 16x256 / 32x128) + parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/kb_geom_r04g.txt; : > $out
for b in kbuild_bench kbuild_bench_w32s256 kbuild_bench_w16s256 kbuild_bench_w32s128; do
  for c in SE SE+SE+WN; do
    echo "== $b $c" >> $out
    KB_ONLY=$c timeout -k 10 120 ./tools/$b 32768 8 >> $out 2>&1 || exit 1
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "buffer or kernel" > gpurun_out/tests_r04g.log 2>&1
rc=$?; tail -5 gpurun_out/tests_r04g.log; exit $rc
