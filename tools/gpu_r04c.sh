set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/kb_r04c.txt
for w in 3 4 6 8 12; do for k in SE SE+SE+WN; do GPR_KBUILD_UWGS=$w KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "upper|sym" | sed "s/^/uwgs=$w /" >> gpurun_out/kb_r04c.txt 2>&1; done; done
for k in SE SE+SE+WN; do KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_nostore | grep -E "upper|sym" | sed 's/^/nostore /' >> gpurun_out/kb_r04c.txt 2>&1; done
cat gpurun_out/kb_r04c.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fit_buffer or kernel_matrix or potrf_dag or fit_predict or fit_kinv" > gpurun_out/tests_r04c.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/tests_r04c.log
