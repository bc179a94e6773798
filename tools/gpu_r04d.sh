set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/kb_r04d.txt
for k in SE SE+SE+WN; do KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "upper|sym" >> gpurun_out/kb_r04d.txt 2>&1; GPR_KBUILD_FULLCOLS=2 KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "sym" | sed 's/^/fullcols2 /' >> gpurun_out/kb_r04d.txt 2>&1; GPR_KBUILD_FULLCOLS=0 KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "sym" | sed 's/^/fullcols0 /' >> gpurun_out/kb_r04d.txt 2>&1; KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_nostore | grep -E "upper|sym" | sed 's/^/nostore /' >> gpurun_out/kb_r04d.txt 2>&1; done
cat gpurun_out/kb_r04d.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fit_buffer or kernel or potrf_dag or fit_predict or fit_kinv or predict" > gpurun_out/tests_r04d.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/tests_r04d.log
