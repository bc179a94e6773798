set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_eigen.py tests/test_integrate.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_r04e.log 2>&1
echo "tests rc=$?"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/tests_r04e.log | tail -40
rm -f gpurun_out/kb_r04e.txt
for k in SE SE+SE+WN; do GPR_KBUILD_FULLCOLS=2 KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "sym|upper" | sed 's/^/fullcols2 /' >> gpurun_out/kb_r04e.txt 2>&1; GPR_KBUILD_FULLCOLS=2 KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_nostore | grep -E "sym" | sed 's/^/nostore fullcols2 /' >> gpurun_out/kb_r04e.txt 2>&1; done
cat gpurun_out/kb_r04e.txt
timeout -k 10 200 python bench_split.py --var-rows 1024 --steps 1 --warmup 1 > gpurun_out/bench_split_full_r04e.json 2> gpurun_out/bench_split_full_r04e.err; echo "split rc=$?"; cat gpurun_out/bench_split_full_r04e.json
timeout -k 10 600 bash tools/gpu_clock_stream.sh; echo "clock rc=$?"; cat gpurun_out/clock_stream/probe.txt
timeout -k 10 60 ./tools/probe/mfma_valu_overlap > gpurun_out/mfma_valu_overlap.txt 2>&1; echo "overlap rc=$?"; cat gpurun_out/mfma_valu_overlap.txt
for r in 1 2; do for k in SE SE+SE+WN; do KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_v1 | grep -E "upper" | sed "s/^/v1 /"; KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench | grep -E "upper" | sed "s/^/v2 /"; KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_nostore | grep -E "upper" | sed "s/^/v2 nostore /"; KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_v2m2 | grep -E "upper" | sed "s/^/v2m2 /"; done; done > gpurun_out/kb_v1v2.txt 2>&1; cat gpurun_out/kb_v1v2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fit_buffer or kernel_matrix or kernel_same or predict_vs_oracle" > gpurun_out/tests_r04e_kb.log 2>&1; echo "kb tests rc=$?"; tail -3 gpurun_out/tests_r04e_kb.log
