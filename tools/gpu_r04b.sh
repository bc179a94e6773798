set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fit_buffer or kernel_matrix or potrf_dag or fit_predict or fit_kinv or mgpu" > gpurun_out/tests_r04b.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/tests_r04b.log
for k in SE SE+SE+WN; do KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench >> gpurun_out/kb_r04b.txt 2>&1; KB_ONLY=$k timeout -k 10 60 ./tools/kbuild_bench_nostore | sed 's/^/nostore /' >> gpurun_out/kb_r04b.txt 2>&1; done
cat gpurun_out/kb_r04b.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 180 --timeout-method thread -k "buffer" > gpurun_out/tests_full_r04b.log 2>&1; echo "full rc=$?"; tail -3 gpurun_out/tests_full_r04b.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-split --steps 5 > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err; echo "bench rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04b.json'));print({k:d[k] for k in ['ms_per_step','kbuild_GBps','kbuild_hbm_frac','kbuild_ms','kbuild_full_GBps','dag_ms','dag_TFLOPs']})"
