set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -ra --maxfail=20 > gpurun_out/t2.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t2.log
timeout -k 10 600 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof1 -o run -f csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/prof1.log 2>&1
echo "rc=$?"
tail -5 gpurun_out/t2.log; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err
