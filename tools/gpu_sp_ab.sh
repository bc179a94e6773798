set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/spab
for k in low high normal; do
  GPR_MGPU_SP=$k timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/spab/$k -o st -- python3 tools/mgpu_stream_probe.py 32768 1 2 > gpurun_out/spab/$k.probe.txt 2>&1 || exit 1
  f=$(find gpurun_out/spab/$k -name "*kernel_trace.csv" | head -1)
  echo "== $k"; python3 tools/stream_overlap.py $f | tail -4
done
