set -o pipefail
mkdir -p gpurun_out
B=./tools/gemm_bench
{
for cfg in "1 1" "8 1" "8 0" "4 1" "16 1"; do
  set -- $cfg
  echo "== group=$1 xcd=$2"
  GPR_GEMM_GROUP=$1 GPR_GEMM_XCD=$2 timeout -k 5 60 $B 16384 128 0 | tail -1
  GPR_GEMM_GROUP=$1 GPR_GEMM_XCD=$2 timeout -k 5 60 $B 16384 256 0 | tail -1
  GPR_GEMM_GROUP=$1 GPR_GEMM_XCD=$2 timeout -k 5 60 $B 16384 128 1 | tail -1
done
echo "== potrf"
timeout -k 5 120 $B 16384 0 2
timeout -k 5 120 $B 32768 0 2
} > gpurun_out/gemm_ab.log 2>&1
cat gpurun_out/gemm_ab.log
