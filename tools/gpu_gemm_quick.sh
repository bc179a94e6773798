set -o pipefail
mkdir -p gpurun_out
B=./tools/gemm_bench
{
timeout -k 5 60 $B 16384 128 0 | tail -1
timeout -k 5 60 $B 16384 256 0 | tail -1
timeout -k 5 60 $B 16384 512 0 | tail -1
timeout -k 5 60 $B 16384 128 1 | tail -1
timeout -k 5 60 $B 32768 128 0 | tail -1
timeout -k 5 60 $B 32768 256 0 | tail -1
timeout -k 5 120 $B 32768 0 2
} > gpurun_out/gemm_quick.log 2>&1
cat gpurun_out/gemm_quick.log
