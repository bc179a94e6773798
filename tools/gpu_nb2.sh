set -o pipefail
mkdir -p gpurun_out
{
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/t4.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t4.log
for nb2 in 128 256 512 768 1024; do
  echo "== nb2=$nb2"; GPR_NB2=$nb2 timeout -k 5 100 ./tools/gemm_bench 32768 0 2 | tail -4
done
GPR_NB2=512 timeout -k 5 100 ./tools/gemm_bench 16384 0 2 | tail -4
} > gpurun_out/nb2.log 2>&1
cat gpurun_out/nb2.log
