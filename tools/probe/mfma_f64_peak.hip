// FP64 MFMA issue-rate probe: every wave issues back-to-back v_mfma_f64_16x16x4f64 (inline
// asm, accumulators pinned in VGPRs) on NA independent accumulators; 1, 2 or 4 workgroups of
// 4 waves per CU.  Answers: can ONE wave per SIMD keep the f64 matrix pipe full?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4v __attribute__((ext_vector_type(4)));

template <int NA>
__global__ __launch_bounds__(256) void peak_kernel(double* out, int iters, double a0, double b0) {
  d4v acc[NA];
  for (int i = 0; i < NA; ++i) acc[i] = d4v{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0;
  for (int i = 0; i < NA; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;
}

int main(int argc, char** argv) {
  // argv[1]: iteration multiplier (1: ~4 ms per launch; 70: ~300 ms, long enough for the
  // clock to settle under load); argv[2] = 1: only the 16-accumulator / 1 WG per CU case
  const int mult = argc > 1 ? atoi(argv[1]) : 1;
  const bool one = argc > 2 && atoi(argv[2]) == 1;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  double* out;
  (void)hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](auto kern, int na) {
    for (int wgpc = 1; wgpc <= (one ? 1 : 2); wgpc *= 2) {
      const int grid = cus * wgpc, iters = 160000 / na * mult;
      kern<<<grid, 256>>>(out, 10, 1.0, 1.0);
      (void)hipEventRecord(e0);
      kern<<<grid, 256>>>(out, iters, 1.0, 1.0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double flops = (double)grid * 4 * iters * na * 2048.0;
      printf("mfma_f64_16x16x4 (asm): acc %2d WG/CU %d: %.2f TFLOP/s (%.3f ms)\n", na, wgpc,
             flops / ms / 1e9, ms);
    }
  };
  if (!one) {
    run(peak_kernel<2>, 2);
    run(peak_kernel<4>, 4);
    run(peak_kernel<8>, 8);
  }
  run(peak_kernel<16>, 16);
  return 0;
}
