// Does an FP64 MFMA (v_mfma_f64_16x16x4f64, 64 cycles) leave the SIMD's FP64 VALU free?
// One wave per SIMD (4 per CU, every CU), a loop of [1 MFMA + F independent v_fma_f64]:
// cycles per iteration (s_memtime) = max(64, F x c_fma) if the two pipes overlap, 64 + F x
// c_fma if the MFMA holds the FP64 VALU.  F = 0 gives the MFMA alone, and MFMA-free runs give
// c_fma.  Answers how the K assembly's Gram-form distance (MFMA) and its exponentials
// (FP64 VALU) can share a SIMD.   Usage: mfma_valu_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int F, bool MF>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double seed) {
  d4 acc0 = {seed, 0, 0, 0}, acc1 = {0, seed, 0, 0};
  double v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed * (i + 1);
  const double a = seed * 0.5, b = seed * 0.25;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MF) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int f = 0; f < F; ++f) v[f % 16] = fma(v[f % 16], 0.999, 1e-3);
    __builtin_amdgcn_sched_barrier(0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = acc0[0] + acc0[1] + acc1[2] + acc1[3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += v[i];
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = (double)(t1 - t0) / iters;
    out[2 * blockIdx.x + 1] = s;
  }
}

template <int F, bool MF>
void run(double* d, double* h, int blocks, int iters) {
  probe<F, MF><<<blocks, 256>>>(d, iters, 1.0);
  probe<F, MF><<<blocks, 256>>>(d, iters, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h, d, sizeof(double) * 2 * blocks, hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; ++b) s += h[2 * b];
  printf("%s + %2d v_fma_f64 per iteration: %7.1f cycles / iteration (one wave per SIMD, %d CUs)\n",
         MF ? "2 MFMA f64 16x16x4" : "no MFMA           ", F, s / blocks, blocks);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount, iters = 20000;
  double *d, h[2 * 1024];
  (void)hipMalloc(&d, sizeof(double) * 2 * 1024);
  run<0, true>(d, h, blocks, iters);
  run<8, true>(d, h, blocks, iters);
  run<16, true>(d, h, blocks, iters);
  run<32, true>(d, h, blocks, iters);
  run<48, true>(d, h, blocks, iters);
  run<16, false>(d, h, blocks, iters);
  run<32, false>(d, h, blocks, iters);
  run<48, false>(d, h, blocks, iters);
  return 0;
}
