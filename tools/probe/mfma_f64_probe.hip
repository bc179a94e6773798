// Probe: v_mfma_f64_16x16x4_f64 fragment layout + issue rate on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));

// D = A(16x4) * B(4x16); lane l supplies A[l&15][l>>4], B[l>>4][l&15]
__global__ void layout_kernel(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A row-major 16x4
  double b = B[(l >> 4) * 16 + (l & 15)];  // B row-major 4x16
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];  // raw dump: lane, reg
}

template <int NACC>
__global__ void rate_kernel(double* out, int iters) {
  int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma_rate_kernel(double* out, int iters) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  double m = 0.999999, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = (i == 4 * k + 1) ? 1.0 : 0.0; // picks rows
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = 100 * k + j;  // asymmetric
  // Reference C = A*B (16x16)
  double *dA, *dB, *dD;
  hipMalloc(&dA, 64 * 8); hipMalloc(&dB, 64 * 8); hipMalloc(&dD, 256 * 8);
  hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
  // test hypothesis: row=(l>>4)+4r, col=l&15
  int bad1 = 0, bad2 = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int col = l & 15;
    int row1 = (l >> 4) + 4 * r, row2 = 4 * (l >> 4) + r;
    auto ref = [&](int row) { double s = 0; for (int k = 0; k < 4; ++k) s += A[row * 4 + k] * B[k * 16 + col]; return s; };
    if (D[l * 4 + r] != ref(row1)) bad1++;
    if (D[l * 4 + r] != ref(row2)) bad2++;
  }
  printf("layout: hyp row=(l>>4)+4r bad=%d ; hyp row=4(l>>4)+r bad=%d\n", bad1, bad2);
  double* dout; hipMalloc(&dout, 256 * 8 * 1024 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 20000;
  for (int wpb : {1, 4, 8}) {
    int blocks = 256 * 2;
    rate_kernel<4><<<blocks, 64 * wpb>>>(dout, 100);
    hipEventRecord(e0);
    rate_kernel<4><<<blocks, 64 * wpb>>>(dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * blocks * wpb;
    printf("mfma_f64 NACC=4 waves/blk=%d blocks=%d: %.3f ms  %.2f TFLOP/s\n", wpb, blocks, ms, flops / ms / 1e9);
  }
  {
    int blocks = 256 * 4;
    rate_kernel<1><<<blocks, 256>>>(dout, 100);
    hipEventRecord(e0);
    rate_kernel<1><<<blocks, 256>>>(dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 16 * 16 * 4 * 1.0 * iters * blocks * 4;
    printf("mfma_f64 NACC=1 (dep chain) 4 waves/blk: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  {
    int blocks = 256 * 8;
    fma_rate_kernel<<<blocks, 256>>>(dout, 100);
    hipEventRecord(e0);
    fma_rate_kernel<<<blocks, 256>>>(dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 8 * iters * blocks * 256.0;
    printf("v_fma_f64 vector: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  // HBM write bandwidth probe: 4 GiB write
  size_t n = (size_t)1 << 29; double* big; hipMalloc(&big, n * 8);
  hipMemsetD32((hipDeviceptr_t)big, 0, n * 2);
  hipEventRecord(e0); hipMemsetD32((hipDeviceptr_t)big, 1, n * 2); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("memset 4GiB: %.3f ms  %.2f TB/s\n", ms, n * 8.0 / ms / 1e9);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz mem=%zu\n", p.gcnArchName, p.multiProcessorCount, p.clockRate, p.totalGlobalMem);
  return 0;
}
