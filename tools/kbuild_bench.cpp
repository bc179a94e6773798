// K-assembly timing through the C ABI: symmetric N x N (SE, SE+WN, SE+SE+WN) and cross
// N x M, d = 8.  Build: make -C gaussianprocessregression.jl_amd/csrc kbench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/gpr_hip.h"

// write-bandwidth ceiling references: plain 16-B/lane streaming stores
__global__ void store16_kernel(double* p, size_t n2) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    reinterpret_cast<d2*>(p)[i] = d2{1.0, 2.0};
}

__global__ void store16nt_kernel(double* p, size_t n2) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(d2{1.0, 2.0}, reinterpret_cast<d2*>(p) + i);
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 32768;
  const int d = argc > 2 ? atoi(argv[2]) : 8;
  const int M = argc > 3 ? atoi(argv[3]) : 8192;
  gpr_ctx_t ctx;
  if (gpr_ctx_create(0, nullptr, &ctx)) return 1;
  std::vector<double> hx((size_t)d * N), hxp((size_t)d * M);
  srand(1);
  for (auto& v : hx) v = rand() / (double)RAND_MAX;
  for (auto& v : hxp) v = rand() / (double)RAND_MAX;
  double *dx, *dxp, *K;
  hipMalloc(&dx, sizeof(double) * hx.size());
  hipMalloc(&dxp, sizeof(double) * hxp.size());
  hipMalloc(&K, sizeof(double) * (size_t)N * N);
  hipMemcpy(dx, hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice);
  hipMemcpy(dxp, hxp.data(), sizeof(double) * hxp.size(), hipMemcpyHostToDevice);
  const double l = 3.0 * std::sqrt(8.0 / d);
  hipStream_t s = (hipStream_t)gpr_ctx_stream(ctx);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  {
    const size_t bytes = sizeof(double) * (size_t)N * N;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0, s);
      hipMemsetAsync(K, 0, bytes, s);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep == 3) printf("hipMemsetAsync %.2f GB: %.3f ms  %.0f GB/s\n", bytes / 1e9, ms, bytes / ms / 1e6);
    }
    for (int g : {1024, 2048, 4096, 16384}) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0, s);
        store16_kernel<<<g, 256, 0, s>>>(K, bytes / 16);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (rep) best = ms < best ? ms : best;
      }
      printf("store16 grid %d: %.3f ms  %.0f GB/s\n", g, best, bytes / best / 1e6);
      best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0, s);
        store16nt_kernel<<<g, 256, 0, s>>>(K, bytes / 16);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (rep) best = ms < best ? ms : best;
      }
      printf("store16 nt grid %d: %.3f ms  %.0f GB/s\n", g, best, bytes / best / 1e6);
    }
  }
  struct Cfg { const char* name; std::vector<int> kinds; };
  std::vector<Cfg> cfgs = {{"SE", {GPR_SE}}, {"SE+WN", {GPR_SE, GPR_WN}}, {"SE+SE+WN", {GPR_SE, GPR_SE, GPR_WN}}};
  for (auto& c : cfgs) {
    std::vector<double> hp;
    for (int k : c.kinds) {
      if (k == GPR_SE) { hp.push_back(1.0); for (int t = 0; t < d; ++t) hp.push_back(l); }
      else hp.push_back(0.1);
    }
    for (int cross = 0; cross < 2; ++cross) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0, s);
        int rc = cross ? gpr_kernel(ctx, c.kinds.data(), (int)c.kinds.size(), hp.data(), d, dx, N, dxp, M, 0, 1e-8, K, N)
                       : gpr_kernel(ctx, c.kinds.data(), (int)c.kinds.size(), hp.data(), d, dx, N, nullptr, N, 1, 1e-8, K, N);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        if (rc) { printf("rc=%d %s\n", rc, gpr_last_error(ctx)); return 1; }
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (rep) best = ms < best ? ms : best;
      }
      const double bytes = 8.0 * N * (double)(cross ? M : N);
      printf("kbuild %-9s %s N=%d M=%d d=%d: %.3f ms  %.0f GB/s (%.1f%% of 8 TB/s)\n", c.name,
             cross ? "cross" : "sym  ", N, cross ? M : N, d, best, bytes / best / 1e6,
             bytes / best / 1e6 / 80.0);
    }
  }
  gpr_ctx_destroy(ctx);
  return 0;
}
