// Standalone timing of launch_gemm_tn (SYRK / TRSM-update shapes) and potrf.
// Build: make -C gaussianprocessregression.jl_amd/csrc bench   (links the library objects)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#include "../gaussianprocessregression.jl_amd/csrc/common.hpp"

__global__ void init_kernel(double* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)(i * 2654435761u) ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
    p[i] = (h & 0xffffff) / 16777216.0 - 0.5;
  }
}

__device__ double init_val(size_t i, unsigned seed) {
  unsigned h = (unsigned)(i * 2654435761u) ^ seed;
  h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
  return (h & 0xffffff) / 16777216.0 - 0.5;
}

// max |C - (C0 - P^T P)| over a strided sample of (m, n) (upper: m <= n only, the rest
// must still hold C0); err as the bit pattern of a non-negative double
__global__ void verify_kernel(const double* P, const double* C, int N, int K, int upper, int stride,
                              unsigned long long* err) {
  const int ns = (N + stride - 1) / stride;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)ns * ns;
       t += (size_t)gridDim.x * blockDim.x) {
    // offsets cycle through every residue mod stride, so all tile positions are hit
    const int m = min(N - 1, (int)(t % ns) * stride + (int)(t / ns) % stride);
    const int n = min(N - 1, (int)(t / ns) * stride + (int)(t % ns) % stride);
    const size_t i = (size_t)m + (size_t)n * N;
    double ref = init_val(i, 2);
    if (!upper || m <= n) {
      double acc = 0.0;
      for (int k = 0; k < K; ++k) acc += P[k + (size_t)m * K] * P[k + (size_t)n * K];
      ref -= acc;
    }
    const double e = fabs(C[i] - ref);
    atomicMax(err, (unsigned long long)__double_as_longlong(e != e ? 1e300 : e));
  }
}

extern "C" void gpr_debug_diag_stamps(unsigned long long* out);
extern "C" int gpr_debug_chain_kernels(gpr_ctx_t ctx, double* A, int lda, int n, int variant,
                                       int reps, float* ms);

int main(int argc, char** argv) {
  int N = argc > 1 ? atoi(argv[1]) : 16384;
  int K = argc > 2 ? atoi(argv[2]) : 128;
  int mode = argc > 3 ? atoi(argv[3]) : 0;  // 0 syrk upper, 1 general (M=N=N, K), 2 potrf
  gpr_ctx_t ctx;
  gpr_ctx_create(0, nullptr, &ctx);
  hipStream_t s = (hipStream_t)gpr_ctx_stream(ctx);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  if (mode == 2) {
    // SPD matrix: K = kernel(SE+WN) of random points via the public API
    int d = 8;
    double *X, *A;
    hipMalloc(&X, sizeof(double) * d * N);
    hipMalloc(&A, sizeof(double) * (size_t)N * N);
    init_kernel<<<1024, 256, 0, s>>>(X, (size_t)d * N, 7);
    int kinds[3] = {GPR_SE, GPR_SE, GPR_WN};
    std::vector<double> hp(2 * (d + 1) + 1, 3.0);
    hp[0] = 1.0; hp[d + 1] = 1.0; hp[2 * (d + 1)] = 0.1;
    for (int rep = 0; rep < 3; ++rep) {
      gpr_kernel(ctx, kinds, 3, hp.data(), d, X, N, nullptr, N, 1, 1e-8, A, N);
      gpr_timing_reset(ctx);
      gpr_timing_enable(ctx, rep == 2);
      hipEventRecord(e0, s);
      int info = 0;
      gpr_potrf_upper(ctx, A, N, N, &info);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("potrf N=%d: %.2f ms  %.2f TFLOP/s info=%d\n", N, ms, (double)N * N * N / 3 / ms / 1e9, info);
    }
    {
      unsigned long long st[16];
      gpr_debug_diag_stamps(st);
      printf("in-kernel diag time: %.2f us avg over %llu calls (all reps)\n", st[8] / 100.0 / (st[9] ? st[9] : 1), st[9]);
      printf("sb0: A1 %.2f A2 %.2f A3 %.2f us\n", (st[5] - st[1]) / 100.0, (st[6] - st[5]) / 100.0, (st[7] - st[6]) / 100.0);
      printf("last diag stamps (us from start, 100 MHz clock): load %.2f factor %.2f copy %.2f inverse %.2f\n",
             (st[1] - st[0]) / 100.0, (st[2] - st[1]) / 100.0, (st[3] - st[2]) / 100.0, (st[4] - st[3]) / 100.0);
    }
    const char* nm[5] = {"kbuild", "syrk", "panel", "trsm", "other"};
    for (int c = 0; c < 5; ++c) {
      double ms, fl; long long ln;
      gpr_timing_get(ctx, c, &ms, &ln, &fl);
      if (ln) printf("  %-6s %8.2f ms %5lld launches %7.2f TF\n", nm[c], ms, ln, fl / ms / 1e9);
    }
    return 0;
  }
  if (mode == 4) {
    // posterior TRSM in context: K (SE+SE+WN) -> potrf -> Kpx (N x K cross) -> U^-T Kpx
    const int d = 8, np = K;
    double *X, *A, *B;
    hipMalloc(&X, sizeof(double) * d * (N + np));
    hipMalloc(&A, sizeof(double) * (size_t)N * N);
    hipMalloc(&B, sizeof(double) * (size_t)N * np);
    init_kernel<<<1024, 256, 0, s>>>(X, (size_t)d * (N + np), 7);
    int kinds[3] = {GPR_SE, GPR_SE, GPR_WN};
    std::vector<double> hp(2 * (d + 1) + 1, 3.0);
    hp[0] = 1.0; hp[d + 1] = 1.0; hp[2 * (d + 1)] = 0.1;
    gpr_kernel(ctx, kinds, 3, hp.data(), d, X, N, nullptr, N, 1, 1e-8, A, N);
    int info = 0;
    gpr_potrf_upper(ctx, A, N, N, &info);
    printf("potrf info=%d\n", info);
    for (int rep = 0; rep < 3; ++rep) {
      gpr_kernel(ctx, kinds, 3, hp.data(), d, X, N, X + (size_t)d * N, np, 0, 1e-8, B, N);
      gpr_timing_reset(ctx);
      gpr_timing_enable(ctx, 1);
      hipEventRecord(e0, s);
      trsm_ut_core(ctx, A, N, N, B, np, N, nullptr, 0);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("trsm N=%d nrhs=%d: %.2f ms  %.2f TFLOP/s\n", N, np, ms, (double)N * N * np / ms / 1e9);
      const char* nm[6] = {"kbuild", "syrk", "panel", "trsm", "other", "gemm_pipe"};
      for (int c = 0; c < 6; ++c) {
        double tms, fl; long long ln;
        gpr_timing_get(ctx, c, &tms, &ln, &fl);
        if (ln) printf("  %-9s %8.2f ms %5lld launches %7.2f TF\n", nm[c], tms, ln, fl / tms / 1e9);
      }
    }
    return 0;
  }
  if (mode == 6) {
    // chain kernels on the diagonal blocks of an SE+WN matrix (gpr_debug_chain_kernels)
    int d = 8;
    double *X, *A;
    hipMalloc(&X, sizeof(double) * d * N);
    hipMalloc(&A, sizeof(double) * (size_t)N * N);
    init_kernel<<<1024, 256, 0, s>>>(X, (size_t)d * N, 7);
    int kinds[2] = {GPR_SE, GPR_WN};
    std::vector<double> hp(d + 2, 3.0);
    hp[0] = 1.0; hp[d + 1] = 0.1;
    const char* nm[2] = {"diag (U + W)", "row TRSM W^T GEMM"};
    gpr_kernel(ctx, kinds, 2, hp.data(), d, X, N, nullptr, N, 1, 1e-8, A, N);
    for (int v = 0; v < 2; ++v) {
      float ms = 0;
      const int info = gpr_debug_chain_kernels(ctx, A, N, N, v, 60, &ms);
      printf("N=%d %-24s %8.2f us per launch (info %d)\n", N, nm[v], ms * 1e3, info);
    }
    return 0;
  }
  if (mode == 5) {
    // the factorisation's trailing SYRK in place: C = A(r:, r:) -= A(k:k+K, r:)^T A(k:k+K, r:)
    // inside an N x N matrix (ld N), trailing width W (argv[4]), vs mode 0's dense operands
    const int W = argc > 4 ? atoi(argv[4]) : N / 2;
    double* A5;
    hipMalloc(&A5, sizeof(double) * (size_t)N * N);
    init_kernel<<<1024, 256, 0, s>>>(A5, (size_t)N * N, 5);
    const int r = N - W, k = r - K;
    GemmArgs g{};
    g.P = A5 + k + (size_t)r * N; g.ldp = N;
    g.Q = g.P; g.ldq = N;
    g.C = A5 + r + (size_t)r * N; g.ldc = N;
    g.M = W; g.N = W; g.K = K; g.alpha = -1.0; g.beta = 1.0; g.upper = 1;
    const double flops = (double)W * (W + 1) * K;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0, s);
      launch_gemm_tn(ctx, g, TC_OTHER);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 2) printf("in-place syrk N=%d W=%d K=%d: %.3f ms  %.2f TFLOP/s\n", N, W, K, ms, flops / ms / 1e9);
    }
    return 0;
  }
  if (mode == 3) {
    // general C (M x N, ldc) -= P^T Q with P K x M (ldp), Q K x N (ld K): TRSM-update shapes
    const int M = argc > 4 ? atoi(argv[4]) : N;
    const int ldp = argc > 5 ? atoi(argv[5]) : K;
    const int ldc = argc > 6 ? atoi(argv[6]) : M;
    double *P3, *Q3, *C3;
    hipMalloc(&P3, sizeof(double) * (size_t)ldp * M);
    hipMalloc(&Q3, sizeof(double) * (size_t)K * N);
    hipMalloc(&C3, sizeof(double) * (size_t)ldc * N);
    init_kernel<<<1024, 256, 0, s>>>(P3, (size_t)ldp * M, 1);
    init_kernel<<<1024, 256, 0, s>>>(Q3, (size_t)K * N, 3);
    init_kernel<<<1024, 256, 0, s>>>(C3, (size_t)ldc * N, 2);
    if (getenv("GEMM_KDATA")) {
      // kernel-matrix data (smooth, wide exponent range) instead of uniform random
      const int d = 8, npt = std::max(std::max(ldp, ldc), std::max(M, N));
      double* X;
      hipMalloc(&X, sizeof(double) * d * npt);
      init_kernel<<<1024, 256, 0, s>>>(X, (size_t)d * npt, 7);
      int kinds[2] = {GPR_SE, GPR_WN};
      std::vector<double> hp(d + 2, 3.0);
      hp[0] = 1.0; hp[d + 1] = 0.1;
      gpr_kernel(ctx, kinds, 2, hp.data(), d, X, ldp, X, M, 0, 1e-8, P3, ldp);
      gpr_kernel(ctx, kinds, 2, hp.data(), d, X, ldc, X, N, 0, 1e-8, C3, ldc);
      gpr_kernel(ctx, kinds, 2, hp.data(), d, X, K, X, N, 0, 1e-8, Q3, K);
      hipStreamSynchronize(s);
    }
    GemmArgs g{};
    g.P = P3; g.ldp = ldp; g.Q = Q3; g.ldq = K; g.C = C3; g.ldc = ldc;
    g.M = M; g.N = N; g.K = K; g.alpha = -1.0; g.beta = 1.0;
    const double flops = 2.0 * M * (double)N * K;
    const int reps = getenv("GEMM_REPS") ? atoi(getenv("GEMM_REPS")) : 5;
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto& e : ev) hipEventCreate(&e);
    // back to back (sustained clock), one event between launches
    hipEventRecord(ev[0], s);
    for (int rep = 0; rep < reps; ++rep) {
      launch_gemm_tn(ctx, g, TC_OTHER);
      hipEventRecord(ev[rep + 1], s);
    }
    hipEventSynchronize(ev[reps]);
    for (int rep = 0; rep < reps; ++rep) {
      float ms; hipEventElapsedTime(&ms, ev[rep], ev[rep + 1]);
      if (rep >= 2 && (rep < 6 || rep % 10 == 0 || rep == reps - 1))
        printf("gemm M=%d N=%d K=%d ldp=%d ldc=%d rep %d: %.3f ms  %.2f TFLOP/s\n", M, N, K, ldp, ldc, rep, ms, flops / ms / 1e9);
    }
    return 0;
  }
  double *P, *C;
  hipMalloc(&P, sizeof(double) * (size_t)K * N);
  hipMalloc(&C, sizeof(double) * (size_t)N * N);
  init_kernel<<<1024, 256, 0, s>>>(P, (size_t)K * N, 1);
  init_kernel<<<1024, 256, 0, s>>>(C, (size_t)N * N, 2);
  GemmArgs g{};
  g.P = P; g.ldp = K; g.Q = P; g.ldq = K; g.C = C; g.ldc = N;
  g.M = N; g.N = N; g.K = K; g.alpha = -1.0; g.beta = 1.0; g.upper = (mode == 0);
  double flops = mode == 0 ? (double)N * (N + 1) * K : 2.0 * N * N * K;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0, s);
    launch_gemm_tn(ctx, g, TC_OTHER);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (rep >= 2) printf("gemm mode=%d N=%d K=%d: %.3f ms  %.2f TFLOP/s\n", mode, N, K, ms, flops / ms / 1e9);
  }
  if (getenv("GEMM_VERIFY")) {
    init_kernel<<<1024, 256, 0, s>>>(C, (size_t)N * N, 2);
    launch_gemm_tn(ctx, g, TC_OTHER);
    unsigned long long* derr;
    hipMalloc(&derr, 8);
    hipMemsetAsync(derr, 0, 8, s);
    verify_kernel<<<2048, 256, 0, s>>>(P, C, N, K, g.upper, 7, derr);
    unsigned long long herr = 0;
    hipStreamSynchronize(s);
    hipMemcpy(&herr, derr, 8, hipMemcpyDeviceToHost);
    double e; memcpy(&e, &herr, 8);
    printf("verify mode=%d N=%d K=%d: max abs err %.3e %s\n", mode, N, K, e, e < 1e-12 * K ? "OK" : "FAIL");
  }
  return 0;
}
