// Latency probe of the 32-pivot band elimination used by diag2_kernel (lanes = columns,
// registers = rows).  One wave; s_memtime around the elimination; variants:
//   0: readlane broadcasts in groups of 8 (diag2_kernel)
//   1: only the critical chain (pivot, rsqrt, scale, update of row j+1)
//   2: variant 0 with the pivot taken by ds_bpermute-free v_readfirstlane after a row move
//   3: rsqrt chain only (no updates at all)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/elim_probe tools/probe/elim_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x * y;
  const double r = fma(-h, y, 0.5);
  return fma(y, r, y);
}

template <int V>
__global__ void elim(const double* in, double* out, long long* cyc) {
  const int lane = threadIdx.x;
  double x[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) x[r] = in[r * 64 + lane];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) asm volatile("" ::"v"(x[r]));
  long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  __builtin_amdgcn_sched_barrier(0);
  const bool dl = lane < 32;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const double piv = readlane_d(x[j], j);
    const double ri = rsqrt_nr(piv);
    const double u = piv * ri;
    const double xs = x[j] * ri;
    if constexpr (V == 3) {
      x[j] = xs;
      if (j + 1 < 32) x[j + 1] = x[j + 1] + 1e-300 * xs;
      continue;
    }
    x[j] = dl ? (lane == j ? u : (lane < j ? x[j] : xs)) : xs;
    if constexpr (V == 6) {  // the update FMAs alone, multiplier from an SGPR constant
      const double uc = in[j];
#pragma unroll
      for (int i = j + 1; i < 32; ++i) x[i] = fma(-uc, x[j], x[i]);
      continue;
    }
    if constexpr (V == 7) {  // the readlanes alone (summed into one register)
      double acc = 0.0;
#pragma unroll
      for (int i = j + 1; i < 32; ++i) acc += readlane_d(x[i & 31], i);
      x[j] = acc;
      continue;
    }
    if constexpr (V == 4 || V == 5) {
      __shared__ double rowb[64];
      typedef double d2l __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_sched_barrier(0);
      rowb[lane] = x[j];
      int i1 = j + 1;
      if (V == 4 && j + 1 < 32) {  // critical element by readlane
        x[j + 1] = fma(-readlane_d(x[j], j + 1), x[j], x[j + 1]);
        i1 = j + 2;
      }
      if (i1 & 1) {
        if (i1 < 32) x[i1] = fma(-rowb[i1], x[j], x[i1]);
        ++i1;
      }
#pragma unroll
      for (int g0 = 0; g0 < 32; g0 += 8) {
        if (g0 + 8 <= i1) continue;
        d2l ub[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (g0 + 2 * t >= i1) ub[t] = *reinterpret_cast<const d2l*>(&rowb[g0 + 2 * t]);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (g0 + 2 * t >= i1) {
            x[g0 + 2 * t] = fma(-ub[t][0], x[j], x[g0 + 2 * t]);
            x[g0 + 2 * t + 1] = fma(-ub[t][1], x[j], x[g0 + 2 * t + 1]);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (V == 1) {
      if (j + 1 < 32) x[j + 1] = fma(-readlane_d(x[j], j + 1), x[j], x[j + 1]);
    } else {
#pragma unroll
      for (int i0 = j + 1; i0 < 32; i0 += 8) {
        double u8[8];
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (i0 + t < 32) u8[t] = readlane_d(x[j], i0 + t);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (i0 + t < 32) x[i0 + t] = fma(-u8[t], x[j], x[i0 + t]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < 32; ++r) asm volatile("" ::"v"(x[r]));
  long long t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
#pragma unroll
  for (int r = 0; r < 32; ++r) out[r * 64 + lane] = x[r];
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  double h[32 * 64];
  // SPD-ish band: column c (lane) rows r; diagonal block = I*40 + small, strip random
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 64; ++c) {
      double v = 0.01 * ((r * 7 + c * 13) % 17);
      if (c < 32) v = (r == c) ? 40.0 : (r < c ? 0.3 : 0.0);
      h[r * 64 + c] = v;
    }
  double *din, *dout;
  long long* dc;
  hipMalloc(&din, sizeof h);
  hipMalloc(&dout, sizeof h);
  hipMalloc(&dc, 8);
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  auto run = [&](auto kern, const char* name) {
    long long best = 1LL << 60;
    for (int it = 0; it < 20; ++it) {
      kern<<<1, 64>>>(din, dout, dc);
      long long c;
      hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    // s_memtime counts shader-clock cycles
    printf("%-28s %6lld cycles  (%.1f cycles / pivot)\n", name, best, best / 32.0);
  };
  run(elim<0>, "readlane groups (diag2)");
  run(elim<1>, "critical chain only");
  run(elim<3>, "rsqrt chain only");
  run(elim<4>, "hybrid readlane+LDS");
  run(elim<5>, "LDS broadcast");
  run(elim<6>, "FMAs only (SGPR mult)");
  run(elim<7>, "readlanes only");
  // correctness of 4/5 against 0
  double r0[32 * 64], r4[32 * 64];
  elim<0><<<1, 64>>>(din, dout, dc);
  hipMemcpy(r0, dout, sizeof r0, hipMemcpyDeviceToHost);
  for (int v = 4; v <= 5; ++v) {
    if (v == 4) elim<4><<<1, 64>>>(din, dout, dc); else elim<5><<<1, 64>>>(din, dout, dc);
    hipMemcpy(r4, dout, sizeof r4, hipMemcpyDeviceToHost);
    double md = 0;
    for (int i = 0; i < 32 * 64; ++i) md = fmax(md, fabs(r0[i] - r4[i]));
    printf("variant %d max |diff| vs 0: %.3e\n", v, md);
  }
  return 0;
}
