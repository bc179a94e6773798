// Latency probe: the diagonal factor's 32-row band elimination (lanes = columns, registers =
// rows; lanes 0-31 the band's 32x32 diagonal block D, lanes 32-63 strip columns), one pivot
// per step (diag_block.hpp today: pivot row through a per-wave LDS buffer) against 4-row
// block steps (one LDS round trip per 4 pivots: the 4x4 pivot block is factored redundantly
// in every lane, each column's rows become w = U4^-T a, and the rest of the column takes
// x_i -= a_i . v with v = U4^-1 w -- the same rank-4 Schur update, 4 FMAs per row).
// One wave per block; s_memtime around the elimination.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/elim4_probe tools/probe/elim4_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef double d2v __attribute__((ext_vector_type(2)));
typedef double d4v __attribute__((ext_vector_type(4)));

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

// today's loop (diag_block.hpp F1, LDS pivot-row variant)
__device__ __forceinline__ int elim1(double (&x)[32], double* pivb, int lane) {
  const bool dl = lane < 32;
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const double piv = readlane_d(x[j], j);
    bad = (bad == 0 && !(piv > 0.0)) ? j + 1 : bad;
    const double ri = rsqrt_nr(piv);
    const double u = piv * ri;
    const double xs = x[j] * ri;
    x[j] = dl ? (lane == j ? u : (lane < j ? x[j] : xs)) : xs;
    if (j < 31) {
      pivb[lane] = x[j];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int g0 = (j + 1) & ~1; g0 < 32; g0 += 16) {
        d2v r2[8];
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (g0 + 2 * t < 32) r2[t] = *reinterpret_cast<const d2v*>(pivb + g0 + 2 * t);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int i0 = g0 + 2 * t;
          if (i0 < 32) {
            if (i0 > j) x[i0] = fma(-r2[t][0], x[j], x[i0]);
            x[i0 + 1] = fma(-r2[t][1], x[j], x[i0 + 1]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("" ::: "memory");
    }
  }
  return bad;
}

// 4-row block steps.  pivb: 64 lanes x 4 doubles (32 B per lane).  The later columns'
// 4-vectors are read in groups of G (each group's reads issued together, then its FMAs)
template <int SB, int G>
__device__ __forceinline__ int elim4(double (&x)[32], double* pivb, int lane) {
  const bool dl = lane < 32;
  int bad = 0;
  d2v* pb = reinterpret_cast<d2v*>(pivb);
#pragma unroll
  for (int j0 = 0; j0 < 32; j0 += 4) {
    // this lane's raw 4-vector of the pivot rows
    const double a0 = x[j0], a1 = x[j0 + 1], a2 = x[j0 + 2], a3 = x[j0 + 3];
    pb[2 * lane] = d2v{a0, a1};
    pb[2 * lane + 1] = d2v{a2, a3};
    asm volatile("" ::: "memory");
    // the pivot block (columns j0..j0+3): its upper 10 entries
    d2v pv[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      pv[t][0] = pb[2 * (j0 + t)];
      if (t >= 2) pv[t][1] = pb[2 * (j0 + t) + 1];
    }
    // the first group's reads before the factorisation's chain
    constexpr int GMAX = 8;
    d2v g[GMAX][2];
#pragma unroll
    for (int q = 0; q < G; ++q)
      if (j0 + 4 + q < 32) {
        g[q][0] = pb[2 * (j0 + 4 + q)];
        g[q][1] = pb[2 * (j0 + 4 + q) + 1];
      }
    if (SB) __builtin_amdgcn_sched_barrier(0);
    const double a00 = pv[0][0][0], a01 = pv[1][0][0], a02 = pv[2][0][0], a03 = pv[3][0][0];
    const double a11 = pv[1][0][1], a12 = pv[2][0][1], a13 = pv[3][0][1];
    const double a22 = pv[2][1][0], a23 = pv[3][1][0], a33 = pv[3][1][1];
    bad = (bad == 0 && !(a00 > 0.0)) ? j0 + 1 : bad;
    const double r0 = rsqrt_nr(a00);
    const double u00 = a00 * r0, u01 = a01 * r0, u02 = a02 * r0, u03 = a03 * r0;
    const double p1 = fma(-u01, u01, a11);
    bad = (bad == 0 && !(p1 > 0.0)) ? j0 + 2 : bad;
    const double r1 = rsqrt_nr(p1);
    const double u11 = p1 * r1, u12 = fma(-u01, u02, a12) * r1, u13 = fma(-u01, u03, a13) * r1;
    const double p2 = fma(-u12, u12, fma(-u02, u02, a22));
    bad = (bad == 0 && !(p2 > 0.0)) ? j0 + 3 : bad;
    const double r2 = rsqrt_nr(p2);
    const double u22 = p2 * r2, u23 = fma(-u12, u13, fma(-u02, u03, a23)) * r2;
    const double p3 = fma(-u23, u23, fma(-u13, u13, fma(-u03, u03, a33)));
    bad = (bad == 0 && !(p3 > 0.0)) ? j0 + 4 : bad;
    const double r3 = rsqrt_nr(p3);
    const double u33 = p3 * r3;
    // w = U4^-T a (this column's rows j0..j0+3 of U), v = U4^-1 w
    const double w0 = a0 * r0;
    const double w1 = fma(-u01, w0, a1) * r1;
    const double w2 = fma(-u12, w1, fma(-u02, w0, a2)) * r2;
    const double w3 = fma(-u23, w2, fma(-u13, w1, fma(-u03, w0, a3))) * r3;
    const double v3 = w3 * r3;
    const double v2 = fma(-u23, v3, w2) * r2;
    const double v1 = fma(-u13, v3, fma(-u12, v2, w1)) * r1;
    const double v0 = fma(-u03, v3, fma(-u02, v2, fma(-u01, v1, w0))) * r0;
    // lanes of D left of / inside the pivot block: no update; inside, rows j0.. from U4
    const int cl = lane - j0;
    const bool left = dl && cl < 0, inblk = dl && cl >= 0 && cl < 4;
    const bool upd = !(left || inblk);
    const double z0 = upd ? v0 : 0.0, z1 = upd ? v1 : 0.0, z2 = upd ? v2 : 0.0, z3 = upd ? v3 : 0.0;
    const double b0 = cl == 0 ? u00 : cl == 1 ? u01 : cl == 2 ? u02 : u03;
    const double b1 = cl == 1 ? u11 : cl == 2 ? u12 : cl == 3 ? u13 : 0.0;
    const double b2 = cl == 2 ? u22 : cl == 3 ? u23 : 0.0;
    const double b3 = cl == 3 ? u33 : 0.0;
    x[j0] = left ? x[j0] : inblk ? b0 : w0;
    x[j0 + 1] = left ? x[j0 + 1] : inblk ? b1 : w1;
    x[j0 + 2] = left ? x[j0 + 2] : inblk ? b2 : w2;
    x[j0 + 3] = left ? x[j0 + 3] : inblk ? b3 : w3;
#pragma unroll
    for (int i0 = j0 + 4; i0 < 32; i0 += G) {
      if (i0 > j0 + 4) {
#pragma unroll
        for (int q = 0; q < G; ++q)
          if (i0 + q < 32) {
            g[q][0] = pb[2 * (i0 + q)];
            g[q][1] = pb[2 * (i0 + q) + 1];
          }
        if (SB) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < G; ++q)
        if (i0 + q < 32) {
          double t = fma(-g[q][0][0], z0, x[i0 + q]);
          t = fma(-g[q][0][1], z1, t);
          t = fma(-g[q][1][0], z2, t);
          x[i0 + q] = fma(-g[q][1][1], z3, t);
          // (pins the update here: without it the FMAs sink to the next use of x, keeping
          // every group's operands live across the step -- spills)
          asm volatile("" : "+v"(x[i0 + q]));
        }
      if (SB) __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" ::: "memory");
  }
  return bad;
}

template <int V>
__global__ __launch_bounds__(64) void elim(const double* in, double* out, long long* cyc) {
  __shared__ double pivb[64 * 4];
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
  int bad;
  if constexpr (V == 0) bad = elim1(x, pivb, lane);
  else if constexpr (V == 1) bad = elim4<0, 4>(x, pivb, lane);
  else if constexpr (V == 2) bad = elim4<1, 4>(x, pivb, lane);
  else if constexpr (V == 3) bad = elim4<0, 8>(x, pivb, lane);
  else bad = elim4<1, 8>(x, pivb, lane);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < 32; ++r) asm volatile("" ::"v"(x[r]));
  long long t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
#pragma unroll
  for (int r = 0; r < 32; ++r) out[r * 64 + lane] = x[r];
  if (lane == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = bad;
  }
}

int main() {
  static double h[32 * 64];
  // band [D | S]: D = R^T R + 32 I restricted to its upper triangle (zeros below), S random
  srand(7);
  double R[32][32];
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) R[i][j] = (rand() / (double)RAND_MAX) - 0.5;
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 64; ++c) {
      double v;
      if (c < 32) {
        double s = (r == c) ? 4.0 : 0.0;
        for (int k = 0; k < 32; ++k) s += R[k][r] * R[k][c];
        v = r <= c ? s : 0.0;
      } else {
        v = (rand() / (double)RAND_MAX) - 0.5;
      }
      h[r * 64 + c] = v;
    }
  double *din, *dout;
  long long* dc;
  hipMalloc(&din, sizeof h);
  hipMalloc(&dout, sizeof h);
  hipMalloc(&dc, 16);
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  static double res[5][32 * 64];
  auto run = [&](auto kern, const char* name, int v) {
    long long best = 1LL << 60;
    long long c[2];
    for (int it = 0; it < 20; ++it) {
      kern<<<1, 64>>>(din, dout, dc);
      hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
      if (c[0] < best) best = c[0];
    }
    hipMemcpy(res[v], dout, sizeof h, hipMemcpyDeviceToHost);
    printf("%-34s %6lld cycles  (%.1f cycles / pivot)  bad=%lld\n", name, best, best / 32.0, c[1]);
  };
  run(elim<0>, "one pivot per step (diag_block)", 0);
  run(elim<1>, "4-row blocks, groups of 4", 1);
  run(elim<2>, "4-row blocks, groups of 4, sched", 2);
  run(elim<3>, "4-row blocks, groups of 8", 3);
  run(elim<4>, "4-row blocks, groups of 8, sched", 4);
  for (int v = 1; v <= 4; ++v) {
    double md = 0, mx = 0;
    for (int i = 0; i < 32 * 64; ++i) {
      md = fmax(md, fabs(res[0][i] - res[v][i]));
      mx = fmax(mx, fabs(res[0][i]));
    }
    printf("variant %d max |diff| vs one-pivot: %.3e (max |x| %.3e)\n", v, md, mx);
  }
  return 0;
}
