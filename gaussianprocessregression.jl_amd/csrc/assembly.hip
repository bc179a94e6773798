// Kernel-matrix assembly on gfx950: SquaredExp / composed K, cross K, dK/dtheta.
//
// Reference: kernel_impl!(::SquaredExp) src/covariance.jl:85-95 (scale x by l, squared
// Euclidean distance src/covariance.jl:72-77, sigma^2 exp(-D)), the +eps jitter rule
// src/covariance.jl:49-58, the composed sum/noise src/compose_covar.jl:47-77 and the GPU
// broadcast seam src/covar_gpu.jl:1-18 this replaces.
//
// Design (HBM-write bound): the inputs are pre-scaled once per SE part (xs = x .* l, the
// reference's own rounding order) into a tiny workspace; a 64x64 output tile per 256-thread
// workgroup keeps the row point's d features in registers and reads the column point's
// features with scalar (wave-uniform) loads.  For the symmetric K only upper tiles are
// computed; each is stored directly and, transposed through LDS, as its mirror tile, so
// every N^2 element is written exactly once with 512-B coalesced column segments and the
// exp work is halved.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "common.hpp"
#include "kexp.hpp"

namespace {

constexpr int KT = 64;  // output tile edge

// 16-B stores need a 16-B aligned K and an even leading dimension (GPR_KBUILD_SCALAR forces
// the 8-B-store kernels, for A/B runs)
// persistent grid of the 16-B-store kernels: 8 workgroups per CU x 256 CUs
inline long long kbuild_grid() { return 256LL * 8; }

inline bool vec_store_ok(const double* K, int ldk) {
  return ((uintptr_t)K & 15) == 0 && (ldk & 1) == 0;
}

// xs[p][k + a*d] = x[k + a*d] * l_p[k]   (x .* ls[:, n], src/covariance.jl:90)
__global__ void scale_inputs_kernel(KParams kp, const double* __restrict__ X, int n,
                                    double* __restrict__ xs) {
  const int d = kp.d;
  const size_t total = (size_t)n * d;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total * kp.nse;
       t += (size_t)gridDim.x * blockDim.x) {
    const int p = (int)(t / total);
    const size_t r = t - p * total;
    const int k = (int)(r % d);
    xs[t] = X[r] * kp.l[p][k];
  }
}

// exp(-D) of the assembly kernels.  GPR_KBUILD_NOEXP (tools/kbuild_bench_noexp only, never
// the library) swaps in a cheap stand-in to separate exp cost from store cost.
__device__ __forceinline__ double kexp_neg(double dist) {
#ifdef GPR_KBUILD_NOEXP
  return fma(dist, -1e-3, 1.0);
#else
  return exp(-1.0 * dist);
#endif
}

// The 16-B-store kernels evaluate exp(-dist) by Tang's table method, ~1 ulp (kexp_s2 below;
// the ocml exp costs ~28 instructions with its range checks and quarter-rate conversions and
// made K-assembly VALU-bound at two SE parts).  x = -dist clamped at -800 (exp underflows to 0
// long before; a NaN dist fails the compare and propagates), n = rint(x 256/ln2),
// r = x - n ln2/256 in two Cody-Waite steps (n L1 exact: L1 has 32 significant bits,
// |n| < 2^19), |r| <= ln2/512, exp(x) = 2^(n>>8) T[n&255] (1 + expm1(r)), with
// T[j] = 2^(j/256) rounded once from extended precision on the host (ctx->dexptab).
#ifndef GPR_KBUILD_MINB  // workgroups per CU the 16-B-store assembly kernels are compiled for
#define GPR_KBUILD_MINB 4
#endif
#ifndef KB_CG  // columns per distance/exp group in kmat_tile_compute (2: 128 VGPRs,
#define KB_CG 2  // 4 waves/SIMD; 8: 178 VGPRs, 2 waves/SIMD, SE+SE+WN 2.45 -> 2.20 ms)
#endif
// D = sum_k (xr_k - xc_k)^2 with xr in registers and xc wave-uniform (scalar loads).
template <int D>
__device__ __forceinline__ double sqdist(const double* xr, const double* __restrict__ xc,
                                         int d) {
  double s = 0.0;
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const double t = xr[k] - xc[k];
      s = fma(t, t, s);
    }
  } else {
    for (int k = 0; k < d; ++k) {
      const double t = xr[k] - xc[k];
      s = fma(t, t, s);
    }
  }
  return s;
}

// Symmetric K (same-object call): upper tiles (bi <= bj) + LDS-transposed mirror.
template <int D>
__global__ __launch_bounds__(256) void kmat_sym_kernel(KParams kp, const double* __restrict__ xs,
                                                       int n, double* __restrict__ K,
                                                       size_t ldk) {
  __shared__ double tr[KT * (KT + 1)];
  const int bid = blockIdx.x;
  int bj = (int)((sqrt(8.0 * bid + 1.0) - 1.0) * 0.5);
  while ((bj + 1) * (bj + 2) / 2 <= bid) ++bj;
  while (bj * (bj + 1) / 2 > bid) --bj;
  const int bi = bid - bj * (bj + 1) / 2;
  const int i0 = bi * KT, j0 = bj * KT;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = kp.d;
  const int i = i0 + lane;
  const bool irow = i < n;

  double vals[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) vals[c] = 0.0;
  // parts outermost so only one part's row features live in registers; the per-element
  // accumulation order stays part 1, part 2, ... as in src/compose_covar.jl:52-56.
  for (int p = 0; p < kp.nse; ++p) {
    const double* xrow = xs + ((size_t)p * n + (irow ? i : 0)) * d;
    double xr[D > 0 ? D : 1];
    if constexpr (D > 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) xr[k] = xrow[k];
    }
    const double s2 = kp.sigma[p] * kp.sigma[p];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int j = j0 + wv + 4 * c;  // wave-uniform column
      if (j < n) {
        const double* xc = xs + ((size_t)p * n + j) * d;
        double dist;
        if constexpr (D > 0) {
          dist = sqdist<D>(xr, xc, d);
        } else {
          dist = sqdist<0>(xrow, xc, d);
        }
        double t = s2 * kexp_neg(dist);
        if (i == j) t += kp.eps;
        vals[c] = (p == 0) ? t : vals[c] + t;
      }
    }
  }
  if (kp.has_noise) {
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (i == j0 + wv + 4 * c) vals[c] += kp.noise2;
  }
  // direct tile: K[i + j*ldk], lanes along i -> 512-B column segments
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int j = j0 + wv + 4 * c;
    if (irow && j < n) K[(size_t)i + (size_t)j * ldk] = vals[c];
  }
  if (bi == bj) return;
  // mirror tile through LDS: tr[jl][il]
#pragma unroll
  for (int c = 0; c < 16; ++c) tr[(wv + 4 * c) * (KT + 1) + lane] = vals[c];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int il = wv + 4 * c;     // row of the original tile
    const int jj = j0 + lane;      // mirrored row index
    const int ii = i0 + il;        // mirrored column index
    if (jj < n && ii < n) K[(size_t)jj + (size_t)ii * ldk] = tr[lane * (KT + 1) + il];
  }
}

// Cross kernel K[n x m] (x !== xp): no eps, no noise.  Rows from xs (n), cols from xps (m).
template <int D>
__global__ __launch_bounds__(256) void kmat_cross_kernel(KParams kp, const double* __restrict__ xs,
                                                         int n, const double* __restrict__ xps,
                                                         int m, double* __restrict__ K,
                                                         size_t ldk, int ntile_i) {
  const int bi = blockIdx.x % ntile_i;
  const int bj = blockIdx.x / ntile_i;
  const int i0 = bi * KT, j0 = bj * KT;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = kp.d;
  const int i = i0 + lane;
  const bool irow = i < n;
  double vals[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) vals[c] = 0.0;
  for (int p = 0; p < kp.nse; ++p) {
    const double* xrow = xs + ((size_t)p * n + (irow ? i : 0)) * d;
    double xr[D > 0 ? D : 1];
    if constexpr (D > 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) xr[k] = xrow[k];
    }
    const double s2 = kp.sigma[p] * kp.sigma[p];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int j = j0 + wv + 4 * c;
      if (j < m) {
        const double* xc = xps + ((size_t)p * m + j) * d;
        double dist;
        if constexpr (D > 0) {
          dist = sqdist<D>(xr, xc, d);
        } else {
          dist = sqdist<0>(xrow, xc, d);
        }
        const double t = s2 * kexp_neg(dist);
        vals[c] = (p == 0) ? t : vals[c] + t;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int j = j0 + wv + 4 * c;
    if (irow && j < m) K[(size_t)i + (size_t)j * ldk] = vals[c];
  }
}

// dK/dtheta for one hyper-parameter (src/deriv_covar.jl:20-29): part p of the composed
// kernel, which = 0 -> (2/|sigma|) K_p (K_p incl. eps on the diagonal),
// which = k+1 -> -2 l_k K_p (x_k,a - x_k,b)^2 with RAW x.
__global__ void kgrad_kernel(KParams kp, const double* __restrict__ X,
                             const double* __restrict__ xs, int n, int p, int which,
                             double* __restrict__ DK, size_t ld) {
  const int d = kp.d;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)n * n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int a = (int)(t % n), b = (int)(t / n);
    const double* xa = xs + ((size_t)p * n + a) * d;
    const double* xb = xs + ((size_t)p * n + b) * d;
    double s = 0.0;
    for (int k = 0; k < d; ++k) {
      const double q = xa[k] - xb[k];
      s = fma(q, q, s);
    }
    double Kp = kp.sigma[p] * kp.sigma[p] * exp(-1.0 * s);
    if (a == b) Kp += kp.eps;
    double v;
    if (which == 0) {
      v = (2.0 / fabs(kp.sigma[p])) * Kp;
    } else {
      const int k = which - 1;
      const double dx = X[(size_t)a * d + k] - X[(size_t)b * d + k];
      v = -2.0 * kp.l[p][k] * Kp * (dx * dx);
    }
    DK[(size_t)a + (size_t)b * ld] = v;
  }
}

__global__ void diag_scaled_identity_kernel(double* __restrict__ A, int n, size_t lda,
                                            double lam) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)n * n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int a = (int)(t % n), b = (int)(t / n);
    A[(size_t)a + (size_t)b * lda] = (a == b) ? lam : 0.0;
  }
}

// lower <- upper^T, in 64x64 tiles through LDS (coalesced both ways)
__global__ __launch_bounds__(256) void mirror_upper_kernel(double* __restrict__ A, int n,
                                                           size_t lda) {
  __shared__ double tr[KT * (KT + 1)];
  const int bid = blockIdx.x;
  int bj = (int)((sqrt(8.0 * bid + 1.0) - 1.0) * 0.5);
  while ((bj + 1) * (bj + 2) / 2 <= bid) ++bj;
  while (bj * (bj + 1) / 2 > bid) --bj;
  const int bi = bid - bj * (bj + 1) / 2;  // bi <= bj: source tile (rows bi, cols bj)
  const int i0 = bi * KT, j0 = bj * KT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int c = 0; c < 16; ++c) {
    const int j = j0 + wv + 4 * c, i = i0 + lane;
    tr[(wv + 4 * c) * (KT + 1) + lane] = (i < n && j < n) ? A[(size_t)i + (size_t)j * lda] : 0.0;
  }
  __syncthreads();
  for (int c = 0; c < 16; ++c) {
    const int il = wv + 4 * c;
    const int jj = j0 + lane, ii = i0 + il;  // destination (jj, ii), jj >= ii region
    if (jj < n && ii < n && jj > ii) A[(size_t)jj + (size_t)ii * lda] = tr[lane * (KT + 1) + il];
  }
}

__global__ void set_identity_kernel(double* __restrict__ A, int n, size_t lda) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)n * n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int a = (int)(t % n), b = (int)(t / n);
    A[(size_t)a + (size_t)b * lda] = (a == b) ? 1.0 : 0.0;
  }
}

int scale_inputs(gpr_ctx* ctx, const KParams& kp, const double* dX, int n, double** buf,
                 size_t* cap) {
  GPR_TRY(ensure_buf(ctx, buf, cap, (size_t)kp.nse * kp.d * n + 1));
  const size_t total = (size_t)kp.nse * kp.d * n;
  int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  if (blocks < 1) blocks = 1;
  scale_inputs_kernel<<<blocks, 256, 0, ctx->stream>>>(kp, dX, n, *buf);
  LAUNCH_CHECK(ctx);
  return 0;
}

// ---- 16-B-store assembly (compile-time d, 16-B aligned K with even ldk) ----------------
// Thread t of the 256 owns rows i0 + 2 (t & 31) + {0,1} and columns j0 + (t >> 5) + 8c,
// c < 8: every direct store is one 16-B pair of adjacent rows (32 lanes = one 512-B column
// segment).  Row features stay in registers; the tile's 64 column points sit in LDS and are
// read as half-wave broadcasts.  The mirror tile goes through LDS (row stride 65 doubles:
// conflict-free scalar writes) and is re-read as row pairs, so it too is stored 16 B/lane.
constexpr int KT_LDS = KT * (KT + 1);  // doubles; also holds the 64 x D column points

// One 64 x 64 tile of K (or cross K), all SE parts summed in part order (src/compose_covar.jl:
// 52-56).  DIAG: a diagonal tile of the symmetric K -- eps per SE part and sigma_n^2 on i == j
// (only these 1/nt of the tiles pay the index compares).  tabs = nse tables of 256 doubles.
template <int D, bool DIAG>
__device__ __forceinline__ void kmat_tile_compute(const KParams& kp, const double* __restrict__ xs,
                                                  int n, const double* __restrict__ xcs, int m,
                                                  int i0, int j0, double* lds, const double* tabs,
                                                  double (&v)[8][2]) {
  constexpr int NFILL = (KT * D + 255) / 256;  // column-point doubles per thread per part
  const int t = threadIdx.x, l32 = t & 31, cg = t >> 5;
  const int ia = min(i0 + 2 * l32, n - 1), ib = min(i0 + 2 * l32 + 1, n - 1);
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c][0] = v[c][1] = 0.0;
  for (int p = 0; p < kp.nse; ++p) {
    const double* xp_rows = xs + (size_t)p * n * D;
    const double* xp_cols = xcs + (size_t)p * m * D;
    // all global loads of this part first (row features + this thread's column-point share)
    double xr0[D], xr1[D], fill[NFILL];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xr0[k] = xp_rows[(size_t)ia * D + k];
      xr1[k] = xp_rows[(size_t)ib * D + k];
    }
#pragma unroll
    for (int f = 0; f < NFILL; ++f) {
      const int e = t + 256 * f;
      const int jl = e / D;
      fill[f] = e < KT * D ? xp_cols[(size_t)min(j0 + jl, m - 1) * D + (e - jl * D)] : 0.0;
    }
    __syncthreads();  // previous part's column points fully consumed
#pragma unroll
    for (int f = 0; f < NFILL; ++f)
      if (t + 256 * f < KT * D) lds[t + 256 * f] = fill[f];
    __syncthreads();
    const double* ts = tabs + 256 * p;
    // columns in groups of KB_CG: KB_CG x 2 independent distance accumulators, k outermost
    // (smaller groups keep fewer exp evaluations in flight: register pressure / occupancy)
#pragma unroll
    for (int cb = 0; cb < 8; cb += KB_CG) {
      double d0[KB_CG], d1[KB_CG];
#pragma unroll
      for (int c = 0; c < KB_CG; ++c) d0[c] = d1[c] = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
#pragma unroll
        for (int c = 0; c < KB_CG; ++c) {
          const double cv = lds[(cg + 8 * (cb + c)) * D + k];
          const double q0 = xr0[k] - cv, q1 = xr1[k] - cv;
          d0[c] = fma(q0, q0, d0[c]);
          d1[c] = fma(q1, q1, d1[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < KB_CG; ++c) {
        double t0 = kexp_s2(d0[c], ts), t1 = kexp_s2(d1[c], ts);
        if (DIAG) {
          const int j = j0 + cg + 8 * (cb + c), i = i0 + 2 * l32;
          if (i == j) t0 += kp.eps;
          if (i + 1 == j) t1 += kp.eps;
        }
        v[cb + c][0] += t0;  // 0 + t == t: part 1 enters unrounded
        v[cb + c][1] += t1;
      }
    }
  }
  if (DIAG && kp.has_noise) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = j0 + cg + 8 * c, i = i0 + 2 * l32;
      if (i == j) v[c][0] += kp.noise2;
      if (i + 1 == j) v[c][1] += kp.noise2;
    }
  }
}

// per-part exp tables s2_p * 2^(j/256) into LDS (256 threads)
__device__ __forceinline__ void load_part_tables(const KParams& kp, double* tabs) {
#if GPR_EXP32
  const double T = kp.exptab[(threadIdx.x & 31) << 3];  // compact 2^(j/32) tables
#else
  const double T = kp.exptab[threadIdx.x];
#endif
  for (int p = 0; p < kp.nse; ++p) tabs[256 * p + threadIdx.x] = (kp.sigma[p] * kp.sigma[p]) * T;
}

typedef double kd2 __attribute__((ext_vector_type(2)));

// K is written once and not re-read by this kernel: non-temporal (streaming) stores
__device__ __forceinline__ void store_pair(double* K, size_t idx, bool ok0, bool ok1, double a,
                                           double b) {
#ifdef GPR_KBUILD_NOSTORE  // diagnostics (tools/kbuild_bench_nostore): compute-only timing
  if (!(a == a) || !(b == b)) K[idx] = a;
  return;
#endif
  if (ok1) {
#ifdef GPR_KBUILD_TEMPORAL
    *reinterpret_cast<kd2*>(K + idx) = kd2{a, b};
#else
    __builtin_nontemporal_store(kd2{a, b}, reinterpret_cast<kd2*>(K + idx));
#endif
  } else if (ok0) {
    K[idx] = a;
  }
}

template <int D>
__global__ __launch_bounds__(256, GPR_KBUILD_MINB) void kmat_sym2_kernel(KParams kp, const double* __restrict__ xs,
                                                        int n, double* __restrict__ K, size_t ldk,
                                                        int ntiles) {
  extern __shared__ double dyn_lds[];  // KT_LDS doubles, then nse exp tables
  double* lds = dyn_lds;
  double* tabs = dyn_lds + KT_LDS;
  const int t = threadIdx.x, l32 = t & 31, cg = t >> 5;
  load_part_tables(kp, tabs);
  __syncthreads();
  // persistent: a workgroup walks tiles, so one tile's math overlaps the previous tile's
  // stores draining to HBM
  for (int bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
    int bj = (int)((sqrt(8.0 * bid + 1.0) - 1.0) * 0.5);
    while ((bj + 1) * (bj + 2) / 2 <= bid) ++bj;
    while (bj * (bj + 1) / 2 > bid) --bj;
    const int bi = bid - bj * (bj + 1) / 2;
    const int i0 = bi * KT, j0 = bj * KT;
    double v[8][2];
    if (bi == bj)
      kmat_tile_compute<D, true>(kp, xs, n, xs, n, i0, j0, lds, tabs, v);
    else
      kmat_tile_compute<D, false>(kp, xs, n, xs, n, i0, j0, lds, tabs, v);
    const int i = i0 + 2 * l32;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = j0 + cg + 8 * c;
      if (j < n) store_pair(K, (size_t)i + (size_t)j * ldk, i < n, i + 1 < n, v[c][0], v[c][1]);
    }
    if (bi == bj) continue;
    __syncthreads();  // column points no longer needed: reuse LDS for the transpose
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int jl = cg + 8 * c;
      lds[(2 * l32) * (KT + 1) + jl] = v[c][0];
      lds[(2 * l32 + 1) * (KT + 1) + jl] = v[c][1];
    }
    __syncthreads();
    // mirror: K[j0 + 2q + {0,1}, i0 + il] = tile[il][2q + {0,1}]
    const int jj = j0 + 2 * l32;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int il = cg + 8 * c;
      if (i0 + il < n)
        store_pair(K, (size_t)jj + (size_t)(i0 + il) * ldk, jj < n, jj + 1 < n,
                   lds[il * (KT + 1) + 2 * l32], lds[il * (KT + 1) + 2 * l32 + 1]);
    }
  }
}

template <int D>
__global__ __launch_bounds__(256, GPR_KBUILD_MINB) void kmat_cross2_kernel(KParams kp, const double* __restrict__ xs,
                                                          int n, const double* __restrict__ xps,
                                                          int m, double* __restrict__ K,
                                                          size_t ldk, int ntile_i, int ntiles) {
  extern __shared__ double dyn_lds[];  // KT * D doubles, then nse exp tables
  double* lds = dyn_lds;
  double* tabs = dyn_lds + KT * D;
  const int t = threadIdx.x, l32 = t & 31, cg = t >> 5;
  load_part_tables(kp, tabs);
  __syncthreads();
  for (int bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
    const int bi = bid % ntile_i, bj = bid / ntile_i;
    const int i0 = bi * KT, j0 = bj * KT;
    double v[8][2];
    kmat_tile_compute<D, false>(kp, xs, n, xps, m, i0, j0, lds, tabs, v);
    const int i = i0 + 2 * l32;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = j0 + cg + 8 * c;
      if (j < m) store_pair(K, (size_t)i + (size_t)j * ldk, i < n, i + 1 < n, v[c][0], v[c][1]);
    }
  }
}

template <int D>
void launch_sym(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, double* K, int ldk) {
  const int nt = (n + KT - 1) / KT;
  const long long nblk = (long long)nt * (nt + 1) / 2;
  if constexpr (D > 0) {
    if (vec_store_ok(K, ldk)) {
      const int grid = (int)std::min<long long>(nblk, kbuild_grid());
      const size_t lds_bytes = sizeof(double) * (KT_LDS + 256 * kp.nse);
      kmat_sym2_kernel<D><<<grid, 256, lds_bytes, ctx->stream>>>(kp, xs, n, K, (size_t)ldk, (int)nblk);
      return;
    }
  }
  kmat_sym_kernel<D><<<(unsigned)nblk, 256, 0, ctx->stream>>>(kp, xs, n, K, (size_t)ldk);
}

template <int D>
void launch_cross(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, const double* xps,
                  int m, double* K, int ldk) {
  const int nti = (n + KT - 1) / KT, ntj = (m + KT - 1) / KT;
  const unsigned nblk = (unsigned)((long long)nti * ntj);
  if constexpr (D > 0) {
    if (vec_store_ok(K, ldk)) {
      const int grid = (int)std::min<long long>(nblk, kbuild_grid());
      const size_t lds_bytes = sizeof(double) * (KT * D + 256 * kp.nse);
      kmat_cross2_kernel<D><<<grid, 256, lds_bytes, ctx->stream>>>(kp, xs, n, xps, m, K, (size_t)ldk,
                                                                   nti, (int)nblk);
      return;
    }
  }
  kmat_cross_kernel<D><<<nblk, 256, 0, ctx->stream>>>(kp, xs, n, xps, m, K, (size_t)ldk, nti);
}

// ---- Gram form of the distance on FP64 MFMA ---------------------------------------------
// -D_ab = (-|y_a|^2 - |y_b|^2) + sum_k (2 y_a,k) y_b,k with y = x .* l - c, where c is the mean of
// (a bounded sample of) the part's scaled training points (distances are translation invariant; centring keeps |y|^2,
// the cancelling terms, small).  Per 16 x 16 block the sum is ceil(d/4) v_mfma_f64_16x16x4f64
// started from C = -|y_a|^2 - |y_b|^2 (one VALU add per element), so the FP64 VALU is left with
// exp (kexp_s2) and the part sum.  Rounding: |error of D| <~ (d + 1) u (|y_a|^2 + |y_b|^2),
// ~1e-15 absolute at the default hp (K within rtol 1e-13 of the reference's difference form,
// tests/test_gpu_parity.py); a same-object diagonal gets D = 0 exactly and diagonal tiles are
// made bitwise symmetric.  GPR_KBUILD_EXACT=1 selects the reference's difference form
// (x .* l - x' .* l)^2 in kmat_sym2/cross2.
// Measured (tools/kbuild_bench, SE+SE+WN N = 32768 d = 8, same box): difference form 2.43 ms,
// the same Gram sum on the VALU 2.36 ms, MFMA with the norms as a third k-step 2.07 ms.
// Operands are prepared once per call in MFMA lane order: for 16-point block b and k-step s,
// 64 doubles, lane l <-> (point 16 b + (l & 15), k = 4 s + (l >> 4)) -- every operand load is one
// coalesced 512-B wave load; points padded to a multiple of 64 (zeros).
typedef double gd4 __attribute__((ext_vector_type(4)));
#ifndef GRAM_EXPG  // exp evaluations the scheduler may interleave (register pressure)
#define GRAM_EXPG 4
#endif

// grid = nse * d workgroups of 256: c[p][k] = mean over the first min(n, GRAM_CENTER_PTS) points
// of xs[p][.][k] (fixed-order tree sum).  Any centre inside the data's spread serves (it only
// sets the size of |y|^2); a bounded sample keeps this a few microseconds at any n.
constexpr int GRAM_CENTER_PTS = 2048;
__global__ __launch_bounds__(256) void gram_center_kernel(const double* __restrict__ xs, int n,
                                                          int d, double* __restrict__ c) {
  __shared__ double red[256];
  const int p = blockIdx.x / d, k = blockIdx.x % d;
  const int cnt = min(n, GRAM_CENTER_PTS);
  double sum = 0.0;
  for (int a = threadIdx.x; a < cnt; a += 256) sum += xs[((size_t)p * n + a) * d + k];
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) c[p * KMAXD + k] = red[0] / (double)cnt;
}

// out[p][blk][s][lane] = scale * y[16 blk + (lane & 15)][4 s + (lane >> 4)] (0 past d or n);
// nrm[p][a] = -|y_a|^2 (0 for padded points)
__global__ void gram_prep_kernel(const double* __restrict__ xs, int n, int d, int S, int nblk,
                                 int nse, const double* __restrict__ c, double scale,
                                 double* __restrict__ out, double* __restrict__ nrm) {
  const size_t total = (size_t)nse * nblk * S * 64;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int lane = (int)(t & 63);
    const size_t r = t >> 6;
    const int s = (int)(r % S);
    const size_t r2 = r / S;
    const int blk = (int)(r2 % nblk), p = (int)(r2 / nblk);
    const int a = blk * 16 + (lane & 15), k = 4 * s + (lane >> 4);
    const double* xa = xs + ((size_t)p * n + a) * d;
    const double* cp = c + p * KMAXD;
    out[t] = (a < n && k < d) ? scale * (xa[k] - cp[k]) : 0.0;
    if (nrm && s == 0 && lane < 16) {
      double q = 0.0;
      if (a < n)
        for (int kk = 0; kk < d; ++kk) {
          const double y = xa[kk] - cp[kk];
          q = fma(y, y, q);
        }
      nrm[(size_t)p * nblk * 16 + a] = -q;
    }
  }
}

// One 64 x 64 tile of K on MFMA + VALU, SE parts summed in order.  Wave w owns the 32 x 32
// quadrant (rows 32 (w & 1), cols 32 (w >> 1)): 2 x 2 blocks of 16 x 16; lane l / register q of
// block (rb, cb) <-> row 16 rb + (l >> 4) + 4 q, col 16 cb + (l & 15).
template <int S, bool DIAG>
__device__ __forceinline__ void gram_tile(const KParams& kp, const double* __restrict__ gA,
                                          const double* __restrict__ gB, const double* __restrict__ nA,
                                          const double* __restrict__ nB, int nblkA, int nblkB,
                                          int i0, int j0, const double* tabs, gd4 (&v)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w & 1, wc = w >> 1;
  const int ba = (i0 >> 4) + 2 * wr, bb = (j0 >> 4) + 2 * wc;  // first 16-blocks
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) v[rb][cb] = gd4{0.0, 0.0, 0.0, 0.0};
  for (int p = 0; p < kp.nse; ++p) {
    const double* Ap = gA + ((size_t)p * nblkA + ba) * S * 64 + lane;
    const double* Bp = gB + ((size_t)p * nblkB + bb) * S * 64 + lane;
    const double* nAp = nA + (size_t)p * nblkA * 16 + ba * 16 + (lane >> 4);
    const double* nBp = nB + (size_t)p * nblkB * 16 + bb * 16 + (lane & 15);
    double a[2][S], b[2][S], nr[2][4], nc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        a[h][s] = Ap[(h * S + s) * 64];
        b[h][s] = Bp[(h * S + s) * 64];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) nr[h][q] = nAp[16 * h + 4 * q];
      nc[h] = nBp[16 * h];
    }
    gd4 acc[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[rb][cb][q] = nr[rb][q] + nc[cb];
#pragma unroll
        for (int s = 0; s < S; ++s)
          acc[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[rb][s], b[cb][s], acc[rb][cb], 0, 0, 0);
      }
    const double* ts = tabs + 256 * p;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          double x = acc[rb][cb][q];  // -D
          bool on_diag = false;
          if (DIAG) {
            on_diag = wr == wc && rb == cb && (lane >> 4) + 4 * q == (lane & 15);
            if (on_diag) x = 0.0;
          }
          double t = kexp_s2(-x, ts);
          if (DIAG && on_diag) t += kp.eps;
          v[rb][cb][q] += t;
          if ((q + 1) % GRAM_EXPG == 0) __builtin_amdgcn_sched_barrier(0);
        }
  }
  if (DIAG && kp.has_noise && wr == wc) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if ((lane >> 4) + 4 * q == (lane & 15)) v[rb][rb][q] += kp.noise2;
  }
}

// tile -> LDS, column-major with column stride 65
__device__ __forceinline__ void gram_to_lds(const gd4 (&v)[2][2], double* T) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = 32 * (w & 1) + (lane >> 4), c0 = 32 * (w >> 1) + (lane & 15);
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) T[(c0 + 16 * cb) * (KT + 1) + r0 + 16 * rb + 4 * q] = v[rb][cb][q];
}

// upper-triangle tile bid -> (bi <= bj), column-by-column order; wave-uniform
__device__ __forceinline__ void tri_tile(int bid, int* bi, int* bj) {
  int j = (int)((sqrt(8.0 * bid + 1.0) - 1.0) * 0.5);
  while ((j + 1) * (j + 2) / 2 <= bid) ++j;
  while (j * (j + 1) / 2 > bid) --j;
  j = __builtin_amdgcn_readfirstlane(j);
  *bj = j;
  *bi = __builtin_amdgcn_readfirstlane(bid - j * (j + 1) / 2);
}

template <int S>
__global__ __launch_bounds__(256, 4) void kmat_symg_kernel(KParams kp, const double* __restrict__ gA,
                                                         const double* __restrict__ gB,
                                                         const double* __restrict__ nrm, int nblk,
                                                         int n, double* __restrict__ K, size_t ldk,
                                                         int ntiles) {
  extern __shared__ double dyn_lds[];  // KT_LDS doubles (tile), then nse exp tables
  double* T = dyn_lds;
  double* tabs = dyn_lds + KT_LDS;
  const int t = threadIdx.x, l32 = t & 31, cg = t >> 5;
  load_part_tables(kp, tabs);
  __syncthreads();
  for (int bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
    int bi, bj;
    tri_tile(bid, &bi, &bj);
    const int i0 = bi * KT, j0 = bj * KT;
    gd4 v[2][2];
    if (bi == bj)
      gram_tile<S, true>(kp, gA, gB, nrm, nrm, nblk, nblk, i0, j0, tabs, v);
    else
      gram_tile<S, false>(kp, gA, gB, nrm, nrm, nblk, nblk, i0, j0, tabs, v);
    __syncthreads();  // previous tile's LDS reads are done
    gram_to_lds(v, T);
    __syncthreads();
    // direct: K[i0 + 2 l32 + {0,1}, j0 + jl] = T[jl][2 l32 + {0,1}]
    const int i = i0 + 2 * l32;
    if (bi == bj) {
      // diagonal tile: the strictly-lower half mirrors the upper, so K == K^T bitwise
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int jl = cg + 8 * c, j = j0 + jl, r0 = 2 * l32, r1 = 2 * l32 + 1;
        const double e0 = r0 <= jl ? T[jl * (KT + 1) + r0] : T[r0 * (KT + 1) + jl];
        const double e1 = r1 <= jl ? T[jl * (KT + 1) + r1] : T[r1 * (KT + 1) + jl];
        if (j < n) store_pair(K, (size_t)i + (size_t)j * ldk, i < n, i + 1 < n, e0, e1);
      }
      continue;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int jl = cg + 8 * c, j = j0 + jl;
      if (j < n)
        store_pair(K, (size_t)i + (size_t)j * ldk, i < n, i + 1 < n, T[jl * (KT + 1) + 2 * l32],
                   T[jl * (KT + 1) + 2 * l32 + 1]);
    }
    // mirror: K[j0 + 2 l32 + {0,1}, i0 + il] = tile(il, 2 l32 + {0,1}) = T[2 l32 + {0,1}][il]
    const int jj = j0 + 2 * l32;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int il = cg + 8 * c;
      if (i0 + il < n)
        store_pair(K, (size_t)jj + (size_t)(i0 + il) * ldk, jj < n, jj + 1 < n,
                   T[(2 * l32) * (KT + 1) + il], T[(2 * l32 + 1) * (KT + 1) + il]);
    }
  }
}

template <int S>
__global__ __launch_bounds__(256, 4) void kmat_crossg_kernel(KParams kp, const double* __restrict__ gA,
                                                           const double* __restrict__ gB,
                                                           const double* __restrict__ nrmA,
                                                           const double* __restrict__ nrmB,
                                                           int nblkA, int nblkB, int n, int m,
                                                           double* __restrict__ K, size_t ldk,
                                                           int ntile_i, int ntiles) {
  extern __shared__ double dyn_lds[];
  double* T = dyn_lds;
  double* tabs = dyn_lds + KT_LDS;
  const int t = threadIdx.x, l32 = t & 31, cg = t >> 5;
  load_part_tables(kp, tabs);
  __syncthreads();
  for (int bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
    const int bi = __builtin_amdgcn_readfirstlane(bid % ntile_i);
    const int bj = __builtin_amdgcn_readfirstlane(bid / ntile_i);
    const int i0 = bi * KT, j0 = bj * KT;
    gd4 v[2][2];
    gram_tile<S, false>(kp, gA, gB, nrmA, nrmB, nblkA, nblkB, i0, j0, tabs, v);
    __syncthreads();
    gram_to_lds(v, T);
    __syncthreads();
    const int i = i0 + 2 * l32;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int jl = cg + 8 * c, j = j0 + jl;
      if (j < m)
        store_pair(K, (size_t)i + (size_t)j * ldk, i < n, i + 1 < n, T[jl * (KT + 1) + 2 * l32],
                   T[jl * (KT + 1) + 2 * l32 + 1]);
    }
  }
}

// ---- upper-only K for a factorisation (the tile-DAG mirrors the rest) -------------------
// Column c gets rows [0, min(n, 128 (c / 128 + 1))): the upper triangle plus the whole 128 x
// 128 diagonal blocks -- everything the tile-DAG reads -- as ONE contiguous run per column;
// the DAG stores each off-diagonal tile it loads, transposed, into the strict lower triangle
// (DAG_MIRROR), so the buffer still ends as upper U / strict lower K with half the bytes here.
// Work item = (strip of 32 columns, segment of 256 rows), one wave each, no LDS but the exp
// tables and no barrier: the strip's column operands and norms stay in registers while the
// wave walks down its segment 32 rows at a time.  The MFMA is oriented so that the D layout is
// the store layout: operand A = column points, B = row points, so lane l, register q of block
// (rb, cb) holds row i0 + 16 rb + (l & 15), column j0 + 16 cb + (l >> 4) + 4 q, and each store
// instruction writes 4 columns x 128 contiguous bytes -- no LDS staging.  Elements of the
// diagonal blocks are computed in both orientations, bitwise equal: (2 y_i) y_j and (2 y_j) y_i
// are the same products, summed over the same k order from the same C = -|y_i|^2 - |y_j|^2.
#ifndef KU_WIDTH  // columns per strip (16 or 32)
#define KU_WIDTH 32
#endif
#ifndef KU_SEGROWS  // rows per work item
#define KU_SEGROWS 128
#endif
constexpr int KU_W = KU_WIDTH;     // strip width (columns)
constexpr int KU_CB = KU_W / 16;   // 16-column blocks per strip
constexpr int KU_H = 32;           // unit height (rows): two 16-row blocks
#ifndef KU_MINB  // workgroups (of 4 independent waves) per CU the upper-only build is compiled for
#define KU_MINB 3
#endif
constexpr int KU_SEG = KU_SEGROWS;
constexpr double KU_NC_LIM = 1.4e6;  // |y|^2 below which the exponentials need no clamp

// rows of column block j0 the factorisation reads
__host__ __device__ inline int kup_rows(int j0, int n) { return min(n, 128 * (j0 / 128 + 1)); }

// One 32 x 32 unit (rows i0.., columns j0..) of the upper-only build.  Per part: the four
// blocks' MFMAs first (their latency overlaps the previous part's / unit's exponentials), then
// the 16 exponentials per lane in groups of GRAM_EXPG.  DIAG: the unit on the diagonal (D = 0
// and eps per part on i == j, sigma_n^2 after the parts); EDGE: rows past r1 / columns past n
// masked.  Interior units store unconditionally, so the compiler counts the stores and the next
// unit's prefetched operands are waited for with vmcnt(stores), not vmcnt(0).
template <int S, int NSE, bool DIAG, bool EDGE, bool CLAMP>
__device__ __forceinline__ void kup_unit(const KParams& kp, const double (&ca)[NSE][KU_CB][S],
                                         const double* cn, const double (&ra)[NSE][2][S],
                                         const double (&rn)[NSE][2], const double* tabs,
                                         double* __restrict__ K, size_t ldk, int i0, int j0,
                                         int r1, int n, int voff) {
  const int lane = threadIdx.x & 63;
  // block by block, software-pipelined: the next block's MFMAs are issued before this block's
  // exponentials (their 64-cycle results are not waited for), then its 4 x NSE exponentials --
  // four independent chains per part, pinned as a group -- then its 4 stores.  The empty asm
  // statements pin each group's finished values where they are made: without them the compiler
  // sank the second half of every exponential down to the stores and kept all 16 in flight
  // (200+ registers, one wave per SIMD); pinned one by one, the chains ran serially (each
  // exponential waited for its own table read)
  auto mfma_block = [&](int blk, gd4 (&acc)[NSE]) {
    const int rb = blk / KU_CB, cb = blk % KU_CB;
#pragma unroll
    for (int p = 0; p < NSE; ++p) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[p][q] = rn[p][rb] + cn[KU_W * p + 16 * cb + (lane >> 4) + 4 * q];
#pragma unroll
      for (int s = 0; s < S; ++s)
        acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[p][cb][s], ra[p][rb][s], acc[p], 0, 0, 0);
    }
  };
  constexpr int NBLK = 2 * KU_CB;
  gd4 acc[NSE], accn[NSE];
  mfma_block(0, acc);
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk) {
    const int rb = blk / KU_CB, cb = blk % KU_CB;
    if (blk < NBLK - 1) mfma_block(blk + 1, accn);
    double v[4];
#pragma unroll
    for (int p = 0; p < NSE; ++p) {
      const double* ts = tabs + 256 * p;
      double e[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double x = acc[p][q];  // -D
        bool on = false;
        if (DIAG) {
          on = i0 + 16 * rb + (lane & 15) == j0 + 16 * cb + (lane >> 4) + 4 * q;
          if (on) x = 0.0;
        }
        e[q] = CLAMP ? kexp_s2(-x, ts) : kexp_s2_nc(-x, ts);
        if (DIAG && on) e[q] += kp.eps;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = p == 0 ? e[q] : v[q] + e[q];
      asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double val = v[q];
      if (DIAG && kp.has_noise && i0 + 16 * rb + (lane & 15) == j0 + 16 * cb + (lane >> 4) + 4 * q)
        val += kp.noise2;
      // uniform base (SGPR) + the lane's 32-bit offset: rows 16 rb + (lane & 15), columns
      // 16 cb + 4 q + (lane >> 4) of the unit
      double* base = K + (size_t)(i0 + 16 * rb) + (size_t)(j0 + 16 * cb + 4 * q) * ldk;
#ifdef GPR_KBUILD_NOSTORE  // diagnostics (tools/kbuild_bench_nostore): compute-only timing
      if (!(val == val)) base[voff] = val;
#else
      if (!EDGE || (i0 + 16 * rb + (lane & 15) < r1 && j0 + 16 * cb + 4 * q + (lane >> 4) < n))
        __builtin_nontemporal_store(val, base + voff);
#endif
    }
    if (blk < NBLK - 1)
#pragma unroll
      for (int p = 0; p < NSE; ++p) acc[p] = accn[p];
  }
}

// One interior item of a single-part build (NSE = 1: 32 columns x KU_SEG rows, no diagonal
// element, no ragged edge; GPR_KBUILD_COLSTORE), its values staged through this wave's LDS 16
// columns at a time and stored as one column's 128 rows per store instruction (1 KB, 16 B per
// lane) instead of the MFMA D layout's 4 columns x 128 B: the fastest upper-only store shape the
// kernel's items allow (bench.py `kbuild_store_ceiling`: items_1k_column_stores).  The same
// MFMAs and exponentials as kup_unit in the same order per element: bit for bit the same K.
constexpr int KU_SP = KU_SEG + 2;  // staging column stride (doubles): +16 B against bank repeats
template <int S, bool CLAMP>
__device__ __forceinline__ void kup_item_cols(const double (&ca)[1][KU_CB][S], const double* cn,
                                              const double* __restrict__ gA,
                                              const double* __restrict__ nrm, const double* tabs,
                                              double* stg, double* __restrict__ K, size_t ldk,
                                              int r0, int j0) {
  constexpr int RB = KU_SEG / 16;  // row blocks of the item
  const int lane = threadIdx.x & 63;
  double ra[RB][S], rn[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int ba = (r0 >> 4) + rb;
#pragma unroll
    for (int s = 0; s < S; ++s) ra[rb][s] = gA[((size_t)ba * S + s) * 64 + lane];
    rn[rb] = nrm[ba * 16 + (lane & 15)];
  }
#pragma unroll
  for (int cb = 0; cb < KU_CB; ++cb) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      gd4 acc;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = rn[rb] + cn[16 * cb + (lane >> 4) + 4 * q];
#pragma unroll
      for (int s = 0; s < S; ++s)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[0][cb][s], ra[rb][s], acc, 0, 0, 0);
      double e[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) e[q] = CLAMP ? kexp_s2(-acc[q], tabs) : kexp_s2_nc(-acc[q], tabs);
      asm volatile("" : "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]));
#pragma unroll
      for (int q = 0; q < 4; ++q) stg[((lane >> 4) + 4 * q) * KU_SP + 16 * rb + (lane & 15)] = e[q];
    }
    // (one wave's LDS operations complete in order: the reads below see the writes above)
#pragma unroll 4
    for (int c = 0; c < 16; ++c) {
      const kd2 v = *reinterpret_cast<const kd2*>(stg + c * KU_SP + 2 * lane);
      double* dst = K + (size_t)r0 + 2 * lane + (size_t)(j0 + 16 * cb + c) * ldk;
#ifdef GPR_KBUILD_NOSTORE  // diagnostics (tools/kbuild_bench_nostore): compute-only timing
      if (!(v.x == v.x)) *dst = v.x;
#else
      __builtin_nontemporal_store(v, reinterpret_cast<kd2*>(dst));
#endif
    }
  }
}

template <int S, int NSE>
__global__ __launch_bounds__(256, KU_MINB) void kmat_symu_kernel(KParams kp, const double* __restrict__ gA,
                                                        const double* __restrict__ gB,
                                                        const double* __restrict__ nrm, int nblk,
                                                        int n, double* __restrict__ K, size_t ldk,
                                                        const int* __restrict__ items, int nitems,
                                                        int full, int colstore) {
  extern __shared__ double tabs[];  // NSE exp tables, then per wave the strip's column norms
                                    // (then, colstore, per wave the 16-column staging)
  load_part_tables(kp, tabs);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  const int voff = (lane & 15) + (lane >> 4) * (int)ldk;  // (< 2^31: ldk < 2^29)
  double* cn = tabs + 256 * NSE + (threadIdx.x >> 6) * (KU_W * NSE);  // this wave's
  for (int t = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); t < nitems;
       t += W) {
    const int code = __builtin_amdgcn_readfirstlane(items[t]);
    const int j0 = (code >> 16) * KU_W, r0 = (code & 0xffff) * KU_SEG;
    const int r1 = min(r0 + KU_SEG, full ? n : kup_rows(j0, n));
    // the strip's column operands (A role, registers) and column norms (this wave's LDS: the
    // lanes of a block read 4 distinct addresses per instruction -- broadcasts)
    double ca[NSE][KU_CB][S];
#pragma unroll
    for (int p = 0; p < NSE; ++p)
#pragma unroll
      for (int cb = 0; cb < KU_CB; ++cb) {
        const int bb = (j0 >> 4) + cb;
#pragma unroll
        for (int s = 0; s < S; ++s) ca[p][cb][s] = gB[(((size_t)p * nblk + bb) * S + s) * 64 + lane];
      }
    __builtin_amdgcn_wave_barrier();  // (the previous item's norm reads are done: one wave)
    // the exponentials skip their range clamp where D = |y_i|^2 + |y_j|^2 - 2 y_i.y_j <=
    // 2 (|y_i|^2 + |y_j|^2) < 5.6e6 provably (kexp_s2_nc): every |y|^2 < KU_NC_LIM here
    bool big = false;
    if (lane < KU_W)
#pragma unroll
      for (int p = 0; p < NSE; ++p) {
        const double c = nrm[(size_t)p * nblk * 16 + j0 + lane];
        cn[KU_W * p + lane] = c;
        big |= !(-c < KU_NC_LIM);
      }
    const bool cols_big = __ballot(big) != 0;
    __builtin_amdgcn_wave_barrier();
    if constexpr (NSE == 1) {
      // an interior item (a full segment of rows, every column inside n, no diagonal element)
      // through the column-store path
      if (colstore && r1 - r0 == KU_SEG && j0 + KU_W <= n && !(j0 >= r0 && j0 < r1)) {
        double* stg = tabs + (256 + 4 * KU_W) * NSE + (threadIdx.x >> 6) * (16 * KU_SP);
        bool rbig = cols_big;
        for (int rb = 0; rb < KU_SEG / 16; ++rb)
          rbig |= !(-nrm[(r0 >> 4) * 16 + rb * 16 + (lane & 15)] < KU_NC_LIM);
        if (__ballot(rbig) != 0)
          kup_item_cols<S, true>(ca, cn, gA, nrm, tabs, stg, K, ldk, r0, j0);
        else
          kup_item_cols<S, false>(ca, cn, gA, nrm, tabs, stg, K, ldk, r0, j0);
        continue;
      }
    }
    // row operands (B role) of a 32-row unit: clamped to the last unit (branch-free prefetch)
    auto load_rows = [&](int i0, double (&ra)[NSE][2][S], double (&rn)[NSE][2]) {
      const int ii = min(i0, r1 - 1) & ~(KU_H - 1);
#pragma unroll
      for (int p = 0; p < NSE; ++p)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int ba = (ii >> 4) + rb;
#pragma unroll
          for (int s = 0; s < S; ++s) ra[p][rb][s] = gA[(((size_t)p * nblk + ba) * S + s) * 64 + lane];
          rn[p][rb] = nrm[(size_t)p * nblk * 16 + ba * 16 + (lane & 15)];
        }
    };
    double ra[NSE][2][S], rn[NSE][2];
    load_rows(r0, ra, rn);
    const bool edge_cols = j0 + KU_W > n;
    for (int i0 = r0; i0 < r1; i0 += KU_H) {
      double nra[NSE][2][S], nrn[NSE][2];
      load_rows(i0 + KU_H, nra, nrn);  // next unit's rows, in flight during this one
      bool rbig = cols_big;
#pragma unroll
      for (int p = 0; p < NSE; ++p) rbig |= !(-rn[p][0] < KU_NC_LIM) || !(-rn[p][1] < KU_NC_LIM);
      const bool clamp = __ballot(rbig) != 0;
      // (wave-uniform branches) the diagonal unit, ragged edges, the interior
      if (j0 >= i0 && j0 < i0 + KU_H)  // (the unit holds diagonal elements)
        kup_unit<S, NSE, true, true, true>(kp, ca, cn, ra, rn, tabs, K, ldk, i0, j0, r1, n, voff);
      else if (edge_cols || i0 + KU_H > r1)
        kup_unit<S, NSE, false, true, true>(kp, ca, cn, ra, rn, tabs, K, ldk, i0, j0, r1, n, voff);
      else if (clamp)
        kup_unit<S, NSE, false, false, true>(kp, ca, cn, ra, rn, tabs, K, ldk, i0, j0, r1, n, voff);
      else
        kup_unit<S, NSE, false, false, false>(kp, ca, cn, ra, rn, tabs, K, ldk, i0, j0, r1, n, voff);
#pragma unroll
      for (int p = 0; p < NSE; ++p)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
          for (int s = 0; s < S; ++s) ra[p][rb][s] = nra[p][rb][s];
          rn[p][rb] = nrn[p][rb];
        }
    }
  }
}

// the Gram form (MFMA distance) for d <= 20 unless the context asks for the reference's
// difference form (GPR_KBUILD_EXACT knob)
inline bool gram_enabled(const gpr_ctx* ctx, int d) { return !ctx->kbuild_exact && d <= 4 * 5; }

template <int S>
int launch_gram(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, const double* xps,
                int m, int same, double* K, int ldk) {
  const int d = kp.d;
  const int nbA = ((n + KT - 1) / KT) * (KT / 16);
  const int nbB = same ? nbA : ((m + KT - 1) / KT) * (KT / 16);
  const size_t opA = (size_t)kp.nse * nbA * S * 64, opB = same ? 0 : (size_t)kp.nse * nbB * S * 64;
  const size_t nA = (size_t)kp.nse * nbA * 16, nB = same ? 0 : (size_t)kp.nse * nbB * 16;
  // dgA: row operands + row norms; dgB: column operands + column norms (cross only)
  GPR_TRY(ensure_buf(ctx, &ctx->dgc, &ctx->gc_cap, (size_t)KMAXP * KMAXD));
  GPR_TRY(ensure_buf(ctx, &ctx->dgA, &ctx->gA_cap, opA + nA + (same ? opA : 0)));
  if (!same) GPR_TRY(ensure_buf(ctx, &ctx->dgB, &ctx->gB_cap, opB + nB));
  double* A = ctx->dgA;
  double* nrmA = A + opA;
  double* B = same ? nrmA + nA : ctx->dgB;
  double* nrmB = same ? nrmA : B + opB;
  gram_center_kernel<<<kp.nse * d, 256, 0, ctx->stream>>>(xs, n, d, ctx->dgc);
  auto prep = [&](const double* src, int cnt, int nblk, double scale, double* out, double* nrm) {
    const size_t total = (size_t)kp.nse * nblk * S * 64;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
    gram_prep_kernel<<<blocks, 256, 0, ctx->stream>>>(src, cnt, d, S, nblk, kp.nse, ctx->dgc,
                                                      scale, out, nrm);
  };
  prep(xs, n, nbA, 2.0, A, nrmA);
  prep(same ? xs : xps, same ? n : m, nbB, 1.0, B, same ? nullptr : nrmB);
  LAUNCH_CHECK(ctx);
  const size_t lds_bytes = sizeof(double) * (KT_LDS + 256 * kp.nse);
  if (same) {
    const int nt = (n + KT - 1) / KT;
    const long long nblk = (long long)nt * (nt + 1) / 2;
    const int grid = (int)std::min<long long>(nblk, kbuild_grid());
    kmat_symg_kernel<S><<<grid, 256, lds_bytes, ctx->stream>>>(kp, A, B, nrmA, nbA, n, K,
                                                               (size_t)ldk, (int)nblk);
  } else {
    const int nti = (n + KT - 1) / KT, ntj = (m + KT - 1) / KT;
    const long long nblk = (long long)nti * ntj;
    const int grid = (int)std::min<long long>(nblk, kbuild_grid());
    kmat_crossg_kernel<S><<<grid, 256, lds_bytes, ctx->stream>>>(kp, A, B, nrmA, nrmB, nbA, nbB,
                                                                 n, m, K, (size_t)ldk, nti,
                                                                 (int)nblk);
  }
  LAUNCH_CHECK(ctx);
  return 0;
}

// the upper-only build (kmat_symu_kernel): operands as launch_gram's same-object path
template <int S, int NSE>
int launch_gram_upper(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, double* K, int ldk,
                      int full) {
  const int d = kp.d;
  const int nbA = ((n + KT - 1) / KT) * (KT / 16);
  const size_t opA = (size_t)NSE * nbA * S * 64, nA = (size_t)NSE * nbA * 16;
  GPR_TRY(ensure_buf(ctx, &ctx->dgc, &ctx->gc_cap, (size_t)KMAXP * KMAXD));
  GPR_TRY(ensure_buf(ctx, &ctx->dgA, &ctx->gA_cap, 2 * opA + nA));
  double* A = ctx->dgA;
  double* nrmA = A + opA;
  double* B = nrmA + nA;
  // GPR_KBUILD_COLSTORE (single-part builds): interior items stored a column's 128 rows per
  // instruction through 16.6 KB of LDS per wave (16-B stores: K 16-B aligned, ldk even), and
  // one item per wave (no persistent loop: the hardware dispatches the items in list order, so
  // the running waves write a narrow, advancing band of columns).  The fit's upper-only build
  // only: for the full column build of gpr_kernel the column stores measured 6 % slower (1.73-
  // 1.76 vs 1.63-1.65 ms at N = 32768).  SE, N = 32768, d = 8, same box (profiles/r06_kbuild_
  // colstore_ab.txt): MFMA-layout stores 0.85-0.86 ms persistent / 0.82-0.83 one item per wave;
  // column stores 0.81-0.82 persistent / 0.70-0.72 one item per wave (0.75-0.78 of 8 TB/s).
  const int colstore = NSE == 1 && !full && ctx->kbuild_colstore && (ldk % 2) == 0 &&
                       ((uintptr_t)K % 16) == 0;
#ifndef KU_WGS  // workgroups per CU of the persistent grid (diagnostic builds: 1 << 20 = one
#define KU_WGS 8  // item per wave, dispatch order)
#endif
  const int wgs = colstore ? (1 << 20) : KU_WGS;  // workgroups per CU of the grid
  // work list, cached per (n, full, grid shape) in a few slots (fold and prior builds of
  // cross-validation alternate two shapes): rebuilding one costs a sync, a free and a copy
  const long long key = 4LL * n + 2 * colstore + full;
  gpr_ctx::KupList* kl = nullptr;
  for (auto& e : ctx->kup)
    if (e.key == key) kl = &e;
  if (!kl) {  // strip-major (bj << 16 | segment), into the least recently used slot
    kl = &ctx->kup[0];
    for (auto& e : ctx->kup)
      if (e.used < kl->used) kl = &e;
    std::vector<int> items;
    for (int bj = 0; bj * KU_W < n; ++bj) {
      const int rows = full ? n : kup_rows(bj * KU_W, n);
      for (int sg = 0; sg * KU_SEG < rows; ++sg) items.push_back((bj << 16) | sg);
    }
    {
      // XCD-aware order: wave w of workgroup b takes items t = 4 b + w (mod 4 grid), and
      // workgroups b, b + 8, ... share an XCD (its L2).  Give the workgroups of each residue
      // b mod 8 the segments sg = residue (mod 8), still strip-major: each XCD then reads one
      // eighth of the row operands (0.6 of 4.7 MB at C3, inside its 4-MB L2) instead of
      // streaming all of them through it for every strip.  (Placement is a speed hint only:
      // any order computes the same values.)
      const int nit = (int)items.size();
      const int W = (int)(4 * std::max(1LL, std::min((long long)(nit + 3) / 4, 256LL * wgs)));
      std::vector<int> q[8];
      for (int it : items) q[(it & 0xffff) % 8].push_back(it);
      size_t pos[8] = {};
      for (int t = 0; t < nit; ++t) {
        int g = ((t % W) / 4) % 8;
        for (int k = 0; k < 8 && pos[g] >= q[g].size(); ++k) g = (g + 1) % 8;
        items[t] = q[g][pos[g]++];
      }
    }
    if (kl->d) {  // (an earlier launch on the stream may still read the evicted list)
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      HIP_TRY(ctx, hipFree(kl->d));
      kl->d = nullptr;
    }
    kl->key = -1;
    HIP_TRY(ctx, hipMalloc((void**)&kl->d, items.size() * sizeof(int)));
    HIP_TRY(ctx, hipMemcpy(kl->d, items.data(), items.size() * sizeof(int),
                           hipMemcpyHostToDevice));
    kl->nitems = (int)items.size();
    kl->key = key;
  }
  kl->used = ++ctx->kup_clock;
  gram_center_kernel<<<NSE * d, 256, 0, ctx->stream>>>(xs, n, d, ctx->dgc);
  {
    const size_t total = opA;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
    gram_prep_kernel<<<blocks, 256, 0, ctx->stream>>>(xs, n, d, S, nbA, NSE, ctx->dgc, 2.0, A, nrmA);
    gram_prep_kernel<<<blocks, 256, 0, ctx->stream>>>(xs, n, d, S, nbA, NSE, ctx->dgc, 1.0, B, nullptr);
  }
  LAUNCH_CHECK(ctx);
  const int grid = (int)std::max(1LL, std::min((long long)(kl->nitems + 3) / 4, 256LL * wgs));
  const size_t lds = sizeof(double) * ((256 + 4 * KU_W) * NSE + (colstore ? 4 * 16 * KU_SP : 0));
  kmat_symu_kernel<S, NSE><<<grid, 256, lds, ctx->stream>>>(
      kp, A, B, nrmA, nbA, n, K, (size_t)ldk, kl->d, kl->nitems, full, colstore);
  LAUNCH_CHECK(ctx);
  return 0;
}

template <int NSE>
int launch_gram_upper_s(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, double* K, int ldk,
                        int full) {
  switch ((kp.d + 3) / 4) {
    case 1: return launch_gram_upper<1, NSE>(ctx, kp, xs, n, K, ldk, full);
    case 2: return launch_gram_upper<2, NSE>(ctx, kp, xs, n, K, ldk, full);
    case 3: return launch_gram_upper<3, NSE>(ctx, kp, xs, n, K, ldk, full);
    case 4: return launch_gram_upper<4, NSE>(ctx, kp, xs, n, K, ldk, full);
    default: return launch_gram_upper<5, NSE>(ctx, kp, xs, n, K, ldk, full);
  }
}

int launch_gram_any(gpr_ctx* ctx, const KParams& kp, const double* xs, int n, const double* xps,
                    int m, int same, double* K, int ldk) {
  switch ((kp.d + 3) / 4) {
    case 1: return launch_gram<1>(ctx, kp, xs, n, xps, m, same, K, ldk);
    case 2: return launch_gram<2>(ctx, kp, xs, n, xps, m, same, K, ldk);
    case 3: return launch_gram<3>(ctx, kp, xs, n, xps, m, same, K, ldk);
    case 4: return launch_gram<4>(ctx, kp, xs, n, xps, m, same, K, ldk);
    default: return launch_gram<5>(ctx, kp, xs, n, xps, m, same, K, ldk);
  }
}

#define DISPATCH_D(FN, ...)                 \
  switch (kp.d) {                           \
    case 1: FN<1>(__VA_ARGS__); break;      \
    case 2: FN<2>(__VA_ARGS__); break;      \
    case 3: FN<3>(__VA_ARGS__); break;      \
    case 4: FN<4>(__VA_ARGS__); break;      \
    case 5: FN<5>(__VA_ARGS__); break;      \
    case 6: FN<6>(__VA_ARGS__); break;      \
    case 7: FN<7>(__VA_ARGS__); break;      \
    case 8: FN<8>(__VA_ARGS__); break;      \
    case 16: FN<16>(__VA_ARGS__); break;    \
    default: FN<0>(__VA_ARGS__); break;     \
  }

// Pairwise split-factor kernel (src/split_kernel.jl:108-159) on pre-scaled points.
//   mode 0: Euclidean      v = s2 * exp(-sum (a-b)^2)
//   mode 1: SplitDistanceA v = s2 * exp(-sum (b^2 + 2 a b))      (a = xe, b = xq)
//   mode 2: SplitDistanceC v = s2 * exp(-sum (-2 a b))            (a = xs, b = xq)
// out[ia*sa + ib*sb]; lanes run along whichever of a/b has unit stride.
__global__ __launch_bounds__(256) void pair_kernel(int mode, int d, const double* __restrict__ xa,
                                                   int na, const double* __restrict__ xb, int nb,
                                                   double s2, double* __restrict__ out, size_t sa,
                                                   size_t sb, int a_fast) {
  const size_t total = (size_t)na * nb;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    int ia, ib;
    if (a_fast) {
      ia = (int)(t % na);
      ib = (int)(t / na);
    } else {
      ib = (int)(t % nb);
      ia = (int)(t / nb);
    }
    const double* pa = xa + (size_t)ia * d;
    const double* pb = xb + (size_t)ib * d;
    double D = 0.0;
    if (mode == 0) {
      for (int k = 0; k < d; ++k) {
        const double q = pa[k] - pb[k];
        D = fma(q, q, D);
      }
    } else if (mode == 1) {
      for (int k = 0; k < d; ++k) D += pb[k] * pb[k] + 2.0 * pa[k] * pb[k];
    } else {
      for (int k = 0; k < d; ++k) D += -2.0 * pa[k] * pb[k];
    }
    out[(size_t)ia * sa + (size_t)ib * sb] = s2 * exp(-1.0 * D);
  }
}

}  // namespace

int launch_kernel_matrix(gpr_ctx* ctx, const KParams& kp, const double* dX, int n,
                         const double* dXp, int m, int same, double* dK, int ldk) {
  if (dK == ctx->kup_ptr) ctx->kup_ptr = nullptr;  // (rebuilt in full)
  if (n <= 0 || (!same && m <= 0)) return 0;
  GPR_TRY(scale_inputs(ctx, kp, dX, n, &ctx->dxs, &ctx->xs_cap));
  if (same) {
    const double el = (double)n * n;
    TimerScope ts(ctx, TC_KBUILD, el * 8.0);  // "flops" slot carries algorithmic bytes
    // (the Gram kernels store 16-B pairs: 16-B aligned K with an even ldk, else difference form)
    // one SE part: both halves computed by the column build (store-bound: one exponential per
    // element is cheaper than the mirrored tiles' store pattern); more parts: upper tiles
    // computed once and mirrored through LDS (the exponentials dominate)
    if (gram_enabled(ctx, kp.d) && kp.nse <= 1)
      return kp.nse == 1 ? launch_gram_upper_s<1>(ctx, kp, ctx->dxs, n, dK, ldk, 1)
                         : launch_gram_upper_s<2>(ctx, kp, ctx->dxs, n, dK, ldk, 1);
    if (gram_enabled(ctx, kp.d) && vec_store_ok(dK, ldk))
      return launch_gram_any(ctx, kp, ctx->dxs, n, nullptr, n, 1, dK, ldk);
    DISPATCH_D(launch_sym, ctx, kp, ctx->dxs, n, dK, ldk);
    LAUNCH_CHECK(ctx);
  } else {
    GPR_TRY(scale_inputs(ctx, kp, dXp, m, &ctx->dxps, &ctx->xps_cap));
    TimerScope ts(ctx, TC_OTHER, 0.0);
    if (gram_enabled(ctx, kp.d) && vec_store_ok(dK, ldk))
      return launch_gram_any(ctx, kp, ctx->dxs, n, ctx->dxps, m, 0, dK, ldk);
    DISPATCH_D(launch_cross, ctx, kp, ctx->dxs, n, ctx->dxps, m, dK, ldk);
    LAUNCH_CHECK(ctx);
  }
  return 0;
}

int launch_kernel_matrix_for_factor(gpr_ctx* ctx, const KParams& kp, const double* dX, int n,
                                    double* dK, int ldk) {
  ctx->kup_ptr = nullptr;
  // upper-only where the tile-DAG will take exactly this matrix directly (potrf_core), with
  // the Gram form (d <= 20) and one or two SE parts; the full symmetric K otherwise
  const bool upper = ctx->kbuild_upper && n > 0 && gram_enabled(ctx, kp.d) && kp.nse <= 2 &&
                     dag_takes_whole(ctx, n, ldk, dK) && dag_shape_ok(n, ldk, dK);
  if (!upper) return launch_kernel_matrix(ctx, kp, dX, n, nullptr, n, 1, dK, ldk);
  GPR_TRY(scale_inputs(ctx, kp, dX, n, &ctx->dxs, &ctx->xs_cap));
  {
    // bytes written: column c gets min(n, 128 (c / 128 + 1)) rows
    double bytes = 0.0;
    for (int c0 = 0; c0 < n; c0 += 128) bytes += 8.0 * std::min(128, n - c0) * kup_rows(c0, n);
    TimerScope ts(ctx, TC_KBUILD, bytes);  // ("flops" slot: bytes written)
    GPR_TRY(kp.nse == 1 ? launch_gram_upper_s<1>(ctx, kp, ctx->dxs, n, dK, ldk, 0)
                        : launch_gram_upper_s<2>(ctx, kp, ctx->dxs, n, dK, ldk, 0));
  }
  ctx->kup_ptr = dK;
  ctx->kup_n = n;
  ctx->kup_ld = ldk;
  return 0;
}

int launch_scale_inputs(gpr_ctx* ctx, const KParams& kp, const double* dX, int n, double* out) {
  const size_t total = (size_t)kp.nse * kp.d * n;
  if (total == 0) return 0;
  int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  scale_inputs_kernel<<<blocks, 256, 0, ctx->stream>>>(kp, dX, n, out);
  LAUNCH_CHECK(ctx);
  return 0;
}

int launch_pair(gpr_ctx* ctx, int mode, int d, const double* xa, int na, const double* xb, int nb,
                double s2, double* out, size_t sa, size_t sb) {
  if (na <= 0 || nb <= 0) return 0;
  const size_t total = (size_t)na * nb;
  int blocks = (int)std::min<size_t>((total + 255) / 256, 65536);
  pair_kernel<<<blocks, 256, 0, ctx->stream>>>(mode, d, xa, na, xb, nb, s2, out, sa, sb,
                                               sa == 1 ? 1 : 0);
  LAUNCH_CHECK(ctx);
  return 0;
}

int launch_mirror_upper(gpr_ctx* ctx, double* A, int n, int lda) {
  if (n <= 1) return 0;
  const int nt = (n + KT - 1) / KT;
  const long long nblk = (long long)nt * (nt + 1) / 2;
  mirror_upper_kernel<<<(unsigned)nblk, 256, 0, ctx->stream>>>(A, n, (size_t)lda);
  LAUNCH_CHECK(ctx);
  return 0;
}

int launch_set_identity(gpr_ctx* ctx, double* A, int n, int lda) {
  int blocks = (int)std::min<long long>(((long long)n * n + 255) / 256, 8192);
  set_identity_kernel<<<blocks, 256, 0, ctx->stream>>>(A, n, (size_t)lda);
  LAUNCH_CHECK(ctx);
  return 0;
}

extern "C" {

int gpr_kernel(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
               const double* dX, int n, const double* dXp, int m, int same, double eps,
               double* dK, int ldk) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (!dX || !dK) return set_err(ctx, GPR_E_ARG, "NULL device pointer");
  if (n < 0) return set_err(ctx, GPR_E_ARG, "n < 0");
  if (same != GPR_CROSS && same != GPR_SELF && same != GPR_SAME_OBJECT)
    return set_err(ctx, GPR_E_ARG, "same=%d is not GPR_CROSS, GPR_SELF or GPR_SAME_OBJECT", same);
  if (same == GPR_SAME_OBJECT) kp.has_noise = 0;  // 5-arg x === xp: eps per SE part, no noise
  if (same) m = n;
  else if (!dXp) return set_err(ctx, GPR_E_ARG, "dXp is NULL for a cross kernel");
  if (ldk < (n > 1 ? n : 1)) return set_err(ctx, GPR_E_ARG, "ldk=%d < n=%d", ldk, n);
  return launch_kernel_matrix(ctx, kp, dX, n, dXp, m, same, dK, ldk);
}

int gpr_kernel_grad(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                    const double* dX, int n, int i, double eps, double* dDK, int ld) {
  KParams kp;
  int D = 0;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, &D));
  if (i < 1 || i > D) return set_err(ctx, GPR_E_ARG, "hp index %d out of 1..%d", i, D);
  if (ld < n) return set_err(ctx, GPR_E_ARG, "ld < n");
  // find_idx (src/compose_covar.jl:109-115)
  int off = 0, se = 0;
  for (int t = 0; t < nk; ++t) {
    const int w = kinds[t] == GPR_SE ? d + 1 : 1;
    if (i - 1 < off + w) {
      const int local = i - 1 - off;
      const int blocks = (int)std::min<long long>(((long long)n * n + 255) / 256, 8192);
      if (kinds[t] == GPR_WN) {  // grad(::WhiteNoise) = 2 sigma_n I  (src/deriv_covar.jl:31)
        diag_scaled_identity_kernel<<<blocks, 256, 0, ctx->stream>>>(dDK, n, (size_t)ld,
                                                                    2.0 * hp[off]);
        LAUNCH_CHECK(ctx);
        return 0;
      }
      GPR_TRY(scale_inputs(ctx, kp, dX, n, &ctx->dxs, &ctx->xs_cap));
      kgrad_kernel<<<blocks, 256, 0, ctx->stream>>>(kp, dX, ctx->dxs, n, se, local, dDK,
                                                    (size_t)ld);
      LAUNCH_CHECK(ctx);
      return 0;
    }
    off += w;
    if (kinds[t] == GPR_SE) ++se;
  }
  return set_err(ctx, GPR_E_ARG, "hp index not found");
}

}  // extern "C"
