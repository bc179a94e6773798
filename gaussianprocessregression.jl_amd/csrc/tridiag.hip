// Symmetric tridiagonal reduction, hand-written for gfx950: the first stage of LAPACK's syevr
// (dsytrd) behind the sample_noise quadrature (src/integrate.jl:71-100, LAPACK.syevr! at :75).
//
//   A = Q T Q^T,  T = tridiag(e, d, e),  Q = H_0 H_1 ... H_{n-3},  H_j = I - tau_j v_j v_j^T
//
// (v_j lives on rows j+1..n-1 with v_j[j+1] = 1; dlarfg's reflector conventions).  The
// quadrature never needs an eigenvector: k1' (K + s I)^{-1} y = (Q^T k1)' (T + s I)^{-1} (Q^T y),
// so after the reduction every column costs one O(n) tridiagonal solve (any shift: Gaussian
// elimination with partial pivoting, dgtsv), and gpr_syev_apply's eigendecomposition
// continues from T with the divide-and-conquer solver (dstedc.hip).
//
// The reduction: ONE persistent launch of P workgroups (~16 columns each, at most one per CU),
// the unblocked two-sided Householder algorithm (dsytd2) on a full symmetric work copy,
// columns dealt round-robin (column c to workgroup c mod P: contiguous, coalesced).  Step j,
// with v_j, tau_j and (j > 0) v_{j-1}, w_{j-1} in every workgroup's LDS:
//   * the pass: every workgroup, over its columns c > j, applies step j-1's rank-2 update
//     A(:, c) -= v_{j-1} w_{j-1}[c] + w_{j-1} v_{j-1}[c] and forms p_j[c] = tau_j A(:, c) . v_j
//     (each column read once and written once, 16-B accesses, 8-16 row pairs in flight per lane);
//     the owner of column j + 1 also publishes that column;
//   * one exchange: each workgroup publishes p_j[c] and its part of p_j . v_j; every
//     workgroup then reads p_j, the partial sums and column j + 1 -- each of them polled until
//     its writer's store has landed (the buffers hold a sentinel until written, so every value
//     is its own arrival flag: no counter, no drain before an arrival) -- and forms w_j =
//     p_j - (tau_j / 2)(p_j . v_j) v_j, column j + 1 after step j and the next reflector
//     (dlarfg) ITSELF -- the same bits everywhere, so no second hop.
// Hand-offs are sc1 (write-through stores, sc1 loads), every handed-off address written once
// per launch (p_j, column j + 1, the partial sums each have their own slot).  Every wait is
// bounded: on a time-out the launch drains and the call reports an error.
//
// Cost per step: the store-to-load latency of one hand-off plus 2 (n - j) + P sc1 loads per
// workgroup, and the pass (16 (n - j)^2 / P bytes per workgroup; the work copy stays in the
// Infinity Cache up to n ~ 4k).
//
// Variants by n: up to TRD_DF_MIN the step vectors sit in LDS (sytrd_kernel<.., GV = false>);
// from TRD_DF_MIN on the updates are deferred by panels of DF_NB steps (sytrd_df_kernel: later
// columns only read per step and corrected, flushed per panel by an MFMA GEMM -- 8 instead of
// 16 (n - j)^2 bytes per step); the per-step global-vector variant (GV = true) remains for
// grids the DF variant does not cover (more than DF_MAXP workgroups or 16 DF_MAXCT columns each).
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace {

constexpr int TRD_THREADS = 512;   // 8 waves: one column per wave at a time
constexpr int TRD_WAVES = TRD_THREADS / 64;
constexpr int TRD_MAXN = 6144;     // 3 LDS vectors of n doubles per workgroup
constexpr int TRD_MAXN_G = 16384;  // beyond TRD_MAXN: the vectors in global memory (GV)
constexpr int TRD_FUSED_M = 1024;  // right-hand sides transformed inside the launch

constexpr int RPT = (TRD_MAXN + TRD_THREADS - 1) / TRD_THREADS;      // rows per thread, one column
constexpr int RPT_G = (TRD_MAXN_G + TRD_THREADS - 1) / TRD_THREADS;  // (the GV variant's)

__device__ __forceinline__ double ld1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld1i(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1i(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the exchange buffers' "not yet written" value: a signalling-NaN payload that no arithmetic
// produces (results are quiet NaNs) -- set before every launch, each address written once
constexpr unsigned long long TRD_UNSET = 0x7FF4D1A60000BEEFull;
__device__ __forceinline__ int trd_unset(double v) {
  return __double_as_longlong(v) == (long long)TRD_UNSET;
}
__global__ void trd_fill_unset_kernel(double* __restrict__ p, size_t cnt) {
  const double u = __longlong_as_double((long long)TRD_UNSET);
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < cnt;
       t += (size_t)gridDim.x * blockDim.x)
    p[t] = u;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Late-wave injection (test build only, GPR_TRD_DELAY = d > 0): at each site, one wave in three
// (rotating with the site, the step and the workgroup) sleeps d x ~8k cycles.  Placed before the
// reads that follow a single-thread / single-wave LDS write and before each hand-off poll, it
// forces the schedules in which a reader is late (or a writer is), so a missing barrier or
// flag shows as a wrong result instead of depending on timing.  (It exposes the round-5 dlarfg
// alpha race deterministically: waves reading alpha after thread 0 replaced it by v's 1.)
#ifdef GPR_TESTING
#define TRD_DELAY(site)                                                                 \
  do {                                                                                  \
    if (a.delay > 0 && ((int)blockIdx.x + (int)(threadIdx.x >> 6) + (site) + j) % 3 == 0) \
      for (int q_ = 0; q_ < a.delay; ++q_) __builtin_amdgcn_s_sleep(127);              \
  } while (0)
#else
#define TRD_DELAY(site) \
  do {                  \
  } while (0)
#endif

#ifdef GPR_TESTING
// phase stamps of workgroups 0 and P-1 (test build only: tools/trd_trace.py)
__device__ long long g_trd_trace[2][TRD_MAXN][6];
// every workgroup's pass start / pass end at every 64th step (the spread across workgroups)
__device__ long long g_trd_wg[TRD_MAXN / 64][256][2];
// every workgroup's XCD (HW_REG_XCC_ID), recorded at the first step
__device__ int g_trd_xcc[256];
#define TRD_XCCSTAMP()                                                          \
  do {                                                                          \
    if (tid == 0 && j == 0 && w < 256) {                                        \
      int x_;                                                                   \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x_));   \
      g_trd_xcc[w] = x_;                                                        \
    }                                                                           \
  } while (0)
#define TRD_WGSTAMP(k)                                                                      \
  do {                                                                                      \
    if (tid == 0 && j >= a.wgoff && ((j - a.wgoff) & 63) == 0 && w < 256 && j < TRD_MAXN)  \
      g_trd_wg[(j - a.wgoff) >> 6][w][k] = (long long)__builtin_amdgcn_s_memrealtime();     \
  } while (0)
// (DF's exchange phase split: after the row chunks, after the reflector -- [2][TRD_MAXN][2])
__device__ long long g_trd_trace2[2][TRD_MAXN][2];
#define TRD_STAMP2(k)                                                                   \
  do {                                                                                  \
    if (tid == 0 && (w == 0 || w == P - 1) && j < TRD_MAXN)                             \
      g_trd_trace2[w == 0 ? 0 : 1][j][k] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TRD_STAMP(k)                                                                   \
  do {                                                                                 \
    if (tid == 0 && (w == 0 || w == P - 1) && j < TRD_MAXN)                            \
      g_trd_trace[w == 0 ? 0 : 1][j][k] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define TRD_STAMP(k) \
  do {               \
  } while (0)
#define TRD_WGSTAMP(k) \
  do {                 \
  } while (0)
#define TRD_STAMP2(k) \
  do {                \
  } while (0)
#define TRD_XCCSTAMP() \
  do {                 \
  } while (0)
#endif

struct TrdArgs {
  double* A;        // n x n work copy (full symmetric), ld lda; columns updated in place
  size_t lda;
  int n, P, ldl;    // ldl: stride of the LDS vectors (n rounded up to 2)
  double* V;        // n x n (ld lda): column j = v_j on rows j+1..n-1 (v_j[j+1] = 1)
  double* cpub;     // n x n (ld lda): column j + 1 after step j - 1, published by its owner
  double* pbuf;     // n x n (ld lda): column j = p_j
  double* parts;    // n x P partial sums p_j . v_j
  double* tau;      // n (tau[n-2], tau[n-1] = 0)
  double* d;        // n: diagonal of T
  double* e;        // n - 1: off-diagonal of T
  double* dlast;    // A(n-1, n-1) after step n - 4's update (from the owner of column n-1)
  int* err;         // set on a wait time-out: every wait then gives up
  long long spin_limit;
#ifdef GPR_TESTING
  int fail_step;    // (test build) workgroup 0 never publishes its partial sum of this step
  int delay;        // (test build) GPR_TRD_DELAY: late-wave injection, see trd_delay
  int wgoff;        // (test build) GPR_TRD_WGOFF: the per-workgroup stamps at steps wgoff + 64 k
#endif
  double* B;        // optional n x m (ld ldb): B <- H_j B at step j (column c to workgroup c mod P)
  size_t ldb;
  int m;
  // GV variant (n > TRD_MAXN): step j's vectors in global memory instead of LDS, shared by all
  // workgroups -- v_j in V's column j (every workgroup writes the same bits there), w_j and
  // column j + 1 after step j in rings of 4 columns (ld lda): wr[(j & 3) lda], xr[(j & 3) lda]
  double* wr;
  double* xr;
  // DF variant (deferred updates, sytrd_df_kernel): w_k in Wv's column k (every workgroup writes
  // the same bits), the panel's dot-product partials in abuf (n x 2 DF_NB x P, each written once),
  // deferred panels for steps j < jt, ncl = ceil(n / P) columns per workgroup
  double* Wv;
  double* abuf;
  int jt, ncl;
};

// workgroup sum of one value per thread (red: >= TRD_WAVES doubles of LDS), deterministic: the
// same inputs give the same bits in every workgroup
__device__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < TRD_WAVES; ++q) s += red[q];
  __syncthreads();
  return s;
}

// dlarfg on col[j+1..n-1] in place -> v_j (v_j[j+1] = 1); returns tau_j, *beta = e_j.  Every
// workgroup computes the same bits (the reflector is formed redundantly everywhere).
// (src == dst: in place, LDS; the GV variant reads A's column and writes V's, since another
// workgroup may still be writing the same source values while this one scales them)
__device__ double trd_reflector(int n, int j, const double* col, double* dst, double* red,
                                double* beta_out) {
  // (alpha is read before block_sum's barriers: thread 0 overwrites col[j+1] below, and a wave
  // still to read it after that write would form a different reflector)
  const double alpha = col[j + 1];
  double s = 0.0;
  for (int r = j + 2 + threadIdx.x; r < n; r += TRD_THREADS) s += col[r] * col[r];
  const double xnorm2 = block_sum(s, red);
  double tau = 0.0, beta = alpha, scal = 0.0;
  if (xnorm2 > 0.0) {
    beta = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
  }
  for (int r = j + 1 + threadIdx.x; r < n; r += TRD_THREADS) dst[r] = r == j + 1 ? 1.0 : col[r] * scal;
  __syncthreads();
  *beta_out = beta;
  return tau;
}

// Poll K handed-off values until none holds the sentinel in the whole workgroup (src[k] ==
// nullptr: inactive).  Bounded like the LDS variant's loop: false on a time-out here or
// elsewhere (the caller then ends the workgroup).
constexpr int TRD_GCH = 4;  // GV exchange: rows per thread per chunk
template <int K>
__device__ bool trd_poll(const TrdArgs& a, int n, int j, int* s_ok, double (&v)[K],
                         const double* const (&src)[K]) {
  const int tid = threadIdx.x;
  for (long long spins = 0;; ++spins) {
    int miss = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) miss |= src[k] != nullptr && trd_unset(v[k]);
    if (!__syncthreads_or(miss)) return true;
    if ((spins & 63) == 63) {
      if (tid == 0) {
        if (spins > a.spin_limit) st1i(a.err, 1);
        *s_ok = ld1i(a.err) == 0;
      }
      __syncthreads();
      const bool ok = *s_ok != 0;
      __syncthreads();
      if (!ok) return false;
    }
    if (n - j > 2048) __builtin_amdgcn_s_sleep(31);
    else __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (src[k] != nullptr && trd_unset(v[k])) v[k] = ld1(src[k]);
  }
}

// trd_poll without pointer arrays (registers): v[k] = base[k * stride] for k < cnt (cnt <= K;
// the rest inactive)
template <int K>
__device__ bool trd_poll_strided(const TrdArgs& a, int n, int j, int* s_ok, double (&v)[K],
                                 const double* base, int stride, int cnt) {
  const int tid = threadIdx.x;
  for (long long spins = 0;; ++spins) {
    int miss = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) miss |= k < cnt && trd_unset(v[k]);
    if (!__syncthreads_or(miss)) return true;
    if ((spins & 63) == 63) {
      if (tid == 0) {
        if (spins > a.spin_limit) st1i(a.err, 1);
        *s_ok = ld1i(a.err) == 0;
      }
      __syncthreads();
      const bool ok = *s_ok != 0;
      __syncthreads();
      if (!ok) return false;
    }
    if (n - j > 2048) __builtin_amdgcn_s_sleep(31);
    else __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < cnt && trd_unset(v[k])) v[k] = ld1(base + (size_t)k * stride);
  }
}

// the exchange's row chunks: v[2k] = p0[r_k], v[2k+1] = p1[r_k], r_k = rb + k TRD_THREADS
// (rows >= n inactive)
template <int G>
__device__ bool trd_poll_rows(const TrdArgs& a, int n, int j, int* s_ok, double (&v)[2 * G],
                              const double* p0, const double* p1, int rb) {
  const int tid = threadIdx.x;
  for (long long spins = 0;; ++spins) {
    int miss = 0;
#pragma unroll
    for (int k = 0; k < G; ++k)
      miss |= rb + k * TRD_THREADS < n && (trd_unset(v[2 * k]) | trd_unset(v[2 * k + 1]));
    if (!__syncthreads_or(miss)) return true;
    if ((spins & 63) == 63) {
      if (tid == 0) {
        if (spins > a.spin_limit) st1i(a.err, 1);
        *s_ok = ld1i(a.err) == 0;
      }
      __syncthreads();
      const bool ok = *s_ok != 0;
      __syncthreads();
      if (!ok) return false;
    }
    if (n - j > 2048) __builtin_amdgcn_s_sleep(31);
    else __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int r = rb + k * TRD_THREADS;
      if (r < n) {
        if (trd_unset(v[2 * k])) v[2 * k] = ld1(p0 + r);
        if (trd_unset(v[2 * k + 1])) v[2 * k + 1] = ld1(p1 + r);
      }
    }
  }
}

// Step j's state, identical in every workgroup: vcur = v_j, tau_j; (j > 0) vprev = v_{j-1},
// wprev = w_{j-1}.  One exchange per step: the pass publishes p_j (and the owner of column
// j + 1 that column), every workgroup then forms w_j, column j + 1 and v_{j+1} itself.
// PU: row pairs in flight per lane in the pass (16 from n ~ 800 on: 1-3 % faster at n = 1100-
// 4096; 8 below, where the extra registers cost more than they hide).  RP: rows per thread of
// the exchange (RPT, RPT_G).  GV: the step's vectors in global memory (n > TRD_MAXN, see TrdArgs;
// every workgroup writes the same bits, and reads a location only after its own write of it has
// completed -- workgroup barrier -- so what it reads is its own value)
template <int PU, int RP, bool GV>
__global__ __launch_bounds__(TRD_THREADS, 1) void sytrd_kernel(TrdArgs a) {
  extern __shared__ double lds[];
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int n = a.n, P = a.P, w = blockIdx.x, L = a.ldl;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // (GV: one LDS vector, v_j -- the most read of the three: the pass's dot, the exchange, the B
  // application -- beside the shared global copies of v_{j-1} and w_{j-1})
  double* red = GV ? lds + L : lds + 3 * (size_t)L;
  int* s_ok = reinterpret_cast<int*>(red + TRD_WAVES);
  double* s_alpha = red + TRD_WAVES + 1;  // column j+1's entry j+2 after step j (dlarfg's alpha)
  int ivp = 0, iwp = 1, ivc = 2;
  double tj;

  {  // v_0 from column 0 (no update before it), redundantly in every workgroup
    double beta;
    double d0;
    const int j = 0;
    (void)j;
    TRD_DELAY(0);  // (a late wave reading dlarfg's alpha)
    if (GV) {  // column 0 of the work copy is never updated: read it in place, write V's
      d0 = a.A[0];
      tj = trd_reflector(n, 0, a.A, a.V, red, &beta);
      for (int r = 1 + tid; r < n; r += TRD_THREADS) lds[r] = a.V[r];  // (own writes, after
      __syncthreads();                                                 //  the reflector's barrier)
    } else {
      double* c = lds + (size_t)ivc * L;
      for (int r = tid; r < n; r += TRD_THREADS) c[r] = a.A[r];
      __syncthreads();
      d0 = c[0];
      tj = trd_reflector(n, 0, c, c, red, &beta);
      if (w == 0)
        for (int r = 1 + tid; r < n; r += TRD_THREADS) a.V[r] = c[r];
    }
    if (w == 0 && tid == 0) {
      a.d[0] = d0;
      a.e[0] = beta;
      a.tau[0] = tj;
    }
  }

  for (int j = 0; j <= n - 3; ++j) {
    // (GV, j = 0: v_{-1} and w_{-1} are never used -- the update is skipped -- but the pass
    // still loads them: point them at v_0, which exists)
    const double* vprev = GV ? a.V + (size_t)(j > 0 ? j - 1 : 0) * a.lda : lds + (size_t)ivp * L;
    const double* wprev = GV ? (j > 0 ? a.wr + (size_t)((j - 1) & 3) * a.lda : a.V)
                             : lds + (size_t)iwp * L;
    const double* vcur = GV ? lds : lds + (size_t)ivc * L;
    // ---- the pass over this workgroup's columns c > j, one wave per column: rows from the
    // even r0 <= j + 1 (16-B accesses; row j, when included, is never read again), PU row pairs
    // in flight per lane
    TRD_STAMP(0);
    TRD_WGSTAMP(0);
    TRD_XCCSTAMP();
    double sp = 0.0;
    const int r0 = (j + 1) & ~1;
    int c0 = w + ((j + 1 - w + P - 1) / P) * P;  // first owned column > j
    if (c0 == j + 1) {
      // column j + 1 (its owner): the whole workgroup, rows split over the threads -- updated,
      // written, published, dotted -- before the other columns (one wave on it, with its
      // publishing stores, made this workgroup the step's straggler: 49.6 against a median
      // 37.6 us at n = 4096, profiles/r06_trd_wg_lds_4096.txt)
      double* col = a.A + (size_t)c0 * a.lda;
      double* pub = a.cpub + (size_t)(j + 1) * a.lda;
      const double wc = j > 0 ? wprev[c0] : 0.0, vc = j > 0 ? vprev[c0] : 0.0;
      double dot = 0.0;
      for (int rb = r0 + 2 * tid; rb < n; rb += 8 * TRD_THREADS) {
        d2 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + 2 * TRD_THREADS * u;
          if (r < n) x[u] = *reinterpret_cast<const d2*>(col + r);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + 2 * TRD_THREADS * u;
          if (r < n) {
            const d2 vv = *reinterpret_cast<const d2*>(vcur + r);
            if (j > 0) {
              const d2 vp = *reinterpret_cast<const d2*>(vprev + r);
              const d2 wp = *reinterpret_cast<const d2*>(wprev + r);
              x[u].x -= vp.x * wc + wp.x * vc;
              x[u].y -= vp.y * wc + wp.y * vc;
              *reinterpret_cast<d2*>(col + r) = x[u];
            }
            st1(pub + r, x[u].x);
            st1(pub + r + 1, x[u].y);
            dot += (r >= j + 1 ? x[u].x * vv.x : 0.0) + (r + 1 < n ? x[u].y * vv.y : 0.0);
          }
        }
      }
      const double p = tj * block_sum(dot, red);
      if (tid == 0) st1(&a.pbuf[(size_t)j * a.lda + c0], p);
      if (wv == 0) sp += p * vcur[c0];
      c0 += P;
    }
    for (int c = c0 + wv * P; c < n; c += TRD_WAVES * P) {
      double* col = a.A + (size_t)c * a.lda;
      const double wc = j > 0 ? wprev[c] : 0.0, vc = j > 0 ? vprev[c] : 0.0;
      double* pub = nullptr;  // (column j + 1: above)
      double dot = 0.0;
      for (int rb = r0 + 2 * lane; rb < n; rb += PU * 128) {
        d2 x[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          const int r = rb + 128 * u;
          if (r < n) x[u] = *reinterpret_cast<const d2*>(col + r);
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          const int r = rb + 128 * u;
          if (r < n) {
            const d2 vp = *reinterpret_cast<const d2*>(vprev + r);
            const d2 wp = *reinterpret_cast<const d2*>(wprev + r);
            const d2 vv = *reinterpret_cast<const d2*>(vcur + r);
            if (j > 0) {
              x[u].x -= vp.x * wc + wp.x * vc;
              x[u].y -= vp.y * wc + wp.y * vc;
              *reinterpret_cast<d2*>(col + r) = x[u];
            }
            if (pub) {
              st1(pub + r, x[u].x);
              st1(pub + r + 1, x[u].y);
            }
            if (c == n - 1 && j == n - 3) {  // A(n-1, n-1) for the last 2 x 2 block
              if (r == n - 1) st1(a.dlast, x[u].x);
              if (r + 1 == n - 1) st1(a.dlast, x[u].y);
            }
            // (row j and, for odd n, the padding row n are outside v_j's support)
            dot += (r >= j + 1 ? x[u].x * vv.x : 0.0) + (r + 1 < n ? x[u].y * vv.y : 0.0);
          }
        }
      }
      const double p = tj * wave_sum(dot);
      if (lane == 0) st1(&a.pbuf[(size_t)j * a.lda + c], p);
      sp += p * vcur[c];
    }
    // ---- publish this workgroup's part of p_j . v_j (no arrival counter: every handed-off
    // value is its own flag, see the exchange)
    TRD_STAMP(1);
    TRD_DELAY(1);  // (a late writer of the wave partial sums)
    if (lane == 0) red[wv] = sp;
    __syncthreads();
    TRD_WGSTAMP(1);  // (every wave's pass done)
    if (tid == 0) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < TRD_WAVES; ++q) s += red[q];
#ifdef GPR_TESTING
      if (!(j == a.fail_step && w == 0))
#endif
        st1(&a.parts[(size_t)j * P + w], s);
    }
    __syncthreads();
    // ---- Q^T B on the fly, inside the wait for the other workgroups: H_j applied to this
    // workgroup's columns of B (v_j is in every workgroup's LDS, so no exchange), b -= tau_j
    // (v_j . b) v_j on rows j+1..n-1.  A few columns: each by the whole workgroup (read once
    // into registers, written once); four or more: one wave per column.
    if (a.m > w) {
      const int mine = (a.m - w + P - 1) / P;
      if (mine < 4) {
        for (int c = w; c < a.m; c += P) {
          double* b = a.B + (size_t)c * a.ldb;
          if constexpr (GV) {  // (no register copy of the column: it would spill; read b twice)
            double dot = 0.0;
            for (int r = j + 1 + tid; r < n; r += TRD_THREADS) dot += b[r] * vcur[r];
            const double f = tj * block_sum(dot, red);
            for (int r = j + 1 + tid; r < n; r += TRD_THREADS) b[r] -= f * vcur[r];
            continue;
          }
          double x[RP];
          double dot = 0.0;
#pragma unroll
          for (int k = 0; k < RP; ++k) {
            const int r = j + 1 + tid + k * TRD_THREADS;
            x[k] = r < n ? b[r] : 0.0;
            dot += r < n ? x[k] * vcur[r] : 0.0;
          }
          const double f = tj * block_sum(dot, red);
#pragma unroll
          for (int k = 0; k < RP; ++k) {
            const int r = j + 1 + tid + k * TRD_THREADS;
            if (r < n) b[r] = x[k] - f * vcur[r];
          }
        }
      } else {
        for (int c = w + wv * P; c < a.m; c += TRD_WAVES * P) {
          double* b = a.B + (size_t)c * a.ldb;
          double dot = 0.0;
          for (int rb = j + 1 + lane; rb < n; rb += 4 * 64) {
            double x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = rb + 64 * u < n ? b[rb + 64 * u] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (rb + 64 * u < n) dot += x[u] * vcur[rb + 64 * u];
          }
          const double f = tj * wave_sum(dot);
          for (int r = j + 1 + lane; r < n; r += 64) b[r] -= f * vcur[r];
        }
      }
    }
    TRD_STAMP(2);
    // ---- the exchange: p_j, the published column j + 1 and the P partial sums.  Every one of
    // these addresses is written once per launch and holds the sentinel until then, so each
    // value is its own arrival flag: all loads are issued at once, and only values still
    // holding the sentinel are loaded again (sc1), until none is left in the workgroup.
    double* wnew = GV ? a.wr + (size_t)(j & 3) * a.lda : lds + (size_t)ivp * L;  // (v_{j-1}'s slot)
    double* cnew = GV ? a.xr + (size_t)(j & 3) * a.lda : lds + (size_t)iwp * L;  // (w_{j-1}'s) -> v_{j+1}
    // v_{j+1}'s destination: in place in LDS; V's column j + 1 for GV (not in place: a slower
    // workgroup may still be writing column j + 1's values into the ring slot)
    double* vnext = GV ? a.V + (size_t)(j + 1) * a.lda : cnew;
    const double* pj = a.pbuf + (size_t)j * a.lda;
    const double* cp = a.cpub + (size_t)(j + 1) * a.lda;
    const double* pp = a.parts + (size_t)j * P;
    TRD_DELAY(2);  // (workgroups arriving late at the exchange: the sentinel protocol)
    double xn = 0.0;
    if constexpr (!GV) {
      double pr[RP], cr[RP];
#pragma unroll
      for (int k = 0; k < RP; ++k) {
        const int r = j + 1 + tid + k * TRD_THREADS;
        pr[k] = r < n ? ld1(&pj[r]) : 0.0;
        cr[k] = r < n ? ld1(&cp[r]) : 0.0;
      }
      double pc = ld1(&pj[j + 1]);
      double pq = tid < P ? ld1(&pp[tid]) : 0.0;
      for (long long spins = 0;; ++spins) {
        int miss = trd_unset(pc) | trd_unset(pq);
#pragma unroll
        for (int k = 0; k < RP; ++k) miss |= trd_unset(pr[k]) | trd_unset(cr[k]);
        if (!__syncthreads_or(miss)) break;
        if ((spins & 63) == 63) {  // bounded: a time-out here or elsewhere ends every workgroup
          if (tid == 0) {
            if (spins > a.spin_limit) st1i(a.err, 1);
            *s_ok = ld1i(a.err) == 0;
          }
          __syncthreads();
          const bool ok = *s_ok != 0;
          __syncthreads();
          if (!ok) return;
        }
        // long steps (workgroups arrive microseconds apart): poll less often, so the early
        // arrivals' re-loads leave the memory system to the passes still streaming
        if (n - j > 2048) __builtin_amdgcn_s_sleep(31);
        else __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < RP; ++k) {
          const int r = j + 1 + tid + k * TRD_THREADS;
          if (trd_unset(pr[k])) pr[k] = ld1(&pj[r]);
          if (trd_unset(cr[k])) cr[k] = ld1(&cp[r]);
        }
        if (trd_unset(pc)) pc = ld1(&pj[j + 1]);
        if (trd_unset(pq)) pq = ld1(&pp[tid]);
      }
      TRD_STAMP(3);
      const double kj = 0.5 * tj * block_sum(pq, red);
      TRD_STAMP(4);
      const double wc = pc - kj * vcur[j + 1], vc = vcur[j + 1];
#pragma unroll
      for (int k = 0; k < RP; ++k) {
        const int r = j + 1 + tid + k * TRD_THREADS;
        if (r < n) {
          const double wr = pr[k] - kj * vcur[r];
          const double x = cr[k] - (vcur[r] * wc + wr * vc);
          wnew[r] = wr;
          cnew[r] = x;
          if (r >= j + 3) xn += x * x;
          if (r == j + 2) *s_alpha = x;
        }
      }
    } else {
      // GV (n > TRD_MAXN): the same exchange in chunks of TRD_GCH rows per thread (all of a
      // column's rows in registers at once would spill): the partial sums and p_j[j + 1] first
      // (w_j needs their sum), then each chunk of p_j and column j + 1 polled and consumed
      double pv[2] = {ld1(&pj[j + 1]), tid < P ? ld1(&pp[tid]) : 0.0};
      const double* ps[2] = {&pj[j + 1], tid < P ? &pp[tid] : nullptr};
      if (!trd_poll<2>(a, n, j, s_ok, pv, ps)) return;
      TRD_STAMP(3);
      const double kj = 0.5 * tj * block_sum(pv[1], red);
      TRD_STAMP(4);
      const double wc = pv[0] - kj * vcur[j + 1], vc = vcur[j + 1];
      for (int k0 = 0; j + 1 + k0 * TRD_THREADS < n; k0 += TRD_GCH) {  // (uniform bound)
        double xv[2 * TRD_GCH];
        const double* xs[2 * TRD_GCH];
#pragma unroll
        for (int k = 0; k < TRD_GCH; ++k) {
          const int r = j + 1 + tid + (k0 + k) * TRD_THREADS;
          xs[2 * k] = r < n ? &pj[r] : nullptr;
          xs[2 * k + 1] = r < n ? &cp[r] : nullptr;
          xv[2 * k] = r < n ? ld1(&pj[r]) : 0.0;
          xv[2 * k + 1] = r < n ? ld1(&cp[r]) : 0.0;
        }
        if (!trd_poll<2 * TRD_GCH>(a, n, j, s_ok, xv, xs)) return;
#pragma unroll
        for (int k = 0; k < TRD_GCH; ++k) {
          const int r = j + 1 + tid + (k0 + k) * TRD_THREADS;
          if (r < n) {
            const double wr = xv[2 * k] - kj * vcur[r];
            const double x = xv[2 * k + 1] - (vcur[r] * wc + wr * vc);
            wnew[r] = wr;
            cnew[r] = x;
            if (r >= j + 3) xn += x * x;
            if (r == j + 2) *s_alpha = x;
          }
        }
      }
    }
    const double xnorm2 = block_sum(xn, red);  // (its barriers publish cnew / wnew)
    const bool out = w == (j + 1) % P;         // (one workgroup writes T and V)
    if (out && tid == 0) a.d[j + 1] = cnew[j + 1];
    if (j + 1 <= n - 3) {
      // dlarfg on cnew[j+2..n-1] -> v_{j+1} in place
      // alpha from its own LDS slot, not cnew[j + 2]: thread 0 overwrites that entry with v's
      // leading 1 below, possibly before another wave has read it (no barrier in between)
      TRD_DELAY(3);  // (a late reader of alpha, after another wave's v stores)
      const double alpha = *s_alpha;
      double tau = 0.0, beta = alpha, scal = 0.0;
      if (xnorm2 > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
        tau = (beta - alpha) / beta;
        scal = 1.0 / (alpha - beta);
      }
      double* vj = a.V + (size_t)(j + 1) * a.lda;
      for (int r = j + 2 + tid; r < n; r += TRD_THREADS) {
        const double v = r == j + 2 ? 1.0 : cnew[r] * scal;
        vnext[r] = v;
        if (GV) lds[r] = v;  // (v_j's reads in this step all precede block_sum's barriers)
        if (out && !GV) vj[r] = v;
      }
      if (out && tid == 0) {
        a.e[j + 1] = beta;
        a.tau[j + 1] = tau;
      }
      tj = tau;
      TRD_DELAY(4);  // (a late writer of v_{j+1} before the next pass reads it)
      __syncthreads();
    } else if (out && tid == 0) {  // the last 2 x 2 block: e_{n-2}, d_{n-1}
      a.e[n - 2] = cnew[n - 1];
      double dl = ld1(a.dlast);  // (written in the last pass by column n-1's owner: polled too)
      for (long long spins = 0; trd_unset(dl) && spins <= a.spin_limit; ++spins) {
        __builtin_amdgcn_s_sleep(1);
        dl = ld1(a.dlast);
      }
      if (trd_unset(dl)) st1i(a.err, 1);
      a.d[n - 1] = dl - 2.0 * vcur[n - 1] * wnew[n - 1];
    }
    TRD_STAMP(5);
    const int t = ivp;
    ivp = ivc;
    ivc = iwp;
    iwp = t;
  }
}

// ---- DF: the reduction with deferred updates (n >= TRD_DF_MIN) ----------------------------
// The pass above reads AND writes every trailing column every step (16 (n - j)^2 bytes): at n =
// 8192 that is ~75 % of the launch, at ~4 TB/s.  DF applies the rank-2 updates by panels of
// DF_NB steps instead (LAPACK's dlatrd idea, inside the same persistent launch):
//   * step j of a panel [j0, j0 + DF_NB): the columns the panel will publish, (j, j0 + DF_NB], are
//     kept up to date as before (eager: read, update, write -- each by its owner's whole
//     workgroup, so no owner becomes the step's straggler); every later column is only READ,
//     A(:, c) . v_j, and corrected by the panel's pending updates
//        p_j[c] = tau_j (A(:, c) . v_j - sum_k (w_k[c] alpha_k + v_k[c] beta_k)),
//        alpha_k = v_k . v_j,  beta_k = w_k . v_j  (k = j0 .. j - 1);
//     v_k[c] and w_k[c] at the workgroup's own columns are kept in LDS as they appear, and the
//     dots are summed from per-workgroup partials over those same indices (all columns of all
//     workgroups cover every row), published when v_j is formed at the end of step j - 1 and
//     polled only after this step's column reads -- long arrived, so no second hop's latency;
//   * the panel's first step (j = j0 > 0) flushes the previous panel: every column c > j gets its
//     DF_NB updates A(r, c) -= sum_k v_k[r] w_k[c] + w_k[r] v_k[c] at once (a K = 2 DF_NB GEMM on
//     the FP64 MFMA, waves splitting the rows), is written once and dotted with v_j;
//   * the last steps (j >= jt, n - jt ~ DF_TAIL) update every column every step, as above.
// Column bytes per step: 8 (n - j)^2 read, plus 16 (n - j)^2 per DF_NB steps for the flush.
// Column j + 1 after step j is formed in LDS (over v_j, once read), w_j goes to Wv's column j.
constexpr int DF_NB = 16;      // updates per panel (the flush: 2 DF_NB registers per row)
constexpr int DF_TAIL = 1024;  // steps at the end with every update applied at once
constexpr int DF_MAXP = 256;   // workgroups (the partials' poll: 16 per thread)
constexpr int DF_MAXCT = 4;    // the flush's column tiles of 16: ncl <= 64 (n <= 16384 at P = 256)
// DF from here on: faster than the LDS variant from n ~ 5400 (profiles/r06_trd_df_vs_lds.txt,
// with the LDS variant's column j + 1 by the whole workgroup: 5632 186.3 vs 190.5 ms, 6144 224.5
// vs 240.8; 5120 153.6 vs 150.0, 4608 124.9 vs 116.0 -- below, the work copy stays in the
// Infinity Cache and the per-step passes are cheap)
constexpr int TRD_DF_MIN = 5376;
constexpr int DF_GCH = 8;  // DF exchange: rows per thread per chunk

__global__ __launch_bounds__(TRD_THREADS, 1) void sytrd_df_kernel(TrdArgs a) {
  extern __shared__ double lds[];
  typedef double d2 __attribute__((ext_vector_type(2)));
  constexpr int PU = 8;  // (16 spills here: 8 row pairs per lane, 64 KB in flight per CU)
  const int n = a.n, P = a.P, w = blockIdx.x, L = a.ldl, ncl = a.ncl;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double* red = lds + L;  // lds[0, n): v_j, then (the exchange) column j + 1 after step j
  int* s_ok = reinterpret_cast<int*>(red + TRD_WAVES);
  double* s_alpha = red + TRD_WAVES + 1;  // column j+1's entry j+2 after step j (dlarfg's alpha)
  double* s_d = red + TRD_WAVES + 2;      // its entry j+1 (d_{j+1})
  double* s_cl = red + TRD_WAVES + 3;     // its entry n-1 at the last step (e_{n-2})
  double* vown = red + TRD_WAVES + 4;     // [DF_NB][ncl]: v_k at this workgroup's columns
  double* wown = vown + DF_NB * ncl;      // [DF_NB][ncl]: w_k there
  double* qraw = wown + DF_NB * ncl;      // [ncl]: later columns' A(:, c) . v_j
  double* qpart = qraw + ncl;             // [TRD_WAVES][ncl]: the flush's per-wave dots
  double* ab = qpart + TRD_WAVES * ncl;   // [2 DF_NB]: alpha_k, beta_k interleaved
  const double* vcur = lds;
  double tj;

  {  // v_0 from column 0 (never updated: read in place, V's column 0 written by every workgroup)
    double beta;
    const int j = 0;
    (void)j;
    TRD_DELAY(0);
    const double d0 = a.A[0];
    tj = trd_reflector(n, 0, a.A, a.V, red, &beta);
    for (int r = 1 + tid; r < n; r += TRD_THREADS) lds[r] = a.V[r];
    __syncthreads();
    if (w == 0 && tid == 0) {
      a.d[0] = d0;
      a.e[0] = beta;
      a.tau[0] = tj;
    }
  }

  for (int j = 0; j <= n - 3; ++j) {
    const bool tail = j >= a.jt;
    const int j0 = tail ? a.jt : j - j % DF_NB;  // this panel's first step
    const int j1 = tail ? n - 1 : j0 + DF_NB;    // columns (j, j1]: updated every step
    const int kk = j - j0;                       // updates pending on the later columns
    const int r0 = (j + 1) & ~1;
    const int i0 = (j + 1 - w + P - 1) / P;      // first own column > j: w + i0 P
    const int id = (j1 + 1 - w + P - 1) / P;     // first own column > j1
    const bool later = !tail && id < ncl && w + id * P < n;  // own columns past j1 (uniform)
    const double* vprev = a.V + (size_t)(j > 0 ? j - 1 : 0) * a.lda;
    const double* wprev = a.Wv + (size_t)(j > 0 ? j - 1 : 0) * a.lda;
    double* pubcol = a.cpub + (size_t)(j + 1) * a.lda;
    double sp = 0.0;  // this thread's share of p_j . v_j
    TRD_STAMP(0);
    TRD_WGSTAMP(0);
    TRD_XCCSTAMP();
    if (j == j0 && j > 0) {
      // ---- flush: the previous panel's DF_NB updates on every own column c > j, then . v_j.
      // A GEMM, X(rows, own columns) -= [V W](rows, 2 DF_NB) [w_k[c]; v_k[c]](2 DF_NB, columns),
      // on the FP64 MFMA 16x16x4: first operand the coefficients (lane l: column l & 15 of the
      // column tile, k = l >> 4 of the k-step), second the panel rows (row l & 15), so the result
      // in lane l, entry q is (column (l >> 4) + 4 q, row l & 15): every load and store of X one
      // 128-B column segment per 16 lanes.  Waves split the 16-row tiles, each tile's 2 DF_NB
      // panel values loaded once for all column tiles.  (The same update as VALU FMAs with the
      // coefficients read from LDS per element took ~5x the flush's own HBM time.)
      const int kb = j0 - DF_NB;
      const int nct = (ncl - i0 + 15) / 16;  // column tiles of the own columns > j (<= DF_MAXCT)
      const int lr = lane & 15, lg = lane >> 4;
      typedef double d4 __attribute__((ext_vector_type(4)));
      for (int i = tid; i < TRD_WAVES * ncl; i += TRD_THREADS) qpart[i] = 0.0;
      __syncthreads();
      for (int rt = r0 + 16 * wv; rt < n; rt += 16 * TRD_WAVES) {
        const int r = rt + lr;
        const bool rin = r < n;
        double bv[4], bw[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const size_t k = kb + lg + 4 * s4;
          bv[s4] = rin ? a.V[k * a.lda + r] : 0.0;
          bw[s4] = rin ? a.Wv[k * a.lda + r] : 0.0;
        }
        const double vr = rin && r >= j + 1 ? vcur[r] : 0.0;
#pragma unroll
        for (int ct = 0; ct < DF_MAXCT; ++ct) {
          if (ct >= nct) break;  // (uniform)
          d4 acc;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = i0 + 16 * ct + lg + 4 * q, c = w + i * P;
            acc[q] = rin && i < ncl && c < n ? a.A[(size_t)c * a.lda + r] : 0.0;
          }
          const int ia = i0 + 16 * ct + lr;
          const bool cin = ia < ncl && w + ia * P < n;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int k = lg + 4 * s4;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(cin ? -wown[k * ncl + ia] : 0.0, bv[s4], acc, 0, 0, 0);
          }
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int k = lg + 4 * s4;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(cin ? -vown[k * ncl + ia] : 0.0, bw[s4], acc, 0, 0, 0);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = i0 + 16 * ct + lg + 4 * q, c = w + i * P;
            if (rin && i < ncl && c < n) {
              a.A[(size_t)c * a.lda + r] = acc[q];
              if (c == j + 1) st1(pubcol + r, acc[q]);
            }
            // the tile's part of column i's dot: summed over its 16 rows (lanes l & 15, fixed
            // order) into the wave's slot (one writer per (wave, column))
            double sq = acc[q] * vr;
            sq += __shfl_xor(sq, 1);
            sq += __shfl_xor(sq, 2);
            sq += __shfl_xor(sq, 4);
            sq += __shfl_xor(sq, 8);
            if (lr == 0 && i < ncl) qpart[wv * ncl + i] += sq;
          }
        }
      }
      __syncthreads();
      for (int i = i0 + tid; i < ncl; i += TRD_THREADS) {
        const int c = w + i * P;
        if (c < n) {
          double sdot = 0.0;
#pragma unroll
          for (int q = 0; q < TRD_WAVES; ++q) sdot += qpart[q * ncl + i];
          const double p = tj * sdot;
          st1(&a.pbuf[(size_t)j * a.lda + c], p);
          sp += p * vcur[c];
        }
      }
    } else {
      // ---- the pass.  A deferred panel's own columns in (j, j1] (one at most for P >= DF_NB):
      // the whole workgroup on each, rows split over the threads -- read, updated (step j - 1),
      // written (one wave per such column made its workgroup the step's straggler: ~1.6x the
      // pass, profiles/r06_trd_wg_df.txt)
      if (!tail)
        for (int i = i0; i < ncl; ++i) {
          const int c = w + i * P;
          if (c > j1 || c >= n) break;  // (uniform)
          double* col = a.A + (size_t)c * a.lda;
          const double wc = j > 0 ? wprev[c] : 0.0, vc = j > 0 ? vprev[c] : 0.0;
          double dot = 0.0;
          for (int rb = r0 + 2 * tid; rb < n; rb += 8 * TRD_THREADS) {
            d2 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int r = rb + 2 * TRD_THREADS * u;
              if (r < n) x[u] = *reinterpret_cast<const d2*>(col + r);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int r = rb + 2 * TRD_THREADS * u;
              if (r < n) {
                const d2 vv = *reinterpret_cast<const d2*>(vcur + r);
                if (j > 0) {
                  const d2 vp = *reinterpret_cast<const d2*>(vprev + r);
                  const d2 wp = *reinterpret_cast<const d2*>(wprev + r);
                  x[u].x -= vp.x * wc + wp.x * vc;
                  x[u].y -= vp.y * wc + wp.y * vc;
                  *reinterpret_cast<d2*>(col + r) = x[u];
                }
                if (c == j + 1) {
                  st1(pubcol + r, x[u].x);
                  st1(pubcol + r + 1, x[u].y);
                }
                dot += (r >= j + 1 ? x[u].x * vv.x : 0.0) + (r + 1 < n ? x[u].y * vv.y : 0.0);
              }
            }
          }
          const double p = tj * block_sum(dot, red);
          if (tid == 0) {
            st1(&a.pbuf[(size_t)j * a.lda + c], p);
            sp += p * vcur[c];
          }
        }
      // one wave per own column: the tail's (every column read + updated + written), or a
      // deferred panel's columns past j1 (read only)
      for (int c = w + ((tail ? i0 : id) + wv) * P; c < n; c += TRD_WAVES * P) {
        double* col = a.A + (size_t)c * a.lda;
        const bool eager = tail;
        double dot = 0.0;
        if (eager) {
          const double wc = j > 0 ? wprev[c] : 0.0, vc = j > 0 ? vprev[c] : 0.0;
          double* pub = c == j + 1 ? pubcol : nullptr;
          for (int rb = r0 + 2 * lane; rb < n; rb += PU * 128) {
            d2 x[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
              const int r = rb + 128 * u;
              if (r < n) x[u] = *reinterpret_cast<const d2*>(col + r);
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
              const int r = rb + 128 * u;
              if (r < n) {
                const d2 vv = *reinterpret_cast<const d2*>(vcur + r);
                if (j > 0) {
                  const d2 vp = *reinterpret_cast<const d2*>(vprev + r);
                  const d2 wp = *reinterpret_cast<const d2*>(wprev + r);
                  x[u].x -= vp.x * wc + wp.x * vc;
                  x[u].y -= vp.y * wc + wp.y * vc;
                  *reinterpret_cast<d2*>(col + r) = x[u];
                }
                if (pub) {
                  st1(pub + r, x[u].x);
                  st1(pub + r + 1, x[u].y);
                }
                if (c == n - 1 && j == n - 3) {  // A(n-1, n-1) for the last 2 x 2 block
                  if (r == n - 1) st1(a.dlast, x[u].x);
                  if (r + 1 == n - 1) st1(a.dlast, x[u].y);
                }
                dot += (r >= j + 1 ? x[u].x * vv.x : 0.0) + (r + 1 < n ? x[u].y * vv.y : 0.0);
              }
            }
          }
          const double p = tj * wave_sum(dot);
          if (lane == 0) {
            st1(&a.pbuf[(size_t)j * a.lda + c], p);
            sp += p * vcur[c];
          }
        } else {
          for (int rb = r0 + 2 * lane; rb < n; rb += PU * 128) {
            d2 x[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
              const int r = rb + 128 * u;
              if (r < n) x[u] = *reinterpret_cast<const d2*>(col + r);
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
              const int r = rb + 128 * u;
              if (r < n) {
                const d2 vv = *reinterpret_cast<const d2*>(vcur + r);
                dot += (r >= j + 1 ? x[u].x * vv.x : 0.0) + (r + 1 < n ? x[u].y * vv.y : 0.0);
              }
            }
          }
          const double sdot = wave_sum(dot);
          if (lane == 0) qraw[(c - w) / P] = sdot;
        }
      }
      __syncthreads();  // (qraw)
      if (later && kk > 0) {
        // alpha_k, beta_k: the P workgroups' partials of step j (published with v_j), 16
        // threads per value, summed in a fixed order
        TRD_DELAY(5);
        constexpr int AK = DF_MAXP / 16;
        const int q = tid >> 4, sub = tid & 15;
        // (workgroups sub, sub + 16, ... of value q: cnt of them, none for q >= 2 kk)
        const int cnt = q < 2 * kk ? (P - sub + 15) / 16 : 0;
        const double* base = &a.abuf[((size_t)j * 2 * DF_NB + (q < 2 * kk ? q : 0)) * P + sub];
        double v[AK];
#pragma unroll
        for (int m = 0; m < AK; ++m) v[m] = m < cnt ? ld1(base + 16 * m) : 0.0;
        if (!trd_poll_strided<AK>(a, n, j, s_ok, v, base, 16, cnt)) return;
        double sq = 0.0;
#pragma unroll
        for (int m = 0; m < AK; ++m) sq += v[m];
        sq += __shfl_xor(sq, 1);
        sq += __shfl_xor(sq, 2);
        sq += __shfl_xor(sq, 4);
        sq += __shfl_xor(sq, 8);
        if (sub == 0 && q < 2 * kk) ab[q] = sq;
        __syncthreads();
      }
      if (later) {
        for (int i = id + tid; i < ncl; i += TRD_THREADS) {
          const int c = w + i * P;
          if (c < n) {
            double sdot = qraw[i];
            for (int k = 0; k < kk; ++k)
              sdot -= wown[k * ncl + i] * ab[2 * k] + vown[k * ncl + i] * ab[2 * k + 1];
            const double p = tj * sdot;
            st1(&a.pbuf[(size_t)j * a.lda + c], p);
            sp += p * vcur[c];
          }
        }
      }
    }
    // ---- this step's entries of the panel: v_j at the own columns (w_j's: the exchange);
    // (the flush and the corrections above read only earlier steps' entries, and the flush's
    // reads of entry 0 precede its barrier)
    if (!tail)
      for (int i = tid; i < ncl; i += TRD_THREADS) {
        const int c = w + i * P;
        vown[kk * ncl + i] = c >= j + 1 && c < n ? vcur[c] : 0.0;
        wown[kk * ncl + i] = 0.0;
      }
    // ---- publish this workgroup's part of p_j . v_j
    TRD_STAMP(1);
    TRD_DELAY(1);
    const double spw = block_sum(sp, red);
    TRD_WGSTAMP(1);
    if (tid == 0) {
#ifdef GPR_TESTING
      if (!(j == a.fail_step && w == 0))
#endif
        st1(&a.parts[(size_t)j * P + w], spw);
    }
    // ---- Q^T B on the fly (as sytrd_kernel's GV variant)
    if (a.m > w) {
      const int mine = (a.m - w + P - 1) / P;
      if (mine < 4) {
        for (int c = w; c < a.m; c += P) {
          double* b = a.B + (size_t)c * a.ldb;
          double dot = 0.0;
          for (int r = j + 1 + tid; r < n; r += TRD_THREADS) dot += b[r] * vcur[r];
          const double f = tj * block_sum(dot, red);
          for (int r = j + 1 + tid; r < n; r += TRD_THREADS) b[r] -= f * vcur[r];
        }
      } else {
        for (int c = w + wv * P; c < a.m; c += TRD_WAVES * P) {
          double* b = a.B + (size_t)c * a.ldb;
          double dot = 0.0;
          for (int rb = j + 1 + lane; rb < n; rb += 4 * 64) {
            double x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = rb + 64 * u < n ? b[rb + 64 * u] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (rb + 64 * u < n) dot += x[u] * vcur[rb + 64 * u];
          }
          const double f = tj * wave_sum(dot);
          for (int r = j + 1 + lane; r < n; r += 64) b[r] -= f * vcur[r];
        }
      }
    }
    __syncthreads();  // (every read of v_j in LDS above precedes the exchange's overwrite)
    TRD_STAMP(2);
    // ---- the exchange: p_j, the published column j + 1 and the P partial sums, polled (their
    // sentinel is the arrival flag); w_j to Wv's column j, column j + 1 after step j over v_j in
    // LDS (each row by the thread that read v_j there; row j + 1 and, at the last step, row n - 1
    // to their own slots: v_j[j + 1] and v_j[n - 1] are still read after the loop)
    double* wnew = a.Wv + (size_t)j * a.lda;
    const double* pj = a.pbuf + (size_t)j * a.lda;
    const double* pp = a.parts + (size_t)j * P;
    TRD_DELAY(2);
    double xn = 0.0;
    {
      double pv[2] = {ld1(&pj[j + 1]), tid < P ? ld1(&pp[tid]) : 0.0};
      const double* ps[2] = {&pj[j + 1], tid < P ? &pp[tid] : nullptr};
      if (!trd_poll<2>(a, n, j, s_ok, pv, ps)) return;
      TRD_STAMP(3);
      const double kj = 0.5 * tj * block_sum(pv[1], red);
      TRD_STAMP(4);
      const double wc = pv[0] - kj * vcur[j + 1], vc = vcur[j + 1];
      for (int k0 = 0; j + 1 + k0 * TRD_THREADS < n; k0 += DF_GCH) {  // (uniform bound)
        double xv[2 * DF_GCH];
#pragma unroll
        for (int k = 0; k < DF_GCH; ++k) {
          const int r = j + 1 + tid + (k0 + k) * TRD_THREADS;
          xv[2 * k] = r < n ? ld1(&pj[r]) : 0.0;
          xv[2 * k + 1] = r < n ? ld1(&pubcol[r]) : 0.0;
        }
        if (!trd_poll_rows<DF_GCH>(a, n, j, s_ok, xv, pj, pubcol, j + 1 + tid + k0 * TRD_THREADS))
          return;
#pragma unroll
        for (int k = 0; k < DF_GCH; ++k) {
          const int r = j + 1 + tid + (k0 + k) * TRD_THREADS;
          if (r < n) {
            const double wr = xv[2 * k] - kj * vcur[r];
            const double x = xv[2 * k + 1] - (vcur[r] * wc + wr * vc);
            wnew[r] = wr;
            if (!tail && r >= w && (r - w) % P == 0) wown[kk * ncl + (r - w) / P] = wr;
            if (r == j + 1) *s_d = x;
            else if (j == n - 3 && r == n - 1) *s_cl = x;
            else lds[r] = x;
            if (r >= j + 3) xn += x * x;
            if (r == j + 2) *s_alpha = x;
          }
        }
      }
    }
    TRD_STAMP2(0);
    const double xnorm2 = block_sum(xn, red);  // (its barriers publish the LDS column, wnew)
    const bool out = w == (j + 1) % P;         // (one workgroup writes T)
    if (out && tid == 0) a.d[j + 1] = *s_d;
    if (j + 1 <= n - 3) {
      TRD_DELAY(3);
      const double alpha = *s_alpha;
      double tau = 0.0, beta = alpha, scal = 0.0;
      if (xnorm2 > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
        tau = (beta - alpha) / beta;
        scal = 1.0 / (alpha - beta);
      }
      double* vj = a.V + (size_t)(j + 1) * a.lda;  // (every workgroup: the same bits)
      for (int r = j + 2 + tid; r < n; r += TRD_THREADS) {
        const double v = r == j + 2 ? 1.0 : lds[r] * scal;
        vj[r] = v;
        lds[r] = v;
      }
      if (out && tid == 0) {
        a.e[j + 1] = beta;
        a.tau[j + 1] = tau;
      }
      tj = tau;
      TRD_DELAY(4);
      __syncthreads();
      // ---- the partials of alpha_k, beta_k for step j + 1 (inside a deferred panel): over the
      // own columns, from LDS only
      TRD_STAMP2(1);
      const int jn = j + 1, kn = jn % DF_NB;
      if (jn < a.jt && kn != 0) {
        TRD_DELAY(6);
        for (int q = wv; q < 2 * kn; q += TRD_WAVES) {
          const double* own = (q & 1) ? wown : vown;
          double sq = 0.0;
          for (int i = lane; i < ncl; i += 64) {
            const int c = w + i * P;
            if (c >= jn + 1 && c < n) sq += own[(q >> 1) * ncl + i] * lds[c];
          }
          sq = wave_sum(sq);
          if (lane == 0) st1(&a.abuf[((size_t)jn * 2 * DF_NB + q) * P + w], sq);
        }
      }
    } else if (out && tid == 0) {  // the last 2 x 2 block: e_{n-2}, d_{n-1}
      a.e[n - 2] = *s_cl;
      double dl = ld1(a.dlast);
      for (long long spins = 0; trd_unset(dl) && spins <= a.spin_limit; ++spins) {
        __builtin_amdgcn_s_sleep(1);
        dl = ld1(a.dlast);
      }
      if (trd_unset(dl)) st1i(a.err, 1);
      a.d[n - 1] = dl - 2.0 * vcur[n - 1] * wnew[n - 1];
    }
    TRD_STAMP(5);
  }
}

// ---- Q^T B by blocks of reflectors (compact WY, dlarft forward / columnwise) --------------
constexpr int QB = 64;  // reflectors per block

// Vb (n2 x QB, ld n2) and VbT (QB x n2, ld QB): column i = v_{j0+i} (zeros above row j0+i+1,
// zero columns past the last reflector)
__global__ void qblock_prep_kernel(const double* __restrict__ V, size_t ldv, int n, int n2,
                                   int j0, int nref, double* __restrict__ Vb,
                                   double* __restrict__ VbT) {
  const size_t tot = (size_t)n2 * QB;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(t % n2), i = (int)(t / n2);
    const int j = j0 + i;
    const double v = (i < nref && r > j && r < n) ? V[(size_t)j * ldv + r] : 0.0;
    Vb[t] = v;
    VbT[(size_t)i + (size_t)r * QB] = v;
  }
}

// [G | W] = Vb^T [Vb | B] for one block, split over the rows (thin outputs -- 64 rows, long K --
// leave a tiled GEMM a few dozen tiles; here every 64-column tile x row slice is a workgroup).
// Workgroup (tile x, slice y): rows [k0, k1) of the slice, output columns [64x, 64x + 64) of the
// Nc = QB + m columns (c < QB: Vb's column c, else B's column c - QB); 16-row stages through
// LDS, each thread a 4 x 4 block of outputs.  part[y] (QB x Nc, ld QB) = the slice's sum.
constexpr int GW_KB = 16;
__global__ __launch_bounds__(256) void qblock_gw_partial_kernel(
    const double* __restrict__ Vb, int n2, const double* __restrict__ B, size_t ldb, int m,
    int r0, int n, int ks, double* __restrict__ part) {
  __shared__ double sP[GW_KB][QB + 2];
  __shared__ double sQ[GW_KB][QB + 2];
  const int tid = threadIdx.x;
  const int nc = QB + m;
  const int c0 = blockIdx.x * 64;
  const int k0 = r0 + blockIdx.y * ks, k1 = min(n, k0 + ks);
  const int ti = (tid & 15) * 4, tc = (tid >> 4) * 4;
  double acc[4][4] = {};
  const int lr = tid & 15, lc = tid >> 4;  // loader: row lr, columns lc + 16 q
  for (int kb = k0; kb < k1; kb += GW_KB) {
    const int r = kb + lr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = lc + 16 * q;
      sP[lr][col] = r < k1 ? Vb[(size_t)col * n2 + r] : 0.0;
      const int c = c0 + col;
      double v = 0.0;
      if (r < k1 && c < nc) v = c < QB ? Vb[(size_t)c * n2 + r] : B[(size_t)(c - QB) * ldb + r];
      sQ[lr][col] = v;
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < GW_KB; ++rr) {
      double a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = sP[rr][ti + u];
        b[u] = sQ[rr][tc + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
    }
    __syncthreads();
  }
  double* out = part + (size_t)blockIdx.y * QB * nc;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int c = c0 + tc + v;
    if (c < nc)
#pragma unroll
      for (int u = 0; u < 4; ++u) out[(size_t)c * QB + ti + u] = acc[u][v];
  }
}

// G (QB x QB) and W (QB x m, ld QB) = the sum of the S slices (fixed order: deterministic)
__global__ void qblock_gw_reduce_kernel(const double* __restrict__ part, int S, int m,
                                        double* __restrict__ G, double* __restrict__ W) {
  const size_t nc = (size_t)QB + m, tot = (size_t)QB * nc;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int y = 0; y < S; ++y) s += part[(size_t)y * tot + t];
    if (t < (size_t)QB * QB) G[t] = s;
    else W[t - (size_t)QB * QB] = s;
  }
}

// T (QB x QB upper, ld QB) from G = Vb^T Vb and tau: T(i,i) = tau_i, T(0:i, i) = -tau_i
// T(0:i, 0:i) G(0:i, i) (dlarft forward / columnwise); unused columns (i >= nref) zero.  G and
// tau are staged in LDS first (the recurrence's 64 steps then never wait on memory).
__global__ __launch_bounds__(QB) void qblock_t_kernel(const double* __restrict__ G,
                                                     const double* __restrict__ tau, int j0,
                                                     int nref, double* __restrict__ T) {
  __shared__ double Ts[QB][QB + 1];
  __shared__ double Gs[QB][QB + 1];
  __shared__ double g[QB];
  __shared__ double ts[QB];
  const int k = threadIdx.x;
  for (int i = 0; i < QB; ++i) {
    Ts[k][i] = 0.0;
    Gs[k][i] = G[k + (size_t)i * QB];
  }
  ts[k] = k < nref ? tau[j0 + k] : 0.0;
  __syncthreads();
  for (int i = 0; i < nref; ++i) {
    const double ti = ts[i];
    g[k] = k < i ? -ti * Gs[k][i] : 0.0;
    __syncthreads();
    double s = 0.0;
    if (k < i)
      for (int l = k; l < i; ++l) s += Ts[k][l] * g[l];
    if (k < i) Ts[k][i] = s;
    if (k == i) Ts[i][i] = ti;
    __syncthreads();
  }
  for (int i = 0; i < QB; ++i) T[k + (size_t)i * QB] = Ts[k][i];
}

// ---- the quadrature's per-column solves on T ---------------------------------------------
// Column j (one thread): x = (T + s_j I)^{-1} c with c = C[:, ny] = Q^T k1 by Gaussian
// elimination with partial pivoting on the tridiagonal (dgtsv: the row interchanges fill a
// second superdiagonal), then out[2j] = C[:, j] . x (= k1' (K + s_j I)^{-1} y_j, Iout) and
// out[2j+1] = k2 - c . x (var).  Columns [j0, j1) of this launch; scratch: 4 n doubles per
// column of the launch, interleaved across the launch's columns (entry i of array k of column
// t at scr[(k n + i) cols + t]) so a wave's 64 columns touch 64 consecutive doubles per step
// (d, e and c are the same for every column: broadcast loads).
__global__ void quad_tridiag_kernel(const double* __restrict__ d, const double* __restrict__ e,
                                    int n, const double* __restrict__ C, size_t ldc, int ny,
                                    int j0, int j1, const double* __restrict__ noise, double k2,
                                    double* __restrict__ scr, double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = j0 + t;
  if (j >= j1) return;
  const size_t cols = (size_t)(j1 - j0);
  const double s = noise[j];
  const double* c = C + (size_t)ny * ldc;
  double* Dm = scr + t;                   // final pivots: Dm[i cols]
  double* U1 = Dm + (size_t)n * cols;     // first superdiagonal
  double* U2 = U1 + (size_t)n * cols;     // second superdiagonal (row interchanges)
  double* x = U2 + (size_t)n * cols;      // right-hand side -> solution
  if (n == 1) {
    const double x0 = c[0] / (d[0] + s);
    out[2 * j] = C[(size_t)j * ldc] * x0;
    out[2 * j + 1] = k2 - c[0] * x0;
    return;
  }
  // running row i: (Di, Ui) on the diagonal / superdiagonal, bi; next row: (L = e_i, Dn, Un)
  double Di = d[0] + s, Ui = e[0], bi = c[0];
  for (int i = 0; i < n - 1; ++i) {
    const size_t at = (size_t)i * cols;
    const double L = e[i];
    const double Dn = d[i + 1] + s;
    const double Un = i + 1 < n - 1 ? e[i + 1] : 0.0;
    const double bn = c[i + 1];
    if (fabs(Di) >= fabs(L)) {  // no interchange
      const double f = L / Di;
      Dm[at] = Di;
      U1[at] = Ui;
      U2[at] = 0.0;
      x[at] = bi;
      Di = Dn - f * Ui;
      Ui = Un;
      bi = bn - f * bi;
    } else {  // rows i and i + 1 swap: row i becomes (L, Dn, Un), the next (Di, Ui, 0) - f row i
      const double f = Di / L;
      Dm[at] = L;
      U1[at] = Dn;
      U2[at] = Un;
      x[at] = bn;
      const double nd = Ui - f * Dn;
      const double nu = -f * Un;
      const double nb = bi - f * bn;
      Di = nd;
      Ui = nu;
      bi = nb;
    }
  }
  // back substitution, dotting as it goes
  const double* cy = C + (size_t)j * ldc;
  double x2 = 0.0, x1 = bi / Di;
  double si = cy[n - 1] * x1, sv = c[n - 1] * x1;
  for (int i = n - 2; i >= 0; --i) {
    const size_t at = (size_t)i * cols;
    const double xi = (x[at] - U1[at] * x1 - U2[at] * x2) / Dm[at];
    si += cy[i] * xi;
    sv += c[i] * xi;
    x2 = x1;
    x1 = xi;
  }
  out[2 * j] = si;
  out[2 * j + 1] = k2 - sv;
}

__global__ void trd_copy_kernel(const double* __restrict__ A, size_t lda, int n,
                                double* __restrict__ W, size_t ldw) {
  const size_t tot = (size_t)n * n;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(t % n), c = (int)(t / n);
    W[(size_t)r + (size_t)c * ldw] = A[(size_t)r + (size_t)c * lda];
  }
}

}  // namespace

namespace {
// the work copy and the exchange buffers (4 n^2 doubles) are not kept past the call once they
// pass 1 GB (n > ~5.8k; re-allocating costs far less than the reduction itself)
int release_eig_scratch(gpr_ctx* ctx) {
  if (ctx->deig && ctx->eig_cap * sizeof(double) > (size_t)(1ull << 30)) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(ctx->deig));
    ctx->deig = nullptr;
    ctx->eig_cap = 0;
  }
  return 0;
}

template <int PU, int RP, bool GV>
const void* trd_kernel_ptr() {
  return reinterpret_cast<const void*>(&sytrd_kernel<PU, RP, GV>);
}
}  // namespace

// A (n x n, lda; symmetric, both triangles read) = Q T Q^T: d[n], e[n-1] (device) and, when
// m > 0, B <- Q^T B (n x m, ldb).  Workspace in ctx->deig.  n <= TRD_MAXN_G.
// Returns GPR_E_UNSUP -- before touching B -- when n is beyond the bound or the launch's
// workgroups cannot all be resident at once (the exchange needs every one of them every step:
// the launch is cooperative, so the runtime refuses it up front rather than letting resident
// workgroups spin on absent ones); the callers then take another route.
int sym_tridiag(gpr_ctx* ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                double* dd, double* de) {
  if (n <= 0) return 0;
  if (n > TRD_MAXN_G) return set_err(ctx, GPR_E_UNSUP, "tridiagonal reduction: n = %d > %d", n, TRD_MAXN_G);
  hipStream_t st = ctx->stream;
  if (ctx->ncu <= 0) {
    hipDeviceProp_t prop;
    HIP_TRY(ctx, hipGetDeviceProperties(&prop, ctx->device));
    ctx->ncu = prop.multiProcessorCount;
  }
  // from TRD_DF_MIN on: the deferred-update variant (DF) when its partials' poll and flush tiles
  // cover the grid, else (beyond TRD_MAXN) the per-step GV variant.  (Test build: GPR_TRD_DF = 0 the GV variant, 2 DF at any n --
  // A/B and small-n parity; GPR_TRD_DF_TAIL the steps left to the tail.)
  int df_mode = 1;
  int df_tail = DF_TAIL;
#ifdef GPR_TESTING
  if (const char* e = getenv("GPR_TRD_DF")) df_mode = atoi(e);
  if (const char* e = getenv("GPR_TRD_DF_TAIL")) df_tail = std::max(2 * DF_NB, atoi(e));
#endif
  size_t ld = (size_t)(n + 15) / 16 * 16;
#ifdef GPR_TESTING
  if (const char* e = getenv("GPR_TRD_LDPAD")) ld += (size_t)std::max(0, atoi(e)) / 16 * 16;  // (A/B)
#endif
  // workgroups: 8 columns each up to n ~ 1500, 16 above (profiles/r05_trd_sweep.txt: 4..24
  // columns change n = 512 / 1100 / 2048 / 4096 by <= 12 / 13 / 11 / 1 %), at most one per CU.
  // (Measured and removed:
  // the last owned columns held in registers through the whole launch -- every column for n <=
  // 2048 -- ran no faster: the per-step exchange, not the pass, bounds small n, and at n = 4096
  // the register pressure cut the pass's loads in flight)
  int cols = n <= 1536 ? 8 : 16;
#ifdef GPR_TESTING
  if (const char* e = getenv("GPR_TRD_COLS")) cols = std::max(1, atoi(e));  // (tuning sweeps)
#endif
  const int P = std::max(1, std::min(std::min(ctx->ncu, TRD_THREADS), (n + cols - 1) / cols));
  const int ncl = (n + P - 1) / P;
  const bool df = P <= DF_MAXP && ncl <= 16 * DF_MAXCT && n >= 3 &&
                  ((n >= TRD_DF_MIN && df_mode == 1) || df_mode == 2);
  const bool gv = n > TRD_MAXN || df;
  const size_t shmem =
      df ? ((size_t)((n + 1) & ~1) + TRD_WAVES + 4 + (2 * DF_NB + 1 + TRD_WAVES) * (size_t)ncl + 2 * DF_NB) *
               sizeof(double)
         : ((gv ? 1 : 3) * (size_t)((n + 1) & ~1) + TRD_WAVES + 2) * sizeof(double);
  const void* kfn = df   ? reinterpret_cast<const void*>(&sytrd_df_kernel)
                    : gv ? trd_kernel_ptr<16, RPT_G, true>()
                         : n >= 800 ? trd_kernel_ptr<16, RPT, false>() : trd_kernel_ptr<8, RPT, false>();
  // co-residency: one workgroup per CU (the launch bound and, for the LDS variant, its vectors
  // allow no more); none at all is refused here, and the cooperative launch below refuses a grid
  // that cannot be resident as a whole
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, TRD_THREADS, shmem) != hipSuccess ||
      per_cu <= 0) {
    (void)hipGetLastError();
    return set_err(ctx, GPR_E_UNSUP, "tridiagonal reduction: no resident workgroup possible");
  }
  // workspace: W, V, cpub, pbuf (ld x n each), parts (n x P), (DF) abuf, tau, dlast, then ints
  const size_t nW = ld * n;
  const size_t nI = (size_t)n + 2;  // counters, err (as doubles: half of it, rounded up)
  const int n2 = (int)ld;
  // B <- Q^T B inside the launch (each workgroup applies H_j to its columns of B as v_j
  // appears) up to TRD_FUSED_M columns; wider B (e.g. gpr_syev_apply on B = I) by blocks of
  // 64 reflectors on the MFMA GEMM afterwards
  const bool fused_b = m > 0 && m <= TRD_FUSED_M;
  // the back-transform's row slices: enough workgroups for the chip (~1024), >= 64 rows each
  const int gw_tiles = (QB + m + 63) / 64;
  const int gw_S = std::max(1, std::min((n + 63) / 64, (1024 + gw_tiles - 1) / gw_tiles));
  const size_t nQ = (m > 0 && !fused_b)
                        ? 2 * (size_t)n2 * QB + 2 * (size_t)QB * QB + 2 * (size_t)QB * m +
                              (size_t)gw_S * QB * (QB + m)
                        : 0;
  // (GV: the w and column-(j+1) rings, 4 columns each; DF: Wv, ld x n)
  const size_t nG = df ? nW : gv ? 8 * ld : 0;
  const size_t nA = df ? (size_t)n * 2 * DF_NB * P : 0;  // (DF: the panel's dot partials)
  const size_t need = 4 * nW + (size_t)n * P + nA + (size_t)n + 8 + nI + nQ + nG;
  GPR_TRY(ensure_buf(ctx, &ctx->deig, &ctx->eig_cap, need));
  double* W = ctx->deig;
  double* V = W + nW;
  double* cpub = V + nW;
  double* pbuf = cpub + nW;
  double* parts = pbuf + nW;
  double* abuf = parts + (size_t)n * P;
  double* tau = abuf + nA;
  double* dlast = tau + n;
  int* ints = reinterpret_cast<int*>(dlast + 8);
  int* err = ints + n;
  double* Vb = reinterpret_cast<double*>(ints) + nI;  // the Q^T B blocks'
  double* rings = Vb + nQ;
  TimerScope ts(ctx, TC_OTHER, 4.0 * n * (double)n * n / 3.0);
  if (n == 1 || n == 2) {  // already tridiagonal: T = A, Q = I
    HIP_TRY(ctx, hipMemcpy2DAsync(dd, sizeof(double), dA, sizeof(double) * (lda + 1),
                                  sizeof(double), n, hipMemcpyDeviceToDevice, st));
    if (n == 2) HIP_TRY(ctx, hipMemcpyAsync(de, dA + 1, sizeof(double), hipMemcpyDeviceToDevice, st));
    return 0;
  }
  trd_copy_kernel<<<1024, 256, 0, st>>>(dA, (size_t)lda, n, W, ld);
  LAUNCH_CHECK(ctx);
  HIP_TRY(ctx, hipMemsetAsync(ints, 0, sizeof(int) * ((size_t)n + 2), st));
  // cpub, pbuf, parts, abuf (contiguous) and dlast start "unset" (the exchange polls on the values)
  trd_fill_unset_kernel<<<1024, 256, 0, st>>>(cpub, 2 * nW + (size_t)n * P + nA);
  trd_fill_unset_kernel<<<1, 64, 0, st>>>(dlast, 1);
  LAUNCH_CHECK(ctx);
  HIP_TRY(ctx, hipMemsetAsync(tau, 0, sizeof(double) * n, st));
  TrdArgs a{};
  a.A = W;
  a.lda = ld;
  a.n = n;
  a.P = P;
  a.ldl = (n + 1) & ~1;
  a.V = V;
  a.cpub = cpub;
  a.pbuf = pbuf;
  a.parts = parts;
  a.tau = tau;
  a.d = dd;
  a.e = de;
  a.dlast = dlast;
  a.err = err;
  a.spin_limit = 1ll << 22;
#ifdef GPR_TESTING
  // (fault injection: GPR_TRD_FAIL_STEP = a step whose hand-off never completes; GPR_TRD_SPIN_LIMIT
  // shortens the bound so the time-out comes quickly)
  a.fail_step = getenv("GPR_TRD_FAIL_STEP") ? atoi(getenv("GPR_TRD_FAIL_STEP")) : -1;
  if (const char* e = getenv("GPR_TRD_SPIN_LIMIT")) a.spin_limit = atoll(e);
  a.delay = getenv("GPR_TRD_DELAY") ? std::max(0, atoi(getenv("GPR_TRD_DELAY"))) : 0;
  a.wgoff = getenv("GPR_TRD_WGOFF") ? std::max(0, std::min(63, atoi(getenv("GPR_TRD_WGOFF")))) : 0;
#endif
  a.B = fused_b ? dB : nullptr;
  a.ldb = (size_t)ldb;
  a.m = fused_b ? m : 0;
  a.wr = gv && !df ? rings : nullptr;
  a.xr = gv && !df ? rings + 4 * ld : nullptr;
  a.Wv = df ? rings : nullptr;
  a.abuf = df ? abuf : nullptr;
  a.jt = df ? std::max(0, (n - df_tail) / DF_NB * DF_NB) : 0;
  a.ncl = ncl;
  // cooperative: all P workgroups resident together, or the runtime refuses the launch (nothing
  // has run then: B is untouched, and the caller falls back)
  void* kargs[] = {&a};
  if (hipLaunchCooperativeKernel(kfn, dim3(P), dim3(TRD_THREADS), kargs, (unsigned)shmem, st) !=
      hipSuccess) {
    (void)hipGetLastError();
    return set_err(ctx, GPR_E_UNSUP, "tridiagonal reduction: cooperative launch of %d workgroups "
                   "refused", P);
  }
  int herr = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(ctx, hipStreamSynchronize(st));
  if (herr) return set_err(ctx, GPR_E_HIP, "tridiagonal reduction: a wait timed out");
  if (m <= 0 || fused_b) return release_eig_scratch(ctx);
  // B <- Q^T B = H_{n-3} ... H_0 B, 64 reflectors per block: B -= V_b (T_b^T (V_b^T B))
  const int nref_all = n - 2;
  double* VbT = Vb + (size_t)n2 * QB;
  double* G = VbT + (size_t)n2 * QB;
  double* T = G + (size_t)QB * QB;
  double* Wm = T + (size_t)QB * QB;
  double* X = Wm + (size_t)QB * m;
  double* Pgw = X + (size_t)QB * m;
  for (int j0 = 0; j0 < nref_all; j0 += QB) {
    const int nref = std::min(QB, nref_all - j0);
    const int r0 = ((j0 + 1) / 16) * 16;  // rows below r0 of this block's V are zero
    qblock_prep_kernel<<<512, 256, 0, st>>>(V, ld, n, n2, j0, nref, Vb, VbT);
    LAUNCH_CHECK(ctx);
    // [G | W] = Vb^T [Vb | B] (rows >= r0), split over row slices
    const int S = std::max(1, std::min(gw_S, (n - r0 + 63) / 64));
    const int ks = ((n - r0 + S - 1) / S + GW_KB - 1) / GW_KB * GW_KB;
    qblock_gw_partial_kernel<<<dim3(gw_tiles, S), 256, 0, st>>>(Vb, n2, dB, (size_t)ldb, m, r0, n,
                                                                 ks, Pgw);
    LAUNCH_CHECK(ctx);
    qblock_gw_reduce_kernel<<<1024, 256, 0, st>>>(Pgw, S, m, G, Wm);
    LAUNCH_CHECK(ctx);
    qblock_t_kernel<<<1, QB, 0, st>>>(G, tau, j0, nref, T);
    LAUNCH_CHECK(ctx);
    GemmArgs x{};  // X = T^T W
    x.P = T; x.ldp = QB;
    x.Q = Wm; x.ldq = QB;
    x.C = X; x.ldc = QB;
    x.M = QB; x.N = m; x.K = QB;
    x.alpha = 1.0; x.beta = 0.0;
    GPR_TRY(launch_gemm_tn(ctx, x, TC_OTHER));
    GemmArgs u{};  // B -= V_b X (rows >= r0)
    u.P = VbT + (size_t)r0 * QB; u.ldp = QB;
    u.Q = X; u.ldq = QB;
    u.C = dB + r0; u.ldc = ldb;
    u.M = n - r0; u.N = m; u.K = QB;
    u.alpha = -1.0; u.beta = 1.0;
    GPR_TRY(launch_gemm_tn(ctx, u, TC_OTHER));
  }
  return release_eig_scratch(ctx);
}

// out[2j] = Iout_j, out[2j+1] = var_j for the quadrature (see quad_tridiag_kernel); C = Q^T [Y | k1]
// (scr: 4 n quad_tridiag_chunk(n, ny) doubles of device scratch; launches of that many columns)
int quad_tridiag_chunk(int n, int ny) {
#ifdef GPR_TESTING
  if (const char* e = getenv("GPR_TRD_QCHUNK")) return std::max(1, std::min(ny, atoi(e)));
#endif
  // ~1 GB of scratch at most (>= 256 columns per launch: 4 waves per CU-sized launch)
  const long long cap = std::max(256ll, (1ll << 27) / (4ll * std::max(n, 1)));
  return (int)std::min<long long>(ny, cap);
}

int quad_tridiag_solves(gpr_ctx* ctx, const double* dd, const double* de, int n, const double* C,
                        int ldc, int ny, const double* dnoise, double k2, double* scr, double* out) {
  const int chunk = quad_tridiag_chunk(n, ny);
  for (int j0 = 0; j0 < ny; j0 += chunk) {
    const int j1 = std::min(ny, j0 + chunk);
    quad_tridiag_kernel<<<(j1 - j0 + 63) / 64, 64, 0, ctx->stream>>>(dd, de, n, C, (size_t)ldc, ny, j0,
                                                                    j1, dnoise, k2, scr, out);
    LAUNCH_CHECK(ctx);
  }
  return 0;
}

bool sym_tridiag_ok(int n) { return n >= 1 && n <= TRD_MAXN_G; }

#ifdef GPR_TESTING
// the last reduction's phase stamps (100 MHz clock): [2][n][6] long longs
// every workgroup's pass start / end at steps 0, 64, 128, ...: [TRD_MAXN / 64][256][2]
extern "C" int gpr_testing_trd_wg_trace(long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trd_wg), sizeof(long long) * (TRD_MAXN / 64) * 256 * 2) !=
      hipSuccess)
    return GPR_E_HIP;
  return 0;
}

extern "C" int gpr_testing_trd_xcc(int* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trd_xcc), sizeof(int) * 256) == hipSuccess ? 0 : GPR_E_HIP;
}

extern "C" int gpr_testing_trd_trace2(long long* out, int n) {
  if (n < 1) return GPR_E_ARG;
  n = std::min(n, TRD_MAXN);
  std::vector<long long> h(2 * (size_t)TRD_MAXN * 2);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_trd_trace2), h.size() * sizeof(long long)) != hipSuccess)
    return GPR_E_HIP;
  for (int k = 0; k < 2; ++k)
    std::copy(h.begin() + (size_t)k * TRD_MAXN * 2, h.begin() + ((size_t)k * TRD_MAXN + n) * 2,
              out + (size_t)k * n * 2);
  return 0;
}

extern "C" int gpr_testing_trd_trace(long long* out, int n) {
  if (n < 1) return GPR_E_ARG;
  n = std::min(n, TRD_MAXN);  // (the first TRD_MAXN steps are stamped)
  std::vector<long long> h(2 * (size_t)TRD_MAXN * 6);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_trd_trace), h.size() * sizeof(long long)) != hipSuccess)
    return GPR_E_HIP;
  for (int k = 0; k < 2; ++k)
    std::copy(h.begin() + (size_t)k * TRD_MAXN * 6, h.begin() + ((size_t)k * TRD_MAXN + n) * 6,
              out + (size_t)k * n * 6);
  return 0;
}
#endif

extern "C" int gpr_sytrd_apply(gpr_ctx_t ctx, const double* dA, int n, int lda, double* dB, int m,
                               int ldb, double* dd, double* de) {
  if (!ctx) return GPR_E_ARG;
  if (n < 0 || m < 0 || lda < std::max(n, 1) || (m > 0 && ldb < std::max(n, 1)) ||
      (n > 0 && (!dA || !dd || (n > 1 && !de))) || (m > 0 && n > 0 && !dB))
    return set_err(ctx, GPR_E_ARG, "bad args");
  return sym_tridiag(ctx, dA, n, lda, dB, m, ldb, dd, de);
}
