// Diagonal-block factorisation device code, shared by potrf.hip (diag2_kernel: one launch per
// 128-block of the blocked factorisation) and dag.hip (the F tasks of the persistent tile-DAG
// factorisation).  One 256-thread workgroup factors a 128 x 128 block held in LDS (packed
// upper) and writes U_bb and W_bb = U_bb^{-1}.
#pragma once
#include "common.hpp"

#ifndef STAMP
#define STAMP(i) \
  do {           \
  } while (0)
#endif
// phase timers of the tile-DAG's diagonal factor (dag.hip's DAG_TRACE build defines them)
#ifndef DSTAMP
#define DSTAMP_INIT() \
  do {                \
  } while (0)
#define DSTAMP(i) \
  do {            \
  } while (0)
#define DSTAMPW(i) \
  do {             \
  } while (0)
#endif

namespace {

constexpr int DIAG_THREADS = 256;

typedef double d4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
// LDS-typed pointers: the tile-DAG calls the factor out of line, and through a generic pointer
// every LDS access became a flat-to-local conversion with its own null check and the trailing
// update's loads were issued one at a time
typedef __attribute__((address_space(3))) double lds_d;
typedef __attribute__((address_space(3))) int lds_i;
typedef __attribute__((address_space(3))) d2v lds_d2v;

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int pk(int r, int c) { return (c * (c + 1) >> 1) + r; }  // r <= c

// 1/sqrt(x) to ~1 ulp: hardware rsq + one Newton step (shorter dependency chain than the
// correctly-rounded sqrt + divide; this is the pivot of every sequential step)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x * y;
  const double r = fma(-h, y, 0.5);
  return fma(y, r, y);
}

// Global store of a result another workgroup of the SAME launch may read after a flag
// (SC1: sc1 = write-through, the line leaves this XCD's L2 -- the MI355X guide's sc1
// hand-off), or a plain store (results read only by later launches).
// (through a global-typed pointer: out of line -- the tile-DAG's factor -- a generic pointer
// made these flat stores, which also count in lgkmcnt, so every later LDS wait of the inverse
// waited for the write-through stores too)
typedef __attribute__((address_space(1))) double glb_d;
template <bool SC1>
__device__ __forceinline__ void st_res(double* p, double v) {
  glb_d* g = (glb_d*)p;
  if constexpr (SC1)
    __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *g = v;
}

// ---- diag kernel v2 (NB = 128, factor mode): no per-pivot workgroup barriers ------------
// Per 32-row band sb (K0 = 32 sb, band = rows [K0, K0+32) x cols [K0, 128)):
//   F1  the band is eliminated by whole waves WITHOUT barriers: a wave holds 64 columns of
//       the band in registers (lane = column, register = row) and broadcasts the pivot row
//       with v_readlane.  Every active wave carries the 32x32 diagonal block D in lanes 0-31
//       (recomputed identically, so no wave waits for another) and 32 further columns in
//       lanes 32-63: 32 strip columns (-> U = D^-T S), or, on the last active wave, the
//       identity (-> D^-T, i.e. the rows of the 32x32 inverse Xd_sb for free).
//   F3  trailing update of the rest of the block on MFMA (all waves).
// Inverse W = U^-1 from U and the Xd: column half (J, jh) of W is a 16-column recurrence
//   X_JJ = Xd_J,  X_IJ = -Xd_I sum_{K=I+1..J} U_IK X_KJ   (I = J-1 .. 0)
// kept entirely in MFMA accumulators (D-layout register q = B operand of k-step q), one
// wave per column half -- blocks 0-1 beside band 2 and block 2 beside band 3 (waves 2-3, idle
// there), block 3 after the last band (the tile-DAG's factor: in Q form on all four waves,
// d2_tail_q / d2_tail_out); W goes to the workspace slot with fire-and-forget stores.  No
// global read-back and no barrier after a global store, so nothing waits on HBM latency
// except the single batched load of the block.
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

constexpr int D2_NB = 128;
constexpr int D2_PK = D2_NB * (D2_NB + 1) / 2;  // packed 128x128 upper (66 KB)
constexpr int D2_PB = 32 * 33 / 2;              // packed 32x32 upper
// the factor's LDS: S (D2_PK), Xd (4 D2_PB), the fail flag (2 doubles' room), then per wave a
// 64-double pivot-row buffer (16-B aligned)
constexpr int D2_PIV = D2_PK + 4 * D2_PB + 2;
constexpr int D2_LDS_DOUBLES = D2_PIV + 4 * 64;
// the tile-DAG's factor (QTAIL) also keeps W's off-diagonal blocks X_01, X_02, X_12 (32 x 33,
// row-major) and the Q^T half-tiles the last column block's waves exchange
constexpr int D2_XO = D2_LDS_DOUBLES;
constexpr int D2_QS = D2_XO + 3 * 32 * 33;
constexpr int D2_LDS_QTAIL = D2_QS + 3 * 2 * 4 * 64;

// column half (J, jh) of W = U^-1 (see above); S = U packed upper (128), Xd = packed diag inverses
// (Xo != nullptr: the off-diagonal blocks X_IJ also go to Xo[I + J - 1], row-major, stride 33)
template <int J, bool SC1>
__device__ __forceinline__ void d2_inv_colhalf(int jh, const lds_d* __restrict__ S,
                                               const lds_d (*__restrict__ Xd)[D2_PB],
                                               double* __restrict__ winv, int kb, int lane,
                                               lds_d* __restrict__ Xo = nullptr) {
  d4v X[J + 1][2];
  const int col = 16 * jh + (lane & 15);  // column within block J
#pragma unroll
  for (int ih = 0; ih < 2; ++ih)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * ih + (lane >> 4) + 4 * r;
      const double v = Xd[J][pk(min(row, col), col)];
      X[J][ih][r] = row <= col ? v : 0.0;
    }
#pragma unroll
  for (int I = J - 1; I >= 0; --I) {
    d4v T[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int K = I + 1; K <= J; ++K)
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int k = 32 * K + 4 * st + (lane >> 4);
        const double b = X[K][st >> 2][st & 3];
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          const double a = S[pk(32 * I + 16 * ih + (lane & 15), k)];
          T[ih] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, T[ih], 0, 0, 0);
        }
      }
#pragma unroll
    for (int ih = 0; ih < 2; ++ih) {
      d4v acc = {0.0, 0.0, 0.0, 0.0};
      const int i = 16 * ih + (lane & 15);
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int m = 4 * st + (lane >> 4);
        const double xv = Xd[I][pk(min(i, m), m)];
        // (-Xd_I as the A operand: the result is X_IJ itself, which feeds the next level's
        // MFMAs straight from the accumulators -- negating acc moved it through VGPRs on the
        // level-to-level chain)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(i <= m ? -xv : 0.0, T[st >> 2][st & 3], acc, 0, 0, 0);
      }
      X[I][ih] = acc;
      if (Xo) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Xo[(I + J - 1) * 32 * 33 + (16 * ih + (lane >> 4) + 4 * r) * 33 + col] = acc[r];
      }
    }
  }
  const int gc = 32 * J + col;
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int ih = 0; ih < 2; ++ih)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = 32 * I + 16 * ih + (lane >> 4) + 4 * r;
        const double v = (I <= J) ? X[I <= J ? I : 0][ih][r] : 0.0;
        st_res<SC1>(&winv[gr + (size_t)gc * 128], (gr < kb && gc < kb) ? v : 0.0);
      }
}

// W's last column block without the recurrence's chain (the tile-DAG's factor): block column 3
// of W U = I gives X_I3 = -Q_I Xd_3 with Q_I = sum_{K=I..2} X_IK U_K3 (X_II = Xd_I), so all
// three row blocks are independent products.  Wave (H, ih) forms the Q^T half-tiles (H, I, ih)
// (48 MFMAs: A = U_K3^T from S, B = X_IK^T from Xd / Xo) -- in D layout they are the B operands
// of X_I3^T = -Xd_3^T Q_I^T directly -- the H = 0 waves pass theirs through Qs, and after one
// barrier each wave writes the X_I3 tiles of its column half (4 (H + 1) MFMAs each) and its
// X_33 tile: 48 + 24 MFMAs on the busiest wave against 144 dependent ones for a column half of
// the recurrence.  The X_I3^T D layout stores 16 consecutive rows per column (128-B segments).
// (two halves around the caller's barrier: the Q^T half-tiles, then the products and stores)
template <int H>
__device__ __forceinline__ void d2_tail_q(int ih, const lds_d* __restrict__ S,
                                          const lds_d (*__restrict__ Xd)[D2_PB],
                                          const lds_d* __restrict__ Xo, lds_d* __restrict__ Qs,
                                          int lane, d4v (&q)[3]) {
  const int n = 16 * ih + (lane & 15);  // row of block I (B operand column)
#pragma unroll
  for (int I = 0; I < 3; ++I) {
    q[I] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int K = I; K < 3; ++K)
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int k = 4 * st + (lane >> 4);
        const double a = S[pk(32 * K + k, 96 + 16 * H + (lane & 15))];
        double b;
        if (K == I) {
          const double v = Xd[I][pk(min(n, k), k)];
          b = n <= k ? v : 0.0;
        } else {
          b = Xo[(I + K - 1) * 32 * 33 + n * 33 + k];
        }
        q[I] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, q[I], 0, 0, 0);
      }
  }
  if constexpr (H == 0) {
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int r = 0; r < 4; ++r) Qs[((I * 2 + ih) * 4 + r) * 64 + lane] = q[I][r];
  }
}

template <int H, bool SC1>
__device__ __forceinline__ void d2_tail_out(int ih, const lds_d (*__restrict__ Xd)[D2_PB],
                                            const lds_d* __restrict__ Qs, const d4v (&q)[3],
                                            double* __restrict__ winv, int kb, int lane) {
  const int n = 16 * ih + (lane & 15);
  const int c = 16 * H + (lane & 15);  // column of block 3 (A operand row)
#pragma unroll
  for (int I = 0; I < 3; ++I) {
    d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int st = 0; st < 4 * (H + 1); ++st) {
      const int m = 4 * st + (lane >> 4);
      const double xv = Xd[3][pk(min(m, c), c)];
      const double b = (st >> 2) == H ? q[I][st & 3] : Qs[((I * 2 + ih) * 4 + (st & 3)) * 64 + lane];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(m <= c ? -xv : 0.0, b, acc, 0, 0, 0);
    }
    const int gr = 32 * I + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gc = 96 + 16 * H + (lane >> 4) + 4 * r;
      st_res<SC1>(&winv[gr + (size_t)gc * 128], (gr < kb && gc < kb) ? acc[r] : 0.0);
    }
  }
  {  // X_33 = Xd_3 (zero below the diagonal)
    const int gr = 96 + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cc = 16 * H + (lane >> 4) + 4 * r, gc = 96 + cc;
      const double v = Xd[3][pk(min(n, cc), cc)];
      st_res<SC1>(&winv[gr + (size_t)gc * 128], (n <= cc && gr < kb && gc < kb) ? v : 0.0);
    }
  }
}

// S <- the upper triangle of the kb x kb block at Ab (identity padding beyond kb), packed.
// Batched loads, 4 x 16 in flight: thread t owns row r = t % 128 of columns c0 + 2e.  Clamped
// addresses + select: every load is issued unconditionally (a branch around a load makes the
// compiler drain vmcnt on the other path, serialising the batch).
__device__ __forceinline__ void diag2_load(lds_d* __restrict__ S, const double* __restrict__ Ab,
                                           size_t lda, int kb) {
  constexpr int PER = D2_NB * D2_NB / DIAG_THREADS;
  const int tid = threadIdx.x;
  const int r = tid & (D2_NB - 1), c0 = tid >> 7;
  const double* src = Ab + min(r, kb - 1);
#pragma unroll 1
  for (int e0 = 0; e0 < PER; e0 += 16) {
    double v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = src[(size_t)min(c0 + 2 * (e0 + e), kb - 1) * lda];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = c0 + 2 * (e0 + e);
      if (r <= c) S[pk(r, c)] = (c < kb) ? v[e] : ((r == c) ? 1.0 : 0.0);
    }
  }
}

// Factor the block in S (packed upper, loaded, identity padding beyond kb; the caller has
// synchronised after filling it), write U to Ab (upper part only) and W = U^{-1} to winv
// (128 x 128, zero outside kb x kb).  Returns 0, or the global order (kglob + row + 1) of
// the first non-positive pivot -- then U is not written (W's workspace slot may hold its first
// column blocks).  Uniform across the workgroup.
// Xd: 4 x D2_PB doubles of LDS; fail: one int of LDS.
template <bool SC1, bool QTAIL = false>
__device__ __forceinline__ int diag2_core(lds_d* __restrict__ S, lds_d (*__restrict__ Xd)[D2_PB],
                                          lds_i* fail, double* __restrict__ Ab, size_t lda, int kb,
                                          int kglob, double* __restrict__ winv) {
  constexpr int NB = D2_NB, PER = NB * NB / DIAG_THREADS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wv == 0) *fail = 0;  // (wave-uniform branch)
  __syncthreads();
  DSTAMP_INIT();
#pragma unroll 1
  for (int sb = 0; sb < 4; ++sb) {
    const int K0 = 32 * sb, W = NB - K0;
    const int nsw = (W - 32) / 32;  // waves carrying strip columns; wave nsw carries I
    if (wv <= nsw) {
      const bool dl = lane < 32;
      const bool il = !dl && wv == nsw;
      const int c = dl ? lane : 32 + 32 * wv + (lane - 32);  // band column (D / strip)
      const int q = lane - 32;                                // identity column
      double x[32];
      // all 32 loads first, unconditionally (identity lanes read any valid address), then the
      // selects: with the select next to each load the compiler put every load in its own
      // exec-masked branch with its own lgkmcnt(0) wait -- 32 serialised LDS round trips
#pragma unroll
      for (int r = 0; r < 32; ++r) {
        const int cc = il ? r : c;
        x[r] = S[pk(K0 + min(r, cc), K0 + cc)];
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = 0; r < 32; ++r) x[r] = il ? (r == q ? 1.0 : 0.0) : ((dl && r > lane) ? 0.0 : x[r]);
      DSTAMPW(9);
      int bad = 0;
#ifndef D2_READLANE_ROWS
      // the pivot row through this wave's own LDS buffer: every lane writes its x[j] (lanes
      // 0-31 hold row j of the band's diagonal block), then every lane reads the entries it
      // needs as 16-B broadcasts -- one ds_write + (31 - j) / 2 ds_reads per step instead of
      // two v_readlane per entry.  A wave's LDS operations complete in order, so the next
      // step's write cannot overtake this step's reads; no other wave touches the buffer.
      lds_d* pivb = S + D2_PIV + 64 * wv;
#endif
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const double piv = readlane_d(x[j], j);
        bad = (bad == 0 && !(piv > 0.0)) ? j + 1 : bad;
        const double ri = rsqrt_nr(piv);
        const double u = piv * ri;
        const double xs = x[j] * ri;
        x[j] = dl ? (lane == j ? u : (lane < j ? x[j] : xs)) : xs;
#ifndef D2_READLANE_ROWS
        if (j < 31) {  // (a condition, not a break: the loop must stay fully unrolled)
        pivb[lane] = x[j];
        asm volatile("" ::: "memory");  // (compiler order only: the LDS unit keeps the wave's)
        // reads issued in groups of 8 pairs before the group's FMAs (left to itself the
        // compiler put every read in the same registers with a wait behind each)
#pragma unroll
        for (int g0 = (j + 1) & ~1; g0 < 32; g0 += 16) {
          d2v r2[8];
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (g0 + 2 * t < 32) r2[t] = *reinterpret_cast<const lds_d2v*>(pivb + g0 + 2 * t);
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
#else
        // row j to every lane in groups of 8: the readlanes of a group are issued back to
        // back (their latency overlaps), then the group's FMAs; sched barriers keep the
        // compiler from hoisting a whole step's readlanes (SGPR pressure)
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
#endif
      }
      DSTAMPW(10);
      if (dl) {
        if (wv == 0) {
#pragma unroll
          for (int r = 0; r < 32; ++r)
            if (r <= lane) S[pk(K0 + r, K0 + lane)] = x[r];
        }
      } else if (il) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
          if (r >= q) Xd[sb][pk(q, r)] = x[r];
      } else {
#pragma unroll
        for (int r = 0; r < 32; ++r) S[pk(K0 + r, K0 + c)] = x[r];
      }
      if (wv == 0 && lane == 0 && bad) *fail = kglob + K0 + bad;
      DSTAMPW(11);
    } else if (sb >= 2 && wv >= 2) {
      // W's early column blocks on the waves the band leaves idle (bands 2 and 3 keep only
      // waves 0-1 / wave 0 busy): column block J needs Xd_0..Xd_J and U's rows above band J,
      // all final once band J's F1 and barrier are past, so J = 0, 1 run beside band 2 and
      // J = 2 beside band 3, and only J = 3 is left after the last band
      const int jh = wv - 2;
      int ln = lane;  // (opaque: keeps the lane-derived LDS addresses from being hoisted out
      asm volatile("" : "+v"(ln));  // of the band loop, live across every elimination)
      lds_d* Xo = QTAIL ? S + D2_XO : nullptr;
      if (sb == 2) {
        d2_inv_colhalf<1, SC1>(jh, S, Xd, winv, kb, ln, Xo);
        d2_inv_colhalf<0, SC1>(jh, S, Xd, winv, kb, ln);
      } else {
        d2_inv_colhalf<2, SC1>(jh, S, Xd, winv, kb, ln, Xo);
      }
    }
    __syncthreads();
    if (sb == 0) STAMP(5);
    DSTAMP(2 * sb);
    const int f = __builtin_amdgcn_readfirstlane(*fail);  // uniform branch around barriers
    if (f) return f;
    const int R = W - 32;
    if (R <= 0) break;
    // F3: U(r, c) -= sum_p U(K0+p, r) U(K0+p, c) for K0+32 <= r <= c < NB, on MFMA.  A wave
    // takes two 16 x 16 tiles per pass (t and t + 4): every operand and the old values are
    // loaded first (a sched barrier keeps the compiler from sinking each load next to its
    // MFMA, which serialised load -> wait -> MFMA), then the two tiles' MFMA chains interleave
    {
      const int nt = R / 16, B0 = K0 + 32;
      const int ntile = nt * (nt + 1) / 2;
      auto tile_of = [&](int t, int& r0, int& q0) {
        int tj = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
        while ((tj + 1) * (tj + 2) / 2 <= t) ++tj;
        while (tj * (tj + 1) / 2 > t) --tj;
        r0 = B0 + 16 * (t - tj * (tj + 1) / 2);
        q0 = B0 + 16 * tj;
      };
      for (int t = wv; t < ntile; t += 2 * (DIAG_THREADS / 64)) {
        const int t1 = t + DIAG_THREADS / 64;
        const bool two = t1 < ntile;  // (wave-uniform)
        int r0, q0, r1, q1;
        tile_of(t, r0, q0);
        tile_of(two ? t1 : t, r1, q1);
        double av0[8], bv0[8], av1[8], bv1[8], o0[4], o1[4];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int p = K0 + 4 * kk + (lane >> 4);
          av0[kk] = S[pk(p, r0 + (lane & 15))];
          bv0[kk] = S[pk(p, q0 + (lane & 15))];
          av1[kk] = S[pk(p, r1 + (lane & 15))];
          bv1[kk] = S[pk(p, q1 + (lane & 15))];
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int c0 = q0 + (lane & 15), rr0 = min(r0 + (lane >> 4) + 4 * qq, c0);
          const int c1 = q1 + (lane & 15), rr1 = min(r1 + (lane >> 4) + 4 * qq, c1);
          o0[qq] = S[pk(rr0, c0)];
          o1[qq] = S[pk(rr1, c1)];
        }
        __builtin_amdgcn_sched_barrier(0);
        d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {  // (the barriers keep the two chains interleaved)
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0[kk], bv0[kk], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av1[kk], bv1[kk], acc1, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
        // branch-free stores: entries below the diagonal (and the second tile when !two) go to
        // this wave's pivot-row buffer, unused here -- with exec-masked stores the compiler
        // sank the second chain's MFMAs behind the first tile's stores
        lds_d* dump = S + D2_PIV + 64 * wv + lane;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int r = r0 + (lane >> 4) + 4 * qq, c = q0 + (lane & 15);
          *(r <= c ? S + pk(r, c) : dump) = o0[qq] - acc0[qq];
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int r = r1 + (lane >> 4) + 4 * qq, c = q1 + (lane & 15);
          *(two && r <= c ? S + pk(r, c) : dump) = o1[qq] - acc1[qq];
        }
      }
    }
    __syncthreads();
    if (sb == 0) STAMP(6);
    DSTAMP(2 * sb + 1);
  }
  STAMP(2);
  // U back to global (fire-and-forget; nothing below waits for these stores).  Ab = nullptr:
  // the caller stores U later (diag2_store_u) -- the tile-DAG, where no task of the launch
  // reads a diagonal tile, publishes W first
  if (Ab) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = tid + e * DIAG_THREADS;
      const int r = idx % NB, c = idx / NB;
      if (r < kb && c < kb && r <= c) st_res<SC1>(&Ab[(size_t)r + (size_t)c * lda], S[pk(r, c)]);
    }
  }
  // W = U^-1: the last column block, one wave per column half (blocks 0-2 went out beside
  // bands 2 and 3).  In one phase here, waves 2-3 (blocks 2, 1, 0: 112 MFMAs and three
  // halves' stores) ran 24.0k cycles against 15.3-17.6k for waves 0-1 (block 3: 144 MFMAs),
  // tools/probe/inv_probe
  if constexpr (QTAIL) {  // wave (H, ih) = (wv / 2, wv % 2)
    d4v q[3];
    if (wv < 2)
      d2_tail_q<0>(wv, S, Xd, S + D2_XO, S + D2_QS, lane, q);
    else
      d2_tail_q<1>(wv - 2, S, Xd, S + D2_XO, S + D2_QS, lane, q);
    __syncthreads();  // the H = 0 half-tiles are in Qs
    if (wv < 2)
      d2_tail_out<0, SC1>(wv, Xd, S + D2_QS, q, winv, kb, lane);
    else
      d2_tail_out<1, SC1>(wv - 2, Xd, S + D2_QS, q, winv, kb, lane);
  } else if (wv < 2) {
    d2_inv_colhalf<3, SC1>(wv, S, Xd, winv, kb, lane);
  }
  STAMP(4);
  DSTAMP(7);
  return 0;
}

// U (kb x kb upper, from S) to Ab: plain stores (read by later launches only), or sc1
// (write-through: read by another stream's kernel while this launch runs)
template <bool SC1>
__device__ __forceinline__ void diag2_store_u(const lds_d* __restrict__ S, double* __restrict__ Ab,
                                              size_t lda, int kb) {
  constexpr int NB = D2_NB, PER = NB * NB / DIAG_THREADS;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int idx = threadIdx.x + e * DIAG_THREADS;
    const int r = idx % NB, c = idx / NB;
    if (r < kb && c < kb && r <= c) st_res<SC1>(&Ab[(size_t)r + (size_t)c * lda], S[pk(r, c)]);
  }
}

}  // namespace
