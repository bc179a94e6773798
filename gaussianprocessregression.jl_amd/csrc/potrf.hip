// Blocked upper Cholesky (dpotrf 'U'), triangular solves and K^{-1} on gfx950.
//
// Replaces cholesky!(Hermitian(K)) (src/cost.jl:77,87,104, src/predict.jl:31),
// ldiv!(alpha, kchol, y) (src/cost.jl:79, src/predict.jl:32), rdiv!(Kxp, U)
// (src/predict.jl:84,90,98) and K^{-1} = ldiv!(kchol, I) (src/cost.jl:90-92).
//
// Right-looking blocked algorithm, panel width nb (64/128).  Per panel k:
//   1. diag kernel (one workgroup, block resident in LDS): U_kk = chol(A_kk) in place and
//      the inverse U_kk^{-1} into a per-block workspace slot (kept for later solves);
//   2. panel TRSM as an MFMA GEMM:  U_k,rest = U_kk^{-T} A_k,rest   (in place);
//   3. trailing SYRK on MFMA:       A_rest,rest -= U_k,rest^T U_k,rest  (upper tiles only).
// The lower triangle of A is never written (dpotrf semantics: test/test_loss.jl:46).
// Non-PD pivots set a device info word (order of the failing minor, LAPACK convention);
// every later kernel of the factorisation reads it and exits.
#include <cmath>

#include "common.hpp"

#ifdef GPR_DIAG_STAMPS
// diagnostic build only (tools/gemm_bench): wall-clock stamps of the diag kernel phases
__device__ unsigned long long g_diag_stamps[16];
#define STAMP(i)                                                                       \
  do {                                                                                 \
    __syncthreads();                                                                   \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_diag_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" void gpr_debug_diag_stamps(unsigned long long* out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_stamps), sizeof(unsigned long long) * 16);
}
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

#include "diag_block.hpp"

namespace {

// ---- blocked diagonal-block kernel ------------------------------------------------------
// Factor (mode 1) / only invert (mode 0) one NB x NB diagonal block, blocked by SB = 32:
//   per sub-block K0:  A1 all 4 waves factor the 32x32 diagonal sub-block (thread owns
//                         4 elements; one barrier per step; pivot via rsq + Newton),
//                      A2 strip TRSM  U(K0:K0+32, K0+32:) = D^{-T} S(...)  (thread/column),
//                      A3 trailing update of the rest of the block on FP64 MFMA.
//   inverse X = U^{-1}: B1 one wave per 32x32 diagonal sub-block inverts it in registers,
//                       B2 off-diagonal blocks by super-diagonal levels on MFMA,
//                          X_IJ = -X_II T,  T = sum_{K=I+1..J} U_IK X_KJ  (T never leaves
//                          the accumulators: the f64 MFMA D layout of register q is exactly
//                          the B-operand layout of k-step 4q).
// Everything runs out of LDS/registers: the block is fetched with ONE batch of loads and
// written back with fire-and-forget stores, because this kernel sits on the critical path
// of the lookahead chain while the trailing SYRK saturates HBM (a dependent global round
// trip then costs microseconds).  LDS is kept to ~84 KB (U packed + the diagonal blocks
// of U^{-1}) so the kernel fits on a CU beside ONE trailing-update GEMM workgroup: with a
// full-CU footprint it waited ~0.7 ms per call for a CU to drain (measured).  Off-diagonal
// blocks of U^{-1} go straight to the workspace slot and are re-read by B2 with one batched
// prefetch per tile.  Padding beyond kb is the identity.

template <int NB>
__device__ __forceinline__ void diag_block_body(double* __restrict__ A, size_t lda, int n,
                                                int kglob, int* __restrict__ info,
                                                double* __restrict__ winv, int mode, int blk) {
  constexpr int SB = 32, NSB = NB / SB, NW = DIAG_THREADS / 64;
  constexpr int PK = NB * (NB + 1) / 2;
  constexpr int PER = NB * NB / DIAG_THREADS;  // elements per thread in the bulk copies
  constexpr int PB = SB * (SB + 1) / 2;
  __shared__ double S[PK];        // U, packed upper (66 KB at NB = 128)
  __shared__ double Xd[NSB][PB];  // diagonal 32x32 blocks of U^{-1}, packed upper (17 KB)
  __shared__ double rb[2][NB];
  __shared__ double wbuf[NW][SB];
  __shared__ int fail;
  if (*info != 0) return;
  // this latency-bound chain shares CUs with the MFMA-saturating trailing update: take
  // issue priority over the co-resident GEMM waves (FP64 VALU and FP64 MFMA share the
  // SIMD's FP64 throughput on gfx950)
  __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  int k0, kb;
  if (mode == 1) {
    k0 = kglob;
    kb = min(NB, n - kglob);
  } else {
    k0 = blk * NB;
    kb = min(NB, n - k0);
    winv += (size_t)blk * NB * NB;
  }
  double* Ab = A + (size_t)k0 + (size_t)k0 * lda;
  STAMP(0);
  // batched loads (16 in flight per thread per batch, 4 batches at NB = 128), then LDS
  constexpr int CH = PER < 16 ? PER : 16;
#pragma unroll 1
  for (int e0 = 0; e0 < PER; e0 += CH) {
    double v[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {  // clamped address + select: no branch around the load
      const int idx = tid + (e0 + e) * DIAG_THREADS;
      const int r = idx % NB, c = idx / NB;
      const double g = Ab[(size_t)min(r, kb - 1) + (size_t)min(c, kb - 1) * lda];
      v[e] = (r <= c && c < kb) ? g : ((r == c) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int idx = tid + (e0 + e) * DIAG_THREADS;
      const int r = idx % NB, c = idx / NB;
      if (r <= c) S[pk(r, c)] = v[e];
    }
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  STAMP(1);
  if (mode == 1) {
    // A1+A2 ownership in the 32-row band [K0, K0+32) x [K0, NB): thread owns rows
    // 4 rg + i (i < 4) of columns K0 + cc + 32 cb (cb < NCB).  Row j = 4 jo + jl lives in
    // slot i = jl (compile-time in the unroll-by-4 inner loop) of the threads rg == jo.
    constexpr int NCB = NB / SB;
    const int cc = tid & 31, rg = tid >> 5;
    for (int sb = 0; sb < NSB; ++sb) {
      const int K0 = sb * SB;
      const int W = NB - K0;  // band width
      // ---- A1+A2: right-looking factorisation of the band (pivots in its first 32 cols)
      double d[4][NCB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rg + i, c = cc + 32 * cb;
          d[i][cb] = (c < W && r <= c) ? S[pk(K0 + r, K0 + c)] : 0.0;
        }
      int bad = 0;
#pragma unroll 1
      for (int jo = 0; jo < SB / 4; ++jo) {
#pragma unroll
        for (int jl = 0; jl < 4; ++jl) {
          const int j = 4 * jo + jl;
          double* b = rb[jl & 1];
          if (rg == jo) {  // owners of band row j publish it
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) b[cc + 32 * cb] = d[jl][cb];
          }
          __syncthreads();
          const double piv = b[j];
          bad = (bad == 0 && !(piv > 0.0)) ? j + 1 : bad;
          const double ri = rsqrt_nr(piv);
          const double u = piv * ri;
          double uc[NCB], ur[4];
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            const int c = cc + 32 * cb;
            const double bc = b[c];
            uc[cb] = (c > j) ? bc * ri : 0.0;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * rg + i;
            const double br = b[r];
            ur[i] = (r > j) ? br * ri : 0.0;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
              const double upd = fma(-ur[i], uc[cb], d[i][cb]);
              if (i == jl) {  // compile-time: this slot holds row j in the owner threads
                const int c = cc + 32 * cb;
                const double rowj = (c == j) ? u : ((c > j) ? uc[cb] : d[i][cb]);
                d[i][cb] = (rg == jo) ? rowj : upd;
              } else {
                d[i][cb] = upd;
              }
            }
        }
      }
      if (bad) {
        if (tid == 0) fail = kglob + K0 + bad;
      } else {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * rg + i, c = cc + 32 * cb;
            if (c < W && r <= c) S[pk(K0 + r, K0 + c)] = d[i][cb];
          }
      }
      __syncthreads();
      if (sb == 0) STAMP(5);
      if (fail) {
        if (tid == 0) *info = fail;
        return;
      }
      const int R = NB - K0 - SB;  // rows/cols of the block after this sub-block
      if (R <= 0) break;
      if (sb == 0) STAMP(6);
      // ---- A3: U(r, c) -= sum_p U(K0+p, r) U(K0+p, c) for K0+32 <= r <= c < NB, on MFMA
      {
        const int nt = R / 16, B0 = K0 + SB;
        const int ntile = nt * (nt + 1) / 2;
        for (int t = wv; t < ntile; t += NW) {
          int tj = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
          while ((tj + 1) * (tj + 2) / 2 <= t) ++tj;
          while (tj * (tj + 1) / 2 > t) --tj;
          const int ti = t - tj * (tj + 1) / 2;
          const int r0 = B0 + 16 * ti, q0 = B0 + 16 * tj;
          d4v acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < SB; kk += 4) {
            const int p = K0 + kk + (lane >> 4);
            const double av = S[pk(p, r0 + (lane & 15))];
            const double bv = S[pk(p, q0 + (lane & 15))];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = r0 + (lane >> 4) + 4 * q, c = q0 + (lane & 15);
            if (r <= c) S[pk(r, c)] -= acc[q];
          }
        }
      }
      __syncthreads();
      if (sb == 0) STAMP(7);
    }
  }
  STAMP(2);
  // U (upper) back to global (mode 1): fire-and-forget stores
  if (mode == 1) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = tid + e * DIAG_THREADS;
      const int r = idx % NB, c = idx / NB;
      if (r < kb && c < kb && r <= c) Ab[(size_t)r + (size_t)c * lda] = S[pk(r, c)];
    }
  }
  STAMP(3);
  // ---- B1: wave w inverts diagonal sub-blocks w, w+NW, ... : X D = I, right-looking over
  // columns r; lane holds X[16h+i][c32]
  const int c32 = lane & 31, h = lane >> 5;
  for (int sbi = wv; sbi < NSB; sbi += NW) {
    const int K0 = sbi * SB;
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = (16 * h + i == c32) ? 1.0 : 0.0;
    double* cb = wbuf[wv];
#pragma unroll 2
    for (int r = 0; r < SB; ++r) {
      const double ir = 1.0 / S[pk(K0 + r, K0 + r)];
      if (c32 == r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          x[i] = x[i] * ir;  // rows i > r are zero here
          cb[16 * h + i] = x[i];
        }
      }
      wave_fence();
      const double urc = S[pk(K0 + min(r, c32), K0 + c32)];
      const double uv = (c32 > r) ? urc : 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ii = 16 * h + i;
        const double xv = cb[ii];
        if (ii <= r) x[i] = fma(-xv, uv, x[i]);
      }
      wave_fence();
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ii = 16 * h + i;
      if (ii <= c32) Xd[sbi][pk(ii, c32)] = x[i];
      // the diagonal block also goes to the workspace slot (zero below its diagonal)
      const bool in = (K0 + ii < kb) && (K0 + c32 < kb);
      winv[(K0 + ii) + (size_t)(K0 + c32) * NB] = (ii <= c32 && in) ? x[i] : 0.0;
    }
  }
  // zero the slot below the diagonal blocks (off-diagonal lower blocks)
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int idx = tid + e * DIAG_THREADS;
    const int r = idx % NB, c = idx / NB;
    if ((r >> 5) > (c >> 5)) winv[idx] = 0.0;
  }
  __syncthreads();
  // ---- B2: off-diagonal blocks, level by level; one wave per 16x16 output tile
  for (int dl = 1; dl < NSB; ++dl) {
    const int nblk = NSB - dl;
    for (int t = wv; t < nblk * 4; t += NW) {
      const int I = t >> 2, ih = t & 1, jh = (t >> 1) & 1, J = I + dl;
      const int jc = J * SB + 16 * jh + (lane & 15);  // output column (B-operand column)
      // T[:, jh] for both 16-row halves of the I block: T = sum_K U_IK X_KJ.
      // X_KJ (K < J) comes from the workspace (previous levels): prefetch it in one batch.
      d4v T0 = {0.0, 0.0, 0.0, 0.0}, T1 = {0.0, 0.0, 0.0, 0.0};
      double bpre[(NSB - 2) * (SB / 4) > 0 ? (NSB - 2) * (SB / 4) : 1];
#pragma unroll
      for (int Kb2 = 0; Kb2 < NSB - 2; ++Kb2) {
        const int Kb = I + 1 + Kb2;
#pragma unroll
        for (int kq = 0; kq < SB / 4; ++kq) {
          const int k = Kb * SB + 4 * kq + (lane >> 4);
          bpre[Kb2 * (SB / 4) + kq] = (Kb < J) ? winv[k + (size_t)jc * NB] : 0.0;
        }
      }
#pragma unroll
      for (int Kb2 = 0; Kb2 < NSB - 1; ++Kb2) {
        const int Kb = I + 1 + Kb2;
        if (Kb > J) break;
#pragma unroll
        for (int kq = 0; kq < SB / 4; ++kq) {
          const int kl = 4 * kq + (lane >> 4), k = Kb * SB + kl;
          double bv;
          if (Kb == J) {  // X_JJ from LDS
            const int jl = jc - J * SB;
            const double xv = Xd[J][pk(min(kl, jl), jl)];
            bv = (kl <= jl) ? xv : 0.0;
          } else {
            bv = bpre[Kb2 * (SB / 4) + kq];
          }
          const double a0 = S[pk(I * SB + (lane & 15), k)];       // U(i, k), i < k
          const double a1 = S[pk(I * SB + 16 + (lane & 15), k)];
          T0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bv, T0, 0, 0, 0);
          T1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv, T1, 0, 0, 0);
        }
      }
      // X_IJ[ih rows, jh cols] = - sum_m X_II[i][m] T[m][j]; T register q = k-step 4q
      d4v acc = {0.0, 0.0, 0.0, 0.0};
      const int il = 16 * ih + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ml = 4 * q + (lane >> 4);
        const double xv = Xd[I][pk(min(il, ml), ml)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64((il <= ml) ? xv : 0.0, T0[q], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ml = 16 + 4 * q + (lane >> 4);
        const double xv = Xd[I][pk(min(il, ml), ml)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64((il <= ml) ? xv : 0.0, T1[q], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = I * SB + 16 * ih + (lane >> 4) + 4 * q;
        winv[i + (size_t)jc * NB] = (i < kb && jc < kb) ? -acc[q] : 0.0;
      }
    }
    __syncthreads();  // workgroup-scope fence: this level's X blocks visible to the next
  }
  STAMP(4);
#ifdef GPR_DIAG_STAMPS
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    atomicAdd(&g_diag_stamps[8], g_diag_stamps[4] - g_diag_stamps[0]);
    atomicAdd(&g_diag_stamps[9], 1ull);
  }
#endif
}

template <int NB>
__global__ __launch_bounds__(DIAG_THREADS, 2) void diag_block_kernel(double* __restrict__ A,
                                                                  size_t lda, int n, int kglob,
                                                                  int* __restrict__ info,
                                                                  double* __restrict__ winv,
                                                                  int mode) {
  diag_block_body<NB>(A, lda, n, kglob, info, winv, mode, blockIdx.x);
}

// One 128-block (factor mode) per launch; the body is diag_block.hpp's diag2_core.
// <= 256 registers per wave: the kernel must fit on a CU beside one running trailing-update
// workgroup (224 registers per wave), or it waits for the CU to drain
// The block lives in DYNAMIC LDS (DIAG2_LDS bytes at launch): with 84 KB of static LDS the
// compiler sees that two workgroups cannot share a CU, drops the 2-per-CU register target and
// allocates ~310 registers per wave, and the kernel would no longer fit beside a trailing-
// update workgroup (224 registers per wave).
constexpr size_t DIAG2_LDS = sizeof(double) * D2_LDS_DOUBLES;
__global__ __launch_bounds__(DIAG_THREADS, 2) void diag2_kernel(double* __restrict__ A, size_t lda,
                                                                int n, int kglob,
                                                                int* __restrict__ info,
                                                                double* __restrict__ winv) {
  extern __shared__ double dsm[];
  lds_d* S = (lds_d*)dsm;                                        // U, packed upper (66 KB)
  lds_d(*Xd)[D2_PB] = reinterpret_cast<lds_d(*)[D2_PB]>(S + D2_PK);  // U^-1 diag blocks
  lds_i* fail = reinterpret_cast<lds_i*>(S + D2_PK + 4 * D2_PB);
  if (*info != 0) return;
  // this latency-bound chain shares CUs with the MFMA-saturating trailing update: take
  // issue priority over the co-resident GEMM waves
  __builtin_amdgcn_s_setprio(3);
  const int kb = min(D2_NB, n - kglob);
  double* Ab = A + (size_t)kglob + (size_t)kglob * lda;
  STAMP(0);
  diag2_load(S, Ab, lda, kb);
  STAMP(1);
  const int f = diag2_core<false>(S, Xd, fail, Ab, lda, kb, kglob, winv);
  if (f && threadIdx.x == 0) *info = f;
#ifdef GPR_DIAG_STAMPS
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    g_diag_stamps[3] = g_diag_stamps[2];
    atomicAdd(&g_diag_stamps[8], g_diag_stamps[4] - g_diag_stamps[0]);
    atomicAdd(&g_diag_stamps[9], 1ull);
  }
#endif
}

// ---- square-panel factorisation: one launch per outer panel ------------------------------
// Factors the kw x kw diagonal square of the outer row panel in place (U upper, lower
// untouched), writes each 128-block's inverse to its winv slot, and forms the square's
// inverse U_sq^{-1} (kw x kw, ld kw, only blocks on/above the diagonal) so the rest of the
// row panel is ONE GEMM (X = U_sq^{-T} A_rest).  Before this, the panel took 8 diag launches
// and 16 GEMM launches per outer step, each waiting ~0.3 ms for a CU slot beside the
// trailing SYRK (trace r01).
//
// Workgroup c (ticket order) owns column tile c (128 columns) of the square.  Step j:
// workgroup j factors block (j, j) (diag_block_body) and publishes; workgroup c > j forms
// U(j, c) = W_j^T A(j, c) in place, publishes, then updates A(i, c) -= U(j, i)^T U(j, c) for
// j < i <= c (U(j, i) from workgroup i).  prog[c] counts the final strips of tile c.  Data
// crosses workgroups only after its final write and through agent-scope release/acquire
// (MI355X guide, inter-workgroup visibility); no workgroup reads another's block before the
// flag that publishes it, so no XCD can hold a stale copy of it.  Inverse, block column c
// (workgroup c): X_cc = W_c, X_ic = -W_i sum_{t=i+1..c} U(i, t) X_tc for i = c-1 .. 0.

// acc[bi][bj][r] += sum_t P[m*pm + t*pt] Q[t*qt + n*qn] for the wave's 64x64 share of a
// 128x128 tile: m = 64 (w & 1) + 16 bi + (lane >> 4) + 4 r... (A-operand rows), n = 64 (w >> 1)
// + 16 bj + (lane & 15).  Operands come straight from L2 (small, hot blocks).
__device__ __forceinline__ void sq_mma(d4v (&acc)[4][4], const double* __restrict__ P,
                                       size_t pm, size_t pt, const double* __restrict__ Q,
                                       size_t qt, size_t qn, int K, int mv, int nv) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mb = 64 * (w & 1), nbase = 64 * (w >> 1);
#pragma unroll 8
  for (int t0 = 0; t0 < K; t0 += 4) {
    const int t = t0 + (lane >> 4);
    double a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mb + 16 * i + (lane & 15);
      a[i] = (t < K && m < mv) ? P[(size_t)m * pm + (size_t)t * pt] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nn = nbase + 16 * j + (lane & 15);
      b[j] = (t < K && nn < nv) ? Q[(size_t)t * qt + (size_t)nn * qn] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// LDS-staged form of sq_mma (16-deep K chunks, register-prefetched, double-buffered).
// PM: P is m-contiguous (element (m, t) at P[m + t*pld]); else t-contiguous (P[t + m*pld]).
// Q element (t, n) at Q[t + n*qld].  lds: 2 buffers x (P image 128x16 + Q image 128x16).
// Images use the GEMM kernel's swizzled [row][16] layout (conflict-free ds_read_b128).
constexpr int SQ_KC = 16;
__device__ __forceinline__ int sq_idx(int row, int chunk) {
  return row * SQ_KC + ((chunk ^ ((row >> 1) & 7)) << 1);
}
template <bool PM>
__device__ __forceinline__ void sq_gemm(d4v (&acc)[4][4], const double* __restrict__ P, size_t pld,
                                        const double* __restrict__ Q, size_t qld, int K, int mv,
                                        int nv, double* lds) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int mb = 64 * (w & 1), nbase = 64 * (w >> 1);
  const int nch = (K + SQ_KC - 1) / SQ_KC;
  double rp[8], rq[8];
  auto gload = [&](int c) {
    const int t0 = c * SQ_KC;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 256 * r;
      int m, t;
      if (PM) { m = e & 127; t = e >> 7; } else { m = e >> 4; t = e & 15; }
      const bool ok = m < mv && t0 + t < K;
      rp[r] = ok ? (PM ? P[(size_t)m + (size_t)(t0 + t) * pld] : P[(size_t)(t0 + t) + (size_t)m * pld]) : 0.0;
      const int nn = e >> 4, tq = e & 15;
      rq[r] = (nn < nv && t0 + tq < K) ? Q[(size_t)(t0 + tq) + (size_t)nn * qld] : 0.0;
    }
  };
  auto lstore = [&](int buf) {
    double* pi = lds + buf * 4096;
    double* qi = pi + 2048;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 256 * r;
      int m, t;
      if (PM) { m = e & 127; t = e >> 7; } else { m = e >> 4; t = e & 15; }
      pi[sq_idx(m, t >> 1) + (t & 1)] = rp[r];
      const int nn = e >> 4, tq = e & 15;
      qi[sq_idx(nn, tq >> 1) + (tq & 1)] = rq[r];
    }
  };
  __syncthreads();  // LDS free (previous users done)
  gload(0);
  lstore(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) gload(c + 1);
    const double* pi = lds + (c & 1) * 4096;
    const double* qi = pi + 2048;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = (lane >> 4) + 4 * p;
      d2 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const d2*>(&pi[sq_idx(mb + 16 * i + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const d2*>(&qi[sq_idx(nbase + 16 * j + (lane & 15), ch)]);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i][h], b[j][h], acc[i][j], 0, 0, 0);
    }
    if (c + 1 < nch) lstore((c + 1) & 1);
    __syncthreads();
  }
}

__device__ __forceinline__ void sq_zero(d4v (&acc)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4v{0.0, 0.0, 0.0, 0.0};
}

// C[m*cm + n*cn] = alpha acc + beta C for m < mv, n < nv (and m <= n when upper)
__device__ __forceinline__ void sq_store(const d4v (&acc)[4][4], double* C, size_t cm, size_t cn,
                                         double alpha, double beta, int mv, int nv, bool upper) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mb = 64 * (w & 1), nbase = 64 * (w >> 1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + 16 * i + (lane >> 4) + 4 * r, nn = nbase + 16 * j + (lane & 15);
        if (m < mv && nn < nv && (!upper || m <= nn)) {
          double* p = C + (size_t)m * cm + (size_t)nn * cn;
          *p = beta != 0.0 ? fma(beta, *p, alpha * acc[i][j][r]) : alpha * acc[i][j][r];
        }
      }
}
// ---- small-RHS triangular solves (TRSV-like, nrhs <= 16 per launch) --------------------
constexpr int RHS_CHUNK = 16;

// y_b <- W^T y_b (trans = 1) or W y_b (trans = 0), W = U_bb^{-1} upper (nb x nb).
__global__ __launch_bounds__(256) void trsv_diag_kernel(const double* __restrict__ W, int nb,
                                                        int kb, double* __restrict__ y,
                                                        size_t ldy, int nrhs, int trans) {
  __shared__ double ys[128 * RHS_CHUNK];
  for (int idx = threadIdx.x; idx < kb * nrhs; idx += 256) {
    const int k = idx % kb, c = idx / kb;
    ys[k + c * 128] = y[(size_t)k + (size_t)c * ldy];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < kb * nrhs; idx += 256) {
    const int m = idx % kb, c = idx / kb;
    double s = 0.0;
    if (trans) {
      for (int k = 0; k <= m; ++k) s = fma(W[k + (size_t)m * nb], ys[k + c * 128], s);
    } else {
      for (int k = m; k < kb; ++k) s = fma(W[m + (size_t)k * nb], ys[k + c * 128], s);
    }
    y[(size_t)m + (size_t)c * ldy] = s;
  }
}

// y[r] -= sum_k U[k + r*ldu] x[k]  for r in [0, nr)  (column r of the row panel, contiguous
// in k): one wave per column r.
__global__ __launch_bounds__(256) void gemv_t_update_kernel(const double* __restrict__ U,
                                                            size_t ldu, int kb, int nr,
                                                            const double* __restrict__ x,
                                                            size_t ldx, double* __restrict__ y,
                                                            size_t ldy, int nrhs) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nr) return;
  const double* col = U + (size_t)r * ldu;
  const double u0 = lane < kb ? col[lane] : 0.0;
  const double u1 = lane + 64 < kb ? col[lane + 64] : 0.0;
  for (int c = 0; c < nrhs; ++c) {
    const double* xc = x + (size_t)c * ldx;
    double s = u0 * (lane < kb ? xc[lane] : 0.0);
    s = fma(u1, lane + 64 < kb ? xc[lane + 64] : 0.0, s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) y[(size_t)r + (size_t)c * ldy] -= s;
  }
}

// y[r] -= sum_k U[r + k*ldu] x[k] for r in [0, nr): thread per r (coalesced over r).
__global__ __launch_bounds__(256) void gemv_n_update_kernel(const double* __restrict__ U,
                                                            size_t ldu, int kb, int nr,
                                                            const double* __restrict__ x,
                                                            size_t ldx, double* __restrict__ y,
                                                            size_t ldy, int nrhs) {
  __shared__ double xs[128 * RHS_CHUNK];
  for (int idx = threadIdx.x; idx < kb * nrhs; idx += 256) {
    const int k = idx % kb, c = idx / kb;
    xs[k + c * 128] = x[(size_t)k + (size_t)c * ldx];
  }
  __syncthreads();
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nr) return;
  double acc[RHS_CHUNK];
  for (int c = 0; c < RHS_CHUNK; ++c) acc[c] = 0.0;
  for (int k = 0; k < kb; ++k) {
    const double u = U[(size_t)r + (size_t)k * ldu];
#pragma unroll
    for (int c = 0; c < RHS_CHUNK; ++c)
      if (c < nrhs) acc[c] = fma(u, xs[k + c * 128], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < RHS_CHUNK; ++c)
    if (c < nrhs) y[(size_t)r + (size_t)c * ldy] -= acc[c];
}

// ---- single-launch blocked triangular sweeps (dpotrs, 1-2 right-hand sides per launch, nb = 128) ------------
// One workgroup per 128-row block, handed out by an atomic ticket so that every block a
// workgroup depends on belongs to a workgroup that is already running. Block results are
// published in order (a block can only finish after all blocks before it in the sweep), so
// one monotonic "blocks done" counter replaces per-block flags. Producer: plain stores ->
// vmcnt drain -> barrier -> agent release -> relaxed counter store; consumer: relaxed poll
// by lane 0 of each wave -> agent acquire -> loads (MI355X guide, inter-workgroup hand-off).
// The hand-off vector lives in its own buffer (hand) that is never read before it is
// written inside the launch, so no L2 line of it can be stale on another XCD.
// sync[0] = ticket, sync[1] = blocks done; both zeroed before the launch.
constexpr int SW_NB = 128, SW_THREADS = 512, SW_COLS = SW_NB / (SW_THREADS / 64);

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// SWEEP_SC1 (default): the hand-off vector is written and read ONLY with sc1 (L2-coherent,
// write-through) accesses and the counter is an sc1 store polled by sc1 loads, each polling
// wave loading only after its own poll matched -- MI355X_MICROARCH.md's first sc1 hand-off
// row (hipMalloc memory, one workgroup per CU), which needs neither the producer's L2
// write-back (release, 1.7-6.5 us) nor the consumer's L1 invalidate (acquire, 1.7-7 us) on
// each of the 256 hops of a sweep.  SWEEP_SC1=0: plain accesses behind agent fences.
#ifndef SWEEP_SC1
#define SWEEP_SC1 1
#endif
__device__ __forceinline__ double hand_ld(const double* p) {
#if SWEEP_SC1
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  return *p;
#endif
}
__device__ __forceinline__ void hand_st(double* p, double v) {
#if SWEEP_SC1
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}

// Block until at least `need` blocks are published; `known` caches the last observed count.
__device__ __forceinline__ void sweep_wait(int* sync, int need, int& known, int lane) {
  if (known >= need) return;
  int v = 0;
  if (lane == 0) {
    while ((v = __hip_atomic_load(&sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need)
      __builtin_amdgcn_s_sleep(1);
  }
  known = __shfl(v, 0);
#if SWEEP_SC1
  // no instruction: keeps the compiler from hoisting the sc1 hand-off loads above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

__device__ __forceinline__ void sweep_publish(int* sync, int value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
  __syncthreads();
  if (threadIdx.x == 0) {
#if !SWEEP_SC1
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __hip_atomic_store(&sync[1], value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Forward sweep U^T z = b: block b needs sum_{k<b} U[k-rows, b-cols]^T z_k, a column-dot per
// b-column; each lane keeps partial dots over rows (2l, 2l+1) for its wave's 16 columns and
// reduces across the wave once at the end. Then z_b = W_b^T r_b (W_b = U_bb^{-1}).
template <int NR>
__global__ __launch_bounds__(SW_THREADS) void trsv_fwd_sweep_kernel(
    const double* __restrict__ U, size_t ldu, int n, const double* __restrict__ W,
    double* __restrict__ B, size_t ldb, double* hand, int* sync) {
  __shared__ int sblk;
  __shared__ double rs[SW_NB * NR];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) sblk = atomicAdd(&sync[0], 1);
  __syncthreads();
  const int b = sblk;
  const int c0 = b * SW_NB, kb = min(SW_NB, n - c0);
  const int i0 = 2 * lane;
  const double* Wb = W + (size_t)b * SW_NB * SW_NB;
  double w0[SW_COLS], w1[SW_COLS];
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj) {
    const int j = w * SW_COLS + jj;
    const double* col = Wb + (size_t)j * SW_NB;
    w0[jj] = (j < kb && i0 <= j) ? col[i0] : 0.0;
    w1[jj] = (j < kb && i0 + 1 <= j) ? col[i0 + 1] : 0.0;
  }
  double p[SW_COLS][NR];
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj)
#pragma unroll
    for (int r = 0; r < NR; ++r) p[jj][r] = 0.0;
  int known = 0;
  for (int k = 0; k < b; ++k) {
    const double* tile = U + (size_t)k * SW_NB + i0 + (size_t)(c0 + w * SW_COLS) * ldu;
    double u0[SW_COLS], u1[SW_COLS];
#pragma unroll
    for (int jj = 0; jj < SW_COLS; ++jj) {
      const bool ok = w * SW_COLS + jj < kb;
      u0[jj] = ok ? tile[(size_t)jj * ldu] : 0.0;
      u1[jj] = ok ? tile[(size_t)jj * ldu + 1] : 0.0;
    }
    sweep_wait(sync, k + 1, known, lane);
    double z0[NR], z1[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      z0[r] = hand_ld(&hand[(size_t)r * n + k * SW_NB + i0]);
      z1[r] = hand_ld(&hand[(size_t)r * n + k * SW_NB + i0 + 1]);
    }
#pragma unroll
    for (int jj = 0; jj < SW_COLS; ++jj)
#pragma unroll
      for (int r = 0; r < NR; ++r) p[jj][r] = fma(u0[jj], z0[r], fma(u1[jj], z1[r], p[jj][r]));
  }
  // r_b = b_b - partial sums
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj) {
    const int j = w * SW_COLS + jj;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const double s = wave_sum(p[jj][r]);
      if (lane == 0) rs[j * NR + r] = j < kb ? B[(size_t)(c0 + j) + (size_t)r * ldb] - s : 0.0;
    }
  }
  __syncthreads();
  // z_m = sum_{i <= m} W[i][m] r_i
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj) {
    const int m = w * SW_COLS + jj;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const double s = wave_sum(fma(w0[jj], rs[i0 * NR + r], w1[jj] * rs[(i0 + 1) * NR + r]));
      if (lane == 0 && m < kb) {
        hand_st(&hand[(size_t)r * n + c0 + m], s);
        B[(size_t)(c0 + m) + (size_t)r * ldb] = s;
      }
    }
  }
  sweep_publish(sync, b + 1);
}

// Backward sweep U x = z: block b (rows) needs sum_{k>b} U[b-rows, k-cols] x_k, a column
// AXPY: lane keeps rows (2l, 2l+1), wave w columns 16w.., reduced across waves in LDS.
template <int NR>
__global__ __launch_bounds__(SW_THREADS) void trsv_bwd_sweep_kernel(
    const double* __restrict__ U, size_t ldu, int n, const double* __restrict__ W,
    double* __restrict__ B, size_t ldb, double* hand, int* sync) {
  constexpr int NW = SW_THREADS / 64;
  __shared__ int sblk;
  __shared__ double part[NW][SW_NB * NR];
  __shared__ double rs[SW_NB * NR];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nblk = (n + SW_NB - 1) / SW_NB;
  if (tid == 0) sblk = atomicAdd(&sync[0], 1);
  __syncthreads();
  const int t = sblk;
  const int b = nblk - 1 - t;
  const int r0 = b * SW_NB, kb = min(SW_NB, n - r0);
  const int i0 = 2 * lane;
  const bool ok0 = i0 < kb, ok1 = i0 + 1 < kb;
  const double* Wb = W + (size_t)b * SW_NB * SW_NB;
  double w0[SW_COLS], w1[SW_COLS];
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj) {
    const int i = w * SW_COLS + jj;  // W column
    const double* col = Wb + (size_t)i * SW_NB;
    w0[jj] = (i < kb && i0 <= i) ? col[i0] : 0.0;
    w1[jj] = (i < kb && i0 + 1 <= i) ? col[i0 + 1] : 0.0;
  }
  double a0[NR], a1[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) a0[r] = a1[r] = 0.0;
  int known = 0;
  for (int k = nblk - 1; k > b; --k) {
    const int kk = min(SW_NB, n - k * SW_NB);
    const double* tile = U + (size_t)r0 + i0 + (size_t)(k * SW_NB + w * SW_COLS) * ldu;
    double u0[SW_COLS], u1[SW_COLS];
#pragma unroll
    for (int jj = 0; jj < SW_COLS; ++jj) {
      const bool ok = w * SW_COLS + jj < kk;
      u0[jj] = ok ? tile[(size_t)jj * ldu] : 0.0;
      u1[jj] = ok ? tile[(size_t)jj * ldu + 1] : 0.0;
    }
    sweep_wait(sync, nblk - k, known, lane);
#pragma unroll
    for (int jj = 0; jj < SW_COLS; ++jj) {
      const int j = w * SW_COLS + jj;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const double x = j < kk ? hand_ld(&hand[(size_t)r * n + k * SW_NB + j]) : 0.0;
        a0[r] = fma(u0[jj], x, a0[r]);
        a1[r] = fma(u1[jj], x, a1[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    part[w][i0 * NR + r] = a0[r];
    part[w][(i0 + 1) * NR + r] = a1[r];
  }
  __syncthreads();
  for (int idx = tid; idx < SW_NB * NR; idx += SW_THREADS) {
    const int i = idx / NR, r = idx - i * NR;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += part[q][idx];
    rs[idx] = i < kb ? B[(size_t)(r0 + i) + (size_t)r * ldb] - s : 0.0;
  }
  __syncthreads();
  // x_m = sum_{i >= m} W[m][i] r_i
#pragma unroll
  for (int r = 0; r < NR; ++r) a0[r] = a1[r] = 0.0;
#pragma unroll
  for (int jj = 0; jj < SW_COLS; ++jj) {
    const int i = w * SW_COLS + jj;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const double x = rs[i * NR + r];
      a0[r] = fma(w0[jj], x, a0[r]);
      a1[r] = fma(w1[jj], x, a1[r]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    part[w][i0 * NR + r] = a0[r];
    part[w][(i0 + 1) * NR + r] = a1[r];
  }
  __syncthreads();
  for (int idx = tid; idx < SW_NB * NR; idx += SW_THREADS) {
    const int i = idx / NR, r = idx - i * NR;
    if (i >= kb) continue;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += part[q][idx];
    hand_st(&hand[(size_t)r * n + r0 + i], s);
    B[(size_t)(r0 + i) + (size_t)r * ldb] = s;
  }
  (void)ok0;
  (void)ok1;
  sweep_publish(sync, t + 1);
}

template <int NR>
static void launch_sweeps(gpr_ctx* ctx, const double* U, size_t ldu, int n, double* B,
                          size_t ldb, int* sync, bool forward, bool backward) {
  const int nblk = (n + SW_NB - 1) / SW_NB;
  if (forward)
    trsv_fwd_sweep_kernel<NR><<<nblk, SW_THREADS, 0, ctx->stream>>>(U, ldu, n, ctx->winv, B, ldb,
                                                                    ctx->dtrsv, sync);
  if (backward)
    trsv_bwd_sweep_kernel<NR><<<nblk, SW_THREADS, 0, ctx->stream>>>(U, ldu, n, ctx->winv, B, ldb,
                                                                  ctx->dtrsv, sync + 2);
}

int launch_diag(gpr_ctx* ctx, double* A, int lda, int n, int kglob, double* winv, int mode,
                int nblocks) {
  const int nb = ctx->nb;
  TimerScope ts(ctx, TC_PANEL, 0.0);
  if (nb == 128 && mode == 1 && nblocks == 1)
    diag2_kernel<<<1, DIAG_THREADS, DIAG2_LDS, ctx->ls>>>(A, (size_t)lda, n, kglob, ctx->dinfo,
                                                       winv);
  else if (nb == 128)
    diag_block_kernel<128><<<nblocks, DIAG_THREADS, 0, ctx->ls>>>(A, (size_t)lda, n, kglob,
                                                                      ctx->dinfo, winv, mode);
  else
    diag_block_kernel<64><<<nblocks, DIAG_THREADS, 0, ctx->ls>>>(A, (size_t)lda, n, kglob,
                                                                     ctx->dinfo, winv, mode);
  LAUNCH_CHECK(ctx);
  return 0;
}

// dst[r + c ldd] = src[r + c lds] for r < rows, c < cols: one workgroup per column chunk,
// 16 B per lane when both sides allow it
__global__ __launch_bounds__(256) void copy_panel_kernel(const double* __restrict__ src, size_t lds,
                                                         double* __restrict__ dst, size_t ldd,
                                                         int rows, int cols, int vec) {
  typedef double d2c __attribute__((ext_vector_type(2)));
  const int c = blockIdx.x;
  if (c >= cols) return;
  const double* sc = src + (size_t)c * lds;
  double* dc = dst + (size_t)c * ldd;
  if (vec) {
    for (int r = 2 * threadIdx.x; r < rows; r += 512)
      *reinterpret_cast<d2c*>(dc + r) = *reinterpret_cast<const d2c*>(sc + r);
  } else {
    for (int r = threadIdx.x; r < rows; r += 256) dc[r] = sc[r];
  }
}

int launch_copy_panel(gpr_ctx* ctx, const double* src, int lds, double* dst, int ldd, int rows,
                      int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int vec = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0) && (lds % 2 == 0) &&
                  (ldd % 2 == 0) && (rows % 2 == 0);
  TimerScope ts(ctx, TC_OTHER, 0.0);
  copy_panel_kernel<<<cols, 256, 0, ctx->ls>>>(src, (size_t)lds, dst, (size_t)ldd, rows, cols, vec);
  LAUNCH_CHECK(ctx);
  return 0;
}

hipEvent_t sync_event(gpr_ctx* ctx, size_t i) {
  while (ctx->sync_events.size() <= i) {
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    ctx->sync_events.push_back(e);
  }
  return ctx->sync_events[i];
}

// Factor the rows [k, k+kw) of the (already updated) trailing matrix: per inner block j:
// diag factor+inverse, in-place panel TRSM over all columns >= j+jb (MFMA GEMM with
// U_jj^{-1}), then the update of the remaining rows of this outer panel (K = nb).
// (Measured and removed in round 5: a square-chain + left-looking strip, an inverse strip,
// recursive halves, inner / block lookahead, a one-launch square-panel kernel and CU masking
// for the diagonal kernel -- every one slower than this per-block panel)
int factor_panel(gpr_ctx* ctx, double* A, int n, int lda, int k, int kw) {
  const int nb = ctx->nb;
  for (int j = k; j < k + kw; j += nb) {
    const int jb = std::min(nb, n - j);
    double* wj = ctx->winv + (size_t)(j / nb) * nb * nb;
    GPR_TRY(launch_diag(ctx, A, lda, n, j, wj, 1, 1));
    if (j + jb >= n) break;
    double* row = A + j + (size_t)(j + jb) * lda;
    GemmArgs g{};
    g.P = wj; g.ldp = nb;
    g.Q = row; g.ldq = lda;
    g.C = row; g.ldc = lda;
    g.M = jb; g.N = n - j - jb; g.K = jb;
    g.alpha = 1.0; g.beta = 0.0;
    g.info = ctx->dinfo;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_PANEL));
    const int rows = k + kw - j - jb;  // panel rows below block j
    if (rows <= 0) continue;
    GemmArgs u{};
    u.P = row; u.ldp = lda;
    u.Q = row; u.ldq = lda;
    u.C = A + (j + jb) + (size_t)(j + jb) * lda; u.ldc = lda;
    u.M = rows; u.N = n - j - jb; u.K = jb;
    u.alpha = -1.0; u.beta = 1.0;
    u.mask_upper = 1;
    u.info = ctx->dinfo;
    GPR_TRY(launch_gemm_tn(ctx, u, TC_PANEL));
  }
  return 0;
}

// All outer-panel square inverses U_sq^{-1} of a finished factor in one launch: grid
// (panel p, block column c).  Block column c of panel p needs only U (final) and the block
// inverses W_i (final), so the workgroups are independent (no hand-offs).
//   X_cc = W_c,  X_ic = -W_i sum_{t=i+1..c} U(i, t) X_tc   (i = c-1 .. 0)
__global__ __launch_bounds__(256, 1) void sqinv_kernel(const double* __restrict__ U, size_t ldu,
                                                       int n, int nb2, int p0,
                                                       const double* __restrict__ winv,
                                                       double* __restrict__ sqinv) {
  constexpr int NB = 128;
  __shared__ double glds[2 * 4096];
  const int p = p0 + blockIdx.x, c = blockIdx.y;
  const int k = p * nb2, kw = min(nb2, n - k);
  if (c * NB >= kw) return;
  auto blk = [&](int i, int j) { return U + (size_t)(k + i * NB) + (size_t)(k + j * NB) * ldu; };
  auto wid = [&](int i) { return min(NB, kw - i * NB); };
  auto W = [&](int i) { return winv + (size_t)((k / NB) + i) * NB * NB; };
  const int cw = wid(c);
  double* X = sqinv + (size_t)p * nb2 * nb2 + (size_t)(c * NB) * kw;
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int r = e % NB, q = e / NB;
    if (r < cw && q < cw) X[(size_t)(c * NB + r) + (size_t)q * kw] = W(c)[r + (size_t)q * NB];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  d4v acc[4][4];
  for (int i = c - 1; i >= 0; --i) {
    const int iw = wid(i);
    sq_zero(acc);
    for (int t = i + 1; t <= c; ++t) sq_gemm<true>(acc, blk(i, t), ldu, X + t * NB, kw, wid(t), iw, cw, glds);
    sq_store(acc, X + i * NB, 1, kw, 1.0, 0.0, iw, cw, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    sq_zero(acc);
    sq_gemm<true>(acc, W(i), NB, X + i * NB, kw, iw, iw, cw, glds);
    __syncthreads();
    sq_store(acc, X + i * NB, 1, kw, -1.0, 0.0, iw, cw, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// norm[j] -= sum_{i<n} B[i + j ldb]^2 for j < ncols: one wave per column (deterministic)
__global__ __launch_bounds__(256) void colnorm_sub_kernel(const double* __restrict__ B, size_t ldb,
                                                          int n, int ncols, double* __restrict__ norm) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= ncols) return;
  const double* col = B + (size_t)j * ldb;
  double s0 = 0.0, s1 = 0.0;
  int i = lane;
  for (; i + 64 < n; i += 128) {
    s0 = fma(col[i], col[i], s0);
    s1 = fma(col[i + 64], col[i + 64], s1);
  }
  if (i < n) s0 = fma(col[i], col[i], s0);
  double s = s0 + s1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) norm[j] -= s;
}

// TRSM panel: X_j = W_j^T B_j for the inner blocks of rows [k, k+kw), each followed by
// the update of the remaining rows of the outer block (K = nb).
int trsm_panel(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int ncols, int ldb,
               double* norm_out, int k, int kw) {
  const int nb = ctx->nb;
  for (int j = k; j < k + kw; j += nb) {
    const int jb = std::min(nb, n - j);
    GemmArgs g{};
    g.P = ctx->winv + (size_t)(j / nb) * nb * nb; g.ldp = nb;
    g.Q = dB + j; g.ldq = ldb;
    g.C = dB + j; g.ldc = ldb;
    g.M = jb; g.N = ncols; g.K = jb;
    g.alpha = 1.0; g.beta = 0.0;
    g.norm_out = norm_out;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_TRSM_GEMM));
    if (j + jb < k + kw) {
      GemmArgs u{};
      u.P = dU + j + (size_t)(j + jb) * ldu; u.ldp = ldu;
      u.Q = dB + j; u.ldq = ldb;
      u.C = dB + j + jb; u.ldc = ldb;
      u.M = k + kw - j - jb; u.N = ncols; u.K = jb;
      u.alpha = -1.0; u.beta = 1.0;
      GPR_TRY(launch_gemm_tn(ctx, u, TC_TRSM_GEMM));
    }
  }
  return 0;
}

// Outer panel k of a right-hand-side block on the square inverse (the loop body of
// trsm_ut_sq): X_k = U_sq_k^{-T} B_k (one GEMM, K range cut at each tile's diagonal), the update
// B_rest -= U_k,rest^T X_k (K = nb2), X_k copied back.  Everything on ctx->ls.
int rhs_panel_step(gpr_ctx* ctx, const double* dU, int n, int ldu, const RhsSpec& r, int k,
                   int nb2, double* panelbuf) {
  const int kw = std::min(nb2, n - k), kend = k + kw;
  const int nc = r.lower_rhs ? std::min(r.nrhs, kend) : r.nrhs;
  GemmArgs g{};
  g.P = ctx->dsqinv + (size_t)(k / nb2) * nb2 * nb2; g.ldp = kw;
  g.Q = r.B + k; g.ldq = r.ldb;
  g.C = panelbuf; g.ldc = kw;
  g.M = kw; g.N = nc; g.K = kw;
  g.alpha = 1.0; g.beta = 0.0;
  g.kend_from_m = 1;
  g.info = ctx->dinfo;
  GPR_TRY(launch_gemm_tn(ctx, g, TC_TRSM_GEMM));
  if (kend < n) {
    GemmArgs b{};
    b.P = dU + k + (size_t)kend * ldu; b.ldp = ldu;
    b.Q = panelbuf; b.ldq = kw;
    b.C = r.B + kend; b.ldc = r.ldb;
    b.M = n - kend; b.N = nc; b.K = kw;
    b.alpha = -1.0; b.beta = 1.0;
    b.info = ctx->dinfo;
    GPR_TRY(launch_gemm_tn(ctx, b, TC_TRSM_GEMM));
  }
  return launch_copy_panel(ctx, panelbuf, kw, r.B + k, r.ldb, kw, nc);
}

}  // namespace

// Debug timing of the chain kernels (tools/gemm_bench mode 6 only), averaged over the
// diagonal blocks 0 .. reps-1 of a freshly assembled SPD matrix A (each factored once):
// variant 0 the diagonal-block kernel (U + W), 1 the W^T GEMM row TRSM (after variant 0).
extern "C" int gpr_debug_chain_kernels(gpr_ctx_t ctx, double* A, int lda, int n, int variant,
                                       int reps, float* ms) {
  GPR_TRY(ensure_winv(ctx, n, 128));
  reps = std::min(reps, n / 128 - 1);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  ctx->ls = ctx->stream;
  HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), ctx->stream));
  hipEventRecord(e0, ctx->stream);
  for (int r = 0; r < reps; ++r) {
    const int j = 128 * r;
    double* wj = ctx->winv + (size_t)r * 128 * 128;
    if (variant == 0) GPR_TRY(launch_diag(ctx, A, lda, n, j, wj, 1, 1));
    if (variant == 1) {
      GemmArgs g{};
      g.P = wj; g.ldp = 128;
      g.Q = A + j + (size_t)(j + 128) * lda; g.ldq = lda;
      g.C = A + j + (size_t)(j + 128) * lda; g.ldc = lda;
      g.M = 128; g.N = n - j - 128; g.K = 128;
      g.alpha = 1.0; g.beta = 0.0;
      g.info = ctx->dinfo;
      GPR_TRY(launch_gemm_tn(ctx, g, TC_PANEL));
    }
  }
  hipEventRecord(e1, ctx->stream);
  hipEventSynchronize(e1);
  hipEventElapsedTime(ms, e0, e1);
  *ms /= reps;
  int hinfo = 0;
  hipMemcpy(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return hinfo;
}

// Two-level right-looking upper Cholesky with depth-1 lookahead.
//   outer panels P_s = rows [s*nb2, (s+1)*nb2)      (nb2 = K of the big MFMA updates)
//   stream2 (panel):  wait b_{s-1}; a_s = update of rows P_{s+1} by P_s; factor P_{s+1}
//   stream  (main):   wait panel_s; b_s = SYRK of rows/cols >= (s+2)*nb2 by P_s
// so the latency-bound diag/TRSM chain of panel s+1 overlaps the big SYRK b_s.
//   srhs (rhs, optional): wait panel_s final; U_sq_s^{-1}; solve outer block s of B and update
//                         the rows below (rhs_panel_step) -- the triangular solve rides in the
//                         bubbles of the lookahead chain instead of running after the factor.
int potrf_core(gpr_ctx* ctx, double* dA, int n, int lda, int* info, const RhsSpec* rhs) {
  const int nb = ctx->nb;
  const int nb2 = std::max(nb, (ctx->nb2 / nb) * nb);
  ctx->fac_valid = false;
  ctx->sqinv_nb2 = 0;
  // dA as the upper-only K assembly left it (launch_kernel_matrix_for_factor): its strict lower
  // off-diagonal tiles are written by the tile-DAG launch (DAG_MIRROR) or, on any other path,
  // mirrored here before the factorisation overwrites the upper triangle
  bool mirror = ctx->kup_ptr == dA && ctx->kup_n == n && ctx->kup_ld == lda;
  ctx->kup_ptr = nullptr;
  GPR_TRY(ensure_winv(ctx, n, nb));
  if (rhs && (nb != 128 || nb2 > 2048 || !ctx->srhs || rhs->nrhs <= 0)) rhs = nullptr;
  ctx->rhs_solved = rhs != nullptr;  // (callers solve a dropped right-hand side afterwards)
  if (rhs) {
    GPR_TRY(ensure_buf(ctx, &ctx->dsqinv, &ctx->sqinv_cap,
                       (size_t)((n + nb2 - 1) / nb2) * nb2 * nb2));
    GPR_TRY(ensure_buf(ctx, &ctx->dpanel_rhs, &ctx->panel_rhs_cap, (size_t)nb2 * rhs->nrhs));
  }
  // a gram (K^{-1} += Z^T Z) rides in the DAG launch for the identity's Z only
  const bool dag_rhs_ok = !rhs || ((!rhs->lower_rhs || rhs->nrhs == n) &&
                                   (!rhs->gram || (rhs->lower_rhs && ctx->dag_gram)));
  if (dag_takes_whole(ctx, n, lda, dA) && dag_rhs_ok) {
    // one persistent launch: tiles handed between workgroups by progress counters; shapes the
    // launch does not take directly go through a padded copy
    HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), ctx->stream));
    int rc = 1;
    if (dag_shape_ok(n, lda, dA))  // (1 = B's layout not taken directly either)
      rc = launch_potrf_dag(ctx, dA, n, lda, rhs ? rhs->B : nullptr, rhs ? rhs->nrhs : 0,
                            rhs ? rhs->ldb : 0, 0, ctx->stream,
                            (rhs && rhs->lower_rhs ? DAG_LOWER : 0) |
                                (rhs && rhs->gram ? DAG_GRAM : 0) | (mirror ? DAG_MIRROR : 0),
                            rhs ? rhs->gram : nullptr, rhs ? rhs->ldg : 0);
    if (rc < 0) return rc;
    if (rc == 0) mirror = false;  // (the launch writes the lower tiles)
    if (mirror) {
      GPR_TRY(launch_mirror_upper(ctx, dA, n, lda));
      mirror = false;
    }
    if (rc == 1 && (!rhs || !rhs->lower_rhs))
      rc = launch_potrf_dag_padded(ctx, dA, n, lda, rhs ? rhs->B : nullptr, rhs ? rhs->nrhs : 0,
                                   rhs ? rhs->ldb : 0);
    if (rc < 0) return rc;
    ctx->gram_full = rc == 0 && rhs && rhs->gram;  // (the DAG wrote every tile of it)
    if (rc == 0) {
      int hinfo = 0;
      HIP_TRY(ctx, hipMemcpyAsync(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost,
                                  ctx->stream));
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      if (hinfo < 0)
        return set_err(ctx, GPR_E_HIP, "tile-DAG factorisation: a dependency wait timed out");
      if (info) *info = hinfo;
      if (hinfo == 0) {
        ctx->fac_valid = true;
        ctx->fac_ptr = dA;
        ctx->fac_n = n;
        ctx->fac_ld = lda;
        ctx->fac_nb = nb;
      }
      return 0;
    }
  }
  if (mirror) GPR_TRY(launch_mirror_upper(ctx, dA, n, lda));
  hipStream_t user = ctx->stream;
  ctx->gram_full = false;
  if (rhs && rhs->gram)  // accumulated panel by panel below (upper; the caller mirrors)
    HIP_TRY(ctx, hipMemset2DAsync(rhs->gram, (size_t)rhs->ldg * sizeof(double), 0,
                                  (size_t)n * sizeof(double), n, user));
  hipStream_t s0 = ctx->stream, s1 = ctx->stream2;
  HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), user));
  size_t ev = 0;
  ctx->ev_next = 1000;  // events of the diag hops use a separate index range
  hipEvent_t e0 = sync_event(ctx, ev++);
  HIP_TRY(ctx, hipEventRecord(e0, user));
  HIP_TRY(ctx, hipStreamWaitEvent(s1, e0, 0));
  if (s0 != user) HIP_TRY(ctx, hipStreamWaitEvent(s0, e0, 0));
  // fused_rhs 1: right-hand sides on their own stream (srhs); 2: on the main stream after each
  // trailing SYRK (serialised with the big updates, overlapping only the panel chain)
  hipStream_t sr = !rhs ? nullptr : (rhs->mode == 2 ? s0 : ctx->srhs);
  if (sr && sr != s0) HIP_TRY(ctx, hipStreamWaitEvent(sr, e0, 0));
  ctx->ls = s1;
  auto panel = [&](int k, int kw) { return factor_panel(ctx, dA, n, lda, k, kw); };
  // outer block k of the right-hand sides once panel k of U is final (event ev_final)
  // U_sq^{-1} of outer panel k on ssq once the panel is final (off the solve's own chain);
  // the square path wrote it already
  auto sq_inverse = [&](int k, hipEvent_t ev_final) -> hipEvent_t {
    if (!sr) return ev_final;
    if (hipStreamWaitEvent(ctx->ssq, ev_final, 0) != hipSuccess) return nullptr;
    ctx->ls = ctx->ssq;
    {
      TimerScope ts(ctx, TC_OTHER, 0.0);
      sqinv_kernel<<<dim3(1, nb2 / nb), 256, 0, ctx->ssq>>>(dA, (size_t)lda, n, nb2, k / nb2,
                                                            ctx->winv, ctx->dsqinv);
    }
    hipEvent_t es = sync_event(ctx, ev++);
    if (hipEventRecord(es, ctx->ssq) != hipSuccess) return nullptr;
    return es;
  };
  // outer block k of the right-hand sides once U_sq^{-1} of panel k exists (event ev_sq)
  auto rhs_step = [&](int k, hipEvent_t ev_sq) -> int {
    if (!sr) return 0;
    ctx->ls = sr;
    HIP_TRY(ctx, hipStreamWaitEvent(sr, ev_sq, 0));
    GPR_TRY(rhs_panel_step(ctx, dA, n, lda, *rhs, k, nb2, ctx->dpanel_rhs));
    if (!rhs->gram) return 0;
    // rows [k, kend) of the solved B are final: gram(0:kend, 0:kend) += B_s^T B_s (upper)
    const int kend = std::min(n, k + nb2);
    GemmArgs g{};
    g.P = rhs->B + k; g.ldp = rhs->ldb;
    g.Q = rhs->B + k; g.ldq = rhs->ldb;
    g.C = rhs->gram; g.ldc = rhs->ldg;
    g.M = kend; g.N = kend; g.K = kend - k;
    g.alpha = 1.0; g.beta = 1.0;
    g.upper = 1;
    g.info = ctx->dinfo;
    return launch_gemm_tn(ctx, g, TC_TRSM_GEMM);
  };
  int rc = panel(0, std::min(nb2, n));
  hipEvent_t ev_p = sync_event(ctx, ev++);
  hipEvent_t ev_b = nullptr;
  if (!rc && hipEventRecord(ev_p, s1) != hipSuccess) rc = GPR_E_HIP;
  // tail hand-off: once the trailing matrix is <= dag_tail, ONE SYRK applies panel s to all of
  // it and the tile-DAG factors it (the blocked path is chain-bound there)
  const bool tail_ok = ctx->dag_tail > 0 && !rhs && nb == 128 && lda % 16 == 0 &&
                       ((uintptr_t)dA & 127) == 0 && n % 16 == 0;
  bool tail_done = false;
  for (int k = 0; !rc && k + nb2 < n; k += nb2) {
    const int kend = k + nb2, w2 = std::min(nb2, n - kend), rest0 = kend + w2;
    if (tail_ok && n - kend <= ctx->dag_tail) {
      ctx->ls = s0;
      if (hipStreamWaitEvent(s0, ev_p, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
      GemmArgs b{};
      b.P = dA + k + (size_t)kend * lda; b.ldp = lda;
      b.Q = b.P; b.ldq = lda;
      b.C = dA + kend + (size_t)kend * lda; b.ldc = lda;
      b.M = n - kend; b.N = n - kend; b.K = kend - k;
      b.alpha = -1.0; b.beta = 1.0;
      b.upper = 1;
      b.info = ctx->dinfo;
      if ((rc = launch_gemm_tn(ctx, b, TC_SYRK))) break;
      rc = launch_potrf_dag(ctx, dA + kend + (size_t)kend * lda, n - kend, lda, nullptr, 0, 0,
                            kend, s0);
      if (rc > 0) rc = set_err(ctx, GPR_E_HIP, "tile-DAG tail: shape not eligible");
      tail_done = true;
      break;
    }
    // ---- square inverse of panel s, then (srhs mode) outer block s of B
    hipEvent_t ev_sq = sq_inverse(k, ev_p);
    if (!ev_sq) { rc = GPR_E_HIP; break; }
    if (sr != s0 && (rc = rhs_step(k, ev_sq))) break;
    // ---- panel stream: a_s (rows P_{s+1} by P_s), then factor panel s+1
    ctx->ls = s1;
    if (ev_b && hipStreamWaitEvent(s1, ev_b, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
    GemmArgs a{};
    a.P = dA + k + (size_t)kend * lda; a.ldp = lda;
    a.Q = a.P; a.ldq = lda;
    a.C = dA + kend + (size_t)kend * lda; a.ldc = lda;
    a.M = w2; a.N = n - kend; a.K = nb2;
    a.alpha = -1.0; a.beta = 1.0;
    a.mask_upper = 1;
    a.info = ctx->dinfo;
    if ((rc = launch_gemm_tn(ctx, a, TC_PANEL))) break;
    if ((rc = panel(kend, w2))) break;
    hipEvent_t ev_p_next = sync_event(ctx, ev++);
    if (hipEventRecord(ev_p_next, s1) != hipSuccess) { rc = GPR_E_HIP; break; }
    // ---- main stream: b_s
    ctx->ls = s0;
    if (hipStreamWaitEvent(s0, ev_p, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
    if (rest0 < n) {
      // b_s: the upper trailing matrix in one launch (round 1's split into column bands, to
      // give the lookahead stream dispatch slots in between, measured no faster)
      const int R = n - rest0;
      GemmArgs b{};
      b.P = dA + k + (size_t)rest0 * lda; b.ldp = lda;
      b.Q = dA + k + (size_t)rest0 * lda; b.ldq = lda;
      b.C = dA + rest0 + (size_t)rest0 * lda; b.ldc = lda;
      b.M = R; b.N = R; b.K = nb2;
      b.alpha = -1.0; b.beta = 1.0;
      b.upper = 1;
      b.info = ctx->dinfo;
      rc = launch_gemm_tn(ctx, b, TC_SYRK);
      if (rc) break;
    }
    ev_b = sync_event(ctx, ev++);
    if (hipEventRecord(ev_b, s0) != hipSuccess) { rc = GPR_E_HIP; break; }
    if (sr == s0 && (rc = rhs_step(k, ev_sq))) break;  // after b_s, beside the panel chain
    ev_p = ev_p_next;
  }
  if (!rc && sr) {  // the last outer block
    const int kl = ((n - 1) / nb2) * nb2;
    hipEvent_t ev_sq = sq_inverse(kl, ev_p);
    rc = ev_sq ? rhs_step(kl, ev_sq) : GPR_E_HIP;
  }
  if (sr && sr != s0) {
    hipEvent_t er = sync_event(ctx, ev++);
    HIP_TRY(ctx, hipEventRecord(er, sr));
    HIP_TRY(ctx, hipStreamWaitEvent(user, er, 0));
  }
  ctx->ls = user;
  hipEvent_t ej = sync_event(ctx, ev++);  // join the panel and main streams into the user's
  HIP_TRY(ctx, hipEventRecord(ej, s1));
  HIP_TRY(ctx, hipStreamWaitEvent(user, ej, 0));
  if (s0 != user) {
    hipEvent_t ek = sync_event(ctx, ev++);
    HIP_TRY(ctx, hipEventRecord(ek, s0));
    HIP_TRY(ctx, hipStreamWaitEvent(user, ek, 0));
  }
  if (rc) return rc;
  int hinfo = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost, user));
  HIP_TRY(ctx, hipStreamSynchronize(user));
  if (tail_done && hinfo < 0)
    return set_err(ctx, GPR_E_HIP, "tile-DAG factorisation: a dependency wait timed out");
  if (info) *info = hinfo;
  if (hinfo == 0 && rhs) {
    ctx->sqinv_nb2 = nb2;
    ctx->sq_ptr = dA;
    ctx->sq_n = n;
    ctx->sq_ld = lda;
  }
  if (hinfo == 0) {
    ctx->fac_valid = true;
    ctx->fac_ptr = dA;
    ctx->fac_n = n;
    ctx->fac_ld = lda;
    ctx->fac_nb = nb;
  }
  return 0;
}

int ensure_factor_inverses(gpr_ctx* ctx, const double* dU, int n, int ldu) {
  if (ctx->fac_valid && ctx->fac_ptr == dU && ctx->fac_n == n && ctx->fac_ld == ldu &&
      ctx->fac_nb == ctx->nb)
    return 0;
  const int nb = ctx->nb;
  GPR_TRY(ensure_winv(ctx, n, nb));
  HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), ctx->stream));
  const int nblk = (n + nb - 1) / nb;
  GPR_TRY(launch_diag(ctx, const_cast<double*>(dU), ldu, n, 0, ctx->winv, 0, nblk));
  ctx->fac_valid = true;
  ctx->fac_ptr = dU;
  ctx->fac_n = n;
  ctx->fac_ld = ldu;
  ctx->fac_nb = nb;
  return 0;
}

// U_sq^{-1} of every outer panel of the factor dU (computed once per factor, reused by all
// solves).  Returns 1 when the square path is usable (nb = 128, nb2 <= 2048).
int ensure_sq_inverses(gpr_ctx* ctx, const double* dU, int n, int ldu) {
  constexpr int NB = 128;
  const int nb2 = std::max(NB, (ctx->nb2 / NB) * NB);
  if (ctx->nb != NB || nb2 > 2048) return 0;
  GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
  if (ctx->sqinv_nb2 == nb2 && ctx->sq_ptr == dU && ctx->sq_n == n && ctx->sq_ld == ldu) return 1;
  const int np = (n + nb2 - 1) / nb2;
  GPR_TRY(ensure_buf(ctx, &ctx->dsqinv, &ctx->sqinv_cap, (size_t)np * nb2 * nb2));
  {
    TimerScope ts(ctx, TC_OTHER, 0.0);
    sqinv_kernel<<<dim3(np, nb2 / NB), 256, 0, ctx->stream>>>(dU, (size_t)ldu, n, nb2, 0,
                                                              ctx->winv, ctx->dsqinv);
    LAUNCH_CHECK(ctx);
  }
  ctx->sqinv_nb2 = nb2;
  ctx->sq_ptr = dU;
  ctx->sq_n = n;
  ctx->sq_ld = ldu;
  return 1;
}

// B <- U^{-T} B (U^T X = B), GEMM-based (any nrhs), two-level with the same lookahead
// structure as potrf_core.  norm_out: optional norm_out[c] -= ||X[:, c]||^2 (fused in the
// panel GEMM epilogue).  lower_rhs: B is lower-triangular (identity RHS) -> outer block s
// only touches columns [0, (s+1) nb2).
// trsm_ut_core on the square inverses: the panel solve of outer block s is ONE GEMM,
// X_s = U_sq_s^{-T} B_s (K range cut at each tile's diagonal, out of place + strided copy
// back), instead of nb2/nb dependent (GEMM, update) pairs.  Same two-stream lookahead.
// norm_out is a deterministic post-pass over the solved B.
static int trsm_ut_sq(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                      int ldb, double* norm_out, int lower_rhs) {
  // One stream, per outer panel s: X_s = U_sq_s^{-T} B_s into a panel buffer (one GEMM with a
  // per-tile K range, heavy/light tiles paired per CU), then ONE update GEMM of all rows below
  // (B_rest -= U_s,rest^T X_s, K = nb2), then X_s copied back into B.  A lookahead stream for
  // the next panel's solve measured no faster (the big update loses to the co-running
  // kernels what the overlap gains) and was dropped.
  const int nb2 = ctx->sqinv_nb2;
  hipStream_t s0 = ctx->stream;
  ctx->ls = s0;
  auto cols = [&](int kend) { return lower_rhs ? std::min(nrhs, kend) : nrhs; };
  GPR_TRY(ensure_buf(ctx, &ctx->dpanel, &ctx->panel_cap, (size_t)nb2 * nrhs));
  for (int k = 0; k < n; k += nb2) {
    const int kw = std::min(nb2, n - k), kend = k + kw;
    const int nc = cols(kend);  // lower_rhs: columns >= kend of B_s are still zero
    GemmArgs g{};
    g.P = ctx->dsqinv + (size_t)(k / nb2) * nb2 * nb2; g.ldp = kw;
    g.Q = dB + k; g.ldq = ldb;
    g.C = ctx->dpanel; g.ldc = kw;
    g.M = kw; g.N = nc; g.K = kw;
    g.alpha = 1.0; g.beta = 0.0;
    g.kend_from_m = 1;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_TRSM_GEMM));
    if (kend < n) {
      GemmArgs b{};
      b.P = dU + k + (size_t)kend * ldu; b.ldp = ldu;
      b.Q = ctx->dpanel; b.ldq = kw;
      b.C = dB + kend; b.ldc = ldb;
      b.M = n - kend; b.N = nc; b.K = kw;
      b.alpha = -1.0; b.beta = 1.0;
      GPR_TRY(launch_gemm_tn(ctx, b, TC_TRSM_GEMM));
    }
    GPR_TRY(launch_copy_panel(ctx, ctx->dpanel, kw, dB + k, ldb, kw, nc));
  }
  if (norm_out) {
    TimerScope ts(ctx, TC_OTHER, 0.0);
    colnorm_sub_kernel<<<(nrhs + 3) / 4, 256, 0, s0>>>(dB, (size_t)ldb, n, nrhs, norm_out);
    LAUNCH_CHECK(ctx);
  }
  return 0;
}

int launch_colnorm_sub(gpr_ctx* ctx, const double* dB, int ldb, int n, int ncols, double* norm) {
  if (ncols <= 0) return 0;
  TimerScope ts(ctx, TC_OTHER, 0.0);
  colnorm_sub_kernel<<<(ncols + 3) / 4, 256, 0, ctx->stream>>>(dB, (size_t)ldb, n, ncols, norm);
  LAUNCH_CHECK(ctx);
  return 0;
}

int trsm_ut_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                 int ldb, double* norm_out, int lower_rhs) {
  // solve-only tile-DAG: GPR_DAG_SOLVE=1 always, 0 never; auto (-1) for the wide solves,
  // where it measured no slower: C5's variance rows (n = 32768, 32768 right-hand sides) 719
  // vs 725 ms per job on one box, 714.8 vs 714.9 on another; POTRI's Z at n = 16384 48.9 vs
  // 49.8 ms.  C3's posterior (8193 right-hand sides: 130.4 vs 127.9 ms) stays blocked.
  const bool dag_solve = ctx->dag_solve > 0 || (ctx->dag_solve < 0 && n >= 8192 && nrhs >= n);
  if (dag_solve && dag_takes_whole(ctx, n, ldu, dU) && nrhs >= 128 &&
      (!lower_rhs || nrhs == n)) {
    // the tile-DAG with every tile of U final: only B's tiles are tasks (left-looking, one
    // long-K accumulation per tile, W_i from the factor's block inverses)
    GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
    // the kernel skips every task while info != 0: clear what an earlier launch left, and
    // read it back afterwards (a timed-out dependency wait leaves B unsolved: report it).
    // The read-back synchronises the host once per solve: for C5's variance rows that is one
    // sync per 32-row batch of ~0.5 s of solve, i.e. the next batch's factor build (tens of
    // microseconds) is no longer hidden behind this one -- < 0.01 % of the job.
    HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), ctx->stream));
    const int rc = launch_potrf_dag(ctx, const_cast<double*>(dU), n, ldu, dB, nrhs, ldb, 0,
                                    ctx->stream, DAG_SOLVE | (lower_rhs ? DAG_LOWER : 0));
    if (rc < 0) return rc;
    if (rc == 0) {
      int hinfo = 0;
      HIP_TRY(ctx, hipMemcpyAsync(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost,
                                  ctx->stream));
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      if (hinfo != 0)
        return set_err(ctx, GPR_E_HIP, "tile-DAG solve: a dependency wait timed out (info %d)",
                       hinfo);
      if (norm_out) GPR_TRY(launch_colnorm_sub(ctx, dB, ldb, n, nrhs, norm_out));
      return 0;
    }
  }
  {
    const int sqok = ensure_sq_inverses(ctx, dU, n, ldu);
    if (sqok < 0) return sqok;
    if (sqok == 1) return trsm_ut_sq(ctx, dU, n, ldu, dB, nrhs, ldb, norm_out, lower_rhs);
  }
  GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
  const int nb = ctx->nb;
  const int nb2 = std::max(nb, (ctx->nb2 / nb) * nb);
  hipStream_t s0 = ctx->stream, s1 = ctx->stream2;
  size_t ev = 0;
  hipEvent_t e0 = sync_event(ctx, ev++);
  HIP_TRY(ctx, hipEventRecord(e0, s0));
  HIP_TRY(ctx, hipStreamWaitEvent(s1, e0, 0));
  auto cols = [&](int kend) { return lower_rhs ? std::min(nrhs, kend) : nrhs; };
  ctx->ls = s1;
  const int w0 = std::min(nb2, n);
  int rc = trsm_panel(ctx, dU, n, ldu, dB, cols(w0), ldb, norm_out, 0, w0);
  hipEvent_t ev_p = sync_event(ctx, ev++);
  hipEvent_t ev_b = nullptr;
  if (!rc && hipEventRecord(ev_p, s1) != hipSuccess) rc = GPR_E_HIP;
  for (int k = 0; !rc && k + nb2 < n; k += nb2) {
    const int kend = k + nb2, w2 = std::min(nb2, n - kend), rest0 = kend + w2;
    const int nc = cols(kend);
    ctx->ls = s1;
    if (ev_b && hipStreamWaitEvent(s1, ev_b, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
    GemmArgs a{};
    a.P = dU + k + (size_t)kend * ldu; a.ldp = ldu;
    a.Q = dB + k; a.ldq = ldb;
    a.C = dB + kend; a.ldc = ldb;
    a.M = w2; a.N = nc; a.K = nb2;
    a.alpha = -1.0; a.beta = 1.0;
    if ((rc = launch_gemm_tn(ctx, a, TC_TRSM_GEMM))) break;
    if ((rc = trsm_panel(ctx, dU, n, ldu, dB, cols(rest0), ldb, norm_out, kend, w2))) break;
    hipEvent_t ev_p_next = sync_event(ctx, ev++);
    if (hipEventRecord(ev_p_next, s1) != hipSuccess) { rc = GPR_E_HIP; break; }
    ctx->ls = s0;
    if (hipStreamWaitEvent(s0, ev_p, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
    if (rest0 < n) {
      GemmArgs b{};
      b.P = dU + k + (size_t)rest0 * ldu; b.ldp = ldu;
      b.Q = dB + k; b.ldq = ldb;
      b.C = dB + rest0; b.ldc = ldb;
      b.M = n - rest0; b.N = nc; b.K = nb2;
      b.alpha = -1.0; b.beta = 1.0;
      if ((rc = launch_gemm_tn(ctx, b, TC_TRSM_GEMM))) break;
    }
    ev_b = sync_event(ctx, ev++);
    if (hipEventRecord(ev_b, s0) != hipSuccess) { rc = GPR_E_HIP; break; }
    ev_p = ev_p_next;
  }
  ctx->ls = s0;
  hipEvent_t ej = sync_event(ctx, ev++);
  HIP_TRY(ctx, hipEventRecord(ej, s1));
  HIP_TRY(ctx, hipStreamWaitEvent(s0, ej, 0));
  return rc;
}

// B <- K^{-1} B with small nrhs (dpotrs): blocked forward U^T z = b, backward U x = z.
int potrs_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs, int ldb,
               bool forward, bool backward) {
  GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
  const int nb = ctx->nb;
  const int nblk = (n + nb - 1) / nb;
  if (nb == SW_NB) {
    GPR_TRY(ensure_buf(ctx, &ctx->dtrsv, &ctx->trsv_cap, (size_t)n * 2));
    int* sync = ctx->dinfo + 4;  // dinfo[4..7]: fwd ticket/done, bwd ticket/done
    for (int c0 = 0; c0 < nrhs; c0 += 2) {
      const int nc = std::min(2, nrhs - c0);
      double* B = dB + (size_t)c0 * ldb;
      HIP_TRY(ctx, hipMemsetAsync(sync, 0, 4 * sizeof(int), ctx->stream));
      TimerScope ts(ctx, TC_OTHER, 0.0);
      if (nc == 1)
        launch_sweeps<1>(ctx, dU, ldu, n, B, ldb, sync, forward, backward);
      else
        launch_sweeps<2>(ctx, dU, ldu, n, B, ldb, sync, forward, backward);
      LAUNCH_CHECK(ctx);
    }
    return 0;
  }
  for (int c0 = 0; c0 < nrhs; c0 += RHS_CHUNK) {
    const int nc = std::min(RHS_CHUNK, nrhs - c0);
    double* B = dB + (size_t)c0 * ldb;
    // forward
    for (int b = 0; forward && b < nblk; ++b) {
      const int k = b * nb, kb = std::min(nb, n - k);
      const double* wk = ctx->winv + (size_t)b * nb * nb;
      trsv_diag_kernel<<<1, 256, 0, ctx->stream>>>(wk, nb, kb, B + k, (size_t)ldb, nc, 1);
      LAUNCH_CHECK(ctx);
      const int rest = n - k - kb;
      if (rest > 0) {
        gemv_t_update_kernel<<<(rest + 3) / 4, 256, 0, ctx->stream>>>(
            dU + k + (size_t)(k + kb) * ldu, (size_t)ldu, kb, rest, B + k, (size_t)ldb,
            B + k + kb, (size_t)ldb, nc);
        LAUNCH_CHECK(ctx);
      }
    }
    // backward
    for (int b = nblk - 1; backward && b >= 0; --b) {
      const int k = b * nb, kb = std::min(nb, n - k);
      const double* wk = ctx->winv + (size_t)b * nb * nb;
      trsv_diag_kernel<<<1, 256, 0, ctx->stream>>>(wk, nb, kb, B + k, (size_t)ldb, nc, 0);
      LAUNCH_CHECK(ctx);
      if (k > 0) {
        gemv_n_update_kernel<<<(k + 255) / 256, 256, 0, ctx->stream>>>(
            dU + (size_t)k * ldu, (size_t)ldu, kb, k, B + k, (size_t)ldb, B, (size_t)ldb, nc);
        LAUNCH_CHECK(ctx);
      }
    }
  }
  return 0;
}

extern "C" {

int gpr_potrf_upper(gpr_ctx_t ctx, double* dA, int n, int lda, int* info) {
  if (!dA && n > 0) return set_err(ctx, GPR_E_ARG, "dA is NULL");
  if (n < 0 || lda < std::max(1, n)) return set_err(ctx, GPR_E_ARG, "bad n/lda (%d, %d)", n, lda);
  if (n == 0) {
    if (info) *info = 0;
    return 0;
  }
  int hinfo = 0;
  GPR_TRY(potrf_core(ctx, dA, n, lda, &hinfo));
  if (info) *info = hinfo;
  return hinfo;
}

int gpr_potrs_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                    int ldb) {
  if (n < 0 || nrhs < 0 || ldu < std::max(1, n) || ldb < std::max(1, n))
    return set_err(ctx, GPR_E_ARG, "bad sizes");
  if (n == 0 || nrhs == 0) return 0;
  return potrs_core(ctx, dU, n, ldu, dB, nrhs, ldb);
}

int gpr_trsm_upper_trans(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                         int ldb) {
  if (n < 0 || nrhs < 0 || ldu < std::max(1, n) || ldb < std::max(1, n))
    return set_err(ctx, GPR_E_ARG, "bad sizes");
  if (n == 0 || nrhs == 0) return 0;
  return trsm_ut_core(ctx, dU, n, ldu, dB, nrhs, ldb, nullptr, 0);
}

int gpr_potri_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dKinv, int ldk) {
  if (n <= 0 || ldu < n || ldk < n) return set_err(ctx, GPR_E_ARG, "bad sizes");
  GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, (size_t)n * n));
  double* Z = ctx->dbig;
  GPR_TRY(launch_set_identity(ctx, Z, n, n));
  GPR_TRY(trsm_ut_core(ctx, dU, n, ldu, Z, n, n, nullptr, 1));  // Z = U^{-T}
  return kinv_from_z(ctx, Z, n, dKinv, ldk);
}

}  // extern "C"

// K^{-1} = Z^T Z (upper, round-robin K-range SYRK) mirrored to the full matrix, Z = U^{-T}
int kinv_from_z(gpr_ctx* ctx, const double* Z, int n, double* dKinv, int ldk) {
  GemmArgs g{};
  g.P = Z; g.ldp = n;
  g.Q = Z; g.ldq = n;
  g.C = dKinv; g.ldc = ldk;
  g.M = n; g.N = n; g.K = n;
  g.alpha = 1.0; g.beta = 0.0;
  g.upper = 1; g.kfrom_n = 1;
  GPR_TRY(launch_gemm_tn(ctx, g, TC_SYRK));   // K^{-1} = Z^T Z (upper)
  GPR_TRY(launch_mirror_upper(ctx, dKinv, n, ldk));
  return 0;
}
