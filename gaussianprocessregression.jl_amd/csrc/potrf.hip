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

namespace {

constexpr int DIAG_THREADS = 512;

// Factor (mode 1) or only invert an existing factor (mode 0) of one NB x NB diagonal block.
// mode 1: one launch per panel, block at A + kglob*(lda+1), size kb = min(NB, n-kglob);
// mode 0: grid = number of blocks, block b at A + b*NB*(lda+1).
//
// Register-owned right-looking algorithm: thread (tr, tc) = (t & 31, t >> 5) owns the
// elements (tr + 32a, tc + 16b) of the block (upper part), so each of the NB sequential
// steps is: owners of the pivot row publish it to a double-buffered LDS row, ONE barrier,
// every thread updates its elements from the broadcast row.  The inverse U^{-1} (needed so
// the panel TRSM becomes an MFMA GEMM) is built the same way (X U = I, right-looking over
// columns) with U read from an LDS copy.  Padding beyond kb is the identity.
template <int NB>
__global__ __launch_bounds__(DIAG_THREADS) void diag_block_kernel(double* __restrict__ A,
                                                                  size_t lda, int n, int kglob,
                                                                  int* __restrict__ info,
                                                                  double* __restrict__ winv,
                                                                  int mode) {
  constexpr int LD = NB + 1;
  constexpr int RA = NB / 32, CB = NB / 16;
  __shared__ double S[NB * LD];
  __shared__ double buf[2][NB];
  if (*info != 0) return;
  const int tid = threadIdx.x;
  const int tr = tid & 31, tc = tid >> 5;
  int k0, kb;
  if (mode == 1) {
    k0 = kglob;
    kb = min(NB, n - kglob);
  } else {
    k0 = blockIdx.x * NB;
    kb = min(NB, n - k0);
    winv += (size_t)blockIdx.x * NB * NB;
  }
  double* Ab = A + (size_t)k0 + (size_t)k0 * lda;
  STAMP(0);
  double a[RA][CB];
#pragma unroll
  for (int ai = 0; ai < RA; ++ai)
#pragma unroll
    for (int bi = 0; bi < CB; ++bi) {
      const int r = tr + 32 * ai, c = tc + 16 * bi;
      double v = (r == c) ? 1.0 : 0.0;
      if (r < kb && c < kb && r <= c) v = Ab[(size_t)r + (size_t)c * lda];
      a[ai][bi] = v;
    }

  STAMP(1);
  if (mode == 1) {
    for (int j = 0; j < kb; ++j) {
      const int p = j & 1;
      if (tr == (j & 31)) {  // owners of row j publish it (entries c < j are never read)
        const int aj = j >> 5;
#pragma unroll
        for (int bi = 0; bi < CB; ++bi) {
          double v = a[0][bi];
#pragma unroll
          for (int ai = 1; ai < RA; ++ai) v = (ai == aj) ? a[ai][bi] : v;
          buf[p][tc + 16 * bi] = v;
        }
      }
      __syncthreads();
      const double dj = buf[p][j];
      if (!(dj > 0.0)) {  // also catches NaN (dpotf2: ajj <= 0 .or. disnan(ajj))
        if (tid == 0) *info = kglob + j + 1;
        return;
      }
      const double u = sqrt(dj);
      const double ri = 1.0 / u;
      double ur[RA], uc[CB];
#pragma unroll
      for (int ai = 0; ai < RA; ++ai) {
        const int r = tr + 32 * ai;
        const double v = buf[p][r];  // unconditional load, then select (no branch/wait)
        ur[ai] = (r > j) ? v * ri : 0.0;
      }
#pragma unroll
      for (int bi = 0; bi < CB; ++bi) {
        const int c = tc + 16 * bi;
        const double v = buf[p][c];
        uc[bi] = (c > j) ? v * ri : 0.0;
      }
      // ur/uc are zero outside the trailing block, so the rank-1 update is a no-op there
      // (elements below the diagonal take garbage that is never stored).  Row/column blocks
      // that are entirely finished (<= j) are skipped with wave-uniform branches.
#pragma unroll
      for (int ai = 0; ai < RA; ++ai) {
        if (32 * ai + 31 < j) continue;
        const int r = tr + 32 * ai;
#pragma unroll
        for (int bi = 0; bi < CB; ++bi) {
          if (16 * bi + 15 < j) continue;
          const int c = tc + 16 * bi;
          const double upd = fma(-ur[ai], uc[bi], a[ai][bi]);
          if (32 * ai <= j) {  // this row block contains row j: finalise U[j][c]
            const double rowj = (c == j) ? u : ((c > j) ? uc[bi] : a[ai][bi]);
            a[ai][bi] = (r == j) ? rowj : upd;
          } else {
            a[ai][bi] = upd;
          }
        }
      }
    }
  }

  STAMP(2);
  // U (upper) -> LDS copy (and back to global in mode 1)
#pragma unroll
  for (int ai = 0; ai < RA; ++ai)
#pragma unroll
    for (int bi = 0; bi < CB; ++bi) {
      const int r = tr + 32 * ai, c = tc + 16 * bi;
      if (r <= c) {
        S[r + c * LD] = a[ai][bi];
        if (mode == 1 && r < kb && c < kb) Ab[(size_t)r + (size_t)c * lda] = a[ai][bi];
      }
    }
  // X = U^{-1}: X U = I, right-looking over columns; X owned like U, starts as I.
#pragma unroll
  for (int ai = 0; ai < RA; ++ai)
#pragma unroll
    for (int bi = 0; bi < CB; ++bi) a[ai][bi] = (tr + 32 * ai == tc + 16 * bi) ? 1.0 : 0.0;
  __syncthreads();
  STAMP(3);
  for (int r = 0; r < kb; ++r) {
    const int p = r & 1;
    const double urr = S[r + r * LD];
    if (tc == (r & 15)) {  // owners of column r finalise it: X[i][r] /= U[r][r]
      const int br = r >> 4;
#pragma unroll
      for (int ai = 0; ai < RA; ++ai) {
        double v = a[ai][0];
#pragma unroll
        for (int bi = 1; bi < CB; ++bi) v = (bi == br) ? a[ai][bi] : v;
        const double x = v / urr;
        const bool fin = (tr + 32 * ai) <= r;
#pragma unroll
        for (int bi = 0; bi < CB; ++bi) a[ai][bi] = (bi == br && fin) ? x : a[ai][bi];
        buf[p][tr + 32 * ai] = x;  // entries i > r are never read
      }
    }
    __syncthreads();
    double xc[RA], ur[CB];
#pragma unroll
    for (int ai = 0; ai < RA; ++ai) {
      const int i = tr + 32 * ai;
      const double v = buf[p][i];
      xc[ai] = (i <= r) ? v : 0.0;
    }
#pragma unroll
    for (int bi = 0; bi < CB; ++bi) {
      const int jj = tc + 16 * bi;
      const double v = S[r + jj * LD];
      ur[bi] = (jj > r) ? v : 0.0;
    }
#pragma unroll
    for (int ai = 0; ai < RA; ++ai) {
      if (32 * ai > r) continue;            // rows i > r untouched
#pragma unroll
      for (int bi = 0; bi < CB; ++bi) {
        if (16 * bi + 15 <= r) continue;    // columns jj <= r finished
        a[ai][bi] = fma(-xc[ai], ur[bi], a[ai][bi]);
      }
    }
  }
  STAMP(4);
  // write U^{-1} (upper, zero below, zero outside kb) to the workspace slot
#pragma unroll
  for (int ai = 0; ai < RA; ++ai)
#pragma unroll
    for (int bi = 0; bi < CB; ++bi) {
      const int r = tr + 32 * ai, c = tc + 16 * bi;
      winv[r + c * NB] = (r <= c && r < kb && c < kb) ? a[ai][bi] : 0.0;
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

int launch_diag(gpr_ctx* ctx, double* A, int lda, int n, int kglob, double* winv, int mode,
                int nblocks) {
  const int nb = ctx->nb;
  TimerScope ts(ctx, TC_PANEL, 0.0);
  if (nb == 128)
    diag_block_kernel<128><<<nblocks, DIAG_THREADS, 0, ctx->ls>>>(A, (size_t)lda, n, kglob,
                                                                      ctx->dinfo, winv, mode);
  else
    diag_block_kernel<64><<<nblocks, DIAG_THREADS, 0, ctx->ls>>>(A, (size_t)lda, n, kglob,
                                                                     ctx->dinfo, winv, mode);
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
    if (j + jb < k + kw) {
      GemmArgs u{};
      u.P = row; u.ldp = lda;
      u.Q = row; u.ldq = lda;
      u.C = A + (j + jb) + (size_t)(j + jb) * lda; u.ldc = lda;
      u.M = k + kw - j - jb; u.N = n - j - jb; u.K = jb;
      u.alpha = -1.0; u.beta = 1.0;
      u.mask_upper = 1;
      u.info = ctx->dinfo;
      GPR_TRY(launch_gemm_tn(ctx, u, TC_PANEL));
    }
  }
  return 0;
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

}  // namespace

// Two-level right-looking upper Cholesky with depth-1 lookahead.
//   outer panels P_s = rows [s*nb2, (s+1)*nb2)      (nb2 = K of the big MFMA updates)
//   stream2 (panel):  wait b_{s-1}; a_s = update of rows P_{s+1} by P_s; factor P_{s+1}
//   stream  (main):   wait panel_s; b_s = SYRK of rows/cols >= (s+2)*nb2 by P_s
// so the latency-bound diag/TRSM chain of panel s+1 overlaps the big SYRK b_s.
int potrf_core(gpr_ctx* ctx, double* dA, int n, int lda, int* info) {
  const int nb = ctx->nb;
  const int nb2 = std::max(nb, (ctx->nb2 / nb) * nb);
  ctx->fac_valid = false;
  GPR_TRY(ensure_winv(ctx, n, nb));
  hipStream_t s0 = ctx->stream, s1 = ctx->stream2;
  HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), s0));
  size_t ev = 0;
  hipEvent_t e0 = sync_event(ctx, ev++);
  HIP_TRY(ctx, hipEventRecord(e0, s0));
  HIP_TRY(ctx, hipStreamWaitEvent(s1, e0, 0));
  ctx->ls = s1;
  int rc = factor_panel(ctx, dA, n, lda, 0, std::min(nb2, n));
  hipEvent_t ev_p = sync_event(ctx, ev++);
  hipEvent_t ev_b = nullptr;
  if (!rc && hipEventRecord(ev_p, s1) != hipSuccess) rc = GPR_E_HIP;
  for (int k = 0; !rc && k + nb2 < n; k += nb2) {
    const int kend = k + nb2, w2 = std::min(nb2, n - kend), rest0 = kend + w2;
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
    if ((rc = factor_panel(ctx, dA, n, lda, kend, w2))) break;
    hipEvent_t ev_p_next = sync_event(ctx, ev++);
    if (hipEventRecord(ev_p_next, s1) != hipSuccess) { rc = GPR_E_HIP; break; }
    // ---- main stream: b_s
    ctx->ls = s0;
    if (hipStreamWaitEvent(s0, ev_p, 0) != hipSuccess) { rc = GPR_E_HIP; break; }
    if (rest0 < n) {
      GemmArgs b{};
      b.P = dA + k + (size_t)rest0 * lda; b.ldp = lda;
      b.Q = b.P; b.ldq = lda;
      b.C = dA + rest0 + (size_t)rest0 * lda; b.ldc = lda;
      b.M = n - rest0; b.N = n - rest0; b.K = nb2;
      b.alpha = -1.0; b.beta = 1.0;
      b.upper = 1;
      b.info = ctx->dinfo;
      if ((rc = launch_gemm_tn(ctx, b, TC_SYRK))) break;
    }
    ev_b = sync_event(ctx, ev++);
    if (hipEventRecord(ev_b, s0) != hipSuccess) { rc = GPR_E_HIP; break; }
    ev_p = ev_p_next;
  }
  ctx->ls = s0;
  hipEvent_t ej = sync_event(ctx, ev++);  // join the panel stream into the main stream
  HIP_TRY(ctx, hipEventRecord(ej, s1));
  HIP_TRY(ctx, hipStreamWaitEvent(s0, ej, 0));
  if (rc) return rc;
  int hinfo = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost, s0));
  HIP_TRY(ctx, hipStreamSynchronize(s0));
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

// B <- U^{-T} B (U^T X = B), GEMM-based (any nrhs), two-level with the same lookahead
// structure as potrf_core.  norm_out: optional norm_out[c] -= ||X[:, c]||^2 (fused in the
// panel GEMM epilogue).  lower_rhs: B is lower-triangular (identity RHS) -> outer block s
// only touches columns [0, (s+1) nb2).
int trsm_ut_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                 int ldb, double* norm_out, int lower_rhs) {
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
int potrs_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs, int ldb) {
  GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
  const int nb = ctx->nb;
  const int nblk = (n + nb - 1) / nb;
  for (int c0 = 0; c0 < nrhs; c0 += RHS_CHUNK) {
    const int nc = std::min(RHS_CHUNK, nrhs - c0);
    double* B = dB + (size_t)c0 * ldb;
    // forward
    for (int b = 0; b < nblk; ++b) {
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
    for (int b = nblk - 1; b >= 0; --b) {
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

}  // extern "C"
