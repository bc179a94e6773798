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

namespace {

constexpr int DIAG_THREADS = 512;

// Factor (mode 1) or only invert an existing factor (mode 0) of one diagonal block.
// mode 1: one launch per panel, blockIdx.x == 0, block at A (lda), size kb, global offset
//         kglob; mode 0: grid = number of blocks, block b at A + b*nb*(lda+1).
template <int NB>
__global__ __launch_bounds__(DIAG_THREADS) void diag_block_kernel(double* __restrict__ A,
                                                                  size_t lda, int n, int kglob,
                                                                  int* __restrict__ info,
                                                                  double* __restrict__ winv,
                                                                  int mode) {
  constexpr int LD = NB + 1;
  __shared__ double S[NB * LD];
  __shared__ double Sd[NB];
  if (*info != 0) return;
  const int tid = threadIdx.x;
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
  for (int idx = tid; idx < NB * NB; idx += DIAG_THREADS) {
    const int r = idx % NB, c = idx / NB;
    double v = (r == c) ? 1.0 : 0.0;
    if (r < kb && c < kb && r <= c) v = Ab[(size_t)r + (size_t)c * lda];
    S[r + c * LD] = v;
  }
  __syncthreads();

  if (mode == 1) {
    for (int j = 0; j < kb; ++j) {
      const double ajj = S[j + j * LD];
      if (!(ajj > 0.0)) {  // also catches NaN (dpotf2: ajj <= 0 .or. disnan(ajj))
        if (tid == 0) *info = kglob + j + 1;
        return;
      }
      const double ujj = sqrt(ajj);
      __syncthreads();
      for (int c = j + tid; c < kb; c += DIAG_THREADS)
        S[j + c * LD] = (c == j) ? ujj : S[j + c * LD] / ujj;
      __syncthreads();
      const int nc = kb - j - 1;
      for (int idx = tid; idx < nc * nc; idx += DIAG_THREADS) {
        const int rr = idx % nc, cc = idx / nc;
        if (rr <= cc) {
          const int r = j + 1 + rr, c = j + 1 + cc;
          S[r + c * LD] -= S[j + r * LD] * S[j + c * LD];
        }
      }
      __syncthreads();
    }
  }

  // W = U^{-T} (lower): U^T W = I, row by row; 8 lanes per column, 64 columns per pass.
  const int sub = tid & 7, colg = tid >> 3;
  for (int r = 0; r < kb; ++r) {
    const double urr = S[r + r * LD];
    for (int c0 = 0; c0 <= r; c0 += DIAG_THREADS / 8) {
      const int c = c0 + colg;
      double s = 0.0;
      if (c <= r) {
        for (int p = c + sub; p < r; p += 8) {
          const double wpc = (p == c) ? Sd[c] : S[p + c * LD];
          s = fma(S[p + r * LD], wpc, s);
        }
      }
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      if (c <= r && sub == 0) {
        if (c == r)
          Sd[r] = 1.0 / urr;
        else
          S[r + c * LD] = (-s) / urr;
      }
    }
    __syncthreads();
  }

  // write U back (mode 1) and U^{-1}[k][m] = W[m][k] (upper) to the workspace slot
  for (int idx = tid; idx < NB * NB; idx += DIAG_THREADS) {
    const int r = idx % NB, c = idx / NB;
    if (mode == 1 && r < kb && c < kb && r <= c) Ab[(size_t)r + (size_t)c * lda] = S[r + c * LD];
    double wv = 0.0;
    if (r < kb && c < kb) wv = (r == c) ? Sd[r] : (r < c ? S[c + r * LD] : 0.0);
    winv[r + c * NB] = wv;
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
    diag_block_kernel<128><<<nblocks, DIAG_THREADS, 0, ctx->stream>>>(A, (size_t)lda, n, kglob,
                                                                      ctx->dinfo, winv, mode);
  else
    diag_block_kernel<64><<<nblocks, DIAG_THREADS, 0, ctx->stream>>>(A, (size_t)lda, n, kglob,
                                                                     ctx->dinfo, winv, mode);
  LAUNCH_CHECK(ctx);
  return 0;
}

}  // namespace

int potrf_core(gpr_ctx* ctx, double* dA, int n, int lda, int* info) {
  const int nb = ctx->nb;
  ctx->fac_valid = false;
  GPR_TRY(ensure_winv(ctx, n, nb));
  HIP_TRY(ctx, hipMemsetAsync(ctx->dinfo, 0, sizeof(int), ctx->stream));
  for (int k = 0; k < n; k += nb) {
    const int kb = std::min(nb, n - k);
    double* wk = ctx->winv + (size_t)(k / nb) * nb * nb;
    GPR_TRY(launch_diag(ctx, dA, lda, n, k, wk, 1, 1));
    const int rest = n - k - kb;
    if (rest <= 0) break;
    double* panel = dA + k + (size_t)(k + kb) * lda;
    GemmArgs g{};
    g.P = wk; g.ldp = nb;
    g.Q = panel; g.ldq = lda;
    g.C = panel; g.ldc = lda;
    g.M = kb; g.N = rest; g.K = kb;
    g.alpha = 1.0; g.beta = 0.0;
    g.info = ctx->dinfo;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_PANEL));
    GemmArgs s{};
    s.P = panel; s.ldp = lda;
    s.Q = panel; s.ldq = lda;
    s.C = dA + (k + kb) + (size_t)(k + kb) * lda; s.ldc = lda;
    s.M = rest; s.N = rest; s.K = kb;
    s.alpha = -1.0; s.beta = 1.0;
    s.upper = 1;
    s.info = ctx->dinfo;
    GPR_TRY(launch_gemm_tn(ctx, s, TC_SYRK));
  }
  int hinfo = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&hinfo, ctx->dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
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

// B <- U^{-T} B (Uᵀ X = B), GEMM-based (any nrhs).  norm_out: optional per-column
// accumulation norm_out[c] -= ||X[:, c]||^2.  lower_rhs: B is lower-triangular
// (identity RHS) -> step b only touches columns [0, (b+1) nb).
int trsm_ut_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                 int ldb, double* norm_out, int lower_rhs) {
  GPR_TRY(ensure_factor_inverses(ctx, dU, n, ldu));
  const int nb = ctx->nb;
  for (int k = 0; k < n; k += nb) {
    const int kb = std::min(nb, n - k);
    const int ncols = lower_rhs ? std::min(nrhs, k + kb) : nrhs;
    double* wk = ctx->winv + (size_t)(k / nb) * nb * nb;
    GemmArgs g{};
    g.P = wk; g.ldp = nb;
    g.Q = dB + k; g.ldq = ldb;
    g.C = dB + k; g.ldc = ldb;
    g.M = kb; g.N = ncols; g.K = kb;
    g.alpha = 1.0; g.beta = 0.0;
    g.norm_out = norm_out;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_TRSM_GEMM));
    const int rest = n - k - kb;
    if (rest <= 0) break;
    GemmArgs s{};
    s.P = dU + k + (size_t)(k + kb) * ldu; s.ldp = ldu;
    s.Q = dB + k; s.ldq = ldb;
    s.C = dB + k + kb; s.ldc = ldb;
    s.M = rest; s.N = ncols; s.K = kb;
    s.alpha = -1.0; s.beta = 1.0;
    GPR_TRY(launch_gemm_tn(ctx, s, TC_TRSM_GEMM));
  }
  return 0;
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
