// Fit, posterior and split-kernel block prediction on gfx950.
//
// gpr_fit      = update_cache!(MllLossCache / GPRPredictCache)  src/cost.jl:74-81,
//                src/predict.jl:29-34
// gpr_predict  = predict!/predict_mean!                         src/predict.jl:36-101
// gpr_split_predict = kernel!(::SplitKernel) + split mean/var  src/split_kernel.jl:137-159,
//                src/split_predict.jl:5-53
//
// Layout choice: the cross kernel is built TRANSPOSED w.r.t. the reference (Kpx = K(x, xp),
// n x m, column j = test point j, contiguous over the training index), so that
//   mu = Kpx^T wt               is a column-GEMV (coalesced), and
//   V  = U^{-T} Kpx             is the same left-upper-transposed TRSM (MFMA GEMMs) as the
//                               POTRF panels -- rdiv!(Kxp, U) of src/predict.jl:84 on Kxp^T,
// with the diagonal variance ||V[:, j]||^2 accumulated in the TRSM's GEMM epilogue
// (src/predict.jl:89-95 without a second pass over V).
#include <algorithm>
#include <cmath>
#include <functional>
#include <mutex>
#include <thread>

#ifdef GPR_TESTING  // (the rocSOLVER comparator of gpr_integrate_noise: test build only)
#include <dlfcn.h>
#include <rocsolver/rocsolver.h>
#endif

#include "common.hpp"

namespace {

// y[j + c*ldy] = sum_i A[i + j*lda] x[i + c*ldx]: one wave per column j.
__global__ __launch_bounds__(256) void colgemv_kernel(const double* __restrict__ A, size_t lda,
                                                      int nrows, int ncols,
                                                      const double* __restrict__ x, size_t ldx,
                                                      int nrhs, double* __restrict__ y, size_t ldy) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= ncols) return;
  const double* col = A + (size_t)j * lda;
  for (int c = 0; c < nrhs; ++c) {
    const double* xc = x + (size_t)c * ldx;
    double s = 0.0;
    for (int i = lane; i < nrows; i += 64) s = fma(col[i], xc[i], s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) y[(size_t)j + (size_t)c * ldy] = s;
  }
}

// The diagonal posterior from V = U^{-T} K(x, xp) and z = U^{-T} y in ONE read of V (one wave
// per column j): mu[j] = V_j^T z, var[j] = prior - ||V_j||^2 (colgemv + fill + colnorm_sub
// fused; the order of each sum as in those kernels' lanes, 16-B loads when n is even)
__global__ __launch_bounds__(256) void colgemv_norm_kernel(const double* __restrict__ V, size_t ldv,
                                                           int n, int m,
                                                           const double* __restrict__ z,
                                                           double prior, double* __restrict__ mu,
                                                           double* __restrict__ var) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= m) return;
  const double* col = V + (size_t)j * ldv;
  double s = 0.0, q = 0.0;
  int i = 2 * lane;
  if (((ldv | n) & 1) == 0 && ((uintptr_t)V & 15) == 0 && ((uintptr_t)z & 15) == 0) {
    for (; i + 1 < n; i += 128) {
      const d2 v = *reinterpret_cast<const d2*>(col + i);
      const d2 w = *reinterpret_cast<const d2*>(z + i);
      s = fma(v.x, w.x, fma(v.y, w.y, s));
      q = fma(v.x, v.x, fma(v.y, v.y, q));
    }
  } else {
    for (i = lane; i < n; i += 64) {
      s = fma(col[i], z[i], s);
      q = fma(col[i], col[i], q);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  if (lane == 0) {
    mu[j] = s;
    var[j] = prior - q;
  }
}

__global__ void fill_kernel(double* __restrict__ p, size_t n, double v) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x)
    p[t] = v;
}

// KxqT[s + (jr*nq + q)*ns] = sum_p (A_p[el][q] * BT_p[s][el]) * C_p[s][q], el = e - e_lo.
// Reference: Kxq .+= A[e,q] .* B[e,s] .* C[s,q]  (src/split_predict.jl:45-47), parts summed
// from zero in order.
__global__ __launch_bounds__(256) void split_kxq_kernel(int nse, const double* __restrict__ A,
                                                        const double* __restrict__ BT,
                                                        const double* __restrict__ C, int ns,
                                                        int nq, int E_loc, int el0, int nrows,
                                                        double* __restrict__ out) {
  const size_t total = (size_t)ns * nq * nrows;
  const size_t szA = (size_t)E_loc * nq, szB = (size_t)ns * E_loc, szC = (size_t)ns * nq;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int s = (int)(t % ns);
    const size_t col = t / ns;
    const int q = (int)(col % nq);
    const int el = el0 + (int)(col / nq);
    double v = 0.0;
    for (int p = 0; p < nse; ++p) {
      const double a = A[p * szA + (size_t)el + (size_t)q * E_loc];
      const double b = BT[p * szB + (size_t)s + (size_t)el * ns];
      const double c = C[p * szC + (size_t)s + (size_t)q * ns];
      v += (a * b) * c;
    }
    out[t] = v;
  }
}

int launch_fill(gpr_ctx* ctx, double* p, size_t n, double v) {
  if (n == 0) return 0;
  int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
  fill_kernel<<<blocks, 256, 0, ctx->stream>>>(p, n, v);
  LAUNCH_CHECK(ctx);
  return 0;
}

// diagonal-variance prior: sigma^2 for a single SE (src/predict.jl:67); composed kernels:
// sum over ALL parts of hp_part[1]^2, noise included (src/predict.jl:56-58).  No eps.
double diag_prior(const int* kinds, int nk, const double* hp, int d) {
  if (nk == 1) return hp[0] * hp[0];
  double s = 0.0;
  int off = 0;
  for (int t = 0; t < nk; ++t) {
    s += hp[off] * hp[off];
    off += kinds[t] == GPR_SE ? d + 1 : 1;
  }
  return s;
}

// ---- Bayesian quadrature of the posterior (src/integrate.jl) ------------------------------
constexpr double RT_PI_BY_2 = 0.88622692545275801365;  // sqrt(pi) / 2

// erf(x, y) = erf(y) - erf(x), evaluated through erfc where both arguments lie on the same
// side beyond 1/sqrt(2) (no cancellation of two values near +-1), as SpecialFunctions' two-
// argument erf the reference calls (src/integrate.jl:4,26)
__host__ __device__ inline double erf_diff(double x, double y) {
  const double t = 0.70710678118654752440;
  if (x > t && y > t) return erfc(x) - erfc(y);
  if (x < -t && y < -t) return erfc(-y) - erfc(-x);
  return erf(y) - erf(x);
}

// k1[j] = prefac * prod_i erf(l_i (a_i - x_ij), l_i (b_i - x_ij))  (antideriv!, :16-31)
__global__ void antideriv_se_kernel(const double* __restrict__ X, int n, int d, KParams kp,
                                    const double* __restrict__ ab, double prefac,
                                    double* __restrict__ k1) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    double v = 1.0;
    for (int i = 0; i < d; ++i) {
      const double l = kp.l[0][i], x = X[(size_t)j * d + i];
      v *= erf_diff(l * (ab[i] - x), l * (ab[d + i] - x));
    }
    k1[j] = v * prefac;
  }
}

// erf_integ(w, a, b) (src/integrate.jl:6-7): the double integral of exp(-w^2 (x - y)^2)
double erf_integ(double w, double a, double b) {
  return 1.0 / (w * w) * (std::exp(-(w * (b - a)) * (w * (b - a))) - 1.0) +
         2.0 * (RT_PI_BY_2 / w) * (b - a) * std::erf(w * (b - a));
}


// ---- cross-validation (src/crossval.jl, losses src/loss_grad.jl:12-30) ---------------------
// xo[:, j] = X[:, idx[j]], yo[j] = y[idx[j]] (the views x[:, tst[i]] etc. of cv_batch :27-30);
// indices were range-checked on the host.
__global__ void cv_gather_kernel(const double* __restrict__ X, const double* __restrict__ y, int d,
                                 const int* __restrict__ idx, int m, double* __restrict__ xo,
                                 double* __restrict__ yo) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < m * (d + 1); t += gridDim.x * blockDim.x) {
    const int j = t / (d + 1), i = t - j * (d + 1);
    const size_t src = (size_t)idx[j];
    if (i < d) xo[(size_t)j * d + i] = X[src * d + i];
    else yo[j] = y[src];
  }
}

// One workgroup: mode GPR_COST_MSE -> sum((yt - yp)^2) / m; GPR_COST_CHISQ -> sum((yt - yp)^2 /
// S_ii); 0 -> sum(yp^2) (yp = L^{-1} (y - yp), Mahalanobis); -1 -> yp <- yt - yp, no reduction.
__global__ __launch_bounds__(256) void cv_loss_kernel(const double* __restrict__ yt,
                                                      double* __restrict__ yp,
                                                      const double* __restrict__ S, size_t lds,
                                                      int m, int mode, double* __restrict__ out) {
  __shared__ double part[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < m; i += 256) {
    if (mode == -1) {
      yp[i] = yt[i] - yp[i];
      continue;
    }
    const double r = mode == 0 ? yp[i] : yt[i] - yp[i];
    s += mode == GPR_COST_CHISQ ? r * r / S[(size_t)i * lds + i] : r * r;
  }
  if (mode == -1) return;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (part[0] + part[1]) + (part[2] + part[3]);
    *out = mode == GPR_COST_MSE ? t / m : t;
  }
}


// Kj = upper(K) + s I (the triangle POTRF reads), column-major, ld n
__global__ void shift_upper_kernel(const double* __restrict__ K, size_t ldk, int n, double s,
                                   double* __restrict__ Kj) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)n * n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % n), j = (int)(t / n);
    if (i <= j) Kj[t] = K[(size_t)j * ldk + i] + (i == j ? s : 0.0);
  }
}

// Kxp of predict!/predict_mean! (src/predict.jl:37,43): kernel!(pc.Kxp, covar, hp, xp, md.x),
// stored transposed here (n x m, ld n).  When the caller passes the training inputs
// themselves (dXp == dX, the C analogue of `xp === md.x`) the reference's 5-arg kernel! takes
// its same-object branch: eps once per SE part on the diagonal and NO noise
// (src/covariance.jl:52-56, src/compose_covar.jl:47-61) -- the symmetric kernel without the
// WhiteNoise term.  Any other xp is a plain cross kernel (no eps, no noise).
int launch_cross_or_same(gpr_ctx* ctx, const KParams& kp, const double* dX, int n,
                         const double* dXp, int m, double* out) {
  if (dXp == dX && m == n) {
    KParams k5 = kp;
    k5.has_noise = 0;
    return launch_kernel_matrix(ctx, k5, dX, n, nullptr, n, 1, out, n);
  }
  return launch_kernel_matrix(ctx, kp, dX, n, dXp, m, 0, out, n);
}

}  // namespace

extern "C" {

int gpr_fit(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d, const double* dX,
            int n, const double* dy, int nrhs, int ldy, double eps, double* dK, int ldk,
            double* dalpha, int* info) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || ldk < n || nrhs <= 0 || ldy < n || !dX || !dy || !dK || !dalpha)
    return set_err(ctx, GPR_E_ARG, "bad args");
  GPR_TRY(launch_kernel_matrix_for_factor(ctx, kp, dX, n, dK, ldk));
  HIP_TRY(ctx, hipMemcpy2DAsync(dalpha, (size_t)n * sizeof(double), dy, (size_t)ldy * sizeof(double),
                                (size_t)n * sizeof(double), nrhs, hipMemcpyDeviceToDevice, ctx->stream));
  int hinfo = 0;
  if (ctx->fuse_y) {
    // z = U^{-T} y solved inside the factorisation (a right-hand-side column of the tile-DAG
    // launch, or the blocked path's side stream), then the backward sweep
    RhsSpec rhs{dalpha, nrhs, n, 0, ctx->fused_rhs == 2 ? 2 : 1, nullptr, 0};
    GPR_TRY(potrf_core(ctx, dK, n, ldk, &hinfo, &rhs));
    if (info) *info = hinfo;
    if (hinfo != 0) return hinfo;
    return potrs_core(ctx, dK, n, ldk, dalpha, nrhs, n, /*forward=*/!ctx->rhs_solved);
  }
  GPR_TRY(potrf_core(ctx, dK, n, ldk, &hinfo));
  if (info) *info = hinfo;
  if (hinfo != 0) return hinfo;
  GPR_TRY(potrs_core(ctx, dK, n, ldk, dalpha, nrhs, n));
  return 0;
}

int gpr_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d, const double* dX,
                int n, const double* dU, int ldu, const double* dwt, int nrhs, const double* dXp,
                int m, int mode, double eps, double* dmu, double* dvar, int ldv, double* dwork) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || m <= 0 || ldu < n || nrhs <= 0 || !dX || !dU || !dwt || !dXp || !dmu)
    return set_err(ctx, GPR_E_ARG, "bad args");
  if (mode != GPR_PREDICT_MEAN && !dvar) return set_err(ctx, GPR_E_ARG, "dvar is NULL");
  if (mode == GPR_PREDICT_FULL && ldv < m) return set_err(ctx, GPR_E_ARG, "ldv < m");
  double* Kpx = dwork;
  if (!Kpx) {
    GPR_TRY(ensure_buf(ctx, &ctx->dbig2, &ctx->big2_cap, (size_t)n * m));
    Kpx = ctx->dbig2;
  }
  GPR_TRY(launch_cross_or_same(ctx, kp, dX, n, dXp, m, Kpx));  // K(x, xp), n x m
  {
    TimerScope ts(ctx, TC_OTHER, 0.0);
    colgemv_kernel<<<(m + 3) / 4, 256, 0, ctx->stream>>>(Kpx, (size_t)n, n, m, dwt, (size_t)n, nrhs,
                                                         dmu, (size_t)m);
    LAUNCH_CHECK(ctx);
  }
  if (mode == GPR_PREDICT_MEAN) return 0;
  if (mode == GPR_PREDICT_DIAG) {
    GPR_TRY(launch_fill(ctx, dvar, (size_t)m, diag_prior(kinds, nk, hp, d)));
    return trsm_ut_core(ctx, dU, n, ldu, Kpx, m, n, dvar, 0);
  }
  // full covariance: Sigma = K(xp, xp) (eps per SE part + noise) - V^T V
  GPR_TRY(trsm_ut_core(ctx, dU, n, ldu, Kpx, m, n, nullptr, 0));
  GPR_TRY(launch_kernel_matrix(ctx, kp, dXp, m, nullptr, m, 1, dvar, ldv));
  GemmArgs g{};
  g.P = Kpx; g.ldp = n;
  g.Q = Kpx; g.ldq = n;
  g.C = dvar; g.ldc = ldv;
  g.M = m; g.N = m; g.K = n;
  g.alpha = -1.0; g.beta = 1.0;
  g.upper = 1;
  GPR_TRY(launch_gemm_tn(ctx, g, TC_OTHER));
  return launch_mirror_upper(ctx, dvar, m, ldv);
}

int gpr_fit_kinv(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                 const double* dX, int n, const double* dy, int nrhs, int ldy, double eps,
                 double* dK, int ldk, double* dalpha, double* dKinv, int ldkinv, int* info) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || ldk < n || ldkinv < n || nrhs <= 0 || ldy < n || !dX || !dy || !dK || !dalpha ||
      !dKinv)
    return set_err(ctx, GPR_E_ARG, "bad args");
  GPR_TRY(launch_kernel_matrix_for_factor(ctx, kp, dX, n, dK, ldk));
  GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, (size_t)n * n));
  double* Z = ctx->dbig;
  GPR_TRY(launch_set_identity(ctx, Z, n, n));
  HIP_TRY(ctx, hipMemcpy2DAsync(dalpha, (size_t)n * sizeof(double), dy, (size_t)ldy * sizeof(double),
                                (size_t)n * sizeof(double), nrhs, hipMemcpyDeviceToDevice, ctx->stream));
  int hinfo = 0;
  // Z = U^{-T} (identity right-hand side, lower triangular) solved in the factorisation's
  // lookahead bubbles (GPR_FUSE_KINV=0: after it, as gpr_potri_upper)
  // GPR_FUSE_KINV=2 (default) also accumulates K^{-1} += Z_s^T Z_s as each row panel Z_s is
  // solved, so the N^3/3-flop Gram product fills the chain-bound half of the factorisation
  // instead of running after it
  RhsSpec rhs{Z, n, n, 1, ctx->fused_rhs == 2 ? 2 : 1, nullptr, 0};
  // auto (-1) = 2: Z and K^{-1} += Z^T Z inside the factorisation -- as right-hand-side and
  // gram tile tasks of the one tile-DAG launch when the DAG takes it (lower right-hand-side
  // rows lagged behind A's rows, GPR_DAG_ZLAG), otherwise in the blocked factorisation's
  // lookahead bubbles.  1: Z alone inside, Z^T Z after; 0: both after the factorisation.
  const int fuse = ctx->fuse_kinv >= 0 ? ctx->fuse_kinv : 2;
  if (fuse == 2) {
    rhs.gram = dKinv;
    rhs.ldg = ldkinv;
  }
  GPR_TRY(potrf_core(ctx, dK, n, ldk, &hinfo, fuse ? &rhs : nullptr));
  if (info) *info = hinfo;
  if (hinfo != 0) return hinfo;
  const bool solved = fuse && ctx->rhs_solved;
  GPR_TRY(potrs_core(ctx, dK, n, ldk, dalpha, nrhs, n));
  if (!solved) GPR_TRY(trsm_ut_core(ctx, dK, n, ldk, Z, n, n, nullptr, 1));
  if (solved && rhs.gram) return ctx->gram_full ? 0 : launch_mirror_upper(ctx, dKinv, n, ldkinv);
  return kinv_from_z(ctx, Z, n, dKinv, ldkinv);
}

int gpr_fit_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                    const double* dX, int n, const double* dy, int nrhs, int ldy, double eps,
                    double* dK, int ldk, double* dalpha, const double* dXp, int m, int mode,
                    double* dmu, double* dvar, int ldv, double* dwork, int* info) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || m <= 0 || ldk < n || nrhs <= 0 || ldy < n || !dX || !dy || !dK || !dXp || !dmu)
    return set_err(ctx, GPR_E_ARG, "bad args");
  if (mode != GPR_PREDICT_MEAN && !dvar) return set_err(ctx, GPR_E_ARG, "dvar is NULL");
  if (mode == GPR_PREDICT_FULL && ldv < m) return set_err(ctx, GPR_E_ARG, "ldv < m");
  // Fused (solve [K(x, xp) | y] inside the factorisation) pays where the factorisation is
  // chain-bound and leaves the GPU idle: measured C2 (n = 8192, np = 8192) 21.0 -> 18.9 ms,
  // n = 16384 70.9 -> 67.3; at n = 32768 the trailing SYRKs fill the GPU and the fused
  // solve slows them (r01: 347 vs 334 ms), so auto fuses only up to fused_rhs_nmax.
  // When the tile-DAG takes the whole factorisation, [K(x, xp) | y] rides in it as right-hand-
  // side tile tasks (the same launch), so auto fuses whenever the DAG applies.
  const int fmode = ctx->fused_rhs < 0
                        ? ((n <= ctx->fused_rhs_nmax || dag_takes_whole(ctx, n, ldk, dK)) ? 2 : 0)
                        : ctx->fused_rhs;
  if (mode == GPR_PREDICT_MEAN || !fmode) {
    // nothing to fuse for the mean alone (mu = K(xp, x) alpha); or the unfused reference order
    double* wt = dalpha;
    if (!wt) {
      GPR_TRY(ensure_buf(ctx, &ctx->dscr_wt, &ctx->scr_wt_cap, (size_t)n * nrhs));
      wt = ctx->dscr_wt;
    }
    int hinfo = 0;
    const int rc = gpr_fit(ctx, kinds, nk, hp, d, dX, n, dy, nrhs, ldy, eps, dK, ldk, wt, &hinfo);
    if (info) *info = hinfo;
    if (rc) return rc;
    return gpr_predict(ctx, kinds, nk, hp, d, dX, n, dK, ldk, wt, nrhs, dXp, m, mode, eps, dmu,
                       dvar, ldv, dwork);
  }
  // W = [K(x, xp) | y] (n x (m + nrhs)); POTRF solves W <- U^{-T} W in its lookahead bubbles:
  // V = U^{-T} K(x, xp) and z = U^{-T} y, then mu = V^T z (= K(xp, x) K^{-1} y) and
  // var = prior - ||V_j||^2; alpha = U^{-1} z by the backward sweep alone.
  double* W = dwork;
  if (!W) {
    GPR_TRY(ensure_buf(ctx, &ctx->dbig2, &ctx->big2_cap, (size_t)n * (m + nrhs)));
    W = ctx->dbig2;
  }
  double* Z = W + (size_t)n * m;
  GPR_TRY(launch_kernel_matrix_for_factor(ctx, kp, dX, n, dK, ldk));
  GPR_TRY(launch_cross_or_same(ctx, kp, dX, n, dXp, m, W));
  HIP_TRY(ctx, hipMemcpy2DAsync(Z, (size_t)n * sizeof(double), dy, (size_t)ldy * sizeof(double),
                                (size_t)n * sizeof(double), nrhs, hipMemcpyDeviceToDevice, ctx->stream));
  RhsSpec rhs{W, m + nrhs, n, 0, fmode == 2 ? 2 : 1, nullptr, 0};
  int hinfo = 0;
  GPR_TRY(potrf_core(ctx, dK, n, ldk, &hinfo, &rhs));
  if (info) *info = hinfo;
  if (hinfo != 0) return hinfo;
  if (!ctx->rhs_solved) GPR_TRY(trsm_ut_core(ctx, dK, n, ldk, W, m + nrhs, n, nullptr, 0));
  const bool diag1 = mode == GPR_PREDICT_DIAG && nrhs == 1;  // mean and variance in one pass
  {
    TimerScope ts(ctx, TC_OTHER, 0.0);
    if (diag1)
      colgemv_norm_kernel<<<(m + 3) / 4, 256, 0, ctx->stream>>>(
          W, (size_t)n, n, m, Z, diag_prior(kinds, nk, hp, d), dmu, dvar);
    else
      colgemv_kernel<<<(m + 3) / 4, 256, 0, ctx->stream>>>(W, (size_t)n, n, m, Z, (size_t)n,
                                                           nrhs, dmu, (size_t)m);
    LAUNCH_CHECK(ctx);
  }
  if (dalpha) {
    HIP_TRY(ctx, hipMemcpy2DAsync(dalpha, (size_t)n * sizeof(double), Z, (size_t)n * sizeof(double),
                                  (size_t)n * sizeof(double), nrhs, hipMemcpyDeviceToDevice,
                                  ctx->stream));
    GPR_TRY(potrs_core(ctx, dK, n, ldk, dalpha, nrhs, n, /*forward=*/false));
  }
  if (mode == GPR_PREDICT_DIAG) {
    if (diag1) return 0;
    GPR_TRY(launch_fill(ctx, dvar, (size_t)m, diag_prior(kinds, nk, hp, d)));
    return launch_colnorm_sub(ctx, W, n, n, m, dvar);
  }
  GPR_TRY(launch_kernel_matrix(ctx, kp, dXp, m, nullptr, m, 1, dvar, ldv));
  GemmArgs g{};
  g.P = W; g.ldp = n;
  g.Q = W; g.ldq = n;
  g.C = dvar; g.ldc = ldv;
  g.M = m; g.N = m; g.K = n;
  g.alpha = -1.0; g.beta = 1.0;
  g.upper = 1;
  GPR_TRY(launch_gemm_tn(ctx, g, TC_OTHER));
  return launch_mirror_upper(ctx, dvar, m, ldv);
}

int gpr_antideriv_se(gpr_ctx_t ctx, int d, const double* hp, const double* dX, int n,
                     const double* a, const double* b, double* dk1, double* k2) {
  if (d <= 0 || d > KMAXD || n <= 0 || !hp || !dX || !a || !b)
    return set_err(ctx, GPR_E_ARG, "bad args");
  // hp[0] = sigma, hp[1..d] = l, whatever kernel they belong to (the reference indexes
  // md.params the same way, src/integrate.jl:19-22)
  KParams kp{};
  kp.d = d;
  for (int i = 0; i < d; ++i) kp.l[0][i] = hp[1 + i];
  double prefac = hp[0] * hp[0] * std::pow(RT_PI_BY_2, d);
  double inv = 1.0;
  for (int i = 0; i < d; ++i) inv *= 1.0 / hp[1 + i];
  prefac *= inv;
  if (k2) {  // antideriv2 (:33-41): integ2 = prod_i erf_integ(l_i, a_i, b_i); * sigma^2
    double i2 = 1.0;
    for (int i = 0; i < d; ++i) i2 *= erf_integ(hp[1 + i], a[i], b[i]);
    *k2 = i2 * hp[0] * hp[0];
  }
  if (!dk1) return 0;
  GPR_TRY(ensure_buf(ctx, &ctx->dscratch, &ctx->scratch_cap, (size_t)2 * d + 2));
  double hab[2 * KMAXD];
  for (int i = 0; i < d; ++i) {
    hab[i] = a[i];
    hab[d + i] = b[i];
  }
  HIP_TRY(ctx, hipMemcpyAsync(ctx->dscratch, hab, sizeof(double) * 2 * d, hipMemcpyHostToDevice,
                              ctx->stream));
  const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  antideriv_se_kernel<<<blocks, 256, 0, ctx->stream>>>(dX, n, d, kp, ctx->dscratch, prefac, dk1);
  LAUNCH_CHECK(ctx);
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // hab is a stack array
  return 0;
}

int gpr_integrate(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                  const double* dX, int n, const double* dy, int ny, int ldy, const double* a,
                  const double* b, double eps, double* dK, int ldk, double* dwt, double* Iout,
                  double* var) {
  if (!a || !b || !Iout || !var || !dwt || ny <= 0) return set_err(ctx, GPR_E_ARG, "bad args");
  // update_cache!(wc, md, hp, nothing) (:64-69): K, cholesky!, wt = K^{-1} y
  int hinfo = 0;
  const int rc = gpr_fit(ctx, kinds, nk, hp, d, dX, n, dy, ny, ldy, eps, dK, ldk, dwt, &hinfo);
  if (rc) return rc;
  // k1, k2 (update_cache!(ac, ...) :106-110)
  GPR_TRY(ensure_buf(ctx, &ctx->dbig2, &ctx->big2_cap, (size_t)2 * n + ny + 1));
  double* k1 = ctx->dbig2;
  double* tt = k1 + n;
  double* dI = tt + n;
  double k2 = 0.0;
  GPR_TRY(gpr_antideriv_se(ctx, d, hp, dX, n, a, b, k1, &k2));
  // Iout = wt' k1 (mean_integ_impl! :124-131)
  colgemv_kernel<<<(ny + 3) / 4, 256, 0, ctx->stream>>>(dwt, (size_t)n, n, ny, k1, (size_t)n, 1,
                                                        dI, 1);
  LAUNCH_CHECK(ctx);
  // var = k2 - ||U^{-T} k1||^2 (var_integ_impl!(.., nothing, ..) :134-147: ldiv!(kchol.L, tt))
  HIP_TRY(ctx, hipMemcpyAsync(tt, k1, sizeof(double) * n, hipMemcpyDeviceToDevice, ctx->stream));
  GPR_TRY(potrs_core(ctx, dK, n, ldk, tt, 1, n, /*forward=*/true, /*backward=*/false));
  GPR_TRY(launch_fill(ctx, dI + ny, 1, k2));
  GPR_TRY(launch_colnorm_sub(ctx, tt, n, n, 1, dI + ny));
  HIP_TRY(ctx, hipMemcpyAsync(Iout, dI, sizeof(double) * ny, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(var, dI + ny, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

// child contexts for independent per-fold / per-column work (see gpr_cv_batch)
static int ensure_children(gpr_ctx* ctx, int nsub) {
  for (int t = 0; t < nsub; ++t) {
    if (ctx->cv_sub[t]) continue;
    const int rc = gpr_ctx_create(ctx->device, nullptr, &ctx->cv_sub[t]);
    if (rc) return set_err(ctx, rc, "creating a child context failed");
  }
  for (int t = 0; t < nsub; ++t) {  // (every call: the parent's settings may have changed)
    ctx->cv_sub[t]->nb = ctx->nb;
    ctx->cv_sub[t]->nb2 = ctx->nb2;
    copy_knobs(ctx, ctx->cv_sub[t]);
  }
  return 0;
}

// Batch size of a batched launch: `want` items of `per` doubles each (+ `fixed`), within the
// context's budget (GB) and half of the device memory free right now -- the buffer being
// replaced (cap doubles, freed by ensure_buf first) counts as free.  At least one.
static int batch_capacity(double budget_gb, size_t per, size_t fixed, size_t cap, int want) {
  double bytes = budget_gb * 1e9;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess)
    bytes = std::min(bytes, 0.5 * (double)fr + 8.0 * (double)cap);
  const double avail = bytes / 8.0 - (double)fixed;
  const double k = avail > 0 ? avail / (double)per : 0.0;
  return (int)std::max(1.0, std::min((double)want, std::floor(k)));
}

// A batched launch's workspace with its batch count halved on an allocation failure (another
// allocator may hold memory hipMemGetInfo counted as free) down to one item; then GPR_E_NOMEM.
static int ensure_batch_buf(gpr_ctx* ctx, int* nb, const std::function<size_t(int)>& need) {
  for (;;) {
    const int rc = ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, need(*nb));
    if (rc != GPR_E_NOMEM || *nb <= 1) return rc;
    (void)hipGetLastError();
    ctx->err.clear();
    *nb = (*nb + 1) / 2;
  }
}

// The batched paths size ctx->dbig to their batch; past a call it is released again when
// large, so a context does not keep gigabytes of scratch between calls.
static void release_big_scratch(gpr_ctx* ctx) {
  if (ctx->dbig && ctx->big_cap * sizeof(double) > (size_t)(1ull << 30)) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->dbig);
    ctx->dbig = nullptr;
    ctx->big_cap = 0;
  }
}

// Cap the number of child contexts so their workspaces (bytes_each, allocated in each child's
// dbig) take at most half of the device memory free right now; at least one child.
static int cap_children_by_memory(int nsub, size_t bytes_each) {
  size_t fr = 0, tot = 0;
  if (nsub <= 1 || bytes_each == 0 || hipMemGetInfo(&fr, &tot) != hipSuccess) return nsub;
  const size_t fit = (fr / 2) / bytes_each;
  return (int)std::max<size_t>(1, std::min<size_t>((size_t)nsub, fit));
}

// run body(child t) for t < nsub on host threads; first info > 0, else first error.  Each
// child's workspace (dbig) is released after the batch, so the extra device memory lives
// only as long as the call (the children's streams and small buffers stay for reuse).
static int run_children(gpr_ctx* ctx, int nsub, const std::function<int(gpr_ctx*, int)>& body) {
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // inputs written on the parent stream
  std::vector<int> rcs(nsub, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nsub; ++t)
    th.emplace_back([&, t] {
      hipSetDevice(ctx->device);
      rcs[t] = body(ctx->cv_sub[t], t);
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < nsub; ++t) {
    gpr_ctx* c = ctx->cv_sub[t];
    if (c && c->dbig) {
      hipStreamSynchronize(c->stream);
      hipFree(c->dbig);
      c->dbig = nullptr;
      c->big_cap = 0;
      if (c->dbig2) hipFree(c->dbig2);  // fused fit+predict workspace of the folds
      c->dbig2 = nullptr;
      if (c->dpadA) hipFree(c->dpadA);  // padded copies of odd-shaped folds
      if (c->dpadB) hipFree(c->dpadB);
      c->dpadA = c->dpadB = nullptr;
      c->padA_cap = c->padB_cap = 0;
      c->big2_cap = 0;
      c->fac_valid = false;  // cached factor data were keyed on pointers into dbig
      c->sqinv_nb2 = 0;
    }
  }
  for (int t = 0; t < nsub; ++t)
    if (rcs[t] > 0) return rcs[t];
  for (int t = 0; t < nsub; ++t)
    if (rcs[t] < 0) return set_err(ctx, rcs[t], "%s", ctx->cv_sub[t]->err.c_str());
  return 0;
}

// Folds f0, f0 + fstep, ... of gpr_cv_batch on context c (indices already range-checked);
// lss is the caller's host array, written only at this context's folds.
static int cv_folds(gpr_ctx* c, const int* kinds, int nk, const double* hp, int d,
                    const double* dX, int n, const double* dy, const int* trn, int ntrn,
                    const int* tst, int ntst, int nfold, int f0, int fstep, int cost, double eps,
                    double* lss) {
  const int nmine = (nfold - f0 + fstep - 1) / fstep;
  const size_t nidx = (size_t)nmine * (ntrn + ntst);
  // workspace (c->dbig, not touched by the fit/predict calls below): K (ntrn^2), Sigma_p
  // (ntst^2), xtrn, xtst, ytrn, ytst, yp, losses, then the int indices
  const size_t szK = (size_t)ntrn * ntrn, szS = (size_t)ntst * ntst;
  const size_t szv = (size_t)d * (ntrn + ntst) + ntrn + 2 * (size_t)ntst + nmine;
  GPR_TRY(ensure_buf(c, &c->dbig, &c->big_cap, szK + szS + szv + (nidx + 1) / 2));
  double* K = c->dbig;
  double* S = K + szK;
  double* xtr = S + szS;
  double* xts = xtr + (size_t)d * ntrn;
  double* ytr = xts + (size_t)d * ntst;
  double* yts = ytr + ntrn;
  double* yp = yts + ntst;
  double* dl = yp + ntst;
  int* di = reinterpret_cast<int*>(dl + nmine);
  std::vector<int> hidx(nidx);
  for (int i = 0; i < nmine; ++i) {
    const size_t f = (size_t)f0 + (size_t)i * fstep;
    std::copy(trn + f * ntrn, trn + (f + 1) * ntrn, hidx.begin() + (size_t)i * ntrn);
    std::copy(tst + f * ntst, tst + (f + 1) * ntst,
              hidx.begin() + (size_t)nmine * ntrn + (size_t)i * ntst);
  }
  HIP_TRY(c, hipMemcpyAsync(di, hidx.data(), nidx * sizeof(int), hipMemcpyHostToDevice,
                            c->stream));
  for (int i = 0; i < nmine; ++i) {
    const int* itr = di + (size_t)i * ntrn;
    const int* its = di + (size_t)nmine * ntrn + (size_t)i * ntst;
    cv_gather_kernel<<<std::min((ntrn * (d + 1) + 255) / 256, 1024), 256, 0, c->stream>>>(
        dX, dy, d, itr, ntrn, xtr, ytr);
    LAUNCH_CHECK(c);
    cv_gather_kernel<<<std::min((ntst * (d + 1) + 255) / 256, 1024), 256, 0, c->stream>>>(
        dX, dy, d, its, ntst, xts, yts);
    LAUNCH_CHECK(c);
    // cv_step! (:46-51): update_cache!(pc, mdt) + predict!(yp, Sigma_p, mdt, xtst, pc)
    int hinfo = 0;
    const int rc = gpr_fit_predict(c, kinds, nk, hp, d, xtr, ntrn, ytr, 1, ntrn, eps, K, ntrn,
                                   nullptr, xts, ntst, GPR_PREDICT_FULL, yp, S, ntst, nullptr,
                                   &hinfo);
    if (rc) return rc;
    if (cost == GPR_COST_MAHALANOBIS) {
      // delta = y - yp; cholesky(Sigma_p); ldiv!(L, delta); dot(delta, delta) (:25-30).
      // Sigma_p = U^T U, so L^{-1} = U^{-T}: the forward sweep
      cv_loss_kernel<<<1, 256, 0, c->stream>>>(yts, yp, S, ntst, ntst, -1, nullptr);
      LAUNCH_CHECK(c);
      GPR_TRY(potrf_core(c, S, ntst, ntst, &hinfo));
      if (hinfo != 0) return hinfo;
      GPR_TRY(potrs_core(c, S, ntst, ntst, yp, 1, ntst, /*forward=*/true, /*backward=*/false));
      cv_loss_kernel<<<1, 256, 0, c->stream>>>(yts, yp, S, ntst, ntst, 0, dl + i);
    } else {
      cv_loss_kernel<<<1, 256, 0, c->stream>>>(yts, yp, S, ntst, ntst, cost, dl + i);
    }
    LAUNCH_CHECK(c);
  }
  std::vector<double> hl(nmine);
  HIP_TRY(c, hipMemcpyAsync(hl.data(), dl, sizeof(double) * nmine, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < nmine; ++i) lss[(size_t)f0 + (size_t)i * fstep] = hl[i];
  return 0;
}

// A[c + c lda] = 1 for n <= c < n2 and zeros above it (the upper triangle of [[A, 0], [0, I]]),
// for nb matrices at stride sA
__global__ void pad_identity_kernel(double* __restrict__ A, size_t lda, size_t sA, int n, int n2,
                                    int nb) {
  const size_t per = (size_t)n2 * (n2 - n), tot = per * nb;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot;
       e += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / per);
    const size_t rem = e - (size_t)b * per;
    const int r = (int)(rem % n2), c = n + (int)(rem / n2);
    if (r <= c) A[(size_t)b * sA + r + (size_t)c * lda] = r == c ? 1.0 : 0.0;
  }
}

// gpr_cv_batch with every fold's factorisation in ONE batched tile-DAG launch (and, for
// Mahalanobis, every fold's Sigma_p factorisation in a second): per fold K_f (padded to n2, a
// multiple of 16, with the identity), W_f = [K(x_tr, x_ts) | y_tr] (zero-padded rows), the prior
// Sigma_f = K(x_ts, x_ts) (padded to s2); the launch leaves V_f = U_f^{-T} W_f, then mu =
// V_kx^T v_y, Sigma_p = Sigma_f - V_kx^T V_kx (upper triangle), and the loss -- gpr_fit_predict's
// FULL path per fold with its chain-bound factorisations batched ("cv needs batched
// small POTRFs").  Returns > 0 as the sequential path does (a fold's info), 0 when done; 1 with
// *declined set when the batched launch does not take the shape (nothing written: the shape
// is the same for every chunk, so only the first launch can decline).
static int cv_folds_batched(gpr_ctx* ctx, const KParams& kp, int d, const double* dX, int n,
                            const double* dy, const int* trn, int ntrn, const int* tst, int ntst,
                            int nfold, int cost, double* lss, bool* declined) {
  *declined = false;
  const int n2 = (ntrn + 15) / 16 * 16, s2 = (ntst + 15) / 16 * 16;
  const size_t szK = (size_t)n2 * n2, szW = (size_t)n2 * (ntst + 1), szS = (size_t)s2 * s2;
  const size_t per = szK + szW + szS + 2 * (size_t)s2 + 1;
  const size_t scratch = (size_t)d * (ntrn + ntst) + ntrn;
  auto need = [&](int k) {
    return per * k + scratch + ((size_t)k * (ntrn + ntst) + 1) / 2 + 16;
  };
  int nfc = batch_capacity(ctx->cv_batch_gb, per + (ntrn + ntst + 1) / 2, scratch + 16,
                           ctx->big_cap, nfold);
  GPR_TRY(ensure_batch_buf(ctx, &nfc, need));
  const size_t nidx = (size_t)nfc * (ntrn + ntst);
  double* Kb = ctx->dbig;                 // nfc x szK
  double* Wb = Kb + szK * nfc;            // nfc x szW
  double* Sb = Wb + szW * nfc;            // nfc x szS
  double* Yp = Sb + szS * nfc;            // nfc x s2: mu, then delta / U^{-T} delta
  double* Yt = Yp + (size_t)s2 * nfc;     // nfc x s2: y_ts
  double* dl = Yt + (size_t)s2 * nfc;     // nfc
  double* xtr = dl + nfc;
  double* xts = xtr + (size_t)d * ntrn;
  double* ytr = xts + (size_t)d * ntst;
  int* di = reinterpret_cast<int*>(ytr + ntrn);
  std::vector<int> hidx(nidx), info(nfc);
  std::vector<double> hl(nfc);
  hipStream_t st = ctx->stream;
  for (int f0 = 0; f0 < nfold; f0 += nfc) {
    const int nb = std::min(nfc, nfold - f0);
    for (int i = 0; i < nb; ++i) {
      const size_t f = (size_t)f0 + i;
      std::copy(trn + f * ntrn, trn + (f + 1) * ntrn, hidx.begin() + (size_t)i * ntrn);
      std::copy(tst + f * ntst, tst + (f + 1) * ntst, hidx.begin() + (size_t)nb * ntrn + (size_t)i * ntst);
    }
    HIP_TRY(ctx, hipMemcpyAsync(di, hidx.data(), (size_t)nb * (ntrn + ntst) * sizeof(int),
                                hipMemcpyHostToDevice, st));
    // zero-padded right-hand sides and vectors; the padded matrices' extra columns by the kernel
    HIP_TRY(ctx, hipMemsetAsync(Wb, 0, sizeof(double) * szW * nb, st));
    HIP_TRY(ctx, hipMemsetAsync(Yp, 0, sizeof(double) * 2 * (size_t)s2 * nfc, st));
    for (int i = 0; i < nb; ++i) {
      const int* itr = di + (size_t)i * ntrn;
      const int* its = di + (size_t)nb * ntrn + (size_t)i * ntst;
      double* K = Kb + szK * i;
      double* W = Wb + szW * i;
      double* S = Sb + szS * i;
      cv_gather_kernel<<<std::min((ntrn * (d + 1) + 255) / 256, 1024), 256, 0, st>>>(dX, dy, d, itr,
                                                                                   ntrn, xtr, ytr);
      LAUNCH_CHECK(ctx);
      cv_gather_kernel<<<std::min((ntst * (d + 1) + 255) / 256, 1024), 256, 0, st>>>(
          dX, dy, d, its, ntst, xts, Yt + (size_t)s2 * i);
      LAUNCH_CHECK(ctx);
      GPR_TRY(launch_kernel_matrix(ctx, kp, xtr, ntrn, nullptr, ntrn, 1, K, n2));
      GPR_TRY(launch_kernel_matrix(ctx, kp, xtr, ntrn, xts, ntst, 0, W, n2));
      HIP_TRY(ctx, hipMemcpyAsync(W + (size_t)n2 * ntst, ytr, sizeof(double) * ntrn,
                                  hipMemcpyDeviceToDevice, st));
      GPR_TRY(launch_kernel_matrix(ctx, kp, xts, ntst, nullptr, ntst, 1, S, s2));
    }
    if (n2 > ntrn) {
      pad_identity_kernel<<<1024, 256, 0, st>>>(Kb, n2, szK, ntrn, n2, nb);
      LAUNCH_CHECK(ctx);
    }
    if (s2 > ntst) {
      pad_identity_kernel<<<1024, 256, 0, st>>>(Sb, s2, szS, ntst, s2, nb);
      LAUNCH_CHECK(ctx);
    }
    int rc = launch_potrf_dag_batch(ctx, Kb, szK, n2, n2, Wb, szW, ntst + 1, n2, nb, info.data());
    if (rc == 1 && f0 == 0) {
      *declined = true;
      return 1;
    }
    if (rc) return rc == 1 ? set_err(ctx, GPR_E_HIP, "batched cross-validation: shape declined") : rc;
    for (int i = 0; i < nb; ++i)
      if (info[i] > 0) return info[i];
    for (int i = 0; i < nb; ++i) {
      const double* W = Wb + szW * i;
      double* S = Sb + szS * i;
      double* yp = Yp + (size_t)s2 * i;
      colgemv_kernel<<<(ntst + 3) / 4, 256, 0, st>>>(W, (size_t)n2, n2, ntst, W + (size_t)n2 * ntst,
                                                      (size_t)n2, 1, yp, (size_t)ntst);
      LAUNCH_CHECK(ctx);
      GemmArgs g{};
      g.P = W; g.ldp = n2;
      g.Q = W; g.ldq = n2;
      g.C = S; g.ldc = s2;
      g.M = ntst; g.N = ntst; g.K = n2;
      g.alpha = -1.0; g.beta = 1.0;
      g.upper = 1;
      GPR_TRY(launch_gemm_tn(ctx, g, TC_OTHER));
      cv_loss_kernel<<<1, 256, 0, st>>>(Yt + (size_t)s2 * i, yp, S, (size_t)s2, ntst,
                                        cost == GPR_COST_MAHALANOBIS ? -1 : cost, dl + i);
      LAUNCH_CHECK(ctx);
    }
    if (cost == GPR_COST_MAHALANOBIS) {
      // delta = y - yp; Sigma_p = U^T U; ||U^{-T} delta||^2 (:25-30) -- the second batch
      rc = launch_potrf_dag_batch(ctx, Sb, szS, s2, s2, Yp, (size_t)s2, 1, s2, nb, info.data());
      if (rc == 1 && f0 == 0) {
        *declined = true;
        return 1;
      }
      if (rc) return rc == 1 ? set_err(ctx, GPR_E_HIP, "batched cross-validation: shape declined") : rc;
      for (int i = 0; i < nb; ++i)
        if (info[i] > 0) return info[i];
      for (int i = 0; i < nb; ++i) {
        cv_loss_kernel<<<1, 256, 0, st>>>(Yt + (size_t)s2 * i, Yp + (size_t)s2 * i, Sb + szS * i,
                                          (size_t)s2, ntst, 0, dl + i);
        LAUNCH_CHECK(ctx);
      }
    }
    HIP_TRY(ctx, hipMemcpyAsync(hl.data(), dl, sizeof(double) * nb, hipMemcpyDeviceToHost, st));
    HIP_TRY(ctx, hipStreamSynchronize(st));
    for (int i = 0; i < nb; ++i) lss[(size_t)f0 + i] = hl[i];
  }
  return 0;
}

int gpr_cv_batch(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                 const double* dX, int n, const double* dy, const int* trn, int ntrn,
                 const int* tst, int ntst, int nfold, int cost, double eps, double* lss) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || ntrn <= 0 || ntst <= 0 || nfold <= 0 || !dX || !dy || !trn || !tst || !lss)
    return set_err(ctx, GPR_E_ARG, "bad args");
  if (cost != GPR_COST_MSE && cost != GPR_COST_CHISQ && cost != GPR_COST_MAHALANOBIS)
    return set_err(ctx, GPR_E_ARG, "unknown cost");
  for (size_t f = 0; f < (size_t)nfold; ++f) {
    for (int j = 0; j < ntrn; ++j)
      if (trn[f * ntrn + j] < 0 || trn[f * ntrn + j] >= n)
        return set_err(ctx, GPR_E_ARG, "training index out of range");
    for (int j = 0; j < ntst; ++j)
      if (tst[f * ntst + j] < 0 || tst[f * ntst + j] >= n)
        return set_err(ctx, GPR_E_ARG, "test index out of range");
  }
  // Every fold's factorisation in one batched tile-DAG launch (default; GPR_CV_BATCH=0: the
  // per-fold path below, folds spread over child contexts -- 1.1-2.7x slower, tools/bench_cv.py;
  // also taken when the batched launch declines the shape)
  if (ctx->cv_batch) {
    bool declined = false;
    const int rc = cv_folds_batched(ctx, kp, d, dX, n, dy, trn, ntrn, tst, ntst, nfold, cost, lss,
                                    &declined);
    release_big_scratch(ctx);
    if (!declined) return rc;
    ctx->err.clear();
  }
  // A fold below ~8k training points is a latency-bound chain of small launches (diag
  // block, panel GEMM, update per 128 columns) that leaves most CUs idle, so independent
  // folds run concurrently, one child context (own streams, own workspace) per host thread.
  int nsub = std::min(std::min(ctx->cv_streams, (int)gpr_ctx::CV_MAX_SUB), nfold);
  if (ntrn > 8192) nsub = 1;
  {  // per-child workspace of cv_folds: K, Sigma_p, inputs/outputs and indices of its folds
    const size_t per = ((size_t)ntrn * ntrn + (size_t)ntst * ntst +
                        (size_t)(d + 1) * (ntrn + ntst) + 2 * (size_t)ntst +
                        (size_t)((nfold + nsub - 1) / std::max(nsub, 1)) * (ntrn + ntst + 1)) * 8;
    nsub = cap_children_by_memory(nsub, per);
  }
  if (nsub <= 1)
    return cv_folds(ctx, kinds, nk, hp, d, dX, n, dy, trn, ntrn, tst, ntst, nfold, 0, 1, cost,
                    eps, lss);
  GPR_TRY(ensure_children(ctx, nsub));
  return run_children(ctx, nsub, [&](gpr_ctx* c, int t) {
    return cv_folds(c, kinds, nk, hp, d, dX, n, dy, trn, ntrn, tst, ntst, nfold, t, nsub, cost,
                    eps, lss);
  });
}

// Columns j0, j0 + jstep, ... of gpr_integrate_noise on context c: (K + noise_j I) = U_j^T U_j,
// wt_j = (K + noise_j I)^{-1} y_j, Iout_j = wt_j' k1, var_j = k2 - ||U_j^{-T} k1||^2.
static int integ_noise_cols(gpr_ctx* c, const double* K, int ldk, int n, const double* dy,
                            int ldy, const double* k1, double k2, const double* noise, int ny,
                            int j0, int jstep, double* Iout, double* var) {
  const int nmine = (ny - j0 + jstep - 1) / jstep;
  GPR_TRY(ensure_buf(c, &c->dbig, &c->big_cap, (size_t)n * n + 2 * (size_t)n + 2 * nmine));
  double* Kj = c->dbig;
  double* w = Kj + (size_t)n * n;
  double* t = w + n;
  double* out = t + n;  // [Iout_i, var_i] per owned column
  const int blocks = (int)std::min<size_t>(((size_t)n * n + 255) / 256, 4096);
  for (int i = 0; i < nmine; ++i) {
    const int j = j0 + i * jstep;
    shift_upper_kernel<<<blocks, 256, 0, c->stream>>>(K, (size_t)ldk, n, noise[j], Kj);
    LAUNCH_CHECK(c);
    int hinfo = 0;
    GPR_TRY(potrf_core(c, Kj, n, n, &hinfo));
    if (hinfo != 0) return hinfo;
    HIP_TRY(c, hipMemcpyAsync(w, dy + (size_t)j * ldy, sizeof(double) * n,
                              hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(t, k1, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
    GPR_TRY(potrs_core(c, Kj, n, n, w, 1, n));
    colgemv_kernel<<<1, 256, 0, c->stream>>>(w, (size_t)n, n, 1, k1, (size_t)n, 1, out + 2 * i, 1);
    LAUNCH_CHECK(c);
    GPR_TRY(potrs_core(c, Kj, n, n, t, 1, n, /*forward=*/true, /*backward=*/false));
    GPR_TRY(launch_fill(c, out + 2 * i + 1, 1, k2));
    GPR_TRY(launch_colnorm_sub(c, t, n, n, 1, out + 2 * i + 1));
  }
  std::vector<double> h(2 * (size_t)nmine);
  HIP_TRY(c, hipMemcpyAsync(h.data(), out, sizeof(double) * 2 * nmine, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < nmine; ++i) {
    Iout[j0 + i * jstep] = h[2 * i];
    var[j0 + i * jstep] = h[2 * i + 1];
  }
  return 0;
}

// Batched form of the per-column path: matrices K + noise_b I for a chunk of columns, each
// padded to n2 = n rounded up to 16 with the identity ([[K + s I, 0], [0, I]] has the factor
// [[U, 0], [0, I]]), only the upper triangle written (the tile-DAG reads nothing else), and
// right-hand sides [y_b | k1] (zero-padded) -- one batched tile-DAG launch factors all of them
// and solves V_b = U_b^{-T} [y_b | k1]; then Iout_b = V_b[:,1] . V_b[:,0] (= k1' (K + s I)^{-1}
// y_b) and var_b = k2 - ||V_b[:,1]||^2.
__global__ void quad_batch_prep_kernel(const double* __restrict__ K, int n, int n2,
                                       const double* __restrict__ noise, const double* __restrict__ dy,
                                       int ldy, const double* __restrict__ k1, double* __restrict__ W,
                                       double* __restrict__ Bm, int nb) {
  const size_t per = (size_t)n2 * n2, tot = per * nb;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += stride) {
    const int b = (int)(e / per);
    const size_t rem = e - (size_t)b * per;
    const int r = (int)(rem % n2), c = (int)(rem / n2);
    if (r > c) continue;  // (the strict lower triangle is never read)
    W[e] = (c < n) ? K[(size_t)r + (size_t)c * n] + (r == c ? noise[b] : 0.0) : (r == c ? 1.0 : 0.0);
  }
  const size_t totb = (size_t)2 * n2 * nb;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < totb; e += stride) {
    const int b = (int)(e / (2 * (size_t)n2));
    const size_t rem = e - (size_t)b * 2 * n2;
    const int r = (int)(rem % n2), c = (int)(rem / n2);
    Bm[e] = r < n ? (c == 0 ? dy[(size_t)b * ldy + r] : k1[r]) : 0.0;
  }
}

__global__ void quad_batch_reduce_kernel(const double* __restrict__ Bm, int n2, double k2,
                                         double* __restrict__ out) {
  const double* V = Bm + (size_t)blockIdx.x * 2 * n2;
  double sv = 0.0, sk = 0.0;
  for (int i = threadIdx.x; i < n2; i += 256) {
    const double a = V[i], c = V[n2 + i];
    sv = fma(a, c, sv);
    sk = fma(c, c, sk);
  }
  __shared__ double red[2][256];
  red[0][threadIdx.x] = sv;
  red[1][threadIdx.x] = sk;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = red[0][0];
    out[2 * blockIdx.x + 1] = k2 - red[1][0];
  }
}

// Returns 0 (done), > 0 the first failing column's info (K + noise_j I not positive
// definite), 1 with *declined set when the batched launch cannot take the shape.
static int integ_noise_batched(gpr_ctx* ctx, const double* K, int n, const double* dy, int ldy,
                               const double* k1, double k2, const double* noise, int ny,
                               double* Iout, double* var, bool* declined) {
  *declined = false;
  const int n2 = (n + 15) / 16 * 16;
  const size_t per = (size_t)n2 * n2 + 2 * (size_t)n2;
  int nbc = batch_capacity(ctx->quad_batch_gb, per + 3, 16, ctx->big_cap, ny);
  GPR_TRY(ensure_batch_buf(ctx, &nbc, [&](int k) { return per * k + (size_t)3 * k + 16; }));
  double* W = ctx->dbig;
  double* Bm = W + (size_t)n2 * n2 * nbc;
  double* dnoise = Bm + (size_t)2 * n2 * nbc;
  double* out = dnoise + nbc;
  std::vector<int> info(nbc);
  std::vector<double> h(2 * (size_t)nbc);
  for (int j0 = 0; j0 < ny; j0 += nbc) {
    const int nb = std::min(nbc, ny - j0);
    HIP_TRY(ctx, hipMemcpyAsync(dnoise, noise + j0, sizeof(double) * nb, hipMemcpyHostToDevice,
                                ctx->stream));
    const size_t tot = (size_t)n2 * n2 * nb;
    const int blocks = (int)std::min<size_t>((tot + 255) / 256, 8192);
    quad_batch_prep_kernel<<<blocks, 256, 0, ctx->stream>>>(K, n, n2, dnoise, dy + (size_t)j0 * ldy,
                                                            ldy, k1, W, Bm, nb);
    LAUNCH_CHECK(ctx);
    const int rc = launch_potrf_dag_batch(ctx, W, (size_t)n2 * n2, n2, n2, Bm, (size_t)2 * n2, 2, n2,
                                          nb, info.data());
    if (rc == 1) {
      *declined = true;
      return 1;
    }
    if (rc) return rc;
    for (int b = 0; b < nb; ++b)
      if (info[b] > 0) return info[b];
    quad_batch_reduce_kernel<<<nb, 256, 0, ctx->stream>>>(Bm, n2, k2, out);
    LAUNCH_CHECK(ctx);
    HIP_TRY(ctx, hipMemcpyAsync(h.data(), out, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (int b = 0; b < nb; ++b) {
      Iout[j0 + b] = h[2 * b];
      var[j0 + b] = h[2 * b + 1];
    }
  }
  return 0;
}

#ifdef GPR_TESTING
// ---- rocSOLVER, dlopen'd (the process's own librocsolver.so.0 if loaded -- torch carries
// one -- else the system's; no link-time dependency), for the eigendecomposition of K
struct RocsolverApi {
  bool tried = false, ok = false;
  decltype(&rocblas_create_handle) create = nullptr;
  decltype(&rocblas_destroy_handle) destroy = nullptr;
  decltype(&rocblas_set_stream) set_stream = nullptr;
  decltype(&rocsolver_dsyevd) dsyevd = nullptr;
};
static RocsolverApi g_rs;
static std::mutex g_rs_mu;

static bool load_rocsolver() {
  std::lock_guard<std::mutex> lk(g_rs_mu);
  if (g_rs.tried) return g_rs.ok;
  g_rs.tried = true;
  void* h = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return false;
  // (dlsym on the rocSOLVER handle also searches its dependency, the rocBLAS it was built on)
  g_rs.create = (decltype(g_rs.create))dlsym(h, "rocblas_create_handle");
  g_rs.destroy = (decltype(g_rs.destroy))dlsym(h, "rocblas_destroy_handle");
  g_rs.set_stream = (decltype(g_rs.set_stream))dlsym(h, "rocblas_set_stream");
  g_rs.dsyevd = (decltype(g_rs.dsyevd))dlsym(h, "rocsolver_dsyevd");
  g_rs.ok = g_rs.create && g_rs.destroy && g_rs.set_stream && g_rs.dsyevd;
  return g_rs.ok;
}

static int rb_destroy_fn(void* hdl) {
  return g_rs.destroy ? (int)g_rs.destroy((rocblas_handle)hdl) : 0;
}

#endif  // GPR_TESTING

// out[2j] = Iout_j = sum_i T[i, j] c_i / (lambda_i + noise_j), out[2j+1] = var_j = k2 - sum_i
// c_i^2 / (lambda_i + noise_j), c = T[:, ny] = P^T k1  (src/integrate.jl:81-87,89-104,149-162:
// Iout_j = wt_j' k1 with wt_j = P (lambda + noise_j)^-1 P' y_j, the same sum reassociated)
__global__ __launch_bounds__(256) void quad_diag_update_kernel(const double* __restrict__ T, int n,
                                                               int ny, const double* __restrict__ lam,
                                                               const double* __restrict__ noise,
                                                               double k2, double* __restrict__ out) {
  __shared__ double red[2][256];
  const int j = blockIdx.x;
  const double* tj = T + (size_t)j * n;
  const double* c = T + (size_t)ny * n;
  const double e = noise[j];
  double si = 0.0, sv = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const double r = 1.0 / (lam[i] + e);
    si += tj[i] * c[i] * r;
    sv += c[i] * c[i] * r;
  }
  red[0][threadIdx.x] = si;
  red[1][threadIdx.x] = sv;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * j] = red[0][0];
    out[2 * j + 1] = k2 - red[1][0];
  }
}

// gpr_integrate_noise by one symmetric eigendecomposition of K (in place: K <- P), as the
// reference: T = P^T [Y | k1] on the MFMA GEMM, then one diagonal update per column.  Returns 1
// (nothing done) when rocSOLVER cannot be loaded.
static int integ_noise_eigen(gpr_ctx* ctx, double* K, const double* k1, double k2, int n,
                             const double* dy, int ny, int ldy, const double* noise, double* Iout,
                             double* var, int method) {
  const bool rocsolver = method == 2;
  if (method == 1 && sym_tridiag_ok(n)) {
    // K = Q T Q^T by the hand-written tridiagonal reduction (tridiag.hip; syevr's first
    // stage), C = Q^T [Y | k1], then per column one tridiagonal solve with (T + noise_j I):
    // Iout_j = C[:, j]' (T + s_j I)^{-1} C[:, ny] = k1' (K + s_j I)^{-1} y_j -- the reference's
    // sum_i (P'y_j)_i (P'k1)_i / (lambda_i + s_j) without the eigenvectors (any shift)
    const size_t nc = (size_t)n * (ny + 1);
    GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap,
                       nc + 2 * (size_t)n + 3 * (size_t)ny +
                           4 * (size_t)n * quad_tridiag_chunk(n, ny)));
    double* C = ctx->dbig;
    double* dd = C + nc;
    double* de = dd + n;
    double* dnoise = de + n;
    double* out = dnoise + ny;
    double* scr = out + 2 * (size_t)ny;
    HIP_TRY(ctx, hipMemcpy2DAsync(C, sizeof(double) * n, dy, sizeof(double) * ldy,
                                  sizeof(double) * n, ny, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(C + (size_t)ny * n, k1, sizeof(double) * n, hipMemcpyDeviceToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dnoise, noise, sizeof(double) * ny, hipMemcpyHostToDevice,
                                ctx->stream));
    const int rc = sym_tridiag(ctx, K, n, n, C, ny + 1, n, dd, de);
    if (rc == GPR_E_UNSUP) {  // refused before it ran (not co-resident): K intact, factor per column
      ctx->err.clear();
      return 1;
    }
    GPR_TRY(rc);
    GPR_TRY(quad_tridiag_solves(ctx, dd, de, n, C, n, ny, dnoise, k2, scr, out));
    std::vector<double> h(2 * (size_t)ny);
    HIP_TRY(ctx, hipMemcpyAsync(h.data(), out, sizeof(double) * 2 * ny, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (int j = 0; j < ny; ++j) {
      Iout[j] = h[2 * j];
      var[j] = h[2 * j + 1];
    }
    return 0;
  }
  if (!rocsolver) {
    // the full eigendecomposition, as the reference (method 3; method 1 beyond the reduction's
    // LDS bound): K = P Lambda P^T by the tridiagonal reduction + divide and conquer, or by block
    // Jacobi (method 4, or n beyond both), lambda and T = P^T [Y | k1] directly, P never formed;
    // then the reference's diagonal update per column
    const size_t nb = (size_t)n * (ny + 1);
    GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, nb + (size_t)n + 3 * (size_t)ny));
    double* T = ctx->dbig;
    double* lam = T + nb;
    double* dnoise = lam + n;
    double* out = dnoise + ny;
    HIP_TRY(ctx, hipMemcpy2DAsync(T, sizeof(double) * n, dy, sizeof(double) * ldy,
                                  sizeof(double) * n, ny, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(T + (size_t)ny * n, k1, sizeof(double) * n, hipMemcpyDeviceToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dnoise, noise, sizeof(double) * ny, hipMemcpyHostToDevice,
                                ctx->stream));
    // relative accuracy for K + s_min I (s_min = the smallest shift when none is negative)
    double smin = noise[0];
    for (int j = 1; j < ny; ++j) smin = std::min(smin, noise[j]);
    GPR_TRY(sym_eig_apply(ctx, K, n, n, T, ny + 1, n, lam, nullptr, std::max(smin, 0.0),
                          method == 4 ? 2 : 0));
    quad_diag_update_kernel<<<ny, 256, 0, ctx->stream>>>(T, n, ny, lam, dnoise, k2, out);
    LAUNCH_CHECK(ctx);
    std::vector<double> h(2 * (size_t)ny);
    HIP_TRY(ctx, hipMemcpyAsync(h.data(), out, sizeof(double) * 2 * ny, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (int j = 0; j < ny; ++j) {
      Iout[j] = h[2 * j];
      var[j] = h[2 * j + 1];
    }
    return 0;
  }
  // GPR_QUAD_EIGEN=2: rocSOLVER dsyevd (a timing comparator for the hand-written solver,
  // compiled into the test build libgpr_hip_testing.so only)
#ifndef GPR_TESTING
  return set_err(ctx, GPR_E_ARG, "quadrature eigen route 2 (rocSOLVER comparator) exists only "
                 "in the test build");
#else
  if (!load_rocsolver()) return 1;
  if (!ctx->rb_handle) {
    rocblas_handle hb = nullptr;
    if (g_rs.create(&hb) != rocblas_status_success)
      return set_err(ctx, GPR_E_HIP, "rocblas_create_handle failed");
    ctx->rb_handle = hb;
    ctx->rb_destroy = rb_destroy_fn;
  }
  rocblas_handle hb = (rocblas_handle)ctx->rb_handle;
  if (g_rs.set_stream(hb, ctx->stream) != rocblas_status_success)
    return set_err(ctx, GPR_E_HIP, "rocblas_set_stream failed");
  // workspace (dbig): B = [Y | k1] (n x (ny+1)), T (n x (ny+1)), lambda, E, noise, out, info
  const size_t nb = (size_t)n * (ny + 1);
  GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, 2 * nb + 2 * (size_t)n + 3 * (size_t)ny + 1));
  double* B = ctx->dbig;
  double* T = B + nb;
  double* lam = T + nb;
  double* E = lam + n;
  double* dnoise = E + n;
  double* out = dnoise + ny;
  int* dinfo = reinterpret_cast<int*>(out + 2 * (size_t)ny);
  HIP_TRY(ctx, hipMemcpy2DAsync(B, sizeof(double) * n, dy, sizeof(double) * ldy,
                                sizeof(double) * n, ny, hipMemcpyDeviceToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(B + (size_t)ny * n, k1, sizeof(double) * n, hipMemcpyDeviceToDevice,
                              ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(dnoise, noise, sizeof(double) * ny, hipMemcpyHostToDevice,
                              ctx->stream));
  // LAPACK.syevr!(ws, 'V', 'A', 'U', kxx, ...) -> eigenvalues ascending, eigenvectors in K.
  // A call the library refuses (e.g. a rocSOLVER without code for this device) leaves K
  // untouched: the caller then factors per column instead
  if (g_rs.dsyevd(hb, rocblas_evect_original, rocblas_fill_upper, n, K, n, lam, E, dinfo) !=
      rocblas_status_success) {
    (void)hipGetLastError();
    return 1;
  }
  int hinfo = 0;
  HIP_TRY(ctx, hipMemcpyAsync(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  // T = P^T B
  GemmArgs g{};
  g.P = K; g.ldp = n;
  g.Q = B; g.ldq = n;
  g.C = T; g.ldc = n;
  g.M = n; g.N = ny + 1; g.K = n;
  g.alpha = 1.0; g.beta = 0.0;
  GPR_TRY(launch_gemm_tn(ctx, g, TC_OTHER));
  quad_diag_update_kernel<<<ny, 256, 0, ctx->stream>>>(T, n, ny, lam, dnoise, k2, out);
  LAUNCH_CHECK(ctx);
  std::vector<double> h(2 * (size_t)ny);
  HIP_TRY(ctx, hipMemcpyAsync(h.data(), out, sizeof(double) * 2 * ny, hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (hinfo != 0)
    return set_err(ctx, GPR_E_HIP, "rocsolver_dsyevd did not converge (info %d)", hinfo);
  for (int j = 0; j < ny; ++j) {
    Iout[j] = h[2 * j];
    var[j] = h[2 * j + 1];
  }
  return 0;
#endif  // GPR_TESTING
}

int gpr_integrate_noise(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                        const double* dX, int n, const double* dy, int ny, int ldy,
                        const double* a, const double* b, const double* noise, double eps,
                        double* Iout, double* var) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (n <= 0 || ny <= 0 || ldy < n || !dX || !dy || !a || !b || !noise || !Iout || !var)
    return set_err(ctx, GPR_E_ARG, "bad args");
  // kernel!(wc.kxx, ...) once (src/integrate.jl:72), k1 / k2 once (:106-110)
  // (in dbig2: the per-column worker factors K + noise_j I in its context's dbig)
  GPR_TRY(ensure_buf(ctx, &ctx->dbig2, &ctx->big2_cap, (size_t)n * n + n));
  double* K = ctx->dbig2;
  double* k1 = K + (size_t)n * n;
  GPR_TRY(launch_kernel_matrix(ctx, kp, dX, n, nullptr, n, 1, K, n));
  double k2 = 0.0;
  GPR_TRY(gpr_antideriv_se(ctx, d, hp, dX, n, a, b, k1, &k2));
  // The reference's path is K = P diag(lambda) P^T once (LAPACK.syevr!, :75), then per column
  // j only diagonal updates (inverse_diagonal_update!, :81-104).  GPR_QUAD_EIGEN picks:
  //   1  the tridiagonal reduction K = Q T Q^T (syevr's first stage, tridiag.hip) and one
  //      pivoted tridiagonal solve per column: k1' (K + s I)^{-1} y = (Q^T k1)' (T + s I)^{-1}
  //      (Q^T y) -- the same function of the same reduction, without the eigenvectors;
  //   3  the full decomposition, as the reference: the reduction + divide and conquer on T
  //      (dstedc.hip), then the diagonal updates; 4 the same by block Jacobi (eigen.hip);
  //   0  K + noise_j I factored per column (batched tile-DAG launch; positive definite shifts
  //      only, PosDefException otherwise); 2 rocSOLVER dsyevd (timing comparator).
  // Unset (-1): per-column factorisations while they cost less than the reduction, else 1 --
  // the crossover from the measured costs (profiles/r05_eig_speed_full.txt: batched ~0.5 + ny (4.3e-12
  // n^3 + 1.4e-8 n^2) ms; reduction + solves ~0.00537 n + 9.3e-10 n^3 + ny 2e-9 n^2 ms below n =
  // 5376 (profiles/r06_trd_probe_lds_wg.txt: 19.0 / 86.0 / 150 ms at 2048 / 4096 / 5120): ny ~ 175
  // at n = 4096, ~220 at 2048, ~330 at 1100, ~700 at 512; from n = 5376 on the reduction's
  // deferred-update variant, 3.2e-6 n^2 + 4.6e-10 n^3 -- profiles/r06_trd_probe_df.txt: 467 ms at
  // n = 8192, 1336 at 12288, 228 at 6144, against the batch's 3.3 / 10 ms per column at 8192 /
  // 12288: ny ~ 140); a batch that meets a K + s I that is not
  // positive definite (a shift at or below -lambda_min(K)) falls back to route 1.  Beyond the
  // reduction's bound (n > 16384) the factorisations, whatever ny.
  int qmode = ctx->quad_eigen;
  bool fallback = false;
  if (qmode < 0) {
    const double dn = n, t_fac = 0.5 + ny * (4.26e-12 * dn * dn * dn + 1.37e-8 * dn * dn);
    const double t_red = n >= 5376 ? 3.2e-6 * dn * dn + 4.6e-10 * dn * dn * dn
                                   : 0.00537 * dn + 9.3e-10 * dn * dn * dn;
    const double t_trd = t_red + ny * 2e-9 * dn * dn;
    qmode = (sym_tridiag_ok(n) && t_trd < t_fac) ? 1 : 0;
    fallback = qmode == 0;
  }
  if (qmode != 0) {
    const int rc = integ_noise_eigen(ctx, K, k1, k2, n, dy, ny, ldy, noise, Iout, var, qmode);
    if (rc != 1) return rc;  // (1: the reduction refused (not co-resident) or rocSOLVER unavailable; K intact)
  }
  if (!ctx->quad_seq) {  // the batched launch (GPR_QUAD_SEQ: one column at a time)
    bool declined = false;
    const int rc = integ_noise_batched(ctx, K, n, dy, ldy, k1, k2, noise, ny, Iout, var, &declined);
    release_big_scratch(ctx);
    if (!declined) {
      if (rc > 0 && fallback) {  // K + s I not numerically positive definite: the eigensolver
        ctx->err.clear();
        return integ_noise_eigen(ctx, K, k1, k2, n, dy, ny, ldy, noise, Iout, var, 1);
      }
      return rc;
    }
    ctx->err.clear();
  }
  int nsub = std::min(std::min(ctx->cv_streams, (int)gpr_ctx::CV_MAX_SUB), ny);
  if (n > 8192) nsub = 1;
  nsub = cap_children_by_memory(nsub, ((size_t)n * n + 2 * (size_t)n + 2 * (size_t)ny) * 8);
  int rc;
  if (nsub <= 1) {
    rc = integ_noise_cols(ctx, K, n, n, dy, ldy, k1, k2, noise, ny, 0, 1, Iout, var);
  } else {
    GPR_TRY(ensure_children(ctx, nsub));
    rc = run_children(ctx, nsub, [&](gpr_ctx* c, int t) {
      return integ_noise_cols(c, K, n, n, dy, ldy, k1, k2, noise, ny, t, nsub, Iout, var);
    });
  }
  if (rc > 0 && fallback) {  // K + s I not numerically positive definite: the eigensolver
    ctx->err.clear();
    return integ_noise_eigen(ctx, K, k1, k2, n, dy, ny, ldy, noise, Iout, var, 1);
  }
  return rc;
}

int gpr_split_factors(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                      const double* dX, int ns, const double* dXe, int ne, const double* dXq,
                      int nq, int part, double* dA, double* dB, double* dC) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, 0.0, &kp, nullptr));
  if (part < 0 || part >= kp.nse) return set_err(ctx, GPR_E_ARG, "part out of range");
  const size_t need = (size_t)kp.nse * d * (ns + ne + nq);
  GPR_TRY(ensure_buf(ctx, &ctx->dxs, &ctx->xs_cap, need));
  double* xs = ctx->dxs;
  double* xes = xs + (size_t)kp.nse * d * ns;
  double* xqs = xes + (size_t)kp.nse * d * ne;
  GPR_TRY(launch_scale_inputs(ctx, kp, dX, ns, xs));
  GPR_TRY(launch_scale_inputs(ctx, kp, dXe, ne, xes));
  GPR_TRY(launch_scale_inputs(ctx, kp, dXq, nq, xqs));
  const int p = part;
  const double s2 = kp.sigma[p] * kp.sigma[p];
  if (dA) GPR_TRY(launch_pair(ctx, 1, d, xes + (size_t)p * d * ne, ne, xqs + (size_t)p * d * nq, nq, 1.0, dA, 1, ne));
  if (dB) GPR_TRY(launch_pair(ctx, 0, d, xes + (size_t)p * d * ne, ne, xs + (size_t)p * d * ns, ns, 1.0, dB, 1, ne));
  if (dC) GPR_TRY(launch_pair(ctx, 2, d, xs + (size_t)p * d * ns, ns, xqs + (size_t)p * d * nq, nq, s2, dC, 1, ns));
  return 0;
}

}  // extern "C"

// Split prediction of several contiguous pieces of grid rows in one call (a rank's shard,
// multi-GPU; gpr_split_predict is the one-piece case).  Factors (src/split_kernel.jl:151-159)
// per SE part p: C_p (ns x nq, sigma^2, SplitDistanceC) built ONCE per call; A_p (E x nq,
// sigma = 1, SplitDistanceA) and B_p^T (ns x E, sigma = 1, Euclidean) per piece of E rows.
// Layout in ctx->dbig2: [C_0..C_{nse-1} | A_0.. | BT_0..] with the A/BT slots sized to the
// largest piece.
struct SplitFactors {
  double *A, *BT, *C;
  double *xs, *xes, *xqs;  // scaled inputs per part: (nse, ns, d), (nse, ne, d), (nse, nq, d)
};

static int split_prepare(gpr_ctx* ctx, const KParams& kp, int d, const double* dX, int ns,
                         const double* dXe, int ne, const double* dXq, int nq, int Emax,
                         SplitFactors* f) {
  const int nse = kp.nse;
  const size_t szC = (size_t)ns * nq;
  GPR_TRY(ensure_buf(ctx, &ctx->dbig2, &ctx->big2_cap,
                     (size_t)nse * (szC + (size_t)Emax * nq + (size_t)ns * Emax)));
  f->C = ctx->dbig2;
  f->A = f->C + nse * szC;
  f->BT = f->A + (size_t)nse * Emax * nq;
  GPR_TRY(ensure_buf(ctx, &ctx->dxs, &ctx->xs_cap, (size_t)nse * d * (ns + ne + nq)));
  f->xs = ctx->dxs;
  f->xes = f->xs + (size_t)nse * d * ns;
  f->xqs = f->xes + (size_t)nse * d * ne;
  TimerScope ts(ctx, TC_OTHER, 0.0);
  GPR_TRY(launch_scale_inputs(ctx, kp, dX, ns, f->xs));
  GPR_TRY(launch_scale_inputs(ctx, kp, dXe, ne, f->xes));
  GPR_TRY(launch_scale_inputs(ctx, kp, dXq, nq, f->xqs));
  for (int p = 0; p < nse; ++p)  // C: sigma, SplitDistanceC(x, xq)
    GPR_TRY(launch_pair(ctx, 2, d, f->xs + (size_t)p * d * ns, ns, f->xqs + (size_t)p * d * nq, nq,
                        kp.sigma[p] * kp.sigma[p], f->C + p * szC, 1, ns));
  return 0;
}

// A and B^T of grid rows [e_lo, e_lo + E)
static int split_piece_factors(gpr_ctx* ctx, const KParams& kp, int d, int ns, int ne, int nq,
                               int e_lo, int E, const SplitFactors& f) {
  TimerScope ts(ctx, TC_OTHER, 0.0);
  const size_t szA = (size_t)E * nq, szB = (size_t)ns * E;
  for (int p = 0; p < kp.nse; ++p) {
    const double* xe = f.xes + ((size_t)p * ne + e_lo) * d;
    GPR_TRY(launch_pair(ctx, 1, d, xe, E, f.xqs + (size_t)p * d * nq, nq, 1.0, f.A + p * szA, 1, E));
    GPR_TRY(launch_pair(ctx, 0, d, xe, E, f.xs + (size_t)p * d * ns, ns, 1.0, f.BT + p * szB, ns, 1));
  }
  return 0;
}

// mu[e, q] = sum_p A_p[e,q] * (B_p diag(wt) C_p)[e,q] for rows [e_lo, e_lo + E)
// (src/split_predict.jl:10-19)
// (dmu: output row of e_lo, leading dimension ldmu)
static int split_mean(gpr_ctx* ctx, int nse, const double* A, const double* BT, const double* C,
                      int ns, int E, int nq, const double* dwt, double* dmu, int ldmu) {
  const size_t szA = (size_t)E * nq, szB = (size_t)ns * E, szC = (size_t)ns * nq;
  for (int p = 0; p < nse; ++p) {
    GemmArgs g{};
    g.P = BT + p * szB; g.ldp = ns;
    g.Q = C + p * szC; g.ldq = ns;
    g.qscale = dwt;
    g.E = A + p * szA; g.lde = E;
    g.C = dmu; g.ldc = ldmu;
    g.M = E; g.N = nq; g.K = ns;
    g.alpha = 1.0; g.beta = (p == 0) ? 0.0 : 1.0;
    GPR_TRY(launch_gemm_tn(ctx, g, TC_OTHER));
  }
  return 0;
}

// Kxq columns of grid rows [e, e + nr) (row e - e_lo of the factors), column (e' - e) nq + q
static int split_kxq(gpr_ctx* ctx, int nse, const double* A, const double* BT, const double* C,
                     int ns, int nq, int E, int erow, int nr, double* out) {
  TimerScope ts(ctx, TC_OTHER, 0.0);
  const size_t total = (size_t)ns * nq * nr;
  int blocks = (int)std::min<size_t>((total + 255) / 256, 65536);
  split_kxq_kernel<<<blocks, 256, 0, ctx->stream>>>(nse, A, BT, C, ns, nq, E, erow, nr, out);
  LAUNCH_CHECK(ctx);
  return 0;
}

// Output rows: full grid layout (compact = false: row e at e, dmu leading dim ldmu = ne) or
// the shard's rows only (compact: the pieces' rows concatenated in order, row e of piece k at
// off_k + e - lo_k; dmu R x nq with leading dim ldmu >= R, dvar R nq).
int split_predict_pieces(gpr_ctx* ctx, const int* kinds, int nk, const double* hp, int d,
                         const double* dX, int ns, const double* dU, int ldu, const double* dwt,
                         const double* dXe, int ne, const double* dXq, int nq, const int* pieces,
                         int npieces, int var_lo, int var_hi, double eps, double* dmu, int ldmu,
                         double* dvar, bool compact) {
  KParams kp;
  GPR_TRY(make_kparams(ctx, kinds, nk, hp, d, eps, &kp, nullptr));
  if (ns <= 0 || ne <= 0 || nq <= 0 || ldu < ns || !dX || !dU || !dwt || !dXe || !dXq || !dmu ||
      !dvar || npieces < 0 || (npieces && !pieces))
    return set_err(ctx, GPR_E_ARG, "bad args");
  int Emax = 0, R = 0;
  for (int k = 0; k < npieces; ++k) {
    const int lo = pieces[2 * k], hi = pieces[2 * k + 1];
    if (lo < 0 || hi > ne || lo > hi) return set_err(ctx, GPR_E_ARG, "bad e range [%d,%d)", lo, hi);
    if (k && lo < pieces[2 * k - 1])
      return set_err(ctx, GPR_E_ARG, "pieces must be sorted and disjoint");
    Emax = std::max(Emax, hi - lo);
    R += hi - lo;
  }
  if (ldmu < (compact ? std::max(R, 1) : ne))
    return set_err(ctx, GPR_E_ARG, "ldmu %d < %d", ldmu, compact ? R : ne);
  if (Emax == 0) return 0;
  const int nse = kp.nse;
  SplitFactors f;
  GPR_TRY(split_prepare(ctx, kp, d, dX, ns, dXe, ne, dXq, nq, Emax, &f));
  const double prior = diag_prior(kinds, nk, hp, d);
  const size_t per_row = (size_t)ns * nq;
  for (int k = 0, off = 0; k < npieces; off += pieces[2 * k + 1] - pieces[2 * k], ++k) {
    const int e_lo = pieces[2 * k], e_hi = pieces[2 * k + 1], E = e_hi - e_lo;
    if (E == 0) continue;
    const int o = compact ? off : e_lo;  // output row of grid row e_lo
    GPR_TRY(split_piece_factors(ctx, kp, d, ns, ne, nq, e_lo, E, f));
    GPR_TRY(split_mean(ctx, nse, f.A, f.BT, f.C, ns, E, nq, dwt, dmu + o, ldmu));
    // ---- variance: prior everywhere in range, then rows e in [var_lo, var_hi) updated
    GPR_TRY(launch_fill(ctx, dvar + (size_t)o * nq, (size_t)E * nq, prior));
    const int v0 = std::max(var_lo, e_lo), v1 = std::min(var_hi, e_hi);
    if (v1 > v0) {
      // <= 8 GiB of right-hand sides per batch (C5: 32 rows of ns = 32768, nq = 1024 in one
      // U^{-T} solve of 32768 columns instead of four of 8192)
      int Eb = (int)std::max<size_t>(1, ((size_t)1 << 30) / per_row);
      Eb = std::min(Eb, v1 - v0);
      GPR_TRY(ensure_buf(ctx, &ctx->dbig, &ctx->big_cap, per_row * Eb));
      for (int e = v0; e < v1; e += Eb) {
        const int nr = std::min(Eb, v1 - e);
        GPR_TRY(split_kxq(ctx, nse, f.A, f.BT, f.C, ns, nq, E, e - e_lo, nr, ctx->dbig));
        GPR_TRY(trsm_ut_core(ctx, dU, ns, ldu, ctx->dbig, nr * nq, ns,
                             dvar + (size_t)(o + e - e_lo) * nq, 0));
      }
    }
  }
  return 0;
}

extern "C" {

int gpr_split_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                      const double* dX, int ns, const double* dU, int ldu, const double* dwt,
                      const double* dXe, int ne, const double* dXq, int nq, int e_lo, int e_hi,
                      int var_lo, int var_hi, double eps, double* dmu, double* dvar) {
  if (e_lo < 0 || e_hi > ne || e_lo > e_hi) return set_err(ctx, GPR_E_ARG, "bad e range [%d,%d)", e_lo, e_hi);
  const int piece[2] = {e_lo, e_hi};
  return split_predict_pieces(ctx, kinds, nk, hp, d, dX, ns, dU, ldu, dwt, dXe, ne, dXq, nq, piece,
                              1, var_lo, var_hi, eps, dmu, ne, dvar, false);
}

int gpr_split_predict_rows(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                           const double* dX, int ns, const double* dU, int ldu, const double* dwt,
                           const double* dXe, int ne, const double* dXq, int nq, const int* pieces,
                           int npieces, int var_lo, int var_hi, double eps, double* dmu,
                           double* dvar) {
  return split_predict_pieces(ctx, kinds, nk, hp, d, dX, ns, dU, ldu, dwt, dXe, ne, dXq, nq, pieces,
                              npieces, var_lo, var_hi, eps, dmu, ne, dvar, false);
}

int gpr_split_predict_shard(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                            const double* dX, int ns, const double* dU, int ldu,
                            const double* dwt, const double* dXe, int ne, const double* dXq,
                            int nq, const int* pieces, int npieces, int var_lo, int var_hi,
                            double eps, double* dmu, int ldmu, double* dvar) {
  return split_predict_pieces(ctx, kinds, nk, hp, d, dX, ns, dU, ldu, dwt, dXe, ne, dXq, nq, pieces,
                              npieces, var_lo, var_hi, eps, dmu, ldmu, dvar, true);
}

}  // extern "C"
