/*
 * gpr_hip.h -- C ABI of libgpr_hip.so, the MI355X (gfx950) exact-GP engine.
 *
 * Drop-in boundary for the dense hot path of GaussianProcessRegression.jl
 * (reference snapshot 2025-03-21).  The reference has no FFI of its own: its extension
 * seams are Julia multiple dispatch on the output-array type (kernel!(::AbstractGPUArray)
 * src/covar_gpu.jl:1) and on the cache type (update_cache!/loss/grad!/predict!,
 * src/cost.jl:40-126, src/predict.jl:29-101, src/split_predict.jl:5-53).  Each entry point
 * below names the reference function it replaces; INTEGRATION.md shows the Julia
 * `ccall` methods a maintainer adds on those seams.
 *
 * Conventions (all of them Julia's, so a Julia caller passes its arrays unchanged):
 *   - fp64 everywhere; matrices are COLUMN-MAJOR with an explicit leading dimension.
 *   - x is d x n column-major (each sample's d features contiguous), like md.x.
 *   - A kernel is described by `kinds[nk]` (GPR_SE / GPR_WN, in `+` order) and the flat
 *     hyper-parameter vector `hp` (HOST pointer) of length sum(dim_hp) -- SE: d+1
 *     ([sigma, l_1..l_d]), WN: 1 ([sigma_n]) -- exactly split(hp, dims)
 *     (src/compose_covar.jl:21-28).
 *   - Pointers named d* are DEVICE pointers (from gpr_malloc, hipMalloc, or a torch
 *     tensor); all other pointers are host pointers.  No pointer is retained after a call
 *     returns.
 *   - Every op is enqueued on the context's stream.  Ops that return host scalars/vectors
 *     (info, mll, grad) synchronise the stream before returning; the others are async.
 *   - A context is not thread-safe: one context (one stream) per host thread.
 *
 * Return codes: 0 ok; >0 LAPACK-style info (gpr_potrf_upper: order of the leading minor
 * that is not positive definite, like dpotrf / Julia's PosDefException(info));
 * <0 errors (GPR_E_*), with a message from gpr_last_error(ctx).
 */
#ifndef GPR_HIP_H
#define GPR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPR_SE 1 /* SquaredExp  src/covariance.jl:15 */
#define GPR_WN 2 /* WhiteNoise  src/covariance.jl:17 */

#define GPR_OK 0
#define GPR_E_ARG (-1)      /* bad argument (message names it)                      */
#define GPR_E_HIP (-2)      /* HIP runtime error                                    */
#define GPR_E_NOMEM (-3)    /* device allocation failed                             */
#define GPR_E_UNSUP (-4)    /* unsupported configuration (e.g. d > GPR_MAX_DIM)      */

#define GPR_MAX_DIM 64      /* max input dimension d                               */
#define GPR_MAX_PARTS 8     /* max kernel parts in a composed kernel                */

/* predict modes (src/predict.jl:14-25) */
#define GPR_PREDICT_MEAN 0  /* predict_mean  src/predict.jl:6-12                     */
#define GPR_PREDICT_DIAG 1  /* predict(...; diagonal_var=true)                       */
#define GPR_PREDICT_FULL 2  /* predict(...; diagonal_var=false)                      */

/* cross-validation losses (src/loss_grad.jl:12-30) */
#define GPR_COST_MSE 1         /* MSE:  sum((y - yp)^2) / length(y)                   */
#define GPR_COST_CHISQ 2       /* ChiSq: sum((y - yp)^2 / Sigma_p[i, i])              */
#define GPR_COST_MAHALANOBIS 3 /* Mahalanobis: ||L^{-1}(y - yp)||^2, Sigma_p = L L^T   */

typedef struct gpr_ctx* gpr_ctx_t;

/* ---- context & memory ------------------------------------------------------------- */
/* stream: a hipStream_t to run on (NULL = the context creates its own non-blocking one). */
int gpr_ctx_create(int device, void* stream, gpr_ctx_t* out);
int gpr_ctx_destroy(gpr_ctx_t ctx);
const char* gpr_last_error(gpr_ctx_t ctx);
const char* gpr_version(void);
int gpr_sync(gpr_ctx_t ctx);
void* gpr_ctx_stream(gpr_ctx_t ctx);
int gpr_malloc(gpr_ctx_t ctx, size_t bytes, void** dptr);
int gpr_free(gpr_ctx_t ctx, void* dptr);
int gpr_upload(gpr_ctx_t ctx, void* dst, const void* src, size_t bytes);   /* sync H2D */
int gpr_download(gpr_ctx_t ctx, void* dst, const void* src, size_t bytes); /* sync D2H */
/* Inner panel width of the blocked factorisations: 64 or 128 (default 128). */
int gpr_set_block(gpr_ctx_t ctx, int nb);
/* Outer panel width = K of the big MFMA trailing updates (default 1024, multiple of nb). */
int gpr_set_outer_block(gpr_ctx_t ctx, int nb2);
/* Per-kernel-class timing with HIP events on the context stream (bench instrumentation).
 * class: 0 K-assembly, 1 POTRF trailing update (SYRK), 2 POTRF panel (diag+TRSM),
 *        3 TRSM trailing GEMM, 4 other (call-site classes), 5 every launch of the
 *        pipelined MFMA GEMM kernel (kernel-level, overlaps 1-4), 6 tile-DAG factorisation
 *        launches (with any right-hand sides they solve), 7 solve-only tile-DAG launches
 *        (U^{-T} B from a finished factor: C5's variance rows, POTRI's Z).
 *        Returns accumulated ms, launch count, flops (bytes for class 0). */
/* Knobs: the library's run-time switches.  Each is a GPR_* environment variable read ONCE,
 * when a context is created, and can be changed on a live context with gpr_set_knob (values
 * are doubles, integer knobs truncate).  None of them changes a result beyond rounding: they
 * pick between equivalent code paths or size workspaces.  Unknown names: GPR_E_ARG.
 *   GPR_DAG            1  factorisations as one persistent tile-DAG launch; 0: the blocked
 *                         two-stream factorisation (inner nb, outer nb2)
 *   GPR_DAG_TAIL   12288  blocked path: the last <= this many columns go to the tile-DAG (0 off)
 *   GPR_DAG_SOLVE     -1  solves from a finished factor as solve-only tile-DAG launches
 *                         (-1 auto: n >= 8192 with >= n right-hand sides; 0 never; 1 always)
 *   GPR_DAG_GRAM       1  gpr_fit_kinv: K^{-1} = Z^T Z as gram tasks of the DAG launch
 *   GPR_DAG_ZLAG       4  DAG: Z = U^{-T}'s row i scheduled after A's row i + lag
 *   GPR_FUSED_RHS     -1  gpr_fit_predict: [K(x, xp) | y] solved inside the factorisation
 *                         (-1 auto, 0 after it, 1 own stream, 2 main stream; blocked path)
 *   GPR_FUSE_Y         1  gpr_fit: z = U^{-T} y inside the factorisation
 *   GPR_FUSE_KINV     -1  gpr_fit_kinv: Z (1) and Z^T Z (2) inside the factorisation (-1 = 2)
 *   GPR_KBUILD_UPPER   1  fits assemble only what dpotrf 'U' reads (the DAG mirrors the rest)
 *   GPR_KBUILD_EXACT   0  1: K by the reference's difference form instead of the Gram form
 *   GPR_KBUILD_COLSTORE 1 single-part (SE) upper builds store 1-KB column segments through LDS;
 *                         0: the MFMA D layout (4 columns x 128 B per store instruction)
 *   GPR_CV_BATCH       1  gpr_cv_batch: every fold in one batched launch; 0: per fold
 *   GPR_CV_BATCH_GB   16  device-memory budget of one batched cross-validation launch
 *   GPR_CV_STREAMS     4  child contexts of the per-fold / per-column paths (<= 8)
 *   GPR_QUAD_EIGEN    -1  gpr_integrate_noise: -1 auto (measured cost model), 0 per-column
 *                         factorisations, 1 tridiagonal reduction + per-column tridiagonal
 *                         solves, 3 full eigendecomposition (reduction + divide and conquer),
 *                         4 the same by block Jacobi (2, rocSOLVER dsyevd as a timing
 *                         comparator, exists only in the test build libgpr_hip_testing.so)
 *   GPR_QUAD_BATCH_GB 16  device-memory budget of one batched quadrature launch
 *   GPR_QUAD_SEQ       0  1: the per-column factorisations one at a time (no batch)
 * A gpr_mgpu handle has knobs of its own, read from the environment once at gpr_mgpu_create
 * and changed with gpr_mgpu_set_knob / gpr_mgpu_get_knob (below):
 *   GPR_MGPU_STREAM   -1  1: stream U out during device 0's fit; 0: after it (-1 auto: only
 *                         for one device)
 *   GPR_MGPU_CHUNKS   16  tile-row chunks of the broadcast (>= 1)
 *   GPR_MGPU_RESERVE_CU 8 CUs the streamed fit's launch leaves to the chunks' packs and RCCL
 * Fault injection (forced wait timeouts, failed unpacks, a one-device handle broadcasting to
 * itself) exists only in the test build libgpr_hip_testing.so. */
int gpr_set_knob(gpr_ctx_t ctx, const char* name, double value);
int gpr_get_knob(gpr_ctx_t ctx, const char* name, double* value);
int gpr_timing_enable(gpr_ctx_t ctx, int on);
int gpr_timing_get(gpr_ctx_t ctx, int cls, double* ms, long long* launches, double* flops);
int gpr_timing_reset(gpr_ctx_t ctx);

/* ---- a2/a3: kernel matrices --------------------------------------------------------- */
/* `same` argument of gpr_kernel: which of the reference's kernel! forms is meant.        */
#define GPR_CROSS 0       /* kernel!(K, cov, hp, x, xp), x !== xp: no eps, no noise         */
#define GPR_SELF 1        /* kernel!(K, cov, hp, x) (4-arg): eps per SE part + sigma_n^2 of  */
                          /* the first WhiteNoise part (add_noise!, src/compose_covar.jl:73) */
#define GPR_SAME_OBJECT 2 /* kernel!(K, cov, hp, x, xp) with x === xp (5-arg): eps per SE  */
                          /* part, NO noise (src/compose_covar.jl:47-61, covariance.jl:52-56)*/

/* K[n x m] (ldk) = kernel(cov, hp, x, xp).  same = GPR_SELF or GPR_SAME_OBJECT: dXp is
 * ignored and m must equal n (the symmetric matrix is written in full).  For a single
 * SquaredExp the two same-object forms coincide (eps only); they differ for composed
 * kernels with a WhiteNoise part, where only the 4-arg form adds sigma_n^2.
 * Replaces kernel!(kern, ::SquaredExp, hp, x, xp) src/covariance.jl:49-58,85-95,
 * kernel!(kern::AbstractGPUArray, ...) src/covar_gpu.jl:1-18 and
 * kernel!(kern, ::ComposedKernel, hp, x[, xp]) src/compose_covar.jl:47-77. */
int gpr_kernel(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
               const double* dX, int n, const double* dXp, int m, int same, double eps,
               double* dK, int ldk);

/* a4: dK/dtheta_i (1-based i) materialised, n x n.  WN part: writes 2*sigma_n*I.
 * Replaces grad!(::SquaredExp, DK, i, hp, x, K) src/deriv_covar.jl:20-32 and the
 * composed index mapping src/compose_covar.jl:109-123. */
int gpr_kernel_grad(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                    const double* dX, int n, int i, double eps, double* dDK, int ld);

/* ---- a5-a7: factor / solve --------------------------------------------------------- */
/* In-place upper Cholesky of the SPD matrix in dA (n x n, lda): upper triangle <- U with
 * K = U^T U, strict lower triangle untouched.  *info = 0 or the order of the failing
 * minor.  Replaces cholesky!(Hermitian(K)) = dpotrf('U') (src/cost.jl:77,87,104,
 * src/predict.jl:31).  The context keeps the inverses of the diagonal blocks for the
 * following gpr_potrs/gpr_trsm/gpr_potri calls on the same factor.
 * Implementation: one persistent tile-DAG launch (128 x 128 tile tasks); n and lda
 * multiples of 16 with a 128-B aligned dA are factored in place, other shapes on a padded
 * device copy (n rounded up to 16: an extra ~8 n^2 bytes of device memory, same result);
 * the knob GPR_DAG=0 selects the blocked two-stream factorisation. */
int gpr_potrf_upper(gpr_ctx_t ctx, double* dA, int n, int lda, int* info);

/* The context caches the factor's block inverses (and the outer squares' inverses) after a
 * factorisation or a first solve, keyed on the factor's device pointer and shape.  A factor
 * written into a buffer by anything other than this context (a broadcast, a copy, another
 * context) must be announced with gpr_forget_factor, or a following solve on the same pointer
 * reuses inverses of the previous contents. */
int gpr_forget_factor(gpr_ctx_t ctx);

/* B <- K^{-1} B for K = U^T U (dU from gpr_potrf_upper), B n x nrhs (ldb).
 * Replaces ldiv!(alpha, kchol, y) = dpotrs (src/cost.jl:79,89,106, src/predict.jl:32). */
int gpr_potrs_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                    int ldb);

/* B <- U^{-T} B (left, upper, transposed triangular solve).  With B = K(x, xp)^T this is
 * rdiv!(Kxp, kchol.U) (src/predict.jl:84,90,98) in the transposed layout. */
int gpr_trsm_upper_trans(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dB,
                         int nrhs, int ldb);

/* Full symmetric K^{-1} (n x n, ldk) from the factor.  Replaces
 * K^-1 = I ; ldiv!(kchol, K^-1) (src/cost.jl:90-92,107-109). */
int gpr_potri_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dKinv, int ldk);

/* ---- a8/a9: marginal likelihood ------------------------------------------------------ */
/* *out = 0.5 (y.alpha + 2 sum log U_ii + n log 2pi)  (src/loss_grad.jl:39-41). */
int gpr_mll(gpr_ctx_t ctx, const double* dU, int n, int ldu, const double* dy,
            const double* dalpha, double* out);

/* grad[D] (host) of the negative log-marginal-likelihood w.r.t. hp, fused over all D
 * hyper-parameters in one pass over the upper triangle of K^{-1} (never materialising
 * dK): g_i = -0.5 sum_ab (alpha_a alpha_b - Kinv_ab) dK_i,ab.  Replaces the grad! loop of
 * src/cost.jl:119-126 with src/loss_grad.jl:43-52 and src/deriv_covar.jl:20-32.
 * log_scale != 0 applies G .*= hp (src/cost.jl:60-70). */
int gpr_mll_grad(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                 const double* dX, int n, const double* dKinv, int ldk,
                 const double* dalpha, double eps, int log_scale, double* grad);

/* One-call fit = update_cache!(MllLossCache / GPRPredictCache) (src/cost.jl:74-81,
 * src/predict.jl:29-34): dK (n x n, ldk) <- kernel, then in-place POTRF, then
 * dalpha <- K^{-1} dy (nrhs columns, ldy).  Returns info > 0 if not PD. */
int gpr_fit(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
            const double* dX, int n, const double* dy, int nrhs, int ldy, double eps,
            double* dK, int ldk, double* dalpha, int* info);

/* ---- a10/a11: posterior ------------------------------------------------------------ */
/* Posterior at m test points from a fitted factor (dU, dwt = K^{-1} y with nrhs cols).
 * mode GPR_PREDICT_MEAN: dmu (m x nrhs, ldmu=m).  GPR_PREDICT_DIAG: + dvar[m] =
 * prior - ||U^{-T} k_j||^2 (prior sigma^2 or sum of all parts' hp[1]^2, no eps:
 * src/predict.jl:51-71,89-95).  GPR_PREDICT_FULL: + dvar (m x m, ldv) = K(xp,xp) -
 * V^T V (src/predict.jl:42-49,83-87).  dwork: optional device scratch of n*m doubles
 * (NULL: the context allocates it).  Replaces predict!/predict_mean! src/predict.jl.
 * Same-object rule: dXp == dX (with m == n) is the C analogue of `xp === md.x`; then
 * K(xp, x) takes the reference's same-object branch of kernel!(Kxp, covar, hp, xp, md.x)
 * (src/predict.jl:37,43): eps once per SE part on its diagonal, no noise
 * (src/covariance.jl:52-56, src/compose_covar.jl:47-61).  Any other dXp: cross kernel. */
int gpr_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                const double* dX, int n, const double* dU, int ldu, const double* dwt,
                int nrhs, const double* dXp, int m, int mode, double eps, double* dmu,
                double* dvar, int ldv, double* dwork);

/* ---- a5/a6/a7 fused: update_cache!(::MllGradCache) = K, cholesky!, alpha, K^{-1} --------- */
/* src/cost.jl:83-111 in one call: K into dK (upper -> U, lower keeps K), alpha = K^{-1} y
 * (n x nrhs), dKinv = full symmetric K^{-1} (ldkinv).  Z = U^{-T} and K^{-1} = Z^T Z are
 * computed inside the factorisation: as right-hand-side and gram tile tasks of the one
 * tile-DAG launch (n a multiple of 16, 128-B aligned dK), else in the blocked
 * factorisation's lookahead bubbles (GPR_FUSE_KINV=1: Z alone inside, 0: both after it).
 * Device workspace: n^2 doubles for Z.  >0: LAPACK info. */
int gpr_fit_kinv(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                 const double* dX, int n, const double* dy, int nrhs, int ldy, double eps,
                 double* dK, int ldk, double* dalpha, double* dKinv, int ldkinv, int* info);

/* ---- a5/a6/a10/a11 fused: predict(md, xp; diagonal_var) from scratch ---------------- */
/* The reference's predict (src/predict.jl:14-25 -> update_cache!(pc, md) :29-34 = K, cholesky!,
 * ldiv!(wt, kchol, md.y), then predict! :36-71) in one call: K(x, x) into dK (upper
 * overwritten by U, lower keeps K, as gpr_fit), posterior mean/variance at m test points as
 * gpr_predict.  With mode DIAG/FULL the triangular solve of [K(x, xp) | y] runs inside the
 * factorisation (right-hand-side tile tasks of the tile-DAG launch; on the blocked path outer
 * block s is solved once panel s of U is final), mu = V^T z with
 * V = U^{-T} K(x, xp), z = U^{-T} y; dalpha (optional, n x nrhs) = K^{-1} y.  dwork: optional
 * n*(m+nrhs) doubles.  Returns >0 (LAPACK info) for a non-PD K.  dXp == dX: the
 * same-object rule of gpr_predict (K(xp, x) gets eps per SE part, no noise). */
int gpr_fit_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                    const double* dX, int n, const double* dy, int nrhs, int ldy, double eps,
                    double* dK, int ldk, double* dalpha, const double* dXp, int m, int mode,
                    double* dmu, double* dvar, int ldv, double* dwork, int* info);

/* ---- 8(f) rank 3: Bayesian quadrature of the posterior (src/integrate.jl) ------------- */
/* antideriv!(k1, SquaredExp(), x, hp, a, b) and antideriv2 (src/integrate.jl:16-46): dk1[n]
 * = sigma^2 (sqrt(pi)/2)^d prod(1/l) prod_i erf(l_i (a_i - x_i), l_i (b_i - x_i)) on the
 * device, *k2 = sigma^2 prod_i erf_integ(l_i, a_i, b_i) (host); hp[0] = sigma, hp[1..d] = l
 * (the first d + 1 entries, as the reference indexes md.params).  a, b: host d-vectors;
 * dk1 or k2 may be NULL. */
int gpr_antideriv_se(gpr_ctx_t ctx, int d, const double* hp, const double* dX, int n,
                     const double* a, const double* b, double* dk1, double* k2);
/* integrate(md, hp, a, b; sample_noise=nothing) (src/integrate.jl:48-167): fit (K into dK ->
 * U, dwt = K^{-1} y, n x ny), Iout[ny] = wt' k1, *var = k2 - ||U^{-T} k1||^2 (host outputs).
 * The sample_noise path (syevr + diagonal updates, :71-104) is gpr_integrate_noise below. */
int gpr_integrate(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                  const double* dX, int n, const double* dy, int ny, int ldy, const double* a,
                  const double* b, double eps, double* dK, int ldk, double* dwt, double* Iout,
                  double* var);

/* cv_batch(md, cost, x, y, (trn, tst)) (src/crossval.jl:13-35): for each fold f, fit the
 * model on the training points trn[f*ntrn .. +ntrn) of (dX, dy) and predict the test points
 * tst[f*ntst .. +ntst) with the FULL posterior covariance (cv_step!, :46-51 = update_cache!
 * + predict!), then lss[f] = loss(cost, ytst, yp, Sigma_p) with cost GPR_COST_*.
 * trn/tst: host arrays of 0-based point indices (< n), fold-major; lss: host, nfold.
 * dX: d x n column-major, dy: n.  Returns info > 0 if a training K (or, for Mahalanobis,
 * Sigma_p) is not positive definite -- the reference's PosDefException. */
int gpr_cv_batch(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                 const double* dX, int n, const double* dy, const int* trn, int ntrn,
                 const int* tst, int ntst, int nfold, int cost, double eps, double* lss);

/* integrate(md, hp, a, b; sample_noise = noise::Vector) (src/integrate.jl:71-100,149-162):
 * per column j of y (ny columns, noise[j] host), Iout[j] = k1' (K + noise_j I)^{-1} y_j and
 * var[j] = k2 - k1' (K + noise_j I)^{-1} k1.  The reference decomposes K = P Lambda P' once
 * (LAPACK syevr) and then only updates a diagonal per column.  Here, by default, one of:
 *  - the tridiagonal reduction K = Q T Q' (syevr's first stage, gpr_sytrd_apply, with
 *    C = Q' [y | k1] formed inside the reduction), then per column one pivoted tridiagonal
 *    solve: Iout[j] = C[:, j]' (T + noise_j I)^{-1} C[:, ny] -- any shift, no factorisation,
 *    never info > 0 (an indefinite K + noise_j I gives the reference's indefinite solve);
 *  - the K + noise_j I factored per column, all in one batched tile-DAG launch that also solves
 *    U_j^{-T} [y_j | k1] (same result within rounding), while that is measured to cost less
 *    (ny below ~175 at n = 4096, ~220 at 2048, ~330 at 1100, ~700 at 512, ~140 at 8192;
 *    always beyond the reduction's bound n > 16384); a factorisation that fails (a shift at or
 *    below -lambda_min(K)) hands the call to the reduction, so the default never returns
 *    info > 0 up to that bound.  A reduction whose cooperative launch the runtime refuses (its
 *    workgroups cannot all be resident) falls back to the factorisations.
 * GPR_QUAD_EIGEN forces a route: 1 the reduction; 3 the reference's full decomposition
 * (reduction + divide and conquer, gpr_syev_apply) and its diagonal updates; 0 always the
 * factorisations (positive definite shifts only; info > 0 -- PosDefException -- otherwise);
 * 2 rocSOLVER dsyevd -- a timing comparator compiled into the test build libgpr_hip_testing.so
 * only (GPR_E_ARG here). */
int gpr_integrate_noise(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                        const double* dX, int n, const double* dy, int ny, int ldy,
                        const double* a, const double* b, const double* noise, double eps,
                        double* Iout, double* var);

/* The symmetric eigendecomposition behind the sample_noise quadrature (LAPACK.syevr! at
 * src/integrate.jl:75), applied instead of returned: A (n x n, ld lda, device, read only,
 * symmetric) = P diag(lam) P'; on return dlam[n] (device) holds the eigenvalues -- in no
 * particular order -- and dB (n x m, ld ldb, device) holds P' B, its rows in the order of
 * dlam.  FP64, as dsyevd: the tridiagonal reduction (gpr_sytrd_apply, B <- Q' B) then Cuppen's
 * divide and conquer on T (deflation, secular equations, Gu-Eisenstat vectors; Z never formed:
 * B <- Z' B merge by merge).  n > 16384, or a reduction whose cooperative launch is refused:
 * two-sided block Jacobi (32-wide blocks, parallel ordering).  *sweeps (may be NULL) = merge levels (Jacobi: sweeps used).  GPR_E_HIP if Jacobi
 * does not converge within 60 sweeps. */
int gpr_syev_apply(gpr_ctx_t ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                   double* dlam, int* sweeps);

/* The first stage of that decomposition on its own (LAPACK dsytrd, inside syevr): A (n x n,
 * ld lda, device, read only, symmetric -- both triangles read) = Q T Q^T with T tridiagonal:
 * dd[n] its diagonal, de[n-1] its off-diagonal (device), and, when m > 0, dB (n x m, ld ldb)
 * <- Q^T dB.  One persistent launch (the unblocked two-sided Householder reduction, columns
 * dealt round-robin over the CUs; for m <= 1024 Q^T B is formed inside it), else the
 * back-transform by 64-reflector blocks on the MFMA GEMM.  The launch is cooperative (every
 * workgroup resident or refused up front: GPR_E_UNSUP, nothing touched); below n = 5376 its
 * step vectors sit in LDS and every step updates every trailing column; from 5376 on the
 * updates are deferred by panels of 16 steps (later columns only read per step, flushed per
 * panel by an MFMA GEMM).  n <= 16384 (GPR_E_UNSUP beyond). */
int gpr_sytrd_apply(gpr_ctx_t ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                    double* dd, double* de);

/* ---- a12-a15: split-kernel block prediction ---------------------------------------- */
/* Test grid x_{e,q} = xe_e + xq_q (Cmap(+, xe, xq), src/split_kernel.jl:1-17).
 * dmu: ne x nq column-major (index e + q*ne, src/split_predict.jl:10-19).
 * dvar: ne*nq diagonal; entries (e*nq + q) for e in [var_lo, var_hi) (0-based,
 * half-open; the reference default var_range=1:3 is [0,3)) get prior - ||U^{-T} k||^2,
 * every other entry is set to the prior (src/split_predict.jl:39-53).
 * e_lo/e_hi restrict the call to grid rows [e_lo, e_hi) (multi-GPU sharding: each rank
 * passes its own row range; dmu/dvar still index the FULL grid layout, only the rows in
 * range are written).  dwt is the 1-column K^{-1} y.
 * Replaces kernel!(::SplitKernel,...) src/split_kernel.jl:137-159 and
 * predict_split_mean_impl!/predict_covar_impl! src/split_predict.jl:5-53. */
int gpr_split_predict(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                      const double* dX, int ns, const double* dU, int ldu,
                      const double* dwt, const double* dXe, int ne, const double* dXq,
                      int nq, int e_lo, int e_hi, int var_lo, int var_hi, double eps,
                      double* dmu, double* dvar);

/* gpr_split_predict over several pieces of grid rows at once: pieces = host array of
 * npieces sorted, disjoint half-open ranges {lo_0, hi_0, lo_1, hi_1, ...} (a rank's shard:
 * an even share of the variance rows plus an even share of the rest, gpr_shard_pieces).  The
 * ns x nq C factor is built once per call instead of once per piece; dmu / dvar index the
 * full grid layout as in gpr_split_predict, only the rows in the pieces are written. */
int gpr_split_predict_rows(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                           const double* dX, int ns, const double* dU, int ldu, const double* dwt,
                           const double* dXe, int ne, const double* dXq, int nq, const int* pieces,
                           int npieces, int var_lo, int var_hi, double eps, double* dmu,
                           double* dvar);

/* gpr_split_predict_rows with outputs sized to the shard, not to the grid: the pieces' R rows
 * concatenated in piece order (row e of piece k at r = off_k + e - lo_k, off_k = rows of the
 * pieces before it).  dmu: R x nq column-major, leading dimension ldmu >= R (index r + q*ldmu);
 * dvar: R*nq (index r*nq + q).  What a rank of a multi-GPU split prediction allocates
 * (R ~ ne / ngpu rows instead of ne). */
int gpr_split_predict_shard(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                            const double* dX, int ns, const double* dU, int ldu,
                            const double* dwt, const double* dXe, int ne, const double* dXq,
                            int nq, const int* pieces, int npieces, int var_lo, int var_hi,
                            double eps, double* dmu, int ldmu, double* dvar);

/* Split factors for inspection/tests (src/split_kernel.jl:151-159), SE part `part`
 * (0-based among SE parts): dA ne x nq, dB ne x ns, dC ns x nq (column-major,
 * leading dims = row counts). */
int gpr_split_factors(gpr_ctx_t ctx, const int* kinds, int nk, const double* hp, int d,
                      const double* dX, int ns, const double* dXe, int ne,
                      const double* dXq, int nq, int part, double* dA, double* dB,
                      double* dC);

/* ---- 8(e): split prediction sharded over the GPUs of one node, one host process ------- */
/* Row pieces of grid row count n for `rank` of `world`: an even share of the variance rows
 * [v_lo, v_hi) plus an even share of the others, as at most 3 sorted, disjoint, merged
 * half-open ranges written to pieces[0..5] ({lo, hi} pairs).  Returns their number (or < 0).
 * Host-only helper (no device work); the same partition as gpr_amd.distributed.shard_pieces. */
int gpr_shard_pieces(int n, int world, int rank, int v_lo, int v_hi, int* pieces);

/* The upper triangle of a column-major n x n factor packed by 128-column blocks (block
 * [j0, j1) keeps rows [0, j1) of its columns): gpr_packed_upper_len(n) ~ n^2/2 + 64 n doubles,
 * half the bytes of U for a broadcast.  Unpacking leaves the rest of dU untouched (no solve
 * reads it).  A Julia MPI caller broadcasting pc.Kxx between processes uses these pairs, then
 * gpr_forget_factor on the receivers. */
size_t gpr_packed_upper_len(int n);
int gpr_pack_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dP);
int gpr_unpack_upper(gpr_ctx_t ctx, const double* dP, int n, double* dU, int ldu);

typedef struct gpr_mgpu* gpr_mgpu_t;
#define GPR_MGPU_BROADCAST 0 /* device 0 fits; RCCL broadcast of packed U + wt (xGMI)   */
#define GPR_MGPU_REPLICATE 1 /* every device fits for itself (no N^2 exchange)          */

/* A set of ngpu devices (distinct ids) with one context each and an RCCL communicator
 * (ncclCommInitAll; librccl.so.1 is dlopen'd: the process's own if loaded, else the
 * system's).  Create once, reuse across calls. */
int gpr_mgpu_create(int ngpu, const int* devices, gpr_mgpu_t* out);
int gpr_mgpu_destroy(gpr_mgpu_t h);
const char* gpr_mgpu_last_error(gpr_mgpu_t h);
/* The handle's knobs (GPR_MGPU_STREAM, GPR_MGPU_CHUNKS, GPR_MGPU_RESERVE_CU; see gpr_set_knob).
 * Unknown names: GPR_E_ARG. */
int gpr_mgpu_set_knob(gpr_mgpu_t h, const char* name, double value);
int gpr_mgpu_get_knob(gpr_mgpu_t h, const char* name, double* value);

/* predict(md, Cmap(+, xe, xq); diagonal_var=true) (src/predict.jl:14-25 ->
 * src/split_predict.jl:5-53) sharded over the handle's GPUs.  HOST arrays in and out (the
 * reference's CPU arrays): X d x ns, y ns, Xe d x ne, Xq d x nq; mu ne x nq column-major
 * (index e + q ne), var ne*nq (index e nq + q; rows outside [var_lo, var_hi) keep the prior).
 * fit_mode GPR_MGPU_BROADCAST / GPR_MGPU_REPLICATE.  Device i computes the rows
 * gpr_shard_pieces(ne, ngpu, i, var_lo, var_hi) and copies them into mu / var itself.
 * Returns > 0 (and *info) when K is not positive definite.  With ngpu = 1 the result equals
 * gpr_fit + gpr_split_predict on that device bit for bit.
 * Broadcast mode streams U out while device 0 factors it: chunks of 128-row tile rows
 * (GPR_MGPU_CHUNKS, default 16, about equal bytes) are packed and broadcast as soon as the
 * tile-DAG launch has finalised them, on a stream of their own and the GPR_MGPU_RESERVE_CU
 * (default 8) CUs the launch leaves free; the receivers unpack each chunk as it lands.
 * GPR_MGPU_STREAM=0 sends the same chunks after the fit instead. */
int gpr_split_predict_mgpu(gpr_mgpu_t h, const int* kinds, int nk, const double* hp, int d,
                           const double* X, int ns, const double* y, const double* Xe, int ne,
                           const double* Xq, int nq, int var_lo, int var_hi, double eps,
                           int fit_mode, double* mu, double* var, int* info);

#ifdef __cplusplus
}
#endif
#endif /* GPR_HIP_H */
