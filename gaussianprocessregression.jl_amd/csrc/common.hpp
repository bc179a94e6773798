// Shared internals of libgpr_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#include "../../include/gpr_hip.h"

#define KMAXP 4   // max SquaredExp parts handled by the fused kernels
#define KMAXD GPR_MAX_DIM

// Kernel description passed BY VALUE to every assembly kernel (< 4 KB of kernargs).
// Mirrors split(hp, dims) of src/compose_covar.jl:21-28: the SE parts in `+` order
// and the first WhiteNoise part (add_noise! src/compose_covar.jl:63-71).
struct KParams {
  int d;          // input dimension
  int nse;        // number of SquaredExp parts (1..KMAXP)
  int has_noise;  // a WhiteNoise part is present
  int hp_off_noise;              // flat hp index of sigma_n (for the gradient)
  double eps;                    // jitter per SE part on a same-object diagonal
  double noise2;                 // sigma_n^2
  double noise_sigma;            // sigma_n
  double sigma[KMAXP];           // sigma of each SE part
  int hp_off[KMAXP];             // flat hp index of each SE part's sigma
  double l[KMAXP][KMAXD];        // inverse length-scales (multipliers) per SE part
  double l2[KMAXP][KMAXD];       // their squares (the gradient pass's distance)
  const double* exptab;          // device table 2^(j/256), j < 256 (ctx->dexptab)
};

// TC_GEMM_PIPE is kernel-level (every launch of the pipelined 2-WG/CU GEMM, whatever its call
// site), recorded in addition to the call-site class.
enum TimingClass {
  TC_KBUILD = 0, TC_SYRK = 1, TC_PANEL = 2, TC_TRSM_GEMM = 3, TC_OTHER = 4, TC_GEMM_PIPE = 5,
  TC_DAG = 6, TC_DAG_SOLVE = 7, TC_N = 8
};

struct TimedLaunch {
  int cls;
  hipEvent_t a, b;
  double flops;
};

struct gpr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  int nb = 128;   // inner panel width (diag blocks, in-place panel GEMMs)
  int nb2 = 1024;  // outer panel width = K of the big trailing updates (multiple of nb)
  hipStream_t ls = nullptr;       // stream the launch helpers enqueue on (default: stream)
  hipStream_t stream2 = nullptr;  // lookahead panel stream (GEMMs of the panel chain)
  hipStream_t srhs = nullptr;     // right-hand-side solves fused into the factorisation
  hipStream_t ssq = nullptr;      // square inverses of finished outer panels (fused solves)
  // gpr_fit_predict: 0 = factor, then solve (default); 1 / 2 = solve inside the factorisation
  // on its own stream / on the main stream (GPR_FUSED_RHS; measured slower at C3: 347 vs 334 ms)
  int fused_rhs = -1;             // gpr_fit_predict: -1 auto (fused, mode 2, when the tile-DAG
                                  // factors or n <= fused_rhs_nmax), 0 off, 1/2 forced
                                  // (GPR_FUSED_RHS)
  int fused_rhs_nmax = 16384;
  int fuse_y = 1;                 // gpr_fit: z = U^{-T} y inside the factorisation, then the
                                  // backward sweep alone (GPR_FUSE_Y=0: both sweeps after it;
                                  // C5's fit on one GPU: 727 -> 714 ms per job)
  int fuse_kinv = -1;             // gpr_fit_kinv (GPR_FUSE_KINV; -1 auto = 2): Z = U^{-T} solved
                                  // inside the factorisation (1), and K^{-1} = Z^T Z too (2) --
                                  // tile-DAG right-hand-side and gram tasks, or the blocked
                                  // factorisation's lookahead bubbles
  // persistent tile-DAG factorisation (dag.hip): 0 off (GPR_DAG=0: the blocked two-stream
  // factorisation), 1 on; the task list is cached per (tiles, rhs tiles).
  // Measured (POTRF alone, blocked -> DAG): N = 8192 9.3 -> 6.8 ms, 16384 34.5 -> 25.0,
  // 32768 193 -> 173.4 (67.7 TF/s); C3 fit + predict in one DAG launch 321.8 -> 305.5 ms.
  int dag_mode = 1;
  long long dag_spin_limit = 1ll << 25;  // DAG dependency wait bound in polls (~4 s); test
                                        // builds let GPR_DAG_SPIN_LIMIT override it per launch
  int dag_zlag = 4;       // lower-triangular right-hand-side rows scheduled after A's row i + lag (GPR_DAG_ZLAG)
  int dag_lag_built = -1;
  // one-shot hook of the next whole-matrix factorisation launch (kglob 0, not a solve), called
  // right after the kernel is enqueued with an event that completes once the launch's progress
  // counters are reset (null if it could not be made): work ordered behind that event runs
  // BESIDE the launch (mgpu.hip streams finished tile rows of U out to the other GPUs); cleared
  // before the call
  // (colprog: the progress counters; ustored[i] = 1 once the diagonal tile U_ii is stored --
  // the launch raises colprog before that store)
  void (*dag_hook)(void* user, const double* dA, int n, int lda, const int* colprog,
                   const int* ustored, int nt, hipEvent_t counters_reset) = nullptr;
  void* dag_hook_user = nullptr;
  int dag_reserve_cu = 0;  // CUs the persistent grid leaves free for such concurrent work
  // set by a hook that left work polling dag_sync on another stream: the next DAG launch on
  // this context waits for it before resetting (or reallocating) the counters
  hipEvent_t dag_sync_readers = nullptr;
  bool dag_sync_readers_pending = false;
  bool rhs_solved = false; // the last potrf_core solved its RhsSpec (not dropped by its block sizes)
  bool gram_full = false; // the last potrf_core wrote its RhsSpec gram in full (the tile-DAG)
  int dag_gram = 1;       // K^{-1} += Z^T Z as gram tile tasks of the DAG launch (GPR_DAG_GRAM)
  int dag_solve = -1;     // solves from a finished factor as solve-only DAG launches (GPR_DAG_SOLVE; -1 auto)
  int dag_tail = 12288;  // blocked factorisations (GPR_DAG=0, ineligible sizes) hand their last
                         // <= dag_tail columns to the DAG (GPR_DAG_TAIL; 0 = off)
  unsigned* dag_tasks = nullptr;
  int dag_ntasks = 0, dag_nt = -1, dag_ntr = -1, dag_flags = -1;
  int* dag_sync = nullptr;
  size_t dag_sync_cap = 0;
  double* dpadA = nullptr;  // padded copies for shapes the DAG launch does not take directly
  size_t padA_cap = 0;
  double* dpadB = nullptr;
  size_t padB_cap = 0;
  // rocSOLVER (dlopen'd, gpr_integrate_noise's eigendecomposition): a rocBLAS handle on this
  // context's stream, created on first use; rb_destroy releases it
  void* rb_handle = nullptr;
  int (*rb_destroy)(void*) = nullptr;
  int ncu = 0;
  std::vector<hipEvent_t> sync_events;
  size_t ev_next = 0;

  // cached inverses of the diagonal blocks of the last factor: winv[b] = U_bb^{-1}
  // (nb x nb, column-major, strictly-lower part zero), one slot per block.
  double* winv = nullptr;
  size_t winv_cap = 0;  // doubles
  const double* fac_ptr = nullptr;
  int fac_n = 0, fac_ld = 0, fac_nb = 0;
  bool fac_valid = false;

  int* dinfo = nullptr;         // device info word
  double* dexptab = nullptr;    // 2^(j/256), j < 256, correctly rounded (assembly exp)
  double* dscratch = nullptr;   // generic scratch (partials, small vectors)
  size_t scratch_cap = 0;       // doubles
  // child contexts that run cross-validation folds concurrently (gpr_cv_batch)
  static constexpr int CV_MAX_SUB = 8;
  struct gpr_ctx* cv_sub[CV_MAX_SUB] = {};
  int cv_streams = 4;  // GPR_CV_STREAMS
  double* dbig = nullptr;       // large scratch (Z for potri, Kpx for predict, ...)
  size_t big_cap = 0;           // doubles
  double* dbig2 = nullptr;
  size_t big2_cap = 0;
  double* dsqinv = nullptr;     // U_sq^{-1} of every outer panel square (nb2^2 per slot)
  size_t sqinv_cap = 0;         // doubles
  int sqinv_nb2 = 0;            // nb2 the slots were written with (0 = none valid)
  const double* sq_ptr = nullptr;  // factor the slots belong to
  int sq_n = 0, sq_ld = 0;
  double* dpanel = nullptr;     // out-of-place result of the panel's rest GEMM
  size_t panel_cap = 0;
  double* dtrsv = nullptr;      // single-launch triangular sweep hand-off vector (n x 2)
  size_t trsv_cap = 0;
  double* dxs = nullptr;        // per-part scaled training inputs  (nse x d x n)
  size_t xs_cap = 0;
  double* dxps = nullptr;       // per-part scaled second inputs    (nse x d x m)
  size_t xps_cap = 0;
  double* dscr_wt = nullptr;     // gpr_fit_predict: K^{-1} y when the caller passes no alpha
  size_t scr_wt_cap = 0;
  double* dpanel_rhs = nullptr;  // solved outer panel of the fused right-hand sides
  size_t panel_rhs_cap = 0;
  double* dgA = nullptr;        // Gram-assembly row operands (MFMA lane order, assembly.hip)
  size_t gA_cap = 0;
  double* dgB = nullptr;        // Gram-assembly column operands
  size_t gB_cap = 0;
  double* dgc = nullptr;        // Gram-assembly centres (KMAXP x KMAXD)
  size_t gc_cap = 0;
  // upper-only K assembly for a factorisation (assembly.hip kmat_symu_kernel): its work list
  // (strip << 16 | segment, built once per n) and the matrix it last left without its strict
  // lower off-diagonal tiles -- the next potrf_core on exactly that matrix has the tile-DAG
  // write them (DAG_MIRROR), or mirrors them first on any other path
  struct KupList {
    long long key = -1;  // 2 n + full
    int nitems = 0;
    int* d = nullptr;
    unsigned long long used = 0;
  };
  KupList kup[4];
  unsigned long long kup_clock = 0;
  const double* kup_ptr = nullptr;
  int kup_n = 0, kup_ld = 0;
  double* dagb = nullptr;       // batched tile-DAG workspace (W slots, task lists, counters)
  size_t dagb_cap = 0;
  double* deig = nullptr;       // eigensolver workspace (eigen.hip, tridiag.hip)
  size_t eig_cap = 0;
  double* ddc = nullptr;        // divide-and-conquer workspace (dstedc.hip)
  size_t dc_cap = 0;
  // its merge tables' pinned host staging buffer, re-filled only after dc_tab_ev (the previous
  // call's upload) has completed
  int* dc_tab_host = nullptr;
  size_t dc_tab_host_cap = 0;
  hipEvent_t dc_tab_ev = nullptr;
  double* dtri = nullptr;       // the tridiagonal T between the two stages
  size_t tri_cap = 0;
  int kbuild_upper = 1;         // GPR_KBUILD_UPPER=0: fits build the full K (mirrored tiles)
  int kbuild_exact = 0;         // GPR_KBUILD_EXACT=1: the reference's difference form for K
  int kbuild_colstore = 1;      // GPR_KBUILD_COLSTORE=0: single-part upper builds store in the
                                // MFMA D layout instead of 1-KB column segments
  int cv_batch = 1;             // GPR_CV_BATCH=0: cv_batch folds one by one on child contexts
  double cv_batch_gb = 16.0;    // GPR_CV_BATCH_GB: device-memory budget of a batched launch
  double quad_batch_gb = 16.0;  // GPR_QUAD_BATCH_GB: the same for the quadrature's columns
  int quad_eigen = -1;          // GPR_QUAD_EIGEN: sample_noise quadrature path (-1 auto)
  int quad_seq = 0;             // GPR_QUAD_SEQ=1: its per-column factorisations one at a time

  bool timing = false;
  std::vector<TimedLaunch> pending;
  std::vector<hipEvent_t> event_pool;
  double t_ms[TC_N] = {};
  long long t_launches[TC_N] = {};
  double t_flops[TC_N] = {};
};

// ---- error helpers -------------------------------------------------------------------
// split prediction of sorted, disjoint row pieces [pieces[2k], pieces[2k+1]) (predict.hip)
int split_predict_pieces(gpr_ctx* ctx, const int* kinds, int nk, const double* hp, int d,
                         const double* dX, int ns, const double* dU, int ldu, const double* dwt,
                         const double* dXe, int ne, const double* dXq, int nq, const int* pieces,
                         int npieces, int var_lo, int var_hi, double eps, double* dmu, int ldmu,
                         double* dvar, bool compact);
int set_err(gpr_ctx* ctx, int code, const char* fmt, ...);
// the knob values of `from` onto `to` (child contexts follow their parent)
void copy_knobs(const gpr_ctx* from, gpr_ctx* to);

#define HIP_TRY(ctx, expr)                                                          \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return set_err(ctx, GPR_E_HIP, "%s failed: %s (%s:%d)", #expr,                \
                     hipGetErrorString(_e), __FILE__, __LINE__);                    \
  } while (0)

#define GPR_TRY(expr)            \
  do {                           \
    int _r = (expr);             \
    if (_r != 0) return _r;      \
  } while (0)

#define LAUNCH_CHECK(ctx) HIP_TRY(ctx, hipGetLastError())

// ---- workspace ------------------------------------------------------------------------
int ensure_buf(gpr_ctx* ctx, double** p, size_t* cap, size_t need_doubles);
int ensure_winv(gpr_ctx* ctx, int n, int nb);

// ---- timing ---------------------------------------------------------------------------
struct TimerScope {
  gpr_ctx* ctx;
  TimedLaunch tl;
  bool on;
  hipStream_t st;
  TimerScope(gpr_ctx* c, int cls, double flops);
  ~TimerScope();
};

// ---- parse a kernel description -------------------------------------------------------
int make_kparams(gpr_ctx* ctx, const int* kinds, int nk, const double* hp, int d,
                 double eps, KParams* kp, int* D_total);

// ---- cross-TU launchers ---------------------------------------------------------------
// C[m,n] = alpha * sum_{k<K} P[k + m*ldp] * Q[k + n*ldq] (* qscale[k]) + beta * C[m,n]
struct GemmArgs {
  const double* P; int ldp;
  const double* Q; int ldq;
  double* C; int ldc;
  int M, N, K;
  double alpha, beta;
  int upper;              // grid over upper tiles only (M == N) + element mask m <= n
  int mask_upper;         // element mask m <= n + mask_off on a general grid
  int mask_off;           // column offset of C relative to its row origin (mask_upper)
  int kfrom_n;            // tile's K loop starts at its n0 (triangular factor, Z^T Z)
  int kend_from_m;        // tile's K loop ends at min(K, m0+TM) (upper-triangular P:
                          // P[t][m] = 0 for t > m, e.g. P = U^{-1})
  const double* qscale;   // optional per-k scale of Q (diag(wt) C)
  const double* E; int lde;  // optional Hadamard factor: C = beta*C + alpha*acc*E
  double* norm_out;       // optional: norm_out[n] -= sum_m (result)^2 (needs M <= tile)
  const int* info;        // optional: skip when *info != 0
  int occ1;               // launch at one workgroup per CU (lookahead co-residence)
};
int launch_gemm_tn(gpr_ctx* ctx, const GemmArgs& g, int timing_class);

int launch_kernel_matrix(gpr_ctx* ctx, const KParams& kp, const double* dX, int n,
                         const double* dXp, int m, int same, double* dK, int ldk);
// K for a factorisation that follows at once (potrf_core on exactly dK): where the tile-DAG
// takes the matrix directly, only what the factorisation reads is assembled -- the upper
// triangle and the whole 128 x 128 diagonal blocks, column-contiguously -- and the DAG writes
// the strict lower off-diagonal tiles from the tiles it loads (DAG_MIRROR); anything else
// gets the full symmetric K.  The buffer ends as the reference's: upper U, strict lower K.
int launch_kernel_matrix_for_factor(gpr_ctx* ctx, const KParams& kp, const double* dX, int n,
                                    double* dK, int ldk);
int launch_mirror_upper(gpr_ctx* ctx, double* A, int n, int lda);
int launch_scale_inputs(gpr_ctx* ctx, const KParams& kp, const double* dX, int n, double* out);
int launch_pair(gpr_ctx* ctx, int mode, int d, const double* xa, int na, const double* xb, int nb,
                double s2, double* out, size_t sa, size_t sb);
int launch_set_identity(gpr_ctx* ctx, double* A, int n, int lda);
// Right-hand sides solved during the factorisation: B <- U^{-T} B (outer panel s of B is
// solved as soon as panel s of U is final, on ctx->srhs beside the trailing updates).
// lower_rhs: B is lower triangular (identity), outer block s touches columns < (s+1) nb2.
struct RhsSpec {
  double* B;
  int nrhs;
  int ldb;
  int lower_rhs;
  int mode;  // 1: own stream (srhs) beside the trailing updates; 2: main stream after each SYRK
  // optional: gram (ldg) = B^T B -- K^{-1} = Z^T Z when B is the identity: gram tile tasks
  // of the tile-DAG launch (all of it), or accumulated panel by panel by the blocked path
  // (X_s^T X_s of each solved panel, upper; potrf_core zeroes it first; the caller mirrors)
  double* gram;
  int ldg;
};
// one-launch tile-DAG factorisation (+ B <- U^{-T} B); 1 = shape not eligible, 0 = launched
// DAG_GRAM (with DAG_LOWER, B = the identity's Z = U^{-T}): also G = Z^T Z (every tile)
// DAG_MIRROR: A holds only its upper triangle and 128 x 128 diagonal blocks (the upper-only
// K assembly): every off-diagonal task also stores its loaded tile A_ij, transposed, into the
// strict lower tile (j, i)
enum { DAG_SOLVE = 1, DAG_LOWER = 2, DAG_GRAM = 4, DAG_MIRROR = 8 };
int launch_potrf_dag(gpr_ctx* ctx, double* dA, int n, int lda, double* dB, int nrhs, int ldb,
                     int kglob, hipStream_t st, int flags = 0, double* dG = nullptr, int ldg = 0);
// true when potrf_core would factor (n, lda, dA) as ONE tile-DAG launch (directly, or for
// other shapes on a padded copy); dag_shape_ok: the launch takes the shape directly
bool dag_takes_whole(const gpr_ctx* ctx, int n, int lda, const double* dA);
bool dag_shape_ok(int n, int lda, const double* dA);
int launch_potrf_dag_batch(gpr_ctx* ctx, double* dA, size_t strA, int n, int lda, double* dB,
                           size_t strB, int nrhs, int ldb, int nbatch, int* info_out);
int launch_potrf_dag_padded(gpr_ctx* ctx, double* dA, int n, int lda, double* dB, int nrhs,
                            int ldb);
int potrf_core(gpr_ctx* ctx, double* dA, int n, int lda, int* info,
               const RhsSpec* rhs = nullptr);
int ensure_factor_inverses(gpr_ctx* ctx, const double* dU, int n, int ldu);
int trsm_ut_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs,
                 int ldb, double* norm_out, int lower_rhs);
int kinv_from_z(gpr_ctx* ctx, const double* Z, int n, double* dKinv, int ldk);
// symmetric eigendecomposition A = P diag(lam) P^T applied to B: lam (n, device) and
// B <- P^T B (n x m, ld ldb), A read only; *sweeps may be null.  method 0: tridiagonal
// reduction + divide and conquer (tridiag.hip, dstedc.hip) where n fits them, else block
// Jacobi (eigen.hip); 2: block Jacobi, whose floor >= 0 asks for the eigenvalues of A + floor I
// to high relative accuracy (what (lam + s)^-1 needs for every s >= floor; 0 = those of A)
int sym_eig_apply(gpr_ctx* ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                  double* dlam, int* sweeps, double floor, int method);
// dstedc.hip: T = tridiag(e, d, e) = Z diag(lam) Z^T, C <- Z^T C; n <= 6144 (tridiag_eig_ok)
int tridiag_eig_apply(gpr_ctx* ctx, const double* dd, const double* de, int n, double* dC, int m,
                      int ldc, double* dlam);
bool tridiag_eig_ok(int n);
// tridiag.hip: A = Q T Q^T (d, e on the device; B <- Q^T B when m > 0), one persistent launch
// (+ blocked WY back-transform for m > 1024); n <= 6144 (sym_tridiag_ok).  Workspace ctx->deig.
int sym_tridiag(gpr_ctx* ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                double* dd, double* de);
bool sym_tridiag_ok(int n);
// the quadrature's columns from T: out[2j] = C[:, j]' (T + s_j I)^{-1} c, out[2j+1] = k2 - c' (T +
// s_j I)^{-1} c with c = C[:, ny]; scr: 4 n quad_tridiag_chunk(n, ny) doubles
int quad_tridiag_chunk(int n, int ny);
int quad_tridiag_solves(gpr_ctx* ctx, const double* dd, const double* de, int n, const double* C,
                        int ldc, int ny, const double* dnoise, double k2, double* scr, double* out);
// norm[j] -= ||B[:, j]||^2 (one wave per column, deterministic), on ctx->stream
int launch_colnorm_sub(gpr_ctx* ctx, const double* dB, int ldb, int n, int ncols, double* norm);
// forward = false: only the backward sweep U x = B (B already holds U^{-T} b);
// backward = false: only the forward sweep U^T z = B
int potrs_core(gpr_ctx* ctx, const double* dU, int n, int ldu, double* dB, int nrhs, int ldb,
               bool forward = true, bool backward = true);
