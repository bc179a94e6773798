/* Threaded CPU restatement of the reference's MLL gradient loop -- the timed C4 CPU baseline.
 * TEST INFRASTRUCTURE ONLY (timed CPU baseline, checker).  Follows, per hyperparameter i:
 *   grad!(∇L, MLL, md, tc)           src/cost.jl:119-126   (loop over all D components)
 *   find_idx + grad!(SE, ∇K, i, ...) src/compose_covar.jl:109-123, src/deriv_covar.jl:20-29:
 *       i = sigma:  ∇K = (2/|sigma|) K_p        (K_p the part's cached matrix, eps included)
 *       i = l_k:    ∇K = -2 l_k K_p .* (x_k,a - x_k,b)^2   (raw x)
 *   grad(MLL, kchol, ∇K, α, K⁻¹, tt) src/loss_grad.jl:43-47:
 *       tt = ∇K α (dgemv); g = -0.5 (tt . α - <K⁻¹, ∇K>_F)
 *   WhiteNoise (UniformScaling)      src/loss_grad.jl:49-52, src/deriv_covar.jl:31-32:
 *       g = -0.5 (2 sigma_n) sum(α^2 - diag K⁻¹)
 * i.e. the reference's memory traffic: one ∇K write, one dgemv read and one Frobenius read of
 * ∇K (plus K_p and K⁻¹) per component -- not the GPU's fused single pass.  OpenMP threads over
 * columns (the reference's BLAS threads for dgemv / dot; its broadcast for ∇K).  All matrices
 * n x n column-major; x d x n column-major. */
#include <math.h>
#include <stddef.h>

/* one SE component: materialise ∇K into dK, then dgemv and the Frobenius dot */
static double se_component(int d, int n, const double* x, const double* Kp, double sigma,
                           const double* l, int i /* 0: sigma, k+1: l_k */,
                           const double* alpha, const double* Kinv, double* dK, double* tt) {
  /* ∇K (grad!(::SquaredExp, DK, i, hp, x, K), the N^2 write) */
#pragma omp parallel for schedule(static)
  for (int b = 0; b < n; ++b) {
    const double* kc = Kp + (size_t)b * n;
    double* g = dK + (size_t)b * n;
    if (i == 0) {
      const double f = 2.0 / fabs(sigma);
      for (int a = 0; a < n; ++a) g[a] = f * kc[a];
    } else {
      const int k = i - 1;
      const double f = -2.0 * l[k];
      const double xb = x[(size_t)b * d + k];
      for (int a = 0; a < n; ++a) {
        const double t = x[(size_t)a * d + k] - xb;
        g[a] = f * kc[a] * t * t;
      }
    }
  }
  /* tt = ∇K α (dgemv, column-major: row blocks per thread, columns streamed) */
#pragma omp parallel
  {
#pragma omp for schedule(static)
    for (int a0 = 0; a0 < n; a0 += 256) {
      const int a1 = a0 + 256 < n ? a0 + 256 : n;
      double acc[256];
      for (int a = a0; a < a1; ++a) acc[a - a0] = 0.0;
      for (int b = 0; b < n; ++b) {
        const double ab = alpha[b];
        const double* g = dK + (size_t)b * n;
        for (int a = a0; a < a1; ++a) acc[a - a0] += g[a] * ab;
      }
      for (int a = a0; a < a1; ++a) tt[a] = acc[a - a0];
    }
  }
  double dta = 0.0, frob = 0.0;
#pragma omp parallel for reduction(+ : dta) schedule(static)
  for (int a = 0; a < n; ++a) dta += tt[a] * alpha[a];
  /* <K⁻¹, ∇K>_F over the whole matrices (dot(K⁻¹, ∇K)) */
#pragma omp parallel for reduction(+ : frob) schedule(static)
  for (int b = 0; b < n; ++b) {
    const double* g = dK + (size_t)b * n;
    const double* q = Kinv + (size_t)b * n;
    double s = 0.0;
    for (int a = 0; a < n; ++a) s += q[a] * g[a];
    frob += s;
  }
  return -0.5 * (dta - frob);
}

/* g[D]: the reference's gradient of the negative log marginal likelihood for a composed kernel
 * of nse SquaredExp parts (Kp: nse matrices, part p at Kp + p n^2, eps included; sigma[p],
 * l[p d + k]) and, when has_noise, one WhiteNoise part (sigma_n) -- hp order = part order,
 * part_kind[q] (1 SE, 2 WN) for q < nparts.  dK, tt: scratch (n^2, n). */
void mll_grad_cpu(int d, int n, const double* x, int nparts, const int* part_kind,
                  const double* Kp, const double* sigma, const double* l, double sigma_n,
                  const double* alpha, const double* Kinv, double* dK, double* tt, double* g) {
  int off = 0, p = 0;
  for (int q = 0; q < nparts; ++q) {
    if (part_kind[q] == 1) {
      for (int i = 0; i <= d; ++i)
        g[off + i] = se_component(d, n, x, Kp + (size_t)p * n * n, sigma[p], l + (size_t)p * d,
                                  i, alpha, Kinv, dK, tt);
      off += d + 1;
      ++p;
    } else {
      double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
      for (int a = 0; a < n; ++a) s += alpha[a] * alpha[a] - Kinv[(size_t)a * n + a];
      g[off] = -0.5 * (2.0 * sigma_n) * s;
      off += 1;
    }
  }
}
