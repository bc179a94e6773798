/* Threaded CPU restatement of the composed SquaredExp kernel-matrix assembly.
 * TEST INFRASTRUCTURE ONLY (timed CPU baseline, checker): follows
 *   kernel_impl!(::SquaredExp)  src/covariance.jl:85-95  (xs = x .* l; D = sum (xs-xs')^2;
 *                                                          K = sigma^2 exp(-D))
 *   +eps per SE part on a same-object diagonal  src/covariance.jl:49-58
 *   composed sum + sigma_n^2                     src/compose_covar.jl:47-77
 * and the reference's threading (threaded_kernel_impl!, src/covariance.jl:97-118) with an
 * OpenMP loop over columns.  x is d x n, xp d x m (NULL = same object), K n x m, all
 * column-major. */
#include <math.h>
#include <stdlib.h>

static double* scale(int d, int n, const double* x, int nse, const double* l) {
  double* xs = (double*)malloc(sizeof(double) * (size_t)nse * d * n);
  for (int p = 0; p < nse; ++p)
    for (int a = 0; a < n; ++a)
      for (int k = 0; k < d; ++k) xs[((size_t)p * n + a) * d + k] = x[(size_t)a * d + k] * l[p * d + k];
  return xs;
}

void kbuild_cpu(int d, int n, const double* x, int m, const double* xp, int nse,
                const double* sigma, const double* l /* nse x d */, int has_noise,
                double noise2, double eps, double* K) {
  const int same = (xp == NULL);
  if (same) m = n;
  double* xs = scale(d, n, x, nse, l);
  double* xps = same ? xs : scale(d, m, xp, nse, l);
#pragma omp parallel for schedule(dynamic, 16)
  for (int b = 0; b < m; ++b) {
    for (int a = 0; a < n; ++a) {
      double v = 0.0;
      for (int p = 0; p < nse; ++p) {
        const double* xa = xs + ((size_t)p * n + a) * d;
        const double* xb = xps + ((size_t)p * m + b) * d;
        double D = 0.0;
        for (int k = 0; k < d; ++k) {
          const double t = xa[k] - xb[k];
          D += t * t;
        }
        double t = sigma[p] * sigma[p] * exp(-1.0 * D);
        if (same && a == b) t += eps;
        v = (p == 0) ? t : v + t;
      }
      if (same && a == b && has_noise) v += noise2;
      K[(size_t)a + (size_t)b * n] = v;
    }
  }
  if (!same) free(xps);
  free(xs);
}
