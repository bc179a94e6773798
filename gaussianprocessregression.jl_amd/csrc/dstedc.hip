// Divide-and-conquer eigensolver of a symmetric tridiagonal T (LAPACK dstedc's algorithm:
// Cuppen's tearing, dlaed2's deflation, dlaed4's secular equation, dlaed3's Gu-Eisenstat
// vectors), hand-written for gfx950 -- the second stage of gpr_syev_apply (LAPACK.syevr! at
// src/integrate.jl:75).  The quadrature needs lambda and P^T B only, so the eigenvector matrix
// Z of T is never formed: every node of the recursion carries Z_node^T applied to its rows of
// [C | e_first | e_last] -- C = Q^T B from the reduction, and the node's first and last
// eigenvector rows, which are all a parent merge needs (z = [last row of Z_L; s first row of
// Z_R]).  A merge D + rho z z^T = U Lambda U^T then maps its rows by U^T (after deflation):
//   Z_node^T [C | f | l] = U^T G^T [Z_L^T [C | f | 0]; Z_R^T [C | 0 | l]]
// with G the deflation's Givens rotations.  Cost per merge of size k with K undeflated roots:
// O(k log k) sort, O(k) deflation scan, O(K^2) secular roots / Gu-Eisenstat / norms, and
// 2 K^2 (m + 2) flops for U^T (m columns of C) instead of the k^3 of forming Z.
//
// Tree: balanced halves down to 1 x 1 leaves (leaf i: d_i - |e_{i-1}| - |e_i|, every adjacent
// pair torn once); all merges of one depth run in the same launches (one workgroup per merge
// for the sort and scan; one wave per root / row for the K^2 parts; tiles of 64 roots x 64
// columns for U^T).  Node outputs are not sorted (undeflated roots ascending, then the
// deflated values); the parent sorts its k values first.  n <= 16384: a merge's sort runs in
// LDS up to 8192 values (12 bytes each), in global memory above (the top merge only).
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace {

constexpr int DC_MAXN = 16384;
constexpr int DC_LDS_SORT = 8192;  // merges of more values sort in global memory
constexpr int DC_SORT_THREADS = 1024;
constexpr double DC_EPS = 2.220446049250313e-16;

struct DcLevel {
  int nmerge;
  const int* ma;   // merge t: rows [ma, mb), split mm
  const int* mm;
  const int* mb;
  const int* rowm; // row -> merge id at this level, -1 if the row is not in a merge
  const int* tiles;// apply tiles: {merge, j0, c0} triples
  int ntiles;
};

struct DcArgs {
  int n, mx;       // rows, columns of X (m + 2: C, first, last)
  double* X;       // n x mx, ld ldx
  double* Xt;      // n x mx scratch, ld ldx
  size_t ldx;
  const double* e; // off-diagonal of T (n - 1)
  double* lam;     // current eigenvalue of each row
  double* lamnew;
  // per row position in its merge's range (scratch)
  int* nd_row;     // undeflated t: X row
  double* nd_d;
  double* nd_z;
  int* df_row;     // output position p >= K: deflated X row
  int* org;        // root j: origin pole index (into nd_d)
  double* tau;     // root j: lambda_j = nd_d[org] + tau
  double* zhat;
  double* nrm;
  int* rr1;        // rotations
  int* rr2;
  double* rc;
  double* rs;
  int* K;          // per merge
  int* nrot;
  double* rho2;    // per merge: 2 |beta|
  int delay;       // (test build) GPR_DC_DELAY: late-wave injection, see DC_DELAY
};

// Late-wave injection (test build only, GPR_DC_DELAY = d > 0): one wave in three (rotating with
// the site and the workgroup) sleeps d x ~8k cycles before reads that follow other waves' LDS or
// global writes, so a missing barrier shows as a wrong result (as tridiag.hip's TRD_DELAY).
#ifdef GPR_TESTING
#define DC_DELAY(site)                                                                  \
  do {                                                                                  \
    if (a.delay > 0 && ((int)blockIdx.x + (int)(threadIdx.x >> 6) + (site)) % 3 == 0)   \
      for (int q_ = 0; q_ < a.delay; ++q_) __builtin_amdgcn_s_sleep(127);              \
  } while (0)
#else
#define DC_DELAY(site) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ double dwave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double dwave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double dwave_prod(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v *= __shfl_xor(v, o);
  return v;
}

// leaves: lam_i = d_i - |e_{i-1}| - |e_i|; X = [C | 1 | 1]
__global__ void dc_init_kernel(const double* __restrict__ d, const double* __restrict__ e, int n,
                               const double* __restrict__ C, size_t ldc, int m,
                               double* __restrict__ X, size_t ldx, double* __restrict__ lam) {
  const size_t tot = (size_t)n * (m + 2);
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % n), c = (int)(t / n);
    X[(size_t)i + (size_t)c * ldx] = c < m ? C[(size_t)i + (size_t)c * ldc] : 1.0;
    if (c == 0) {
      double v = d[i];
      if (i > 0) v -= fabs(e[i - 1]);
      if (i < n - 1) v -= fabs(e[i]);
      lam[i] = v;
    }
  }
}

// K1: gather d and z, fix the first / last columns, sort by d, tolerance, deflation scan
// (dlaed2), one workgroup per merge.  key[kp], idx[kp] (int) in LDS, or (GSORT: kp >
// DC_LDS_SORT) in global scratch gkey / gidx (kp per merge); z in zhat's rows of the merge
// (free until dc_zhat_kernel).  Global scratch is read only by the workgroup that wrote it, after
// a barrier.
template <bool GSORT>
__global__ __launch_bounds__(DC_SORT_THREADS) void dc_prep_kernel(DcArgs a, DcLevel L, int kp,
                                                                  double* gkey, int* gidx) {
  extern __shared__ double sm[];
  const int t = blockIdx.x;
  const int lo = L.ma[t], mid = L.mm[t], hi = L.mb[t];
  const int k = hi - lo, k1 = mid - lo;
  double* key = GSORT ? gkey + (size_t)t * kp : sm;
  int* idx = GSORT ? gidx + (size_t)t * kp : reinterpret_cast<int*>(key + kp);
  double* zz = a.zhat + lo;
  __shared__ double red[2][DC_SORT_THREADS / 64];
  const double beta = a.e[mid - 1];
  const double sgn = beta >= 0.0 ? 1.0 : -1.0;
  const double rho = 2.0 * fabs(beta);
  const int tid = threadIdx.x;
  const double* colf = a.X + (size_t)(a.mx - 2) * a.ldx;
  const double* coll = a.X + (size_t)(a.mx - 1) * a.ldx;
  double dmax = 0.0, zmax = 0.0;
  for (int i = tid; i < kp; i += DC_SORT_THREADS) {
    if (i < k) {
      const int row = lo + i;
      const double dv = a.lam[row];
      // z = [last rows of Z_L; s * first rows of Z_R] / sqrt(2) (|z| = 1), rho -> 2 |beta|
      const double zv = (i < k1 ? coll[row] : sgn * colf[row]) * 0.70710678118654752440;
      key[i] = dv;
      idx[i] = i;
      zz[i] = zv;
      dmax = fmax(dmax, fabs(dv));
      zmax = fmax(zmax, fabs(zv));
    } else {
      key[i] = INFINITY;
      idx[i] = i;
    }
  }
  __syncthreads();
  // the node's own first / last columns: [f_L; 0] and [0; l_R]
  for (int i = tid; i < k; i += DC_SORT_THREADS) {
    const int row = lo + i;
    if (i >= k1) a.X[row + (size_t)(a.mx - 2) * a.ldx] = 0.0;
    else a.X[row + (size_t)(a.mx - 1) * a.ldx] = 0.0;
  }
  dmax = dwave_max(dmax);
  zmax = dwave_max(zmax);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = dmax;
    red[1][tid >> 6] = zmax;
  }
  // bitonic sort of (key, idx) ascending
  for (int size = 2; size <= kp; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      DC_DELAY(size + stride);  // (a late wave of the previous stage's exchanges)
      for (int i = tid; i < kp / 2; i += DC_SORT_THREADS) {
        const int lo_i = 2 * i - (i & (stride - 1));
        const int hi_i = lo_i + stride;
        const bool up = (lo_i & size) == 0;
        const double k0 = key[lo_i], k1v = key[hi_i];
        if ((k0 > k1v) == up) {
          key[lo_i] = k1v;
          key[hi_i] = k0;
          const int x = idx[lo_i];
          idx[lo_i] = idx[hi_i];
          idx[hi_i] = x;
        }
      }
    }
  DC_DELAY(1);
  __syncthreads();
  if (tid == 0) {
    double dm = 0.0, zm = 0.0;
    for (int q = 0; q < DC_SORT_THREADS / 64; ++q) {
      dm = fmax(dm, red[0][q]);
      zm = fmax(zm, red[1][q]);
    }
    const double tol = 8.0 * DC_EPS * fmax(dm, zm);
    // dlaed2's scan over the sorted values: small z deflates; a pending candidate and the next
    // value close enough (|t c s| <= tol) deflate the candidate by a rotation into the next
    int K = 0, nd = 0, nr = 0;
    int pj = -1;
    double pd = 0.0, pz = 0.0;
    for (int p = 0; p < k; ++p) {
      const int li = idx[p];
      const double dv = key[p], zv = zz[li];
      if (rho * fabs(zv) <= tol) {
        a.df_row[hi - 1 - nd] = lo + li;
        a.lamnew[hi - 1 - nd] = dv;
        ++nd;
        continue;
      }
      if (pj < 0) {
        pj = li;
        pd = dv;
        pz = zv;
        continue;
      }
      const double tau = hypot(zv, pz);
      const double tt = dv - pd;
      const double c = zv / tau, s = -pz / tau;
      if (fabs(tt * c * s) <= tol) {
        a.rr1[lo + nr] = lo + pj;
        a.rr2[lo + nr] = lo + li;
        a.rc[lo + nr] = c;
        a.rs[lo + nr] = s;
        ++nr;
        a.df_row[hi - 1 - nd] = lo + pj;
        a.lamnew[hi - 1 - nd] = pd * c * c + dv * s * s;
        ++nd;
        pd = pd * s * s + dv * c * c;
        pz = tau;
        pj = li;
      } else {
        a.nd_row[lo + K] = lo + pj;
        a.nd_d[lo + K] = pd;
        a.nd_z[lo + K] = pz;
        ++K;
        pj = li;
        pd = dv;
        pz = zv;
      }
    }
    if (pj >= 0) {
      a.nd_row[lo + K] = lo + pj;
      a.nd_d[lo + K] = pd;
      a.nd_z[lo + K] = pz;
      ++K;
    }
    a.K[t] = K;
    a.nrot[t] = nr;
    a.rho2[t] = rho;
  }
}

// K1b: the deflation rotations on X's rows, in order, one thread per column of a merge:
// x1' = c x1 + s x2, x2' = c x2 - s x1 (dlaed2's DROT); a chain of rotations through the same
// row keeps it in a register
__global__ void dc_rot_kernel(DcArgs a, DcLevel L) {
  const int t = blockIdx.y;
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= a.mx) return;
  const int lo = L.ma[t];
  const int nr = a.nrot[t];
  double* X = a.X + (size_t)col * a.ldx;
  int cur = -1;
  double cv = 0.0;
  for (int q = 0; q < nr; ++q) {
    const int r1 = a.rr1[lo + q], r2 = a.rr2[lo + q];
    const double c = a.rc[lo + q], s = a.rs[lo + q];
    const double x1 = r1 == cur ? cv : X[r1];
    const double x2 = X[r2];
    X[r1] = c * x1 + s * x2;
    cv = c * x2 - s * x1;
    cur = r2;
    const int nxt = q + 1 < nr ? a.rr1[lo + q + 1] : -1;
    if (nxt != r2) {
      X[r2] = cv;
      cur = -1;
    }
  }
}

// K2: root j of its merge's secular equation 1/rho + sum z_i^2 / (d_i - lambda) = 0 (rho > 0,
// d ascending): lambda_j = d_o + tau with o the closer end of its interval, tau by a
// bracketed "middle way" iteration (two-pole rational model matching value and slope),
// bisection when a step leaves the bracket.  One wave per root.
__global__ __launch_bounds__(256) void dc_secular_kernel(DcArgs a, DcLevel L) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.n) return;
  const int t = L.rowm[row];
  if (t < 0) return;
  const int lo = L.ma[t];
  const int K = a.K[t];
  const int j = row - lo;
  if (j >= K) return;
  const double* dl = a.nd_d + lo;
  const double* z = a.nd_z + lo;
  const double rho = a.rho2[t], rinv = 1.0 / rho;
  if (K == 1) {
    if (lane == 0) {
      a.org[row] = 0;
      a.tau[row] = rho * z[0] * z[0];
      a.lamnew[row] = dl[0] + rho * z[0] * z[0];
    }
    return;
  }
  // f(tau) pieces relative to origin o: delta_i = (dl_i - dl_o) - tau
  auto eval = [&](int o, double tau, int split, double* psi, double* dpsi, double* phi,
                  double* dphi, double* asum) {
    double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0, s = 0.0;
    const double dlo = dl[o];
    for (int i = lane; i < K; i += 64) {
      const double del = (dl[i] - dlo) - tau;
      const double zi2 = z[i] * z[i];
      const double tt = zi2 / del;
      if (i <= split) {
        p0 += tt;
        p1 += tt / del;
      } else {
        q0 += tt;
        q1 += tt / del;
      }
      s += fabs(tt);
    }
    *psi = dwave_sum(p0);
    *dpsi = dwave_sum(p1);
    *phi = dwave_sum(q0);
    *dphi = dwave_sum(q1);
    *asum = dwave_sum(s);
  };
  int o;
  double lo_t, hi_t, tau;
  double ps, dps, ph, dph, as;
  if (j < K - 1) {
    const double del = dl[j + 1] - dl[j];
    eval(j, 0.5 * del, j, &ps, &dps, &ph, &dph, &as);
    if (rinv + ps + ph >= 0.0) {  // root in (d_j, mid]
      o = j;
      lo_t = 0.0;
      hi_t = 0.5 * del;
    } else {
      o = j + 1;
      lo_t = -0.5 * del;
      hi_t = 0.0;
    }
    tau = 0.5 * (lo_t + hi_t);
  } else {
    o = K - 1;
    double zs = 0.0;
    for (int i = lane; i < K; i += 64) zs += z[i] * z[i];
    zs = dwave_sum(zs);
    lo_t = 0.0;
    hi_t = rho * zs;
    tau = 0.5 * hi_t;
  }
  const double dlo = dl[o];
  const double dL = dl[j] - dlo;                              // left pole (tau coordinates)
  const double dR = j < K - 1 ? dl[j + 1] - dlo : INFINITY;   // right pole
  for (int it = 0; it < 120; ++it) {
    eval(o, tau, j, &ps, &dps, &ph, &dph, &as);
    const double f = rinv + ps + ph;
    const double tolf = DC_EPS * (8.0 * as + 2.0 * rinv + 3.0 * fabs(tau) * (dps + dph));
    if (fabs(f) <= tolf) break;
    if (f < 0.0) lo_t = tau;
    else hi_t = tau;
    if (hi_t - lo_t <= 2.0 * DC_EPS * fmax(fabs(lo_t), fabs(hi_t))) break;
    const double DL = dL - tau, DR = dR - tau;  // DL < 0 < DR
    const double b1 = dps * DL * DL, a1 = ps - b1 / DL;
    double u;
    bool ok = true;
    if (j < K - 1) {
      const double b2 = dph * DR * DR, a2 = ph - b2 / DR;
      const double c = rinv + a1 + a2;
      const double B = c * (DL + DR) + b1 + b2;
      const double C0 = f * DL * DR;
      if (c == 0.0) {
        u = B != 0.0 ? C0 / B : 0.0;
      } else {
        const double disc = fmax(B * B - 4.0 * c * C0, 0.0);
        const double q = 0.5 * (B + copysign(sqrt(disc), B));
        const double u1 = q / c, u2 = q != 0.0 ? C0 / q : 0.0;
        u = (u2 > DL && u2 < DR) ? u2 : u1;
      }
    } else {
      const double c = rinv + a1 + ph;
      ok = c > 0.0;
      u = ok ? DL + b1 / c : 0.0;
    }
    double tn = tau + u;
    if (!ok || !(tn > lo_t && tn < hi_t)) tn = 0.5 * (lo_t + hi_t);
    if (tn == tau) break;
    tau = tn;
  }
  if (lane == 0) {
    a.org[row] = o;
    a.tau[row] = tau;
    a.lamnew[row] = dlo + tau;
  }
}

// delta_j(i) = d_i - lambda_j, accurately: (d_i - d_{o_j}) - tau_j
__device__ __forceinline__ double dc_delta(const double* dl, const int* org, const double* tau,
                                           int i, int j) {
  return (dl[i] - dl[org[j]]) - tau[j];
}

// K3: Gu-Eisenstat zhat_i = sign(z_i) sqrt(|prod_j delta_j(i) / prod_{j != i} (d_i - d_j)|)
// (dlaed3), one wave per i
__global__ __launch_bounds__(256) void dc_zhat_kernel(DcArgs a, DcLevel L) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.n) return;
  const int t = L.rowm[row];
  if (t < 0) return;
  const int lo = L.ma[t], K = a.K[t], i = row - lo;
  if (i >= K) return;
  const double* dl = a.nd_d + lo;
  const int* org = a.org + lo;
  const double* tau = a.tau + lo;
  double p = 1.0;
  for (int j = lane; j < K; j += 64) {
    const double del = dc_delta(dl, org, tau, i, j);
    p *= j == i ? del : del / (dl[i] - dl[j]);
  }
  p = dwave_prod(p);
  if (lane == 0) a.zhat[row] = copysign(sqrt(fabs(p)), a.nd_z[row]);
}

// K4: norm of eigenvector j, (sum_i (zhat_i / delta_j(i))^2)^(1/2), one wave per j
__global__ __launch_bounds__(256) void dc_norm_kernel(DcArgs a, DcLevel L) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.n) return;
  const int t = L.rowm[row];
  if (t < 0) return;
  const int lo = L.ma[t], K = a.K[t], j = row - lo;
  if (j >= K) return;
  const double* dl = a.nd_d + lo;
  const int* org = a.org + lo;
  const double* tau = a.tau + lo;
  const double* zh = a.zhat + lo;
  double s = 0.0;
  for (int i = lane; i < K; i += 64) {
    const double u = zh[i] / dc_delta(dl, org, tau, i, j);
    s += u * u;
  }
  s = dwave_sum(s);
  if (lane == 0) a.nrm[row] = 1.0 / sqrt(s);
}

// K5: output rows [lo, hi) of a merge into Xt: root j < K: sum_i U(i, j) X(nd_row_i, :) with
// U(i, j) = zhat_i / delta_j(i) / |.|_j; position p >= K: the deflated row df_row[p].
// Tile: 64 output rows x 64 columns per 256-thread workgroup (4 x 4 per thread), i in LDS
// chunks of 16.
__global__ __launch_bounds__(256) void dc_apply_kernel(DcArgs a, DcLevel L) {
  __shared__ double Us[16][65];
  __shared__ double Xs[16][65];
  const int t = L.tiles[3 * blockIdx.x], j0 = L.tiles[3 * blockIdx.x + 1],
            c0 = L.tiles[3 * blockIdx.x + 2];
  const int lo = L.ma[t], hi = L.mb[t], K = a.K[t];
  const int k = hi - lo;
  const int tid = threadIdx.x;
  const int tj = tid & 15, tc = tid >> 4;  // rows j0 + tj + 16 q, columns c0 + tc + 16 r
  double acc[4][4] = {};
  const double* dl = a.nd_d + lo;
  const int* org = a.org + lo;
  const double* tau = a.tau + lo;
  const double* zh = a.zhat + lo;
  const int jend = min(j0 + 64, K);
  if (j0 < K) {
    for (int i0 = 0; i0 < K; i0 += 16) {
      for (int e = tid; e < 16 * 64; e += 256) {
        const int ii = e >> 6, q = e & 63;
        const int i = i0 + ii;
        const int jj = j0 + q, cc = c0 + q;
        Us[ii][q] = (i < K && jj < jend) ? zh[i] / dc_delta(dl, org, tau, i, jj) * a.nrm[lo + jj] : 0.0;
        Xs[ii][q] = (i < K && cc < a.mx) ? a.X[(size_t)a.nd_row[lo + i] + (size_t)cc * a.ldx] : 0.0;
      }
      DC_DELAY(i0);  // (a late writer of the staged U / X chunk)
      __syncthreads();
#pragma unroll 4
      for (int ii = 0; ii < 16; ++ii) {
        double u[4], x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          u[q] = Us[ii][tj + 16 * q];
          x[q] = Xs[ii][tc + 16 * q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[q][r] = fma(u[q], x[r], acc[q][r]);
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int jj = j0 + tj + 16 * q;
    if (jj >= k) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cc = c0 + tc + 16 * r;
      if (cc >= a.mx) continue;
      const double v = jj < K ? acc[q][r] : a.X[(size_t)a.df_row[lo + jj] + (size_t)cc * a.ldx];
      a.Xt[(size_t)(lo + jj) + (size_t)cc * a.ldx] = v;
    }
  }
}

// K6: the merged rows back into X, their eigenvalues into lam
__global__ void dc_copyback_kernel(DcArgs a, DcLevel L) {
  const size_t tot = (size_t)a.n * a.mx;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot;
       e += (size_t)gridDim.x * blockDim.x) {
    const int row = (int)(e % a.n), c = (int)(e / a.n);
    if (L.rowm[row] < 0) continue;
    a.X[(size_t)row + (size_t)c * a.ldx] = a.Xt[(size_t)row + (size_t)c * a.ldx];
    if (c == 0) a.lam[row] = a.lamnew[row];
  }
}

__global__ void dc_out_kernel(const double* __restrict__ X, size_t ldx, int n, int m,
                              double* __restrict__ C, size_t ldc) {
  const size_t tot = (size_t)n * m;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot;
       e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % n), c = (int)(e / n);
    C[(size_t)i + (size_t)c * ldc] = X[(size_t)i + (size_t)c * ldx];
  }
}

struct Node {
  int a, m, b, depth;
};

void build_tree(int a, int b, int depth, std::vector<Node>& out, int* maxdepth) {
  if (b - a < 2) return;
  const int m = a + (b - a) / 2;
  out.push_back({a, m, b, depth});
  *maxdepth = std::max(*maxdepth, depth);
  build_tree(a, m, depth + 1, out, maxdepth);
  build_tree(m, b, depth + 1, out, maxdepth);
}

}  // namespace

bool tridiag_eig_ok(int n) { return n >= 1 && n <= DC_MAXN; }

// T = tridiag(e, d, e) (device d[n], e[n-1]) = Z diag(lam) Z^T: lam[n] (device; order: the
// root merge's output, not sorted) and C <- Z^T C (n x m, ld ldc; m >= 0)
int tridiag_eig_apply(gpr_ctx* ctx, const double* dd, const double* de, int n, double* dC, int m,
                      int ldc, double* dlam) {
  if (n <= 0) return 0;
  if (n > DC_MAXN) return set_err(ctx, GPR_E_UNSUP, "tridiagonal eigensolver: n = %d > %d", n, DC_MAXN);
  hipStream_t st = ctx->stream;
  const int mx = m + 2;
  const size_t ldx = (size_t)(n + 1) / 2 * 2;
  // tree and per-depth merge lists (host)
  std::vector<Node> nodes;
  int maxd = -1;
  build_tree(0, n, 0, nodes, &maxd);
  std::vector<std::vector<int>> byd(maxd + 1);
  for (int q = 0; q < (int)nodes.size(); ++q) byd[nodes[q].depth].push_back(q);
  // device tables: per depth: ma, mm, mb (nmerge each), rowm (n), tiles (3 per tile)
  std::vector<int> tab;
  struct LvlOff {
    size_t ma, mm, mb, rowm, tiles;
    int nmerge, ntiles, kmax;
  };
  std::vector<LvlOff> off(maxd + 1);
  for (int dpt = maxd; dpt >= 0; --dpt) {
    LvlOff& o = off[dpt];
    const auto& ids = byd[dpt];
    o.nmerge = (int)ids.size();
    o.kmax = 0;
    o.ma = tab.size();
    for (int q : ids) tab.push_back(nodes[q].a);
    o.mm = tab.size();
    for (int q : ids) tab.push_back(nodes[q].m);
    o.mb = tab.size();
    for (int q : ids) tab.push_back(nodes[q].b);
    o.rowm = tab.size();
    tab.resize(tab.size() + n, -1);
    for (int t = 0; t < (int)ids.size(); ++t) {
      const Node& nd = nodes[ids[t]];
      o.kmax = std::max(o.kmax, nd.b - nd.a);
      for (int r = nd.a; r < nd.b; ++r) tab[o.rowm + r] = t;
    }
    o.tiles = tab.size();
    o.ntiles = 0;
    for (int t = 0; t < (int)ids.size(); ++t) {
      const Node& nd = nodes[ids[t]];
      for (int j0 = 0; j0 < nd.b - nd.a; j0 += 64)
        for (int c0 = 0; c0 < mx; c0 += 64) {
          tab.push_back(t);
          tab.push_back(j0);
          tab.push_back(c0);
          ++o.ntiles;
        }
    }
  }
  // workspace (doubles): X, Xt, lam-new, 9 n-vectors, per-merge K/nrot/rho2, the tables
  const size_t nX = ldx * mx;
  const size_t nvec = 16 * (size_t)n + 3 * (size_t)nodes.size() + 64;
  const size_t ntab = (tab.size() + 1) / 2 + 1;
  // global sort scratch for the merges beyond the LDS sort (kp values: a double and an int each)
  size_t gsort_cap = 0;
  for (int dpt = 0; dpt <= maxd; ++dpt) {
    int kp = 2;
    while (kp < off[dpt].kmax) kp <<= 1;
    if (kp > DC_LDS_SORT) gsort_cap = std::max(gsort_cap, (size_t)off[dpt].nmerge * kp);
  }
  GPR_TRY(ensure_buf(ctx, &ctx->ddc, &ctx->dc_cap, 2 * nX + nvec + ntab + gsort_cap + (gsort_cap + 1) / 2));
  double* X = ctx->ddc;
  double* Xt = X + nX;
  double* v = Xt + nX;
  DcArgs a{};
  a.n = n;
  a.mx = mx;
  a.X = X;
  a.Xt = Xt;
  a.ldx = ldx;
  a.e = de;
  a.lam = dlam;
  a.lamnew = v;
  a.nd_d = v + n;
  a.nd_z = v + 2 * (size_t)n;
  a.tau = v + 3 * (size_t)n;
  a.zhat = v + 4 * (size_t)n;
  a.nrm = v + 5 * (size_t)n;
  a.rc = v + 6 * (size_t)n;
  a.rs = v + 7 * (size_t)n;
  a.rho2 = v + 8 * (size_t)n;                      // (nodes.size() <= n)
  int* iv = reinterpret_cast<int*>(v + 9 * (size_t)n);
  a.nd_row = iv;
  a.df_row = iv + n;
  a.org = iv + 2 * (size_t)n;
  a.rr1 = iv + 3 * (size_t)n;
  a.rr2 = iv + 4 * (size_t)n;
  a.K = iv + 5 * (size_t)n;
  a.nrot = iv + 6 * (size_t)n;
  int* dtab = reinterpret_cast<int*>(v + nvec);
  double* gkey = v + nvec + ntab;
  int* gidx = reinterpret_cast<int*>(gkey + gsort_cap);
  // the tables go up from a context-owned pinned buffer (the call returns with the copy still
  // queued): the previous call's upload must have read it before it is refilled
  if (ctx->dc_tab_ev) HIP_TRY(ctx, hipEventSynchronize(ctx->dc_tab_ev));
  else HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->dc_tab_ev, hipEventDisableTiming));
  if (ctx->dc_tab_host_cap < tab.size()) {
    if (ctx->dc_tab_host) HIP_TRY(ctx, hipHostFree(ctx->dc_tab_host));
    ctx->dc_tab_host = nullptr;
    ctx->dc_tab_host_cap = 0;
    HIP_TRY(ctx, hipHostMalloc((void**)&ctx->dc_tab_host, tab.size() * sizeof(int)));
    ctx->dc_tab_host_cap = tab.size();
  }
  if (!tab.empty()) {
    std::copy(tab.begin(), tab.end(), ctx->dc_tab_host);
    HIP_TRY(ctx, hipMemcpyAsync(dtab, ctx->dc_tab_host, tab.size() * sizeof(int),
                                hipMemcpyHostToDevice, st));
    HIP_TRY(ctx, hipEventRecord(ctx->dc_tab_ev, st));
  }
#ifdef GPR_TESTING
  a.delay = getenv("GPR_DC_DELAY") ? std::max(0, atoi(getenv("GPR_DC_DELAY"))) : 0;
#endif
  TimerScope ts(ctx, TC_OTHER, 0.0);
  dc_init_kernel<<<512, 256, 0, st>>>(dd, de, n, dC, (size_t)ldc, m, X, ldx, dlam);
  LAUNCH_CHECK(ctx);
  for (int dpt = maxd; dpt >= 0; --dpt) {
    const LvlOff& o = off[dpt];
    if (!o.nmerge) continue;
    DcLevel L{};
    L.nmerge = o.nmerge;
    L.ma = dtab + o.ma;
    L.mm = dtab + o.mm;
    L.mb = dtab + o.mb;
    L.rowm = dtab + o.rowm;
    L.tiles = dtab + o.tiles;
    L.ntiles = o.ntiles;
    int kp = 2;
    while (kp < o.kmax) kp <<= 1;
    if (kp <= DC_LDS_SORT) {
      const size_t sh = (size_t)kp * (sizeof(double) + sizeof(int));
      dc_prep_kernel<false><<<o.nmerge, DC_SORT_THREADS, sh, st>>>(a, L, kp, nullptr, nullptr);
    } else {
      if ((size_t)o.nmerge * kp > gsort_cap)
        return set_err(ctx, GPR_E_HIP, "divide and conquer: sort scratch too small");
      dc_prep_kernel<true><<<o.nmerge, DC_SORT_THREADS, 0, st>>>(a, L, kp, gkey, gidx);
    }
    LAUNCH_CHECK(ctx);
    dc_rot_kernel<<<dim3((mx + 63) / 64, o.nmerge), 64, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
    const int wgs = (n + 3) / 4;
    dc_secular_kernel<<<wgs, 256, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
    dc_zhat_kernel<<<wgs, 256, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
    dc_norm_kernel<<<wgs, 256, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
    dc_apply_kernel<<<o.ntiles, 256, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
    dc_copyback_kernel<<<1024, 256, 0, st>>>(a, L);
    LAUNCH_CHECK(ctx);
  }
  if (m > 0) {
    dc_out_kernel<<<512, 256, 0, st>>>(X, ldx, n, m, dC, (size_t)ldc);
    LAUNCH_CHECK(ctx);
  }
  return 0;
}
