// Symmetric eigendecomposition applied to right-hand sides, hand-written for gfx950: the
// sample_noise branch of Bayesian quadrature (src/integrate.jl:71-100, LAPACK.syevr! at :75)
// needs lambda = eig(K) and P^T [Y | k1] only -- never P itself.
//
// Method: two-sided BLOCK Jacobi with a parallel (round-robin) ordering.  K (padded to a
// multiple of 64 with zero rows/columns, which stay decoupled) is split into 32-wide blocks;
// a round pairs every block with another (the circle method: nb - 1 rounds per sweep meet
// every pair once).  Per round:
//   1. one workgroup per pair (I, J) runs one sweep of scalar parallel Jacobi on its 64 x 64
//      subproblem S = K[I u J, I u J] in LDS (32 disjoint rotations per step, 63 steps;
//      GPR_EIG_INNER sweeps: 1, 2 and 8 measured 111 / 183 / 177 ms at n = 1100 with 13 outer
//      sweeps each, profiles/r04_eig_probe.txt), re-orthogonalises the accumulated rotation R
//      by one Newton-Schulz step (without it R's drift set the eigenvalue error: 3-9 n eps
//      |K|, orthogonality of P 300-15000 eps; with it 0.03-0.2 n eps |K| and 3-54 eps) and
//      writes it (64 x 64);
//   2. every 64 x 64 tile of K in pair coordinates becomes R_k^T K[P_k, P_l] R_l (computed for
//      k <= l and mirrored, so K stays exactly symmetric) and the pair's rows of B become
//      R_k^T B[P_k, :] -- all pairs' transforms at once, J^T K J with J = diag(R_k).
// A sweep that rotates nothing anywhere ends it: lambda = diag(K), B = P^T B_in.  Rotations
// follow Rutishauser's stable formulas and are skipped when |s_pq| <= 1e-15 sqrt((|s_pp| + f)
// (|s_qq| + f)) (the Demmel-Veselic criterion for K + f I: its eigenvalues to high relative
// accuracy -- f = 0 for K itself; the quadrature passes f = its smallest nonnegative shift,
// which is all (lambda + s)^-1 needs for every shift s >= f) or when the angle is below
// rounding (|tan| < 1e-17), so a converged matrix is left exactly as it is (R = I is applied
// exactly).
//
// Cost: per round one small latency-bound launch (nb/2 workgroups, 63 dependent steps: ~95 us,
// ~70 % of the time) and one pass over K (16 n^2 bytes, 2 x 64^3 FP64 MFMA per tile, ~38 us);
// nb - 1 rounds per sweep, 9-25 sweeps (n = 1100: 56 ms random, 110 ms SE kernel).
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace {

constexpr int EB = 32;        // Jacobi block width
constexpr int ES = 2 * EB;    // subproblem / tile edge
constexpr int ELD = ES + 1;   // LDS row stride (doubles) of a 64 x 64 image

// circle method over m slots (m even): round r pairs slot 0 with L[0] and L[i] with L[m-1-i],
// L = (1..m-1) rotated by r
__device__ __forceinline__ void circle_pair(int m, int r, int k, int* a, int* b) {
  const int mm = m - 1;
  auto L = [&](int i) { return (i + r) % mm + 1; };
  if (k == 0) {
    *a = 0;
    *b = L(0);
  } else {
    *a = L(k);
    *b = L(mm - k);
  }
}

// global index of pair-local row i (0..63) of pair (I, J)
__device__ __forceinline__ int pair_row(int I, int J, int i) {
  return i < EB ? EB * I + i : EB * J + (i - EB);
}

// thread t computes the 4 x 4 block rows 4 (t % 16).., columns 4 (t / 16).. of the 64 x 64
// product C = TA ? X^T Y : X Y  (X, Y in LDS, row stride ELD)
template <bool TA>
__device__ __forceinline__ void gemm64(const double* X, const double* Y, double (&c)[4][4]) {
  const int t = threadIdx.x, i0 = 4 * (t % 16), j0 = 4 * (t / 16);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) c[a][b] = 0.0;
  for (int kk = 0; kk < ES; ++kk) {
    double x[4], y[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) x[a] = TA ? X[kk + (i0 + a) * ELD] : X[(i0 + a) + kk * ELD];
#pragma unroll
    for (int b = 0; b < 4; ++b) y[b] = Y[kk + (j0 + b) * ELD];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) c[a][b] = fma(x[a], y[b], c[a][b]);
  }
}

typedef double ed4 __attribute__((ext_vector_type(4)));

// The same 64 x 64 product on the FP64 matrix cores: wave w owns the 32 x 32 quadrant rows
// 32 (w & 1).., columns 32 (w >> 1)..; v_mfma_f64_16x16x4f64 takes lane l's A[l & 15][l >> 4]
// and B[l >> 4][l & 15] and leaves C[(l >> 4) + 4 q][l & 15] in register q.  Written into Z
// (LDS, row stride ELD) -- Z may alias X or Y: the barrier before the stores orders them after
// every wave's last operand read.
template <bool TA>
__device__ __forceinline__ void gemm64_mfma(const double* X, const double* Y, double* Z) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = 32 * (w & 1), c0 = 32 * (w >> 1);
  ed4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = ed4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int ks = 0; ks < ES / 4; ++ks) {
    const int k = 4 * ks + (lane >> 4);
    double xa[2], yb[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int i = r0 + 16 * a + (lane & 15);
      xa[a] = TA ? X[k + i * ELD] : X[i + k * ELD];
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) yb[b] = Y[k + (c0 + 16 * b + (lane & 15)) * ELD];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a], yb[b], acc[a][b], 0, 0, 0);
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        Z[(r0 + 16 * a + (lane >> 4) + 4 * q) + (c0 + 16 * b + (lane & 15)) * ELD] = acc[a][b][q];
  __syncthreads();
}

// 1. per pair: diagonalise S = A[P, P] by parallel Jacobi in LDS, R = accumulated rotation.
//    MERGED (default; GPR_EIG_SUBK=0 selects the first form: two passes, 256 threads, rotations
//    skipped by branches): 1024 threads, one 2 x 2 block of S and two entries of R each; per
//    step the rotations from one division and two square roots, then S's two-sided update and
//    R's in one straight-line pass, one barrier each.  Same box, n = 1100: 165 -> 95 us per
//    launch (profiles/r04_eig_speed.txt)
template <bool MERGED, int NT>
__global__ __launch_bounds__(NT) void eig_subproblem_kernel(const double* __restrict__ A, size_t lda,
                                                            int nb, int round,
                                                            double* __restrict__ Rbuf,
                                                            int* __restrict__ rotations,
                                                            int max_inner, int reorth, double sig) {
  __shared__ double S[ES * ELD];
  __shared__ double R[ES * ELD];
  __shared__ double cs[ES / 2][2];
  __shared__ int pr[ES / 2][2];
  __shared__ int rot_sweep, rot_total;
  const int k = blockIdx.x, t = threadIdx.x;
  int I, J;
  circle_pair(nb, round, k, &I, &J);
  for (int e = t; e < ES * ES; e += NT) {
    const int i = e % ES, j = e / ES;
    S[i + j * ELD] = A[(size_t)pair_row(I, J, i) + (size_t)pair_row(I, J, j) * lda];
    R[i + j * ELD] = i == j ? 1.0 : 0.0;
  }
  if (t == 0) rot_total = 0;
  __syncthreads();
  if (MERGED) {
    // a pair none of whose off-diagonal entries passes the rotation test rotates nothing this
    // round (its S would stay exactly as it is): R = I, flag 0, no 63-step sweep -- in the
    // late sweeps most pairs
    bool need = false;
    for (int e = t; e < ES * ES; e += NT) {
      const int i = e % ES, j = e / ES;
      if (i < j) {
        const double apq = S[i + j * ELD];
        need |= apq != 0.0 &&
                apq * apq > 1e-30 * ((fabs(S[i + i * ELD]) + sig) * (fabs(S[j + j * ELD]) + sig));
      }
    }
    if (!__syncthreads_or(need)) {
      double* Rk = Rbuf + (size_t)k * ES * ES;
      for (int e = t; e < ES * ES; e += NT) Rk[e] = (e % ES) == (e / ES) ? 1.0 : 0.0;
      if (t == 0) rotations[2 + k] = 0;
      return;
    }
  }
  for (int sweep = 0; sweep < max_inner; ++sweep) {
    if (t == 0) rot_sweep = 0;
    __syncthreads();
    for (int step = 0; step < ES - 1; ++step) {
      if (MERGED) {
        // rotations: wave 0, lane t < 32 for pair t.  t = tan of the angle that zeroes s_pq,
        // Rutishauser's root sign(theta) / (|theta| + sqrt(1 + theta^2)), theta = (s_qq -
        // s_pp) / (2 s_pq), written with one division: |h| / (|d| + sqrt(d^2 + h^2)), d = s_qq -
        // s_pp, h = 2 s_pq; the skip test squared (no square root)
        if (t < 64) {
          bool rot = false;
          if (t < ES / 2) {
            int p, q;
            circle_pair(ES, step, t, &p, &q);
            if (p > q) { const int w = p; p = q; q = w; }
            const double app = S[p + p * ELD], aqq = S[q + q * ELD], apq = S[p + q * ELD];
            double c = 1.0, s = 0.0;
            if (apq != 0.0 && apq * apq > 1e-30 * ((fabs(app) + sig) * (fabs(aqq) + sig))) {
              const double d = aqq - app, h = 2.0 * apq;
              const bool pos = d == 0.0 || ((d > 0.0) == (h > 0.0));
              const double ah = pos ? fabs(h) : -fabs(h);
              const double tt = ah / (fabs(d) + sqrt(fma(d, d, h * h)));
              if (fabs(tt) >= 1e-17) {
                c = 1.0 / sqrt(fma(tt, tt, 1.0));
                s = tt * c;
                rot = true;
              }
            }
            cs[t][0] = c;
            cs[t][1] = s;
            pr[t][0] = p;
            pr[t][1] = q;
          }
          const unsigned long long m = __ballot(rot);
          if (t == 0 && m) rot_sweep += __popcll(m);
        }
        __syncthreads();
        // S <- J^T S J by 2 x 2 blocks (row pair a, column pair b: the row rotation, then the
        // column rotation of the row-rotated values) and R <- R J, straight-line: a pair that
        // did not rotate has c = 1, s = 0, which leaves every value exactly as it is
        const int b = t & 31;
        const double cb = cs[b][0], sb = cs[b][1];
        const int pb = pr[b][0], qb = pr[b][1];
#pragma unroll
        for (int u = 0; u < 1024 / NT; ++u) {
          const int a = (t >> 5) + (NT / 32) * u;
          const double ca = cs[a][0], sa = cs[a][1];
          const int pa = pr[a][0], qa = pr[a][1];
          const double x00 = S[pa + pb * ELD], x01 = S[pa + qb * ELD];
          const double x10 = S[qa + pb * ELD], x11 = S[qa + qb * ELD];
          const double y00 = ca * x00 - sa * x10, y10 = sa * x00 + ca * x10;
          const double y01 = ca * x01 - sa * x11, y11 = sa * x01 + ca * x11;
          S[pa + pb * ELD] = cb * y00 - sb * y01;
          S[pa + qb * ELD] = sb * y00 + cb * y01;
          S[qa + pb * ELD] = cb * y10 - sb * y11;
          S[qa + qb * ELD] = sb * y10 + cb * y11;
        }
        const int i = t & 63;
#pragma unroll
        for (int u = 0; u < 2048 / NT; ++u) {
          const int pk = (t >> 6) + (NT / 64) * u;
          const double c = cs[pk][0], s = cs[pk][1];
          const int p = pr[pk][0], q = pr[pk][1];
          const double rp = R[i + p * ELD], rq = R[i + q * ELD];
          R[i + p * ELD] = c * rp - s * rq;
          R[i + q * ELD] = s * rp + c * rq;
        }
        __syncthreads();
        continue;
      }
      if (t < ES / 2) {
        int p, q;
        circle_pair(ES, step, t, &p, &q);
        if (p > q) { const int w = p; p = q; q = w; }
        const double app = S[p + p * ELD], aqq = S[q + q * ELD], apq = S[p + q * ELD];
        double c = 1.0, s = 0.0;
        if (apq != 0.0 && fabs(apq) > 1e-15 * sqrt(fabs(app * aqq))) {
          // Rutishauser: theta = (aqq - app) / (2 apq), t = sign(theta) / (|theta| + sqrt(1 + theta^2))
          const double theta = (aqq - app) / (2.0 * apq);
          const double tt = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(1.0 + theta * theta));
          if (fabs(tt) >= 1e-17) {
            c = 1.0 / sqrt(1.0 + tt * tt);
            s = tt * c;
            atomicAdd(&rot_sweep, 1);
          }
        }
        cs[t][0] = c;
        cs[t][1] = s;
        pr[t][0] = p;
        pr[t][1] = q;
      }
      __syncthreads();
      // rows p, q of S: S <- J^T S   (J: c at (p,p), (q,q); s at (p,q); -s at (q,p))
      for (int e = t; e < (ES / 2) * ES; e += NT) {
        const int pk = e / ES, j = e % ES;
        const double c = cs[pk][0], s = cs[pk][1];
        if (s == 0.0) continue;
        const int p = pr[pk][0], q = pr[pk][1];
        const double sp = S[p + j * ELD], sq = S[q + j * ELD];
        S[p + j * ELD] = c * sp - s * sq;
        S[q + j * ELD] = s * sp + c * sq;
      }
      __syncthreads();
      // columns p, q of S and of R: S <- S J, R <- R J
      for (int e = t; e < (ES / 2) * ES; e += NT) {
        const int pk = e / ES, i = e % ES;
        const double c = cs[pk][0], s = cs[pk][1];
        if (s == 0.0) continue;
        const int p = pr[pk][0], q = pr[pk][1];
        const double sp = S[i + p * ELD], sq = S[i + q * ELD];
        S[i + p * ELD] = c * sp - s * sq;
        S[i + q * ELD] = s * sp + c * sq;
        const double rp = R[i + p * ELD], rq = R[i + q * ELD];
        R[i + p * ELD] = c * rp - s * rq;
        R[i + q * ELD] = s * rp + c * rq;
      }
      __syncthreads();
    }
    const int rs = rot_sweep;
    if (t == 0) rot_total += rs;
    __syncthreads();  // (every thread has read rot_sweep before thread 0 resets it)
    if (rs == 0) break;
  }
  // R accumulated hundreds of rotations and drifted from orthogonality by ~sqrt(count) ulps;
  // applied round after round, that drift (not the rotations' own rounding) set the
  // eigenvalue error.  One Newton-Schulz step R <- R (3 I - R^T R) / 2 takes it to rounding
  // level (quadratic: 1e-14 -> 1e-28) -- two 64^3 products in LDS, S's space holding R^T R.
  if (reorth && rot_total) {  // (the products on the first 256 threads)
    const bool on = t < 256;
    const int i0 = 4 * (t % 16), j0 = 4 * ((t / 16) % 16);
    double c[4][4];
    if (on) {
      gemm64<true>(R, R, c);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) S[(i0 + a) + (j0 + b) * ELD] = c[a][b];
    }
    __syncthreads();
    double r[4][4];
    if (on) {
      gemm64<false>(R, S, c);  // R (R^T R)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) r[a][b] = 1.5 * R[(i0 + a) + (j0 + b) * ELD] - 0.5 * c[a][b];
    }
    __syncthreads();
    if (on)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) R[(i0 + a) + (j0 + b) * ELD] = r[a][b];
    __syncthreads();
  }
  double* Rk = Rbuf + (size_t)k * ES * ES;
  for (int e = t; e < ES * ES; e += NT) Rk[e] = R[(e % ES) + (e / ES) * ELD];
  if (t == 0) {
    if (rot_total) atomicAdd(rotations, rot_total);
    rotations[2 + k] = rot_total != 0;  // R_k != I: the transform skips identity factors
  }
}

// 2. A[P_k, P_l] <- R_k^T A[P_k, P_l] R_l for every tile k <= l (mirrored into (l, k)), and
//    B[P_k, cols] <- R_k^T B[P_k, cols] for every pair k and 64-column chunk of B
//    MF: the two products on the matrix cores, staged through LDS and stored by columns
//    (default; GPR_EIG_TMFMA=0: the VALU form).  rflag (default; GPR_EIG_SKIPI=0 passes null):
//    the pairs that rotated this round -- identity factors are skipped
template <bool MF>
__global__ __launch_bounds__(256) void eig_transform_kernel(double* __restrict__ A, size_t lda,
                                                           int nb, int round,
                                                           const double* __restrict__ Rbuf,
                                                           double* __restrict__ B, size_t ldb,
                                                           int m, int ntiles,
                                                           const int* __restrict__ rflag) {
  __shared__ double lds[4 * ES * ELD];  // 133 KB: one workgroup per CU
  double* T = lds;               // tile (then U = T R_l)
  double* Rl = T + ES * ELD;
  double* Rk = Rl + ES * ELD;
  double* U = Rk + ES * ELD;
  const int t = threadIdx.x, np = nb / 2;
  const int i0 = 4 * (t % 16), j0 = 4 * (t / 16);
  int bid = blockIdx.x;
  if (bid < ntiles) {
    // tile (k, l), k <= l, from the linear upper-triangle index
    int l = (int)((sqrt(8.0 * bid + 1.0) - 1.0) * 0.5);
    while ((l + 1) * (l + 2) / 2 <= bid) ++l;
    while (l * (l + 1) / 2 > bid) --l;
    const int k = bid - l * (l + 1) / 2;
    // a pair that rotated nothing this round has R = I exactly, and a product with I is exact
    // (every other term is a signed zero): such factors are skipped, bitwise the same result
    const bool fk = !rflag || rflag[k] != 0, fl = !rflag || rflag[l] != 0;
    if (!fk && !fl) return;
    int Ik, Jk, Il, Jl;
    circle_pair(nb, round, k, &Ik, &Jk);
    circle_pair(nb, round, l, &Il, &Jl);
    const double* Rkg = Rbuf + (size_t)k * ES * ES;
    const double* Rlg = Rbuf + (size_t)l * ES * ES;
    for (int e = t; e < ES * ES; e += 256) {
      const int i = e % ES, j = e / ES;
      T[i + j * ELD] = A[(size_t)pair_row(Ik, Jk, i) + (size_t)pair_row(Il, Jl, j) * lda];
      Rl[i + j * ELD] = Rlg[e];
      Rk[i + j * ELD] = Rkg[e];
    }
    __syncthreads();
    if (MF) {
      double* res = T;
      if (fl) {
        gemm64_mfma<false>(T, Rl, U);  // U = T R_l
        res = U;
      }
      if (fk) {
        gemm64_mfma<true>(Rk, res, T);  // T = R_k^T U
        res = T;
      }
      // column runs of 32 contiguous rows (the pair's two blocks) per 64-lane store
      for (int e = t; e < ES * ES; e += 256) {
        const int i = e % ES, j = e / ES;
        const double v = (k == l && i > j) ? res[j + i * ELD] : res[i + j * ELD];
        A[(size_t)pair_row(Ik, Jk, i) + (size_t)pair_row(Il, Jl, j) * lda] = v;
      }
      if (k != l)  // the mirror (l, k): its column j is row j of T
        for (int e = t; e < ES * ES; e += 256) {
          const int i = e % ES, j = e / ES;
          A[(size_t)pair_row(Il, Jl, i) + (size_t)pair_row(Ik, Jk, j) * lda] = res[j + i * ELD];
        }
      return;
    }
    double c[4][4];
    gemm64<false>(T, Rl, c);  // U = T R_l
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) U[(i0 + a) + (j0 + b) * ELD] = c[a][b];
    __syncthreads();
    gemm64<true>(Rk, U, c);   // R_k^T U
    if (k == l) {             // exactly symmetric: the upper half, mirrored
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) T[(i0 + a) + (j0 + b) * ELD] = c[a][b];
      __syncthreads();
      for (int e = t; e < ES * ES; e += 256) {
        const int i = e % ES, j = e / ES;
        const double v = i <= j ? T[i + j * ELD] : T[j + i * ELD];
        A[(size_t)pair_row(Ik, Jk, i) + (size_t)pair_row(Il, Jl, j) * lda] = v;
      }
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int gi = pair_row(Ik, Jk, i0 + a), gj = pair_row(Il, Jl, j0 + b);
          A[(size_t)gi + (size_t)gj * lda] = c[a][b];
          A[(size_t)gj + (size_t)gi * lda] = c[a][b];
        }
    }
    return;
  }
  // B rows of pair k, 64-column chunk ch
  bid -= ntiles;
  const int nch = (m + ES - 1) / ES;
  const int k = bid / nch, ch = bid % nch;
  if (k >= np || (rflag && !rflag[k])) return;
  int Ik, Jk;
  circle_pair(nb, round, k, &Ik, &Jk);
  const double* Rkg = Rbuf + (size_t)k * ES * ES;
  for (int e = t; e < ES * ES; e += 256) {
    const int i = e % ES, j = e / ES, col = ch * ES + j;
    T[i + j * ELD] = col < m ? B[(size_t)pair_row(Ik, Jk, i) + (size_t)col * ldb] : 0.0;
    Rk[i + j * ELD] = Rkg[e];
  }
  __syncthreads();
  if (MF) {
    gemm64_mfma<true>(Rk, T, U);
    for (int e = t; e < ES * ES; e += 256) {
      const int i = e % ES, j = e / ES, col = ch * ES + j;
      if (col < m) B[(size_t)pair_row(Ik, Jk, i) + (size_t)col * ldb] = U[i + j * ELD];
    }
    return;
  }
  double c[4][4];
  gemm64<true>(Rk, T, c);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int col = ch * ES + j0 + b;
      if (col < m) B[(size_t)pair_row(Ik, Jk, i0 + a) + (size_t)col * ldb] = c[a][b];
    }
}

__global__ void eig_pad_kernel(const double* __restrict__ A, size_t lda, int n,
                               double* __restrict__ W, int n2) {
  const size_t tot = (size_t)n2 * n2;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot;
       e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % n2), j = (int)(e / n2);
    W[e] = (i < n && j < n) ? A[(size_t)i + (size_t)j * lda] : 0.0;
  }
}

__global__ void eig_diag_kernel(const double* __restrict__ W, int n2, int n, double* __restrict__ lam) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    lam[i] = W[(size_t)i + (size_t)i * n2];
}

}  // namespace

// lambda (n, device) = eigenvalues of the symmetric A (n x n, ld lda; read only), and
// B (n x m, ld ldb) <- P^T B with A = P diag(lambda) P^T.  Eigenvalues in no particular order,
// B's rows in the same order.  *sweeps: outer sweeps used.  Returns GPR_E_HIP (with a message)
// if the iteration does not converge within GPR_EIG_MAX_SWEEPS (default 60).
static int jacobi_eig_apply(gpr_ctx* ctx, const double* dA, int n, int lda, double* dB, int m,
                            int ldb, double* dlam, int* sweeps_out, double floor) {
  if (n <= 0) return 0;
  const int n2 = (n + ES - 1) / ES * ES;
  const int nb = n2 / EB, np = nb / 2;
  const int ntiles = np * (np + 1) / 2;
  // workspace: W (n2 x n2), Bp (n2 x m), R (np x 64 x 64), rotation counter
  const size_t need = (size_t)n2 * n2 + (size_t)n2 * std::max(m, 1) + (size_t)np * ES * ES + 2 + np;
  GPR_TRY(ensure_buf(ctx, &ctx->deig, &ctx->eig_cap, need));
  double* W = ctx->deig;
  double* Bp = W + (size_t)n2 * n2;
  double* Rb = Bp + (size_t)n2 * std::max(m, 1);
  int* rot = reinterpret_cast<int*>(Rb + (size_t)np * ES * ES);  // [0] count, [2 + k] flags
  hipStream_t s = ctx->stream;
  eig_pad_kernel<<<1024, 256, 0, s>>>(dA, (size_t)lda, n, W, n2);
  LAUNCH_CHECK(ctx);
  if (m > 0) {
    HIP_TRY(ctx, hipMemset2DAsync(Bp, (size_t)n2 * sizeof(double), 0, (size_t)n2 * sizeof(double), m, s));
    HIP_TRY(ctx, hipMemcpy2DAsync(Bp, (size_t)n2 * sizeof(double), dB, (size_t)ldb * sizeof(double),
                                  (size_t)n * sizeof(double), m, hipMemcpyDeviceToDevice, s));
  }
  // (measured variants -- the unmerged 256-thread subproblem, the VALU round transform, no
  // identity skipping, more inner sweeps -- were all slower; round 4)
  constexpr int max_sweeps = 60, max_inner = 1, reorth = 1;
  const int nch = m > 0 ? (m + ES - 1) / ES : 0;
  int sweep = 0, hrot = 1;
  TimerScope ts(ctx, TC_OTHER, 0.0);
  for (; sweep < max_sweeps && hrot; ++sweep) {
    HIP_TRY(ctx, hipMemsetAsync(rot, 0, sizeof(int), s));
    for (int r = 0; r < nb - 1; ++r) {
      eig_subproblem_kernel<true, 1024><<<np, 1024, 0, s>>>(W, (size_t)n2, nb, r, Rb, rot, max_inner, reorth, floor);
      eig_transform_kernel<true><<<ntiles + np * nch, 256, 0, s>>>(W, (size_t)n2, nb, r, Rb, Bp,
                                                                  (size_t)n2, m, ntiles, rot + 2);
    }
    LAUNCH_CHECK(ctx);
    HIP_TRY(ctx, hipMemcpyAsync(&hrot, rot, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
  }
  if (sweeps_out) *sweeps_out = sweep;
  if (hrot) return set_err(ctx, GPR_E_HIP, "block Jacobi eigensolver: not converged after %d sweeps", sweep);
  eig_diag_kernel<<<(n + 255) / 256, 256, 0, s>>>(W, n2, n, dlam);
  LAUNCH_CHECK(ctx);
  if (m > 0)
    HIP_TRY(ctx, hipMemcpy2DAsync(dB, (size_t)ldb * sizeof(double), Bp, (size_t)n2 * sizeof(double),
                                  (size_t)n * sizeof(double), m, hipMemcpyDeviceToDevice, s));
  return 0;
}

// The symmetric eigendecomposition applied to B: by default the tridiagonal reduction
// (tridiag.hip: A = Q T Q^T, B <- Q^T B inside its launch) followed by divide and conquer on T
// (dstedc.hip: lam, B <- Z^T B) -- LAPACK syevr's two stages; block Jacobi (above) for n beyond
// their bounds (16384), when the reduction's cooperative launch is refused (its workgroups cannot
// all be resident: another context's persistent work on the device), or when asked for (method 2).  *sweeps: Jacobi sweeps, or the depth of the
// divide-and-conquer tree.
int sym_eig_apply(gpr_ctx* ctx, const double* dA, int n, int lda, double* dB, int m, int ldb,
                  double* dlam, int* sweeps_out, double floor, int method) {
  if (n <= 0) {
    if (sweeps_out) *sweeps_out = 0;
    return 0;
  }
  if (method != 2 && sym_tridiag_ok(n) && tridiag_eig_ok(n)) {
    GPR_TRY(ensure_buf(ctx, &ctx->dtri, &ctx->tri_cap, 2 * (size_t)n + 2));
    double* d = ctx->dtri;
    double* e = d + n + 1;
    const int rc = sym_tridiag(ctx, dA, n, lda, dB, m, ldb, d, e);
    if (rc == GPR_E_UNSUP) {  // refused before it ran (not co-resident): B untouched -> Jacobi
      ctx->err.clear();
      return jacobi_eig_apply(ctx, dA, n, lda, dB, m, ldb, dlam, sweeps_out, floor);
    }
    GPR_TRY(rc);
    GPR_TRY(tridiag_eig_apply(ctx, d, e, n, dB, m, ldb, dlam));
    if (sweeps_out) {
      int depth = 0;
      while ((1 << depth) < n) ++depth;
      *sweeps_out = depth;
    }
    return 0;
  }
  return jacobi_eig_apply(ctx, dA, n, lda, dB, m, ldb, dlam, sweeps_out, floor);
}

extern "C" int gpr_syev_apply(gpr_ctx_t ctx, const double* dA, int n, int lda, double* dB, int m,
                              int ldb, double* dlam, int* sweeps) {
  if (!ctx) return GPR_E_ARG;
  if (n < 0 || m < 0 || lda < std::max(n, 1) || (m > 0 && ldb < std::max(n, 1)) ||
      (n > 0 && (!dA || !dlam)) || (m > 0 && n > 0 && !dB))
    return set_err(ctx, GPR_E_ARG, "bad args");
  return sym_eig_apply(ctx, dA, n, lda, dB, m, ldb, dlam, sweeps, 0.0, 0);
}
