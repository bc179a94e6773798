// FP64 MFMA GEMM for gfx950:  C[m,n] = alpha * sum_k P[k,m] Q[k,n] + beta * C[m,n]
//
// Both operands are "K-contiguous" (column m of P and column n of Q are contiguous in k),
// which is how every product on the GP hot path is laid out in this engine:
//   * POTRF trailing SYRK   A22 -= U12^T U12          (row panel of the upper factor)
//   * POTRF/TRSM panel      X = U_bb^{-T} B_b          (P = U_bb^{-1}, Q = B_b)
//   * TRSM trailing update  B_c -= U_bc^T X_b
//   * K^{-1} = Z^T Z        (Z = U^{-T}; upper tiles, K-range from the tile's n0)
//   * split mean            mu = A o (B^T . diag(wt) C)   (Hadamard epilogue, qscale)
// so a single kernel with a few epilogue switches covers them all.
//
// v_mfma_f64_16x16x4_f64: lane l supplies A[l&15][k=l>>4] and B[k=l>>4][l&15] (one f64
// each); D lane l reg r = D[row (l>>4)+4r][col l&15] (verified on MI355X,
// tools/probe/mfma_f64_probe.hip).  We feed the Q fragment as A and the P fragment as B,
// so D = (Q^T P) has rows = n and cols = m: lanes 0..15 of a register hold 16 consecutive
// m of one column n -> 128-B contiguous segments on the C read/write.
//
// Tile 128 x 128 x 16, 256 threads = 4 waves in 2(m) x 2(n), 64x64 per wave = 4x4 MFMA
// blocks (16 f64x4 accumulators, 128 VGPRs).  Double-buffered LDS (rows padded to 17
// doubles), next stage prefetched into registers while the current stage's 64 MFMAs per
// wave run; one barrier per stage.  A K=16 stage is 64 MFMAs x ~64 cycles per wave, so
// global latency is fully hidden at 2 workgroups per CU.
#include <cstdlib>

#include "common.hpp"

namespace {

constexpr int TM = 128, TN = 128, TK = 16, LDT = TK + 1;
typedef double d4 __attribute__((ext_vector_type(4)));

struct GemmK {
  GemmArgs g;
  int tiles_m, tiles_n;
  int gm, gn;           // super-tile edges (tiles)
  int xcd_remap;
  int super_m;          // super-tiles along m (general grid)
};

__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(GemmK a) {
  const GemmArgs& g = a.g;
  if (g.info && *g.info != 0) return;
  __shared__ double Ps[2][TM * LDT];
  __shared__ double Qs[2][TN * LDT];
  __shared__ double red[2][TN];

  // XCD-aware, super-tile-grouped tile order.  Blocks b and b+8 share an XCD (round-robin
  // dispatch), so the bijective remap hands each XCD a contiguous range of logical ids;
  // logical ids walk GxG super-tiles, so the P/Q panels of the ~64 tiles an XCD has in
  // flight (2G panels of 128 x K) stay in its 4 MB L2.  Placement only affects speed.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int L = a.xcd_remap ? (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3)
                            : bid;
  const int Gm = a.gm, Gn = a.gn;
  const int sidx = L / (Gm * Gn), wl = L % (Gm * Gn);
  int SI, SJ;
  if (g.upper) {  // upper super-tiles SI <= SJ, triangular order
    int sj = (int)((sqrt(8.0 * sidx + 1.0) - 1.0) * 0.5);
    while ((sj + 1) * (sj + 2) / 2 <= sidx) ++sj;
    while (sj * (sj + 1) / 2 > sidx) --sj;
    SJ = sj;
    SI = sidx - sj * (sj + 1) / 2;
  } else {
    SI = sidx % a.super_m;
    SJ = sidx / a.super_m;
  }
  const int tm = SI * Gm + (wl % Gm), tn = SJ * Gn + (wl / Gm);
  if (tm >= a.tiles_m || tn >= a.tiles_n || (g.upper && tm > tn)) return;
  const int m0 = tm * TM, n0 = tn * TN;
  if (g.mask_upper && m0 > n0 + TN - 1 + g.mask_off) return;  // tile entirely below diagonal
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;

  const int kbeg = g.kfrom_n ? n0 : 0;
  const int kend = g.K;
  const int nst = kend > kbeg ? (kend - kbeg + TK - 1) / TK : 0;

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  double rp[8], rq[8];
  // global -> registers for stage s
  auto gload = [&](int s) {
    const int k0 = kbeg + s * TK;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int idx = tid + 256 * r;
      const int col = idx >> 4, kk = idx & 15;
      const int k = k0 + kk;
      const bool kin = k < kend;
      const int m = m0 + col, n = n0 + col;
      rp[r] = (kin && m < g.M) ? g.P[(size_t)k + (size_t)m * g.ldp] : 0.0;
      double q = (kin && n < g.N) ? g.Q[(size_t)k + (size_t)n * g.ldq] : 0.0;
      if (g.qscale) q *= (kin ? g.qscale[k] : 0.0);
      rq[r] = q;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int idx = tid + 256 * r;
      const int col = idx >> 4, kk = idx & 15;
      Ps[buf][col * LDT + kk] = rp[r];
      Qs[buf][col * LDT + kk] = rq[r];
    }
  };

  if (nst > 0) {
    gload(0);
    lstore(0);
    __syncthreads();
  }
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) gload(s + 1);
    const double* ps = Ps[buf];
    const double* qs = Qs[buf];
#pragma unroll
    for (int k4 = 0; k4 < TK / 4; ++k4) {
      double af[4], bf[4];
      const int kk = k4 * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = qs[(wn * 64 + i * 16 + (lane & 15)) * LDT + kk];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = ps[(wm * 64 + j * 16 + (lane & 15)) * LDT + kk];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nst) lstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: all loads first (C, E), then all stores -- interleaving them through
  // possibly-aliasing pointers would serialise one HBM round trip per element.
  double* __restrict__ Cp = g.C;
  const double* __restrict__ Ep = g.E;
  const bool has_beta = g.beta != 0.0;
  const bool has_e = Ep != nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * 64 + i * 16 + (lane >> 4) + 4 * r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + (lane & 15);
        const bool in = m < g.M && n < g.N && (!(g.upper || g.mask_upper) || m <= n + g.mask_off);
        double v = acc[i][j][r];
        if (has_e) v = v * (in ? Ep[(size_t)m + (size_t)n * g.lde] : 0.0);
        v = g.alpha * v;
        if (has_beta) v = v + g.beta * (in ? Cp[(size_t)m + (size_t)n * g.ldc] : 0.0);
        acc[i][j][r] = v;
      }
    }
  const bool do_norm = g.norm_out != nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * 64 + i * 16 + (lane >> 4) + 4 * r;
      double nsum = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + (lane & 15);
        if (m < g.M && n < g.N && (!(g.upper || g.mask_upper) || m <= n + g.mask_off)) {
          const double v = acc[i][j][r];
          Cp[(size_t)m + (size_t)n * g.ldc] = v;
          nsum = fma(v, v, nsum);
        }
      }
      if (do_norm) {
        nsum += __shfl_xor(nsum, 1);
        nsum += __shfl_xor(nsum, 2);
        nsum += __shfl_xor(nsum, 4);
        nsum += __shfl_xor(nsum, 8);
        if ((lane & 15) == 0) red[wm][wn * 64 + i * 16 + (lane >> 4) + 4 * r] = nsum;
      }
    }
  }
  if (do_norm) {
    __syncthreads();
    if (tid < TN) {
      const int n = n0 + tid;
      if (n < g.N) g.norm_out[n] -= red[0][tid] + red[1][tid];
    }
  }
}

}  // namespace

int launch_gemm_tn(gpr_ctx* ctx, const GemmArgs& g, int timing_class) {
  if (g.M <= 0 || g.N <= 0) return 0;
  if (g.norm_out && g.M > TM) return set_err(ctx, GPR_E_ARG, "gemm norm epilogue needs M<=%d", TM);
  GemmK a;
  a.g = g;
  a.tiles_m = (g.M + TM - 1) / TM;
  a.tiles_n = (g.N + TN - 1) / TN;
  static const int genv = getenv("GPR_GEMM_GROUP") ? atoi(getenv("GPR_GEMM_GROUP")) : 8;
  static const int xenv = getenv("GPR_GEMM_XCD") ? atoi(getenv("GPR_GEMM_XCD")) : 1;
  a.xcd_remap = xenv;
  a.gm = std::max(1, std::min(genv, a.tiles_m));
  a.gn = std::max(1, std::min(genv, a.tiles_n));
  if (g.upper) a.gn = a.gm;
  a.super_m = (a.tiles_m + a.gm - 1) / a.gm;
  const long long super_n = (a.tiles_n + a.gn - 1) / a.gn;
  long long nblk;
  double flops;
  if (g.upper) {
    if (a.tiles_m != a.tiles_n) return set_err(ctx, GPR_E_ARG, "upper gemm needs M == N");
    nblk = super_n * (super_n + 1) / 2 * a.gm * a.gn;
    flops = (double)g.M * (g.M + 1) * g.K;  // 2 * M(M+1)/2 * K
    if (g.kfrom_n) flops = (double)g.M * g.M * g.M / 3.0;
  } else {
    nblk = (long long)a.super_m * super_n * a.gm * a.gn;
    flops = 2.0 * g.M * (double)g.N * g.K;
    if (g.mask_upper) {  // exclude the masked corner rows m > n + mask_off
      const double rows_below = std::max(0.0, (double)g.M - g.mask_off);
      const double cut = std::min(rows_below, (double)g.N);
      flops = 2.0 * g.K * ((double)g.M * g.N - (cut * (cut - 1) / 2.0 + std::max(0.0, rows_below - g.N) * g.N));
    }
  }
  TimerScope ts(ctx, timing_class, flops);
  // g.occ1: reserve LDS so only ONE such workgroup fits per CU, leaving the other half of
  // every CU to a concurrent (lookahead) stream
  static const size_t pad_env = getenv("GPR_GEMM_PAD") ? (size_t)atoi(getenv("GPR_GEMM_PAD")) : 0;
  const size_t pad = g.occ1 ? 20 * 1024 : pad_env;
  gemm_tn_kernel<<<(unsigned)nblk, 256, pad, ctx->ls>>>(a);
  LAUNCH_CHECK(ctx);
  return 0;
}
