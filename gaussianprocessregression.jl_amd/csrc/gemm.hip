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

constexpr int TM = 128, TN = 128, TK = 16, LDT = TK;
// LDS rows hold the 16 k-values of one column as eight 16-B chunks; chunk c of row r is
// stored at chunk position c ^ ((r >> 1) & 7).  Lane l of an MFMA fragment reads row l & 15,
// chunk (l >> 4) + 4p with ONE ds_read_b128 (k-steps 2p and 2p+1): with this swizzle each of
// the four 16-lane groups of ds_read_b128 hits 16 distinct bank quads (conflict-free), and
// the 8-lane groups of the 16-B stores write one whole row each.
__device__ __forceinline__ int lds_idx(int row, int chunk) {
  return row * LDT + ((chunk ^ ((row >> 1) & 7)) << 1);
}
typedef double d4 __attribute__((ext_vector_type(4)));

struct GemmK {
  GemmArgs g;
  int tiles_m, tiles_n;
  int gm, gn;           // super-tile edges (tiles)
  int xcd_remap;
  int super_m;          // super-tiles along m (general grid)
};

__device__ __forceinline__ bool tile_coords(const GemmK& a, int& m0, int& n0) {
  const GemmArgs& g = a.g;
  // XCD-aware, super-tile-grouped tile order.  Blocks b and b+8 share an XCD (round-robin
  // dispatch), so the bijective remap hands each XCD a contiguous range of logical ids;
  // logical ids walk GxG super-tiles, so the P/Q panels of the ~64 tiles an XCD has in
  // flight (2G panels of 128 x K) stay in its 4 MB L2.  Placement only affects speed.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  if (g.kend_from_m && !g.upper && !g.mask_upper) {
    // triangular P: row-tile tm costs (tm + 1) K-steps.  Heavy rows first; with an even
    // number of row tiles, block b and block b + T/2 (same XCD, and the pair that shares a
    // CU when the grid is two workgroups per CU) get complementary rows tm + tm' = tiles_m - 1,
    // so every CU carries the same K work.
    const int tmn = a.tiles_m, tnn = a.tiles_n, half = (tmn / 2) * tnn;
    if (bid >= tmn * tnn) return false;
    int tm, tn;
    if ((tmn & 1) == 0 && bid >= half) {
      tm = (bid - half) / tnn;
      tn = (bid - half) % tnn;
    } else {
      tm = tmn - 1 - bid / tnn;
      tn = bid % tnn;
    }
    m0 = tm * TM;
    n0 = tn * TN;
    return true;
  }
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int L = a.xcd_remap ? (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3)
                            : bid;
  const int Gm = a.gm, Gn = a.gn;
  int tm, tn;
  if (g.upper) {  // upper super-tiles SI <= SJ, triangular order
    const int sidx = L / (Gm * Gn), wl = L % (Gm * Gn);
    int sj = (int)((sqrt(8.0 * sidx + 1.0) - 1.0) * 0.5);
    while ((sj + 1) * (sj + 2) / 2 <= sidx) ++sj;
    while (sj * (sj + 1) / 2 > sidx) --sj;
    tm = (sidx - sj * (sj + 1) / 2) * Gm + (wl % Gm);
    tn = sj * Gn + (wl / Gm);
  } else {
    // the grid holds exactly tiles_m x tiles_n blocks: column bands of Gn tiles (the last one
    // narrower), each walked in Gm-row super-tiles (the last one shorter).  A grid padded to
    // whole super-tiles would put all the empty blocks at the end of the logical order, i.e.
    // on the last XCD, and overload the other seven (+14 % at 8193 right-hand sides).
    const int tmn = a.tiles_m, tnn = a.tiles_n;
    const int SJ = L / (tmn * Gn);
    const int bw = min(Gn, tnn - SJ * Gn);
    const int t = L - SJ * tmn * Gn;
    const int fr = (tmn / Gm) * Gm;  // rows covered by whole super-tiles
    if (t < fr * bw) {
      const int SI = t / (Gm * bw), r = t - SI * Gm * bw;
      tm = SI * Gm + r % Gm;
      tn = SJ * Gn + r / Gm;
    } else {
      const int t2 = t - fr * bw, h = tmn - fr;
      tm = fr + t2 % h;
      tn = SJ * Gn + t2 / h;
    }
  }
  if (tm >= a.tiles_m || tn >= a.tiles_n || (g.upper && tm > tn)) return false;
  m0 = tm * TM;
  n0 = tn * TN;
  return !(g.mask_upper && m0 > n0 + TN - 1 + g.mask_off);  // tile entirely below diagonal
}

// C = alpha * acc (o E) + beta * C on the tile, optional column sum-of-squares into norm_out.
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, d4 (&acc)[4][4], int m0, int n0,
                                              double* red, bool preloaded = false) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  // ---- epilogue: all loads first (C, E), then all stores -- interleaving them through
  // possibly-aliasing pointers would serialise one HBM round trip per element.
  double* __restrict__ Cp = g.C;
  const double* __restrict__ Ep = g.E;
  // preloaded: the accumulators started at (beta/alpha) C, so C is not read again here
  const bool has_beta = g.beta != 0.0 && !preloaded;
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
        if ((lane & 15) == 0) red[wm * TN + wn * 64 + i * 16 + (lane >> 4) + 4 * r] = nsum;
      }
    }
  }
  if (do_norm) {
    __syncthreads();
    if (tid < TN) {
      const int n = n0 + tid;
      if (n < g.N) g.norm_out[n] -= red[tid] + red[TN + tid];
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(GemmK a) {
  const GemmArgs& g = a.g;
  if (g.info && *g.info != 0) return;
  __shared__ double Ps[2][TM * LDT];
  __shared__ double Qs[2][TN * LDT];
  __shared__ double red[2][TN];

  int m0, n0;
  if (!tile_coords(a, m0, n0)) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;

  const int kbeg = g.kfrom_n ? n0 : 0;
  const int kend = g.kend_from_m ? min(g.K, m0 + TM) : g.K;
  const int nst = kend > kbeg ? (kend - kbeg + TK - 1) / TK : 0;

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  // VEC: 16-B loads of k-pairs (8 lanes cover one 128-B column segment), branch-free with
  // clamped addresses; out-of-range elements are zeroed when the stage is written to LDS.
  // Needs 16-B aligned operands, even ld and even K (checked by the launcher), no qscale.
  // Scalar path: one f64 per lane per load, any alignment, optional qscale.
  constexpr int NR = VEC ? 4 : 8;
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2 vp[VEC ? 4 : 1], vq[VEC ? 4 : 1];
  double rp[VEC ? 1 : 8], rq[VEC ? 1 : 8];
  // global -> registers for stage s
  auto gload = [&](int s) {
    const int k0 = kbeg + s * TK;
    if constexpr (VEC) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int idx = tid + 256 * r;
        const int col = idx >> 3, k = k0 + 2 * (idx & 7);
        const int kc = k < kend ? k : kbeg;
        const int m = min(m0 + col, g.M - 1), n = min(n0 + col, g.N - 1);
        vp[r] = *reinterpret_cast<const d2*>(g.P + (size_t)kc + (size_t)m * g.ldp);
        vq[r] = *reinterpret_cast<const d2*>(g.Q + (size_t)kc + (size_t)n * g.ldq);
      }
    } else {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
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
    }
  };
  auto lstore = [&](int buf, int s) {
    const int k0 = kbeg + s * TK;
    if constexpr (VEC) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int idx = tid + 256 * r;
        const int col = idx >> 3, kp = idx & 7;
        const bool kin = k0 + 2 * kp < kend;
        const d2 z = {0.0, 0.0};
        *reinterpret_cast<d2*>(&Ps[buf][lds_idx(col, kp)]) = (kin && m0 + col < g.M) ? vp[r] : z;
        *reinterpret_cast<d2*>(&Qs[buf][lds_idx(col, kp)]) = (kin && n0 + col < g.N) ? vq[r] : z;
      }
    } else {
      (void)k0;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int idx = tid + 256 * r;
        const int col = idx >> 4, kk = idx & 15;
        Ps[buf][lds_idx(col, kk >> 1) + (kk & 1)] = rp[r];
        Qs[buf][lds_idx(col, kk >> 1) + (kk & 1)] = rq[r];
      }
    }
  };

  if (nst > 0) {
    gload(0);
    lstore(0, 0);
    __syncthreads();
  }
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) gload(s + 1);
    const double* ps = Ps[buf];
    const double* qs = Qs[buf];
    // k-step 2p+h, lane group g = lane >> 4 consumes k = 2 (g + 4p) + h for both operands
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = (lane >> 4) + 4 * p;
      d2 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const d2*>(&qs[lds_idx(wn * 64 + i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const d2*>(&ps[lds_idx(wm * 64 + j * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i][h], bf[j][h], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nst) lstore(buf ^ 1, s + 1);
    __syncthreads();
  }

  gemm_epilogue(g, acc, m0, n0, &red[0][0]);
}

// ---- deep-pipelined variant: one workgroup per CU, four LDS stages fed by LDS-DMA ------
// One wave per SIMD keeps the f64 matrix pipe full on its own (back-to-back
// v_mfma_f64_16x16x4 from one wave: 77.7 TF/s measured, tools/probe/mfma_f64_peak.hip), so
// this variant spends the doubled register budget (launch bounds 256 x 1) on a second
// fragment set instead of a second workgroup: while stage s's 64 MFMAs per wave issue, the
// ds_read_b128 of stage s+1 are already in flight, and the global->LDS DMA
// (global_load_lds_dwordx4, no VGPRs, swizzle applied on the source address) runs 2-3
// stages ahead.  Per stage: one counted vmcnt wait (own DMA of stage s+1 retired) and ONE
// raw s_barrier (stage s+1 visible to all waves; stage s-1's buffer free for the DMA of
// stage s+3).  Eligible when K - kbeg is a multiple of 16, operands 16-B aligned with even
// leading dimensions and no qscale (the launcher checks; other calls use gemm_tn_kernel).
// acc = 0, produced in AGPRs (an MFMA with zero operands and inline-constant C = 0), so every
// definition of the accumulators is AGPR-class and the loop never copies them
__device__ __forceinline__ void mfma_agpr_zero(d4& acc) {
  asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, 0" : "=a"(acc) : "v"(0.0));
}

template <int VM>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
}

constexpr int PBUF = 4;  // LDS stages of the pipelined kernels

// Stage image: TKS doubles per row (NCH = TKS/2 chunks of 16 B), chunk c of row r stored at
// c ^ swz(r): conflict-free for the 16-lane groups of ds_read_b128 (checked exhaustively for
// both row lengths: NCH = 8 -> (r >> 1) & 7, NCH = 4 -> (r >> 1) & 2).
template <int TKS>
__device__ __forceinline__ int pipe_swz(int row) {
  return TKS == 16 ? ((row >> 1) & 7) : ((row >> 1) & 2);
}
template <int TKS>
__device__ __forceinline__ int pipe_idx(int row, int chunk) {
  return row * TKS + ((chunk ^ pipe_swz<TKS>(row)) << 1);
}

// TKS = 16, OCC = 1: one workgroup per CU (512 registers per lane), 32-KB stages, 64 MFMAs
//   per wave per stage -- best for long K (72 TF/s at 8192^3 vs 65 for gemm_tn_kernel).
// TKS = 8, OCC = 2: two workgroups per CU, 16-KB stages, 32 MFMAs per stage -- a second
//   workgroup hides each tile's prologue fill and C epilogue, which matter at short K (the
//   K = nb2 trailing updates of POTRF and the TRSM).
template <int TKS, bool PRELOAD>
__device__ __forceinline__ void gemm_tn_pipe_body(const GemmK& a) {
  constexpr int STAGE_D = (TM + TN) * TKS;      // doubles per stage (P image, then Q)
  constexpr int NCH = TKS / 2;                  // 16-B chunks per row
  constexpr int ROWS_PER_DMA = 64 / NCH;        // rows covered by one wave-wide 1-KB DMA
  constexpr int NDMA = TM / (4 * ROWS_PER_DMA); // DMA instructions per wave per operand
  constexpr int VM_STAGE = 2 * NDMA;            // vmcnt increments per stage
  constexpr int NP = TKS / 8;                   // fragment blocks (2 k-steps each) per stage
  typedef double d2 __attribute__((ext_vector_type(2)));
  const GemmArgs& g = a.g;
  if (g.info && *g.info != 0) return;
  __shared__ double lds[PBUF * STAGE_D + 2 * TN];
  int m0, n0;
  if (!tile_coords(a, m0, n0)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  const int kbeg = g.kfrom_n ? n0 : 0;
  const int nst = ((g.kend_from_m ? min(g.K, m0 + TM) : g.K) - kbeg) / TKS;

  // DMA sources: instruction r of wave w fills rows ROWS_PER_DMA (4r + w) + (L / NCH); lane
  // L lands at physical chunk L % NCH of its row, so it fetches the logical chunk
  // (L % NCH) ^ swz(row) (the swizzle is applied on the source side; LDS-DMA writes
  // lane-linearly).  Rows past M/N are clamped: a row of P only feeds its own output row,
  // which is never stored.
  const double* srcP[NDMA];
  const double* srcQ[NDMA];
#pragma unroll
  for (int r = 0; r < NDMA; ++r) {
    const int row = ROWS_PER_DMA * (4 * r + w) + lane / NCH;
    const int c = (lane % NCH) ^ pipe_swz<TKS>(row);
    srcP[r] = g.P + kbeg + 2 * c + (size_t)min(m0 + row, g.M - 1) * g.ldp;
    srcQ[r] = g.Q + kbeg + 2 * c + (size_t)min(n0 + row, g.N - 1) * g.ldq;
  }
  // DMA of stage s into buffer s % PBUF.  Stages past the end re-fetch the last stage into a
  // buffer that is never read again: the loop body stays branch-free (one register
  // assignment for the accumulators) and the vmcnt count uniform.
  auto issue = [&](int s) {
    double* base = lds + (s % PBUF) * STAGE_D;
    const size_t ko = (size_t)min(s, nst - 1) * TKS;
#pragma unroll
    for (int r = 0; r < NDMA; ++r) {
      __builtin_amdgcn_global_load_lds(srcP[r] + ko, base + (4 * r + w) * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(srcQ[r] + ko, base + TM * TKS + (4 * r + w) * 128, 16, 0, 0);
    }
  };
  // fragment set of one stage: [p][i] Q-side (A operand), [p][4 + j] P-side (B operand);
  // lane group g = lane >> 4 reads chunk g + 4p, i.e. k = 2 (g + 4p) + h for k-step 2p + h
  auto read_frags = [&](d2 (&F)[NP][8], int s) {
    const double* ps = lds + (s % PBUF) * STAGE_D;
    const double* qs = ps + TM * TKS;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int ch = (lane >> 4) + 4 * p;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        F[p][i] = *reinterpret_cast<const d2*>(&qs[pipe_idx<TKS>(wn * 64 + i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        F[p][4 + j] = *reinterpret_cast<const d2*>(&ps[pipe_idx<TKS>(wm * 64 + j * 16 + (lane & 15), ch)]);
    }
  };
  // PRELOAD (host picks it for beta != 0, alpha != 0, no Hadamard factor): the tile of C
  // is read up front into the accumulators as (beta/alpha) C -- 64 independent loads per
  // lane in one batch instead of a dependent load->store round trip in the epilogue (which
  // bounds the short-K chain GEMMs); the epilogue then only stores alpha acc.  A compile-
  // time switch: a runtime branch merging two accumulator initialisations miscompiles.
  d4 acc[4][4];
  if constexpr (PRELOAD) {
    const double sc = g.beta / g.alpha;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = n0 + wn * 64 + i * 16 + (lane >> 4) + 4 * r;
        const double* col = g.C + (size_t)min(nn, g.N - 1) * g.ldc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // clamped address + select: branch-free, all 64 loads in flight together
          const int mm = m0 + wm * 64 + j * 16 + (lane & 15);
          const double c = col[min(mm, g.M - 1)];
          acc[i][j][r] = (mm < g.M && nn < g.N) ? sc * c : 0.0;
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mfma_agpr_zero(acc[i][j]);
  }
  auto mfma_stage = [&](const d2 (&F)[NP][8]) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[p][i][h], F[p][4 + j][h], acc[i][j], 0, 0, 0);
  };
  // one pipeline step: stage s computes from Fc while stage s+1's fragments load into Fn
  // (past the end they read a stale buffer and are discarded)
  auto step = [&](int s, d2 (&Fc)[NP][8], d2 (&Fn)[NP][8]) {
    wait_vmcnt<VM_STAGE>();  // own DMA of stage s+1 retired, stage s+2 still in flight
    __builtin_amdgcn_s_barrier();
    issue(s + 3);
    read_frags(Fn, s + 1);
    mfma_stage(Fc);
    // interleave: the DMAs one per MFMA, then the fragment reads one per two MFMAs, so the
    // matrix pipe never waits behind a block of memory instructions
#pragma unroll
    for (int t = 0; t < VM_STAGE; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
#pragma unroll
    for (int t = 0; t < 8 * NP; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32 * NP - VM_STAGE - 16 * NP, 0);
    // retire Fn's reads here (they completed under the MFMAs): lgkmcnt holds at most 15, so
    // the compiler would otherwise wait for ALL next-stage reads before the first MFMA of
    // the next step.  A real s_waitcnt (builtin), which the waitcnt pass accounts for.
    __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  };

  d2 F0[NP][8], F1[NP][8];
  if (nst > 0) {
    issue(0);
    issue(1);
    issue(2);
    wait_vmcnt<2 * VM_STAGE>();
    __builtin_amdgcn_s_barrier();
    read_frags(F0, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  int s = 0;
  for (; s + 1 < nst; s += 2) {
    step(s, F0, F1);
    step(s + 1, F1, F0);
  }
  if (s < nst) mfma_stage(F0);
  wait_vmcnt<0>();
  __syncthreads();  // the epilogue's norm reduction reuses LDS
  gemm_epilogue(g, acc, m0, n0, lds + PBUF * STAGE_D, PRELOAD);
}

// pipe8: C preloaded (beta != 0, the SYRK / TRSM updates); pipe8z: zero-initialised
__global__ __launch_bounds__(256, 2) void gemm_tn_pipe8_kernel(GemmK a) { gemm_tn_pipe_body<8, true>(a); }
__global__ __launch_bounds__(256, 2) void gemm_tn_pipe8z_kernel(GemmK a) { gemm_tn_pipe_body<8, false>(a); }

// ---- narrow-tile variant for short-K launches with few 128x128 tiles -------------------
// The latency-bound panel chain of the factorisation issues K <= 128..256 GEMMs with one
// or a few 128-row tile rows (row TRSM M = 128, in-panel updates): at 128 x 128 tiles such a
// launch occupies a fraction of the CUs and each tile's K loop runs at one CU's MFMA rate
// (128 x 128 x 128 = 13.7 us at 0.31 TF/s per CU).  A 128 x 32 tile spreads the same work
// over 4x the CUs: wave w owns rows 32w..32w+31 and all 32 columns (2 x 2 blocks of
// 16 x 16, 128 MFMAs per K = 128).  Each tile still covers whole 128-row spans of K, so the
// in-place row TRSM (C = Q, M = 128) stays safe: a tile reads all K rows of its columns
// before its epilogue writes them.  Register-prefetched, double-buffered LDS stages of 16 k.
constexpr int NTN = 32;
__global__ __launch_bounds__(256, 4) void gemm_tn_narrow_kernel(GemmK a) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const GemmArgs& g = a.g;
  if (g.info && *g.info != 0) return;
  __shared__ double Ps[2][TM * LDT];
  __shared__ double Qs[2][NTN * LDT];
  const int bid = blockIdx.x;
  const int tm = bid % a.tiles_m, tn = bid / a.tiles_m;
  if (tn >= a.tiles_n) return;
  const int m0 = tm * TM, n0 = tn * NTN;
  if ((g.upper || g.mask_upper) && m0 > n0 + NTN - 1 + g.mask_off) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kbeg = g.kfrom_n ? n0 : 0;
  const int kend = g.kend_from_m ? min(g.K, m0 + TM) : g.K;
  const int nst = kend > kbeg ? (kend - kbeg + TK - 1) / TK : 0;
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  // stage loads: P 128 rows x 8 k-pairs (4 per thread), Q 32 rows x 8 k-pairs (1 per thread);
  // clamped addresses, out-of-range pairs zeroed at the LDS store (K even: pairs whole)
  d2 vp[4], vq;
  auto gload = [&](int st) {
    const int k0 = kbeg + st * TK;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + 256 * r;
      const int row = idx >> 3, k = k0 + 2 * (idx & 7);
      const int kc = k < kend ? k : kbeg;
      vp[r] = *reinterpret_cast<const d2*>(g.P + (size_t)kc + (size_t)min(m0 + row, g.M - 1) * g.ldp);
    }
    const int row = tid >> 3, k = k0 + 2 * (tid & 7);
    const int kc = k < kend ? k : kbeg;
    vq = *reinterpret_cast<const d2*>(g.Q + (size_t)kc + (size_t)min(n0 + row, g.N - 1) * g.ldq);
  };
  auto lstore = [&](int buf, int st) {
    const int k0 = kbeg + st * TK;
    const d2 z = {0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + 256 * r;
      const int row = idx >> 3, kp = idx & 7;
      *reinterpret_cast<d2*>(&Ps[buf][lds_idx(row, kp)]) = (k0 + 2 * kp < kend) ? vp[r] : z;
    }
    const int row = tid >> 3, kp = tid & 7;
    *reinterpret_cast<d2*>(&Qs[buf][lds_idx(row, kp)]) = (k0 + 2 * kp < kend) ? vq : z;
  };
  if (nst > 0) {
    gload(0);
    lstore(0, 0);
    __syncthreads();
  }
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload(st + 1);
    const double* ps = Ps[buf];
    const double* qs = Qs[buf];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = (lane >> 4) + 4 * p;
      d2 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const d2*>(&qs[lds_idx(i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const d2*>(&ps[lds_idx(w * 32 + j * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i][h], bf[j][h], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nst) lstore(buf ^ 1, st + 1);
    __syncthreads();
  }
  // epilogue: D lane l reg r = (n = (l >> 4) + 4r, m = l & 15) of each 16 x 16 block; all C
  // loads first, then the stores
  const bool has_beta = g.beta != 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + i * 16 + (lane >> 4) + 4 * r;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = m0 + w * 32 + j * 16 + (lane & 15);
        const bool in = m < g.M && n < g.N && (!(g.upper || g.mask_upper) || m <= n + g.mask_off);
        double v = g.alpha * acc[i][j][r];
        if (has_beta) v = v + g.beta * (in ? g.C[(size_t)m + (size_t)n * g.ldc] : 0.0);
        acc[i][j][r] = v;
      }
    }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + i * 16 + (lane >> 4) + 4 * r;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = m0 + w * 32 + j * 16 + (lane & 15);
        if (m < g.M && n < g.N && (!(g.upper || g.mask_upper) || m <= n + g.mask_off))
          g.C[(size_t)m + (size_t)n * g.ldc] = acc[i][j][r];
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
  constexpr int genv = 8;  // super-tile edge (tiles) of the XCD-aware walk
  // the XCD remap hands each XCD a contiguous range of tiles (L2 locality); with per-tile
  // K ranges (kfrom_n / kend_from_m) that range would hold all the heavy tiles of one end
  // of the triangle, so those launches keep the round-robin dispatch order (balanced XCDs)
  a.xcd_remap = !g.kfrom_n && !g.kend_from_m;
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
    nblk = (long long)a.tiles_m * a.tiles_n;  // exactly the tiles (see tile_coords)
    flops = 2.0 * g.M * (double)g.N * g.K;
    if (g.kend_from_m)  // upper-triangular P: row m of the product uses K-range [0, m]
      flops = (double)g.N * g.M * (g.M + 1);
    if (g.mask_upper) {  // exclude the masked corner rows m > n + mask_off
      const double rows_below = std::max(0.0, (double)g.M - g.mask_off);
      const double cut = std::min(rows_below, (double)g.N);
      flops = 2.0 * g.K * ((double)g.M * g.N - (cut * (cut - 1) / 2.0 + std::max(0.0, rows_below - g.N) * g.N));
    }
  }
  TimerScope ts(ctx, timing_class, flops);
  // g.occ1: reserve LDS so only ONE such workgroup fits per CU, leaving the other half of
  // every CU to a concurrent (lookahead) stream
  const size_t pad = g.occ1 ? 20 * 1024 : 0;
  const bool vec = !g.qscale && ((uintptr_t)g.P & 15) == 0 && ((uintptr_t)g.Q & 15) == 0 &&
                   (g.ldp & 1) == 0 && (g.ldq & 1) == 0 && (g.K & 1) == 0;
  // pipelined variants need K - kbeg to be a whole number of stages (kbeg is 0 or a
  // multiple of TN).  Few 128 x 128 tiles at short K: the narrow-tile kernel spreads them
  // over 4x the CUs (up to 384 tiles)
  constexpr int narrow_max = 384;
  if (vec && !g.occ1 && !g.E && !g.norm_out && g.K <= 256 && nblk <= narrow_max &&
      !(g.upper && g.kfrom_n)) {
    GemmK an = a;
    an.tiles_n = (g.N + NTN - 1) / NTN;
    const long long nb_n = (long long)an.tiles_m * an.tiles_n;
    gemm_tn_narrow_kernel<<<(unsigned)nb_n, 256, 0, ctx->ls>>>(an);
    LAUNCH_CHECK(ctx);
    return 0;
  }
  // the pipelined 2-WG/CU kernel (faster than its 1-WG/CU, 16-deep form at every measured
  // shape: 74.3 vs 71.9 TF/s at 8192^3, 66.3 vs 52.0 at 16384^2 x 768)
  const bool pipe = vec && (g.K % TK) == 0 && !g.occ1;
  if (pipe) {
    TimerScope tk(ctx, TC_GEMM_PIPE, flops);
    if (g.beta != 0.0 && g.alpha != 0.0 && !g.E)
      gemm_tn_pipe8_kernel<<<(unsigned)nblk, 256, 0, ctx->ls>>>(a);
    else
      gemm_tn_pipe8z_kernel<<<(unsigned)nblk, 256, 0, ctx->ls>>>(a);
  }
  else if (vec)
    gemm_tn_kernel<true><<<(unsigned)nblk, 256, pad, ctx->ls>>>(a);
  else
    gemm_tn_kernel<false><<<(unsigned)nblk, 256, pad, ctx->ls>>>(a);
  LAUNCH_CHECK(ctx);
  return 0;
}
