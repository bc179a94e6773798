// Persistent tile-DAG Cholesky (dpotrf 'U', in place) with optional fused right-hand sides
// B <- U^{-T} B, in ONE launch.
//
// Replaces the same reference calls as potrf_core (cholesky!(Hermitian(K)), src/cost.jl:77,
// src/predict.jl:31) and, with B, the first half of ldiv!/rdiv! against the factor
// (src/predict.jl:32,84: V = U^{-T} K(x, xp) and z = U^{-T} y in gpr_fit_predict).
//
// Left-looking by 128 x 128 tile: the task of upper tile (i, j) of A owns that tile for its
// whole life:
//     acc  = A_ij - sum_{k<i} U_ki^T U_kj          (one long-K FP64 MFMA accumulation)
//     i == j:  U_ii = chol(acc), W_i = U_ii^{-1}   (diag_block.hpp, in LDS)
//     i <  j:  U_ij = W_i^T acc                     (one K = 128 product)
// and the task of right-hand-side tile (i, c) the same with B's column block c in place of
// A's column block j.  A tile is written by its task only, and read by other tasks only
// after it is final, so no XCD's L2 or CU's L1 can hold a stale copy of data another
// workgroup reads: final tiles (and W_i) are stored with sc1 (write-through; the line leaves
// the writer's L2), then a per-column progress counter is raised with an sc1 store after
// the stores drained (the MI355X guide's sc1 hand-off: no L2 write-back, no L1 invalidate).
// colprog[j] = number of final tiles at the top of column block j of A (tiles (0..p-1, j));
// rhsprog[c] likewise for B.  Column tiles finalise top-down, so one counter per column
// suffices; a task accumulates row blocks as their tiles become final (k < min(colprog[i],
// colprog[j])), so only its last row block waits for the previous row.
//
// Scheduling: one workgroup per CU (128 KB of LDS: four 32-KB DMA stages of the GEMM
// pipeline, or the diagonal block), tasks claimed from an atomic ticket in a host-built
// topological order (row i of A's tiles, then row i of B's tiles, for i = 0, 1, ...): every
// tile a task waits for belongs to an earlier ticket, i.e. to a workgroup that is already
// running, so the grid cannot deadlock whatever the residency.  Every wait is bounded
// (~seconds): on timeout the launch flags info = -1 and every task still publishes, so the
// grid always drains.  A non-positive pivot sets info (first failure wins; later pivots
// depend on it) and the remaining tasks skip their arithmetic.
//
// Conditions (checked by the host): tiles of 128, n % 16 == 0, lda % 16 == 0 (and ldb),
// 128-B aligned bases -- every 128-B line then belongs to exactly one tile.
#include <algorithm>
#include <cstdint>

#include "common.hpp"

#ifdef DAG_TRACE
// diagnostic build: the diagonal factor's phases (band sb elimination: 2 sb, its trailing
// update: 2 sb + 1, the inverse: 7; realtime ticks summed over the launch's diagonal tasks)
__device__ unsigned long long g_diag_ph[16];
#define DSTAMP_INIT() unsigned long long _dst_t = __builtin_amdgcn_s_memrealtime()
#define DSTAMP(i)                                                   \
  do {                                                              \
    __syncthreads();                                                \
    if (threadIdx.x == 0) {                                         \
      const unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
      atomicAdd(&g_diag_ph[i], _t - _dst_t);                        \
      if ((i) == 7) atomicAdd(&g_diag_ph[8], 1ull);                 \
      _dst_t = _t;                                                  \
    }                                                               \
  } while (0)
// wave 0 only, no barrier (inside the band elimination): 9 loads, 10 elimination, 11 stores
#define DSTAMPW(i)                                                  \
  do {                                                              \
    const unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
    if (threadIdx.x == 0) atomicAdd(&g_diag_ph[i], _t - _dst_t);    \
    _dst_t = _t;                                                    \
  } while (0)
extern "C" void gpr_debug_diag_phases(unsigned long long* out, int reset) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_ph), sizeof(unsigned long long) * 16);
  if (reset) {
    unsigned long long z[16] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_diag_ph), z, sizeof z);
  }
}
#endif

#include "diag_block.hpp"

#ifdef DAG_TRACE
// diagnostic build only (tools/probe/dag_probe): per-workgroup progress words
__device__ int g_dag_trace[4096];
#define DTRACE(slot, v)                                                                   \
  do {                                                                                    \
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)                            \
      __hip_atomic_store(&g_dag_trace[blockIdx.x * 8 + (slot)], (v), __ATOMIC_RELAXED,     \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                      \
  } while (0)
extern "C" void gpr_debug_dag_trace(int* out, void* stream) {
  hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_dag_trace), sizeof(int) * 4096, 0,
                           hipMemcpyDeviceToHost, (hipStream_t)stream);
  hipStreamSynchronize((hipStream_t)stream);
}
// phase timers (100 MHz realtime ticks), summed per workgroup into trace slots 2..7
#define PROF(var, ...)                                  \
  do {                                                  \
    const unsigned long long _t0 = __builtin_amdgcn_s_memrealtime(); \
    __VA_ARGS__;                                        \
    var += __builtin_amdgcn_s_memrealtime() - _t0;      \
  } while (0)
#else
#define DTRACE(slot, v) \
  do {                  \
  } while (0)
#define PROF(var, ...) \
  do {                 \
    __VA_ARGS__;       \
  } while (0)
#endif

namespace {

constexpr int DT = 128;                     // tile edge
constexpr int DTK = 16;                     // K rows per pipeline stage
#ifndef DAG_DPB
#define DAG_DPB 4
#endif
constexpr int DPB = DAG_DPB;                // LDS stages (DMA DPB - 1 stages ahead)
constexpr int DSTAGE = (DT + DT) * DTK;     // doubles per stage (P image, then Q)
constexpr int DLDS = DPB * DSTAGE;          // 16384 doubles = 128 KB at DPB = 4
// the task loop's three LDS ints: after the stages when they fit in the 160 KB, else in the
// last stage's final 16 bytes -- they are live only between accumulations (every dag_accum
// ends with a barrier after its last LDS read; the ints are read before the next one starts)
constexpr int DINT = (DLDS + 2) * 8 <= 160 * 1024 ? DLDS : DLDS - 2;
constexpr int DALLOC = DINT + 2;
constexpr int DNCH = DTK / 2;               // 16-B chunks per LDS row
constexpr int DRPD = 64 / DNCH;             // rows per wave-wide 1-KB DMA
constexpr int DNDMA = DT / (4 * DRPD);      // DMA instructions per wave per operand
constexpr int DVM = 2 * DNDMA;              // vmcnt increments per stage
constexpr int DNP = DTK / 8;                // fragment blocks (2 k-steps each) per stage
static_assert(D2_LDS_QTAIL <= DLDS, "diagonal block must fit in the stage buffers");

typedef double d2 __attribute__((ext_vector_type(2)));

struct DagArgs {
  double* A;
  size_t lda;
  int n, nt;
  double* B;  // optional right-hand sides (n x nrhs, ld ldb)
  size_t ldb;
  int nrhs, ntr;
  double* winv;  // W_i = U_ii^{-1} in slot i (128 x 128)
  int kglob;     // global index of row 0 (reported pivot orders)
  int* info;
  int* sync;     // [0] ticket, [2 + j] colprog[j], [2 + nt + c] rhsprog[c]
  int* ustored;  // optional (a launch hook reads U while the launch runs): ustored[i] = 1 once
                 // U_ii's (post-publish) store has drained -- colprog alone does not cover it
  const unsigned* tasks;
  int ntasks;
  int lower;     // B is lower triangular (the identity's solve Z = U^{-T}): tile (i, c) exists
                 // for i >= c only and accumulates row blocks [c, i)
  double* G;     // optional (lower B only): G += B^T B, upper tiles (i <= j), ld ldg --
  size_t ldg;    // K^{-1} = Z^T Z; tickets >= gbase are these tiles
  int gbase;
  long long spin_limit;  // polls before a wait gives up (~4 s at 2^25; GPR_DAG_SPIN_LIMIT, tests)
  int mirror;  // DAG_MIRROR: off-diagonal tasks store their loaded A_ij, transposed, at (j, i)
  // batched launches (launch_potrf_dag_batch): task t belongs to matrix tbatch[t], whose A, B,
  // W slots, progress counters and info word sit at these strides from the base pointers (the
  // ticket stays a.sync[0])
  const int* tbatch;
  size_t strA, strB, strW;
  int strS;
};

__device__ __forceinline__ int ld_sc1(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int VM>
__device__ __forceinline__ void dag_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
}

__device__ __forceinline__ int dag_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int dag_idx(int row, int chunk) {
  return row * DTK + ((chunk ^ dag_swz(row)) << 1);
}

// acc[i][j][r] += sum_{k < 16 nst} P[k + m ldp] Q[k + n ldq] for the tile element
// (m, n) = (64 wm + 16 j + (lane & 15), 64 wn + 16 i + (lane >> 4) + 4 r)  (gemm.hip's layout:
// the Q fragment is the MFMA A operand).  Rows m >= mv / n >= nv are clamped (their results
// are never stored).  The pipelined gemm.hip body at one workgroup per CU: four LDS stages
// fed by LDS-DMA (global_load_lds_dwordx4, swizzle applied on the source address), DMA three
// stages ahead, next stage's fragments read during the current stage's MFMAs.  Leaves the
// LDS free (ends with a barrier).
//
// TRI (the W-products U_ij = W_i^T B, K = 128, P = W_i upper triangular: P[k + m ldp] = 0 for
// k > m): stage s (k in [16 s, 16 s + 16)) only feeds the 16-row blocks mb >= s of the result,
// so the MFMAs of the others are skipped.  The two wave rows take interleaved row blocks --
// wm = 0: {0, 3, 4, 7}, wm = 1: {1, 2, 5, 6}, 18 block-stages each -- instead of halves (10 and
// 26), so the waves stay balanced: 20 of 32 stage-slots of MFMA work per wave, with the same
// accumulators and fragment registers.  Element (m, n) of acc[i][j][r]: m = 16 dag_mblk(wm, j)
// + (lane & 15).
__device__ __forceinline__ int dag_mblk(int wm, int j) {
  return 4 * (j >> 1) + (wm ? 1 + (j & 1) : 3 * (j & 1));
}

template <bool TRI = false>
__device__ __forceinline__ void dag_accum(d4v (&acc)[4][4], const double* __restrict__ P,
                                          size_t ldp, int mv, const double* __restrict__ Q,
                                          size_t ldq, int nv, int nst, double* lds) {
  if (nst <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  const double* srcP[DNDMA];
  const double* srcQ[DNDMA];
#pragma unroll
  for (int r = 0; r < DNDMA; ++r) {
    const int row = DRPD * (4 * r + w) + lane / DNCH;
    const int c = (lane % DNCH) ^ dag_swz(row);
    srcP[r] = P + 2 * c + (size_t)min(row, mv - 1) * ldp;
    srcQ[r] = Q + 2 * c + (size_t)min(row, nv - 1) * ldq;
  }
  auto issue = [&](int s) {
    double* base = lds + (s % DPB) * DSTAGE;
    const size_t ko = (size_t)min(s, nst - 1) * DTK;
#pragma unroll
    for (int r = 0; r < DNDMA; ++r) {
      __builtin_amdgcn_global_load_lds(srcP[r] + ko, base + (4 * r + w) * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(srcQ[r] + ko, base + DT * DTK + (4 * r + w) * 128, 16, 0, 0);
    }
  };
  auto read_frags = [&](d2 (&F)[DNP][8], int s) {
    const double* ps = lds + (s % DPB) * DSTAGE;
    const double* qs = ps + DT * DTK;
#pragma unroll
    for (int p = 0; p < DNP; ++p) {
      const int ch = (lane >> 4) + 4 * p;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        F[p][i] = *reinterpret_cast<const d2*>(&qs[dag_idx(wn * 64 + i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int mrow = TRI ? 16 * dag_mblk(wm, j) : wm * 64 + j * 16;
        F[p][4 + j] = *reinterpret_cast<const d2*>(&ps[dag_idx(mrow + (lane & 15), ch)]);
      }
    }
  };
  auto mfma_stage = [&](const d2 (&F)[DNP][8], int s) {
    (void)s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (TRI && dag_mblk(wm, j) < s) continue;  // (wave-uniform: W_i's zeros)
#pragma unroll
      for (int p = 0; p < DNP; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[p][i][h], F[p][4 + j][h], acc[i][j], 0, 0, 0);
    }
  };
  auto step = [&](int s, d2 (&Fc)[DNP][8], d2 (&Fn)[DNP][8]) {
    // keep the previous stage's MFMAs ahead of this barrier: issued just before it, they run
    // while the wave waits there (sunk past it, the matrix pipe idles through the wait)
    __builtin_amdgcn_sched_barrier(0);
    // the previous step's fragment reads retired before the barrier lets other waves' DMA
    // overwrite that stage (waited here, after the step's last MFMAs, not right behind them)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
    dag_vmcnt<DVM * (DPB - 3)>();  // own DMA of stage s+1 retired, s+2.. still in flight
    __builtin_amdgcn_s_barrier();
    issue(s + DPB - 1);
    read_frags(Fn, s + 1);
    mfma_stage(Fc, s);
    if constexpr (TRI) return;  // (variable MFMA counts: the compiler's own order)
// instruction order inside a stage (same-box C3 DAG launch, profiles/r02e_ab_dag_sched_
// variants.txt): 0 (default) 299.8 ms, 1 300.1, 2 313.6, 3 314.1
#ifndef DAG_SCHED
#define DAG_SCHED 0
#endif
#if DAG_SCHED == 0
#pragma unroll
    for (int t = 0; t < DVM; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
#pragma unroll
    for (int t = 0; t < 8 * DNP; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32 * DNP - DVM - 16 * DNP, 0);
#elif DAG_SCHED == 1  // DMA spread over twice as many MFMAs
#pragma unroll
    for (int t = 0; t < DVM; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
#pragma unroll
    for (int t = 0; t < 8 * DNP; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32 * DNP - 2 * DVM - 16 * DNP, 0);
#elif DAG_SCHED == 2  // fragment reads first, then the DMA
#pragma unroll
    for (int t = 0; t < 8 * DNP; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
#pragma unroll
    for (int t = 0; t < DVM; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32 * DNP - 2 * DVM - 8 * DNP, 0);
#endif  // DAG_SCHED == 3: the compiler's own order
  };
  d2 F0[DNP][8], F1[DNP][8];
#pragma unroll
  for (int t = 0; t < DPB - 1; ++t) issue(t);
  dag_vmcnt<DVM * (DPB - 2)>();
  __builtin_amdgcn_s_barrier();
  read_frags(F0, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  int s = 0;
  for (; s + 1 < nst; s += 2) {
    step(s, F0, F1);
    step(s + 1, F1, F0);
  }
  if (s < nst) mfma_stage(F0, s);
  dag_vmcnt<0>();
  __syncthreads();
}

// Control flow around barriers must be WAVE-UNIFORM: a thread-0-only region (exec-masked)
// next to the barriers of the task loop was structurised by the compiler so that the publish
// store ran under a mask no lane satisfied and the grid hung.  So every "one lane" action
// below is done by all 64 lanes of wave 0 behind a scalar branch on the wave index (same
// value to the same address), and values steering branches are readfirstlane'd.

// Block until min(pa, pb) > have (wave 0 polls with sc1 loads, sleeping between polls);
// returns min(pa, pb, cap), uniform across the workgroup.  Bounded: after ~2^25 polls the
// launch is flagged (info = -1) and the wait returns cap (results are garbage, the grid drains).
__device__ __forceinline__ int dag_wait(const int* pa, const int* pb, int have, int cap,
                                        int* info, long long limit, int* sh) {
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    int v = 0;
    long long spins = 0;
    for (;;) {
      v = __builtin_amdgcn_readfirstlane(min(ld_sc1(pa), ld_sc1(pb)));
      if (v > have) break;
      if (++spins > limit) {
        atomicCAS(info, 0, -1);
        v = cap;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    *sh = min(v, cap);
  }
  // no instruction: keeps the compiler from hoisting the data loads above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  __syncthreads();
  const int r = __builtin_amdgcn_readfirstlane(*sh);
  __syncthreads();  // *sh may be rewritten by the next wait
  return r;
}

// stores of the drained task become visible before the counter: every storing wave waits
// for its stores, then wave 0 raises the counter (sc1)
__device__ __forceinline__ void dag_publish(int* prog, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)
    __hip_atomic_store(prog, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The F task's factorisation, out of line: inlined, its readlane-heavy elimination (SGPR
// spills into VGPR lanes) shares the allocation with the GEMM pipeline's live state and
// spilled to scratch; as a call it is allocated on its own.
// (U_ii itself is NOT stored here: no task of the launch reads a diagonal tile -- every
// accumulation takes U_ki with k < i, the off-diagonal and right-hand-side tiles take W_i -- so
// the task publishes once W_i is out and stores U_ii afterwards, off the chain: dag_store_u)
__device__ __attribute__((noinline)) int dag_factor(double* S, int mv, int kglob, double* winv) {
  lds_d* L = (lds_d*)S;  // (one conversion; see diag_block.hpp)
  lds_d(*Xd)[D2_PB] = reinterpret_cast<lds_d(*)[D2_PB]>(L + D2_PK);
  lds_i* fail = reinterpret_cast<lds_i*>(L + D2_PK + 4 * D2_PB);
  return diag2_core<true, true>(L, Xd, fail, nullptr, 0, mv, kglob, winv);
}

// (sc1: a launch hook's kernel reads U_ii on another stream while the launch runs -- a plain
// store would sit in this XCD's L2 until the launch ends)
__device__ __attribute__((noinline)) void dag_store_u(const double* S, double* T, size_t lda, int mv,
                                                      bool sc1) {
  const lds_d* L = (const lds_d*)S;
  if (sc1)
    diag2_store_u<true>(L, T, lda, mv);
  else
    diag2_store_u<false>(L, T, lda, mv);
}

// A gram task: K^{-1} = Z^T Z tile (i, j), i <= j.  Inlined into the GRAM instance of the
// kernel only (out of line, the calls' register saves slowed every task by ~2 %; inlined
// into the one kernel, its second copy of the pipeline cost the plain factorisation ~0.3 %)
__device__ __forceinline__ void dag_gram_task(const DagArgs& a, int i_, int j_,
                                                        double* lds, int* s_wait,
                                                        unsigned long long& p_wait,
                                                        unsigned long long& p_acc) {
  (void)p_wait;
  (void)p_acc;
  // (values steering the loop around the barriers are readfirstlane'd: see the kernel)
  const int i = __builtin_amdgcn_readfirstlane(i_), j = __builtin_amdgcn_readfirstlane(j_);
  const int n = __builtin_amdgcn_readfirstlane(a.n), nt = __builtin_amdgcn_readfirstlane(a.nt);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  const int* rhsprog = a.sync + 2 + nt;
  double* T = a.G + (size_t)i * DT + (size_t)j * DT * a.ldg;
  const int mv = min(DT, n - i * DT), nv = min(DT, n - j * DT);
  d4v acc[4][4];
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = d4v{0.0, 0.0, 0.0, 0.0};
  const double* Pcol = a.B + (size_t)i * DT * a.ldb;
  const double* Qcol = a.B + (size_t)j * DT * a.ldb;
  int done = j;
  while (done < nt) {
    int r = 0;
    PROF(p_wait, r = dag_wait(rhsprog + i, rhsprog + j, done, nt, a.info, a.spin_limit, s_wait));
    const int nst = (min(r * DT, n) - done * DT) / DTK;  // (the last block may be short)
    PROF(p_acc, dag_accum(acc, Pcol + (size_t)done * DT, a.ldb, mv, Qcol + (size_t)done * DT, a.ldb,
                          nv, nst, lds));
    done = r;
  }
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int mm = wm * 64 + jj * 16 + (lane & 15);
        if (mm < mv && nn < nv && (i != j || mm <= nn))
          T[(size_t)mm + (size_t)nn * a.ldg] = acc[ii][jj][r];
      }
    }
  // the mirror (a diagonal tile's strict lower half from its own upper half, so G is
  // exactly symmetric): each store covers 32 B of 16 columns, and the 4 values of r
  // fill 128-B lines that the L2 merges before write-back
  double* Tm = a.G + (size_t)j * DT + (size_t)i * DT * a.ldg;
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
        const int mm = wm * 64 + jj * 16 + (lane & 15);
        if (mm < mv && nn < nv && (i != j || mm < nn))
          Tm[(size_t)nn + (size_t)mm * a.ldg] = acc[ii][jj][r];
      }
}

template <bool GRAM, bool BATCH>
__global__ __launch_bounds__(256, 1) void potrf_dag_kernel(DagArgs a0) {
  DagArgs a = a0;  // (BATCH: re-pointed at each task's matrix)
  // ONE LDS variable: with separate __shared__ scalars the accesses get alias scopes, and
  // the waitcnt pass then made every fragment read wait for ALL in-flight LDS-DMA (an
  // s_waitcnt vmcnt(0) per stage: the DMA never ran ahead; accumulation at 0.23 instead of
  // ~0.28 TF/s per CU)
  __shared__ double lds[DALLOC];
  int& s_task = reinterpret_cast<int*>(lds + DINT)[0];
  int& s_skip = reinterpret_cast<int*>(lds + DINT)[1];
  int& s_wait = reinterpret_cast<int*>(lds + DINT)[2];
  int s_fok = 0;  // this diagonal task factored its tile (uniform)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  int* colprog = a.sync + 2;
  int* rhsprog = colprog + a.nt;
  unsigned long long p_wait = 0, p_acc = 0, p_fac = 0, p_tri = 0, p_all = 0, p_n = 0;
#ifdef DAG_PROF_PUB
  unsigned long long p_pub = 0, p_tri_unused = 0;
#define p_tri p_tri_unused
#endif
  (void)p_wait; (void)p_acc; (void)p_fac; (void)p_tri; (void)p_all; (void)p_n;
#ifdef DAG_TRACE
  const unsigned long long p_start = __builtin_amdgcn_s_memrealtime();
#endif
  for (;;) {
    if (w == 0) {  // one ticket: lane 0 adds 1, the other lanes 0 (a wave-wide atomic)
      const int tk = atomicAdd(&a0.sync[0], lane == 0 ? 1 : 0);
      const int tk0 = __builtin_amdgcn_readlane(tk, 0);
      s_task = tk0;
      if (!BATCH) {
        s_skip = __builtin_amdgcn_readfirstlane(ld_sc1(a.info)) != 0;
      } else if (tk0 < a0.ntasks) {
        const int b = __builtin_amdgcn_readfirstlane(a0.tbatch[tk0]);
        s_skip = __builtin_amdgcn_readfirstlane(ld_sc1(a0.info + b)) != 0;
      }
    }
    __syncthreads();
    // wave-uniform (SGPR) copies: the loop exit and every branch around the barriers below
    // must be provably uniform, or the compiler structurises them as divergent and the
    // thread-0 publish ends up under a mask no lane satisfies (observed: the grid hangs)
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    const bool skip = __builtin_amdgcn_readfirstlane(s_skip);
    DTRACE(0, t);
    DTRACE(1, 1);
    if (t >= a.ntasks) break;
    if (BATCH) {
      const int b = __builtin_amdgcn_readfirstlane(a0.tbatch[t]);
      a.A = a0.A + (size_t)b * a0.strA;
      a.B = a0.B + (size_t)b * a0.strB;
      a.winv = a0.winv + (size_t)b * a0.strW;
      a.info = a0.info + b;
      colprog = a0.sync + (size_t)b * a0.strS + 2;
      rhsprog = colprog + a.nt;
    }
    const unsigned code = __builtin_amdgcn_readfirstlane(a.tasks[t]);  // (a vector load)
    if (GRAM && t >= a.gbase) {
      // G_ij = sum_{k >= j} B_ki^T B_kj (i <= j; B lower triangular, so row blocks k < j
      // of B_kj vanish), row blocks taken as both columns of B finalise them; written to
      // tile (i, j) and, transposed, to (j, i); no one waits for G, so nothing is published
      if (!skip) dag_gram_task(a, (code >> 16) & 0x7fff, code & 0xffff, lds, &s_wait, p_wait, p_acc);
      ++p_n;
      __syncthreads();  // every wave has read s_task before wave 0 takes the next ticket
      continue;
    }
    const bool rhs = code >> 31;
    const int i = (code >> 16) & 0x7fff, j = code & 0xffff;
    const bool diag = !rhs && i == j;
    double* T = rhs ? a.B + (size_t)i * DT + (size_t)j * DT * a.ldb
                    : a.A + (size_t)i * DT + (size_t)j * DT * a.lda;
    const size_t ldt = rhs ? a.ldb : a.lda;
    const double* Qcol = rhs ? a.B + (size_t)j * DT * a.ldb : a.A + (size_t)j * DT * a.lda;
    const double* Pcol = a.A + (size_t)i * DT * a.lda;
    int* pj = rhs ? rhsprog + j : colprog + j;
    const int mv = min(DT, a.n - i * DT);                        // rows of the tile
    const int nv = min(DT, (rhs ? a.nrhs : a.n) - j * DT);       // columns of the tile
    if (!skip) {
      // acc = -T (the result is -acc after the accumulation), branch-free clamped loads
      d4v acc[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
          const double* col = T + (size_t)min(nn, nv - 1) * ldt;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int mm = wm * 64 + jj * 16 + (lane & 15);
            const double c = col[min(mm, mv - 1)];
            acc[ii][jj][r] = (mm < mv && nn < nv) ? -c : 0.0;
          }
        }
      // DAG_MIRROR: the K assembly left the strict lower triangle to this launch -- the loaded
      // tile, transposed, into tile (j, i) (K there, as dpotrf 'U' leaves it).  Lanes with one
      // (lane & 15) store 32 contiguous bytes of one column per register r; the four r fill a
      // 128-B line, which the L2 merges before writing back.  Nothing in the launch reads it.
      if (a.mirror && !rhs && !diag) {
        double* Tm = a.A + (size_t)j * DT + (size_t)i * DT * a.lda;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
              const int mm = wm * 64 + jj * 16 + (lane & 15);
              if (mm < mv && nn < nv) Tm[(size_t)nn + (size_t)mm * a.lda] = -acc[ii][jj][r];
            }
      }
      // acc += sum_{k<i} U_ki^T X_kj, row blocks taken as soon as both columns have them final
      DTRACE(1, 2);
      int done = (rhs && a.lower) ? j : 0;
      while (done < i) {
        int r = 0;
        PROF(p_wait, r = dag_wait(colprog + i, pj, done, i, a.info, a.spin_limit, &s_wait));
        PROF(p_acc, dag_accum(acc, Pcol + (size_t)done * DT, a.lda, mv, Qcol + (size_t)done * DT,
                              ldt, nv, (r - done) * (DT / DTK), lds));
        done = r;
      }
      if (diag) {
        // factor -acc in LDS (packed upper, identity padding beyond mv), U_ii and W_i out (sc1)
        double* S = lds;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int mm = wm * 64 + jj * 16 + (lane & 15);
              if (mm <= nn) S[pk(mm, nn)] = nn < mv ? -acc[ii][jj][r] : (mm == nn ? 1.0 : 0.0);
            }
          }
        __syncthreads();
        DTRACE(1, 3);
        int f = 0;
        PROF(p_fac, f = dag_factor(S, mv, a.kglob + i * DT, a.winv + (size_t)i * DT * DT));
        if (f && w == 0) atomicCAS(a.info, 0, f);
        s_fok = f == 0;
        DTRACE(1, 4);
      } else {
        // B_ij = -acc into the tile (own tile: only this workgroup reads it back), then
        // U_ij = W_i^T B_ij once W_i is final
        if (i > 0) {  // (row 0: acc = -A_0j exactly, nothing to write)
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                const int mm = wm * 64 + jj * 16 + (lane & 15);
                if (mm < mv && nn < nv) T[(size_t)mm + (size_t)nn * ldt] = -acc[ii][jj][r];
              }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        PROF(p_wait, dag_wait(colprog + i, colprog + i, i, i + 1, a.info, a.spin_limit, &s_wait));  // W_i final
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = d4v{0.0, 0.0, 0.0, 0.0};
        // (full tiles: the triangular form; the last tile row, mv < 128, the plain one)
        const bool tri = mv == DT;
        if (tri)
          PROF(p_tri, dag_accum<true>(acc, a.winv + (size_t)i * DT * DT, DT, mv, T, ldt, nv, DT / DTK, lds));
        else
          PROF(p_tri, dag_accum(acc, a.winv + (size_t)i * DT * DT, DT, mv, T, ldt, nv, mv / DTK, lds));
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = wn * 64 + ii * 16 + (lane >> 4) + 4 * r;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int mm = (tri ? 16 * dag_mblk(wm, jj) : wm * 64 + jj * 16) + (lane & 15);
              if (mm < mv && nn < nv) st_res<true>(&T[(size_t)mm + (size_t)nn * ldt], acc[ii][jj][r]);
            }
          }
      }
    } else if (a.mirror && !rhs && !diag) {
      // a skipped task (a pivot failed: dpotrf stops there) still owes the strict lower tile
      // its K values -- its own upper tile was written by no one, so it still holds A_ij
      double* Tm = a.A + (size_t)j * DT + (size_t)i * DT * a.lda;
      for (int e = tid; e < DT * DT; e += 256) {
        const int mm = e & (DT - 1), nn = e >> 7;
        if (mm < mv && nn < nv) Tm[(size_t)nn + (size_t)mm * a.lda] = T[(size_t)mm + (size_t)nn * ldt];
      }
    }
    DTRACE(1, 5);
#ifdef DAG_PROF_PUB
    // (probe build: the "trsm" slot times the diagonal tasks' publish -- W_i's store drain)
    if (diag) PROF(p_pub, dag_publish(pj, i + 1)); else dag_publish(pj, i + 1);
#else
    dag_publish(pj, i + 1);
#endif
    DTRACE(1, 6);
    // U_ii after the publish (read by later launches only; the LDS still holds it)
    if (diag && !skip && __builtin_amdgcn_readfirstlane(s_fok))
      dag_store_u(lds, T, a.lda, mv, a.ustored != nullptr);
    // ... and by a launch hook's readers (the streamed broadcast's row gates): they wait for
    // ustored[i] too, raised once the (then write-through) store drained -- also after a
    // failure, so no gate waits out its limit; the host reports the error
    if (diag && a.ustored) dag_publish(a.ustored + i, 1);
    ++p_n;
  }
  DTRACE(1, 7);
#ifdef DAG_TRACE
  p_all = __builtin_amdgcn_s_memrealtime() - p_start;
  DTRACE(2, (int)p_wait);
  DTRACE(3, (int)p_acc);
  DTRACE(4, (int)p_fac);
#ifdef DAG_PROF_PUB
#undef p_tri
  DTRACE(5, (int)p_pub);
  (void)p_tri_unused;
#else
  DTRACE(5, (int)p_tri);
#endif
  DTRACE(6, (int)p_all);
  DTRACE(7, (int)p_n);
#endif
}

}  // namespace

// Progress counters of a launch that starts from a finished factor (DAG_SOLVE: every tile of
// U final, colprog[j] = j + 1) and/or a lower-triangular B (DAG_LOWER: tiles (k < c, c) of B
// are the identity's zeros, final from the start: rhsprog[c] = c).
__global__ void dag_init_kernel(int* sync, int nt, int ntr, int solve, int lower) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt + ntr; t += gridDim.x * blockDim.x)
    sync[2 + t] = t < nt ? (solve ? t + 1 : 0) : (lower ? t - nt : 0);
}

// Bound on every dependency wait of a launch, in polls (~4 s).  Test builds only
// (libgpr_hip_testing.so) let GPR_DAG_SPIN_LIMIT shorten it per launch, so the timeout tests
// can force the bound to expire around one call.
static long long dag_spin_limit(const gpr_ctx* ctx) {
#ifdef GPR_TESTING
  if (const char* sl = getenv("GPR_DAG_SPIN_LIMIT")) return std::max(1ll, atoll(sl));
#endif
  return ctx->dag_spin_limit;
}

// The launch's own shape conditions: every 128-B line belongs to one tile (leading dimensions
// multiples of 16 doubles, 128-B aligned bases) and every K range is a multiple of the 16-row
// pipeline stage (n % 16 == 0).
bool dag_shape_ok(int n, int lda, const double* dA) {
  return n > 0 && n % 16 == 0 && lda % 16 == 0 && ((uintptr_t)dA & 127) == 0 && n <= DT * 32767;
}

// true when potrf_core factors (n, lda, dA) as one tile-DAG launch: directly, or for any other
// shape through a padded copy (dag_padded)
bool dag_takes_whole(const gpr_ctx* ctx, int n, int lda, const double* dA) {
  (void)lda;
  (void)dA;
  return ctx->dag_mode && ctx->nb == DT && n > 0 &&
         n <= DT * 32767 - 16;
}

// upper triangle of A (n x n, ld lda) into W (n2 x n2, ld n2), identity beyond n: the padded
// matrix [[A, 0], [0, I]] has the factor [[U, 0], [0, I]] and the same block inverses on its
// first n rows, and the tile-DAG's arithmetic on the first n rows is unchanged by the padding
__global__ void dag_pad_in_kernel(const double* __restrict__ A, size_t lda, int n,
                                  double* __restrict__ W, int n2) {
  const size_t tot = (size_t)n2 * n2;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(t % n2), c = (int)(t / n2);
    if (r <= c) W[t] = c < n ? A[(size_t)r + (size_t)c * lda] : (r == c ? 1.0 : 0.0);
  }
}

// U (upper, first n rows / columns of W) back into A; A's strict lower triangle untouched
__global__ void dag_pad_out_kernel(double* __restrict__ A, size_t lda, int n,
                                   const double* __restrict__ W, int n2) {
  const size_t tot = (size_t)n * n;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(t % n), c = (int)(t / n);
    if (r <= c) A[(size_t)r + (size_t)c * lda] = W[(size_t)r + (size_t)c * n2];
  }
}

// The factorisation (and B <- U^{-T} B) of a shape the launch does not take directly, on a
// padded copy: n2 = n rounded up to 16, ld n2.  Costs one read + write of the upper triangle
// each way (and of B); returns 1 when the workspace cannot be allocated (caller falls back).
int launch_potrf_dag_padded(gpr_ctx* ctx, double* dA, int n, int lda, double* dB, int nrhs,
                            int ldb) {
  const int n2 = (n + 15) / 16 * 16;
  hipStream_t st = ctx->stream;
  if (ensure_buf(ctx, &ctx->dpadA, &ctx->padA_cap, (size_t)n2 * n2) != 0 ||
      (dB && ensure_buf(ctx, &ctx->dpadB, &ctx->padB_cap, (size_t)n2 * nrhs) != 0)) {
    ctx->err.clear();
    (void)hipGetLastError();  // do not leave the allocation failure for the next launch check
    return 1;
  }
  const int blocks = 2048;
  dag_pad_in_kernel<<<blocks, 256, 0, st>>>(dA, (size_t)lda, n, ctx->dpadA, n2);
  LAUNCH_CHECK(ctx);
  if (dB) {
    HIP_TRY(ctx, hipMemcpy2DAsync(ctx->dpadB, (size_t)n2 * sizeof(double), dB,
                                  (size_t)ldb * sizeof(double), (size_t)n * sizeof(double), nrhs,
                                  hipMemcpyDeviceToDevice, st));
    if (n2 > n)
      HIP_TRY(ctx, hipMemset2DAsync(ctx->dpadB + n, (size_t)n2 * sizeof(double), 0,
                                    (size_t)(n2 - n) * sizeof(double), nrhs, st));
  }
  const int rc = launch_potrf_dag(ctx, ctx->dpadA, n2, n2, dB ? ctx->dpadB : nullptr, nrhs, n2, 0,
                                  st, 0);
  if (rc) return rc < 0 ? rc : set_err(ctx, GPR_E_HIP, "padded tile-DAG: shape not eligible");
  dag_pad_out_kernel<<<blocks, 256, 0, st>>>(dA, (size_t)lda, n, ctx->dpadA, n2);
  LAUNCH_CHECK(ctx);
  if (dB)
    HIP_TRY(ctx, hipMemcpy2DAsync(dB, (size_t)ldb * sizeof(double), ctx->dpadB,
                                  (size_t)n2 * sizeof(double), (size_t)n * sizeof(double), nrhs,
                                  hipMemcpyDeviceToDevice, st));
  return 0;
}

// Factor A (n x n, ld lda) in place and, when B != nullptr, B <- U^{-T} B (n x nrhs, ld ldb),
// in one launch on st.  Writes W_i into ctx->winv slots (block inverses for the solves).
// kglob: global index of A's first row/column (the trailing matrix of a blocked factorisation:
// block inverses go to winv slots kglob/128 + i, pivot orders are global).  flags: DAG_SOLVE
// (A already holds U and winv its block inverses: only B's tiles are tasks), DAG_LOWER (B is
// lower triangular, e.g. the identity).  Returns 1 when the shape does not qualify (caller
// falls back), 0 when launched.
int launch_potrf_dag(gpr_ctx* ctx, double* dA, int n, int lda, double* dB, int nrhs, int ldb,
                     int kglob, hipStream_t st, int flags, double* dG, int ldg) {
  const bool solve = flags & DAG_SOLVE, lower = flags & DAG_LOWER, gram = flags & DAG_GRAM;
  const bool mirror = flags & DAG_MIRROR;
  if ((solve || lower) && (!dB || kglob)) return 1;
  if (mirror && (solve || kglob)) return 1;
  if (gram && (!lower || !dG || ldg < n || nrhs != n)) return 1;
  if (ctx->nb != DT || n <= 0 || n % 16 || lda % 16 || ((uintptr_t)dA & 127) || n > DT * 32767 ||
      kglob % DT)
    return 1;
  if (dB && (nrhs <= 0 || ldb % 16 || ((uintptr_t)dB & 127) || nrhs > DT * 65535)) return 1;
  const int nt = (n + DT - 1) / DT, ntr = dB ? (nrhs + DT - 1) / DT : 0;
  GPR_TRY(ensure_winv(ctx, kglob + n, DT));
  if (ctx->dag_nt != nt || ctx->dag_ntr != ntr || ctx->dag_flags != (flags & ~DAG_MIRROR) ||
      ctx->dag_lag_built != ctx->dag_zlag) {
    std::vector<unsigned> tasks;
    tasks.reserve((size_t)nt * (nt + 1) + (size_t)nt * ntr);
    // right-hand-side row i after A's row i + lag: a lower-triangular B's tiles (i, c) near
    // the diagonal accumulate only i - c row blocks and would otherwise sit waiting for W_i
    // (the diagonal task of the same row, still accumulating i blocks); the order stays
    // topological (every dependency of a task has an earlier ticket)
    // (a lag for the other right-hand sides, 1, 2 or 4 rows, measured no faster for C2 / C3)
    const int lag = solve || !lower ? 0 : std::min(ctx->dag_zlag, nt);
    auto rhs_row = [&](int i) {
      for (int c = 0; c < (lower ? std::min(ntr, i + 1) : ntr); ++c)
        tasks.push_back(0x80000000u | ((unsigned)i << 16) | (unsigned)c);
    };
    // (the diagonal task F(i + 1) right behind T(i, i + 1) instead of behind all of row i
    // measured within 0.1-0.4 % either way for C2 / C3 / C4, so row order it is)
    for (int i = 0; i < nt; ++i) {
      if (!solve)
        for (int j = i; j < nt; ++j) tasks.push_back(((unsigned)i << 16) | (unsigned)j);
      if (i - lag >= 0) rhs_row(i - lag);
    }
    for (int i = std::max(nt - lag, 0); i < nt; ++i) rhs_row(i);
    // G's upper tiles last, by column: G_ij sums B's row blocks k >= j, so the low columns
    // (the longest sums, whose first blocks are final earliest) go first
    if (gram)
      for (int j = 0; j < nt; ++j)
        for (int i = 0; i <= j; ++i) tasks.push_back(((unsigned)i << 16) | (unsigned)j);
    // a previous launch on this context may still be reading the old list (a factorisation
    // launch returns without synchronising; a solve-only launch syncs to read its info, but
    // the list may belong to a factorisation): drain the context's stream before freeing it
    if (ctx->dag_tasks) {
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (every DAG launch joins it)
      HIP_TRY(ctx, hipFree(ctx->dag_tasks));
    }
    ctx->dag_tasks = nullptr;
    ctx->dag_nt = ctx->dag_ntr = -1;
    HIP_TRY(ctx, hipMalloc((void**)&ctx->dag_tasks, tasks.size() * sizeof(unsigned)));
    HIP_TRY(ctx, hipMemcpy(ctx->dag_tasks, tasks.data(), tasks.size() * sizeof(unsigned),
                           hipMemcpyHostToDevice));
    ctx->dag_ntasks = (int)tasks.size();
    ctx->dag_nt = nt;
    ctx->dag_ntr = ntr;
    ctx->dag_flags = flags & ~DAG_MIRROR;  // (the task list does not depend on it)
    ctx->dag_lag_built = ctx->dag_zlag;
  }
  // a previous launch's hook may have left readers of the counters (row gates on another
  // stream): they must drain before the counters are reset or reallocated
  if (ctx->dag_sync_readers_pending) {
    HIP_TRY(ctx, hipStreamWaitEvent(st, ctx->dag_sync_readers, 0));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->dag_sync_readers, 0));
    ctx->dag_sync_readers_pending = false;
  }
  // [2 + nt + ntr + i]: ustored[i] (hook launches; zeroed with the rest)
  const size_t nsync = 2 + (size_t)nt + ntr + nt;
  if (ctx->dag_sync_cap < nsync) {
    if (ctx->dag_sync) {
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (every DAG launch joins it)
      HIP_TRY(ctx, hipFree(ctx->dag_sync));
    }
    ctx->dag_sync = nullptr;
    ctx->dag_sync_cap = 0;
    HIP_TRY(ctx, hipMalloc((void**)&ctx->dag_sync, nsync * sizeof(int)));
    ctx->dag_sync_cap = nsync;
  }
  HIP_TRY(ctx, hipMemsetAsync(ctx->dag_sync, 0, nsync * sizeof(int), st));
  if (solve || lower) {
    dag_init_kernel<<<(nt + ntr + 255) / 256, 256, 0, st>>>(ctx->dag_sync, nt, ntr, solve, lower);
    LAUNCH_CHECK(ctx);
  }
  if (ctx->ncu <= 0) {
    hipDeviceProp_t prop;
    HIP_TRY(ctx, hipGetDeviceProperties(&prop, ctx->device));
    ctx->ncu = prop.multiProcessorCount;
  }
  DagArgs a{};
  a.A = dA;
  a.lda = (size_t)lda;
  a.n = n;
  a.nt = nt;
  a.B = dB;
  a.ldb = (size_t)(dB ? ldb : 0);
  a.nrhs = dB ? nrhs : 0;
  a.ntr = ntr;
  a.winv = ctx->winv + (size_t)(kglob / DT) * DT * DT;
  a.kglob = kglob;
  a.info = ctx->dinfo;
  a.sync = ctx->dag_sync;
  a.tasks = ctx->dag_tasks;
  a.ntasks = ctx->dag_ntasks;
  a.lower = lower;
  a.G = gram ? dG : nullptr;
  a.ldg = (size_t)(gram ? ldg : 0);
  a.gbase = gram ? ctx->dag_ntasks - nt * (nt + 1) / 2 : ctx->dag_ntasks;
  a.mirror = mirror;
  a.spin_limit = dag_spin_limit(ctx);
  const int grid = std::min(ctx->dag_ntasks, std::max(1, ctx->ncu - ctx->dag_reserve_cu));
  // the one-shot hook (common.hpp): an event between the counters' reset and the launch, the
  // hook itself only after the launch is enqueued -- work it orders behind the event can then
  // never sit ahead of the launch in a hardware queue that two streams share
  auto hook = (ctx->dag_hook && !solve && !lower && kglob == 0) ? ctx->dag_hook : nullptr;
  a.ustored = hook ? ctx->dag_sync + 2 + nt + ntr : nullptr;
  hipEvent_t hook_ev = nullptr;
  if (hook) {
    ctx->dag_hook = nullptr;
    if (hipEventCreateWithFlags(&hook_ev, hipEventDisableTiming) != hipSuccess) hook_ev = nullptr;
    if (hook_ev && hipEventRecord(hook_ev, st) != hipSuccess) {
      hipEventDestroy(hook_ev);
      hook_ev = nullptr;
    }
    (void)hipGetLastError();
  }
  // factorisation n^3/3; U^{-T} B: n^2 per column, ~n^3/3 for a lower-triangular n x n B
  const double flops = (solve ? 0.0 : (double)n * n * n / 3.0) +
                       (lower ? (double)n * n * n / 3.0 : (double)n * n * (dB ? nrhs : 0)) +
                       (gram ? (double)n * n * n / 3.0 : 0.0);
  {
    hipStream_t ls = ctx->ls;
    ctx->ls = st;  // TimerScope records on ctx->ls
    TimerScope ts(ctx, solve ? TC_DAG_SOLVE : TC_DAG, flops);  // (solve-only launches apart)
    if (gram)
      potrf_dag_kernel<true, false><<<grid, 256, 0, st>>>(a);
    else
      potrf_dag_kernel<false, false><<<grid, 256, 0, st>>>(a);
    ctx->ls = ls;
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
      if (hook_ev) hipEventDestroy(hook_ev);  // (the hook is not called: nothing was launched)
      return set_err(ctx, GPR_E_HIP, "tile-DAG launch: %s", hipGetErrorString(le));
    }
  }
  if (hook) {
    hook(ctx->dag_hook_user, dA, n, lda, ctx->dag_sync + 2, a.ustored, nt, hook_ev);
    if (hook_ev) hipEventDestroy(hook_ev);
  }
  return 0;
}

// nbatch independent factorisations A_b = U_b^T U_b (A_b = dA + b strA, n x n, ld lda) and
// B_b <- U_b^{-T} B_b (dB + b strB, n x nrhs, ld ldb; optional) in ONE persistent launch: the
// tasks of every matrix in one ticket list, row by row across the matrices (row i of each A_b,
// then row i of each B_b), so the independent chains fill the CUs that one chain leaves idle
// (a per-matrix launch of a small N is chain-bound).  Per-matrix W slots, progress counters and
// info words in ctx->dagb; info_out[b] (host) = matrix b's LAPACK info.  The shape conditions
// are the single launch's (n % 16, 128-B aligned tiles: strides multiples of 16 doubles).
// Returns 1 when they do not hold (nothing launched), 0 after the launch has completed.
int launch_potrf_dag_batch(gpr_ctx* ctx, double* dA, size_t strA, int n, int lda, double* dB,
                           size_t strB, int nrhs, int ldb, int nbatch, int* info_out) {
  hipStream_t st = ctx->stream;
  if (nbatch <= 0) return 0;
  // (its W slots are its own, so the context's inner block size does not matter)
  if (n <= 0 || n % 16 || lda % 16 || strA % 16 || ((uintptr_t)dA & 127) || n > DT * 32767)
    return 1;
  if (dB && (nrhs <= 0 || ldb % 16 || strB % 16 || ((uintptr_t)dB & 127) || nrhs > DT * 65535))
    return 1;
  const int nt = (n + DT - 1) / DT, ntr = dB ? (nrhs + DT - 1) / DT : 0;
  std::vector<unsigned> tasks;
  std::vector<int> tb;
  const size_t per = (size_t)nt * (nt + 1) / 2 + (size_t)nt * ntr;
  tasks.reserve(per * nbatch);
  tb.reserve(per * nbatch);
  for (int i = 0; i < nt; ++i) {
    for (int b = 0; b < nbatch; ++b)
      for (int j = i; j < nt; ++j) {
        tasks.push_back(((unsigned)i << 16) | (unsigned)j);
        tb.push_back(b);
      }
    for (int b = 0; b < nbatch; ++b)
      for (int c = 0; c < ntr; ++c) {
        tasks.push_back(0x80000000u | ((unsigned)i << 16) | (unsigned)c);
        tb.push_back(b);
      }
  }
  const int ntasks = (int)tasks.size();
  const int strS = 2 + nt + ntr;
  // workspace (doubles): W slots | tasks | tbatch | sync | info (ints packed two per double)
  const size_t nW = (size_t)nbatch * nt * DT * DT;
  const size_t nI = (size_t)ntasks * 2 + (size_t)nbatch * strS + (size_t)nbatch;
  GPR_TRY(ensure_buf(ctx, &ctx->dagb, &ctx->dagb_cap, nW + (nI + 1) / 2 + 1));
  double* W = ctx->dagb;
  unsigned* dtasks = reinterpret_cast<unsigned*>(W + nW);
  int* dtb = reinterpret_cast<int*>(dtasks + ntasks);
  int* dsync = dtb + ntasks;
  int* dinfo = dsync + (size_t)nbatch * strS;
  HIP_TRY(ctx, hipMemcpyAsync(dtasks, tasks.data(), sizeof(unsigned) * ntasks, hipMemcpyHostToDevice, st));
  HIP_TRY(ctx, hipMemcpyAsync(dtb, tb.data(), sizeof(int) * ntasks, hipMemcpyHostToDevice, st));
  HIP_TRY(ctx, hipMemsetAsync(dsync, 0, sizeof(int) * ((size_t)nbatch * strS + nbatch), st));
  if (ctx->ncu <= 0) {
    hipDeviceProp_t prop;
    HIP_TRY(ctx, hipGetDeviceProperties(&prop, ctx->device));
    ctx->ncu = prop.multiProcessorCount;
  }
  DagArgs a{};
  a.A = dA;
  a.lda = (size_t)lda;
  a.n = n;
  a.nt = nt;
  a.B = dB;
  a.ldb = (size_t)(dB ? ldb : 0);
  a.nrhs = dB ? nrhs : 0;
  a.ntr = ntr;
  a.winv = W;
  a.kglob = 0;
  a.info = dinfo;
  a.sync = dsync;
  a.tasks = dtasks;
  a.ntasks = ntasks;
  a.gbase = ntasks;
  a.spin_limit = dag_spin_limit(ctx);
  a.tbatch = dtb;
  a.strA = strA;
  a.strB = strB;
  a.strW = (size_t)nt * DT * DT;
  a.strS = strS;
  const int grid = std::min(ntasks, std::max(1, ctx->ncu));
  const double flops = nbatch * ((double)n * n * n / 3.0 + (double)n * n * (dB ? nrhs : 0));
  {
    TimerScope ts(ctx, TC_DAG, flops);
    potrf_dag_kernel<false, true><<<grid, 256, 0, st>>>(a);
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess) return set_err(ctx, GPR_E_HIP, "batched tile-DAG launch: %s", hipGetErrorString(le));
  }
  std::vector<int> h(nbatch);
  HIP_TRY(ctx, hipMemcpyAsync(h.data(), dinfo, sizeof(int) * nbatch, hipMemcpyDeviceToHost, st));
  HIP_TRY(ctx, hipStreamSynchronize(st));
  for (int b = 0; b < nbatch; ++b) {
    if (h[b] < 0) return set_err(ctx, GPR_E_HIP, "batched tile-DAG: a dependency wait timed out");
    if (info_out) info_out[b] = h[b];
  }
  return 0;
}
