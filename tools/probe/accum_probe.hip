// Accumulation-pipeline probe for the tile-DAG (dag.hip dag_accum): one persistent workgroup
// per CU computes acc += P^T Q over a long K, P = 128 TMR columns, Q = 128 columns of a
// K-contiguous (column-major, ld = K) matrix, TMR = 1: 4 waves (each 64 x 64, today's kernel),
// TMR = 2: 8 waves over a 256 x 128 tile (2 waves per SIMD; Q shared by both row halves: 48 KB
// of operands per 16-deep stage for twice the flops of a 32-KB 128 x 128 stage).
// Answers: per-CU FP64 MFMA rate and HBM traffic per flop of the two shapes before the DAG
// is restructured around either.   Usage: accum_probe [K] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4v __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int DT = 128, DTK = 16, DNCH = DTK / 2, DRPD = 64 / DNCH;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int lidx(int row, int chunk) { return row * DTK + ((chunk ^ swz(row)) << 1); }

template <int VM>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
}

// TMR: 128-row tiles of P (1 or 2); NW: waves (4 = one per SIMD, 8 = two); each wave owns
// (128 TMR / (NW / 2)) rows x 64 columns; NSTG: LDS stages; DBUF: next stage's fragments read
// into a second register set during the current stage's MFMAs.
template <int TMR, int NW, int NSTG, bool DBUF>
__global__ __launch_bounds__(NW * 64, 1) void accum_kernel(const double* __restrict__ M, size_t ld,
                                                          int ncolblk, int nst, int mode,
                                                          double* out) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass cannot instantiate the amdgcn builtins)
  constexpr int PR = DT * TMR;             // P rows (tile rows)
  constexpr int WR = NW / 2;               // wave row groups
  constexpr int RB = PR / WR / 16;         // 16-row blocks per wave
  constexpr int DSTAGE = (PR + DT) * DTK;  // doubles per stage
  constexpr int NDP = PR / (NW * DRPD);    // DMA per wave for P
  constexpr int NDQ = DT / (NW * DRPD);    // DMA per wave for Q
  constexpr int DVM = NDP + NDQ;
  constexpr int DNP = DTK / 8;
  constexpr int NF = 4 + RB;
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w % WR, wn = w / WR;
  const int b = blockIdx.x;
  // mode 0 (hot): every workgroup reads the same P (panels 0..TMR-1) and Q (panel TMR):
  // the pipeline's own rate.  mode 1 (DAG-like): P shared by groups of 32 workgroups (a row
  // of tasks), Q distinct per workgroup (every task its own column panel).  P spans TMR
  // consecutive panels, so it starts at most at panel ncolblk - TMR - 1.
  const int np_ = ncolblk - TMR - 1;
  // mode 2 (L2-resident): mode 0's operands, K wrapped at 1024 rows (64 stages): 2 MB of
  // operands per launch, held in every XCD's 4-MB L2 -- the same MFMA work with no HBM stream
  const int pp = mode == 1 ? (b / 32) % np_ : 0, qp = mode == 1 ? TMR + (b % np_) : TMR;
  const double* P = M + (size_t)pp * DT * ld;
  const double* Q = M + (size_t)qp * DT * ld;
  d4v acc[4][RB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      if (NW == 4)  // one wave per SIMD: accumulators defined in AGPRs (gemm.hip's idiom), so
                    // the loop never copies them between register files
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(0.0));
      else
        acc[i][j] = d4v{0, 0, 0, 0};
    }
  const double* srcP[NDP];
  const double* srcQ[NDQ];
#pragma unroll
  for (int r = 0; r < NDP; ++r) {
    const int row = DRPD * (NW * r + w) + lane / DNCH;
    srcP[r] = P + 2 * ((lane % DNCH) ^ swz(row)) + (size_t)row * ld;
  }
#pragma unroll
  for (int r = 0; r < NDQ; ++r) {
    const int row = DRPD * (NW * r + w) + lane / DNCH;
    srcQ[r] = Q + 2 * ((lane % DNCH) ^ swz(row)) + (size_t)row * ld;
  }
  auto issue = [&](int s) {
    double* base = lds + (s % NSTG) * DSTAGE;
    const size_t ko = (size_t)(mode == 2 ? min(s, nst - 1) & 63 : min(s, nst - 1)) * DTK;
#pragma unroll
    for (int r = 0; r < NDP; ++r)
      __builtin_amdgcn_global_load_lds(srcP[r] + ko, base + (NW * r + w) * 128, 16, 0, 0);
#pragma unroll
    for (int r = 0; r < NDQ; ++r)
      __builtin_amdgcn_global_load_lds(srcQ[r] + ko, base + PR * DTK + (NW * r + w) * 128, 16, 0, 0);
  };
  auto read_frags = [&](d2 (&F)[DNP][NF], int s) {
    const double* ps = lds + (s % NSTG) * DSTAGE;
    const double* qs = ps + PR * DTK;
#pragma unroll
    for (int p = 0; p < DNP; ++p) {
      const int ch = (lane >> 4) + 4 * p;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        F[p][i] = *reinterpret_cast<const d2*>(&qs[lidx(wn * 64 + i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < RB; ++j)
        F[p][4 + j] = *reinterpret_cast<const d2*>(&ps[lidx(wm * 16 * RB + j * 16 + (lane & 15), ch)]);
    }
  };
  auto mfma_stage = [&](const d2 (&F)[DNP][NF]) {
#pragma unroll
    for (int p = 0; p < DNP; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < RB; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[p][i][h], F[p][4 + j][h], acc[i][j], 0, 0, 0);
  };
  constexpr int NMF = DNP * 2 * 4 * RB, NDS = DNP * NF;
  auto sched = [&]() {
#pragma unroll
    for (int t = 0; t < DVM; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
    if (DBUF) {
#pragma unroll
      for (int t = 0; t < NDS; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMF - DVM - 2 * NDS, 0);
    } else {
      __builtin_amdgcn_sched_group_barrier(0x008, NMF - DVM, 0);
    }
  };
  d2 F0[DNP][NF], F1[DNP][NF];
#pragma unroll
  for (int t = 0; t < NSTG - 1; ++t) issue(t);
  if (DBUF) {
    vmcnt<DVM * (NSTG - 2)>();
    __builtin_amdgcn_s_barrier();
    read_frags(F0, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    auto step = [&](int s, d2 (&Fc)[DNP][NF], d2 (&Fn)[DNP][NF]) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      vmcnt<DVM * (NSTG - 3)>();
      __builtin_amdgcn_s_barrier();
      issue(s + NSTG - 1);
      read_frags(Fn, s + 1);
      mfma_stage(Fc);
      sched();
    };
    int s = 0;
    for (; s + 1 < nst; s += 2) {
      step(s, F0, F1);
      step(s + 1, F1, F0);
    }
    if (s < nst) mfma_stage(F0);
  } else {
    // one fragment set: stage s's fragments read right after the barrier that makes it
    // complete (the other wave on the SIMD covers the LDS latency)
    for (int s = 0; s < nst; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      vmcnt<DVM * (NSTG - 2)>();
      __builtin_amdgcn_s_barrier();
      issue(s + NSTG - 1);
      read_frags(F0, s);
      mfma_stage(F0);
      sched();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // own fragment reads of stage s done before the
    }                                       // next barrier frees the stage for re-fill
  }
  vmcnt<0>();
  __syncthreads();
  double t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < RB; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 512 + tid] = t;
#endif
}

// Barrier-free variant: every wave DMAs its OWN operand rows (its 64 P rows and 64 Q rows)
// into a private LDS region, so a wave waits only for its own DMA (vmcnt) and never for the
// other waves (no s_barrier in the loop); each P / Q row is fetched by two waves (L2 hits).
// PK-deep stages (8: 4 chunks per row, swizzle (row >> 2) & 3; 16: 8 chunks, (row >> 1) & 7),
// NSTG stages, next stage's fragments prefetched into a second register set.
template <int PK, int NSTG>
__global__ __launch_bounds__(256, 1) void accum_priv_kernel(const double* __restrict__ M, size_t ld,
                                                           int ncolblk, int nst, int mode,
                                                           double* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int NCH = PK / 2;              // 16-B chunks per LDS row
  constexpr int RPD = 64 / NCH;            // rows per wave-wide 1-KB DMA
  constexpr int ND = 64 / RPD;             // DMA per operand per wave per stage
  constexpr int WSTAGE = 2 * 64 * PK;      // doubles per wave per stage (P rows, then Q rows)
  constexpr int DNP = PK / 8;              // fragment blocks (2 k-steps each) per stage
  constexpr int DVM = 2 * ND;
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  const int b = blockIdx.x;
  const int np_ = ncolblk - 2;
  const int pp = mode ? (b / 32) % np_ : 0, qp = mode ? 1 + (b % np_) : 1;
  const double* P = M + (size_t)pp * DT * ld + (size_t)wm * 64 * ld;
  const double* Q = M + (size_t)qp * DT * ld + (size_t)wn * 64 * ld;
  auto sw = [](int row) { return PK == 8 ? ((row >> 2) & 3) : ((row >> 1) & 7); };
  d4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(0.0));
  const double* srcP[ND];
  const double* srcQ[ND];
#pragma unroll
  for (int r = 0; r < ND; ++r) {
    const int row = RPD * r + lane / NCH;
    const int c = (lane % NCH) ^ sw(row);
    srcP[r] = P + 2 * c + (size_t)row * ld;
    srcQ[r] = Q + 2 * c + (size_t)row * ld;
  }
  double* mine = lds + w * WSTAGE;
  auto issue = [&](int s) {
    double* base = mine + (s % NSTG) * 4 * WSTAGE;
    const size_t ko = (size_t)min(s, nst - 1) * PK;
#pragma unroll
    for (int r = 0; r < ND; ++r) {
      __builtin_amdgcn_global_load_lds(srcP[r] + ko, base + r * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(srcQ[r] + ko, base + 64 * PK + r * 128, 16, 0, 0);
    }
  };
  auto read_frags = [&](d2 (&F)[DNP][8], int s) {
    const double* ps = mine + (s % NSTG) * 4 * WSTAGE;
    const double* qs = ps + 64 * PK;
#pragma unroll
    for (int p = 0; p < DNP; ++p) {
      const int ch = (lane >> 4) + 4 * p;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = i * 16 + (lane & 15);
        F[p][i] = *reinterpret_cast<const d2*>(&qs[row * PK + 2 * (ch ^ sw(row))]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = j * 16 + (lane & 15);
        F[p][4 + j] = *reinterpret_cast<const d2*>(&ps[row * PK + 2 * (ch ^ sw(row))]);
      }
    }
  };
  auto mfma_stage = [&](const d2 (&F)[DNP][8]) {
#pragma unroll
    for (int p = 0; p < DNP; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[p][i][h], F[p][4 + j][h], acc[i][j], 0, 0, 0);
  };
  auto step = [&](int s, d2 (&Fc)[DNP][8], d2 (&Fn)[DNP][8]) {
    __builtin_amdgcn_sched_barrier(0);
    // stage s - 1's buffer: its fragments were read (and waited for) a step ago
    issue(s + NSTG - 1);
    vmcnt<DVM * (NSTG - 2)>();  // own DMA of stage s + 1 landed (s + 2 .. s + NSTG - 1 in flight)
    read_frags(Fn, s + 1);
    mfma_stage(Fc);
#pragma unroll
    for (int t = 0; t < 8 * DNP; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 32 * DNP - 16 * DNP, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): Fn in registers before the next issue
  };
  d2 F0[DNP][8], F1[DNP][8];
#pragma unroll
  for (int t = 0; t < NSTG - 1; ++t) issue(t);
  vmcnt<DVM * (NSTG - 2)>();
  read_frags(F0, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  int s = 0;
  for (; s + 1 < nst; s += 2) {
    step(s, F0, F1);
    step(s + 1, F1, F0);
  }
  if (s < nst) mfma_stage(F0);
  vmcnt<0>();
  double t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 512 + tid] = t;
#endif
}

template <int PK, int NSTG>
void run_priv(const double* M, size_t ld, int ncolblk, int K, int reps, int mode, double* out, int cus) {
  constexpr size_t lds = sizeof(double) * NSTG * 4 * 2 * 64 * PK;
  if (hipFuncSetAttribute((const void*)accum_priv_kernel<PK, NSTG>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    printf("priv PK=%d NSTG=%d: cannot set %zu B of LDS\n", PK, NSTG, lds);
    return;
  }
  const int nst = K / PK;
  hipLaunchKernelGGL((accum_priv_kernel<PK, NSTG>), dim3(cus), dim3(256), lds, 0, M, ld, ncolblk, 8, mode, out);
  hipError_t le = hipGetLastError();
  if (le == hipSuccess) le = hipDeviceSynchronize();
  if (le != hipSuccess) {
    printf("priv PK=%d NSTG=%d: launch failed: %s\n", PK, NSTG, hipGetErrorString(le));
    return;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((accum_priv_kernel<PK, NSTG>), dim3(cus), dim3(256), lds, 0, M, ld, ncolblk, nst, mode, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * DT * DT * (double)nst * PK * cus * reps;
  printf("%s private-buffer 128x128, 4 waves, %2d-deep x %d stages (%3zu KB), no barrier: "
         "%.2f TFLOP/s = %.4f per CU (%.3f ms per launch)\n", mode ? "dag-like" : "hot     ",
         PK, NSTG, lds / 1024, flops / ms / 1e9, flops / ms / 1e9 / cus, ms / reps);
}

template <int TMR, int NW, int NSTG, bool DBUF>
void run(const double* M, size_t ld, int ncolblk, int K, int reps, int mode, double* out, int cus) {
  constexpr size_t lds = sizeof(double) * NSTG * (DT * TMR + DT) * DTK;
  auto kern = accum_kernel<TMR, NW, NSTG, DBUF>;
  if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess) {
    printf("TMR=%d NW=%d NSTG=%d: cannot set %zu B of LDS\n", TMR, NW, NSTG, lds);
    return;
  }
  const int nst = K / DTK;
  hipLaunchKernelGGL(kern, dim3(cus), dim3(NW * 64), lds, 0, M, ld, ncolblk, 8, mode, out);
  hipError_t le = hipGetLastError();
  if (le == hipSuccess) le = hipDeviceSynchronize();
  if (le != hipSuccess) {
    printf("TMR=%d NW=%d NSTG=%d: launch failed: %s\n", TMR, NW, NSTG, hipGetErrorString(le));
    return;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, dim3(cus), dim3(NW * 64), lds, 0, M, ld, ncolblk, nst, mode, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * DT * TMR * DT * (double)nst * DTK * cus * reps;
  const double bytes = 8.0 * (DT * TMR + DT) * (double)nst * DTK * cus * reps;
  printf("%s tile %3dx128, %d waves, %d stages (%3zu KB), %s fragments: %.2f TFLOP/s = %.4f per CU, "
         "%.1f flop/B, operand stream %.2f TB/s (%.3f ms per launch)\n",
         mode == 1 ? "dag-like" : mode == 2 ? "L2-held " : "hot     ",
         DT * TMR, NW, NSTG, lds / 1024, DBUF ? "2-set" : "1-set", flops / ms / 1e9,
         flops / ms / 1e9 / cus, flops / bytes, bytes / ms / 1e9, ms / reps);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 16384;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int ncolblk = 64;                         // 64 panels of 128 columns, K deep
  const size_t ld = K, ncols = (size_t)ncolblk * DT;
  double *M, *out;
  if (hipMalloc(&M, sizeof(double) * ld * ncols) != hipSuccess ||
      hipMalloc(&out, sizeof(double) * cus * 512) != hipSuccess)
    return 1;
  std::vector<double> h(ld * ncols);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  (void)hipMemcpy(M, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
  const int cfg = argc > 3 ? atoi(argv[3]) : 0;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  printf("K = %d, %d CUs, %d reps, config %d\n", K, cus, reps, cfg);
  switch (cfg) {
    case 0: run<1, 4, 4, true>(M, ld, ncolblk, K, reps, mode, out, cus); break;   // today's dag_accum
    case 1: run<2, 4, 3, false>(M, ld, ncolblk, K, reps, mode, out, cus); break;  // 256 x 128, 1 wave/SIMD
    case 2: run<2, 8, 3, false>(M, ld, ncolblk, K, reps, mode, out, cus); break;  // 256 x 128, 2 waves/SIMD
    case 3: run<1, 4, 4, false>(M, ld, ncolblk, K, reps, mode, out, cus); break;
    case 4: run_priv<8, 4>(M, ld, ncolblk, K, reps, mode, out, cus); break;   // 128 KB
    case 5: run_priv<8, 5>(M, ld, ncolblk, K, reps, mode, out, cus); break;   // 160 KB
    case 6: run_priv<16, 2>(M, ld, ncolblk, K, reps, mode, out, cus); break;  // 128 KB
    case 7: run<1, 8, 4, true>(M, ld, ncolblk, K, reps, mode, out, cus); break;   // 128 x 128, 2 waves/SIMD (32 x 64 each)
    case 8: run<1, 8, 4, false>(M, ld, ncolblk, K, reps, mode, out, cus); break;
  }
  return 0;
}
