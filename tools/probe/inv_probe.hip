// Latency probe: one column half of the diagonal factor's inverse (diag_block.hpp
// d2_inv_colhalf<3>: 144 FP64 MFMAs in a 3-level recurrence) on one wave, s_memtime cycles,
// with and without its W stores, and the tile-DAG's Q-form last block (d2_tail_q/_out).  S / Xd hold a well-conditioned synthetic U (values only
// matter for finiteness).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I gaussianprocessregression.jl_amd/csrc \
//          -o tools/probe/inv_probe tools/probe/inv_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "diag_block.hpp"

template <int V>
__global__ __launch_bounds__(256) void inv_kernel(double* winv, long long* cyc) {
  extern __shared__ double dsm[];
  lds_d* S = (lds_d*)dsm;
  lds_d(*Xd)[D2_PB] = reinterpret_cast<lds_d(*)[D2_PB]>(S + D2_PK);
  for (int e = threadIdx.x; e < D2_LDS_QTAIL; e += blockDim.x)
    S[e] = 1.0 / (1.0 + (e % 97));
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  long long t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  __builtin_amdgcn_sched_barrier(0);
  if (V == 0) {  // today's split: waves 0-1 J=3, waves 2-3 J=2,1,0
    if (wv == 0) d2_inv_colhalf<3, true>(0, S, Xd, winv, 128, lane);
    else if (wv == 1) d2_inv_colhalf<3, true>(1, S, Xd, winv, 128, lane);
    else {
      d2_inv_colhalf<2, true>(wv - 2, S, Xd, winv, 128, lane);
      d2_inv_colhalf<1, true>(wv - 2, S, Xd, winv, 128, lane);
      d2_inv_colhalf<0, true>(wv - 2, S, Xd, winv, 128, lane);
    }
  } else if (V == 1) {  // one column half alone, wave 0 (plain stores)
    if (wv == 0) d2_inv_colhalf<3, false>(0, S, Xd, winv, 128, lane);
  } else {  // the tile-DAG's last column block in Q form (all four waves, one barrier)
    d4v q[3];
    if (wv < 2)
      d2_tail_q<0>(wv, S, Xd, S + D2_XO, S + D2_QS, lane, q);
    else
      d2_tail_q<1>(wv - 2, S, Xd, S + D2_XO, S + D2_QS, lane, q);
    __syncthreads();
    if (wv < 2)
      d2_tail_out<0, true>(wv, Xd, S + D2_QS, q, winv, 128, lane);
    else
      d2_tail_out<1, true>(wv - 2, Xd, S + D2_QS, q, winv, 128, lane);
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (lane == 0) cyc[wv] = t1 - t0;
}

int main() {
  double* w;
  long long* c;
  hipMalloc(&w, 128 * 128 * 8);
  hipMalloc(&c, 4 * 8);
  const size_t lds = sizeof(double) * D2_LDS_QTAIL;
  auto run = [&](auto k, const char* name) {
    long long best[4] = {1ll << 60, 1ll << 60, 1ll << 60, 1ll << 60}, h[4];
    for (int it = 0; it < 20; ++it) {
      hipMemset(c, 0, 32);
      k<<<1, 256, lds>>>(w, c);
      hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
      for (int q = 0; q < 4; ++q) best[q] = h[q] < best[q] ? h[q] : best[q];
    }
    printf("%-40s cycles per wave: %lld %lld %lld %lld\n", name, best[0], best[1], best[2], best[3]);
  };
  run(inv_kernel<0>, "4 waves as in diag2_core (sc1 stores)");
  run(inv_kernel<1>, "wave 0 alone, J=3 (plain stores)");
  run(inv_kernel<2>, "block 3 in Q form, 4 waves (sc1 stores)");
  return 0;
}
