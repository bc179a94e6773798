// store_ceiling.hip -- bench instrumentation, not product code (libgpr_store_probe.so, loaded by
// bench.py only).  Times pure-store kernels that write exactly the bytes of the fit's upper-only
// K build (kmat_symu_kernel, assembly.hip: column c gets rows [0, min(n, 128 (c / 128 + 1))),
// ~4 n^2 bytes) with no arithmetic, so the bench line carries, from the same box and process,
// the store rate the K-assembly is bounded by:
//   pattern 0  the kernel's own shape: one wave per (32-column strip, 128-row segment) item,
//              persistent grid (256 CUs x 8 workgroups of 4 waves), 8-B stores, each store
//              instruction = 4 columns x 128 contiguous bytes (the MFMA D layout)
//   pattern 1  the same items, one wave per item (no persistent loop: dispatch order)
//   pattern 2  1-KB column chunks in column order, one chunk per wave (16-B stores: each
//              instruction one column's 128 rows) -- the fastest upper-only order measured
//   pattern 3  the kernel's items and persistent grid, but each store instruction one column's
//              128 rows (1 KB, 16-B lanes): what an LDS-transposed D layout would write
//   pattern 4  as 3 with 16-column strips
//   pattern 5  as 3, one item per wave (no persistent loop): the shape of the fit's single-part
//              build since round 6 (GPR_KBUILD_COLSTORE)
// Each is launched `reps` times after one warm-up; the best time is returned.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

namespace {

__host__ __device__ inline int up_rows(int c, int n) { return min(n, 128 * (c / 128 + 1)); }

__global__ __launch_bounds__(256) void st_kup(double* K, int n, size_t ld, const int* items,
                                              int nitems, double v) {
  const int lane = threadIdx.x & 63;
  const int voff = (lane & 15) + (lane >> 4) * (int)ld;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < nitems; t += gridDim.x * 4) {
    const int code = items[t];
    const int j0 = (code >> 16) * 32, r0 = (code & 0xffff) * 128;
    const int r1 = min(r0 + 128, up_rows(j0, n));
    for (int i0 = r0; i0 < r1; i0 += 32)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = i0 + 16 * rb + (lane & 15), c = j0 + 16 * cb + 4 * q + (lane >> 4);
            if (r < r1 && c < n)
              __builtin_nontemporal_store(
                  v, K + (size_t)(i0 + 16 * rb) + (size_t)(j0 + 16 * cb + 4 * q) * ld + voff);
          }
  }
}

template <int W>
__global__ __launch_bounds__(256) void st_kup_col(double* K, int n, size_t ld, const int* items,
                                                  int nitems, double v) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < nitems; t += gridDim.x * 4) {
    const int code = items[t];
    const int j0 = (code >> 16) * W, r0 = (code & 0xffff) * 128;
    const int r1 = min(r0 + 128, up_rows(j0, n));
    const int r = r0 + 2 * lane;
#pragma unroll 4
    for (int c = j0; c < min(j0 + W, n); ++c) {
      if (r + 1 < r1)
        __builtin_nontemporal_store(d2{v, v}, reinterpret_cast<d2*>(K + (size_t)r + (size_t)c * ld));
      else if (r < r1)
        __builtin_nontemporal_store(v, K + (size_t)r + (size_t)c * ld);
    }
  }
}

__global__ __launch_bounds__(256) void st_flat(double* K, int n, size_t ld,
                                               const long long* chunks, int nch, double v) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= nch) return;
  const long long code = chunks[t];
  const int c = (int)(code >> 20), r = (int)(code & 0xfffff) + 2 * lane;
  const int r1 = up_rows(c, n);
  if (r + 1 < r1)
    __builtin_nontemporal_store(d2{v, v}, reinterpret_cast<d2*>(K + (size_t)r + (size_t)c * ld));
  else if (r < r1)
    __builtin_nontemporal_store(v, K + (size_t)r + (size_t)c * ld);
}

}  // namespace

extern "C" {

// K: device buffer of n x n doubles (leading dimension n), overwritten.  Returns 0 and the best
// time (ms) and the bytes written per launch; negative on a HIP error.
int gpr_probe_upper_store(void* stream, int n, double* K, int pattern, int reps, double* best_ms,
                          double* bytes) {
  if (n <= 0 || !K || !best_ms || !bytes || pattern < 0 || pattern > 5) return -1;
  hipStream_t s = (hipStream_t)stream;
  const size_t ld = (size_t)n;
  std::vector<int> items;
  std::vector<long long> chunks;
  const int W = pattern == 4 ? 16 : 32;
  double nb = 0.0;
  for (int c = 0; c < n; ++c) nb += 8.0 * up_rows(c, n);
  for (int bj = 0; bj * W < n; ++bj)
    for (int sg = 0; sg * 128 < up_rows(bj * W, n); ++sg) items.push_back((bj << 16) | sg);
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < up_rows(c, n); r += 128) chunks.push_back(((long long)c << 20) | r);
  int* ditems = nullptr;
  long long* dch = nullptr;
  if (hipMalloc(&ditems, items.size() * sizeof(int)) != hipSuccess ||
      hipMalloc(&dch, chunks.size() * sizeof(long long)) != hipSuccess)
    return -2;
  hipMemcpy(ditems, items.data(), items.size() * sizeof(int), hipMemcpyHostToDevice);
  hipMemcpy(dch, chunks.data(), chunks.size() * sizeof(long long), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  const int nit = (int)items.size(), nch = (int)chunks.size();
  for (int rep = 0; rep <= std::max(1, reps); ++rep) {
    hipEventRecord(e0, s);
    if (pattern == 0)
      st_kup<<<std::max(1, std::min((nit + 3) / 4, 256 * 8)), 256, 0, s>>>(K, n, ld, ditems, nit, 1.0);
    else if (pattern == 1)
      st_kup<<<(nit + 3) / 4, 256, 0, s>>>(K, n, ld, ditems, nit, 1.0);
    else if (pattern == 2)
      st_flat<<<(nch + 3) / 4, 256, 0, s>>>(K, n, ld, dch, nch, 1.0);
    else if (pattern == 3)
      st_kup_col<32><<<std::max(1, std::min((nit + 3) / 4, 256 * 8)), 256, 0, s>>>(K, n, ld, ditems, nit, 1.0);
    else if (pattern == 4)
      st_kup_col<16><<<std::max(1, std::min((nit + 3) / 4, 256 * 8)), 256, 0, s>>>(K, n, ld, ditems, nit, 1.0);
    else
      st_kup_col<32><<<(nit + 3) / 4, 256, 0, s>>>(K, n, ld, ditems, nit, 1.0);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep) best = std::min(best, ms);  // (rep 0: warm-up)
  }
  const bool ok = hipGetLastError() == hipSuccess;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(ditems);
  hipFree(dch);
  *best_ms = best;
  *bytes = nb;
  return ok ? 0 : -3;
}

}  // extern "C"
