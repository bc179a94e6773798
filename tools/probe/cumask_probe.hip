// How does hipExtStreamCreateWithCUMask map mask bits to CUs on a multi-XCD gfx950?
// For a few masks, a grid of short spinning blocks records (XCC_ID, HW_ID) per block; the
// probe prints how many distinct CUs each XCD used.  Used to build XCD-balanced CU masks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <utility>
#include <vector>

__global__ void where_kernel(int* out) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = (int)(xcc & 0xf);
    out[2 * blockIdx.x + 1] = (int)((hw >> 8) & 0xff);  // cu, sh, se
  }
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) {
  }
}

static void run(const char* name, const std::vector<uint32_t>& m, int* d, int nb) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) {
    printf("%s: mask stream failed\n", name);
    return;
  }
  std::vector<int> h(2 * nb);
  where_kernel<<<nb, 64, 0, s>>>(d);
  (void)hipMemcpyAsync(h.data(), d, 2 * nb * sizeof(int), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  std::set<std::pair<int, int>> all;
  std::vector<std::set<int>> per(8);
  for (int b = 0; b < nb; ++b) {
    all.insert({h[2 * b], h[2 * b + 1]});
    if (h[2 * b] >= 0 && h[2 * b] < 8) per[h[2 * b]].insert(h[2 * b + 1]);
  }
  printf("%-28s distinct CUs %3zu  per XCD:", name, all.size());
  for (int x = 0; x < 8; ++x) printf(" %2zu", per[x].size());
  printf("\n");
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  const int words = (ncu + 31) / 32;
  const int nb = 65536;
  int* d;
  (void)hipMalloc(&d, 2 * nb * sizeof(int));
  printf("ncu=%d\n", ncu);
  auto mk = [&](auto keep) {
    std::vector<uint32_t> m(words, 0u);
    for (int c = 0; c < ncu; ++c)
      if (keep(c)) m[c >> 5] |= 1u << (c & 31);
    return m;
  };
  run("full", mk([](int) { return true; }), d, nb);
  run("drop bits 0..7", mk([](int c) { return c >= 8; }), d, nb);
  run("drop bits 0..31", mk([](int c) { return c >= 32; }), d, nb);
  run("drop bits 0..63", mk([](int c) { return c >= 64; }), d, nb);
  run("drop c%32<4", mk([](int c) { return c % 32 >= 4; }), d, nb);
  run("drop c%8==0", mk([](int c) { return c % 8 != 0; }), d, nb);
  run("keep bits 0..7", mk([](int c) { return c < 8; }), d, nb);
  run("keep bits 0..31", mk([](int c) { return c < 32; }), d, nb);
  run("keep c%32<4", mk([](int c) { return c % 32 < 4; }), d, nb);
  run("keep c%8==0", mk([](int c) { return c % 8 == 0; }), d, nb);
  return 0;
}
