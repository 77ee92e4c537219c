// Micro-benchmark (diagnostic): CPU write bandwidth into plain, hipHostRegister'ed
// and hipHostMalloc'ed host memory (the control-op staging buffers).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
using clk = std::chrono::steady_clock;
static double bench(void *p, size_t n) {
  std::memset(p, 1, n);
  auto t0 = clk::now();
  for (int r = 0; r < 20; r++) std::memset(p, r, n);
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count() / 20;
}
int main() {
  const size_t n = 256 << 10;
  void *a = std::aligned_alloc(4096, n);
  printf("plain      %.4f ms per 256 KiB\n", bench(a, n));
  void *b = std::aligned_alloc(4096, n);
  if (hipHostRegister(b, n, hipHostRegisterMapped) != hipSuccess) return 1;
  printf("registered %.4f ms per 256 KiB\n", bench(b, n));
  void *c = nullptr;
  if (hipHostMalloc(&c, n) != hipSuccess) return 1;
  printf("hostmalloc %.4f ms per 256 KiB\n", bench(c, n));
  void *d = nullptr;
  if (hipHostMalloc(&d, n, hipHostMallocNonCoherent) != hipSuccess) return 1;
  printf("noncoher.  %.4f ms per 256 KiB\n", bench(d, n));
  return 0;
}
