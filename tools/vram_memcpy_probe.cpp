// tools/vram_memcpy_probe.cpp -- host memcpy cost into pinned host memory vs
// fine-grained device memory (the service inbox).
// build: hipcc -O2 -mavx2 --offload-arch=gfx950 tools/vram_memcpy_probe.cpp -o tools/vram_probe2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include <immintrin.h>
int main() {
  unsigned char* p = nullptr; unsigned char* h = nullptr;
  if (hipExtMallocWithFlags((void**)&p, 1 << 20, hipDeviceMallocFinegrained) != hipSuccess) return 1;
  if (hipHostMalloc((void**)&h, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
  static unsigned char src[8192];
  for (int i = 0; i < 8192; ++i) src[i] = (unsigned char)i;
  for (int sz : {64, 4096, 8192}) {
    for (int dst = 0; dst < 2; ++dst) {
      unsigned char* d = dst ? p : h;
      double best = 1e9, sum = 0;
      for (int r = 0; r < 2000; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        memcpy(d + (r % 64) * 8192 % (1 << 19), src, sz);
        _mm_sfence();
        auto t1 = std::chrono::steady_clock::now();
        double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (us < best) best = us; sum += us;
      }
      printf("%s %d B: best %.3f us mean %.3f us\n", dst ? "vram" : "pinned", sz, best, sum / 2000);
    }
  }
  // read back cost from vram (CPU reads)
  static unsigned char back[4096];
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < 100; ++r) memcpy(back, p, 4096);
  auto t1 = std::chrono::steady_clock::now();
  printf("vram read 4096 B: %.3f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  return 0;
}
