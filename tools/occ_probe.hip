// tools/occ_probe.hip -- how many one-wave workgroups with a given static
// LDS size a gfx950 CU holds at once (the LDS allocation granularity decides
// the encoder's occupancy: DESIGN.md 4.1).  Each wave holds its LDS and
// spins for kSpinUs; k workgroups per CU take one spin period while all k
// are resident, two once they are not.
//   build: hipcc -O2 --offload-arch=gfx950 tools/occ_probe.hip -o tools/occ_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr unsigned kSpinUs = 200;

template <int LDS, int W>
__global__ __launch_bounds__(64 * W) void hold(unsigned* sink) {
  __shared__ unsigned char buf[LDS];
  buf[threadIdx.x * (LDS / (64 * W))] = (unsigned char)threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();           // 100 MHz
  while (wall_clock64() - t0 < kSpinUs * 100ull) __builtin_amdgcn_s_sleep(8);
  if (buf[(threadIdx.x * 7) % LDS] == 0xfe) sink[threadIdx.x] = 1;   // keep buf live
}

// The largest k for which k one-wave workgroups per CU finish in one spin
// period (all resident at once).
template <int LDS, int W = 1>
static void run(int cus, unsigned* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int fit = 0;
  for (int k = (W == 1 ? 8 : 1); k <= 32 / W; ++k) {
    (void)hipGetLastError();
    hold<LDS, W><<<cus * k, 64 * W>>>(sink);               // warm-up
    hipEventRecord(a);
    hold<LDS, W><<<cus * k, 64 * W>>>(sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (ms * 1000.0 > 1.5 * kSpinUs) break;
    fit = k;
  }
  printf("lds %6d B per %2d-wave workgroup -> %2d workgroups = %2d waves/CU resident\n", LDS, W,
         fit, fit * W);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs, %zu B LDS per block max\n", p.gcnArchName, cus, p.sharedMemPerBlock);
  unsigned* sink;
  if (hipMalloc(&sink, 4096) != hipSuccess) return 1;
  run<4096>(cus, sink);
  run<8000>(cus, sink);
  run<8192>(cus, sink);
  run<8384>(cus, sink);
  run<8448>(cus, sink);
  run<8704>(cus, sink);
  run<8768>(cus, sink);
  run<8960>(cus, sink);
  run<9216>(cus, sink);
  run<10240>(cus, sink);
  run<10304>(cus, sink);
  run<12352>(cus, sink);
  run<16768, 2>(cus, sink);
  run<25152, 3>(cus, sink);
  run<75456, 9>(cus, sink);
  run<78912, 9>(cus, sink);
  run<83840, 10>(cus, sink);
  run<81920, 10>(cus, sink);
  run<92160, 11>(cus, sink);
  run<163840, 16>(cus, sink);
  hipFree(sink);
  return 0;
}
