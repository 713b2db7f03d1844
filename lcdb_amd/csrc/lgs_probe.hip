// HBM copy probe: the achievable-bandwidth yardstick bench.py reports beside
// the spec peak (SURVEY §8d asks for an achievable rate, not only 8 TB/s).
// Not on the codec path.  Each lane moves four 16-byte vectors, all four
// loads issued before the first store, so a wave keeps 4 x 1 KiB in flight;
// a 256-lane workgroup covers 16 KiB and a 1 GiB copy is 65 536 workgroups,
// far past the 256 CUs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lgs_launch.h"

namespace lgs {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kCopyThreads = 256;
constexpr int kCopyVec = 4;                 // uint4 per lane
constexpr size_t kCopyTile = (size_t)kCopyThreads * kCopyVec * 16;

__global__ __launch_bounds__(kCopyThreads) void hbm_copy_kernel(v4u* __restrict__ dst,
                                                                const v4u* __restrict__ src,
                                                                size_t nvec) {
  size_t base = (size_t)blockIdx.x * (kCopyThreads * kCopyVec) + threadIdx.x;
  v4u v[kCopyVec];
  if (base + (kCopyVec - 1) * kCopyThreads < nvec) {
#pragma unroll
    for (int k = 0; k < kCopyVec; ++k) v[k] = __builtin_nontemporal_load(&src[base + k * kCopyThreads]);
#pragma unroll
    for (int k = 0; k < kCopyVec; ++k) __builtin_nontemporal_store(v[k], &dst[base + k * kCopyThreads]);
  } else {
    for (int k = 0; k < kCopyVec; ++k) {
      size_t i = base + k * kCopyThreads;
      if (i < nvec) dst[i] = src[i];
    }
  }
}

}  // namespace

hipError_t launch_hbm_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  size_t nvec = bytes / 16;
  size_t grid = (bytes + kCopyTile - 1) / kCopyTile;
  if (grid == 0) return hipSuccess;
  if (grid > 0x7fffffffu) return hipErrorInvalidValue;
  hbm_copy_kernel<<<(unsigned)grid, kCopyThreads, 0, s>>>((v4u*)dst, (const v4u*)src, nvec);
  return hipGetLastError();
}

}  // namespace lgs
