// lgs_bloom.hip -- lcdb's bloom filter on gfx950:
// ldb_hash (src/util/hash.c:22-58) and the builtin policy's build and match
// (src/util/bloom.c:82-165), for many filters / queries per launch.
//
//  * build: one wave per filter.  The filter's bits live in LDS (zeroed, then
//    every key's k probe bits set with ds_or_b32 -- bit `pos` of the
//    reference's byte array is bit pos % 32 of little-endian dword pos / 32),
//    then written out with dword stores plus the trailing k byte
//    (bloom.c:102-119).  Filters over kLdsBytes bytes set their bits with
//    global atomics on the zeroed output instead.  One lane hashes one key.
//  * match: one lane per (filter, key) query (bloom.c:121-165).
// `h % bits` uses a 64-bit reciprocal, exact for 32-bit operands.
#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {
namespace {

constexpr uint32_t kBloomSeed = 0xbc9f1d34u;   // bloom.c:64-67
constexpr uint32_t kHashMul = 0xc6a4a793u;     // hash.c:25
constexpr uint32_t kBloomWaves = 4;
constexpr uint32_t kLdsBytes = 8192;           // per wave

typedef uint32_t u32_u __attribute__((aligned(1)));

// Little-endian dword at an arbitrary byte address (reads the aligned dwords
// around it: up to 7 bytes past p).
__device__ __forceinline__ uint32_t ld32u(gptr<const uint8_t> p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const gptr<const uint32_t> w = (gptr<const uint32_t>)(a & ~3ull);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}

// hash.c:22-58 of p[0 .. n), seed kBloomSeed (bloom.c:64-67).
__device__ __forceinline__ uint32_t bloom_hash(gptr<const uint8_t> p, uint32_t n) {
  uint32_t h = kBloomSeed ^ (n * kHashMul);
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    h += ld32u(p + i);
    h *= kHashMul;
    h ^= h >> 16;
  }
  const uint32_t rest = n - i;
  if (rest) {
    const uint32_t w = ld32u(p + i);
    h += rest == 3 ? (w & 0xffffffu) : (rest == 2 ? (w & 0xffffu) : (w & 0xffu));
    h *= kHashMul;
    h ^= h >> 24;
  }
  return h;
}

// h % d for 32-bit h and d > 0, with m = floor((2^64 - 1) / d) + 1.
__device__ __forceinline__ uint32_t fastmod(uint32_t h, uint64_t m, uint32_t d) {
  const uint64_t low = m * h;
  return (uint32_t)__umul64hi(low, (uint64_t)d);
}

// bloom.c:69-80: bytes of filter bits for n keys.
__device__ __forceinline__ uint32_t filter_bytes(uint32_t n, uint32_t bpk) {
  uint64_t bits = (uint64_t)n * bpk;
  if (bits < 64) bits = 64;
  return (uint32_t)((bits + 7) / 8);
}

template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void bloom_build_kernel(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_len, const uint32_t* __restrict__ first,
    uint32_t nfilters, uint32_t bpk, uint32_t k, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off) {
  __shared__ uint32_t s_bits[WAVES][kLdsBytes / 4];
  const uint32_t wv = uni(threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  uint32_t* const sb = s_bits[wv];
  for (uint32_t f = blockIdx.x * WAVES + wv; f < nfilters; f += gridDim.x * WAVES) {
    const uint32_t k0 = uni(first[f]), k1 = uni(first[f + 1]);
    if (k1 <= k0) continue;                                  // empty filter: no bytes
    const uint32_t n = k1 - k0;
    const uint32_t bytes = filter_bytes(n, bpk);
    const uint32_t bits = 8 * bytes;
    const uint64_t m = ~0ull / bits + 1;
    const gptr<uint8_t> o = to_global(out) + uni64(out_off[f]);
    const uint64_t oa = (uint64_t)(uintptr_t)o;
    const bool in_lds = bytes <= kLdsBytes;
    if (in_lds) {
      for (uint32_t w = lane; w < (bytes + 3) / 4; w += kWave) sb[w] = 0;
    } else {
      for (uint32_t b = lane; b < bytes; b += kWave) o[b] = 0;
      __builtin_amdgcn_s_waitcnt(0x0f70);                    // zeros land before the ORs
    }
    order();
    for (uint32_t i = k0 + lane; i < k1; i += kWave) {      // bloom_add, bloom.c:82-100
      uint32_t h = bloom_hash(to_global(keys) + key_off[i], key_len[i]);
      const uint32_t delta = (h >> 17) | (h << 15);
      for (uint32_t j = 0; j < k; ++j) {
        const uint32_t pos = fastmod(h, m, bits);
        if (in_lds) {
          atomicOr(&sb[pos >> 5], 1u << (pos & 31u));
        } else {                                             // aligned dword holding byte pos / 8
          const uint64_t ba = oa + (pos >> 3);
          atomicOr((uint32_t*)(uintptr_t)(ba & ~3ull), 1u << (8 * (ba & 3u) + (pos & 7u)));
        }
        h += delta;
      }
    }
    order();
    if (in_lds) {                                            // whole dwords, then 1-3 bytes
      for (uint32_t w = lane; w < bytes / 4; w += kWave) *(gptr<u32_u>)(o + 4 * w) = sb[w];
      const uint32_t tail = bytes & ~3u;
      if (lane < (bytes & 3u)) o[tail + lane] = (uint8_t)(sb[tail / 4] >> (8 * lane));
    }
    if (lane == 0) o[bytes] = (uint8_t)k;                    // bloom.c:118
  }
}

__global__ __launch_bounds__(256) void bloom_match_kernel(
    const uint8_t* __restrict__ filters, const uint64_t* __restrict__ filter_off,
    const uint32_t* __restrict__ filter_len, const uint32_t* __restrict__ qfilter,
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_len, uint8_t* __restrict__ match, uint32_t nq) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const uint32_t f = qfilter[q];
  const gptr<const uint8_t> fp = to_global(filters) + filter_off[f];
  const uint32_t len = filter_len[f];
  uint8_t r;
  if (len < 2) {                                             // bloom.c:130-131
    r = 0;
  } else {
    const uint32_t bits = (len - 1) * 8;
    const uint32_t k = fp[len - 1];
    if (k > 30) {                                            // bloom.c:137-141
      r = 1;
    } else {
      const uint64_t m = ~0ull / bits + 1;
      uint32_t h = bloom_hash(to_global(keys) + key_off[q], key_len[q]);
      const uint32_t delta = (h >> 17) | (h << 15);
      r = 1;
      for (uint32_t j = 0; j < k; ++j) {
        const uint32_t pos = fastmod(h, m, bits);
        if ((fp[pos >> 3] & (1u << (pos & 7u))) == 0) {
          r = 0;
          break;
        }
        h += delta;
      }
    }
  }
  match[q] = r;
}

}  // namespace

hipError_t launch_bloom_build(const uint8_t* keys, const uint64_t* key_off,
                              const uint32_t* key_len, const uint32_t* first, uint32_t nfilters,
                              uint32_t bpk, uint32_t k, uint8_t* out, const uint64_t* out_off,
                              hipStream_t s) {
  if (nfilters == 0) return hipSuccess;
  const uint32_t want = (nfilters + kBloomWaves - 1) / kBloomWaves;
  const uint32_t grid = want < 4096 ? want : 4096;
  hipLaunchKernelGGL(bloom_build_kernel<kBloomWaves>, dim3(grid), dim3(64 * kBloomWaves), 0, s,
                     keys, key_off, key_len, first, nfilters, bpk, k, out, out_off);
  return hipGetLastError();
}

hipError_t launch_bloom_match(const uint8_t* filters, const uint64_t* filter_off,
                              const uint32_t* filter_len, const uint32_t* qfilter,
                              const uint8_t* keys, const uint64_t* key_off,
                              const uint32_t* key_len, uint8_t* match, uint32_t nq,
                              hipStream_t s) {
  if (nq == 0) return hipSuccess;
  hipLaunchKernelGGL(bloom_match_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, filters,
                     filter_off, filter_len, qfilter, keys, key_off, key_len, match, nq);
  return hipGetLastError();
}

}  // namespace lgs
