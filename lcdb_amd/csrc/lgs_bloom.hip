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

// The hashed length of a key: ldb_ifp_build/_match (dbformat.c:308-334) drop
// the 8-byte trailer of internal keys (trim = 8); shorter keys, an assert in
// the reference, hash as empty.
__device__ __forceinline__ uint32_t trimmed(uint32_t len, uint32_t trim) {
  return len > trim ? len - trim : 0u;
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
    const uint64_t* __restrict__ out_off, uint32_t trim) {
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
      uint32_t h = bloom_hash(to_global(keys) + key_off[i], trimmed(key_len[i], trim));
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

// bloom.c:121-165: filter fp[0 .. len) against the key at kp (klen bytes).
__device__ __forceinline__ uint8_t bloom_probe(gptr<const uint8_t> fp, uint32_t len,
                                               gptr<const uint8_t> kp, uint32_t klen) {
  if (len < 2) return 0;                                     // bloom.c:130-131
  const uint32_t bits = (len - 1) * 8;
  const uint32_t k = fp[len - 1];
  if (k > 30) return 1;                                      // bloom.c:137-141
  const uint64_t m = ~0ull / bits + 1;
  uint32_t h = bloom_hash(kp, klen);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (uint32_t j = 0; j < k; ++j) {
    const uint32_t pos = fastmod(h, m, bits);
    if ((fp[pos >> 3] & (1u << (pos & 7u))) == 0) return 0;
    h += delta;
  }
  return 1;
}

__global__ __launch_bounds__(256) void bloom_match_kernel(
    const uint8_t* __restrict__ filters, const uint64_t* __restrict__ filter_off,
    const uint32_t* __restrict__ filter_len, const uint32_t* __restrict__ qfilter,
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_len, uint8_t* __restrict__ match, uint32_t nq) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const uint32_t f = qfilter[q];
  match[q] = bloom_probe(to_global(filters) + filter_off[f], filter_len[f],
                         to_global(keys) + key_off[q], key_len[q]);
}

// ---- the filter block of one table (src/table/filter_block.c) ----
//
// The table builder adds data block b's keys, writes the block, then calls
// ldb_filtergen_start_block(offset after it) (table_builder.c:242-243,
// 276-277): filters are generated until there is one per started 2 KiB, the
// first taking the pending keys.  Offsets only grow, so block b's keys land
// in filter win(b) = (b == 0 ? 0 : block_off[b] >> 11) -- the filter
// ldb_filter_matches(block_off[b]) reads (filter_block.c:203) -- and the
// filters are win's runs.  Their count F is data_end >> 11, plus one when
// the last window's keys are still pending at ldb_filtergen_finish
// (:131-135).

constexpr uint32_t kFilterBaseLg = 11;                       // filter_block.c:31

__device__ __forceinline__ uint64_t win_of(const uint64_t* block_off, uint32_t b) {
  return b == 0 ? 0 : block_off[b] >> kFilterBaseLg;
}

// kf[j] = first key of filter j = block_first[first block whose window is
// >= j], j in [0, fmax]: lane b writes the j in (win(b-1), win(b)], lane
// nblocks the rest (its keys end the table).  meta = {last window, data_end
// >> 11, nblocks > 0} for filter_count.
__global__ __launch_bounds__(256) void filter_layout_kernel(
    const uint32_t* __restrict__ block_first, const uint64_t* __restrict__ block_off,
    uint32_t nblocks, uint64_t data_end, uint32_t fmax, uint32_t* __restrict__ kf,
    uint32_t* __restrict__ meta) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b > nblocks) return;
  const uint64_t lo = b == 0 ? 0 : win_of(block_off, b - 1) + 1;
  const uint64_t hi = b < nblocks ? win_of(block_off, b) : (uint64_t)fmax;
  const uint32_t v = block_first[b];
  for (uint64_t j = lo; j <= hi && j <= fmax; ++j) kf[j] = v;
  if (b == nblocks) {
    const uint64_t wl = nblocks ? win_of(block_off, nblocks - 1) : 0;
    meta[0] = (uint32_t)(wl < fmax ? wl : fmax);
    meta[1] = (uint32_t)(data_end >> kFilterBaseLg);
    meta[2] = nblocks > 0;
  }
}

// F, the number of filters: one per started 2 KiB, plus one when the last
// window's keys are still pending at ldb_filtergen_finish (:131-135).  kf[fmax]
// = all keys; F <= fmax since the last window is at most data_end >> 11.
__device__ __forceinline__ uint32_t filter_count(const uint32_t* kf, const uint32_t* meta,
                                                 uint32_t fmax) {
  if (meta[2] == 0) return 0;
  const uint32_t wl = meta[0], e = meta[1];
  if (e > wl) return e;
  return kf[fmax] > kf[wl] ? wl + 1 : wl;
}

// Filter sizes -> offsets foff[j] (j <= F), then the offset array, its start
// and base_lg (filter_block.c:137-149); size[0] = block bytes.  A three-pass
// scan: tile sums, one workgroup over the tile sums (part[nparts] = total),
// tile scans writing the results.  Tiles of kTile filters, 8 per thread.
constexpr uint32_t kScanT = 256, kScanPer = 8, kTile = kScanT * kScanPer;

__device__ __forceinline__ uint64_t filter_size_at(const uint32_t* kf, uint32_t f, uint32_t bpk,
                                                   uint32_t j) {
  if (j >= f || kf[j + 1] <= kf[j]) return 0;
  return filter_bytes(kf[j + 1] - kf[j], bpk) + 1ull;
}

// Exclusive scan of one u64 per thread over the workgroup; returns the total.
__device__ __forceinline__ uint64_t wg_scan64(uint64_t* s_wave, uint64_t v, uint64_t* excl) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint64_t x = v;
  for (uint32_t d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  if (lane == kWave - 1) s_wave[wv] = x;
  __syncthreads();
  uint64_t before = 0, total = 0;
  for (uint32_t w = 0; w < kScanT / kWave; ++w) {
    if (w < wv) before += s_wave[w];
    total += s_wave[w];
  }
  __syncthreads();
  *excl = before + x - v;
  return total;
}

__global__ __launch_bounds__(kScanT) void filter_part_kernel(const uint32_t* __restrict__ kf,
                                                             const uint32_t* __restrict__ meta,
                                                             uint32_t fmax, uint32_t bpk,
                                                             uint64_t* __restrict__ part) {
  __shared__ uint64_t s_wave[kScanT / kWave];
  const uint32_t f = filter_count(kf, meta, fmax);
  const uint32_t j0 = blockIdx.x * kTile + threadIdx.x * kScanPer;
  uint64_t sum = 0;
  for (uint32_t q = 0; q < kScanPer; ++q) sum += filter_size_at(kf, f, bpk, j0 + q);
  uint64_t ex;
  const uint64_t tot = wg_scan64(s_wave, sum, &ex);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanT) void filter_top_kernel(uint64_t* __restrict__ part,
                                                            uint32_t nparts) {
  __shared__ uint64_t s_wave[kScanT / kWave];
  const uint32_t per = (nparts + kScanT - 1) / kScanT;
  const uint32_t j0 = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) sum += part[j];
  uint64_t ex;
  const uint64_t tot = wg_scan64(s_wave, sum, &ex);
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) {
    const uint64_t v = part[j];
    part[j] = ex;
    ex += v;
  }
  if (threadIdx.x == 0) part[nparts] = tot;
}

__global__ __launch_bounds__(kScanT) void filter_out_kernel(
    const uint32_t* __restrict__ kf, const uint32_t* __restrict__ meta, uint32_t fmax,
    uint32_t bpk, const uint64_t* __restrict__ part, uint32_t nparts, uint64_t* __restrict__ foff,
    uint8_t* __restrict__ out, uint64_t* __restrict__ size) {
  __shared__ uint64_t s_wave[kScanT / kWave];
  const uint32_t f = filter_count(kf, meta, fmax);
  const uint32_t j0 = blockIdx.x * kTile + threadIdx.x * kScanPer;
  uint64_t v[kScanPer];
  uint64_t sum = 0;
  for (uint32_t q = 0; q < kScanPer; ++q) {
    v[q] = filter_size_at(kf, f, bpk, j0 + q);
    sum += v[q];
  }
  uint64_t ex;
  wg_scan64(s_wave, sum, &ex);
  const uint64_t total = part[nparts];
  const gptr<uint8_t> arr = to_global(out) + total;          // the offset array
  uint64_t at = part[blockIdx.x] + ex;
  for (uint32_t q = 0; q < kScanPer; ++q) {
    const uint32_t j = j0 + q;
    if (j < f) {
      foff[j] = at;
      for (uint32_t b = 0; b < 4; ++b) arr[4ull * j + b] = (uint8_t)(at >> (8 * b));
    } else if (j == f) {                                     // array start, base_lg
      foff[j] = at;
      for (uint32_t b = 0; b < 4; ++b) arr[4ull * f + b] = (uint8_t)(total >> (8 * b));
      arr[4ull * f + 4] = (uint8_t)kFilterBaseLg;
      size[0] = total + 4ull * f + 5;
    }
    at += v[q];
  }
}

// ldb_filter_init + ldb_filter_matches (filter_block.c:170-225): query q is
// (data block at qoff[q], key q); one lane per query.
__device__ __forceinline__ uint32_t le32(gptr<const uint8_t> p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(256) void filter_match_kernel(
    const uint8_t* __restrict__ blk, uint64_t n, const uint64_t* __restrict__ qoff,
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_len, uint32_t trim, uint8_t* __restrict__ match,
    uint32_t nq) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const gptr<const uint8_t> d = to_global(blk);
  uint8_t r = 1;                                  // no filter: "errors are potential matches"
  if (n >= 5) {
    const uint32_t base_lg = d[n - 1] & 63u;
    const uint64_t last_word = le32(d + n - 5);
    if (last_word <= n - 5) {
      const uint64_t num = (n - 5 - last_word) / 4;
      const uint64_t index = qoff[q] >> base_lg;
      if (index < num) {
        const uint32_t start = le32(d + last_word + 4 * index);
        const uint32_t limit = le32(d + last_word + 4 * index + 4);
        if (start <= limit && limit <= last_word)
          r = bloom_probe(d + start, limit - start, to_global(keys) + key_off[q],
                          trimmed(key_len[q], trim));
        else if (start == limit)
          r = 0;
      }
    }
  }
  match[q] = r;
}

}  // namespace

hipError_t launch_bloom_build(const uint8_t* keys, const uint64_t* key_off,
                              const uint32_t* key_len, const uint32_t* first, uint32_t nfilters,
                              uint32_t bpk, uint32_t k, uint8_t* out, const uint64_t* out_off,
                              uint32_t trim, hipStream_t s) {
  if (nfilters == 0) return hipSuccess;
  const uint32_t want = (nfilters + kBloomWaves - 1) / kBloomWaves;
  const uint32_t grid = want < 4096 ? want : 4096;
  hipLaunchKernelGGL(bloom_build_kernel<kBloomWaves>, dim3(grid), dim3(64 * kBloomWaves), 0, s,
                     keys, key_off, key_len, first, nfilters, bpk, k, out, out_off, trim);
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

hipError_t launch_filter_block_build(const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, const uint32_t* block_first,
                                     const uint64_t* block_off, uint32_t nblocks,
                                     uint64_t data_end, uint32_t bpk, uint32_t k, uint32_t trim,
                                     uint8_t* out, uint64_t* size, uint32_t* kf, uint64_t* foff,
                                     uint64_t* part, uint32_t* meta, hipStream_t s) {
  const uint32_t fmax = (uint32_t)(data_end >> kFilterBaseLg) + 1;
  hipLaunchKernelGGL(filter_layout_kernel, dim3(nblocks / 256 + 1), dim3(256), 0, s,
                     block_first, block_off, nblocks, data_end, fmax, kf, meta);
  const uint32_t nparts = (fmax + 1 + kTile - 1) / kTile;
  hipLaunchKernelGGL(filter_part_kernel, dim3(nparts), dim3(kScanT), 0, s, kf, meta, fmax, bpk,
                     part);
  hipLaunchKernelGGL(filter_top_kernel, dim3(1), dim3(kScanT), 0, s, part, nparts);
  hipLaunchKernelGGL(filter_out_kernel, dim3(nparts), dim3(kScanT), 0, s, kf, meta, fmax, bpk,
                     part, nparts, foff, out, size);
  // Filters past F are empty (kf constant there): the build skips them.
  return launch_bloom_build(keys, key_off, key_len, kf, fmax, bpk, k, out, foff, trim, s);
}

size_t filter_block_parts(uint64_t data_end) {
  return (size_t)(((data_end >> kFilterBaseLg) + 2 + kTile - 1) / kTile) + 1;
}

hipError_t launch_filter_block_match(const uint8_t* blk, uint64_t n, const uint64_t* qoff,
                                     const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, uint32_t trim, uint8_t* match,
                                     uint32_t nq, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  hipLaunchKernelGGL(filter_match_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, blk, n, qoff,
                     keys, key_off, key_len, trim, match, nq);
  return hipGetLastError();
}

}  // namespace lgs
