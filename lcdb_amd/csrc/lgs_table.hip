// lgs_table.hip -- SSTable block framing on gfx950:
//
//  * CRC32C of a block and its type byte, masked: the 5-byte block trailer
//    of src/table/table_builder.c:134-147 (crc32c.c:643-750, crc32c.h:38-57);
//  * the batched data-block writer: snappy encode (lgs_encode.hip), the
//    12.5 % rule of table_builder.c:190, trailers, and the blocks packed at
//    their file offsets (table_builder.c:123-153), byte-identical to
//    ldb_tablegen_write_block called once per block;
//  * the batched block reader: format.c:162-270 per block handle -- the
//    truncation check, the trailer CRC check (verify_checksums), the type
//    dispatch, raw copy or snappy decode (lgs_decode.hip).
//
// CRC on a wave (one block per wave, any length).  CRC32C is linear over
// GF(2), so the wave splits a block into 64-byte segments, one per lane,
// and combines them:
//  * the block is virtually left-padded with zeros to a multiple of 4096
//    bytes (a 4096-byte "pass" = 64 lanes x 64 bytes).  Leading zeros do not
//    change the unconditioned CRC (register 0 stays 0), and the ~0
//    pre-conditioning equals complementing the message's first 4 bytes, so
//    every pass is 64 equal segments and every lane does identical work;
//  * a lane folds its 16 dwords with slice-by-4 tables (4 LDS lookups per
//    dword);
//  * six butterfly levels (ds_bpermute) combine lane pairs: shift the left
//    CRC by 64 * 2^k zero bytes (multiply by x^(512 * 2^k) mod P, eight
//    nibble-table lookups) and xor the right one; passes combine the same
//    way with the 4096-byte shift.
// The block is staged pass by pass in LDS with 16-byte aligned loads; the
// same LDS image feeds the copy to the destination (the file image on the
// write path, the output slot of a raw block on the read path).
#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {
namespace {

constexpr uint32_t kPoly = 0x82f63b78u;       // CRC32C (Castagnoli), reflected
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.h:38
constexpr uint32_t kTrailer = 5;              // type byte + fixed32 crc (format.h)
constexpr uint32_t kSeg = 64;                 // bytes per lane per pass
constexpr uint32_t kPass = kSeg * kWave;      // 4096
constexpr uint32_t kLevels = 7;               // shifts by 64 * 2^k bytes, k = 0..6
constexpr uint32_t kTabWords = 4 * 256 + kLevels * 128;

// a * b mod P over GF(2), reflected (bit 31 is x^0).
constexpr uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
  }
  return p;
}

struct CrcTables {
  uint32_t w[kTabWords];
  // w[k*256 + b]          slice-by-4: byte b followed by k zero bytes
  // w[1024 + k*128 + 16j + v]  v << 4j times x^(512 * 2^k)
  constexpr CrcTables() : w() {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
      w[b] = c;
    }
    for (uint32_t k = 1; k < 4; ++k)
      for (uint32_t b = 0; b < 256; ++b) {
        const uint32_t prev = w[(k - 1) * 256 + b];
        w[k * 256 + b] = (prev >> 8) ^ w[prev & 0xffu];
      }
    uint32_t xp = 0x40000000u;                       // x^1
    for (int j = 0; j < 9; ++j) xp = gf_mul(xp, xp); // x^512: 64 zero bytes
    for (uint32_t k = 0; k < kLevels; ++k) {
      for (uint32_t j = 0; j < 8; ++j)
        for (uint32_t v = 0; v < 16; ++v) w[1024 + k * 128 + 16 * j + v] = gf_mul(xp, v << (4 * j));
      xp = gf_mul(xp, xp);
    }
  }
};

__constant__ CrcTables kCrc = CrcTables();

// The tables in LDS (one copy per workgroup).
struct Crc {
  const uint32_t* w;
  // Four more bytes (little-endian dword) into an unconditioned register.
  __device__ __forceinline__ uint32_t dword(uint32_t crc, uint32_t x) const {
    const uint32_t c = crc ^ x;
    return w[768 + (c & 255u)] ^ w[512 + ((c >> 8) & 255u)] ^ w[256 + ((c >> 16) & 255u)] ^
           w[c >> 24];
  }
  __device__ __forceinline__ uint32_t byte(uint32_t crc, uint32_t b) const {
    return w[(crc ^ b) & 255u] ^ (crc >> 8);
  }
  // crc followed by 64 * 2^k zero bytes.
  __device__ __forceinline__ uint32_t shift(uint32_t k, uint32_t a) const {
    const uint32_t* n = w + 1024 + k * 128;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) r ^= n[16 * j + ((a >> (4 * j)) & 15u)];
    return r;
  }
};

__device__ __forceinline__ void load_tables(uint32_t* s) {
  for (uint32_t i = threadIdx.x; i < kTabWords; i += blockDim.x) s[i] = kCrc.w[i];
  __syncthreads();
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {          // crc32c.h:46-50
  return ((c >> 15) | (c << 17)) + kMaskDelta;
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {        // crc32c.h:53-57
  const uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
}

// One pass staged in LDS as its 1024 virtual dwords V_m (bytes 4m .. 4m+3
// of the pass), re-aligned to the pass's byte 0 and stored at dword index
// m + m / 16: lane L's segment (V_16L .. V_16L+15) starts at dword 17 L, so
// the 64 lanes reading dword j of their segments hit 64 different banks.
constexpr uint32_t kImgWords = kPass / 4 + kPass / 64 + 8;
__device__ __forceinline__ uint32_t pidx(uint32_t m) { return m + (m >> 4); }

// A pass's source granules in registers: this lane's granule k is the
// aligned 16 bytes at g_lo + 16 (lane + 64 k), plus the dword after them;
// a pass covers at most 4 096 data bytes, so 5 granules a lane reach past it.
constexpr uint32_t kPassGr = 5;
struct PassLoad {
  u32x4 q[kPassGr];
  uint32_t nx[kPassGr];
};

// Issues the loads of the pass covering data [a, b) (all of them before any
// is used, so their latencies overlap; never a granule without a byte of
// src[a .. b + 16)).
__device__ __forceinline__ void load_pass(PassLoad& r, gptr<const uint8_t> src, uint32_t a,
                                          uint32_t b) {
  if (a >= b) return;
  const uint64_t s0 = (uint64_t)(uintptr_t)src;
  const uint64_t g_lo = (s0 + a) & ~15ull, g_hi = (s0 + b + 15) & ~15ull;
#pragma unroll
  for (uint32_t k = 0; k < kPassGr; ++k) {
    const uint64_t g = g_lo + 16ull * (lane_id() + kWave * k);
    if (g < g_hi) {
      r.q[k] = *(gptr<const u32x4>)(src + (int64_t)(g - s0));
      r.nx[k] = *(gptr<const uint32_t>)(src + (int64_t)(g + 16 - s0));
    }
  }
}

// Stages the pass whose virtual byte 0 is data index lo from its loads: every
// V_m holding a data byte of [a, b) (m < 1024).  Other dwords are left as
// they were.
__device__ __forceinline__ void store_pass(uint32_t* img, const PassLoad& r,
                                           gptr<const uint8_t> src, int64_t lo, uint32_t a,
                                           uint32_t b) {
  if (a >= b) return;
  const uint64_t s0 = (uint64_t)(uintptr_t)src;
  const uint64_t sb = s0 + (uint64_t)lo;                     // address of virtual byte 0
  const uint32_t sh = (uint32_t)(sb & 3u);
  const uint64_t ab = sb - sh;                               // V_m = bytes ab + 4m + sh ..
  const uint64_t g_lo = (s0 + a) & ~15ull, g_hi = (s0 + b + 15) & ~15ull;
#pragma unroll
  for (uint32_t k = 0; k < kPassGr; ++k) {
    const uint64_t g = g_lo + 16ull * (lane_id() + kWave * k);
    if (g < g_hi) {
      const u32x4 q = r.q[k];
      const uint32_t nx = r.nx[k];
      const int32_t i0 = (int32_t)((int64_t)(g - ab) >> 2);  // dword index of q.x
      const uint32_t v[5] = {__builtin_amdgcn_alignbyte(q.x, 0u, sh),   // bytes before g: never data
                             __builtin_amdgcn_alignbyte(q.y, q.x, sh),
                             __builtin_amdgcn_alignbyte(q.z, q.y, sh),
                             __builtin_amdgcn_alignbyte(q.w, q.z, sh),
                             __builtin_amdgcn_alignbyte(nx, q.w, sh)};
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int32_t m = i0 - 1 + t;
        if ((t > 0 || g == g_lo) && m >= 0 && m < (int32_t)(kPass / 4)) img[pidx((uint32_t)m)] = v[t];
      }
    }
  }
}

__device__ __forceinline__ void stage_pass(uint32_t* img, gptr<const uint8_t> src, int64_t lo,
                                           uint32_t a, uint32_t b) {
  PassLoad r;
  load_pass(r, src, a, b);
  store_pass(img, r, src, lo, a, b);
}

// Byte v (0 <= v < 4096 + 16) of a staged pass.
__device__ __forceinline__ uint32_t img_byte(const uint32_t* img, uint32_t v) {
  return (img[pidx(v >> 2)] >> (8 * (v & 3u))) & 0xffu;
}

// Writes data indices [a, e) of the staged pass (virtual byte 0 = data index
// lo) to dst + k, any alignment: whole 16-byte destination granules with one
// 16-byte store, the ragged granules at either end byte by byte.
__device__ __forceinline__ void copy_out(const uint32_t* img, int64_t lo, gptr<uint8_t> dst,
                                         uint32_t a, uint32_t e) {
  if (a >= e) return;
  const uint64_t d0 = (uint64_t)(uintptr_t)dst;
  const uint64_t g_lo = (d0 + a) & ~15ull, g_hi = (d0 + e + 15) & ~15ull;
  for (uint64_t g = g_lo + 16ull * lane_id(); g < g_hi; g += 16ull * kWave) {
    const int64_t k0 = (int64_t)(g - d0);                    // data index of the granule
    if (g >= d0 + a && g + 16 <= d0 + e) {
      const uint32_t v0 = (uint32_t)(k0 - lo), m0 = v0 >> 2, t = v0 & 3u;
      const uint32_t w0 = img[pidx(m0)], w1 = img[pidx(m0 + 1)], w2 = img[pidx(m0 + 2)],
                     w3 = img[pidx(m0 + 3)], w4 = img[pidx(m0 + 4)];
      const u32x4 v{__builtin_amdgcn_alignbyte(w1, w0, t), __builtin_amdgcn_alignbyte(w2, w1, t),
                    __builtin_amdgcn_alignbyte(w3, w2, t), __builtin_amdgcn_alignbyte(w4, w3, t)};
      *(gptr<u32x4>)(dst + k0) = v;
    } else {
      for (uint32_t t = 0; t < 16; ++t) {
        const int64_t k = k0 + t;
        if (k >= (int64_t)a && k < (int64_t)e) dst[k] = (uint8_t)img_byte(img, (uint32_t)(k - lo));
      }
    }
  }
}

// Conditioned CRC32C (crc32c.c:643-750) of src[0 .. len) followed by the
// byte `type` when has_type -- the trailer CRC of table_builder.c:139-140
// before masking.  When `copy`, src[0 .. len) is also written to dst, and
// the type byte after it when copy_type.  want_crc == false: copy only.
// Uniform result.  Reads may touch the 16 bytes after src[len - 1].
__device__ uint32_t wave_crc(const Crc& T, uint32_t* img, gptr<const uint8_t> src, uint32_t len,
                             uint32_t has_type, uint32_t type, gptr<uint8_t> dst, bool copy,
                             bool copy_type, bool want_crc) {
  const uint32_t lane = lane_id();
  const uint32_t total = len + has_type;                      // message length L'
  if (total < 4) {                                            // tiny: one byte at a time
    uint32_t c = ~0u;
    for (uint32_t k = 0; k < len; ++k) c = T.byte(c, src[k]);
    if (has_type) c = T.byte(c, type);
    const uint32_t ncopy = len + (copy_type ? has_type : 0u);
    if (copy && lane < ncopy) dst[lane] = lane < len ? src[lane] : (uint8_t)type;
    return ~c;
  }
  const uint32_t passes = (total + kPass - 1) / kPass;
  const uint32_t pad = passes * kPass - total;                // leading virtual zeros
  uint32_t acc = 0;
  for (uint32_t p = 0; p < passes; ++p) {
    const int64_t lo = (int64_t)p * kPass - pad;              // data index of virtual byte 0
    const uint32_t a = lo < 0 ? 0u : (uint32_t)lo;
    const uint32_t b = (uint32_t)(lo + kPass < (int64_t)len ? lo + kPass : (int64_t)len);
    const bool last = p + 1 == passes;
    stage_pass(img, src, lo, a, b);
    order();
    if (last && has_type && lane == 0) {                      // virtual byte 4095
      reinterpret_cast<uint8_t*>(img)[4 * pidx(kPass / 4 - 1) + 3] = (uint8_t)type;
    }
    order();
    if (want_crc) {
      uint32_t c = 0;
      const int64_t k0 = lo + (int64_t)(kSeg * lane);         // data index of the segment
      if (k0 + (int64_t)kSeg > 0) {                           // lanes wholly in the padding skip
#pragma unroll 4
        for (uint32_t j = 0; j < kSeg / 4; ++j) {
          const int32_t k = (int32_t)(k0 + 4 * j);            // data index of the dword
          const uint32_t raw = img[17 * lane + j];
          const uint32_t nk = (uint32_t)(-k);
          const uint32_t part = ~0u << (8 * (nk & 3u));       // used for -4 < k < 0
          const uint32_t vm = k >= 0 ? ~0u : (k <= -4 ? 0u : part);
          const uint32_t head = ~0u >> (8 * ((uint32_t)k & 3u)); // used for 0 <= k < 4
          const uint32_t cm = (k >= 4 || k <= -4) ? 0u : (k >= 0 ? head : part);
          c = T.dword(c, (raw & vm) ^ cm);                    // ~0 pre-conditioning
        }
      }
      // Six levels: lane i (i a multiple of 2^(lv+1)) joins its group with
      // the next one, c = c * x^(512 * 2^lv) ^ c(i + 2^lv).  Only those lanes
      // do the shift's 8 table lookups (all 64 doing them was ~half of the
      // kernel's LDS reads).
#pragma unroll
      for (uint32_t lv = 0; lv < 6; ++lv) {
        const uint32_t other = (uint32_t)__shfl_down((int)c, 1u << lv);
        if ((lane & ((2u << lv) - 1u)) == 0) c = T.shift(lv, c) ^ other;
      }
      const uint32_t pc = uni(c);                             // lane 0: the whole pass
      acc = p == 0 ? pc : uni(T.shift(6, vec(acc)) ^ pc);
    }
    if (copy) copy_out(img, lo, dst, a, last && copy_type ? b + has_type : b);
    order();
  }
  return ~acc;
}

// ---- row 1: masked (or plain) CRC32C per block -------------------------

template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void crc_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, const uint8_t* __restrict__ type,
    uint32_t masked, uint32_t* __restrict__ crc_out, uint32_t n) {
  __shared__ uint32_t s_tab[kTabWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_img[WAVES][kImgWords];
  load_tables(s_tab);
  const Crc T{s_tab};
  const uint32_t wv = uni(threadIdx.x >> 6);
  for (uint32_t i = blockIdx.x * WAVES + wv; i < n; i += gridDim.x * WAVES) {
    const uint32_t len = uni(in_len[i]);
    const uint32_t ty = type ? uni(type[i]) : 0u;
    const uint32_t c = wave_crc(T, s_img[wv], to_global(in) + uni64(in_off[i]), len,
                                type ? 1u : 0u, ty, nullptr, false, false, true);
    if (lane_id() == 0) crc_out[i] = masked ? crc_mask(c) : c;
  }
}

// ---- row 2: data-block framing ------------------------------------------

// Size of item i's region in one of three layouts:
//   MODE 0: encode slot, 16-byte aligned encode bound (snappy.c:354);
//   MODE 1: framed block in the file: contents (compressed only when that
//           saves more than 12.5 %, table_builder.c:190) + 5-byte trailer;
//   MODE 2: the encoded bytes alone, packed (lgs_encode_batch_host).
template <int MODE>
__device__ __forceinline__ uint64_t item_size(const uint32_t* raw_len, const uint32_t* enc_len,
                                              uint32_t i) {
  if (MODE == 2) return enc_len[i];
  const uint32_t L = raw_len[i];
  if (MODE == 0) return ((uint64_t)32 + L + L / 6 + 15) & ~15ull;
  const uint32_t e = enc_len ? enc_len[i] : 0xffffffffu;
  return (uint64_t)(e < L - L / 8 ? e : L) + kTrailer;
}

constexpr uint32_t kScanT = 256, kScanPer = 8, kScanItems = kScanT * kScanPer;

// Exclusive scan of u64 values inside one workgroup; returns the total.
__device__ __forceinline__ uint64_t wg_scan(uint64_t* s, uint64_t v, uint64_t* excl) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kScanT; d <<= 1) {
    const uint64_t t = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  *excl = s[threadIdx.x] - v;
  const uint64_t tot = s[kScanT - 1];
  __syncthreads();
  return tot;
}

template <int MODE>
__global__ __launch_bounds__(kScanT) void scan_part_kernel(const uint32_t* __restrict__ raw_len,
                                                           const uint32_t* __restrict__ enc_len,
                                                           uint64_t* __restrict__ part,
                                                           uint32_t n) {
  __shared__ uint64_t s[kScanT];
  const uint32_t i0 = blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  uint64_t sum = 0;
  for (uint32_t j = 0; j < kScanPer; ++j)
    if (i0 + j < n) sum += item_size<MODE>(raw_len, enc_len, i0 + j);
  uint64_t ex;
  const uint64_t tot = wg_scan(s, sum, &ex);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanT) void scan_top_kernel(uint64_t* __restrict__ part,
                                                          uint32_t nparts) {
  __shared__ uint64_t s[kScanT];
  const uint32_t per = (nparts + kScanT - 1) / kScanT;
  const uint32_t j0 = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) sum += part[j];
  uint64_t ex;
  wg_scan(s, sum, &ex);
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) {
    const uint64_t v = part[j];
    part[j] = ex;
    ex += v;
  }
}

template <int MODE>
__global__ __launch_bounds__(kScanT) void scan_out_kernel(const uint32_t* __restrict__ raw_len,
                                                          const uint32_t* __restrict__ enc_len,
                                                          const uint64_t* __restrict__ part,
                                                          uint64_t base, uint64_t* __restrict__ off,
                                                          uint64_t* __restrict__ end, uint32_t n) {
  __shared__ uint64_t s[kScanT];
  const uint32_t i0 = blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  uint64_t v[kScanPer];
  uint64_t sum = 0;
  for (uint32_t j = 0; j < kScanPer; ++j) {
    v[j] = i0 + j < n ? item_size<MODE>(raw_len, enc_len, i0 + j) : 0;
    sum += v[j];
  }
  uint64_t ex;
  wg_scan(s, sum, &ex);
  uint64_t at = base + part[blockIdx.x] + ex;
  for (uint32_t j = 0; j < kScanPer; ++j) {
    if (i0 + j < n) {
      off[i0 + j] = at;
      if (end && i0 + j == n - 1) *end = at + v[j];
    }
    at += v[j];
  }
}

// One wave per block: pick the contents (table_builder.c:182-199), write
// them and the trailer (:123-153) at file offset off[i] (file[0] is offset
// `base`), record the handle.
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void frame_kernel(
    const uint8_t* __restrict__ raw, const uint64_t* __restrict__ raw_off,
    const uint32_t* __restrict__ raw_len, const uint8_t* __restrict__ enc,
    const uint64_t* __restrict__ enc_off, const uint32_t* __restrict__ enc_len,
    uint8_t* __restrict__ file, uint64_t base, const uint64_t* __restrict__ foff,
    uint64_t* __restrict__ handle_off, uint64_t* __restrict__ handle_size, uint32_t n) {
  __shared__ uint32_t s_tab[kTabWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_img[WAVES][kImgWords];
  load_tables(s_tab);
  const Crc T{s_tab};
  const uint32_t wv = uni(threadIdx.x >> 6);
  for (uint32_t i = blockIdx.x * WAVES + wv; i < n; i += gridDim.x * WAVES) {
    const uint32_t L = uni(raw_len[i]);
    const uint32_t e = enc_len ? uni(enc_len[i]) : 0xffffffffu;
    const bool comp = e < L - L / 8;                                  // :190
    const uint32_t size = comp ? e : L;
    const gptr<const uint8_t> src = comp ? to_global((const uint8_t*)enc) + uni64(enc_off[i])
                                         : to_global(raw) + uni64(raw_off[i]);
    const uint64_t at = uni64(foff[i]);
    const gptr<uint8_t> dst = to_global(file) + (at - base);
    const uint32_t c = wave_crc(T, s_img[wv], src, size, 1u, comp ? 1u : 0u, dst, true, true, true);
    const uint32_t m = crc_mask(c);                                   // :142
    if (lane_id() < 4) dst[size + 1 + lane_id()] = (uint8_t)(m >> (8 * lane_id()));
    if (lane_id() == 0) {
      handle_off[i] = at;                                             // :128-129
      handle_size[i] = size;
    }
  }
}

// ---- row 3: block reads --------------------------------------------------

constexpr uint8_t kPending = 0xff;   // snappy block: status decided by the decoder

// format.c:162-231, 263-267 per handle; snappy blocks (:233-261) are handed
// to the decoder through dec_in_off/dec_len/dec_off/dec_cap (others get an
// empty input at file offset 0 and a zero-capacity dummy slot, so the
// decoder cannot touch their output).
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void check_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint32_t verify, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    uint64_t* __restrict__ dec_in_off, uint32_t* __restrict__ dec_len,
    uint64_t* __restrict__ dec_off, uint32_t* __restrict__ dec_cap, uint64_t dummy_off,
    uint32_t n) {
  __shared__ uint32_t s_tab[kTabWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_img[WAVES][kImgWords];
  load_tables(s_tab);
  const Crc T{s_tab};
  const uint32_t wv = uni(threadIdx.x >> 6);
  for (uint32_t i = blockIdx.x * WAVES + wv; i < n; i += gridDim.x * WAVES) {
    const uint64_t off = uni64(hoff[i]), size = uni64(hsize[i]);
    const uint32_t cap = uni(out_cap[i]);
    const uint64_t oo = uni64(out_off[i]);
    uint32_t st;
    uint32_t olen = 0;
    bool snappy = false;
    if (size > ~0ull - kTrailer) {                                    // :174-175
      st = kStCorrupt;
    } else if (off > file_len || file_len - off < size + kTrailer) {  // :195-198
      st = kStIoErr;
    } else if (size > 0x7fffffffull) {                                // beyond this ABI
      st = kStNoSpace;
    } else {
      const gptr<const uint8_t> data = to_global(file) + off;
      const uint32_t sz = (uint32_t)size;
      const uint32_t ty = uni(data[sz]);
      const bool raw_fits = ty == 0 && sz <= cap;
      bool ok = true;
      if (verify) {                                                   // :203-211
        const uint32_t stored = (uint32_t)data[sz + 1] | ((uint32_t)data[sz + 2] << 8) |
                                ((uint32_t)data[sz + 3] << 16) | ((uint32_t)data[sz + 4] << 24);
        const uint32_t c = wave_crc(T, s_img[wv], data, sz, 1u, ty, to_global(out) + oo,
                                    raw_fits, false, true);
        ok = crc_unmask(uni(stored)) == c;
      } else if (raw_fits) {
        wave_crc(T, s_img[wv], data, sz, 0u, 0u, to_global(out) + oo, true, false, false);
      }
      if (!ok) {
        st = kStBadCrc;
      } else if (ty == 0) {                                           // :213-231
        st = raw_fits ? kStOk : kStNoSpace;
        olen = raw_fits ? sz : 0u;
      } else if (ty == 1) {                                           // :233-261
        st = kPending;
        snappy = true;
      } else {                                                        // :263-267
        st = kStBadType;
      }
    }
    if (lane_id() == 0) {
      status[i] = (uint8_t)st;
      out_len[i] = olen;
      dec_in_off[i] = snappy ? off : 0u;   // never an out-of-range address
      dec_len[i] = snappy ? (uint32_t)size : 0u;
      dec_off[i] = snappy ? oo : dummy_off;
      dec_cap[i] = snappy ? cap : 0u;
    }
  }
}

__global__ __launch_bounds__(256) void merge_kernel(uint8_t* __restrict__ status,
                                                    uint32_t* __restrict__ out_len,
                                                    const uint8_t* __restrict__ dec_status,
                                                    const uint32_t* __restrict__ dec_out_len,
                                                    uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || status[i] != kPending) return;
  status[i] = dec_status[i];      // LGS_ST_CORRUPT / OK / NOSPACE, format.c:237-252
  out_len[i] = dec_out_len[i];
}

// Grid for the one-wave-per-block framing kernels: every workgroup
// resident at once (CUs x the occupancy the kernel's LDS allows), each
// loading the tables once and striding over blocks -- no second, partial
// round of workgroups.
constexpr uint32_t kFrameWaves = 4;
template <class K>
uint32_t frame_grid(K kernel, uint32_t n) {
  static uint32_t resident = 0;   // same on every device of the node
  if (resident == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64 * kFrameWaves, 0) !=
            hipSuccess ||
        cus <= 0 || per <= 0) {
      cus = 256;
      per = 4;
    }
    resident = (uint32_t)(cus * per);
  }
  const uint32_t want = (n + kFrameWaves - 1) / kFrameWaves;
  return want < resident ? (want ? want : 1u) : resident;
}

}  // namespace

hipError_t launch_crc(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      const uint8_t* type, int masked, uint32_t* crc, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(crc_kernel<kFrameWaves>, dim3(frame_grid(crc_kernel<kFrameWaves>, n)), dim3(64 * kFrameWaves),
                     0, s, in, in_off, in_len, type, (uint32_t)(masked != 0), crc, n);
  return hipGetLastError();
}

size_t scan_parts(uint32_t n) { return (n + kScanItems - 1) / kScanItems; }

hipError_t launch_scan(int mode, const uint32_t* raw_len, const uint32_t* enc_len, uint64_t* part,
                       uint64_t base, uint64_t* off, uint64_t* end, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t np = (uint32_t)scan_parts(n);
  if (mode == 0) {
    hipLaunchKernelGGL(scan_part_kernel<0>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  } else if (mode == 1) {
    hipLaunchKernelGGL(scan_part_kernel<1>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  } else {
    hipLaunchKernelGGL(scan_part_kernel<2>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  }
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanT), 0, s, part, np);
  if (mode == 0) {
    hipLaunchKernelGGL(scan_out_kernel<0>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  } else if (mode == 1) {
    hipLaunchKernelGGL(scan_out_kernel<1>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  } else {
    hipLaunchKernelGGL(scan_out_kernel<2>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  }
  return hipGetLastError();
}

// Item i's len[i] bytes from src + src_off[i] to dst + dst_off[i], one wave
// per item: whole 16-byte destination granules with one (unaligned) 16-byte
// load and one aligned store, the ragged ends byte by byte.
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void pack_kernel(const uint8_t* __restrict__ src,
                                                         const uint64_t* __restrict__ src_off,
                                                         const uint32_t* __restrict__ len,
                                                         uint8_t* __restrict__ dst,
                                                         const uint64_t* __restrict__ dst_off,
                                                         uint32_t n) {
  typedef u32x4 u32x4_g __attribute__((aligned(1)));
  for (uint32_t i = uni(blockIdx.x * WAVES + (threadIdx.x >> 6)); i < n;
       i += gridDim.x * WAVES) {
    const gptr<const uint8_t> s = to_global(src) + src_off[i];
    const gptr<uint8_t> d = to_global(dst) + dst_off[i];
    const uint32_t e = len[i];
    const uint64_t d0 = (uint64_t)(uintptr_t)d;
    const uint64_t g_lo = d0 & ~15ull, g_hi = (d0 + e + 15) & ~15ull;
    for (uint64_t g = g_lo + 16ull * lane_id(); g < g_hi; g += 16ull * kWave) {
      const int64_t k0 = (int64_t)(g - d0);
      if (g >= d0 && g + 16 <= d0 + e) {
        *(gptr<u32x4>)(d + k0) = *(gptr<const u32x4_g>)(s + k0);
      } else {
        for (uint32_t t = 0; t < 16; ++t) {
          const int64_t k = k0 + t;
          if (k >= 0 && k < (int64_t)e) d[k] = s[k];
        }
      }
    }
  }
}

hipError_t launch_pack(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                       uint8_t* dst, const uint64_t* dst_off, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pack_kernel<kFrameWaves>, dim3(frame_grid(pack_kernel<kFrameWaves>, n)),
                     dim3(64 * kFrameWaves), 0, s, src, src_off, len, dst, dst_off, n);
  return hipGetLastError();
}

hipError_t launch_frame(const FrameArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(frame_kernel<kFrameWaves>, dim3(frame_grid(frame_kernel<kFrameWaves>, a.n)), dim3(64 * kFrameWaves), 0,
                     s, a.raw, a.raw_off, a.raw_len, a.enc, a.enc_off, a.enc_len, a.file, a.base,
                     a.foff, a.handle_off, a.handle_size, a.n);
  return hipGetLastError();
}

hipError_t launch_check(const CheckArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(check_kernel<kFrameWaves>, dim3(frame_grid(check_kernel<kFrameWaves>, a.n)), dim3(64 * kFrameWaves), 0,
                     s, a.file, a.file_len, a.hoff, a.hsize, a.verify, a.out, a.out_off,
                     a.out_cap, a.out_len, a.status, a.dec_in_off, a.dec_len, a.dec_off, a.dec_cap,
                     a.dummy_off, a.n);
  return hipGetLastError();
}

hipError_t launch_merge(uint8_t* status, uint32_t* out_len, const uint8_t* dec_status,
                        const uint32_t* dec_out_len, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(merge_kernel, dim3((n + 255) / 256), dim3(256), 0, s, status, out_len,
                     dec_status, dec_out_len, n);
  return hipGetLastError();
}

}  // namespace lgs
