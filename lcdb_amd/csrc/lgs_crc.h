// lgs_crc.h -- CRC32C of SSTable block trailers on gfx950 (crc32c.c:643-750,
// crc32c.h:38-57): the tables, the lane-segment fold and the copy helpers
// of the framing kernels (lgs_table.hip, whose header describes the method).
#pragma once

#include "lgs_device.h"

namespace lgs {
namespace {


constexpr uint32_t kPoly = 0x82f63b78u;       // CRC32C (Castagnoli), reflected
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.h:38
constexpr uint32_t kTrailer = 5;              // type byte + fixed32 crc (format.h)
// Geometry (round 6): kHalf lanes per block (64: one block per
// wave; 32: two), kNG 16-byte granules per lane.  64 x 48 bytes by default:
// one 3 KB pass for C2's ~2.3 KB blocks.  A lane's fold is a chain of
// dependent table lookups, and that chain, not the padding lanes, bounds the
// pass: short segments over all 64 lanes beat two blocks per wave.
#ifndef LGS_CRC_LANES
#define LGS_CRC_LANES 64
#define LGS_CRC_NG 3
#endif
constexpr uint32_t kHalf = LGS_CRC_LANES;     // lanes per block
constexpr uint32_t kNG = LGS_CRC_NG;          // granules per lane
constexpr uint32_t kBpw = kWave / kHalf;      // blocks per wave
constexpr uint32_t kLvl = kHalf == 64 ? 6 : 5;  // butterfly levels
constexpr uint32_t kSeg = 16 * kNG;           // bytes per lane per pass
constexpr uint32_t kPass = kSeg * kHalf;      // 2560
constexpr uint32_t kLaneBase = 2048;          // after the slice-by-8 tables
constexpr uint32_t kLaneStride = 129;         // 128 words a lane, +1 spreads the banks
constexpr uint32_t kInitBase = kLaneBase + kLaneStride * kHalf;   // kSeg start registers
constexpr uint32_t kBflyBase = kInitBase + kSeg;                  // 5 x 128: shifts by kSeg * 2^k bytes
constexpr uint32_t kTabWords = kBflyBase + kLvl * 128;            // copied to LDS (full image)
constexpr uint32_t kInvBase = kTabWords;                          // 16 x 128: divide by x^(8t), t < 16
constexpr uint32_t kAllWords = kInvBase + 16 * 128;
// The small LDS image (verify_kernel): slice-by-4 and the five butterfly
// shifts, 6.6 KB -- small enough to sit beside the ring decoder's 8 waves.
constexpr uint32_t kSmallWords = 1024 + kLvl * 128;
static_assert(kTabWords % 4 == 0 && kSmallWords % 4 == 0, "tables copied 16 bytes at a time");

// a * b mod P over GF(2), reflected (bit 31 is x^0).
constexpr uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
  }
  return p;
}

// t[16j + v] = (v << 4j) * m: multiplication by m as eight nibble lookups.
constexpr void nibbles(uint32_t* t, uint32_t m) {
  uint32_t bx[32] = {};                              // bx[i] = m * x^i
  bx[0] = m;
  for (int i = 1; i < 32; ++i) bx[i] = (bx[i - 1] & 1u) ? (bx[i - 1] >> 1) ^ kPoly : (bx[i - 1] >> 1);
  for (uint32_t j = 0; j < 8; ++j) {
    t[16 * j] = 0;
    for (uint32_t v = 1; v < 16; ++v) {
      uint32_t b = 0;
      while (!((v >> b) & 1u)) ++b;
      t[16 * j + v] = t[16 * j + (v & (v - 1))] ^ bx[31 - (4 * j + b)];  // bit 4j+b is x^(31-4j-b)
    }
  }
}

struct alignas(16) CrcTables {
  uint32_t w[kAllWords];
  // w[k*256 + b]          slice-by-8: byte b followed by k zero bytes (k < 4: slice-by-4)
  // w[kLaneBase + 129*L + 16j + v]  (v << 4j) times x^(8 kSeg (31 - L)): lane L's
  //                        segment followed by the 31 - L segments after it
  // w[kInitBase + z]       the register that z zero bytes turn into ~0
  // w[kBflyBase + 128k + 16j + v]  (v << 4j) times x^(8 kSeg 2^k)
  // w[kInvBase + 128t + 16j + v]   (v << 4j) times x^(-8t)
  constexpr CrcTables() : w() {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
      w[b] = c;
    }
    for (uint32_t k = 1; k < 8; ++k)
      for (uint32_t b = 0; b < 256; ++b) {
        const uint32_t prev = w[(k - 1) * 256 + b];
        w[k * 256 + b] = (prev >> 8) ^ w[prev & 0xffu];
      }
    uint32_t x8 = 0x40000000u;                           // x^1
    for (int j = 0; j < 3; ++j) x8 = gf_mul(x8, x8);     // x^8: one zero byte
    uint32_t xs = 0x80000000u;                           // x^(8 kSeg): one segment
    for (uint32_t j = 0; j < kSeg; ++j) xs = gf_mul(xs, x8);
    uint32_t xp = 0x80000000u;                           // x^0 for lane 31
    for (int L = (int)kHalf - 1; L >= 0; --L) {
      nibbles(w + kLaneBase + kLaneStride * (uint32_t)L, xp);
      xp = gf_mul(xp, xs);
    }
    for (uint32_t k = 0, xk = xs; k < kLvl; ++k, xk = gf_mul(xk, xk)) nibbles(w + kBflyBase + 128 * k, xk);
    // One zero byte maps c to T[c & 255] ^ (c >> 8), whose top byte is the
    // top byte of T[c & 255]; those 256 top bytes are distinct, so the step
    // inverts: find the index by the top byte, then undo the xor and shift.
    uint32_t inv_top[256] = {};
    for (uint32_t b = 0; b < 256; ++b) inv_top[w[b] >> 24] = b;
    uint32_t r = ~0u, m = 0x80000000u;                   // m = x^(-8t)
    for (uint32_t z = 0; z < kSeg; ++z) {
      w[kInitBase + z] = r;
      if (z < 16) nibbles(w + kInvBase + 128 * z, m);
      uint32_t idx = inv_top[r >> 24];
      r = ((r ^ w[idx]) << 8) | idx;
      idx = inv_top[m >> 24];
      m = ((m ^ w[idx]) << 8) | idx;
    }
  }
};

__constant__ CrcTables kCrc = CrcTables();

// a ^ b ^ c in one instruction (v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Xor over each half wave, in every lane of the half: a prefix within each
// row of 16 lanes (DPP row_shr 1, 2, 4, 8; lanes shifted in from outside the
// row read 0), then the half's two rows' last lanes.
__device__ __forceinline__ uint32_t half_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  const uint32_t a = lane_val(v, 15) ^ lane_val(v, 31), b = lane_val(v, 47) ^ lane_val(v, 63);
  if (kHalf == 64) return a ^ b;
  return lane_id() < kHalf ? a : b;
}

// Slice-by-4 in LDS at w[0 .. 1024).
struct CrcSlice {
  const uint32_t* w;
  // x = crc ^ dword 0 of the lane's segment: the register after all N
  // dwords (v[1 ..] follow), four bytes per dependent step.
  template <uint32_t N>
  __device__ __forceinline__ uint32_t fold(uint32_t x, const uint32_t (&v)[N]) const {
#pragma unroll
    for (uint32_t i = 0; i < N; ++i) x = step(x, i + 1 < N ? v[i + 1] : 0u);
    return x;
  }
  // x = crc ^ (four more bytes): the register after them, xor `next`.
  __device__ __forceinline__ uint32_t step(uint32_t x, uint32_t next) const {
    return xor3(xor3(w[768 + (x & 255u)], w[512 + ((x >> 8) & 255u)], w[256 + ((x >> 16) & 255u)]),
                w[x >> 24], next);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t crc, uint32_t b) const {
    return w[(crc ^ b) & 255u] ^ (crc >> 8);
  }
};

// The full image (kTabWords): slice-by-8 (a lane's chain is latency-bound:
// eight bytes per dependent step halve it), then each lane multiplies its
// segment's CRC by x^(8 kSeg (lanes - 1 - lane)) with its own table and one
// xor over the block's lanes.
struct Crc : CrcSlice {
  template <uint32_t N>
  __device__ __forceinline__ uint32_t fold(uint32_t x, const uint32_t (&v)[N]) const {
    static_assert(N % 2 == 0, "whole 8-byte steps");
#ifdef LGS_CRC_S4
    return CrcSlice::fold(x, v);                      // probe build: slice-by-4
#endif
#pragma unroll
    for (uint32_t i = 0; i < N; i += 2) {
      const uint32_t d = v[i + 1];
      x = xor3(xor3(w[1792 + (x & 255u)], w[1536 + ((x >> 8) & 255u)], w[1280 + ((x >> 16) & 255u)]),
               xor3(w[1024 + (x >> 24)], w[768 + (d & 255u)], w[512 + ((d >> 8) & 255u)]),
               xor3(w[256 + ((d >> 16) & 255u)], w[d >> 24], i + 2 < N ? v[i + 2] : 0u));
    }
    return x;
  }
  __device__ __forceinline__ uint32_t combine(uint32_t a, uint32_t lane) const {
    const uint32_t* n = w + kLaneBase + kLaneStride * (lane & (kHalf - 1));
    uint32_t t[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) t[j] = n[16 * j + ((a >> (4 * j)) & 15u)];
    return half_xor(xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]));
  }
  __device__ __forceinline__ uint32_t init(uint32_t z) const { return w[kInitBase + z]; }
};

// The small image (kSmallWords): a five-level butterfly per half -- lane i
// (a multiple of 2^(k+1)) joins the next 2^k lanes' CRC:
// c * x^(8 kSeg 2^k) ^ c(i + 2^k).
struct CrcSmall : CrcSlice {
  __device__ __forceinline__ uint32_t shift(uint32_t k, uint32_t a) const {
    const uint32_t* n = w + 1024 + 128 * k;
    uint32_t t[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) t[j] = n[16 * j + ((a >> (4 * j)) & 15u)];
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
  }
  __device__ __forceinline__ uint32_t combine(uint32_t c, uint32_t lane) const {
    uint32_t o;
    // k = 0..3 inside rows of 16 lanes (DPP row_shl: lane i reads lane i + 2^k).
    o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x101, 0xf, 0xf, false);
    if (!(lane & 1u)) c = shift(0, c) ^ o;
    o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x102, 0xf, 0xf, false);
    if (!(lane & 3u)) c = shift(1, c) ^ o;
    o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x104, 0xf, 0xf, false);
    if (!(lane & 7u)) c = shift(2, c) ^ o;
    o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x108, 0xf, 0xf, false);
    if (!(lane & 15u)) c = shift(3, c) ^ o;
    o = (uint32_t)__shfl_down((int)c, 16);
    if (!(lane & 31u)) c = shift(4, c) ^ o;
    if (kHalf == 64) {
      o = (uint32_t)__shfl_down((int)c, 32);
      if (lane == 0) c = shift(5, c) ^ o;
      return lane_val(c, 0);
    }
    return lane < kHalf ? lane_val(c, 0) : lane_val(c, kHalf & 63);
  }
  __device__ __forceinline__ uint32_t init(uint32_t z) const { return kCrc.w[kInitBase + z]; }
};

// A register with its last t zero bytes divided out (t may differ between
// the halves: vector loads of the constant tables).
__device__ __forceinline__ uint32_t unshift(uint32_t a, uint32_t t) {
  const uint32_t* n = kCrc.w + kInvBase + 128 * t;
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) r ^= n[16 * j + ((a >> (4 * j)) & 15u)];
  return r;
}

// The first `words` words of kCrc into LDS, every load issued before the
// first LDS store: one memory latency per workgroup, not one per 16 bytes.
template <uint32_t NT, uint32_t WORDS>
__device__ __forceinline__ void load_tables(uint32_t* s) {
  constexpr uint32_t kQ = WORDS / 4, kPer = (kQ + NT - 1) / NT;
  const u32x4* g = reinterpret_cast<const u32x4*>(kCrc.w);
  u32x4* l = reinterpret_cast<u32x4*>(s);
  u32x4 v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * NT;
    // (The small image is slice-by-4 then the butterfly shifts.)
    const uint32_t gi = WORDS == kSmallWords && i >= 256 ? i - 256 + kBflyBase / 4 : i;
    v[k] = g[i < kQ ? gi : 0];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * NT;
    if (i < kQ) l[i] = v[k];
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {          // crc32c.h:46-50
  return ((c >> 15) | (c << 17)) + kMaskDelta;
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {        // crc32c.h:53-57
  const uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
}

typedef u32x4 u32x4_a1 __attribute__((aligned(1)));

// src[0 .. e) to dst (e >= 16) by the 32 lanes of a half (hl = lane in the
// half): whole aligned 16-byte granules of the destination, each read as 16
// unaligned bytes of src; the ragged first and last granules as the 16 bytes
// that start at dst and end at dst + e (overlapping stores of equal bytes).
// Reads stay inside src[0 .. e).
__device__ __forceinline__ void copy_bytes(gptr<const uint8_t> src, gptr<uint8_t> dst, uint32_t e,
                                           uint32_t hl) {
  const uint64_t d0 = (uint64_t)(uintptr_t)dst;
  const uint32_t a = (uint32_t)((16u - (d0 & 15u)) & 15u);   // first aligned granule
  for (uint32_t k = a + 16 * hl; k + 16 <= e; k += 16 * kHalf)
    *(gptr<u32x4>)(dst + k) = *(gptr<const u32x4_a1>)(src + k);
  if (hl == 0 && a) *(gptr<u32x4_a1>)dst = *(gptr<const u32x4_a1>)src;
  if (hl == 1 && ((d0 + e) & 15u))
    *(gptr<u32x4_a1>)(dst + (e - 16)) = *(gptr<const u32x4_a1>)(src + (e - 16));
}

// Bytes [0, n) of a granule kept, the rest zero (n <= 16).
__device__ __forceinline__ u32x4 keep_below(uint32_t n) {
  u32x4 m;
#pragma unroll
  for (uint32_t d = 0; d < 4; ++d) {
    const uint32_t nd = n > 4 * d ? n - 4 * d : 0u;
    m[d] = nd >= 4 ? ~0u : (nd == 0 ? 0u : ~0u >> (32 - 8 * nd));
  }
  return m;
}

// src[0 .. len) to dst by a half: a byte a lane up to 32 bytes, else copy_bytes.
__device__ __forceinline__ void copy_block(gptr<const uint8_t> src, gptr<uint8_t> dst, uint32_t len,
                                           uint32_t hl) {
  if (len > kHalf) {
    copy_bytes(src, dst, len, hl);
  } else if (hl < len) {
    dst[hl] = src[hl];
  }
}

// Conditioned CRC32C (crc32c.c:643-750) of src[0 .. len) followed by the
// byte `type` when has_type -- the trailer CRC of table_builder.c:139-140
// before masking -- of one block per half wave; `on` false: no block (the
// result is unused).  Every lane of a half gets its block's CRC.  Reads
// only the aligned 16-byte granules holding a byte of src[0 .. len).  Called
// by the whole wave (cross-lane steps), never under divergent control flow.
// (Copies are a pass of their own, copy_block: the CRC pass storing its
// chunks cost 8-16 us more on C2's framing, profiles/r6m.)
template <class Tab>
__device__ __forceinline__ uint32_t half_crc(const Tab& T, gptr<const uint8_t> src, uint32_t len,
                                             uint32_t has_type, uint32_t type, bool on) {
  const uint32_t lane = lane_id(), hl = lane & (kHalf - 1);
  const uint32_t total = len + has_type;                      // message length L'
  uint32_t res = 0;
  if (on & (total < 4)) {                                     // tiny: one byte at a time
    uint32_t c = ~0u;
    for (uint32_t k = 0; k < len; ++k) c = T.byte(c, src[k]);
    if (has_type) c = T.byte(c, type);
    res = ~c;
  }
  const bool gen = on & (total >= 4);
  const uint64_t s0 = (uint64_t)(uintptr_t)src;
  const uint32_t t = (uint32_t)(0u - (uint32_t)(s0 + total)) & 15u;  // trailing zeros
  const uint32_t vtotal = total + t;
  const uint32_t passes = gen ? (vtotal + kPass - 1) / kPass : 0u;
  const uint32_t pad = passes * kPass - vtotal;               // leading zeros
  const uint64_t base = s0 - pad;                             // virtual byte 0: 16-aligned
  // The granule holding src[0] (pass 0) and the one holding index len (the
  // type byte's place, or the first byte after the block).
  const uint32_t vh = pad - (uint32_t)(s0 & 15u);
  const uint32_t lh = vh / kSeg, ih = (vh % kSeg) >> 4;
  const u32x4 keep_h = ~keep_below((uint32_t)(s0 & 15u));
  const uint32_t vt = (uint32_t)(((s0 + len) & ~15ull) - base);
  const uint32_t pt = vt / kPass, lt = (vt % kPass) / kSeg, it = ((vt % kPass) % kSeg) >> 4;
  const uint32_t ot = (uint32_t)((s0 + len) & 15u);          // index len's byte in it
  u32x4 keep_t = keep_below(ot), put_t = u32x4{0, 0, 0, 0};
  if (has_type) put_t[ot >> 2] = type << (8 * (ot & 3u));
  const uint32_t p0 = lane_val(passes, 0), p1 = lane_val(passes, kHalf & 63);
  const uint32_t maxp = p0 > p1 ? p0 : p1;
  uint32_t acc = 0;
  for (uint32_t p = 0; p < maxp; ++p) {
    const bool act = p < passes;
    const uint64_t seg = base + (uint64_t)p * kPass + (uint64_t)(kSeg * hl);
    u32x4 g[kNG];
#pragma unroll
    for (uint32_t i = 0; i < kNG; ++i) {
      const uint64_t a = seg + 16ull * i;
      g[i] = u32x4{0, 0, 0, 0};
      if (act & (a + 16 > s0) & (a < s0 + len)) g[i] = *(gptr<const u32x4>)(src + (int64_t)(a - s0));
    }
#pragma unroll
    for (uint32_t i = 0; i < kNG; ++i) {
      if ((p == 0) & (i == ih) & (hl == lh)) g[i] &= keep_h;  // bytes before src[0]
      if ((p == pt) & (i == it) & (hl == lt)) g[i] = (g[i] & keep_t) | put_t;
    }
    // Lane lane_h holds data index 0 at segment byte pad % kSeg (pass 0); the
    // lanes before it are all padding.  Its chain starts from the register
    // that those zero bytes turn into ~0 (the pre-conditioning); lane 0's
    // from the CRC of the passes before.
    const uint32_t lane_h = p == 0 ? pad / kSeg : 0u;
    uint32_t x = 0;
    if (act & (hl >= lane_h)) {
      const uint32_t init = p == 0 ? T.init(pad % kSeg) : acc;
      uint32_t v[4 * kNG];
#pragma unroll
      for (uint32_t i = 0; i < kNG; ++i) {
        v[4 * i] = g[i].x;
        v[4 * i + 1] = g[i].y;
        v[4 * i + 2] = g[i].z;
        v[4 * i + 3] = g[i].w;
      }
      x = T.fold(v[0] ^ (hl == lane_h ? init : 0u), v);
    }
    const uint32_t c = T.combine(x, lane);
    acc = act ? c : acc;
  }
  return gen ? ~unshift(acc, t) : res;
}

}  // namespace
}  // namespace lgs
