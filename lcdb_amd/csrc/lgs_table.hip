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
// CRC on half a wave (two blocks per wave, any length).  CRC32C is linear
// over GF(2), so the 32 lanes of a half split a block into 80-byte
// segments, one per lane, and combine them:
//  * the block's bytes are taken where they lie, as the aligned 16-byte
//    granules that hold them (only those: never another page), extended by
//    t < 16 trailing zeros to the end of the last granule and by leading
//    zeros to a multiple of 2560 bytes (a "pass" = 32 lanes x 80 bytes).
//    Leading zeros leave a register that is 0 at 0; the ~0
//    pre-conditioning is the start register of the lane holding byte 0
//    (the register that its leading zeros turn into ~0); the trailing
//    zeros are divided out at the end (a multiplication by x^(-8t));
//  * a lane folds its 20 dwords with slice-by-4 tables (4 LDS lookups per
//    dword), then multiplies its CRC by x^(640 (31 - lane)) -- the zero
//    bytes after its segment -- with a table of its own (eight nibble
//    lookups), and one xor-reduction over the half (DPP) gives the pass's
//    CRC.  The CRC of the passes before enters as lane 0's start register.
// Copies to the destination (the file image on the write path, the output
// slot of a raw block on the read path) are a pass of their own over whole
// aligned destination granules (copy_bytes).
#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {
namespace {

constexpr uint32_t kPoly = 0x82f63b78u;       // CRC32C (Castagnoli), reflected
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.h:38
constexpr uint32_t kTrailer = 5;              // type byte + fixed32 crc (format.h)
// Two blocks per wave (round 6): half a wave (32 lanes) per block, 80 bytes
// (five granules) per lane, so a pass is 2 560 bytes -- one pass for C2's
// ~2.3 KB blocks, where a 64-lane, 4 096-byte pass spent 43 % of its
// instructions on padding lanes.
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

// ---- row 1: masked (or plain) CRC32C per block -------------------------

template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void crc_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, const uint8_t* __restrict__ type,
    uint32_t masked, uint32_t* __restrict__ crc_out, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
  load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint32_t len = on ? in_len[i] : 0u;
    const uint32_t ty = type && on ? type[i] : 0u;
    const uint32_t c = half_crc(T, to_global(in) + (on ? in_off[i] : 0), len, type ? 1u : 0u, ty, on);
    if (on & (hl == 0)) crc_out[i] = masked ? crc_mask(c) : c;
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
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
  load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint32_t L = on ? raw_len[i] : 0u;
    const uint32_t e = enc_len && on ? enc_len[i] : 0xffffffffu;
    const bool comp = e < L - L / 8;                                  // :190
    const uint32_t size = comp ? e : L;
    const gptr<const uint8_t> src = !on ? to_global(raw)
                                  : comp ? to_global((const uint8_t*)enc) + enc_off[i]
                                         : to_global(raw) + raw_off[i];
    const uint64_t at = on ? foff[i] : base;
    const gptr<uint8_t> dst = to_global(file) + (at - base);
    const uint32_t c = half_crc(T, src, size, 1u, comp ? 1u : 0u, on);
    if (on) {
      copy_block(src, dst, size, hl);
      if (hl == 0) dst[size] = (uint8_t)(comp ? 1u : 0u);
      const uint32_t m = crc_mask(c);                                 // :142
      if (hl < 4) dst[size + 1 + hl] = (uint8_t)(m >> (8 * hl));
      if (hl == 0) {
        handle_off[i] = at;                                           // :128-129
        handle_size[i] = size;
      }
    }
  }
}

// ---- row 3: block reads --------------------------------------------------

constexpr uint8_t kPending = 0xff;   // snappy block: status decided by the decoder

// format.c:162-231, 263-267 per handle; snappy blocks (:233-261) are handed
// to the decoder through dec_in_off/dec_len/dec_off/dec_cap (others get an
// empty input at file offset 0 and a zero-capacity dummy slot, so the
// decoder cannot touch their output).
template <uint32_t WAVES, bool CRC>
__global__ __launch_bounds__(64 * WAVES) void check_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint32_t verify, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    uint64_t* __restrict__ dec_in_off, uint32_t* __restrict__ dec_len,
    uint64_t* __restrict__ dec_off, uint32_t* __restrict__ dec_cap, uint64_t dummy_off,
    uint32_t n) {
  // Without CRC (verify == 0, or the checks run in verify_kernel) no tables:
  // this instance holds no LDS and runs beside verify_kernel.
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[CRC ? kTabWords : 4];
  if (CRC) load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint64_t off = on ? hoff[i] : 0, size = on ? hsize[i] : 0;
    const uint32_t cap = on ? out_cap[i] : 0u;
    const uint64_t oo = on ? out_off[i] : 0;
    uint32_t st = kStCorrupt;
    uint32_t olen = 0;
    bool snappy = false;
    // The checks of format.c:174-198 first; the trailer CRC (:203-211) of
    // every block that passes them, by the whole wave (half_crc).
    const bool bad_size = size > ~0ull - kTrailer;                    // :174-175
    const bool io = !bad_size && (off > file_len || file_len - off < size + kTrailer);  // :195-198
    const bool big = !bad_size && !io && size > 0x7fffffffull;        // beyond this ABI
    const bool body = on && !bad_size && !io && !big;
    const gptr<const uint8_t> data = to_global(file) + (body ? off : 0);
    const uint32_t sz = body ? (uint32_t)size : 0u;
    const uint32_t ty = body ? (uint32_t)data[sz] : 0u;
    uint32_t c = 0;
    if (CRC) c = half_crc(T, data, sz, 1u, ty, body && verify);
    if (bad_size) {
      st = kStCorrupt;
    } else if (io) {
      st = kStIoErr;
    } else if (big) {
      st = kStNoSpace;
    } else if (on) {
      const bool raw_fits = ty == 0 && sz <= cap;
      bool ok = true;
      if (CRC && verify) {                                            // :203-211
        const uint32_t stored = (uint32_t)data[sz + 1] | ((uint32_t)data[sz + 2] << 8) |
                                ((uint32_t)data[sz + 3] << 16) | ((uint32_t)data[sz + 4] << 24);
        ok = crc_unmask(stored) == c;
      }
      if (raw_fits) copy_block(data, to_global(out) + oo, sz, hl);   // (unspecified if the CRC fails)
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
    if (on & (hl == 0)) {
      status[i] = (uint8_t)st;
      out_len[i] = olen;
      dec_in_off[i] = snappy ? off : 0u;   // never an out-of-range address
      dec_len[i] = snappy ? (uint32_t)size : 0u;
      dec_off[i] = snappy ? oo : dummy_off;
      dec_cap[i] = snappy ? cap : 0u;
    }
  }
}

// The trailer checks of format.c:203-211 on their own (check_kernel then
// runs without them): bad[i] = 1 when block i's stored CRC does not match.
// Its 6.6 KB of tables let one workgroup sit on every CU beside the ring
// decoder's eight waves (151.5 of 160 KB of LDS), so it runs while the
// blocks decode (table_read).
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void verify_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint8_t* __restrict__ bad, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kSmallWords];
  load_tables<64 * WAVES, kSmallWords>(s_tab);
  const CrcSmall T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint64_t off = on ? hoff[i] : 0, size = on ? hsize[i] : 0;
    const bool body = on && size <= ~0ull - kTrailer && off <= file_len &&
                      file_len - off >= size + kTrailer && size <= 0x7fffffffull;  // as check_kernel
    const gptr<const uint8_t> data = to_global(file) + (body ? off : 0);
    const uint32_t sz = body ? (uint32_t)size : 0u;
    const uint32_t ty = body ? (uint32_t)data[sz] : 0u;
    const uint32_t c = half_crc(T, data, sz, 1u, ty, body);
    uint32_t b = 0;
    if (body) {
      const uint32_t stored = (uint32_t)data[sz + 1] | ((uint32_t)data[sz + 2] << 8) |
                              ((uint32_t)data[sz + 3] << 16) | ((uint32_t)data[sz + 4] << 24);
      b = crc_unmask(stored) != c;
    }
    if (on & (hl == 0)) bad[i] = (uint8_t)b;
  }
}

__global__ __launch_bounds__(256) void merge_kernel(uint8_t* __restrict__ status,
                                                    uint32_t* __restrict__ out_len,
                                                    const uint8_t* __restrict__ dec_status,
                                                    const uint32_t* __restrict__ dec_out_len,
                                                    const uint8_t* __restrict__ bad, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (bad && bad[i]) {            // format.c:203-211 before the type dispatch
    status[i] = kStBadCrc;
    out_len[i] = 0;
    return;
  }
  if (status[i] != kPending) return;
  status[i] = dec_status[i];      // LGS_ST_CORRUPT / OK / NOSPACE, format.c:237-252
  out_len[i] = dec_out_len[i];
}

// Grid for the one-wave-per-block framing kernels: every workgroup
// resident at once (CUs x the occupancy the kernel's LDS allows), each
// loading the tables once and striding over blocks -- no second, partial
// round of workgroups.
constexpr uint32_t kFrameWaves = 8;
uint32_t g_res_crc = 0, g_res_pack = 0, g_res_frame = 0, g_res_check = 0, g_res_check_plain = 0;
template <class K>
uint32_t frame_grid(K kernel, uint32_t n, uint32_t& resident) {   // resident: per kernel,
  if (resident == 0) {                                              // same on every device
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
  // (Two blocks per wave: half_crc.)
  const uint32_t want = (n + kBpw * kFrameWaves - 1) / (kBpw * kFrameWaves);
  return want < resident ? (want ? want : 1u) : resident;
}

}  // namespace

hipError_t launch_crc(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      const uint8_t* type, int masked, uint32_t* crc, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(crc_kernel<kFrameWaves>, dim3(frame_grid(crc_kernel<kFrameWaves>, n, g_res_crc)), dim3(64 * kFrameWaves),
                     0, s, in, in_off, in_len, type, (uint32_t)(masked != 0), crc, n);
  return hipGetLastError();
}

size_t scan_parts(uint32_t n) { return (n + kScanItems - 1) / kScanItems; }

__global__ __launch_bounds__(256) void fill_stride_kernel(uint64_t* __restrict__ off,
                                                          uint64_t stride, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) off[i] = (uint64_t)i * stride;
}

hipError_t launch_fill_stride(uint64_t* off, uint64_t stride, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_stride_kernel, dim3((n + 255) / 256), dim3(256), 0, s, off, stride, n);
  return hipGetLastError();
}

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
  hipLaunchKernelGGL(pack_kernel<kFrameWaves>, dim3(frame_grid(pack_kernel<kFrameWaves>, n, g_res_pack)),
                     dim3(64 * kFrameWaves), 0, s, src, src_off, len, dst, dst_off, n);
  return hipGetLastError();
}

hipError_t launch_frame(const FrameArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(frame_kernel<kFrameWaves>, dim3(frame_grid(frame_kernel<kFrameWaves>, a.n, g_res_frame)), dim3(64 * kFrameWaves), 0,
                     s, a.raw, a.raw_off, a.raw_len, a.enc, a.enc_off, a.enc_len, a.file, a.base,
                     a.foff, a.handle_off, a.handle_size, a.n);
  return hipGetLastError();
}

hipError_t launch_check(const CheckArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (a.verify) {
    hipLaunchKernelGGL((check_kernel<kFrameWaves, true>),
                       dim3(frame_grid(check_kernel<kFrameWaves, true>, a.n, g_res_check)),
                       dim3(64 * kFrameWaves), 0, s, a.file, a.file_len, a.hoff, a.hsize, a.verify,
                       a.out, a.out_off, a.out_cap, a.out_len, a.status, a.dec_in_off, a.dec_len,
                       a.dec_off, a.dec_cap, a.dummy_off, a.n);
  } else {
    hipLaunchKernelGGL((check_kernel<kFrameWaves, false>),
                       dim3(frame_grid(check_kernel<kFrameWaves, false>, a.n, g_res_check_plain)),
                       dim3(64 * kFrameWaves), 0, s, a.file, a.file_len, a.hoff, a.hsize, a.verify,
                       a.out, a.out_off, a.out_cap, a.out_len, a.status, a.dec_in_off, a.dec_len,
                       a.dec_off, a.dec_cap, a.dummy_off, a.n);
  }
  return hipGetLastError();
}

hipError_t launch_merge(uint8_t* status, uint32_t* out_len, const uint8_t* dec_status,
                        const uint32_t* dec_out_len, const uint8_t* bad, uint32_t n,
                        hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(merge_kernel, dim3((n + 255) / 256), dim3(256), 0, s, status, out_len,
                     dec_status, dec_out_len, bad, n);
  return hipGetLastError();
}

// One workgroup of 8 waves per CU: the verify pass keeps to the LDS the ring
// decoder leaves free.
constexpr uint32_t kVerifyWaves = 8;
hipError_t launch_verify(const uint8_t* file, uint64_t file_len, const uint64_t* hoff,
                         const uint64_t* hsize, uint8_t* bad, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  static uint32_t cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
              ? (uint32_t)c : 256u;
  }
  const uint32_t want = (n + kBpw * kVerifyWaves - 1) / (kBpw * kVerifyWaves);
  hipLaunchKernelGGL(verify_kernel<kVerifyWaves>, dim3(want < cus ? want : cus),
                     dim3(64 * kVerifyWaves), 0, s, file, file_len, hoff, hsize, bad, n);
  return hipGetLastError();
}

}  // namespace lgs
