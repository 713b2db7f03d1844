// lgs_encode.hip -- batched Snappy block encoder for gfx950 (MI355X),
// byte-identical to lcdb's src/util/snappy.c:104-195 (encode_block) and
// snappy.c:364-384 (snappy_encode).
//
// One wave owns one work item (a whole block <= 64 KiB, or one 64 KiB chunk
// of a larger block).  The chunk is staged in LDS at address 0, the
// 2048-entry u16 hash table (snappy.c:25,107) right after it at a constant
// offset that the table's LDS instructions carry in their offset field.  The
// greedy parse is serial by definition; the wave makes each serial step
// cheap instead of parallel-but-different:
//
//  * search batches: the probe positions of snappy.c:138-143 depend only on
//    the probe's index k since the search started (skip = 32, += skip >> 5),
//    so lanes 2..63 take 62 probes at once; lanes 0-1 are the re-probe after
//    a copy (snappy.c:172-186: A at at-1, B at at with lcdb's 64-bit compare
//    of :182), off in a batch that does not follow a copy.  Each lane swaps
//    its position into its hash's u16 entry with one ds_mskor_rtn_b32; lanes
//    of one instruction that hit the same dword apply in lane order, so each
//    lane receives the entry the serial loop would read and the table ends as
//    the serial loop leaves it.  The first matching lane ends the search;
//    lanes after it store back what they received.  A lane receiving a later
//    position than its own would mean the order broke: the batch then undoes
//    its swaps and replays lane by lane (never seen on gfx950).
//  * one path per round: the loop is rotated so a batch is its only exit
//    test, and lane validity is recomputed per batch rather than carried
//    (a carried bool becomes a lane-mask phi merged with exec on every path).
//  * match extension (snappy.c:163-164): 64 byte compares per step, the
//    first mismatch found by ballot.  (Sizing copies shorter than 8 bytes
//    from an 8-byte candidate compare in the batch was measured 3 % slower:
//    the third dword read sits on every batch's critical path.)
//  * emission (snappy.c:53-102): each op is recorded in lane k of two VGPRs;
//    every 64 ops flush_ops writes the literals and copy tags lane-parallel,
//    a wave scan placing them, straight to the output slot.
#include "lgs_device.h"
#include "lgs_probe_hooks.h"
#include "lgs_launch.h"
#include "lgs_service.h"

namespace lgs {

__constant__ ProbeTable kProbe = ProbeTable();

// Output slot of one block as a raw buffer: byte offset = SGPR cursor +
// VGPR lane offset, so stores need no 64-bit address arithmetic, and the
// hardware range check (num_records = the encode bound) keeps every store
// inside the slot.
struct OutSlot {
  __amdgpu_buffer_rsrc_t r;
  __device__ void put(uint32_t soff, uint32_t voff, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, (int)voff, (int)soff, 0);
  }
  // 2, 4, 8 or 16 bytes at any byte offset (gfx950 buffer stores need no
  // alignment).
  __device__ void put2(uint32_t soff, uint32_t voff, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, r, (int)voff, (int)soff, 0);
  }
  __device__ void put4(uint32_t soff, uint32_t voff, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, 0);
  }
  __device__ void put8(uint32_t soff, uint32_t voff, uint32_t lo, uint32_t hi) const {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo, hi}, r, (int)voff, (int)soff, 0);
  }
  __device__ void put16(uint32_t soff, uint32_t voff, u32x4 v) const {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, (int)soff, 0);
  }
};

// Where encode_chunk reads its chunk.  LdsIn: the whole chunk staged in LDS
// (every class up to 16 KiB, and C2).  WinIn: the 64 KiB class's window, a
// W-byte LDS ring of the chunk with the chunk in HBM behind it, so four
// waves fit a CU instead of two.  lcdb's 2 048-entry table keeps candidates
// from anywhere in the chunk, but on fillseq only ~40 of a 64 KiB block's
// 26 600 probes find one more than 28 000 bytes back (tools/
// sim_candidate_age.py), so reads outside the ring take a slow path: a
// wave-uniform test, then global loads for the lanes that need them.
struct LdsIn {
  static constexpr bool kWin = false;
  const uint8_t* x;
  // (Aligned dwords + v_alignbyte: the same reads as unaligned ds_read_b64 /
  // b32 took C2 encode from 783 to 1 515 us, profiles/r3d_unaligned_lds_ab.txt.)
  __device__ uint64_t rd64(uint32_t p) const { return lds_ld64(x, p); }
  __device__ Raw64 raw64(uint32_t p) const { return lds_raw64(x, p); }
  __device__ Raw32 raw32(uint32_t p) const { return lds_raw32(x, p); }
  __device__ uint32_t byte(uint32_t p) const { return x[p]; }
  __device__ u32x4 lit128(uint32_t p) const { return lds_ld128(x, p); }
  __device__ uint32_t litbyte(uint32_t p) const { return x[p]; }
  __device__ bool oow(uint32_t, uint32_t) const { return false; }
  __device__ void ensure(uint32_t) {}
  __device__ uint64_t g64(uint32_t) const { return 0; }
  __device__ uint32_t g32(uint32_t) const { return 0; }
  __device__ uint32_t gbyte(uint32_t) const { return 0; }
};

template <uint32_t W>
struct WinIn {
  static constexpr bool kWin = true;
  uint8_t* ring;                 // W bytes + a 16-byte mirror of ring[0..15]
  gptr<const uint8_t> gal;       // the chunk's first byte's 16-byte granule
  uint32_t sh;                   // chunk start & 15: position p is u = p + sh
  uint32_t n;                    // chunk length
  uint32_t hu;                   // staged below u = hu (a multiple of 16); valid: u >= hu - W
  __device__ uint32_t ri(uint32_t p) const { return (p + sh) & (W - 1); }
  __device__ uint64_t rd64(uint32_t p) const { return lds_ld64(ring, ri(p)); }
  __device__ Raw64 raw64(uint32_t p) const { return lds_raw64(ring, ri(p)); }
  __device__ Raw32 raw32(uint32_t p) const { return lds_raw32(ring, ri(p)); }
  __device__ uint32_t byte(uint32_t p) const { return ring[ri(p)]; }
  // bytes p .. p+k-1 are not in the ring
  __device__ bool oow(uint32_t p, uint32_t k) const {
    const uint32_t u = p + sh;
    return (u + W < hu) | (u + k > hu);
  }
  // Global dword d (of the granule-aligned view), clamped to the chunk's last
  // dword: reads never leave the granules that hold the chunk's bytes.
  __device__ uint32_t gdw(uint32_t d) const {
    const uint32_t last = (n + sh - 1) >> 2;
    return *(gptr<const uint32_t>)(gal + 4 * (d < last ? d : last));
  }
  __device__ uint64_t g64(uint32_t p) const {
    const uint32_t u = p + sh, d = u >> 2, b = u & 3u;
    const uint32_t a = gdw(d), c = gdw(d + 1), e = gdw(d + 2);
    return ((uint64_t)__builtin_amdgcn_alignbyte(e, c, b) << 32) | __builtin_amdgcn_alignbyte(c, a, b);
  }
  __device__ uint32_t g32(uint32_t p) const {
    const uint32_t u = p + sh;
    return __builtin_amdgcn_alignbyte(gdw((u >> 2) + 1), gdw(u >> 2), u & 3u);
  }
  __device__ uint32_t gbyte(uint32_t p) const {
    const uint32_t u = p + sh;
    return (gdw(u >> 2) >> (8 * (u & 3u))) & 0xffu;
  }
  // Emission reads literals from HBM (a literal may start anywhere behind).
  __device__ u32x4 lit128(uint32_t p) const {
    const uint32_t u = p + sh, d = u >> 2, b = u & 3u;
    const uint32_t a0 = gdw(d), a1 = gdw(d + 1), a2 = gdw(d + 2), a3 = gdw(d + 3), a4 = gdw(d + 4);
    return u32x4{__builtin_amdgcn_alignbyte(a1, a0, b), __builtin_amdgcn_alignbyte(a2, a1, b),
                 __builtin_amdgcn_alignbyte(a3, a2, b), __builtin_amdgcn_alignbyte(a4, a3, b)};
  }
  __device__ uint32_t litbyte(uint32_t p) const { return gbyte(p); }
  // Stage 4 KiB more (16-byte granules, each lane four), waiting for them.
  __device__ void stage() {
    const uint32_t lane = lane_id(), gend = (n + sh + 15) >> 4;
    u32x4 v[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t g = (hu >> 4) + lane + 64 * j;
      v[j] = g < gend ? *(gptr<const u32x4>)(gal + 16 * g) : u32x4{0, 0, 0, 0};
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);                          // vmcnt(0)
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t r = (hu + 16 * (lane + 64 * j)) & (W - 1);
      *reinterpret_cast<u32x4*>(ring + r) = v[j];
      if (r < 16) *reinterpret_cast<u32x4*>(ring + W + r) = v[j];
    }
    order();
    hu += 4096;
  }
  // Positions below P staged (as far as the chunk goes).
  __device__ void ensure(uint32_t P) {
    const uint32_t want = (P < n ? P : n) + sh;
    while (hu < want) stage();
  }
};

// A literal's bytes [from, from + len) of the chunk to slot offset `to`,
// 16 bytes per lane and four pieces in flight (WinIn reads them from HBM:
// a byte per lane and load would wait a memory round trip per 64 bytes).
// The last < 16 bytes go out as exact 8/4/2/1-byte stores.
template <class IN>
__device__ __forceinline__ void copy_lit16(const OutSlot& o, uint32_t op, const IN& x,
                                           uint32_t to, uint32_t from, uint32_t len) {
  constexpr uint32_t kOff = 0x40000000u;            // dropped by the range check
  const uint32_t lane = lane_id();
  const uint32_t whole = len & ~15u;
#pragma clang loop unroll(disable)
  for (uint32_t t0 = 0; t0 < whole; t0 += 4096) {
    u32x4 v[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t t = t0 + 1024 * k + 16 * lane;
      v[k] = x.lit128(from + (t < whole ? t : 0u));
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t t = t0 + 1024 * k + 16 * lane;
      o.put16(op, t < whole ? to + t : kOff, v[k]);
    }
  }
  const uint32_t rem = len - whole;
  if (rem) {
    u32x4 v = x.lit128(from + whole);
    uint32_t at = to + whole;
    const bool l0 = lane == 0;
    o.put8(op, l0 && (rem & 8) ? at : kOff, v.x, v.y);
    if (rem & 8) v = u32x4{v.z, v.w, 0, 0};
    at += rem & 8;
    o.put4(op, l0 && (rem & 4) ? at : kOff, v.x);
    if (rem & 4) v.x = v.y;
    at += rem & 4;
    o.put2(op, l0 && (rem & 2) ? at : kOff, v.x);
    if (rem & 2) v.x >>= 16;
    at += rem & 2;
    o.put(op, l0 && (rem & 1) ? at : kOff, v.x);
  }
}

// snappy.c:53-73: literal of len >= 1 taken from lds[from ..], written at o:
// header (1-3 bytes) and bytes in one pass, lane j writing output byte j.
// Returns bytes written.
template <class IN>
__device__ __forceinline__ uint32_t emit_literal(const OutSlot& o, uint32_t op, const IN& in,
                                                 uint32_t from, uint32_t len) {
  const uint32_t lane = lane_id();
  const uint32_t m = len - 1;
  const uint32_t hl = m < 60 ? 1u : (m < 256 ? 2u : 3u);
  const uint32_t h0 = m < 60 ? (m << 2) : (m < 256 ? 0xf0u : 0xf4u);
  const uint32_t hdr = h0 | ((m & 0xffu) << 8) | ((m >> 8) << 16);   // little-endian header
  const uint32_t total = hl + len;
  if (IN::kWin || len > kWave) {
    if (lane < hl) o.put(op, lane, hdr >> (8 * lane));
    copy_lit16(o, op, in, hl, from, len);
    return total;
  }
#pragma clang loop unroll(disable) vectorize(disable)
  for (uint32_t j0 = 0; j0 < total; j0 += kWave) {
    const uint32_t j = j0 + lane;
    // Unconditional (clamped) LDS read, then a select: no branch around it.
    const uint32_t lb = in.litbyte(from + (j >= hl ? j - hl : 0));
    const uint32_t v = j < hl ? (hdr >> (8 * j)) : lb;
    if (j < total) o.put(op, j, v);
  }
  return total;
}

// snappy.c:75-102: 64-byte COPY2 pieces while len >= 68, a 60-byte COPY2 if
// then len > 64, then COPY2 (len >= 12 or dist >= 2048) or COPY1.  Lane b
// writes byte b of the emitted sequence.
__device__ __forceinline__ uint32_t emit_copy(const OutSlot& o, uint32_t op, uint32_t dist,
                                              uint32_t len) {
  const uint32_t lane = lane_id();
  const uint8_t lo = (uint8_t)(dist & 0xffu), hi = (uint8_t)((dist >> 8) & 0xffu);
  if (len < 68) {                                   // no 64-byte pieces (almost always)
    const uint32_t has60 = len > 64 ? 1u : 0u;
    const uint32_t rest = len - 60 * has60;
    const bool c1 = rest < 12 && dist < 2048;
    const uint32_t first = c1 ? (((dist >> 8) << 5) | ((rest - 4) << 2) | 1u)
                              : (((rest - 1) << 2) | 2u);
    // bytes: [0xee lo hi] (if has60), then first lo [hi]
    const uint32_t total = 3 * has60 + (c1 ? 2u : 3u);
    const uint32_t r = lane - 3 * has60;           // index inside the final piece
    const uint32_t v = lane < 3 * has60 ? (lane == 0 ? 0xeeu : (lane == 1 ? lo : hi))
                                        : (r == 0 ? first : (r == 1 ? lo : hi));
    if (lane < total) o.put(op, lane, v);
    return total;
  }
  const uint32_t n64 = (len - 68) / 64 + 1;
  uint32_t rest = len - 64 * n64;
  const uint32_t has60 = rest > 64 ? 1u : 0u;
  rest -= 60 * has60;
  const bool c1 = rest < 12 && dist < 2048;
  const uint32_t head = 3 * (n64 + has60);
  const uint32_t total = head + (c1 ? 2u : 3u);
  const uint8_t last0 = c1 ? (uint8_t)(((dist >> 8) << 5) | ((rest - 4) << 2) | 1u)
                           : (uint8_t)(((rest - 1) << 2) | 2u);
#pragma clang loop unroll(disable) vectorize(disable)
  for (uint32_t b0 = 0; b0 < total; b0 += kWave) {
    const uint32_t b = b0 + lane;
    if (b < total) {
      uint8_t v;
      if (b < head) {
        const uint32_t r = b % 3;
        const bool is60 = has60 && b >= 3 * n64;
        v = r == 0 ? (is60 ? (uint8_t)0xee : (uint8_t)0xfe) : (r == 1 ? lo : hi);
      } else {
        const uint32_t r = b - head;
        v = r == 0 ? last0 : (r == 1 ? lo : hi);
      }
      o.put(op, b, v);
    }
  }
  return total;
}

// The recorded ops of one chunk, emitted lane-parallel: lane k holds op k
// (recA = copy end << 16 | copy start, recB = the copy's source), each op
// being the literal from the previous op's end (lit0 for op 0) to its copy
// start, then the copy (snappy.c:156, :166).  Every lane sizes its op
// (snappy.c:53-102), a wave scan places it, then
//   1. literal bytes, each lane its own op's: 16 bytes per trip from LDS
//      with one unaligned 16-byte store, then the last < 16 bytes with
//      exact-size stores (byte stores, one per byte, measured 3 % slower in
//      encode time);
//   2. literals over kLongLit bytes: all lanes on one op at a time;
//   3. literal headers and copy tags; copies of 68+ bytes (several pieces,
//      rare) through emit_copy, one op at a time.
// Returns the output cursor after the k ops.
constexpr uint32_t kLongLit = 256;

// r = v in the lanes whose bit of the SGPR mask sel is set (one lane: the
// op's record slot).  A plain v_cndmask with the mask as its condition; in
// C++ the per-lane bit of an SGPR mask costs a shift and a compare.
__device__ __forceinline__ void rec_lane(uint32_t& r, uint32_t v, uint64_t sel) {
  asm("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(v), "s"(sel));
}
template <class IN>
__device__ __forceinline__ uint32_t flush_ops(const OutSlot& o, uint32_t op, const IN& x,
                                              uint32_t recA, uint32_t recB, uint32_t k,
                                              uint32_t lit0) {
  const uint32_t lane = lane_id();
  const bool live = lane < k;
  // (The copy's end is kept mod 2^16: it is 65 536 when a copy ends a 64 KiB
  // chunk; the length, at most 65 535, is exact mod 2^16.)
  const uint32_t base = recA & 0xffffu, clen = ((recA >> 16) - base) & 0xffffu, dist = base - recB;
  const uint32_t pend = (uint32_t)__shfl_up((int)(base + clen), 1);
  const uint32_t lit = lane == 0 ? lit0 : pend;
  const uint32_t LL = live ? base - lit : 0u;
  const uint32_t m = LL - 1;                                          // snappy.c:55-66
  const uint32_t hl_big = m < 256 ? 2u : 3u;
  const uint32_t hl = LL == 0 ? 0u : (m < 60 ? 1u : hl_big);
  const uint32_t h0_big = m < 256 ? 0xf0u : 0xf4u;
  const uint32_t h0 = m < 60 ? (m << 2) : h0_big;
  const uint32_t hdr = h0 | ((m & 0xffu) << 8) | ((m >> 8) << 16);
  const bool longc = live && clen >= 68;
  const uint32_t has60 = clen > 64 ? 3u : 0u;                         // snappy.c:84-89
  const uint32_t rest = clen - 20 * has60;
  const bool c1 = rest < 12 && dist < 2048;                           // snappy.c:91
  const uint32_t first = c1 ? (((dist >> 8) << 5) | ((rest - 4) << 2) | 1u)
                            : (((rest - 1) << 2) | 2u);
  uint32_t ntag = has60 + (c1 ? 2u : 3u);
  if (longc) {                                                        // snappy.c:80-89
    const uint32_t n64 = (clen - 68) / 64 + 1;
    uint32_t r = clen - 64 * n64;
    const uint32_t h60 = r > 64 ? 1u : 0u;
    r -= 60 * h60;
    ntag = 3 * (n64 + h60) + ((r < 12 && dist < 2048) ? 2u : 3u);
  }
  const uint32_t size = live ? hl + LL + ntag : 0u;
  uint32_t incl = size;
#pragma unroll
  for (uint32_t d = 1; d < kWave; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, d);
    incl += lane >= d ? t : 0u;
  }
  const uint32_t excl = incl - size;
  const uint32_t total = lane_val(incl, kWave - 1);
  const uint32_t lat = excl + hl;                                     // literal's first byte
  const uint32_t tat = lat + LL;                                      // copy's first tag byte
  constexpr uint32_t kOff = 0x40000000u;                              // dropped by the range check
  // 1. short literals, lane-parallel: whole 16-byte pieces, then the last
  //    < 16 bytes with one 8-, 4-, 2- and 1-byte store each (lanes that do
  //    not need one aim it past the slot), so no byte lands past a literal.
  const uint32_t LLs = LL > kLongLit ? 0u : LL;
  const uint32_t whole = LLs & ~15u;
#pragma clang loop unroll(disable)
  for (uint32_t t = 0; ballot(t < whole); t += 16) {
    const bool on = t < whole;
    o.put16(op, on ? lat + t : kOff, x.lit128(on ? lit + t : 0u));
  }
  {
    const uint32_t rem = LLs - whole;                 // 0..15
    u32x4 v = x.lit128(LLs ? lit + whole : 0u);
    uint32_t at = lat + whole;
    o.put8(op, (rem & 8) ? at : kOff, v.x, v.y);
    if (rem & 8) v = u32x4{v.z, v.w, 0, 0};
    at += rem & 8;
    o.put4(op, (rem & 4) ? at : kOff, v.x);
    if (rem & 4) v.x = v.y;
    at += rem & 4;
    o.put2(op, (rem & 2) ? at : kOff, v.x);
    if (rem & 2) v.x >>= 16;
    at += rem & 2;
    o.put(op, (rem & 1) ? at : kOff, v.x);
  }
  // 2. long literals, all lanes on one op at a time (rare).
  for (uint64_t big = ballot(LL > kLongLit); big; big &= big - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(big);
    const uint32_t from = lane_val(lit, l), len = lane_val(LL, l), to = lane_val(lat, l);
    copy_lit16(o, op, x, to, from, len);
  }
  // 3. headers and tags.
  o.put(op, hl > 0 ? excl : kOff, hdr);
  o.put(op, hl > 1 ? excl + 1 : kOff, hdr >> 8);
  o.put(op, hl > 2 ? excl + 2 : kOff, hdr >> 16);
  const bool shortc = live && !longc;
  const uint32_t fb = tat + has60;                                    // final piece
  o.put(op, shortc && has60 ? tat : kOff, 0xeeu);
  o.put(op, shortc && has60 ? tat + 1 : kOff, dist);
  o.put(op, shortc && has60 ? tat + 2 : kOff, dist >> 8);
  o.put(op, shortc ? fb : kOff, first);
  o.put(op, shortc ? fb + 1 : kOff, dist);
  o.put(op, shortc && !c1 ? fb + 2 : kOff, dist >> 8);
  for (uint64_t lc = ballot(longc); lc; lc &= lc - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(lc);
    emit_copy(o, op + lane_val(tat, l), lane_val(dist, l), lane_val(clen, l));
  }
  return op + total;
}

// snappy.c:138-143's probe schedule in closed form (skip += skip >> 5 from
// 32: steps of 1 to probe 32, 2 to 48, 3 to 59, 4 to 67); equal to
// kProbe.off[k] for k <= 67 (the table serves longer searches).
__host__ __device__ constexpr uint32_t probe_off(uint32_t k) {
  return k + (k > 32 ? k - 32 : 0u) + (k > 48 ? k - 48 : 0u) + (k > 59 ? k - 59 : 0u);
}
constexpr uint32_t kProbeClosed = 67;
constexpr bool probe_off_matches_table() {
  constexpr ProbeTable t;
  for (uint32_t k = 0; k <= kProbeClosed; ++k)
    if (probe_off(k) != t.off[k]) return false;
  return true;
}
static_assert(probe_off_matches_table(), "closed-form probe schedule != snappy.c:138-143");

// The table (2 048 u16 entries + a sink) sits at the start of the wave's
// LDS, the chunk image right after it (EncLds below).  Lanes that must not
// touch a real entry aim their table access at the sink dword instead of
// branching around it (keeps the batch free of exec-mask regions, whose
// save/branch/restore is scalar work).
constexpr uint32_t kSink = kTableCap;

// LDS address (32-bit, address space 3) of a __shared__ pointer.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// One LDS atomic on the table dword at byte offset a (the table itself at
// LDS offset TAB, folded into the instruction): mem = (mem & ~mask) | data,
// returning the old dword.  The lanes of one such instruction that hit the
// same dword are applied in ascending lane order, each seeing its
// predecessors' writes (measured on gfx950, tools/lds_atomic_probe.hip;
// encode_chunk verifies it per batch).
template <uint32_t TAB>
__device__ __forceinline__ uint32_t lds_mskor_rtn(uint32_t a, uint32_t mask, uint32_t data) {
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3 offset:%4\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(old) : "v"(a), "v"(mask), "v"(data), "i"(TAB) : "memory");
  return old;
}
// The same without the result (and without a wait: LDS operations of one
// wave execute in issue order).
template <uint32_t TAB>
__device__ __forceinline__ void lds_mskor(uint32_t a, uint32_t mask, uint32_t data) {
  asm volatile("ds_mskor_b32 %0, %1, %2 offset:%3" : : "v"(a), "v"(mask), "v"(data), "i"(TAB)
               : "memory");
}

// Per-lane constants of a batch.  Every batch has lanes 0 and 1 reserved
// for the re-probe that follows a copy (snappy.c:172-186): lane 0 is its A
// at at - 1, lane 1 its B at at; lanes l >= 2 are search probes k + l - 2 of
// the literal search (snappy.c:138-143), 62 per batch.  A chunk's first
// batch and a search's later batches leave lanes 0 and 1 off.  e0: offset of
// lane l's probe from the search start at + 1 in the batch after a copy; e1:
// offset of the probe after it (the bound check of snappy.c:143; A and B
// always pass it: the batch runs only while at < last); bm: 0xffffff in B's
// lane (its 64-bit compare, snappy.c:182), else 0.
struct PostLanes {
  uint32_t e0, e1, bm;
};
constexpr uint32_t kProbesPerBatch = kWave - 2;
__device__ __forceinline__ PostLanes post_lanes(uint32_t lane) {
  const uint32_t pk = lane >= 2 ? lane - 2 : 0;
  return PostLanes{lane == 0 ? 0xfffffffeu : (lane == 1 ? 0xffffffffu : probe_off(pk)),
                   lane < 2 ? 0u : probe_off(pk + 1), lane == 1 ? 0xffffffu : 0u};
}
// Offset of the last lane's probe in the first batch of a search (WinIn staging).
constexpr uint32_t kPostLast = probe_off(kProbesPerBatch - 1);

// Encode one chunk x[0..n), 17 <= n <= 65536, held in LDS.  `tab` is the
// u16 hash table (with a sink slot).  Writes to o, returns bytes written.
// Mirrors snappy.c:104-195 step for step.
//
// Literal-search batches.  Lane l takes the batch's probe l (lane 0 the
// earliest).  Each valid lane swaps its probe position into tab[hash] with
// one LDS atomic (lds_mskor_rtn on the entry's dword).  Because a wave's
// atomics on one address apply in lane order, every lane gets back exactly
// what snappy.c:146-148 would read at that probe -- the position of the
// batch's latest earlier probe with the same hash, else the entry as the
// batch found it -- and the table ends as the serial loop would leave it
// after all 64 probes.  Any number of probes may share a hash.  The first
// lane whose 4-byte compare matches ends the search; the probes after it
// must not have written, so in each slot they touched the first of them
// restores the value it received (its received value is a committed position
// or an old entry exactly when it is at most the match's position: positions
// grow with the lane, old entries lie before the batch).  A lane receiving a
// position later than its own would mean the order assumption broke; then
// the batch restores the table and replays the swaps one lane at a time.
//
// The re-probe after a copy (PostLanes) is two ordinary probes to the table
// swap, which gives the serial order's table semantics (B's candidate is
// at-1 when A and B share a hash); A never matches, and B's match is the
// re-match of snappy.c:182.  Folding the re-probe into the batch removes its
// three dependent LDS round trips from every copy.
//
// A found match is extended and recorded: lane k of recA/recB holds op k,
// and 64 ops at a time are emitted lane-parallel (flush_ops), a few VALU per
// op instead of one 64-lane pass.  (The per-op pass measured 176 against
// 213 GiB/s.)
//
// Round 4: the hot path is one loop with one exit -- batch, match,
// extension, record, the batch after the copy -- and a batch without a
// match leaves it, to the outer loop that places a search's later batches
// from the probe table.  The batch after the chunk's last copy runs with
// every lane off, so the end of the chunk is that same exit.  Every batch
// has the same lane layout, so B's mask and the lanes that may match need
// no per-batch state, and validity is computed per batch, not carried.
// Table addresses come straight from the hash (the image at LDS 0,
// the table at a constant offset folded into the instruction), and an op is
// recorded by a one-hot lane mask (rec_lane) instead of v_writelane
// through M0.
template <uint32_t TAB, class IN>
__device__ __forceinline__ uint32_t encode_chunk(IN& x, uint32_t n, uint16_t* tab,
                                                 const OutSlot& o, uint32_t op0,
                                                 const PostLanes& pl) {
  const uint32_t lane = lane_id();
  const uint32_t last = n - kMargin;                  // snappy.c:106

  uint32_t tsize = 256, shift = 24;                   // snappy.c:108-125
  while (tsize < kTableCap && tsize < n) {
    tsize <<= 1;
    --shift;
  }
  // snappy.c:129, 16 bytes (8 entries) per lane and store: tsize >= 256
  // entries is a whole number of 64-lane rows.
  for (uint32_t e = lane; e < tsize / 8; e += kWave)
    reinterpret_cast<u32x4*>(tab)[e] = u32x4{0, 0, 0, 0};
  order();
  // h2 = (x * kHashMul) >> (shift - 1) = 2 * hash32(x, shift) + one more bit:
  // the entry's dword is at TAB + (h2 & ~3) and its half of that dword is
  // (h2 & 2) << 3.  (TAB, the table's LDS offset, goes into the instruction.)
  const uint32_t hsh = shift - 1;
  constexpr uint32_t kSinkOff = 2 * kSink;            // the sink dword, from the table

  uint32_t op = op0;     // output cursor (byte offset in the slot)
  uint32_t at = 0;       // end of the last copy (snappy.c:167 "emit")
  uint32_t start = 1;    // first probe position of the current search (snappy.c:112)
  uint32_t kb = 0;       // the search's probe index in lane 2 of the batch
  uint32_t recA = 0, recB = 0, lit0 = 0;
  uint64_t sel = 1;      // one-hot: the lane that records the next op

  // The batch in flight: each lane's probe position, the lanes that are
  // probes (vmask), and the read of bytes p .. p+7 (issued when the batch
  // is placed, combined at first use).
  uint32_t p;
  uint64_t vmask = 0;
  Raw64 xr;
  // The batch's table state, kept for the copy that follows a match.
  uint32_t prev = 0, h2 = 0, ta = 0, sh = 0, mask = 0;
  // ---- one batch: snappy.c:146-152 for its 64 probes, `valid` the lanes
  // that are probes.  Returns the lanes that match.  (Validity is passed in,
  // not kept: a bool carried around the loop becomes a lane-mask phi merged
  // with exec on every path.)
  auto batch = [&](bool valid) -> uint64_t {
    vmask = ballot(valid);
    uint32_t xv = xr.lo(), xh = xr.hi();
    if constexpr (IN::kWin) {
      const bool o8 = valid & x.oow(p, 8);
      if (ballot(o8)) {
        const uint64_t g = x.g64(p);
        xv = o8 ? (uint32_t)g : xv;
        xh = o8 ? (uint32_t)(g >> 32) : xh;
      }
    }
    h2 = (xv * kHashMul) >> hsh;                                  // snappy.c:44-47
    ta = valid ? (h2 & ~3u) : kSinkOff;
    sh = (h2 << 3) & 16u;
    mask = 0xffffu << sh;
    const uint32_t old = lds_mskor_rtn<TAB>(ta, mask, p << sh);   // snappy.c:146-148
    prev = (old >> sh) & 0xffffu;
    Raw32 yr = x.raw32(prev);                                     // the candidate's bytes
    // (Checked under the read's latency; the rare path reads them again.)
    // (A probe build takes this path on every batch, lgs_probe_hooks.h.)
    if (LGS_ENC_REPLAY(prev > p, vmask)) {
      // Not in lane order (never seen on gfx950): put back each touched
      // slot's entry as the batch found it (the one lane per slot that
      // received a value from before the batch), then swap lane by lane.
      const uint32_t p0 = lane_val(p, (uint32_t)__builtin_ctzll(vmask));
      lds_mskor<TAB>(prev < p0 ? ta : kSinkOff, mask, prev << sh);
      for (uint64_t r = vmask; r; r &= r - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(r);
        const uint32_t got = lds_mskor_rtn<TAB>(lane == l ? ta : kSinkOff, mask, p << sh);
        prev = lane == l ? (got >> sh) & 0xffffu : prev;
      }
      yr = x.raw32(prev);
    }
    uint32_t yv = yr.value();
    if constexpr (IN::kWin) {
      const bool o4 = valid & x.oow(prev, 4);
      if (ballot(o4)) yv = o4 ? x.g32(prev) : yv;
    }
    // snappy.c:152; lane B: lcdb's 64-bit compare (snappy.c:182), bytes
    // at..at+6 against a zero-extended 4-byte load; A never matches.
    return ballot(((xv ^ yv) | (xh & pl.bm)) == 0) & vmask & ~1ull;
  };
  // A chunk's first batch: the post-copy layout from start = 1, A and B off.
  bool evalid = (lane >= 2) & (pl.e1 <= last - 1);
  p = evalid ? 1 + pl.e0 : 0;
  if constexpr (IN::kWin) x.ensure(1 + kPostLast + 16);
  xr = x.raw64(p);
  for (;;) {
    const uint32_t at_in = at;
    // Rotated: the batch is the loop's last step, so its match test is the
    // loop's only exit (a test in the middle became a selector variable).
    for (uint64_t mm = batch(evalid); mm;
         mm = batch((int32_t)(last - start) >= (int32_t)pl.e1)) {
      // ---- the copy (snappy.c:156-169)
      const uint32_t m = (uint32_t)__builtin_ctzll(mm);           // the matching probe
      const uint32_t base = lane_val(p, m);
      const uint32_t ref = lane_val(prev, m);
      // The probes after it did not happen: in each slot they touched, the
      // first of them puts back what it received.  A plain u16 store: the
      // lanes with nothing to put back all aim at the sink, and same-address
      // LDS atomics serialise where same-address stores do not (as an
      // ds_mskor this store took bank conflicts per launch from 1.0e8 to
      // 2.5e8, profiles/r4b_pmc_mskor_restore.txt).
      // (Lanes that are no probe have ta at the sink: their received value
      // is the sink's and must not reach a real entry.)
      *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(tab) +
                                   (((lane > m) & (prev <= base)) ? (ta | (h2 & 2u)) : kSinkOff)) =
          (uint16_t)prev;
      const uint32_t dist = base - ref;
      uint32_t at_n = base + 4;
#pragma clang loop unroll(disable)
      for (;;) {                                                  // snappy.c:163-164
        const uint32_t q = at_n + lane;
        if constexpr (IN::kWin) x.ensure(at_n + kWave);
        // Unconditional reads, unclamped: lanes at q >= n read at most 63
        // bytes past the chunk (the LDS image has that slack; the window
        // ring masks its index), and count as a mismatch.
        uint32_t bq = x.byte(q), br = x.byte(q - dist);
        if constexpr (IN::kWin) {
          const bool orq = x.oow(q - dist, 1) || x.oow(q, 1);
          if (ballot(orq)) {
            br = orq ? x.gbyte(q - dist) : br;
            bq = orq ? x.gbyte(q) : bq;
          }
        }
        const uint64_t diff = ballot(br != bq) | ballot(q >= n);
        if (diff) {
          at_n += (uint32_t)__builtin_ctzll(diff);
          break;
        }
        at_n += kWave;
      }
      // The batch after the copy (snappy.c:172-186 + the next search): its
      // read goes out now, under the op's bookkeeping.  Past the limit
      // (snappy.c:169) no lane of it is on, so it finds no match and ends the
      // chunk.
      start = at_n + 1;
      p = start + pl.e0;
      if constexpr (IN::kWin) x.ensure(start + kPostLast + 16);
      xr = x.raw64(p);
      // snappy.c:156 + 166: the literal before the copy (empty after a
      // re-match), then the copy -- recorded, emitted by flush_ops.
      at = at_n;
      rec_lane(recA, base | (at_n << 16), sel);
      rec_lane(recB, ref, sel);
      sel <<= 1;
      if (!sel) {                                                 // every 64 ops
        op = flush_ops(o, op, x, recA, recB, kWave, lit0);
        sel = 1;
        lit0 = at_n;
      }
    }
    if (at >= last) break;
    // No match in the batch: the search ends if a probe of the batch was
    // past the limit (snappy.c:143), else continues with its next 62 probes,
    // from the probe table.
    if ((vmask | 3ull) != ~0ull) break;
    kb = (at != at_in ? 0u : kb) + kProbesPerBatch;
    const uint32_t kk = kb + lane - 2;
    const bool in_tab = (lane >= 2) & (kk < kProbeTab);
    const uint32_t kc = in_tab ? kk : 0u;
    const uint32_t o0 = kProbe.off[kc], o1 = kProbe.off[kc + 1];
    // Wait for these two loads here, on the rare path.  Left to the
    // compiler, the wait lands where the paths merge as vmcnt(0) -- and
    // vmcnt also counts the output stores, so every batch would stall
    // until the previous copy's bytes had reached memory.
    __builtin_amdgcn_s_waitcnt(0x0f70);                           // vmcnt(0)
    evalid = in_tab & (o1 <= last - start);                       // snappy.c:143
    p = evalid ? start + o0 : 0;
    if constexpr (IN::kWin) x.ensure(start + lane_val(o0, kWave - 1) + 16);
    xr = x.raw64(p);
  }
  const uint32_t nops = (uint32_t)__builtin_ctzll(sel);
  if (nops) op = flush_ops(o, op, x, recA, recB, nops, lit0);

  if (at < n) op += emit_literal(o, op, x, at, n - at);           // snappy.c:190-192
  return op;
}

// varint32 header hv (coding.h:140-167) at the slot's start, unless hv is
// 0xffffffff (a later chunk of a > 64 KiB block).  Returns its length.
__device__ __forceinline__ uint32_t emit_header(const OutSlot& o, uint32_t hv) {
  if (hv == 0xffffffffu) return 0;
  const uint32_t lane = lane_id();
  const uint32_t hl = hv < (1u << 7) ? 1 : hv < (1u << 14) ? 2 : hv < (1u << 21) ? 3
                    : hv < (1u << 28) ? 4 : 5;
  if (lane < hl) {
    uint32_t b = (hv >> (7 * lane)) & 0x7fu;
    if (lane + 1 < hl) b |= 0x80u;
    o.put(0, lane, b);
  }
  return hl;
}

__device__ __forceinline__ OutSlot out_slot(uint8_t* out, uint64_t off, uint32_t len) {
  return OutSlot{__builtin_amdgcn_make_buffer_rsrc(out + off, 0, (int)(32 + len + len / 6),
                                                   0x00020000)};
}

// One wave's LDS: the chunk image at LDS 0 (its reads need no base: a
// ds_read2_b32 offset reaches only 1 KiB), then the hash table and its sink
// at the constant offset IMG, which the table's LDS atomics carry in their
// 16-bit offset field.  Each kernel declares this as its only __shared__
// object, so it is placed at LDS 0 (checked at the kernel's start).
template <uint32_t IMG>
struct EncLds {
  static_assert(IMG % 16 == 0 && IMG <= 65535 - 2 * kSink - 16, "table offset");
  uint8_t img[IMG];
  uint16_t tab[kTableCap + 8];                        // + the sink
};

// Work item i: input in[in_off[i] .. + in_len[i]), output at out + out_off[i].
// hdr == nullptr: item is a whole block, prefixed with its varint32 length
// (snappy.c:368).  Otherwise hdr[i] is the varint value to prefix, or
// 0xffffffff for none (a later chunk of a > 64 KiB block).  One wave per
// work item, one-wave workgroups (a static partition over persistent waves
// balances worse).
// One block (or a > 64 KiB block's chunks, one after the other) of `len`
// bytes at src, encoded into o with the varint header hv (0xffffffff: none).
// s: the wave's LDS (the kernel's only __shared__ object, at LDS 0).
template <uint32_t IN_CAP>
__device__ __forceinline__ uint32_t encode_item(EncLds<IN_CAP + 112>& s, gptr<const uint8_t> src,
                                                uint32_t len, uint32_t hv, const OutSlot& o) {
  // Image: + 48 the zero granule past it (and spare), + 64 the match
  // extension's reads past the chunk (encode_chunk).  8 832 B with the
  // table: 18 waves per CU (the 1 280-byte LDS granule).
  constexpr uint32_t kImg = IN_CAP + 112;
  const PostLanes pl = post_lanes(lane_id());
  LGS_ENC_PH_DECL;
  uint32_t op = emit_header(o, hv);

  // snappy.c:370-381: independent 64 KiB chunks, a short tail as a literal.
  // (IN_CAP >= min(len, 65536) is guaranteed by the launcher.)
  for (uint32_t c0 = 0; c0 < len; c0 += kChunk) {
    const uint32_t clen = len - c0 < kChunk ? len - c0 : kChunk;
    // Byte k of the chunk at img[k]: the image's dword reads are aligned
    // for any input alignment (unaligned LDS dword reads took C2 encode from
    // 0.78 to 1.5 ms, see LdsIn).
    constexpr uint32_t kR = (IN_CAP + 16 + 1023) / 1024 < 8 ? (IN_CAP + 16 + 1023) / 1024 : 8;
    stage_in_linear<kR>(s.img, src + c0, clen);
    LdsIn x{s.img};
    order();
    LGS_ENC_PH_STAGED();
    if (clen >= kMinBlock) {
      op = encode_chunk<kImg>(x, clen, s.tab, o, op, pl);
    } else {
      op += emit_literal(o, op, x, 0, clen);                    // snappy.c:379-380
    }
    order();
  }
  LGS_ENC_PH_END(o, len);
  return op;
}

// Work item i: input in[in_off[i] .. + in_len[i]), output at out + out_off[i].
// hdr == nullptr: item is a whole block, prefixed with its varint32 length
// (snappy.c:368).  Otherwise hdr[i] is the varint value to prefix, or
// 0xffffffff for none (a later chunk of a > 64 KiB block).  One wave per
// work item, one-wave workgroups (a static partition over persistent waves
// balances worse).
#ifndef LGS_ENCODE_SERVICE_ONLY
template <uint32_t IN_CAP>
__global__ __launch_bounds__(64) void encode_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
    const uint32_t* __restrict__ hdr, const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count, const Item1 one) {
  __shared__ __attribute__((aligned(16))) EncLds<IN_CAP + 112> s;
  if (lds_addr(&s) != 0) __builtin_trap();            // encode_chunk<kImg> assumes it

  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);

  uint64_t ioff, ooff;
  uint32_t len, hv;
  if (one.on) {                                     // the drop-in's item, by value
    ioff = one.in_off; ooff = one.out_off; len = one.in_len; hv = one.aux;
  } else {
    ioff = uni64(in_off[i]); ooff = uni64(out_off[i]); len = uni(in_len[i]);
    hv = uni(hdr ? hdr[i] : len);
  }
  const uint32_t op = encode_item<IN_CAP>(s, to_global(in) + ioff, len, hv, out_slot(out, ooff, len));
  if (lane_id() == 0) out_len[i] = op;
}

#endif  // !LGS_ENCODE_SERVICE_ONLY

// The batch kernels and the service kernel are compiled apart (build.py):
// the batch kernels with the max-ILP machine scheduler (C2 encode -1 %), the
// resident service wave without it (its latency, +1.8 us a call with it;
// DESIGN 4.1).  lgs_encode_service.hip includes this file for the latter.
#ifndef LGS_ENCODE_BATCH_ONLY
// The drop-in service's encode waves (lgs_launch.h): wave k serves mailbox
// k, one block of <= kSvcMaxItem bytes at a time, from its slot's arena.
__global__ __launch_bounds__(64) void encode_service_kernel(SvcMailbox* __restrict__ mb,
                                                            uint64_t idle,
                                                            SvcControl* __restrict__ ctl) {
  __shared__ __attribute__((aligned(16))) EncLds<kSvcMaxItem + 112> s;
  if (lds_addr(&s) != 0) __builtin_trap();
  svc_loop(mb + blockIdx.x, idle, ctl,
           [&](uint32_t len, uint64_t input, uint64_t arena, uint32_t* status, uint32_t* out_len) {
             uint8_t* a = reinterpret_cast<uint8_t*>(arena);
             len = len < kSvcMaxItem ? len : kSvcMaxItem;    // (the host never posts more)
             *out_len = encode_item<kSvcMaxItem>(s, to_global(reinterpret_cast<const uint8_t*>(input)),
                                                 len, len, out_slot(a, kSvcOut, len));
             *status = 1;
           });
}

hipError_t launch_encode_service(SvcMailbox* mb, uint32_t nslots, uint64_t idle,
                                 SvcControl* ctl, hipStream_t s) {
  hipLaunchKernelGGL(encode_service_kernel, dim3(nslots), dim3(64), 0, s, mb, idle, ctl);
  return hipGetLastError();
}
#endif  // !LGS_ENCODE_BATCH_ONLY

#ifndef LGS_ENCODE_SERVICE_ONLY
// The 64 KiB class with its chunk in a W-byte LDS ring (WinIn): 32 KiB +
// the table is 37 KB, four waves per CU (the whole-chunk image, 70 KB,
// fits two), so C3's 1 024 blocks of 64 KiB run as one generation.
template <uint32_t W>
__global__ __launch_bounds__(64) void encode_win_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
    const uint32_t* __restrict__ hdr, const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count) {
  __shared__ __attribute__((aligned(16))) EncLds<W + 16> s;    // ring + its 16-byte mirror
  if (lds_addr(&s) != 0) __builtin_trap();            // encode_chunk<W + 16> assumes it

  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);
  const uint32_t lane = lane_id();
  const PostLanes pl = post_lanes(lane);
  const uint32_t len = uni(in_len[i]);
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  const OutSlot o = out_slot(out, uni64(out_off[i]), len);
  uint32_t op = emit_header(o, uni(hdr ? hdr[i] : len));
  for (uint32_t c0 = 0; c0 < len; c0 += kChunk) {               // snappy.c:370-381
    const uint32_t clen = len - c0 < kChunk ? len - c0 : kChunk;
    const gptr<const uint8_t> g = src + c0;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
    WinIn<W> x{s.img, g - sh, sh, clen, 0};
    if (clen >= kMinBlock) {
      x.ensure(W / 4);
      op = encode_chunk<W + 16>(x, clen, s.tab, o, op, pl);
    } else {
      op += emit_literal(o, op, x, 0, clen);                    // snappy.c:379-380
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);   // the chunk's emission reads, before the ring is reused
    order();
  }
  if (lane == 0) out_len[i] = op;
}

// The 64 KiB class (and longer blocks, chunk by chunk).
static hipError_t launch_encode_big(const EncodeArgs& a, hipStream_t s);

template <uint32_t IN_CAP>
static hipError_t launch_encode_cls(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((encode_kernel<IN_CAP>), dim3(a.n), dim3(64), 0, s, a.in,
                     a.in_off, a.in_len, a.out, a.out_off, a.out_len, a.hdr, a.index, a.n,
                     a.count, a.one);
  return hipGetLastError();
}

constexpr uint32_t kEncCap0 = 4608;

// The <= 4 608-byte class.  (Two blocks per wave in lockstep, half a wave
// each, was byte-exact and slower: 1.83 against 1.21 ms on C2 -- see
// DESIGN.md 4.1.)
static hipError_t launch_encode_small(const EncodeArgs& a, hipStream_t s) {
  // (Persistent waves that prefetch the next block into registers while
  // parsing one were byte-exact and 15 % slower, 1 286 against 1 118 us on
  // C2: a wave's wait for its next block also drains its previous block's
  // output stores (vmcnt counts both), and a static partition of blocks over
  // waves balances worse than dispatching one-wave workgroups.)
  return launch_encode_cls<kEncCap0>(a, s);
}
constexpr uint32_t kEncCap1 = 16896;

static hipError_t launch_encode_big(const EncodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((encode_win_kernel<32768>), dim3(a.n), dim3(64), 0, s, a.in, a.in_off,
                     a.in_len, a.out, a.out_off, a.out_len, a.hdr, a.index, a.n, a.count);
  return hipGetLastError();
}

// max_in: largest item length in the launch (<= 65536).
// Blocks longer than 64 KiB are encoded chunk by chunk by their wave.
hipError_t launch_encode(const EncodeArgs& a, uint32_t max_in, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  // A by-value item stands for item 0 of a one-item launch; with more items
  // or an index list every slot would encode item 0.
  if (a.one.on && (a.n != 1 || a.index)) return hipErrorInvalidValue;
  if (max_in <= kEncCap0) return launch_encode_small(a, s);
  if (a.index || a.n < kSplitMinBlocks || !options().split) {
    if (max_in <= kEncCap1) return launch_encode_cls<kEncCap1>(a, s);
    return launch_encode_big(a, s);
  }
  // A mixed-size batch: each size class in its own kernel (see
  // launch_decode_split), so small blocks keep their small LDS images.
  const size_t list_bytes = (size_t)3 * a.n * sizeof(uint32_t);
  Scratch scratch(list_bytes + 16, s);
  hipError_t e = scratch.status();
  if (e != hipSuccess) return e;
  uint32_t* list = (uint32_t*)scratch.get();
  uint32_t* cnt = (uint32_t*)((uint8_t*)scratch.get() + list_bytes);
  EncodeArgs c = a;
  if ((e = hipMemsetAsync(cnt, 0, 16, s)) != hipSuccess ||
      (e = launch_classify(a.in_len, a.n, kEncCap0, kEncCap1, 0xffffffffu, list, cnt, s)) !=
          hipSuccess)
    return e;
  c.index = list; c.count = cnt;
  if ((e = launch_encode_small(c, s)) != hipSuccess) return e;
  c.index = list + a.n; c.count = cnt + 1;
  if ((e = launch_encode_cls<kEncCap1>(c, s)) != hipSuccess) return e;
  c.index = list + 2 * (size_t)a.n; c.count = cnt + 2;
  if (max_in > kEncCap1 && (e = launch_encode_big(c, s)) != hipSuccess) return e;
  return scratch.release();
}
#endif  // !LGS_ENCODE_SERVICE_ONLY

}  // namespace lgs
