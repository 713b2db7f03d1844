// lgs_decode_common.h -- device helpers shared by the gfx950 decoders
// (lgs_decode.hip, and the probe-only decoders of lgs_decode_probe.hip):
// 16-byte global and LDS accesses, byte-exact stores, the output flush of
// the wave decoders and the tag parse of snappy.c:210-324 with its rejects.
#pragma once

#include "lgs_device.h"

namespace lgs {

// Byte source over the stream in global memory (oversized blocks only).
// Window bytes at or past `len` read as zero and are never consumed.
struct GlobalStream {
  gptr<const uint8_t> base;
  uint32_t len;
  __device__ uint64_t win(uint32_t pos) const {
    uint64_t v = 0;
    for (uint32_t i = 0; i < 8; ++i)
      if (pos + i < len) v |= (uint64_t)base[pos + i] << (8 * i);
    return uni64(v);
  }
  __device__ uint8_t byte(uint32_t pos) const { return base[pos]; }
};

// Decode one stream held in global memory (blocks whose compressed length
// exceeds the LDS staging area) into `o` (LDS).  Returns 1 ok / 0 corrupt /
// 2 too big.
template <class Src>
__device__ uint32_t decode_stream(const Src& src, uint32_t slen, uint8_t* o,
                                  uint32_t cap, uint32_t* want_out) {
  const uint32_t lane = lane_id();

  // varint32 header, coding.h:169-204 (<= 5 bytes, continuation on the
  // fifth byte or running out of input is a failure).
  uint64_t w = src.win(0);
  uint32_t want = 0, pos = 0;
  bool hdr_ok = false;
  for (uint32_t i = 0; i < 5 && i < slen; ++i) {
    uint32_t b = (uint32_t)(w >> (8 * i)) & 0xffu;
    if ((b & 0x80u) == 0) {
      want |= b << (7 * i);
      pos = i + 1;
      hdr_ok = true;
      break;
    }
    want |= (b & 0x7fu) << (7 * i);
  }
  if (!hdr_ok || want > 0x7fffffffu) return 0;   // snappy.c:405-409
  if (want > cap) return 2;
  *want_out = want;

  uint32_t left = slen - pos;
  uint32_t made = 0;

  while (left > 0) {                                // snappy.c:208
    const uint64_t t = src.win(pos);
    const uint32_t tag = (uint32_t)t & 0xffu;
    const uint32_t kind = tag & 3u;

    if (kind == 0) {                                // literal, snappy.c:210-273
      uint32_t m = tag >> 2;
      uint32_t hl = 1;
      if (m >= 60) {
        const uint32_t extra = m - 59;              // 1..4 length bytes
        if (left - 1 < extra) return 0;
        const uint32_t hi = (uint32_t)(t >> 8);
        m = extra == 4 ? hi : (hi & ((1u << (8 * extra)) - 1u));
        hl += extra;
      }
      if (m >= 0x7fffffffu) return 0;               // snappy.c:258
      const uint32_t len = m + 1;
      pos += hl;
      left -= hl;
      if (len > want - made || len > left) return 0;  // snappy.c:263
      for (uint32_t j0 = 0; j0 < len; j0 += kWave) {
        const uint32_t j = j0 + lane;
        if (j < len) o[made + j] = src.byte(pos + j);
      }
      order();
      made += len;
      pos += len;
      left -= len;
      continue;
    }

    uint32_t len, dist, hl;
    if (kind == 1) {                                // COPY1, snappy.c:276-287
      if (left < 2) return 0;
      len = 4 + ((tag >> 2) & 7u);
      dist = ((tag & 0xe0u) << 3) | ((uint32_t)(t >> 8) & 0xffu);
      hl = 2;
    } else if (kind == 2) {                         // COPY2, snappy.c:289-301
      if (left < 3) return 0;
      len = 1 + (tag >> 2);
      dist = (uint32_t)(t >> 8) & 0xffffu;
      hl = 3;
    } else {                                        // COPY4, snappy.c:303-317
      if (left < 5) return 0;
      len = 1 + (tag >> 2);
      dist = (uint32_t)(t >> 8);
      hl = 5;
    }
    pos += hl;
    left -= hl;
    if (dist == 0 || dist >= 0x80000000u) return 0;   // snappy.c:320
    if (made < dist || len > want - made) return 0;   // snappy.c:323

    // len <= 64: one lane per output byte.  An overlapping copy (dist <
    // len) repeats the dist-byte pattern, which is what the reference's
    // forward byte loop (snappy.c:329-330) produces.
    if (lane < len) {
      const uint32_t from = made - dist + (dist >= len ? lane : lane % dist);
      const uint8_t v = o[from];
      o[made + lane] = v;
    }
    order();
    made += len;
  }

  return made == want ? 1u : 0u;                    // snappy.c:337
}

// Stream the decoded bytes lds[shift .. shift+len) to dst, where
// shift == dst & 15 (lds is the 16-byte aligned base of the output image):
// every full granule is one 16-byte store.
__device__ __forceinline__ void flush_out(gptr<uint8_t> dst, const uint8_t* o, uint32_t len) {  // o: LDS base
  const uint32_t shift = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  const gptr<uint8_t> g = dst - shift;
  const uint32_t end = shift + len;
  const uint32_t n16 = (end + 15u) >> 4;
  for (uint32_t c = lane_id(); c < n16; c += kWave) {
    const uint32_t lo = c << 4, hi = lo + 16;
    if (lo >= shift && hi <= end) {
      *(gptr<u32x4>)(g + lo) = *reinterpret_cast<const u32x4*>(o + lo);
    } else {
      for (uint32_t b = lo; b < hi; ++b)
        if (b >= shift && b < end) g[b] = o[b];
    }
  }
}

// ---------------------------------------------------------------------------
// Per-lane helpers of the ring decoder below (one lane decodes one block).
// Reads may touch 16 bytes past a block's input (see lgs_decode_batch_dev).
// (A kernel that moved every byte as a 16-byte global access of its own
// lane, straight HBM to HBM, ran C2 at 373 GiB/s: its texture addresser was
// 93 % busy and 3.4x the output bytes reached HBM.  Removed in round 2.)
// ---------------------------------------------------------------------------
typedef u32x4 u32x4_u __attribute__((aligned(1)));

__device__ __forceinline__ u32x4 ld16(gptr<const uint8_t> p) {
  return *(gptr<const u32x4_u>)p;
}
__device__ __forceinline__ void st16(gptr<uint8_t> p, u32x4 v) { *(gptr<u32x4_u>)p = v; }

__device__ __forceinline__ uint32_t pick(u32x4 v, uint32_t d) {   // v[d], d < 4
  const uint32_t lo = d == 0 ? v.x : v.y;
  const uint32_t hi = d == 2 ? v.z : v.w;
  return d < 2 ? lo : hi;
}

__device__ __forceinline__ uint32_t byte_of(u32x4 v, uint32_t j) {   // byte j < 16
  return (pick(v, j >> 2) >> (8 * (j & 3u))) & 0xffu;
}

// 8 bytes starting at p (>= 5 meaningful), via two aligned dword loads.
__device__ __forceinline__ uint64_t view8(gptr<const uint8_t> p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const gptr<const uint32_t> w = (gptr<const uint32_t>)(a & ~(uintptr_t)3);
  const uint64_t v = ((uint64_t)w[1] << 32) | w[0];
  return v >> ((a & 3u) * 8);
}

// Store the first `len` bytes of the 16-byte value v at p, byte-exact.
// The byte stores are inline asm: written as C++ they made the compiler's
// wait-count analysis put a vmcnt(0) at the head of the decode loop (paid on
// every tag, i.e. waiting for that tag's stores), although nothing a later
// instruction reads is in flight.  The trailing s_nop covers the VMEM-store
// data hazard, which the hazard recognizer cannot see through inline asm.
__device__ __forceinline__ void st_exact(gptr<uint8_t> p, u32x4 v, uint32_t len) {
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
  for (uint32_t b = 0; b < len; ++b) {
    const uint32_t byte = byte_of(v, b);
    asm volatile("global_store_byte %0, %1, off\n\ts_nop 1" ::"v"(p + b), "v"(byte)
                 : "memory");
  }
}

// One parsed tag (snappy.c:210-324) of a lane's stream.
struct Tag {
  uint32_t kind, len, hl, dist, next;
  bool bad;
};

__device__ __forceinline__ Tag parse_tag(u32x4 tv, uint32_t pos, uint32_t slen, uint32_t want,
                                         uint32_t made) {
  // Every field is computed for both kinds and selected: lanes of a wave
  // parse literals and copies together, so branches would run both sides
  // anyway and add the exec-mask bookkeeping.
  Tag t;
  const uint32_t tag = tv.x & 0xffu, kind = tag & 3u, m0 = tag >> 2;
  const uint32_t left = slen - pos;
  const uint32_t b1 = (tv.x >> 8) | (tv.y << 24);              // bytes 1..4
  const bool lit = kind == 0;
  // literal, snappy.c:210-256: m0 < 60, or m0 - 59 length bytes
  const uint32_t extra = m0 >= 60 ? m0 - 59 : 0u;
  const uint32_t emask = extra >= 4 ? 0xffffffffu : (1u << (8 * (extra & 3u))) - 1u;
  const uint32_t m = extra ? (b1 & emask) : m0;
  // copies, snappy.c:276-317
  const uint32_t clen = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;
  const uint32_t cdist = kind == 1 ? ((tag & 0xe0u) << 3) | (b1 & 0xffu)
                                   : (kind == 2 ? b1 & 0xffffu : b1);
  t.kind = kind;
  t.len = lit ? m + 1 : clen;
  t.hl = lit ? 1 + extra : (kind == 3 ? 5u : kind + 1);
  t.dist = lit ? 0u : cdist;
  // The rejects, folded: the tag's header must fit the stream (:240-256,
  // :276-317); len > want - made is :263 / :323's length bound; a literal
  // also needs m < 2^31 - 1 (:258) and its bytes in the stream (:263); a
  // copy needs 0 < dist <= made (:320, :323): dist - 1 >= made as unsigned
  // covers dist == 0 and dist >= 2^31 too, since made < 2^31.
  // (As lane masks, not a select of two bools: a select of bools goes
  // through a VGPR and back.)
  t.bad = (t.hl > left) | (t.len > want - made) |
          (lit & ((m >= 0x7fffffffu) | (t.hl + t.len > left))) | (!lit & (cdist - 1 >= made));
  t.next = pos + t.hl + (lit ? t.len : 0u);
  return t;
}

// LDS byte address of a __shared__ pointer (for inline-asm ds_* operands).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// One byte of global memory through an agent-scope load (not served from a
// possibly stale L1 line): the wide decoder's reads of output it flushed.
__device__ __forceinline__ uint8_t gl_byte(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint8_t)(v >> (8 * (a & 3u)));
}

typedef u32x4 u32x4_l1 __attribute__((aligned(1)));
__device__ __forceinline__ u32x4 lrd16(const uint8_t* p) { return *(const u32x4_l1*)p; }
__device__ __forceinline__ void lwr16(uint8_t* p, u32x4 v) { *(u32x4_l1*)p = v; }

}  // namespace lgs
