// lgs_device.h -- device-side helpers shared by the gfx950 Snappy kernels.
//
// Format constants and arithmetic follow lcdb's src/util/snappy.c (file:line
// cited per item).  Everything here is wave64 code: "uniform" values live in
// SGPRs (v_readfirstlane) so control flow is scalar, and lane-parallel byte
// work uses the 64 lanes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lgs {

constexpr uint32_t kWave = 64;
constexpr uint32_t kTableCap = 2048;      // MAX_TABLE_SIZE, snappy.c:25
constexpr uint32_t kMargin = 15;          // INPUT_MARGIN, snappy.c:26
constexpr uint32_t kMinBlock = 17;        // MIN_BLOCK_SIZE, snappy.c:27
constexpr uint32_t kChunk = 65536;        // MAX_BLOCK_SIZE, snappy.c:28
constexpr uint32_t kHashMul = 0x1e35a7bdu;  // snappy.c:46

// Probe schedule of the literal search (snappy.c:138-143): probe k sits at
// start + kProbeOff[k]; skip starts at 32 and grows by skip >> 5 after each
// probe.  The schedule depends only on k, so a wave can place 64 probes at
// once.  384 entries cover a 64 KiB chunk (the offset passes 65536 near k=250).
constexpr int kProbeTab = 384;
struct ProbeTable {
  uint32_t off[kProbeTab + 1];
  constexpr ProbeTable() : off() {
    uint32_t skip = 32, at = 0;
    for (int k = 0; k <= kProbeTab; ++k) {
      off[k] = at;
      at += skip >> 5;
      skip += skip >> 5;
    }
  }
};

// Global-memory pointers.  Offsets added to a kernel-argument pointer after a
// v_readfirstlane keep hipcc's address-space inference; casting through an
// integer does not, and flat_* accesses also count on lgkmcnt (so every LDS
// wait would wait for them too).  Everything that touches HBM goes through
// these types.
template <class T>
using gptr = __attribute__((address_space(1))) T*;

// 16-byte vector (a plain clang vector: HIP's uint4 struct has no
// address-space-qualified assignment).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ gptr<T> to_global(T* p) {
  return (gptr<T>)p;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Moves a wave-uniform value into a VGPR and hides that it is uniform, so
// arithmetic on the result is issued on the VALU.  A CU has one scalar unit
// for its four SIMDs but twice the scalar unit's instruction rate in VALU
// issue, and the encoder's per-copy bookkeeping otherwise lands on the SALU.
__device__ __forceinline__ uint32_t vec(uint32_t v) {
  asm("" : "+v"(v));
  return v;
}

// Wave ballot as a plain compare into an SGPR pair (HIP's __ballot adds a
// v_cndmask/v_cmp round trip).
__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

// Value of v in lane l (l wave-uniform): v_readlane, no LDS round trip.
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t l) {
  return __builtin_amdgcn_readlane(v, l);
}

// snappy.c:44-47 (argument truncated to 32 bits at every call site).
__device__ __forceinline__ uint32_t hash32(uint32_t v, uint32_t shift) {
  return (v * kHashMul) >> shift;
}

// Compiler-only barrier: LDS accesses of one wave execute in issue order in
// hardware; this stops hipcc from reordering a lane's LDS load above another
// lane's earlier LDS store that it cannot see it depends on.
__device__ __forceinline__ void order() { asm volatile("" ::: "memory"); }

// Unaligned little-endian 32-bit load from a 4-byte-aligned LDS base: two
// aligned dwords + v_alignbyte (coding.h:33-40 semantics).
__device__ __forceinline__ uint32_t lds_ld32(const uint8_t* base, uint32_t at) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (at & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], at & 3u);
}

// 8 bytes starting at `at` (bytes at..at+7).
__device__ __forceinline__ uint64_t lds_ld64(const uint8_t* base, uint32_t at) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (at & ~3u));
  uint32_t a = w[0], b = w[1], c = w[2];
  uint32_t s = at & 3u;
  uint32_t lo = __builtin_amdgcn_alignbyte(b, a, s);
  uint32_t hi = __builtin_amdgcn_alignbyte(c, b, s);
  return ((uint64_t)hi << 32) | lo;
}

// lds_ld64 in two halves: the three dword reads now, the combine at first
// use (so the reads' latency can pass under other work in between).  `s` is
// the unmasked byte address: v_alignbyte_b32 reads only its low two bits.
struct Raw64 {
  uint32_t a, b, c, s;
  __device__ uint32_t lo() const { return __builtin_amdgcn_alignbyte(b, a, s); }
  __device__ uint32_t hi() const { return __builtin_amdgcn_alignbyte(c, b, s); }
  __device__ uint64_t value() const { return ((uint64_t)hi() << 32) | lo(); }
};
__device__ __forceinline__ Raw64 lds_raw64(const uint8_t* base, uint32_t at) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (at & ~3u));
  return Raw64{w[0], w[1], w[2], at};
}
// The same for lds_ld32: two dword reads now, the combine at first use.
struct Raw32 {
  uint32_t a, b, s;
  __device__ uint32_t value() const { return __builtin_amdgcn_alignbyte(b, a, s); }
};
__device__ __forceinline__ Raw32 lds_raw32(const uint8_t* base, uint32_t at) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (at & ~3u));
  return Raw32{w[0], w[1], at};
}

// 16 bytes starting at `at` (bytes at..at+15): five aligned dwords.
__device__ __forceinline__ u32x4 lds_ld128(const uint8_t* base, uint32_t at) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (at & ~3u));
  const uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
  const uint32_t s = at & 3u;
  return u32x4{__builtin_amdgcn_alignbyte(b, a, s), __builtin_amdgcn_alignbyte(c, b, s),
               __builtin_amdgcn_alignbyte(d, c, s), __builtin_amdgcn_alignbyte(e, d, s)};
}

// Copy `len` bytes global->LDS with byte k of the source at lds[k] (lds
// 16-byte aligned), so dword reads of the image are aligned whatever the
// source's alignment.  The global reads are 16 bytes per lane at any byte
// address, all inside [src, src + len): a ragged last granule is read as
// the 16 bytes that end at src + len and shifted into place (a block that
// ends flush with the end of a page or allocation must not fault), and a
// block under 16 bytes is read a byte per lane.  The image's bytes past len
// in its last granule are zero, and one zero granule is written past it.
// Up to R loads per lane are in flight before the first LDS write, so a
// 4 KiB block (257 granules, R = 5) costs one memory round trip, not one
// per 1 KiB.
template <uint32_t R>
__device__ __forceinline__ void stage_in_linear(uint8_t* lds, gptr<const uint8_t> src,
                                                uint32_t len) {
  typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
  u32x4* l = reinterpret_cast<u32x4*>(lds);
  const uint32_t n16 = (len + 15u) >> 4, lane = lane_id();
#ifdef LGS_PROBE_OLD_STAGE
  // Probe build: round 3's staging (reads up to 15 bytes past the block).
  for (uint32_t c0 = 0; c0 < n16; c0 += R * kWave) {
    u32x4 v[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      v[k] = *(gptr<const u32x4_a1>)(src + 16 * (c < n16 ? c : 0u));
    }
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      if (c < n16) l[c] = v[k];
    }
  }
  if (lane == 0) l[n16] = u32x4{0, 0, 0, 0};
  return;
#endif
  if (len < 16) {                                   // one ragged granule, no full one
    if (lane < 16) lds[lane] = lane < len ? src[lane] : (uint8_t)0;
    if (lane == 0) l[1] = u32x4{0, 0, 0, 0};
    return;
  }
  // The whole granules, then (d != 0) the ragged last one, nfull, read as
  // the 16 bytes that end at src + len by lane 0, its load issued first.
  const uint32_t nfull = len >> 4, d = (16u - (len & 15u)) & 15u;
  u32x4 tail = u32x4{0, 0, 0, 0};
  if ((d != 0) & (lane == 0)) tail = *(gptr<const u32x4_a1>)(src + (len - 16));
#pragma clang loop unroll(disable)
  for (uint32_t c0 = 0; c0 < nfull; c0 += R * kWave) {
    u32x4 v[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      v[k] = *(gptr<const u32x4_a1>)(src + 16 * (c < nfull ? c : 0u));
    }
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      if (c < nfull) l[c] = v[k];
    }
  }
  if ((d != 0) & (lane == 0)) {
    // Shift it down by d bytes, zeros in: word i of the granule is bytes
    // 4i + d .. 4i + d + 3 of the loaded 16.
    const uint32_t w[8] = {tail.x, tail.y, tail.z, tail.w, 0, 0, 0, 0};
    const uint32_t q = d >> 2, r = d & 3u;
    uint32_t o[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t lo = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
      const uint32_t hi = q == 0 ? w[i + 1] : q == 1 ? w[i + 2] : q == 2 ? w[i + 3] : w[i + 4];
      o[i] = __builtin_amdgcn_alignbyte(hi, lo, r);
    }
    l[nfull] = u32x4{o[0], o[1], o[2], o[3]};
  }
  if (lane == 0) l[n16] = u32x4{0, 0, 0, 0};
}

// Copy `len` bytes global->LDS: the LDS image keeps the source's alignment
// mod 16 (byte k of the source lands at lds[(src & 15) + k]) so that every
// lane moves one aligned 16-byte granule.  Returns the LDS shift (src & 15).
// Reads may touch the aligned 16-byte granules that contain the first and
// last byte, never a different page.  Up to R granules per lane are in
// flight before the first LDS write (one memory round trip per R KiB).
template <uint32_t R = 1>
__device__ __forceinline__ uint32_t stage_in(uint8_t* lds, gptr<const uint8_t> src, uint32_t len) {
  const uint32_t shift = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15u);
  gptr<const u32x4> g = (gptr<const u32x4>)(src - shift);
  u32x4* l = reinterpret_cast<u32x4*>(lds);
  const uint32_t n16 = (shift + len + 15u) >> 4, lane = lane_id();
#pragma clang loop unroll(disable)
  for (uint32_t c0 = 0; c0 < n16; c0 += R * kWave) {
    u32x4 v[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      v[k] = g[c < n16 ? c : 0u];
    }
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t c = c0 + k * kWave + lane;
      if (c < n16) l[c] = v[k];
    }
  }
  // Zero pad one granule past the end so fixed-width window reads are defined.
  if (lane == 0) l[n16] = u32x4{0, 0, 0, 0};
  return shift;
}

}  // namespace lgs
