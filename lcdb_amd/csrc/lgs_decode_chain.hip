// lgs_decode_chain.hip -- wave-per-block Snappy decoder for the batches where
// latency, not throughput, is the bound: the drop-in's single blocks and
// other batches of a few blocks.  PROBE LIBRARY ONLY (-DLGS_PROBE_DECODERS):
// exact, but it loses -- 36 us for one 4 KiB block against the wave
// decoder's 28 (profiles/r4i_session.txt): a lone wave pays ~4 cycles an
// instruction whatever they depend on, and walking the chain then moving
// the bytes issues about as many instructions as doing both per tag.
//
// Semantics: lcdb src/util/snappy.c:386-412 and decode_blocks (:201-341),
// with every reject of :216-338 and :337.  The other decoders move each
// op's bytes as they reach its tag, so every tag of the serial chain waits
// for an LDS round trip (a lone wave: ~345 cycles a tag, 28 us for a 4 KiB
// block).  Here the chain and the byte moves are apart:
//   * walk: lanes parse the tag that would start at each of 64 stream
//     positions (its step and output length); the scalar chain then steps
//     through the window with two v_readlane per tag, recording tag k's
//     stream position and output offset in lane k of two VGPRs (one
//     compare, two selects; 64 tags a batch).  No LDS access and no check
//     on the chain;
//   * execute the batch: each lane parses its recorded tag again and checks
//     every reject (parse_tag: the stream-only ones and :263 / :323 against
//     its recorded output offset); any failure rejects the block before a
//     byte of the batch is written.  Literals are written by their own
//     lanes at once (a literal over 64 bytes by the whole wave); copies then
//     run in order, each one LDS read and one write by the wave.
// Writes never leave their op's bytes, so ops of one batch never clobber
// each other; a copy reads only bytes before its own output, all written by
// then.  A stream longer than the LDS staging area (never a valid 4 KiB
// block from lcdb) is decoded by decode_stream from global memory.
#ifndef LGS_PROBE_DECODERS
#error "lgs_decode_chain.hip is built into the probe library only (build.py build_probe)"
#endif
#include "lgs_device.h"
#include "lgs_decode_common.h"
#include "lgs_launch.h"

namespace lgs {
namespace chn {

typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
typedef uint16_t u16_u __attribute__((aligned(1)));

// The first n < 16 bytes of v at LDS p, as 8/4/2/1-byte pieces.
__device__ __forceinline__ void put_short(uint8_t* p, u32x4 v, uint32_t n) {
  uint32_t off = 0, a = v.x, b = v.y;
  if (n & 8) {
    *(u64_u*)p = ((uint64_t)b << 32) | a;
    a = v.z;
    b = v.w;
    off = 8;
  }
  if (n & 4) {
    *(u32_u*)(p + off) = a;
    a = b;
    off += 4;
  }
  if (n & 2) {
    *(u16_u*)(p + off) = (uint16_t)a;
    a >>= 16;
    off += 2;
  }
  if (n & 1) p[off] = (uint8_t)a;
}

// Decode the stream in[0 .. S) (LDS, zero padding after it) into o[0 ..
// want).  Returns 1 ok / 0 corrupt / 2 larger than cap.
__device__ uint32_t chain_decode(const uint8_t* in, uint32_t S, uint8_t* o, uint32_t cap,
                                 uint32_t* want_out) {
  const uint32_t lane = lane_id();
  // varint32 header, coding.h:169-204; snappy.c:405-409.
  const uint64_t h8 = uni64(lds_ld64(in, 0));
  uint32_t want = 0, hlen = 0;
  for (uint32_t k = 0; k < 5 && k < S; ++k) {
    const uint32_t b = (uint32_t)(h8 >> (8 * k)) & 0xffu;
    want |= (b & 0x7fu) << (7 * k);
    if ((b & 0x80u) == 0) {
      hlen = k + 1;
      break;
    }
  }
  if (hlen == 0 || want > 0x7fffffffu) return 0;
  if (want > cap) return 2;
  *want_out = want;

  uint32_t p = hlen, m = 0;                      // next tag, output it starts at
  while (p < S) {                                // snappy.c:208
    // ---- walk up to 64 tags
    uint32_t k = 0, recp = 0, recm = 0;
    do {
      const uint32_t w = p;
      const uint32_t q = w + lane;
      const uint64_t t8 = lds_ld64(in, q);
      const uint32_t tag = (uint32_t)t8 & 0xffu, kind = tag & 3u, m0 = tag >> 2;
      const bool lit = kind == 0;
      const uint32_t extra = (lit & (m0 >= 60)) ? m0 - 59 : 0u;
      const uint32_t b1 = (uint32_t)(t8 >> 8);
      const uint32_t emask = extra >= 4 ? 0xffffffffu : (1u << (8 * (extra & 3u))) - 1u;
      const uint32_t mval = extra ? (b1 & emask) : m0;
      const uint32_t len = lit ? mval + 1 : (kind == 1 ? 4 + (m0 & 7u) : m0 + 1);
      const uint32_t hl = lit ? 1 + extra : (kind == 3 ? 5u : kind + 1);
      // The step, clamped so that a tag running past the stream ends the walk
      // (its rejects are found when the batch executes).
      const uint64_t step = (uint64_t)hl + (lit ? (uint64_t)mval + 1 : 0u);
      const uint32_t left = S - q;
      const uint32_t stepv = step > left ? left + 1 : (uint32_t)step;
      do {
        const uint32_t d = p - w;
        const uint32_t sp = __builtin_amdgcn_readlane(stepv, d);
        const uint32_t ln = __builtin_amdgcn_readlane(len, d);
        const bool here = lane == k;
        recp = here ? p : recp;
        recm = here ? m : recm;
        p += sp;
        m += ln;
        ++k;
      } while ((k < 64) & (p - w < 64) & (p < S));
    } while ((k < 64) & (p < S));

    // ---- execute tags 0 .. k-1 (lane j: tag j)
    const bool has = lane < k;
    const uint64_t tv8 = lds_ld64(in, recp);
    const Tag tg = parse_tag(u32x4{(uint32_t)tv8, (uint32_t)(tv8 >> 32), 0u, 0u}, recp, S, want,
                             recm);
    if (ballot(has & tg.bad)) return 0;
    const bool lit = has & (tg.kind == 0);
    const uint32_t ls = recp + tg.hl, ln = tg.len;
    uint8_t* const dst = o + recm;
    // literals of <= 64 bytes, one lane each: 16-byte chunks, the last one
    // ending at the literal's end; under 16 bytes, 8/4/2/1-byte pieces
    const bool sl = lit & (ln <= 64);
    if (ballot(sl & (ln >= 16))) {
      if (sl & (ln >= 16)) {
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) {
          if (16 * c < ln) {
            const uint32_t off = 16 * c + 16 <= ln ? 16 * c : ln - 16;
            lwr16(dst + off, lrd16(in + ls + off));
          }
        }
      }
    }
    if (ballot(sl & (ln < 16))) {
      if (sl & (ln < 16)) put_short(dst, lrd16(in + ls), ln);
    }
    // longer literals by the whole wave
    for (uint64_t lm = ballot(lit & (ln > 64)); lm; lm &= lm - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(lm);
      const uint32_t jm = lane_val(recm, j), js = lane_val(ls, j), jl = lane_val(ln, j);
      for (uint32_t c = 16 * lane; c < jl; c += 16 * kWave) {
        const uint32_t off = c + 16 <= jl ? c : jl - 16;
        lwr16(o + jm + off, lrd16(in + js + off));
      }
    }
    order();
    // copies in stream order, each by the wave (snappy.c:320-331)
    for (uint64_t cm = ballot(has & (tg.kind != 0)); cm; cm &= cm - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(cm);
      const uint32_t jm = lane_val(recm, j), jl = lane_val(ln, j), jd = lane_val(tg.dist, j);
      if (jd >= jl) {
        if (jl >= 16) {
          if (16 * lane < jl) {
            const uint32_t off = 16 * lane + 16 <= jl ? 16 * lane : jl - 16;
            lwr16(o + jm + off, lrd16(o + jm - jd + off));
          }
        } else if (lane < jl) {
          const uint8_t b = o[jm - jd + lane];
          o[jm + lane] = b;
        }
      } else if (lane < jl) {
        // overlapping (dist < len): the dist bytes before it, repeated --
        // what the reference's forward byte loop (snappy.c:329-330) writes
        const uint8_t b = o[jm - jd + lane % jd];
        o[jm + lane] = b;
      }
      order();
    }
  }
  return m == want ? 1u : 0u;                    // snappy.c:337
}

}  // namespace chn

template <uint32_t OUT_CAP, uint32_t IN_CAP>
__global__ __launch_bounds__(64) void decode_chain_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n, const uint32_t* __restrict__ count) {
  __shared__ __attribute__((aligned(16))) uint8_t s_img[OUT_CAP + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_in[IN_CAP + 128];
  const uint32_t lane = lane_id();
  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  const uint32_t S = uni(in_len[i]);
  const gptr<uint8_t> dst = to_global(out) + uni64(out_off[i]);
  const uint32_t cap = uni(out_cap[i] < OUT_CAP ? out_cap[i] : OUT_CAP);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  uint8_t* const o = s_img + sh;                 // output byte k at o[k]

  uint32_t want = 0, st;
  if (S <= IN_CAP) {
    // stage the stream: 16-byte granules, zero past it (reads stay within
    // 15 bytes past the stream), plus 128 bytes of zero padding
    for (uint32_t c = lane; c < (S + 15) / 16 + 8; c += kWave) {
      u32x4 v = {0, 0, 0, 0};
      if (16 * c < S) {
        v = ld16(src + 16 * c);
        const uint32_t kk = S - 16 * c;
        if (kk < 16) {
#pragma unroll
          for (uint32_t d = 0; d < 4; ++d) {
            const uint32_t lo = 4 * d;
            v[d] &= kk <= lo ? 0u : (kk >= lo + 4 ? 0xffffffffu : (1u << (8 * (kk - lo))) - 1u);
          }
        }
      }
      lwr16(s_in + 16 * c, v);
    }
    order();
    st = S ? chn::chain_decode(s_in, S, o, cap, &want) : 0u;
  } else {
    st = decode_stream(GlobalStream{src, S}, S, o, cap, &want);
  }
  order();
  if (st == 1) flush_out(dst, s_img, want);
  if (lane == 0) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

// One wave per block; outputs up to the 16 KiB class.  The stream is staged
// whole when it is at most twice the class (every lcdb block; longer streams
// decode from global memory).
hipError_t launch_decode_chain(const DecodeArgs& a, uint32_t max_out, hipStream_t s) {
  if (max_out <= 4608) {
    hipLaunchKernelGGL((decode_chain_kernel<4608, 9216>), dim3(a.n), dim3(64), 0, s, a.in,
                       a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                       a.index, a.n, a.count);
  } else {
    hipLaunchKernelGGL((decode_chain_kernel<16896, 33792>), dim3(a.n), dim3(64), 0, s, a.in,
                       a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                       a.index, a.n, a.count);
  }
  return hipGetLastError();
}

}  // namespace lgs
