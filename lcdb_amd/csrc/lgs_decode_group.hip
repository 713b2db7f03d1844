// lgs_decode_group.hip -- workgroup-per-block Snappy decoder for gfx950
// (MI355X), PROBE LIBRARY ONLY (-DLGS_PROBE_DECODERS; tests/test_gpu_probe_
// decoders.py).  Built for the batches where the lane- and wave-per-block
// decoders leave the chip idle (single blocks, the 64 KiB class); exact, but
// it loses: pointer jumping moves every stream position and output byte
// through LDS ~15 times, and the CU's LDS is the bound -- 32 us for one
// 4 KiB block against the wave decoder's 28, C3 fillseq 64 KiB 44 against
// 144 GiB/s (profiles/r4h_session.txt).
//
// Semantics: lcdb src/util/snappy.c:386-412 and decode_blocks (:201-341);
// every reject of :216-338 and :337, so the per-block accept/reject bit and
// the output bytes equal the reference's.  The serial tag walk is replaced
// by data-parallel steps over a window of the stream:
//
//  1. stage: IN_WIN stream bytes (+ lookahead) into LDS, one 16-byte load
//     per thread;
//  2. parse: at every window position the tag that would start there
//     (parse_tag: its step and the rejects that depend only on the stream);
//     J0[r] = the next tag's window position, or TERM when the step leaves
//     the window or the tag is bad;
//  3. mark: tag starts = the positions reachable from the window's first tag.
//     Round k marks J^(2^k)(r) from every marked r, then doubles J
//     (double-buffered, so each round jumps exactly 2^k tags); after round k
//     tags 0 .. 2^(k+1)-1 of the chain are marked, and the rounds stop when
//     the first tag's jump leaves the window (ceil(log2(tags)) rounds);
//  4. ops: a scan of the marked tags' lengths gives each op's output offset;
//     each op is checked against the output-dependent rejects (:263, :323);
//  5. fill: literal bytes into the LDS image of the block's output; each
//     copied byte's source (output position - dist) into R;
//  6. resolve: R[o] <- R[R[o]] until every copied byte points at a literal
//     byte or at output of an earlier window (ceil(log2(copy chain depth))
//     rounds); then one gather;
//  7. flush whole 16-byte granules of the finished output to HBM.
// A window's output is bounded by OUT_WIN (R's size): a window whose tags
// produce more is cut after the last op that fits, and the next window
// starts at the next tag (a single literal longer than OUT_WIN is copied
// alone).  Windows follow each other until the stream ends.
#ifndef LGS_PROBE_DECODERS
#error "lgs_decode_group.hip is built into the probe library only (build.py build_probe)"
#endif
#include "lgs_device.h"
#include "lgs_decode_common.h"
#include "lgs_launch.h"

namespace lgs {
namespace grp {

constexpr uint16_t kTerm = 0xffffu;
// ctl[] words
constexpr uint32_t kBad = 0, kNext = 1, kCut = 2;

template <uint32_t OUT_CAP, uint32_t IN_WIN, uint32_t OUT_WIN, uint32_t NT>
struct Lds {
  static_assert(IN_WIN % NT == 0 && OUT_WIN % NT == 0 && NT % 64 == 0, "shape");
  static_assert(IN_WIN <= 32768 && OUT_WIN <= 65536, "16-bit window positions");
  static constexpr uint32_t kSw = IN_WIN + 96;   // window + lookahead (literal bytes)
  static constexpr uint32_t kOps = IN_WIN / 2 + 4;   // a tag takes >= 2 stream bytes
  static constexpr uint32_t kImg = (OUT_CAP + 32 + 15) & ~15u;
  uint8_t img[kImg];         // output byte o of the block at img[sh + o], sh = dst & 15
  uint8_t sw[kSw];           // stream bytes ws .. ws + kSw (zero past the stream)
  uint16_t J[2][IN_WIN];     // jump pointers (window positions), double-buffered
  uint8_t M[IN_WIN];         // 1: a tag of the chain starts here
  uint32_t oo[kOps];         // op k's output offset in the window; oo[nops] = the total
  uint32_t os[kOps];         // literal: stream position of its first byte; copy: dist
  uint16_t opos[kOps];       // window position of op k's tag | 0x8000 for a literal
  uint32_t R[OUT_WIN];       // source (block output position) of the window's byte o
  uint32_t cov[NT];          // op covering each thread's first output byte
  uint32_t red[2][NT / 64];  // per-wave partials of the block scans
  uint32_t ctl[4];
};

// The 8 bytes at LDS byte offset `at` (any alignment) of a 4-aligned base.
__device__ __forceinline__ u32x4 tag_bytes(const uint8_t* base, uint32_t at) {
  const uint64_t v = lds_ld64(base, at);
  return u32x4{(uint32_t)v, (uint32_t)(v >> 32), 0u, 0u};
}

// Exclusive block-wide scan of (a, b) pairs; totals in *ta, *tb.  Ends with a
// barrier, so red[] is free again when it returns.
template <uint32_t NT>
__device__ __forceinline__ void scan2(uint32_t a, uint32_t b, uint32_t (*red)[NT / 64],
                                      uint32_t* ea, uint32_t* eb, uint32_t* ta, uint32_t* tb) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t x = a, y = b;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t px = __shfl_up(x, d), py = __shfl_up(y, d);
    if (lane >= d) { x += px; y += py; }
  }
  if (lane == 63) { red[0][w] = x; red[1][w] = y; }
  __syncthreads();
  uint32_t ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
  for (uint32_t k = 0; k < NT / 64; ++k) {
    const uint32_t ra = red[0][k], rb = red[1][k];
    ba += k < w ? ra : 0u;
    bb += k < w ? rb : 0u;
    sa += ra;
    sb += rb;
  }
  *ea = ba + x - a;
  *eb = bb + y - b;
  *ta = sa;
  *tb = sb;
  __syncthreads();
}

// Inclusive block-wide max-scan.
template <uint32_t NT>
__device__ __forceinline__ uint32_t scan_max(uint32_t v, uint32_t (*red)[NT / 64]) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t px = __shfl_up(x, d);
    if (lane >= d) x = px > x ? px : x;
  }
  if (lane == 63) red[0][w] = x;
  __syncthreads();
  uint32_t b = 0;
#pragma unroll
  for (uint32_t k = 0; k < NT / 64; ++k) {
    const uint32_t r = red[0][k];
    b = ((k < w) & (r > b)) ? r : b;
  }
  __syncthreads();
  return x > b ? x : b;
}

}  // namespace grp

template <uint32_t OUT_CAP, uint32_t IN_WIN, uint32_t OUT_WIN, uint32_t NT>
__global__ __launch_bounds__(NT) void decode_group_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n, const uint32_t* __restrict__ count) {
  using namespace grp;
  using L = Lds<OUT_CAP, IN_WIN, OUT_WIN, NT>;
  constexpr uint32_t P = IN_WIN / NT;       // window positions per thread
  constexpr uint32_t C = OUT_WIN / NT;      // window output bytes per thread
  __shared__ __attribute__((aligned(16))) L s;

  const uint32_t t = threadIdx.x;
  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;            // the whole workgroup
  const uint32_t i = uni(index ? index[slot] : slot);
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  const uint32_t S = uni(in_len[i]);
  const gptr<uint8_t> dst = to_global(out) + uni64(out_off[i]);
  const uint32_t cap = uni(out_cap[i] < OUT_CAP ? out_cap[i] : OUT_CAP);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  const gptr<uint8_t> dsta = dst - sh;                       // 16-byte aligned

  // varint32 header, coding.h:169-204; snappy.c:405-409.
  uint32_t want = 0, hlen = 0;
  {
    const uint64_t h = S ? view8(src) : 0;
    for (uint32_t k = 0; k < 5 && k < S; ++k) {
      const uint32_t b = (uint32_t)(h >> (8 * k)) & 0xffu;
      want |= (b & 0x7fu) << (7 * k);
      if ((b & 0x80u) == 0) {
        hlen = k + 1;
        break;
      }
    }
  }
  uint32_t st = (hlen == 0 || want > 0x7fffffffu) ? 0u : (want > cap ? 2u : 1u);

  // One 16-byte granule of the window that starts at stream offset `base`
  // (thread t's; zero past the stream; loads stay within 15 bytes past it).
  static_assert(L::kSw / 16 <= NT, "one staging granule per thread");
  auto fetch = [&](uint32_t base) -> u32x4 {
    u32x4 v = {0, 0, 0, 0};
    const uint32_t o = 16 * t;
    if ((t < L::kSw / 16) & (base < S) && o < S - base) {
      v = ld16(src + base + o);
      const uint32_t k = S - base - o;        // bytes 0..k-1 are the stream's
      if (k < 16) {
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
          const uint32_t lo = 4 * d;
          const uint32_t keep = k <= lo ? 0u : (k >= lo + 4 ? 0xffffffffu : (1u << (8 * (k - lo))) - 1u);
          v[d] &= keep;
        }
      }
    }
    return v;
  };

  uint32_t ws = hlen, wo = 0;                 // window start (stream), output made
  uint32_t F = sh ? 16u : 0u;                 // image offset flushed up to (granules)
  // The next window's granule, loaded while the current one decodes (its
  // start is known once the current window's ops are placed).
  u32x4 pf = fetch(ws);
  while ((st == 1) & (ws < S)) {               // snappy.c:208
    const uint32_t wn = S - ws < IN_WIN ? S - ws : IN_WIN;
    // ---- 1. stage the window
    if (t < L::kSw / 16) lwr16(s.sw + 16 * t, pf);
    __syncthreads();
    // ---- 2. parse every position (stream-only rejects: made/want checks off)
#pragma unroll
    for (uint32_t j = 0; j < P; ++j) {
      const uint32_t r = t * P + j;
      uint16_t jr = kTerm;
      if (r < wn) {
        const Tag tg = parse_tag(tag_bytes(s.sw, r), ws + r, S, 0xffffffffu, 0x7fffffffu);
        if (!tg.bad && tg.next - ws < wn) jr = (uint16_t)(tg.next - ws);
      }
      s.J[0][r] = jr;
      s.M[r] = r == 0;
    }
    s.cov[t] = 0;
    if (t == 0) {
      s.ctl[kBad] = 0;
      s.ctl[kNext] = S;
      s.ctl[kCut] = 0xffffffffu;
    }
    __syncthreads();
    // ---- 3. mark the chain from position 0 by pointer doubling
    uint32_t cur = 0;
    while (s.J[cur][0] != kTerm) {
#pragma unroll
      for (uint32_t j = 0; j < P; ++j) {
        const uint32_t r = t * P + j;
        const uint32_t a = s.J[cur][r];
        uint16_t nx = kTerm;
        if (a != kTerm) {
          if (s.M[r]) s.M[a] = 1;
          nx = s.J[cur][a];
        }
        s.J[cur ^ 1][r] = nx;
      }
      __syncthreads();
      cur ^= 1;
    }
    // ---- 4. ops: output offsets by a scan, output-dependent rejects
    uint32_t cnt = 0, sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < P; ++j) {
      const uint32_t r = t * P + j;
      if ((r < wn) && s.M[r]) {
        const Tag tg = parse_tag(tag_bytes(s.sw, r), ws + r, S, 0xffffffffu, 0x7fffffffu);
        ++cnt;
        sum += tg.bad ? 0u : tg.len;
      }
    }
    uint32_t kb, mb, nops, lw;
    scan2<NT>(cnt, sum, s.red, &kb, &mb, &nops, &lw);
#pragma unroll
    for (uint32_t j = 0; j < P; ++j) {
      const uint32_t r = t * P + j;
      if ((r < wn) && s.M[r]) {
        const uint32_t made = wo + mb;
        const Tag tg = parse_tag(tag_bytes(s.sw, r), ws + r, S, want, made);
        const bool lit = tg.kind == 0;
        const uint32_t len = tg.bad ? 0u : tg.len;
        s.oo[kb] = mb;
        s.os[kb] = lit ? ws + r + tg.hl : tg.dist;
        s.opos[kb] = (uint16_t)(r | (lit ? 0x8000u : 0u));
        if (tg.bad) s.ctl[kBad] = 1;
        else if (tg.next - ws >= wn) s.ctl[kNext] = tg.next;   // the window's last tag
        if ((mb <= OUT_WIN) & (mb + len > OUT_WIN)) s.ctl[kCut] = kb;
        const uint32_t c0 = (mb + C - 1) / C;
        if ((c0 < NT) & (c0 * C < mb + len)) s.cov[c0] = kb;
        ++kb;
        mb += len;
      }
    }
    if (t == 0) s.oo[nops] = lw;
    __syncthreads();
    if (s.ctl[kBad]) {
      st = 0;
      break;
    }
    uint32_t wl, nws;
    const uint32_t cut = s.ctl[kCut];
    const bool solo = (lw > OUT_WIN) & (cut == 0);
    if (lw <= OUT_WIN) {
      wl = lw;
      nws = s.ctl[kNext];
    } else if (!solo) {
      wl = s.oo[cut];
      nws = ws + (s.opos[cut] & 0x7fffu);
    } else {
      wl = s.oo[1];
      nws = nops > 1 ? ws + (s.opos[1] & 0x7fffu) : s.ctl[kNext];
    }
    pf = fetch(nws);
    // ---- 5-6. literal bytes and copy sources; resolve; gather
    if (!solo) {
      uint32_t k = scan_max<NT>(s.cov[t], s.red);
      const uint32_t o0 = t * C;
#pragma unroll 1
      for (uint32_t jj = 0; jj < C; ++jj) {
        const uint32_t o = o0 + jj;
        if (o >= wl) break;
        while (s.oo[k + 1] <= o) ++k;
        const uint32_t v = s.os[k];
        if (s.opos[k] & 0x8000u) {
          const uint32_t q = v + (o - s.oo[k]);
          const uint32_t b = q - ws < L::kSw ? s.sw[q - ws] : src[q];
          s.img[sh + wo + o] = (uint8_t)b;
          s.R[o] = wo + o;
        } else {
          s.R[o] = wo + o - v;
        }
      }
      bool changed;
      do {
        __syncthreads();
        changed = false;
#pragma unroll 1
        for (uint32_t jj = 0; jj < C; ++jj) {
          const uint32_t o = o0 + jj;
          if (o >= wl) break;
          const uint32_t r0 = s.R[o];
          if ((r0 >= wo) & (r0 != wo + o)) {
            const uint32_t r1 = s.R[r0 - wo];
            if (r1 != r0) {
              s.R[o] = r1;
              changed = true;
            }
          }
        }
      } while (__syncthreads_or(changed));
#pragma unroll 1
      for (uint32_t jj = 0; jj < C; ++jj) {
        const uint32_t o = o0 + jj;
        if (o >= wl) break;
        const uint32_t r0 = s.R[o];
        if (r0 != wo + o) s.img[sh + wo + o] = s.img[sh + r0];
      }
    } else {
      // A literal longer than OUT_WIN alone: straight from the stream in
      // 16-byte granules of the image (aligned LDS writes); the granules at
      // either end only take their own bytes (the first holds earlier
      // output).  Loads may run 15 bytes past the literal, inside the stream
      // or its read slack.
      const uint32_t lp = s.os[0];
      const uint32_t i0 = sh + wo, i1 = i0 + wl;          // image range
      for (uint32_t g = (i0 & ~15u) + 16 * t; g < i1; g += 16 * NT) {
        const int32_t d = (int32_t)g - (int32_t)i0;        // literal offset of byte g
        if ((d >= 0) & (g + 16 <= i1)) {
          lwr16(s.img + g, ld16(src + lp + (uint32_t)d));
        } else {
#pragma unroll 1
          for (uint32_t b = g; b < g + 16; ++b)
            if ((b >= i0) & (b < i1)) s.img[b] = src[lp + (b - i0)];
        }
      }
    }
    __syncthreads();
    // ---- 7. flush the window's whole granules
    const uint32_t E = (sh + wo + wl) & ~15u;
    for (uint32_t g = F + 16 * t; g < E; g += 16 * NT) st16(dsta + g, lrd16(s.img + g));
    F = E > F ? E : F;
    wo += wl;
    ws = nws;
    __syncthreads();
  }
  if ((st == 1) & (wo != want)) st = 0;        // snappy.c:337
  if (st == 1) {
    // the partial first and last granules, byte by byte
    const uint32_t G0 = sh ? 16u : 0u;
    for (uint32_t b = sh + t; b < sh + want; b += NT)
      if ((b < G0) | (b >= F)) dsta[b] = s.img[b];
  }
  if (t == 0) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

// One workgroup per block.  The 64 KiB class: 1 024 threads (16 waves) and
// 142 KB of LDS, so one block per CU at a time; smaller classes (single
// blocks, small batches): 97 KB.
hipError_t launch_decode_group(const DecodeArgs& a, uint32_t max_out, hipStream_t s) {
  if (max_out <= 16896) {
    hipLaunchKernelGGL((decode_group_kernel<16896, 4096, 8192, 1024>), dim3(a.n), dim3(1024), 0, s,
                       a.in, a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                       a.index, a.n, a.count);
  } else {
    hipLaunchKernelGGL((decode_group_kernel<66048, 4096, 8192, 1024>), dim3(a.n), dim3(1024), 0, s,
                       a.in, a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                       a.index, a.n, a.count);
  }
  return hipGetLastError();
}

}  // namespace lgs
