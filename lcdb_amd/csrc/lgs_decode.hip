// lgs_decode.hip -- batched Snappy block decoder for gfx950 (MI355X).
//
// Semantics: lcdb src/util/snappy.c:386-412 (snappy_decode_size/decode) and
// decode_blocks (snappy.c:201-341), restated for a wave64:
//   * one wave owns one block; WAVES independent waves per workgroup;
//   * the compressed block is staged global->LDS with 16-byte lanes, the
//     decoded block is built in LDS and streamed out with 16-byte stores;
//   * the tag walk is a scalar (SGPR) loop over tags that the lanes parse in
//     parallel, 64 stream positions at a time; each op's bytes are moved by
//     the lanes (decode_win);
//   * every reject condition of the reference is checked in the same order,
//     so the per-block accept/reject bit equals the reference's.
// Blocks whose compressed length exceeds the class's LDS staging area are
// decoded from global memory by the same loop (still on the GPU).  Outputs
// over the 16 KiB class go to decode_wide_kernel (rings, any size); large
// batches of small blocks to decode_ring_kernel (one lane per block).
//
// status[i]: 1 = ok, 0 = corrupt (reference returns 0), 2 = decoded length
// exceeds out_cap[i] (batch-API capacity check; the drop-in sizes the output
// from the header so it never sees 2).
#include "lgs_device.h"
#include "lgs_decode_common.h"
#include "lgs_launch.h"
#include "lgs_probe_hooks.h"
#include "lgs_service.h"

#include <mutex>

namespace lgs {

// Wave-per-block decode of an LDS-staged stream: stream byte k sits at
// base[sh + k] (base 16-byte aligned).  The tag walk is serial, so the parse
// is taken off it: per window of 64 stream positions w .. w+63, lane l
// parses, in parallel with the others, the tag that would start at w + l --
// its length, its step to the next tag, its source (a literal's first byte)
// or distance (a copy), and the reject conditions of snappy.c:210-324 that
// depend only on the stream.  The walk then reads the three packed fields of
// the tag at apos with v_readlane, checks the conditions that depend on the
// output produced so far (:263, :323) and moves the op's bytes (the lanes, one
// byte each); when it leaves the window the next one starts at apos.  (Round
// 2: 1 240 -> 1 083 us for C2 on this decoder, 16 KiB fillseq 108 -> 119
// GiB/s, 64 KiB 40 -> 43, against a walk that parsed each tag on the SALU.)
//
// Deferred write: an op's byte is read from LDS and written only after the
// next tag's checks, so the read's latency hides behind them; it is written
// before the next op reads anything (a copy may read it).  Until the first op
// it aims at the stream's never-consumed pad.
//
// In place: the stream is staged at the top of the same LDS buffer the output
// grows into from the bottom, o + gap == base.  Every write must end at or
// below the next unread stream byte (made + len <= gap + next), so no byte is
// overwritten before it is read; a stream that would break this (its output
// running ahead of its input by more than the class margin) returns 3 and is
// decoded again from global memory.  A literal needs made <= gap + from: its
// lanes read a 64-byte piece before writing it, and each piece's writes end
// where that piece's reads began, below every later piece.
__device__ uint32_t decode_win(const uint8_t* base, uint32_t sh, uint32_t slen, uint8_t* o,
                               int32_t gap, uint32_t cap, uint32_t* want_out) {
  const uint32_t lane = lane_id();

  // varint32 header, coding.h:169-204.
  const uint64_t w8 = uni64(lds_ld64(base, sh));
  uint32_t want = 0, hlen = 0;
  for (uint32_t i = 0; i < 5 && i < slen; ++i) {
    const uint32_t b = (uint32_t)(w8 >> (8 * i)) & 0xffu;
    if ((b & 0x80u) == 0) {
      want |= b << (7 * i);
      hlen = i + 1;
      break;
    }
    want |= (b & 0x7fu) << (7 * i);
  }
  if (hlen == 0 || want > 0x7fffffffu) return 0;    // snappy.c:405-409
  if (want > cap) return 2;
  *want_out = want;

  uint32_t apos = sh + hlen;                        // absolute LDS offset of the next tag
  const uint32_t aend = sh + slen;
  uint32_t made = 0;
  // The stream's never-consumed pad: the deferred write's target until the
  // first op.
  const uint32_t pad = (uint32_t)((int32_t)aend + gap) + kWave + lane;
  uint32_t pend = pad, pv = 0, res = 1;

  while (apos < aend) {                             // snappy.c:208
    // ---- the window: lane l looks at the tag that would start at q = w + l
    // (reads stay inside the staging pad past the stream end; lanes past it
    // are never used) and decides whether it is a *common* tag: a literal
    // with a one-byte header (<= 60 bytes) or a COPY1 / COPY2 whose bytes do
    // not overlap (dist >= len), inside the stream.  For those it packs what
    // the walk needs; every other tag, and every common tag that fails the
    // walk's one test, is decoded by the exact scalar path below.
    const uint32_t w = apos;
    const uint32_t q = w + lane;
    const uint32_t t = lds_ld32(base, q);
    const uint32_t tag = t & 0xffu, kind = tag & 3u, m0 = tag >> 2;
    const bool lit = kind == 0;
    const uint32_t len = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;       // snappy.c:216, 276, 289
    const uint32_t dist = kind == 1 ? ((tag & 0xe0u) << 3) | ((t >> 8) & 0xffu)
                                    : (t >> 8) & 0xffffu;            // snappy.c:279, 292
    const uint32_t step = lit ? len + 1 : kind + 1;
    // The walk accepts the tag when lo <= made <= hmax: made >= dist is
    // snappy.c:323's source bound, made <= want - len the length bound of
    // :263 / :323, and made <= gap + lim - 64 the in-place bound (a copy's
    // stream ends at q + step, a literal reads from q + 1).
    const int32_t lim = (int32_t)q + (int32_t)(lit ? 1u : step);
    const int32_t hi0 = (int32_t)want - (int32_t)len, hi1 = gap + lim - (int32_t)kWave;
    const int32_t hmax = hi0 < hi1 ? hi0 : hi1;
    const uint32_t lo = lit ? 0u : dist;
    const bool common = (lit ? m0 < 60 : (kind != 3) & (dist >= len) & (dist != 0)) &
                        (step <= aend - q);
    const bool fast = common & (hmax >= (int32_t)lo);
    const uint32_t flo = fast ? lo : 0xffffffffu;
    const uint32_t frng = fast ? (uint32_t)(hmax - (int32_t)lo) : 0u;
    // The op's first source byte relative to o: a literal's in the staged
    // stream (base == o + gap), a copy's at made - dist (made added below).
    const uint32_t fsrc = lit ? (uint32_t)(gap + (int32_t)q + 1) : 0u - dist;
    const uint32_t fpk = len | (step << 8) | (lit ? 0u : 0x10000u);

    // ---- the serial walk over this window's tags.  Both paths end in one
    // deferred write + one read, so the read's register is never copied
    // (a copy would wait for the read).
    const uint32_t wend = aend - w < kWave ? aend : w + kWave;
    do {
      const uint32_t d = apos - w;
      const uint32_t rlo = __builtin_amdgcn_readlane(flo, d);
      const uint32_t rrng = __builtin_amdgcn_readlane(frng, d);
      uint32_t n = 0, adv = 0, from = 0;
      if (made - rlo <= rrng) {
        const uint32_t pk = __builtin_amdgcn_readlane(fpk, d);
        const uint32_t src = __builtin_amdgcn_readlane(fsrc, d);
        n = pk & 0xffu;
        adv = (pk >> 8) & 0xffu;
        from = src + ((pk >> 16) ? made : 0u) + lane;
      } else {
        // The exact tag step of snappy.c:210-324, on the SALU.
        const uint64_t tv = uni64(lds_ld64(base, apos));
        const uint32_t tg = (uint32_t)tv & 0xffu, kd = tg & 3u;
        const uint32_t hi = (uint32_t)(tv >> 8), left = aend - apos;
        bool bad = false;
        uint32_t x = 0, ds = 0;
        int32_t lm = 0;
        if (kd == 0) {                              // literal, snappy.c:210-273
          uint32_t m = tg >> 2, hl = 1;
          if (m >= 60) {
            const uint32_t extra = m - 59;          // 1..4 length bytes
            bad = left - 1 < extra;
            m = extra == 4 ? hi : (hi & ((1u << (8 * (extra & 3u))) - 1u));
            hl += extra;
          }
          n = m + 1;
          bad = bad || m >= 0x7fffffffu || n > left - hl || n > want - made;   // :258, :263
          x = apos + hl;
          adv = hl + n;
          lm = (int32_t)x;
        } else {                                    // copies, snappy.c:276-324
          const uint32_t chl = kd == 1 ? 2u : (kd == 2 ? 3u : 5u);
          n = kd == 1 ? 4 + ((tg >> 2) & 7u) : 1 + (tg >> 2);
          ds = kd == 1 ? ((tg & 0xe0u) << 3) | (hi & 0xffu) : (kd == 2 ? hi & 0xffffu : hi);
          bad = left < chl || ds == 0 || ds >= 0x80000000u || made < ds || n > want - made;
          adv = chl;
          lm = (int32_t)(apos + chl);
        }
        const bool ahead = (int32_t)(made + kWave) - lm > gap;   // the in-place bound
        if (bad | ahead) {
          // One exit per loop (no selector chains from loop-exit
          // unification): end both walks; the tail below writes nothing
          // that matters (a corrupt block is not flushed, a run-ahead one
          // is decoded again from global memory into o).
          res = bad ? 0u : 3u;
          apos = aend;
          adv = 0;
          n = 0;
          from = made + lane;
        } else if (kd == 0) {
          if (n <= kWave) {
            from = (uint32_t)gap + x + lane;                     // base[x + lane]
          } else {
            o[pend] = (uint8_t)pv;                               // before the piece writes
            order();
            // 16 bytes a lane (unaligned ds_read/write_b128), then the last
            // < 16 bytes one a lane.  In place, a piece's writes end 64+
            // bytes below the next piece's reads (the in-place bound).
            typedef u32x4 u32x4_b __attribute__((aligned(1)));
            const uint32_t n16 = n & ~15u;
            for (uint32_t j = 16 * lane; j < n16; j += 16 * kWave)
              *(u32x4_b*)(o + made + j) = *(const u32x4_b*)(base + x + j);
            order();
            for (uint32_t j = n16 + lane; j < n; j += kWave) o[made + j] = base[x + j];
            pend = pad;                                          // the write below: harmless
            from = made + lane;
          }
        } else if (ds >= n) {
          from = made - ds + lane;
        } else {
          from = made - ds + lane % ds;             // lanes >= n: wild, overwritten later
        }
      }
      o[pend] = (uint8_t)pv;
      pv = o[from];
      pend = made + lane;
      order();
      made += n;
      apos += adv;
    } while (apos < wend);
  }
  o[pend] = (uint8_t)pv;
  if (res != 1) return res;

  return made == want ? 1u : 0u;                    // snappy.c:337
}

// One in-place buffer per wave: the output image grows from the bottom, the
// compressed stream is staged at the top (+ 48 for its alignment shift and
// zero pad, + 256 so the window reads of decode_win never read past the
// array).  kMargin is how far the output may run ahead of the input (literal
// headers still unread); half the LDS of separate input and output images,
// so twice the waves per CU.
template <uint32_t OUT_CAP>
struct DecBuf {
  static constexpr uint32_t kMargin = 512 + OUT_CAP / 64;
  static constexpr uint32_t kBuf = (OUT_CAP + 32 + kMargin + 48 + 256 + 15) & ~15u;
};

// One block: the stream src[0 .. slen) decoded into dst (capacity cap),
// built in the wave's LDS buffer buf (DecBuf<OUT_CAP>::kBuf bytes).  Returns
// the status (1 ok, 0 corrupt, 2 no space), *want_out the decoded length.
template <uint32_t OUT_CAP>
__device__ __forceinline__ uint32_t decode_item(uint8_t* buf, gptr<const uint8_t> src,
                                                uint32_t slen, gptr<uint8_t> dst, uint32_t cap0,
                                                uint32_t* want_out) {
  constexpr uint32_t kBuf = DecBuf<OUT_CAP>::kBuf;
  LGS_DEC_PH_DECL;
  const uint32_t cap = cap0 < OUT_CAP ? cap0 : OUT_CAP;
  const uint32_t oshift = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  uint8_t* o = buf + oshift;

  uint32_t want = 0, st = 3;
  if (slen <= kBuf - 48 - 256) {
    const uint32_t ib = (kBuf - slen - 48 - 256) & ~15u;
    constexpr uint32_t kR = (kBuf + 1023) / 1024 < 8 ? (kBuf + 1023) / 1024 : 8;
    const uint32_t sh = stage_in<kR>(buf + ib, src, slen);
    order();
    LGS_DEC_PH_STAGED();
    st = decode_win(buf + ib, sh, slen, o, (int32_t)ib - (int32_t)oshift, cap, &want);
    order();
    LGS_DEC_PH_END(flush_out(dst, buf, want), (gptr<uint32_t>)(dst + ((cap0 - 16) & ~3u)));
  }
  if (st == 3) st = decode_stream(GlobalStream{src, slen}, slen, o, cap, &want);
  if (st == 1) flush_out(dst, buf, want);
  *want_out = want;
  return st;
}

template <uint32_t OUT_CAP, uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void decode_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count, const Item1 one) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[WAVES][DecBuf<OUT_CAP>::kBuf];

  // Per-wave scalars go through v_readfirstlane so hipcc keeps the whole
  // tag walk on the SALU (it cannot prove threadIdx.x >> 6 wave-uniform).
  const uint32_t wv = uni(threadIdx.x >> 6);
  const uint32_t slot = blockIdx.x * WAVES + wv;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);

  uint64_t ioff, ooff;
  uint32_t slen, cap;
  if (one.on) {                                     // the drop-in's item, by value
    ioff = one.in_off; ooff = one.out_off; slen = one.in_len; cap = one.aux;
  } else {
    ioff = uni64(in_off[i]); ooff = uni64(out_off[i]); slen = uni(in_len[i]); cap = uni(out_cap[i]);
  }
  uint32_t want = 0;
  const uint32_t st = decode_item<OUT_CAP>(&s_buf[wv][0], to_global(in) + ioff, slen,
                                           to_global(out) + ooff, cap, &want);
  if (lane_id() == 0) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

// The drop-in service's decode waves (lgs_launch.h): wave k serves mailbox
// k, one stream whose output is <= kSvcMaxItem bytes at a time (the host
// checked the header), from its slot's arena.
__global__ __launch_bounds__(64) void decode_service_kernel(SvcMailbox* __restrict__ mb,
                                                            uint64_t idle,
                                                            SvcControl* __restrict__ ctl) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[DecBuf<kSvcMaxItem>::kBuf];
  svc_loop(mb + blockIdx.x, idle, ctl,
           [&](uint32_t len, uint64_t input, uint64_t arena, uint32_t* status, uint32_t* out_len) {
             uint8_t* a = reinterpret_cast<uint8_t*>(arena);
             len = len < kSvcOut - kSvcIn - 16 ? len : kSvcOut - kSvcIn - 16;   // (never more)
             uint32_t want = 0;
             const uint32_t st = decode_item<kSvcMaxItem>(s_buf, to_global(reinterpret_cast<const uint8_t*>(input)), len,
                                                          to_global(a) + kSvcOut, kSvcMaxItem,
                                                          &want);
             *status = st;
             *out_len = st == 1 ? want : 0;
           });
}

hipError_t launch_decode_service(SvcMailbox* mb, uint32_t nslots, uint64_t idle,
                                 SvcControl* ctl, hipStream_t s) {
  hipLaunchKernelGGL(decode_service_kernel, dim3(nslots), dim3(64), 0, s, mb, idle, ctl);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Wide decoder: outputs over the 16 KiB class (the 64 KiB class and larger).
// decode_kernel held a whole 64 KiB block in LDS (68 KB: two waves per CU,
// so 1 024 such blocks ran as two generations of one serial walk each: 70
// GiB/s on C3's 64 KiB fillseq class), and a global-memory walk for larger
// outputs waited for memory on every copy.  Here a wave keeps
//   * a 32 KiB ring of its output, flushed to HBM in 16-byte granules once
//     8 KiB are pending at a window start, and
//   * a 4 KiB ring of its stream (+ an 80-byte mirror of its start), staged
//     2 KiB at a time from registers prefetched one refill ahead,
// 37 KB in all: four waves per CU.  The walk is decode_win's (one range test
// per common tag, an exact scalar step for the rest) without the in-place
// bound; a copy reaching further back than the ring (dist > 32 704) reads
// the flushed output from HBM after its stores have drained.
// ---------------------------------------------------------------------------

// OUT / IN: the output and input ring sizes (powers of two, IN >= 2048).
template <uint32_t OUT, uint32_t IN>
__global__ __launch_bounds__(64) void decode_wide_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count) {
  constexpr uint32_t kOut = OUT;             // output ring
  constexpr uint32_t kIn = IN;               // input ring
  constexpr uint32_t kMirror = 80;           // stream bytes kIn.. mirror ring offsets 0..79
  constexpr uint32_t kBuf = kOut + kIn + kMirror + kWave;   // + a pad for harmless writes
  constexpr uint32_t kPad = kOut + kIn + kMirror;
  constexpr uint32_t kRefill = kIn / 2;      // stream bytes per refill
  constexpr uint32_t kGran = kRefill / 1024; // 16-byte granules per lane and refill
  // Pending output that triggers a flush.  A window makes <= 4 KiB, so the
  // unflushed bytes stay under kFlushAt + 4 160 < kOut - 64 (the pending
  // write's wild lanes never reach an unflushed byte), and a far copy's
  // source (dist > kFar) ends below F.
  constexpr uint32_t kFlushAt = kOut / 4;
  constexpr uint32_t kFar = kOut - kWave;    // copies up to this distance read the ring
  static_assert(kFlushAt + 4224 <= kOut && (kGran == 1 || kGran == 2), "ring sizes");
  __shared__ __attribute__((aligned(16))) uint8_t sb[kBuf];
  uint8_t* const ib = sb + kOut;            // input ring

  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);
  const uint32_t lane = lane_id();
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  const uint32_t slen = uni(in_len[i]);
  const uint64_t doff = uni64(out_off[i]);
  const gptr<uint8_t> dst = to_global(out) + doff;
  const uint8_t* const dgen = out + doff;   // (generic, for the agent-scope far-copy loads)
  const uint32_t cap = uni(out_cap[i]);
  const uint32_t oshift = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  const gptr<uint8_t> dal = dst - oshift;  // 16-byte aligned; byte b is at dal + b + oshift

  // varint32 header, coding.h:169-204 (reads stay inside the 16-byte slack).
  uint32_t st = 1, want = 0, hlen = 0;
  {
    const uint64_t h = uni64(view8(src));
    for (uint32_t k = 0; k < 5 && k < slen; ++k) {
      const uint32_t b = (uint32_t)(h >> (8 * k)) & 0xffu;
      if ((b & 0x80u) == 0) {
        want |= b << (7 * k);
        hlen = k + 1;
        break;
      }
      want |= (b & 0x7fu) << (7 * k);
    }
    if (hlen == 0 || want > 0x7fffffffu) st = 0;              // snappy.c:405-409
    else if (want > cap) st = 2;
  }

  // ---- input ring: stream position p at ib[p & (kIn - 1)], positions with
  // p & (kIn - 1) < kMirror also at ib[kIn + ...].  Lane l prefetches the
  // granules l and l + 64 of the next chunk.
  uint32_t staged = 0;
  u32x4 pf0 = {0, 0, 0, 0}, pf1 = pf0;
  auto prefetch = [&]() {
    const uint32_t c0 = staged + 16 * lane, c1 = c0 + 1024;
    if (c0 < slen) pf0 = ld16(src + c0);
    if (kGran == 2 && c1 < slen) pf1 = ld16(src + c1);
  };
  auto land = [&]() {       // the prefetched chunk into the ring, then the next prefetch
    __builtin_amdgcn_s_waitcnt(0x0f70);                       // vmcnt(0)
    const uint32_t r0 = (staged + 16 * lane) & (kIn - 1), r1 = (r0 + 1024) & (kIn - 1);
    *reinterpret_cast<u32x4*>(ib + r0) = pf0;
    if (r0 < kMirror) *reinterpret_cast<u32x4*>(ib + kIn + r0) = pf0;
    if (kGran == 2) {
      *reinterpret_cast<u32x4*>(ib + r1) = pf1;
      if (r1 < kMirror) *reinterpret_cast<u32x4*>(ib + kIn + r1) = pf1;
    }
    order();
    staged += kRefill;
    prefetch();
  };

  // ---- output ring: output byte b at sb[(b + oshift) & (kOut - 1)].
  uint32_t made = 0, F = 0;
  auto flush = [&](uint32_t to) {           // bytes [F, to) to HBM; to: a granule edge or want
    const uint32_t g0 = (F + oshift) >> 4, g1 = (to + oshift + 15) >> 4;
    for (uint32_t g = g0 + lane; g < g1; g += kWave) {
      const uint32_t lo = 16 * g, hi = lo + 16;                // in dal coordinates
      const u32x4 v = *reinterpret_cast<const u32x4*>(sb + (lo & (kOut - 1)));
      if (lo >= F + oshift && hi <= to + oshift) {
        *(gptr<u32x4>)(dal + lo) = v;
      } else {
        for (uint32_t b = lo; b < hi; ++b)
          if (b >= F + oshift && b < to + oshift) dal[b] = (uint8_t)byte_of(v, b - lo);
      }
    }
    F = to;
  };

  uint32_t apos = hlen;
  const uint32_t aend = slen;
  if (st == 1) {
    prefetch();
    land();
    land();
  }
  // The deferred write: pending byte pv goes to sb[pend] (the pad until the
  // first op), written before the next op reads anything.
  const uint32_t pad = kPad + lane;
  uint32_t pend = pad, pv = 0;
  uint32_t w = 0, wend = 0, flo = 0, frng = 0, fsrc = 0, fpk = 0;
  while (st == 1 && apos < aend) {                            // snappy.c:208
    // ---- window start: stage the stream (>= 144 bytes past w, the reach of
    // this window's literals), flush once 8 KiB are pending, and parse.
    w = apos;
    wend = aend - w < kWave ? aend : w + kWave;
    while (staged < aend && staged <= w + kRefill) land();   // (staged may trail w after a long literal)
    if (made - F >= kFlushAt) {
      sb[pend] = (uint8_t)pv;                 // the last op's bytes, before they are flushed
      pend = pad;
      order();
      flush(((made + oshift) & ~15u) - oshift);
    }
    {
      const uint32_t q = w + lane;
      const uint32_t t = lds_ld32(ib, q & (kIn - 1));
      const uint32_t tag = t & 0xffu, kind = tag & 3u, m0 = tag >> 2;
      const bool lit = kind == 0;
      const uint32_t len = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;     // snappy.c:216, 276, 289
      const uint32_t dist = kind == 1 ? ((tag & 0xe0u) << 3) | ((t >> 8) & 0xffu)
                                      : (t >> 8) & 0xffffu;          // snappy.c:279, 292
      const uint32_t step = lit ? len + 1 : kind + 1;
      // Accepted when lo <= made <= hi: snappy.c:323's source bound and the
      // length bound of :263 / :323.
      const int32_t hi = (int32_t)want - (int32_t)len;
      const uint32_t lo = lit ? 0u : dist;
      const bool common = (lit ? m0 < 60 : (kind != 3) & (dist >= len) & (dist != 0) &
                                           (dist <= kFar)) & (step <= aend - q);
      const bool fast = common & (hi >= (int32_t)lo);
      flo = fast ? lo : 0xffffffffu;
      frng = fast ? (uint32_t)(hi - (int32_t)lo) : 0u;
      // A literal's first byte in the input ring (linear through the
      // mirror), a copy's output position less made, shifted into the ring.
      fsrc = lit ? kOut + ((q + 1) & (kIn - 1)) : oshift - dist;
      fpk = len | (step << 8) | (lit ? 0u : 0x10000u);
    }
    do {
      const uint32_t d = apos - w;
      const uint32_t rlo = __builtin_amdgcn_readlane(flo, d);
      const uint32_t rrng = __builtin_amdgcn_readlane(frng, d);
      uint32_t nb = 0, adv = 0, from = 0;
      if (made - rlo <= rrng) {
        const uint32_t pk = __builtin_amdgcn_readlane(fpk, d);
        const uint32_t sr = __builtin_amdgcn_readlane(fsrc, d);
        nb = pk & 0xffu;
        adv = (pk >> 8) & 0xffu;
        from = (pk >> 16) ? ((sr + made + lane) & (kOut - 1)) : sr + lane;
      } else {
        // The exact tag step of snappy.c:210-324, on the SALU.
        const uint64_t tv = uni64(lds_ld64(ib, apos & (kIn - 1)));
        const uint32_t tg = (uint32_t)tv & 0xffu, kd = tg & 3u;
        const uint32_t hi = (uint32_t)(tv >> 8), left = aend - apos;
        bool bad = false;
        uint32_t x = 0, ds = 0;
        if (kd == 0) {                              // literal, snappy.c:210-273
          uint32_t m = tg >> 2, hl = 1;
          if (m >= 60) {
            const uint32_t extra = m - 59;          // 1..4 length bytes
            bad = left - 1 < extra;
            m = extra == 4 ? hi : (hi & ((1u << (8 * (extra & 3u))) - 1u));
            hl += extra;
          }
          nb = m + 1;
          bad = bad || m >= 0x7fffffffu || nb > left - hl || nb > want - made;   // :258, :263
          x = apos + hl;
          adv = hl + nb;
        } else {                                    // copies, snappy.c:276-324
          const uint32_t chl = kd == 1 ? 2u : (kd == 2 ? 3u : 5u);
          nb = kd == 1 ? 4 + ((tg >> 2) & 7u) : 1 + (tg >> 2);
          ds = kd == 1 ? ((tg & 0xe0u) << 3) | (hi & 0xffu) : (kd == 2 ? hi & 0xffffu : hi);
          bad = left < chl || ds == 0 || ds >= 0x80000000u || made < ds || nb > want - made;
          adv = chl;
        }
        if (bad) {
          // One exit per loop: end the walk through the loop conditions.
          st = 0;
          apos = aend;
          adv = 0;
          nb = 0;
          from = pad;
        } else if (kd == 0 && nb <= kWave) {
          from = kOut + (x & (kIn - 1)) + lane;    // staged: x + 64 <= w + 136
        } else if (kd == 0) {
          // A long literal: piece by piece from the input ring (refilled as
          // it drains) into the output ring (flushed as it fills).  The
          // pending write goes first: its wild lanes may cover these bytes.
          sb[pend] = (uint8_t)pv;
          pend = pad;
          order();
          // Bytes up to the output ring's next 16-byte edge one a lane,
          // then whole granules straight from HBM (16 bytes a lane, 4 KiB in
          // flight: the input ring is bypassed and restaged after), then the
          // last < 16 bytes one a lane.  Reads stay within the block's
          // 16-byte read slack.
          const uint32_t u0 = made + oshift;
          const uint32_t head0 = (16u - (u0 & 15u)) & 15u;
          const uint32_t head = head0 < nb ? head0 : nb;
          const uint32_t body = (nb - head) & ~15u;
          const gptr<const uint8_t> ls = src + x;
          if (lane < head) sb[(u0 + lane) & (kOut - 1)] = ls[lane];
          order();
          for (uint32_t j = head; j < head + body; j += 4096) {
            if (made + j - F >= kFlushAt) flush(((made + j + oshift) & ~15u) - oshift);
            u32x4 v[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
              const uint32_t jj = j + 16 * (lane + 64 * k);
              if (jj < head + body) v[k] = ld16(ls + jj);
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
              const uint32_t jj = j + 16 * (lane + 64 * k);
              if (jj < head + body)
                *reinterpret_cast<u32x4*>(sb + ((u0 + jj) & (kOut - 1))) = v[k];
            }
            order();
          }
          if (made + nb - F >= kFlushAt) flush(((made + head + body + oshift) & ~15u) - oshift);
          {
            const uint32_t jj = head + body + lane;
            if (jj < nb) sb[(u0 + jj) & (kOut - 1)] = ls[jj];
          }
          order();
          // The stream resumes at x + nb: restage from there.
          if (x + nb > staged) {
            __builtin_amdgcn_s_waitcnt(0x0f70);                   // the old prefetch
            staged = (x + nb) & ~15u;
            prefetch();
          }
          from = (made + oshift + lane) & (kOut - 1);
        } else if (ds > kFar) {
          // Beyond the ring: the flushed output, once its stores have
          // drained (ds > kFar puts the source below F; never overlapping).
          sb[pend] = (uint8_t)pv;
          pend = pad;
          __builtin_amdgcn_s_waitcnt(0x0f70);                     // vmcnt(0)
          const uint8_t v = gl_byte(dgen + made - ds + lane);
          sb[(made + oshift + lane) & (kOut - 1)] = v;
          order();
          from = (made + oshift + lane) & (kOut - 1);
        } else if (ds >= nb) {
          from = (made - ds + oshift + lane) & (kOut - 1);
        } else {
          from = (made - ds + oshift + lane % ds) & (kOut - 1);  // lanes >= nb: wild
        }
      }
      sb[pend] = (uint8_t)pv;
      pv = sb[from];
      pend = (made + oshift + lane) & (kOut - 1);
      order();
      made += nb;
      apos += adv;
    } while (apos < wend);
  }
  sb[pend] = (uint8_t)pv;
  order();
  if (st == 1 && made != want) st = 0;                        // snappy.c:337
  if (st == 1) flush(want);
  if (lane == 0) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

}  // namespace lgs

// ---------------------------------------------------------------------------
// Launchers (internal; the C ABI is in lgs_api.cpp).
// Decode classes by the largest output a launch must hold in LDS.
// ---------------------------------------------------------------------------
namespace lgs {

template <uint32_t OUT_CAP, uint32_t WAVES>
static hipError_t launch_decode_cls(const DecodeArgs& a, hipStream_t s) {
  const uint32_t grid = (a.n + WAVES - 1) / WAVES;
  hipLaunchKernelGGL((decode_kernel<OUT_CAP, WAVES>), dim3(grid), dim3(64 * WAVES), 0, s,
                     a.in, a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                     a.index, a.n, a.count, a.one);
  return hipGetLastError();
}

// Class limits (bytes of decoded output held in LDS per wave).
// ---------------------------------------------------------------------------
// Ring decoder: lane-per-block with LDS staging (large batches).
//
// The lane kernel above moves every byte as a 16-byte access of its own
// lane, so each memory instruction touches 64 cache lines: on C2 the
// texture addresser is ~93 % busy and partially written lines are evicted
// and rewritten (3.4x the output bytes reach HBM).  Here each lane keeps
//   * an input window: a 128-byte ring of its compressed stream, refilled
//     64 bytes at a time by 4 cooperating lanes (one coalesced line), and
//   * an output ring of 256 bytes, flushed 128 bytes at a time by 8
//     cooperating lanes (whole lines, written once),
// both in LDS with a 64-byte mirror after the ring so that any read of up
// to 64 bytes from a ring offset is linear.  Literals and copies with
// dist <= kNear move LDS to LDS; farther copies read the already flushed
// output from memory, issued when the tag is parsed and used a trip later.
// A trip = one piece (<= 64 bytes) of one op per lane; every memory
// operation issued in a trip is waited for once, at the top of the next.
// TWO (the default): a trip has a second op slot after the flush -- the
// piece of the op just parsed, if its bytes are in LDS, and the tag after
// it -- so a literal and a near copy take one trip instead of two.  The
// ring bounds still hold: the flush leaves < 128 unflushed bytes, each slot
// adds <= 64, and the next trip's first piece starts below 192.  A far copy
// met in the second slot is taken only when its source is flushed already.
// BL: blocks per wave.  With BL = 32 (the default) lanes 32-63 only serve
// the refill and flush jobs; the rings then fit eight waves in a CU's LDS,
// two per SIMD, which overlap each other's once-per-trip memory waits.
// ---------------------------------------------------------------------------
namespace ring {
constexpr uint32_t kInRing = 128, kInStride = 208;     // ring + 64 mirror + 16 sink
// 16 pad + ring + 64 mirror + 16, + 16 for the ring's shift by the
// destination's alignment (below).  Still 15 LDS granules per wave.
constexpr uint32_t kOutRing = 256, kOutStride = 368;
constexpr uint32_t kNear = 240;                         // ring minus one wild chunk
constexpr uint32_t kFlush = 128;
constexpr uint32_t kInSink = kInRing + 64;             // a lane's sink slot (its slack)
}  // namespace ring


// The tag's 5 bytes (parse_tag reads tv.x and the low byte of tv.y) from
// two aligned dwords: an unaligned ds_read_b128 is replayed (+~60 LDS
// cycles; the ring's SQ_LDS_UNALIGNED_STALL was 55 % of its LDS-busy
// cycles on C2, profiles/r5c_pmc.txt).  (The pieces' 16-byte accesses stay
// ds_read/write_b128: as aligned dwords (5 reads + v_alignbyte, a write as
// 3 bytes + 4 dwords) they are exact and slower, 339 against 274 us, and
// even wrong-byte aligned b128s gain only 3 % -- the instructions, not the
// LDS cycles, are what a trip waits on; profiles/r5d_ab.txt.)
__device__ __forceinline__ u32x4 rrd_tag(const uint8_t* p) {
  const uint32_t r = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - r);
  const uint32_t d0 = w[0], d1 = w[1];
  return u32x4{__builtin_amdgcn_alignbyte(d1, d0, r), d1 >> (8 * r), 0u, 0u};
}

// 16 bytes at output offset p of a lane's ring (ob = ring start): the ring
// copy, plus the mirror copy (r < 64) or the wrapped part (r > 240), which
// only those lanes write.
__device__ __forceinline__ void out_put(uint8_t* ob, uint32_t p, u32x4 v) {
  const uint32_t r = p & (ring::kOutRing - 1);
  lwr16(ob + r, v);
  // r < 64 or r > 240 as one unsigned compare; the second copy's offset as
  // one select (its value for the other lanes is never used).  (Written by
  // every lane, to a pad for the others, it cost 1.5 %; the whole trip
  // branch-free that way, 35 %: LDS stores cost by the lanes they move,
  // profiles/r4h_session.txt.)
  if (r - 64 > 176u) lwr16(ob + (int32_t)r + (r < 64 ? 256 : -256), v);
}

// A cooperative job (a refill or a flush) of one lane, 16 bytes: the lane
// rides in the top byte of the pointer's high word (virtual addresses are
// 48-bit).
struct RingJob {
  uint32_t off, cnt, plo, phil;
  __device__ RingJob() = default;
  __device__ RingJob(uint32_t ln, uint32_t o, uint32_t c, uint64_t p)
      : off(o), cnt(c), plo((uint32_t)p), phil((uint32_t)(p >> 32) | (ln << 24)) {}
  __device__ uint32_t lane() const { return phil >> 24; }
  __device__ uint64_t ptr() const { return ((uint64_t)(phil & 0xffffffu) << 32) | plo; }
};

template <bool TWO, uint32_t BL>
__global__ __launch_bounds__(64) void decode_ring_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count) {
  using namespace ring;
  // BL lanes decode (BL blocks per wave); with BL < 64 the others only help
  // with refills and flushes.  At most BL lanes post a flush job and at most
  // min(BL, 32) a refill job per trip.
  constexpr uint32_t kJobs = BL > 32 ? BL : 32;
  __shared__ __attribute__((aligned(16))) uint8_t s_in[BL * kInStride];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[BL * kOutStride];
  __shared__ __attribute__((aligned(16))) RingJob s_job[kJobs];

  // Every lane stays to the end: lanes without a block still work for the
  // cooperative refills and flushes.
  const uint32_t lane = threadIdx.x;
  const uint32_t slot = blockIdx.x * BL + lane;
  if (count) n = *count;
  if (blockIdx.x * BL >= n) return;   // a whole wave without blocks
  const bool exists = lane < BL && slot < n;
  const uint32_t i = exists ? (index ? index[slot] : slot) : 0;
  const gptr<const uint8_t> src = to_global(in) + (exists ? in_off[i] : 0);
  const uint32_t slen = exists ? in_len[i] : 0;
  const gptr<uint8_t> dst = to_global(out) + (exists ? out_off[i] : 0);
  const uint32_t cap = exists ? out_cap[i] : 0;
  uint8_t* const ib = s_in + (lane < BL ? lane : 0) * kInStride;     // (helpers: unused)
  // The output ring is shifted by the destination's alignment (dst & 15), so
  // a flush job's 16-byte reads (which end on the destination's line
  // boundaries) are aligned in LDS whatever the slot's alignment: unaligned,
  // they cost 6 % of C2 decode with outputs 1 byte off (303 against 286 us).
  uint8_t* const ob = s_out + (lane < BL ? lane : 0) * kOutStride + 16 +
                      ((uint32_t)reinterpret_cast<uintptr_t>(dst) & 15u);

  // varint32 header, coding.h:169-204.  st: 1 decoding/ok, 0 corrupt,
  // 2 no space, 3 no block.
  uint32_t st = exists ? 1u : 3u, want = 0, hlen = 0;
  if (exists) {
    const uint64_t h = view8(src);
    for (uint32_t k = 0; k < 5 && k < slen; ++k) {
      const uint32_t b = (uint32_t)(h >> (8 * k)) & 0xffu;
      if ((b & 0x80u) == 0) {
        want |= b << (7 * k);
        hlen = k + 1;
        break;
      }
      want |= (b & 0x7fu) << (7 * k);
    }
    if (hlen == 0 || want > 0x7fffffffu) st = 0;                // snappy.c:405-409
    else if (want > cap) st = 2;
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);

  uint32_t pos = hlen;               // next tag (stream offset)
  uint32_t made = 0, F = 0;          // output produced / flushed
  uint32_t in_req = 0, in_have = 0;  // input requested / landed (64-byte units)
  uint32_t orem = 0, okind = 0, odist = 0, olp = 0;   // current op: bytes left, ...
  bool ofar = false;
  u32x4 fa0 = {0, 0, 0, 0}, fa1 = fa0, fa2 = fa0, fa3 = fa0;   // far-copy bytes
  u32x4 rv0 = fa0, rv1 = fa0;                                  // refill bytes (worker)
  // A lane's sink for dropped refill writes: its own slack (helpers share a
  // decoding lane's).
  const uint32_t sink = (lane < BL ? lane : (lane - BL) % BL) * kInStride + kInSink;
  uint32_t ra0 = sink, rm0 = sink, ra1 = sink, rm1 = sink;

  // One piece (<= 64 bytes) of the current op (snappy.c:210-331) for every
  // lane whose bytes are in LDS (literal from the window, copy from the ring).
  auto piece = [&]() {
    const bool lit = okind == 0;
    const uint32_t piece = orem < 64 ? orem : 64;
    // (One condition, one exec-mask region.)
    if ((st == 1) & (orem > 0) & !ofar & (!lit | (in_have >= olp + piece))) {
      {
        const uint32_t dist = odist;
        const bool overlap = !lit & (dist < piece);
        const bool pat = overlap & (dist <= 8) & ((dist & (dist - 1)) == 0);
        if (overlap & !pat) {
          // Period not dividing 16: chunk by chunk, each reading bytes the
          // previous ones wrote (LDS program order); chunk 0 of a period
          // < 16 is built byte by byte, later chunks copy from qq back
          // (qq = a multiple of the period >= 16).
          const uint32_t qq = dist >= 16 ? dist : dist * ((16 + dist - 1) / dist);
          u32x4 p0;
          if (dist >= 16) {
            p0 = lrd16(ob + ((made - dist) & (kOutRing - 1)));
          } else {
            const u32x4 c0 = lrd16(ob + ((made - dist) & (kOutRing - 1)));
            uint32_t w[4] = {0, 0, 0, 0};
            uint32_t r = 0;
  #pragma clang loop unroll(disable)
            for (uint32_t j = 0; j < 16; ++j) {
              w[j >> 2] |= byte_of(c0, r) << (8 * (j & 3u));
              r = r + 1 == dist ? 0 : r + 1;
            }
            p0 = u32x4{w[0], w[1], w[2], w[3]};
          }
          out_put(ob, made, p0);
          order();
  #pragma clang loop unroll(disable)
          for (uint32_t k = 1; 16 * k < piece; ++k) {
            const u32x4 v = lrd16(ob + ((made + 16 * k - qq) & (kOutRing - 1)));
            out_put(ob, made + 16 * k, v);
            order();
          }
        } else {
          // A literal reads the input window, a copy the output ring.
          const uint8_t* sp = lit ? ib + (olp & (kInRing - 1))
                                  : ob + ((made - dist) & (kOutRing - 1));
          const u32x4 c0 = lrd16(sp);
          // Period 1/2/4/8: the dist bytes before d as a 16-byte pattern
          // (byte 0 four times, bytes 0-1 twice: one v_perm each, not a
          // quarter-rate v_mul_lo_u32).
          const uint32_t w1 = __builtin_amdgcn_perm(c0.x, c0.x, 0x00000000u);
          const uint32_t w2 = __builtin_amdgcn_perm(c0.x, c0.x, 0x01000100u);
          const uint32_t px = dist == 1 ? w1 : (dist == 2 ? w2 : c0.x);
          const uint32_t py = dist == 8 ? c0.y : px;
          const u32x4 pv = {px, py, px, py};
          out_put(ob, made, pat ? pv : c0);
          // Later chunks are read only when the piece has them (and not for
          // a pattern).  A source chunk can share ring slots only with a
          // later destination chunk (dist <= 240), so reading chunk k just
          // before writing chunk k keeps every read ahead of its clobber.
          // (All four reads issued before the first write -- legal here, no
          // source chunk holds a byte the piece writes -- is slower: 292-294
          // against 273-275 us on C2, profiles/r5b_ab.txt.  The LDS pipe, not
          // the round trips, is what a piece waits on.)
          if (piece > 16) out_put(ob, made + 16, pat ? pv : lrd16(sp + 16));
          if (piece > 32) out_put(ob, made + 32, pat ? pv : lrd16(sp + 32));
          if (piece > 48) out_put(ob, made + 48, pat ? pv : lrd16(sp + 48));
        }
        made += piece;
        orem -= piece;
        if (lit) olp += piece;
      }
    }
  };


  // Parse the next tag (its bytes are in the window); a far copy's bytes are
  // loaded from the flushed output for the next trip.
  auto parse = [&](bool second) {
    // Computed on every lane and committed with selects: one exec-mask
    // region (the far-copy loads) instead of three nested ones.  Lanes that
    // are not parsing read their own ring (in range) and discard the tag.
    const uint32_t need_to = slen - pos < 5 ? slen : pos + 5;
    const bool ready = (st == 1) & (orem == 0) & (pos < slen) & (in_have >= need_to);
    const Tag t = parse_tag(rrd_tag(ib + (pos & (kInRing - 1))), pos, slen, want, made);
    const bool far = (t.kind != 0) & (t.dist > kNear);
    if (ready & t.bad) st = 0;
    // (A far copy parsed in the second slot must find its source flushed
    // already; otherwise it waits for the next trip's first.)
    const bool take = ready & !t.bad & (!second | !far | (made - F + t.len <= t.dist));
    orem = take ? t.len : orem;
    okind = take ? (t.kind == 0 ? 0u : 1u) : okind;
    odist = take ? t.dist : odist;
    olp = take ? pos + t.hl : olp;
    pos = take ? t.next : pos;
    ofar = take ? far : ofar;
    if (take & far) {
      // The copy's own bytes are flushed already (first slot: they end <=
      // made - kNear + 64 < F; second slot: the take test above).  A granule
      // reads up to 15 bytes past the copy; they lie inside [0, made) of this
      // block (dist > kNear), may be bytes not yet flushed, and are never
      // used (the landing writes only orem bytes' worth that count).
      const gptr<const uint8_t> sp = (gptr<const uint8_t>)(dst + (made - odist));   // 32-bit offset
      fa0 = LGS_RING_FAR_LD16(sp);
      // Only the 16-byte granules the copy has: most far copies are 4-6
      // bytes (a key's shared prefix), and loading all 64 fetched 232 MB for
      // 70 MB used on C2.  Same time, less traffic
      // (profiles/r5b_ab.txt).
      if (t.len > 16) {
        fa1 = LGS_RING_FAR_LD16(sp + 16);
        if (t.len > 32) {
          fa2 = LGS_RING_FAR_LD16(sp + 32);
          if (t.len > 48) fa3 = LGS_RING_FAR_LD16(sp + 48);
        }
      }
    }
  };

  // Rotated: the loop's test is its last step (a test at the top became a
  // selector variable and a bool round trip through a VGPR).  A trip with no
  // active lane (every block's header corrupt) does nothing.
  LGS_RING_TRIPS_DECL;
  LGS_RING_PH_DECL;
  do {
    LGS_RING_TRIP();
    LGS_RING_PH_TRIP();
    LGS_RING_PH(7);                    // (the loop test, from the last trip)

    // ---- one piece of the current op for every lane whose bytes are in LDS;
    // this runs before the wait, so last trip's loads land meanwhile.
    piece();
    order();
    LGS_RING_PH(0);

    // ---- everything issued last trip has landed: far-copy pieces (never
    // overlapping, <= 64 bytes), then the input refills.
    __builtin_amdgcn_s_waitcnt(0x0f70);                         // vmcnt(0)
    LGS_RING_PH(1);
    if ((st == 1) & (orem > 0) & ofar) {
      out_put(ob, made, fa0);
      if (orem > 16) out_put(ob, made + 16, fa1);
      if (orem > 32) out_put(ob, made + 32, fa2);
      if (orem > 48) out_put(ob, made + 48, fa3);
      made += orem;
      orem = 0;
      ofar = false;
    }
    // (Lanes without a refill chunk, or a chunk without a mirror copy, hold
    // the sink: they skip the write.)
    if (ra0 != sink) lwr16(s_in + ra0, rv0);
    if (rm0 != sink) lwr16(s_in + rm0, rv0);
    if (ra1 != sink) lwr16(s_in + ra1, rv1);
    if (rm1 != sink) lwr16(s_in + rm1, rv1);
    order();
    in_have = in_req;
    LGS_RING_PH(2);

    // ---- flush finished bytes; the block's last ones once the stream is
    // consumed (snappy.c:337: it must end exactly at want).
    if ((st == 1) & (orem == 0) & (pos >= slen) & (made != want)) st = 0;
    const bool fin = (st == 1) & (orem == 0) & (pos >= slen);
    // Flush whole 128-byte lines of the destination: up to the last line
    // boundary at or below dst + made, so every interior line is written by
    // one job, once (a block's first and last lines are shared with its
    // neighbours), then the tail after the last boundary once the block is
    // finished.  A trip makes <= 128 bytes and F sits on a boundary (or at
    // the block's start, before its first one), so a job is <= 128 bytes
    // and D = made - F < 128 after the flush.
    const uint64_t dpa = reinterpret_cast<uint64_t>(dst);
    const uint64_t lb = (dpa + made) & ~(uint64_t)(kFlush - 1);
    const uint32_t lim = lb > dpa ? (uint32_t)(lb - dpa) : 0u;
    const uint32_t fcnt = lim > F ? lim - F : (fin ? made - F : 0u);
    {
      const bool need = (st == 1) & (fcnt > 0);
      const uint64_t m = ballot(need);
      const uint32_t j = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      const uint32_t total = uni((uint32_t)__builtin_popcountll(m));
      if (need) {
        const uint64_t dp = reinterpret_cast<uint64_t>(dst);
        s_job[j] = RingJob(lane, F, fcnt, dp);
      }
      order();
      // 4 lanes a job, 32 bytes each (bytes 16w.. and 64 + 16w..): 16 jobs
      // per round, so a trip's flush is one round of two LDS round trips
      // (a job record, then the ring) whenever at most 16 blocks flush.
      // (8 lanes a job, 8 jobs a round: 274 against 268 us on C2,
      // profiles/r5e_ab.txt.)
#pragma clang loop unroll(disable)
      for (uint32_t base = 0; base < total; base += 16) {
        const uint32_t jj = base + (lane >> 2), w = lane & 3u;
        // jj < base + 16 <= kJobs: the record is in range (stale past total).
        const RingJob jb = s_job[jj];
        if ((jj < total) & (16 * w < jb.cnt)) {
          const uint8_t* rb = s_out + (jb.lane() & (BL - 1)) * kOutStride + 16 +
                              ((uint32_t)jb.ptr() & 15u);
          const u32x4 v0 = lrd16(rb + ((jb.off + 16 * w) & (kOutRing - 1)));
          const bool two = 64 + 16 * w < jb.cnt;
          u32x4 v1 = v0;
          if (two) v1 = lrd16(rb + ((jb.off + 64 + 16 * w) & (kOutRing - 1)));
          const gptr<uint8_t> g = (gptr<uint8_t>)jb.ptr() + jb.off + 16 * w;
          LGS_RING_FLUSH_ST(g, v0, jb.cnt - 16 * w);
          if (two) LGS_RING_FLUSH_ST(g + 64, v1, jb.cnt - 64 - 16 * w);
        }
      }
      order();
      if (need) F += fcnt;
    }
    LGS_RING_PH(3);

    // ---- parse the next tag.  TWO: then a second op slot -- its piece, if
    // its bytes are in LDS, and the tag after it.
    parse(false);
    LGS_RING_PH(4);
    if (TWO) {
      order();
      piece();
      order();
      parse(true);
    }
    LGS_RING_PH(5);

    // ---- refill requests: the next 64 input bytes, once the 64 they
    // overwrite in the ring are consumed.
    // 4 lanes per request, <= 32 a trip.  (Each lane loading its own
    // block's 64 bytes instead: the same time, profiles/r5f_ab.txt.)
    {
      const uint32_t cons = ((orem > 0) & (okind == 0)) ? olp : pos;
      const bool need = (st == 1) & (in_req < slen) & (in_req <= cons + 64);
      const uint64_t m = ballot(need);
      const uint32_t j = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      const uint32_t total = uni((uint32_t)__builtin_popcountll(m));
      if (need & (j < 32)) {
        const uint64_t sp = reinterpret_cast<uint64_t>(src);
        s_job[j] = RingJob(lane, in_req, slen, sp);
      }
      order();
      ra0 = rm0 = ra1 = rm1 = sink;
      const uint32_t w = lane & 3u;
      if ((lane >> 2) < total) {
        const RingJob jb = s_job[lane >> 2];
        const uint32_t o = jb.off + 16 * w;
        const gptr<const uint8_t> g = (gptr<const uint8_t>)jb.ptr();
        // (A granule past the stream reloads its first: never consumed.)
        rv0 = ld16(g + (o < jb.cnt ? o : 0u));
        const uint32_t r = o & (kInRing - 1);
        ra0 = jb.lane() * kInStride + r;
        rm0 = r < 64 ? ra0 + kInRing : sink;
      }
      if (16 + (lane >> 2) < total) {
        const RingJob jb = s_job[16 + (lane >> 2)];
        const uint32_t o = jb.off + 16 * w;
        const gptr<const uint8_t> g = (gptr<const uint8_t>)jb.ptr();
        rv1 = ld16(g + (o < jb.cnt ? o : 0u));
        const uint32_t r = o & (kInRing - 1);
        ra1 = jb.lane() * kInStride + r;
        rm1 = r < 64 ? ra1 + kInRing : sink;
      }
      order();
      if (need & (j < 32)) in_req += 64;
    }
    LGS_RING_PH(6);
  } while (ballot(st == 1) & ~(ballot(orem == 0) & ballot(pos >= slen) & ballot(F >= made)));

  if (exists) {
    status[i] = (uint8_t)st;
    out_len[i] = LGS_RING_PH_VALUE(lane, LGS_RING_OUT_LEN(st == 1 ? want : 0));
  }
}

hipError_t launch_decode_ring(const DecodeArgs& a, hipStream_t s) {
  // Two op slots per trip, 32 blocks per wave: the rings for 32 lanes take
  // 20 KB of LDS, so eight waves fit a CU, two per SIMD, and each hides the
  // other's memory waits.  (64 blocks per wave: 746 -> 709 GiB/s on C2; one
  // op slot: 632.  Those variants were removed in round 2.)
#ifndef LGS_RING_BL
#define LGS_RING_BL 32
#endif
  hipLaunchKernelGGL((decode_ring_kernel<true, LGS_RING_BL>), dim3((a.n + LGS_RING_BL - 1) / LGS_RING_BL), dim3(64), 0, s, a.in,
                     a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                     a.index, a.n, a.count);
  return hipGetLastError();
}





constexpr uint32_t kDecCap0 = 4608;    // fillseq "4 KiB" blocks (max 4208 B)
constexpr uint32_t kDecCap1 = 16896;   // 16 KiB class
constexpr uint32_t kDecCap2 = 66048;   // 64 KiB class (+ block-builder overshoot)

// Batches of at least this many blocks go to the lane-per-block ring
// kernel, smaller ones to the wave-per-block kernel.  Measured on 4 KiB
// fillseq blocks (tools/sweep_decoders.py, round 2): ring 292 / wave 268 us
// at 32 768 blocks, 316 / 328 at 40 960 (the ring's time is one generation
// of its trips until the chip is full, the wave kernel's grows with the
// batch).  On incompressible blocks the wave kernel wins at every size
// (98 against 163 us at 49 152), but a launch does not know the ratio.
constexpr uint32_t kLaneMinBlocks = 36864;

// ---------------------------------------------------------------------------
// Mixed-size batches.  One launch sized for its largest block runs every
// block in that class's LDS image (a 4 KiB block in a 64 KiB wave: two waves
// per CU) or, in the ring decoder, lets one lane walk a 64 KiB block while
// the rest of the chip idles.  So a batch whose largest block is over the
// smallest class is first sorted into classes on the device, and each class
// runs in its own kernel over its index list; the device-side count ends
// the grid's surplus waves at once.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void classify_kernel(const uint32_t* __restrict__ len,
                                                       uint32_t n, uint32_t b0, uint32_t b1,
                                                       uint32_t b2, uint32_t* __restrict__ list,
                                                       uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const bool here = i < n;
  const uint32_t v = here ? len[i] : 0;
  const uint32_t c = v <= b0 ? 0 : v <= b1 ? 1 : v <= b2 ? 2 : 3;
  const uint32_t lane = lane_id();
  for (uint32_t k = 0; k < 4; ++k) {
    const uint64_t m = __ballot(here && c == k);
    if (m == 0) continue;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&cnt[k], (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (here && c == k) list[(size_t)k * n + base + __popcll(m & ((1ull << lane) - 1))] = i;
  }
}

hipError_t launch_classify(const uint32_t* len, uint32_t n, uint32_t b0, uint32_t b1, uint32_t b2,
                           uint32_t* list, uint32_t* cnt, hipStream_t s) {
  hipLaunchKernelGGL(classify_kernel, dim3((n + 255) / 256), dim3(256), 0, s, len, n, b0, b1, b2,
                     list, cnt);
  return hipGetLastError();
}

// One private pool per device, created on first use and kept: freed
// scratch stays mapped (release threshold 256 MiB), so a split launch does
// not map memory every time.
static hipMemPool_t scratch_pool(int dev, hipError_t* err) {
  static std::mutex mu;
  static hipMemPool_t pools[64] = {};
  std::lock_guard<std::mutex> g(mu);
  if (dev < 0 || dev >= 64) {
    *err = hipErrorInvalidDevice;
    return nullptr;
  }
  if (!pools[dev]) {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t p = nullptr;
    if ((*err = hipMemPoolCreate(&p, &props)) != hipSuccess) return nullptr;
    uint64_t keep = 256ull << 20;
    (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
    pools[dev] = p;
  }
  *err = hipSuccess;
  return pools[dev];
}

Scratch::Scratch(size_t bytes, hipStream_t s) : s_(s) {
  int dev = 0;
  err_ = hipGetDevice(&dev);
  if (err_ != hipSuccess) return;
  hipMemPool_t pool = scratch_pool(dev, &err_);
  if (err_ != hipSuccess) return;
  err_ = hipMallocFromPoolAsync(&p_, bytes, pool, s);
  if (err_ != hipSuccess) p_ = nullptr;
}

#define LGS_TRY(x) do { const hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

// Outputs over the 16 KiB class: the wide decoder (any size; the 64 KiB class
// decoded 70 GiB/s in decode_kernel<66048>, two waves per CU).
template <uint32_t OUT, uint32_t IN>
static hipError_t launch_decode_wide(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((decode_wide_kernel<OUT, IN>), dim3(a.n), dim3(64), 0, s, a.in, a.in_off,
                     a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status, a.index, a.n,
                     a.count);
  return hipGetLastError();
}
// The wide class: the one-tag walk (a probe build can select the trip
// decoder of lgs_decode_probe.hip).
// max_out: the largest capacity the launch may hold (the probe library's
// workgroup decoder takes the 64 KiB class, never larger outputs).
static hipError_t launch_decode_big(const DecodeArgs& a, uint32_t max_out, hipStream_t s) {
  (void)max_out;
#ifdef LGS_PROBE_DECODERS
  if (options().wide.load(std::memory_order_relaxed) == kWideTrips)
    return launch_decode_trips(a, s);
#endif
#ifdef LGS_PROBE_DECODERS
  if (max_out <= kGroupMaxOut && (options().wide.load(std::memory_order_relaxed) == kWideGroup ||
                                  options().decoder.load(std::memory_order_relaxed) == kDecGroup))
    return launch_decode_group(a, max_out, s);
#endif
  return launch_decode_wide<32768, 4096>(a, s);
}
// The 16 KiB class stays in decode_kernel's in-place image (18 KB, eight
// waves per CU): the rings at 8 KiB + 2 KiB (10.4 KB, fourteen waves) were
// slower on C3's 16 KiB classes (fillseq 212 -> 204 GiB/s, random 838 -> 690).
static hipError_t launch_decode_mid(const DecodeArgs& a, hipStream_t s) {
  return launch_decode_cls<kDecCap1, 1>(a, s);
}

static hipError_t launch_decode_split(const DecodeArgs& a, uint32_t max_out, hipStream_t s) {
  const int force = options().decoder.load(std::memory_order_relaxed);
  const size_t list_bytes = (size_t)4 * a.n * sizeof(uint32_t);
  Scratch scratch(list_bytes + 16, s);
  LGS_TRY(scratch.status());
  uint32_t* list = (uint32_t*)scratch.get();
  uint32_t* cnt = (uint32_t*)((uint8_t*)scratch.get() + list_bytes);
  LGS_TRY(hipMemsetAsync(cnt, 0, 16, s));
  LGS_TRY(launch_classify(a.out_cap, a.n, kDecCap0, kDecCap1, kDecCap2, list, cnt, s));
  DecodeArgs c = a;
  c.index = list; c.count = cnt;
#ifdef LGS_PROBE_DECODERS
  if (options().decoder.load(std::memory_order_relaxed) == kDecOps) {
    LGS_TRY(launch_decode_ops(c, s));
  } else
#endif
  LGS_TRY((a.n >= kLaneMinBlocks || force == kDecRing ? launch_decode_ring(c, s)
                                                      : launch_decode_cls<kDecCap0, 1>(c, s)));
  c.index = list + a.n; c.count = cnt + 1;
  LGS_TRY(launch_decode_mid(c, s));
  if (max_out > kDecCap1) {            // (classes above max_out are empty)
    c.index = list + 2 * (size_t)a.n; c.count = cnt + 2;
    LGS_TRY(launch_decode_big(c, kDecCap2, s));
  }
  if (max_out > kDecCap2) {
    c.index = list + 3 * (size_t)a.n; c.count = cnt + 3;
    LGS_TRY(launch_decode_big(c, max_out, s));
  }
  return scratch.release();
}

hipError_t launch_decode(const DecodeArgs& a, uint32_t max_out, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  // (As launch_encode: a by-value item only in a one-item launch.)
  if (a.one.on && (a.n != 1 || a.index)) return hipErrorInvalidValue;
  const int force = options().decoder.load(std::memory_order_relaxed);
#ifdef LGS_PROBE_DECODERS
  if (force == kDecOps && max_out <= kDecCap0) return launch_decode_ops(a, s);
  if (force == kDecQuad) return launch_decode_quad(a, s);
#endif
  if ((force == kDecAuto || force == kDecOps || force == kDecRing) &&
      !a.index && max_out > kDecCap0 && a.n >= kSplitMinBlocks &&
      options().split.load(std::memory_order_relaxed))
    return launch_decode_split(a, max_out, s);
  if (force == kDecRing || (force == kDecAuto && a.n >= kLaneMinBlocks))
    return launch_decode_ring(a, s);
#ifdef LGS_PROBE_DECODERS
  if (force == kDecGroup && max_out <= kGroupMaxOut) return launch_decode_group(a, max_out, s);
  if (force == kDecChain && max_out <= kChainMaxOut) return launch_decode_chain(a, max_out, s);
#endif
  if (max_out <= kDecCap0) return launch_decode_cls<kDecCap0, 1>(a, s);
  if (max_out <= kDecCap1) return launch_decode_mid(a, s);
  return launch_decode_big(a, max_out, s);
}

}  // namespace lgs
