// lgs_decode_probe.hip -- decoders that lost their A/B against the product
// kernels, kept as test and measurement probes.  Compiled only
// into the probe library (lcdb_amd/liblcdb_gpu_snappy_probe.so, built with
// -DLGS_PROBE_DECODERS by lcdb_amd/build.py's build_probe()); the product
// library that lcdb loads has only the ring, wave and wide decoders, and its
// lgs_set_option("decoder", "quad" | "ops") / ("wide", "trips") return
// LGS_EINVAL.  Every kernel here keeps every reject of snappy.c:216-338, and
// tests/test_gpu_probe_decoders.py runs them against the reference.
//   * decode_trips_kernel: the wide class, up to 8 tags per step (C3 fillseq
//     64 KiB 80 against the walk's 129 GiB/s);
//   * decode_quad_kernel: four lanes per block (C2 305 against the ring's
//     285 us);
//   * tag_scan_kernel + op_exec_kernel: the two-pass decoder, op lists in
//     HBM (C2 432-464 us).
#ifndef LGS_PROBE_DECODERS
#error "lgs_decode_probe.hip belongs to the probe library only (-DLGS_PROBE_DECODERS)"
#endif
#include "lgs_device.h"
#include "lgs_decode_common.h"
#include "lgs_launch.h"

namespace lgs {

// ---------------------------------------------------------------------------
// Trip decoder (round 3): decode_wide_kernel's rings, staging and flushes,
// but the walk moves up to G = 8 tags per step ("trip") instead of one.
// C3's fillseq 64 KiB class decoded at ~130 GiB/s in the wide decoder: 1 024
// blocks are 1 024 serial walks, one per SIMD, and each tag cost ~380 cycles
// of one wave's dependent instructions and LDS round trips (3 072 tags per
// block).  A trip:
//   * chain (scalar): from apos, follow the window's parsed tags while each
//     passes its one range test (the same test as the wide walk: a common tag
//     whose snappy.c:263 / :323 bounds hold at its own output offset), up to
//     G tags and the window's end; op k's window lane and output offset go to
//     lane group k (lanes 8k .. 8k+7);
//   * moves (lane groups): op k's bytes i = j, j+8, .. (j = lane & 7), one
//     byte per LDS access, ring-masked, so the writes are exact and never
//     touch a neighbour's bytes;
//   * rounds: a copy whose source reaches into this trip's output (dependent)
//     must read after the ops it depends on have written.  Op k runs in round
//     r_k = the number of dependent ops among 0..k; every round reads, then
//     writes (one wave's LDS accesses execute in issue order).  r_k is larger
//     than every earlier op's round exactly when op k is dependent.
// A tag that fails the test (long literal, overlapping, COPY4 or far copy,
// or a bound) ends the chain; if it is the trip's first, the exact scalar step
// of the wide walk decodes it alone.  By simulation on fillseq 64 KiB blocks
// (G = 8, 64-byte windows): 5.7 tags per trip, 2.0 rounds per trip.
// Measured (profiles/r3s_wide_trips_ab.txt): exact, but C3's fillseq 64 KiB
// class decodes at 80 GiB/s against the walk's 129.  A lone wave per SIMD
// runs ~10 cycles per instruction; the walk spends ~28 instructions per tag,
// a trip ~340 for 5.7 tags (the scalar chain alone ~25 per tag).  Not the
// default; lgs_set_option("wide", "trips") selects it.
// ---------------------------------------------------------------------------
template <uint32_t OUT, uint32_t IN>
__global__ __launch_bounds__(64) void decode_trips_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count) {
  constexpr uint32_t kG = 8;                 // ops per trip (8 lanes each)
  constexpr uint32_t kOut = OUT;             // output ring
  constexpr uint32_t kIn = IN;               // input ring
  constexpr uint32_t kMirror = 80;           // stream bytes kIn.. mirror ring offsets 0..79
  constexpr uint32_t kSink = kOut + kIn + kMirror;   // a dword per lane for unused writes
  constexpr uint32_t kBuf = kSink + 4 * kWave;
  constexpr uint32_t kRefill = kIn / 2;
  constexpr uint32_t kGran = kRefill / 1024;
  constexpr uint32_t kFlushAt = kOut / 4;
  constexpr uint32_t kFar = kOut - kWave;
  static_assert(kFlushAt + 4224 <= kOut && (kGran == 1 || kGran == 2), "ring sizes");
  __shared__ __attribute__((aligned(16))) uint8_t sb[kBuf];
  uint8_t* const ib = sb + kOut;

  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t i = uni(index ? index[slot] : slot);
  const uint32_t lane = lane_id();
  const uint32_t grp = lane >> 3, sub = lane & 7u;
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  const uint32_t slen = uni(in_len[i]);
  const uint64_t doff = uni64(out_off[i]);
  const gptr<uint8_t> dst = to_global(out) + doff;
  const uint8_t* const dgen = out + doff;
  const uint32_t cap = uni(out_cap[i]);
  const uint32_t oshift = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  const gptr<uint8_t> dal = dst - oshift;

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

  uint32_t staged = 0;
  u32x4 pf0 = {0, 0, 0, 0}, pf1 = pf0;
  auto prefetch = [&]() {
    const uint32_t c0 = staged + 16 * lane, c1 = c0 + 1024;
    if (c0 < slen) pf0 = ld16(src + c0);
    if (kGran == 2 && c1 < slen) pf1 = ld16(src + c1);
  };
  auto land = [&]() {
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

  uint32_t made = 0, F = 0;
  auto flush = [&](uint32_t to) {
    const uint32_t g0 = (F + oshift) >> 4, g1 = (to + oshift + 15) >> 4;
    for (uint32_t g = g0 + lane; g < g1; g += kWave) {
      const uint32_t lo = 16 * g, hi = lo + 16;
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
  while (st == 1 && apos < aend) {                            // snappy.c:208
    const uint32_t w = apos;
    const uint32_t wend = aend - w < kWave ? aend : w + kWave;
    while (staged < aend && staged <= w + kRefill) land();
    if (made - F >= kFlushAt) flush(((made + oshift) & ~15u) - oshift);
    uint32_t flo, frng, fsrc, fpk;
    {
      const uint32_t q = w + lane;
      const uint32_t t = lds_ld32(ib, q & (kIn - 1));
      const uint32_t tag = t & 0xffu, kind = tag & 3u, m0 = tag >> 2;
      const bool lit = kind == 0;
      const uint32_t len = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;     // snappy.c:216, 276, 289
      const uint32_t dist = kind == 1 ? ((tag & 0xe0u) << 3) | ((t >> 8) & 0xffu)
                                      : (t >> 8) & 0xffffu;          // snappy.c:279, 292
      const uint32_t step = lit ? len + 1 : kind + 1;
      const int32_t hi = (int32_t)want - (int32_t)len;
      const uint32_t lo = lit ? 0u : dist;
      const bool common = (lit ? m0 < 60 : (kind != 3) & (dist >= len) & (dist != 0) &
                                           (dist <= kFar)) & (step <= aend - q);
      const bool fast = common & (hi >= (int32_t)lo);
      flo = fast ? lo : 0xffffffffu;
      frng = fast ? (uint32_t)(hi - (int32_t)lo) : 0u;
      // A literal's first stream position; a copy's source less its output offset.
      fsrc = lit ? q + 1 : 0u - dist;
      fpk = len | (step << 8) | (lit ? 0u : 0x10000u);
    }
    do {
      // ---- chain: up to kG tags from apos, each passing its range test.
      uint32_t nops = 0, m = made, maxlen = 0;
      uint32_t my_d = 0, my_m = 0;
      while (nops < kG && apos < wend) {
        const uint32_t d = apos - w;
        const uint32_t rlo = __builtin_amdgcn_readlane(flo, d);
        const uint32_t rrng = __builtin_amdgcn_readlane(frng, d);
        if (m - rlo > rrng) break;
        const uint32_t pk = __builtin_amdgcn_readlane(fpk, d);
        if (grp == nops) {
          my_d = d;
          my_m = m;
        }
        const uint32_t ln = pk & 0xffu;
        maxlen = ln > maxlen ? ln : maxlen;
        m += ln;
        apos += (pk >> 8) & 0xffu;
        ++nops;
      }
      if (nops > 0) {
        // ---- the trip's moves, in rounds.
        const bool act = grp < nops;
        const uint32_t opk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(my_d << 2), (int)fpk);
        const uint32_t os = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(my_d << 2), (int)fsrc);
        const uint32_t L = act ? (opk & 0xffu) : 0u;
        const bool lit = (opk >> 16) == 0;
        const uint32_t s0 = lit ? os : my_m + os + oshift;     // ring coordinate of byte 0
        const uint32_t smask = lit ? kIn - 1 : kOut - 1;
        const uint32_t sbase = lit ? kOut : 0u;
        const uint32_t d0 = my_m + oshift;
        const bool dep = act & !lit & (my_m + os + L > made);   // source reaches into this trip
        const uint64_t db = ballot(dep);
        const uint64_t upto = grp == 7 ? ~0ull : ((1ull << (8 * grp + 8)) - 1ull);
        const uint32_t rnd = (uint32_t)__builtin_popcountll(db & upto) >> 3;
        const uint32_t nr = ((uint32_t)__builtin_popcountll(db) >> 3) + 1;
        const uint32_t T = (maxlen + 7) >> 3;
        // Byte slot t of this lane: op byte sub + 8t.  Reads are harmless
        // anywhere in the rings (ring-masked), so only writes are steered:
        // bytes outside this round's ops go to the lane's own sink dword.
        uint32_t ra[8], wa[8];
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) {
          ra[t] = sbase + ((s0 + sub + 8 * t) & smask);
          wa[t] = (d0 + sub + 8 * t) & (kOut - 1);
        }
        const uint32_t sink = kSink + 4 * lane;
        const uint32_t lb = lds_addr(sb);
        for (uint32_t r = 0; r < nr; ++r) {
          const bool go = rnd == r;
          // Reads of slots 0-3 always, 4-7 when an op is longer than 32
          // bytes; one wait; then the writes.  (Written as C++ with per-slot
          // conditions, hipcc put an lgkmcnt(0) before every read.)
          uint32_t v0, v1, v2, v3, v4 = 0, v5 = 0, v6 = 0, v7 = 0;
          asm volatile(
              "ds_read_u8 %0, %4\n\tds_read_u8 %1, %5\n\t"
              "ds_read_u8 %2, %6\n\tds_read_u8 %3, %7"
              : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
              : "v"(lb + ra[0]), "v"(lb + ra[1]), "v"(lb + ra[2]), "v"(lb + ra[3])
              : "memory");
          if (T > 4)
            asm volatile(
                "ds_read_u8 %0, %4\n\tds_read_u8 %1, %5\n\t"
                "ds_read_u8 %2, %6\n\tds_read_u8 %3, %7"
                : "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
                : "v"(lb + ra[4]), "v"(lb + ra[5]), "v"(lb + ra[6]), "v"(lb + ra[7])
                : "memory");
          uint32_t w[8];
#pragma unroll
          for (uint32_t t = 0; t < 8; ++t) w[t] = lb + ((go & (sub + 8 * t < L)) ? wa[t] : sink);
          asm volatile(
              "s_waitcnt lgkmcnt(0)\n\t"
              "ds_write_b8 %0, %4\n\tds_write_b8 %1, %5\n\t"
              "ds_write_b8 %2, %6\n\tds_write_b8 %3, %7"
              :
              : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(v0), "v"(v1), "v"(v2), "v"(v3)
              : "memory");
          if (T > 4)
            asm volatile(
                "ds_write_b8 %0, %4\n\tds_write_b8 %1, %5\n\t"
                "ds_write_b8 %2, %6\n\tds_write_b8 %3, %7"
                :
                : "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(v4), "v"(v5), "v"(v6), "v"(v7)
                : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        made = m;
        continue;
      }
      // ---- the exact tag step of snappy.c:210-324 for one tag.
      const uint64_t tv = uni64(lds_ld64(ib, apos & (kIn - 1)));
      const uint32_t tg = (uint32_t)tv & 0xffu, kd = tg & 3u;
      const uint32_t hi = (uint32_t)(tv >> 8), left = aend - apos;
      bool bad = false;
      uint32_t x = 0, ds = 0, nb = 0, adv = 0;
      if (kd == 0) {                                // literal, snappy.c:210-273
        uint32_t mm = tg >> 2, hl = 1;
        if (mm >= 60) {
          const uint32_t extra = mm - 59;
          bad = left - 1 < extra;
          mm = extra == 4 ? hi : (hi & ((1u << (8 * (extra & 3u))) - 1u));
          hl += extra;
        }
        nb = mm + 1;
        bad = bad || mm >= 0x7fffffffu || nb > left - hl || nb > want - made;   // :258, :263
        x = apos + hl;
        adv = hl + nb;
      } else {                                      // copies, snappy.c:276-324
        const uint32_t chl = kd == 1 ? 2u : (kd == 2 ? 3u : 5u);
        nb = kd == 1 ? 4 + ((tg >> 2) & 7u) : 1 + (tg >> 2);
        ds = kd == 1 ? ((tg & 0xe0u) << 3) | (hi & 0xffu) : (kd == 2 ? hi & 0xffffu : hi);
        bad = left < chl || ds == 0 || ds >= 0x80000000u || made < ds || nb > want - made;
        adv = chl;
      }
      if (bad) {
        st = 0;
        break;
      }
      const uint32_t u0 = made + oshift;
      if (kd == 0 && nb <= kWave) {
        uint32_t v = 0;
        if (lane < nb) v = ib[(x + lane) & (kIn - 1)];
        order();
        if (lane < nb) sb[(u0 + lane) & (kOut - 1)] = (uint8_t)v;
        order();
      } else if (kd == 0) {
        // A long literal, as in decode_wide_kernel.
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
        if (x + nb > staged) {
          __builtin_amdgcn_s_waitcnt(0x0f70);
          staged = (x + nb) & ~15u;
          prefetch();
        }
      } else if (ds > kFar) {
        // Beyond the ring: the flushed output, once its stores have drained.
        __builtin_amdgcn_s_waitcnt(0x0f70);                       // vmcnt(0)
        uint8_t v = 0;
        if (lane < nb) v = gl_byte(dgen + made - ds + lane);
        if (lane < nb) sb[(u0 + lane) & (kOut - 1)] = v;
        order();
      } else {
        // dist < len repeats the dist-byte pattern (snappy.c:329-330).
        uint32_t v = 0;
        if (lane < nb) v = sb[(u0 - ds + (ds >= nb ? lane : lane % ds)) & (kOut - 1)];
        order();
        if (lane < nb) sb[(u0 + lane) & (kOut - 1)] = (uint8_t)v;
        order();
      }
      made += nb;
      apos += adv;
    } while (apos < wend);
  }
  order();
  if (st == 1 && made != want) st = 0;                        // snappy.c:337
  if (st == 1) flush(want);
  if (lane == 0) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

hipError_t launch_decode_trips(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((decode_trips_kernel<32768, 4096>), dim3(a.n), dim3(64), 0, s, a.in,
                     a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                     a.index, a.n, a.count);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Quad decoder: four lanes per block, up to four consecutive ops per trip.
//
// The ring decoder above is bound by its per-wave instruction stream: one
// lane walks each block, so a wave's life is ~110 trips of ~560 dependent
// instructions whatever the lane count (profiles/r3e_ringprobe.txt: dropping
// every flush store and far-copy load moves it by < 5 %).  Here the four
// lanes of a DPP quad own one block (16 blocks per wave, 16 waves per CU
// for C2) and a trip takes the block's next ops as far as four tags, 128
// output bytes, the landed input and one far copy go:
//   * parse: the quad's lanes walk the four tags together (identical work on
//     each lane, no cross-lane traffic); lane g keeps tag g.  Every reject
//     of snappy.c:216-338 is checked in the reference's order (parse_tag).
//   * a copy whose source lies inside the trip's last literal reads that
//     literal's bytes from the input ring (no dependency on this trip's
//     writes); a copy reading other bytes this trip writes waits a round
//     (all lower slots written first; ~6 % of trips need one).
//   * every round reads all of its sources before it writes (reads-first),
//     and writes exactly the op's bytes (16-byte chunks + an 8/4/2/1 tail),
//     so ops of one round never clobber each other or the near window.
//   * a far copy (beyond the 240-byte near window) is the trip's one load:
//     the quad fetches its <= 64 bytes from the flushed output, 16 a lane,
//     and they land at the start of the next trip; later ops of the trip go
//     on unless they read them.
//   * flushes and refills are the quad's own 16-byte lanes: 64 contiguous
//     bytes per instruction per block, no job records.
// So a block takes ~50 trips instead of ~110, each of a similar number of
// instructions for four times as many lanes of useful work.
// ---------------------------------------------------------------------------
namespace quad {
constexpr uint32_t kIR = 128, kIS = 208;     // input ring; stride (ring + 64 mirror + 16 sink)
constexpr uint32_t kOR = 256, kOS = 352;     // output ring; stride (16 pad + ring + 64 mirror + 16 sink)
constexpr uint32_t kNear = 240;               // ring minus one 16-byte granule of slack
constexpr uint32_t kBudget = 128;             // output bytes per block and trip
constexpr uint32_t kBW = 16;                  // blocks per wave
}  // namespace quad

// Exact-size LDS writes of the first t < 16 bytes of v at p (8/4/2/1-byte
// pieces; lanes that skip a piece aim it at their sink).
__device__ __forceinline__ void lds_tail(uint8_t* p, u32x4 v, uint32_t t, uint8_t* sink) {
  typedef uint64_t u64_a1 __attribute__((aligned(1)));
  typedef uint32_t u32_a1 __attribute__((aligned(1)));
  typedef uint16_t u16_a1 __attribute__((aligned(1)));
  uint8_t* q = p;
  *(u64_a1*)((t & 8) ? q : sink) = ((uint64_t)v.y << 32) | v.x;
  if (t & 8) v = u32x4{v.z, v.w, 0, 0};
  q += t & 8;
  *(u32_a1*)((t & 4) ? q : sink) = v.x;
  if (t & 4) v.x = v.y;
  q += t & 4;
  *(u16_a1*)((t & 2) ? q : sink) = (uint16_t)v.x;
  if (t & 2) v.x >>= 16;
  q += t & 2;
  *((t & 1) ? q : sink) = (uint8_t)v.x;
}

// Write n <= 64 bytes (c0..c3 = bytes 0..63) at output position at of a
// quad lane's output ring ob: whole 16-byte chunks, then the exact tail,
// each also into the mirror (ring offsets < 64) or the pre-pad (pieces that
// wrap past 256) so any read of <= 64 bytes at a ring offset is linear.
__device__ __forceinline__ void qo_put(uint8_t* ob, uint32_t at, uint32_t n, u32x4 c0, u32x4 c1,
                                       u32x4 c2, u32x4 c3, uint8_t* sink) {
  using namespace quad;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const u32x4 v = k == 0 ? c0 : (k == 1 ? c1 : (k == 2 ? c2 : c3));
    const uint32_t r = (at + 16 * k) & (kOR - 1);
    if (16 * k + 16 <= n) {
      lwr16(ob + r, v);
      if (r - 64 > 176u) lwr16(ob + (int32_t)r + (r < 64 ? 256 : -256), v);
    } else if (16 * k < n) {
      const uint32_t t = n - 16 * k;
      lds_tail(ob + r, v, t, sink);
      // the mirror copy of the tail: ring offsets < 64 also at +256, a tail
      // running past 256 also at -256 (the pre-pad holds offsets -16..-1)
      const bool mir = (r < 64) | (r + t > kOR);
      lds_tail(mir ? ob + (int32_t)r + (r < 64 ? 256 : -256) : sink, v, mir ? t : 0u, sink);
    }
  }
}

// Bytes [b0, b1) of the 16-byte value v to p + b0 .. p + b1 - 1 (global),
// one byte store each (inline asm: see st_exact).
__device__ __forceinline__ void st_range(gptr<uint8_t> p, u32x4 v, uint32_t b0, uint32_t b1) {
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t byte = byte_of(v, b);
    asm volatile("global_store_byte %0, %1, off\n\ts_nop 1" ::"v"(p + b), "v"(byte) : "memory");
  }
}

// 16 bytes at stream position p of a quad's input ring (linear through the
// mirror for reads of <= 64 bytes).
__device__ __forceinline__ u32x4 qi_get(const uint8_t* ib, uint32_t p) {
  return lrd16(ib + (p & (quad::kIR - 1)));
}

// A 16-byte ring write of the lanes with `on`, plus its mirror copy (ring
// offsets < 64 also at +256, a write running past 256 also at -256), so
// reads of <= 64 bytes at any ring offset are linear.  Exec-masked, not
// aimed at a sink: an LDS store costs by the lanes it moves, and sink
// stores doubled the quad decoder's LDS traffic (419 against 315 us on C2).
__device__ __forceinline__ void qo_put16(uint8_t* ob, uint32_t at, u32x4 v, bool on, uint8_t*) {
  const uint32_t r = at & (quad::kOR - 1);
  if (on) {
    lwr16(ob + r, v);
    if (r - 64 > 176u) lwr16(ob + (int32_t)r + (r < 64 ? 256 : -256), v);   // r < 64 or r > 240
  }
}

// The trip's independent ops (round one): every source chunk was read
// before any write (reads-first), so ops of one round never read each
// other's bytes.  Chunks 3, 2, 1 are written whole even past the op's end
// (their spill lies inside the next op's first 16 bytes, or past the trip's
// output), then every op's first 16 bytes exactly (a whole chunk, or the
// 8/4/2/1-byte pieces of an op under 16 bytes), which rewrites any spill.
// Spill past the trip's end only touches output not yet made and, in the
// ring, bytes older than the 240-byte near window.
__device__ __forceinline__ void qo_put_round1(uint8_t* ob, uint32_t at, uint32_t n, bool on,
                                              u32x4 c0, u32x4 c1, u32x4 c2, u32x4 c3,
                                              uint8_t* sink) {
  using namespace quad;
  if (ballot(on & (n > 48))) qo_put16(ob, at + 48, c3, on & (n > 48), sink);
  if (ballot(on & (n > 32))) qo_put16(ob, at + 32, c2, on & (n > 32), sink);
  if (ballot(on & (n > 16))) qo_put16(ob, at + 16, c1, on & (n > 16), sink);
  qo_put16(ob, at, c0, on & (n >= 16), sink);
  const bool sh = on & (n < 16);
  if (sh) {
    const uint32_t r = at & (kOR - 1);
    lds_tail(ob + r, c0, n, sink);
    if ((r < 64) | (r + n > kOR)) lds_tail(ob + (int32_t)r + (r < 64 ? 256 : -256), c0, n, sink);
  }
}

__global__ __launch_bounds__(64) void decode_quad_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n,
    const uint32_t* __restrict__ count) {
  using namespace quad;
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kBW * kIS];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kBW * kOS];

  const uint32_t lane = threadIdx.x;
  const uint32_t qb = lane >> 2, g = lane & 3u;      // block in the wave, slot in the quad
  const uint32_t qs = lane & ~3u;                    // the quad's first lane
  const uint32_t slot = blockIdx.x * kBW + qb;
  if (count) n = *count;
  if (blockIdx.x * kBW >= n) return;                // a whole wave without blocks
  const bool exists = slot < n;
  const uint32_t i = exists ? (index ? index[slot] : slot) : 0;
  const gptr<const uint8_t> src = to_global(in) + (exists ? in_off[i] : 0);
  const uint32_t slen = exists ? in_len[i] : 0;
  const gptr<uint8_t> dst = to_global(out) + (exists ? out_off[i] : 0);
  const uint32_t cap = exists ? out_cap[i] : 0;
  uint8_t* const ib = s_in + qb * kIS;
  uint8_t* const ob = s_out + qb * kOS + 16;
  uint8_t* const isink = ib + kIR + 64;             // 16 bytes per lane quad: harmless writes
  uint8_t* const osink = ob + kOR + 64;

  // varint32 header, coding.h:169-204.  st: 1 decoding/ok, 0 corrupt, 2 no
  // space, 3 no block.
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

  // Prologue: the stream's first 128 bytes (two 16-byte granules a lane).
  uint32_t in_req = 0, in_have = 0;
  {
    u32x4 a = {0, 0, 0, 0}, b = a;
    const uint32_t o0 = 16 * g, o1 = 64 + 16 * g;
    if ((st == 1) & (o0 < slen)) a = ld16(src + o0);
    if ((st == 1) & (o1 < slen)) b = ld16(src + o1);
    __builtin_amdgcn_s_waitcnt(0x0f70);                         // vmcnt(0)
    lwr16(ib + o0, a);
    lwr16(ib + o1, b);
    lwr16(ib + kIR + o0, a);                                    // mirror of offsets 0..63
    order();
    in_req = in_have = st == 1 ? (slen < kIR ? slen : kIR) : 0u;
  }

  uint32_t pos = hlen;               // next tag (stream offset)
  uint32_t made = 0, F = 0;          // output produced / flushed
  uint32_t orem = 0, olp = 0;        // a long literal's bytes left / their stream position
  // The far copy in flight (in the lane whose slot took it): its output
  // position and length, and its <= 64 bytes.
  uint32_t fat = 0, flen = 0;
  u32x4 fv0 = {0, 0, 0, 0}, fv1 = fv0, fv2 = fv0, fv3 = fv0;
  // Refills in flight: up to two 16-byte granules a lane and their ring
  // offsets (the sink when none).
  u32x4 rv0 = fv0, rv1 = fv0;
  uint8_t *ra0 = isink, *ra1 = isink, *rm0 = isink, *rm1 = isink;
  const uint64_t dpa = reinterpret_cast<uint64_t>(dst);
  const uint32_t dsh = (uint32_t)(dpa & 15u);

#ifndef LGS_PROBE_QUAD_TOP_REFILL
#define LGS_PROBE_QUAD_TOP_REFILL 0
#endif
  // The refill requests (below: at the end of the trip).  Probe builds
  // (the round-3 silent corruption): LGS_PROBE_QUAD_TOP_REFILL=1
  // issues them at the top of the trip, after the landing and after in_have
  // takes the landed requests; =2 issues them there but before in_have is
  // updated, so in_have also counts the requests just issued.
  auto refill = [&]() {
    const uint32_t cons = orem > 0 ? olp : pos;
    const bool q0 = (st == 1) & (in_req < slen) & (in_req <= cons + 64);
    const uint32_t o0 = in_req + 16 * g;
    if (q0 & (o0 < slen)) rv0 = ld16(src + o0);
    ra0 = q0 ? ib + (o0 & (kIR - 1)) : isink;
    rm0 = (q0 & ((o0 & (kIR - 1)) < 64)) ? ib + kIR + (o0 & (kIR - 1)) : isink;
    in_req = q0 ? in_req + 64 : in_req;
    const bool q1 = q0 & (in_req < slen) & (in_req <= cons + 64);
    const uint32_t o1 = in_req + 16 * g;
    if (q1 & (o1 < slen)) rv1 = ld16(src + o1);
    ra1 = q1 ? ib + (o1 & (kIR - 1)) : isink;
    rm1 = (q1 & ((o1 & (kIR - 1)) < 64)) ? ib + kIR + (o1 & (kIR - 1)) : isink;
    in_req = q1 ? in_req + 64 : in_req;
  };
  for (;;) {
    // ---- everything issued last trip has landed: the far copy's bytes (the
    // trip's last op: nothing past it is written yet, so whole chunks), then
    // the refills.
    __builtin_amdgcn_s_waitcnt(0x0f70);                         // vmcnt(0)
    if (flen > 0) {
      qo_put16(ob, fat, fv0, true, osink);
      qo_put16(ob, fat + 16, fv1, flen > 16, osink);
      qo_put16(ob, fat + 32, fv2, flen > 32, osink);
      qo_put16(ob, fat + 48, fv3, flen > 48, osink);
      flen = 0;
    }
    if (ra0 != isink) lwr16(ra0, rv0);
    if (rm0 != isink) lwr16(rm0, rv0);
    if (ra1 != isink) lwr16(ra1, rv1);
    if (rm1 != isink) lwr16(rm1, rv1);
    ra0 = ra1 = rm0 = rm1 = isink;
#if LGS_PROBE_QUAD_TOP_REFILL == 2
    refill();
#endif
    in_have = in_req;
    order();
#if LGS_PROBE_QUAD_TOP_REFILL == 1
    refill();
#ifdef LGS_PROBE_QUAD_REFILL_SYNC
    __builtin_amdgcn_s_waitcnt(0x0f70);   // probe: the refills complete here
#endif
#endif

    // ---- flush: whole 64-byte segments of the destination up to made, the
    // block's tail once its stream is consumed (snappy.c:337: it must end
    // exactly at want).
    if ((st == 1) & (orem == 0) & (pos >= slen) & (made != want)) st = 0;
    const bool fin = (st == 1) & (orem == 0) & (pos >= slen);
    // Output flushed by earlier trips: their stores were waited for at the
    // top of this trip, so loads (of other lanes) see it.  A far copy must
    // read only such bytes (this trip's flush stores are still in flight).
    const uint32_t F0 = F;
    {
      const uint64_t lb = (dpa + made) & ~(uint64_t)63;
      const uint32_t lim = lb > dpa ? (uint32_t)(lb - dpa) : 0u;
      const uint32_t T = (st != 1) ? F : (fin ? made : (lim > F ? lim : F));
      if (ballot(T > F)) {
        const uint32_t g0 = (F + dsh) >> 4, g1 = (T + dsh + 15) >> 4;
        const gptr<uint8_t> A = dst - dsh;                       // 16-byte aligned
#pragma clang loop unroll(disable)
        for (uint32_t j = g0 + g; ballot(j < g1); j += 4) {
          if (j < g1) {
            const uint32_t lo = 16 * j - dsh;                    // output position
            const u32x4 v = lrd16(ob + (lo & (kOR - 1)));
            if ((16 * j >= F + dsh) & (16 * j + 16 <= T + dsh)) {
              st16(A + 16 * j, v);
            } else {
              // the block's first or last granule: only bytes [F, T)
              const uint32_t b0 = F + dsh > 16 * j ? F + dsh - 16 * j : 0u;
              const uint32_t b1 = T + dsh < 16 * j + 16 ? T + dsh - 16 * j : 16u;
              st_range(A + 16 * j, v, b0, b1);
            }
          }
        }
      }
      F = T;
    }
    const bool active = (st == 1) & !(fin & (F >= made));
    if (ballot(active) == 0) break;

    // ---- parse: up to four tags.  The quad's lanes first walk the tag
    // chain together (identical work on every lane, each tag's length and
    // step only, snappy.c:210-317's header forms), lane g keeping tag g's
    // bytes and start; then each lane checks its own tag in full (every
    // reject of snappy.c:216-338, in the reference's order) and the quad
    // takes the longest prefix of slots that pass -- at most one far copy or
    // long literal, as its last.
    uint32_t my_n = 0, my_src = 0, my_at = 0, my_kind = 0, my_dist = 0;
    // kinds: 0 input ring (a literal, or a copy of the previous slot's
    // literal), 1 output ring, 2 far (global), 3 overlapping copy (dist < n)
    bool my_dep = false, my_far = false;
    const uint32_t made0 = made;
    if (ballot(active & (orem > 0))) {
      // a long literal's next piece, in slot 0 only
      const uint32_t pc = orem < 64 ? orem : 64u;
      const bool go = active & (orem > 0) & (olp + pc <= in_have);
      if (go & (g == 0)) {
        my_n = pc;
        my_src = olp;
        my_at = made;
      }
      made = go ? made + pc : made;
      olp = go ? olp + pc : olp;
      orem = go ? orem - pc : orem;
    }
    if (ballot(active & (orem == 0) & (pos < slen))) {
      const bool live = active & (orem == 0) & (pos < slen) & (made == made0);
      uint32_t p = pos, m = made;
      uint32_t my_p = p, my_m = m, my_lo = 0, my_b4 = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        // bytes p .. p+4 from two aligned dwords of the ring (offset p & 127;
        // the mirror keeps them linear)
        const uint32_t r = p & (kIR - 1);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(ib + (r & ~3u));
        const uint32_t w0 = w[0], w1 = w[1];
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, r & 3u);
        const uint32_t b4 = __builtin_amdgcn_alignbyte(0u, w1, r & 3u);   // byte 4 in bits 0..7
        my_p = g == k ? p : my_p;
        my_m = g == k ? m : my_m;
        my_lo = g == k ? lo : my_lo;
        my_b4 = g == k ? b4 : my_b4;
        const uint32_t tag = lo & 0xffu, kind = tag & 3u, m0 = tag >> 2;
        const uint32_t extra = m0 >= 60 ? m0 - 59 : 0u;
        const uint32_t b1 = (lo >> 8) | (b4 << 24);
        const uint32_t emask = extra >= 4 ? 0xffffffffu : (1u << (8 * (extra & 3u))) - 1u;
        const uint32_t llen = (extra ? (b1 & emask) : m0) + 1;
        const uint32_t clen = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;
        const bool lit = kind == 0;
        p += lit ? 1 + extra + llen : (kind == 3 ? 5u : kind + 1);
        m += lit ? llen : clen;
      }
      // this lane's tag, in full (snappy.c:210-324): header form, length,
      // distance, and the rejects
      const uint32_t tag = my_lo & 0xffu, kind = tag & 3u, m0 = tag >> 2;
      const bool lit = kind == 0;
      const uint32_t extra = (lit & (m0 >= 60)) ? m0 - 59 : 0u;
      const uint32_t b1 = (my_lo >> 8) | (my_b4 << 24);
      const uint32_t emask = extra >= 4 ? 0xffffffffu : (1u << (8 * (extra & 3u))) - 1u;
      const uint32_t mval = extra ? (b1 & emask) : m0;                 // literal length - 1
      const uint32_t len = lit ? mval + 1 : (kind == 1 ? 4 + (m0 & 7u) : m0 + 1);
      const uint32_t hl = lit ? 1 + extra : (kind == 3 ? 5u : kind + 1);
      const uint32_t dist = kind == 1 ? ((tag & 0xe0u) << 3) | (b1 & 0xffu)
                                      : (kind == 2 ? b1 & 0xffffu : b1);
      const uint32_t left = slen - my_p;
      // :240-256 / :276-317 header in the stream; :263 / :323 length within
      // want; :258 literal length; :263 literal bytes in the stream; :320 /
      // :323 0 < dist <= made (dist - 1 >= made also covers dist >= 2^31).
      const bool bad = (hl > left) | (len > want - my_m) |
                       (lit ? (mval >= 0x7fffffffu) | (hl + len > left) : (dist - 1 >= my_m));
      const bool hdr = live & (my_p < slen) & (in_have >= (left < 5 ? slen : my_p + 5));
      const bool longl = lit & (len > 64);
      const uint32_t pc = longl ? 64u : len;
      const uint32_t lp = my_p + hl;                           // a literal's first byte
      const uint32_t cs = my_m - dist;                         // a copy's first source byte
#ifdef LGS_PROBE_QUAD_OLD_NEAR
      // Round 3's rule: the near window grew with the slot's
      // offset in the trip, which admits 256 < dist <= 368 as ring reads --
      // a slot an earlier op of the same trip has already overwritten.
      const bool far = !lit & (dist > kNear + (my_m - made0));
#else
      // Near = in the 256-byte ring and not overwritten by this trip: a
      // constant bound below the ring size, as in the ring decoder.
      const bool far = !lit & (dist > kNear);
#endif
      const bool ok = hdr & !bad & (!lit | (lp + pc <= in_have)) & (!far | (cs + len <= F0)) &
                      ((g == 0) | (my_m + pc - made0 <= kBudget)) & !(longl & (g > 0));
      // the longest prefix of passing slots, none after a far copy or a long
      // literal (quad nibbles of wave ballots)
      const uint32_t low = (1u << g) - 1u;
      const uint32_t okm = (uint32_t)(ballot(ok) >> qs) & 0xfu;
      const uint32_t stopm = (uint32_t)(ballot(ok & (far | longl)) >> qs) & 0xfu;
      const bool prefix = ((okm & low) == low) & ((stopm & low) == 0);
      const bool take = ok & prefix;
      // the first slot that does not pass, with its header in: a reject
      if ((uint32_t)(ballot(prefix & !ok & hdr & bad) >> qs) & 0xfu) st = 0;
      const uint32_t nt = (uint32_t)__builtin_popcount((uint32_t)(ballot(take) >> qs) & 0xfu);
      // a copy that reads the previous slot's literal reads its bytes from
      // the input ring (no dependency on this trip's writes)
      const uint32_t pm = __builtin_amdgcn_mov_dpp(my_m, 0x90, 0xf, 0xf, false);    // quad_perm [0,0,1,2]
      const uint32_t ppc = __builtin_amdgcn_mov_dpp(pc, 0x90, 0xf, 0xf, false);
      const uint32_t plp = __builtin_amdgcn_mov_dpp(lp, 0x90, 0xf, 0xf, false);
      const uint32_t plit = __builtin_amdgcn_mov_dpp((uint32_t)lit, 0x90, 0xf, 0xf, false);
      const bool remap = !lit & (g > 0) & (plit != 0) & (cs >= pm) & (cs + len <= pm + ppc);
      const bool ovl = !lit & (dist < len);
      my_n = take ? pc : my_n;
      my_at = take ? my_m : my_at;
      my_dist = take ? dist : my_dist;
      my_far = take & far;
      my_kind = take ? (lit ? 0u : (far ? 2u : (remap ? 0u : (ovl ? 3u : 1u)))) : my_kind;
      my_src = take ? (lit ? lp : (remap ? plp + (cs - pm) : cs)) : my_src;
      // reads bytes this trip writes (or a period that is not 1/2/4/8):
      // after every lower slot, with exact writes
      const bool pat = ovl & (dist <= 8) & ((dist & (dist - 1)) == 0);
      my_dep = take & !lit & !far & !remap &
               ((cs + (ovl ? dist : len) > made0) | (ovl & !pat));
      // the block's new position and output: the end of the last taken
      // slot's tag and op (a long literal: after its first piece; the rest
      // continues next trip from olp)
      const uint32_t nxt = my_p + hl + (lit ? len : 0u), mend = my_m + pc;
      const uint32_t n0 = __builtin_amdgcn_mov_dpp(nxt, 0x00, 0xf, 0xf, false);   // quad_perm [0,0,0,0]
      const uint32_t n1 = __builtin_amdgcn_mov_dpp(nxt, 0x55, 0xf, 0xf, false);   // [1,1,1,1]
      const uint32_t n2 = __builtin_amdgcn_mov_dpp(nxt, 0xaa, 0xf, 0xf, false);   // [2,2,2,2]
      const uint32_t n3 = __builtin_amdgcn_mov_dpp(nxt, 0xff, 0xf, 0xf, false);   // [3,3,3,3]
      const uint32_t e0 = __builtin_amdgcn_mov_dpp(mend, 0x00, 0xf, 0xf, false);
      const uint32_t e1 = __builtin_amdgcn_mov_dpp(mend, 0x55, 0xf, 0xf, false);
      const uint32_t e2 = __builtin_amdgcn_mov_dpp(mend, 0xaa, 0xf, 0xf, false);
      const uint32_t e3 = __builtin_amdgcn_mov_dpp(mend, 0xff, 0xf, 0xf, false);
      const uint32_t l0 = __builtin_amdgcn_mov_dpp(len, 0x00, 0xf, 0xf, false);
      const uint32_t lp0 = __builtin_amdgcn_mov_dpp(lp, 0x00, 0xf, 0xf, false);
      const bool long0 = (uint32_t)(ballot(take & longl) >> qs) & 1u;
      const uint32_t nq = nt > 2 ? (nt > 3 ? n3 : n2) : (nt > 1 ? n1 : n0);
      const uint32_t eq = nt > 2 ? (nt > 3 ? e3 : e2) : (nt > 1 ? e1 : e0);
      pos = nt ? nq : pos;
      made = nt ? eq : made;
      orem = long0 ? l0 - 64 : orem;
      olp = long0 ? lp0 + 64 : olp;
    }

    // ---- the far copy's bytes from output flushed by earlier trips (F0),
    // issued now, landed at the start of the next trip.
    if (ballot(my_far)) {
      const gptr<const uint8_t> fp = (gptr<const uint8_t>)(dst + (my_far ? my_src : 0u));
#ifdef LGS_PROBE_QUAD_FAR_WAIT
      __builtin_amdgcn_s_waitcnt(0x0f70);    // probe: nothing in flight before them
#endif
      if (my_far) {
#ifdef LGS_PROBE_QUAD_FARBYPASS
        // probe: agent-scope dword loads (never served from the CU's L1)
        auto gl4 = [&](gptr<const uint8_t> q) {
          const uintptr_t a = reinterpret_cast<uintptr_t>(q);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
          const uint32_t sh8 = 8 * (uint32_t)(a & 3u);
          uint32_t d[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) d[k] = __hip_atomic_load(w + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          u32x4 v;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            v[k] = sh8 ? (d[k] >> sh8) | (d[k + 1] << (32 - sh8)) : d[k];
          return v;
        };
        fv0 = gl4(fp);
        fv1 = gl4(fp + 16);
        fv2 = gl4(fp + 32);
        fv3 = gl4(fp + 48);
#else
        fv0 = ld16(fp);
        fv1 = ld16(fp + 16);
        fv2 = ld16(fp + 32);
        fv3 = ld16(fp + 48);
#endif
      }
      fat = my_far ? my_at : fat;
      flen = my_far ? my_n : 0u;
    }

    // ---- move the bytes, in rounds: an op that reads bytes this trip writes
    // (or copies with a period other than 1/2/4/8) starts a new round, so a
    // slot's round is the number of such ops at or before it.  In a round
    // every source is read before any write; writes may spill up to 15
    // bytes past an op's end, into later ops of the same or a later round
    // (rewritten after) or past the trip's output (not made yet; in the ring,
    // older than the 240-byte near window) -- see qo_put_round1.
    {
      const bool mv = (my_n > 0) & !my_far;
      const uint32_t depm = (uint32_t)(ballot(mv & my_dep) >> qs) & 0xfu;
      const uint32_t rnd = (uint32_t)__builtin_popcount(depm & ((2u << g) - 1u));
      const bool pat = (my_kind == 3u) & (my_dist <= 8) & ((my_dist & (my_dist - 1)) == 0);
      const bool slow = (my_kind == 3u) & !pat;
#pragma clang loop unroll(disable)
      for (uint32_t r = 0; ballot(mv & (rnd >= r)); ++r) {
        const bool on = mv & (rnd == r);
        u32x4 c0, c1 = {0, 0, 0, 0}, c2 = c1, c3 = c1;
        const uint8_t* sp = my_kind == 0u ? ib + (my_src & (kIR - 1)) : ob + (my_src & (kOR - 1));
        // period 1/2/4/8 (snappy.c:329-330): the dist bytes before my_at repeat
        const uint32_t d = my_dist;
        const u32x4 s0 = lrd16(pat ? ob + ((my_at - d) & (kOR - 1)) : sp);
        const uint32_t b0 = s0.x & 0xffu, h0 = s0.x & 0xffffu;
        const uint32_t px = d == 1 ? b0 * 0x01010101u : (d == 2 ? h0 | (h0 << 16) : s0.x);
        const uint32_t py = d == 8 ? s0.y : px;
        c0 = pat ? u32x4{px, py, px, py} : s0;
        if (ballot(on & !pat & (my_n > 16))) c1 = lrd16(sp + 16);
        if (ballot(on & !pat & (my_n > 32))) c2 = lrd16(sp + 32);
        if (ballot(on & !pat & (my_n > 48))) c3 = lrd16(sp + 48);
        c1 = pat ? c0 : c1;
        c2 = pat ? c0 : c2;
        c3 = pat ? c0 : c3;
        order();
        qo_put_round1(ob, my_at, my_n, on & !slow, c0, c1, c2, c3, osink);
        order();
        if (ballot(on & slow)) {
          // other periods (dist < n, not 1/2/4/8): byte by byte, the
          // reference's forward loop (never in fillseq)
          if (on & slow) {
#pragma clang loop unroll(disable)
            for (uint32_t b = 0; b < my_n; ++b) {
              const uint8_t v = ob[(my_at + b - my_dist) & (kOR - 1)];
              order();
              const uint32_t rr = (my_at + b) & (kOR - 1);
              ob[rr] = v;
              if (rr < 64) ob[rr + kOR] = v;
              order();
            }
          }
          order();
        }
      }
    }

    // ---- refills: the next 64 stream bytes once the 64 they overwrite in
    // the ring are consumed; up to two a trip, landed at the top of the next.
    // (Issued at the top of the trip instead, from the trip's start
    // position, they decoded C2 wrongly -- an unexplained failure, see
    // DESIGN.md 4.2 -- and were slower: 312 against 305 us.)
#if LGS_PROBE_QUAD_TOP_REFILL
    (void)0;   // issued at the top of the trip instead (probe)
#else
    refill();
#endif
  }

  if (exists & (g == 0)) {
    status[i] = (uint8_t)st;
    out_len[i] = st == 1 ? want : 0;
  }
}

hipError_t launch_decode_quad(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(decode_quad_kernel, dim3((a.n + quad::kBW - 1) / quad::kBW), dim3(64), 0, s,
                     a.in, a.in_off, a.in_len, a.out, a.out_off, a.out_cap, a.out_len, a.status,
                     a.index, a.n, a.count);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Two-pass decoder (round 3): large batches of small blocks (outputs of the
// 4 608-byte class; C2, C4).
//
// The ring decoder's time is one wave's serial stream of walk *and* byte
// moves (~340 instructions per tag step at ~10 cycles each).
// Here the two are split over two kernels with the op list in HBM between:
//
//   pass 1, tag_scan_kernel: one lane per block walks the block's tags
//     (snappy.c:208-324, every reject in the reference's order) and writes
//     one 4-byte record per op.  The walk reads its stream from a 512-byte
//     LDS ring per lane that LDS-DMA loads (global_load_lds) fill one
//     256-byte segment ahead, so a step waits on LDS, never on HBM; the
//     walk moves no output byte, so a step is ~50 instructions.
//   pass 2, op_exec_kernel: one wave per block executes the block's records
//     64 at a time in an LDS image of the output: every literal at once
//     (16 bytes a lane, read from the stream in HBM), then every copy whose
//     source holds no byte of an earlier copy of the batch at once, then the
//     remaining copies in order; the image is written out whole.
//
// Record (bit 31 = copy): a literal is (len - 1) << 17 | its first byte's
// stream offset; a copy 1 << 31 | (len - 1) << 17 | distance.  Output
// offsets are the running sum of the lengths (pass 2 scans them).  A block
// with more than kK ops (average op under 4.5 bytes: only synthetic
// streams) is decoded by pass 2 from its stream alone (decode_stream), as is
// one whose stream is too long for the 17-bit offsets.
// ---------------------------------------------------------------------------
namespace ops {
constexpr uint32_t kSeg = 256;        // stream bytes per ring segment; two per lane
constexpr uint32_t kK = 1024;         // records per block
constexpr uint32_t kOut = 4608;       // output class
constexpr uint32_t kMaxStream = 131072 - 64;   // literal offsets fit 17 bits
constexpr uint32_t kExec = 1u << 30, kSelf = 2u << 30;   // pass-2 states (meta.x top bits)
#ifndef LGS_OPS_BL
#define LGS_OPS_BL 64
#endif
constexpr uint32_t kBL = LGS_OPS_BL;  // blocks (lanes) per pass-1 wave
}  // namespace ops

// LDS-DMA: 16 bytes per active lane from gaddr to LDS byte address
// lds_base + 16 * lane (global_load_lds_dwordx4).  Inline asm, so hipcc
// neither counts it nor waits for it: the pass-1 walk tracks it itself.
__device__ __forceinline__ void glds16(uint64_t gaddr, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep) : "v"(gaddr), "s"(lds_base) : "memory");
}

// s_waitcnt immediate for vmcnt(n) (gfx9: bits 3:0 and 15:14; lgkmcnt and
// expcnt left at their maximum, i.e. not waited for).
constexpr int vmcnt_imm(int n) { return 0x0f70 | (n & 15) | ((n >> 4) << 14); }

// Wave-wide inclusive prefix sum / max (DPP: rows of 16, then the row
// broadcasts of gfx9).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return x;
}
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = umax(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
// Value of x in the lane below (0 in lane 0): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}

template <uint32_t BL>
__global__ __launch_bounds__(64) void tag_scan_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n, const uint32_t* __restrict__ count,
    uint32_t* __restrict__ rec, uint2* __restrict__ meta) {
  using namespace ops;
  // Half h of lane j's ring: s_ring[(h * BL + j) * kSeg ..].  Segment s (of
  // the stream's 16-byte-aligned view) lives in half s & 1.
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[2 * BL * kSeg];
  const uint32_t lane = threadIdx.x;
  if (count) n = uni(*count);
  if (blockIdx.x * BL >= n) return;
  const uint32_t slot = blockIdx.x * BL + lane;
  const bool exists = (lane < BL) & (slot < n);
  const uint32_t i = exists ? (index ? index[slot] : slot) : 0;
  const uint64_t sp = reinterpret_cast<uint64_t>(in) + (exists ? in_off[i] : 0);
  const uint32_t slen = exists ? in_len[i] : 0;
  const uint32_t cap = exists ? out_cap[i] : 0;
  // Stream byte p is byte u = p + sh of the aligned view starting at gb.
  const uint32_t sh = (uint32_t)sp & 15u;
  const uint64_t gb = sp - sh;
  const uint32_t lastg = slen ? (sh + slen - 1) >> 4 : 0;   // last granule holding a byte
  const uint32_t ring0 = lds_addr(s_ring);
  const uint8_t* const mine = s_ring + (lane < BL ? lane : 0) * kSeg;

  // Vector-memory instructions issued (LDS-DMA and record stores: vmcnt
  // counts both); every one below jret has completed.  jh0 / jh1: index of
  // the last DMA into this lane's half 0 / 1.
  uint32_t J = 0, jret = 0;
  int32_t jh0 = -1, jh1 = -1;
  // DMA of segment seg (per lane) for the lanes in m: one instruction per
  // lane, 16 lanes x 16 bytes, granules clamped to the stream's last.
  auto issue = [&](uint64_t m, uint32_t seg) {
    for (; m; m &= m - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      const uint32_t sj = lane_val(seg, j), lj = lane_val(lastg, j);
      const uint64_t gj = ((uint64_t)lane_val((uint32_t)(gb >> 32), j) << 32) |
                          lane_val((uint32_t)gb, j);
      if (lane < 16) {
        const uint32_t g = 16 * sj + lane;
        glds16(gj + 16ull * (g < lj ? g : lj), ring0 + ((sj & 1) * BL + j) * kSeg);
      }
      const bool me = lane == j;
      jh0 = (me & !(sj & 1)) ? (int32_t)J : jh0;
      jh1 = (me & (sj & 1)) ? (int32_t)J : jh1;
      ++J;
    }
  };
  // Bytes u .. u+4 of the lane's view from its ring (two aligned dwords):
  // x = bytes u..u+3, y's low byte = byte u+4.
  auto rd = [&](uint32_t u, uint32_t* x, uint32_t* y) {
    const uint32_t d0 = u & ~3u, d1 = d0 + 4;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(mine + ((d0 >> 8) & 1) * BL * kSeg + (d0 & 255));
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(mine + ((d1 >> 8) & 1) * BL * kSeg + (d1 & 255));
    *x = __builtin_amdgcn_alignbyte(w1, w0, u & 3u);
    *y = w1 >> (8 * (u & 3u));
  };

  issue(ballot(exists), 0u);
  issue(ballot(exists & (lastg >= 16)), 1u);
  __builtin_amdgcn_s_waitcnt(0x0f70);                       // vmcnt(0)
  jret = J;

  // varint32 header, coding.h:169-204.  st: 1 walking/ok, 0 corrupt,
  // 2 no space, 3 no block, 4 decoded by pass 2 from the stream.
  uint32_t st = exists ? 1u : 3u, want = 0, hlen = 0;
  {
    uint32_t x, y;
    rd(sh, &x, &y);
    for (uint32_t k = 0; k < 5; ++k) {
      const uint32_t b = ((k < 4 ? x >> (8 * k) : y)) & 0xffu;
      if (k < slen && hlen == 0) {
        want |= (b & 0x7fu) << (7 * k);
        if ((b & 0x80u) == 0) hlen = k + 1;
      }
    }
    if (exists) {
      if (hlen == 0 || want > 0x7fffffffu) st = 0;              // snappy.c:405-409
      else if (want > cap) st = 2;
      else if (slen > kMaxStream) st = 4;
    }
  }

  uint32_t pos = hlen, made = 0, k = 0, segl = 0;
  u32x4 rb = {0, 0, 0, 0};                                    // four records, then one store
  gptr<u32x4> const rq = (gptr<u32x4>)(to_global(rec) + (size_t)slot * kK);
  for (;;) {
    const bool act = (st == 1) & (pos < slen);                // snappy.c:208
    if (!ballot(act)) break;
    const uint32_t u = pos + sh, s = u >> 8;
    // Leaving segment segl: load segment s + 1 into the half just left
    // (after a long literal: segments s and s + 1).
    const bool adv = act & (s != segl);
    if (ballot(adv)) {
      const bool jump = s > segl + 1;
      const uint32_t sa = jump ? s : s + 1;
      issue(ballot(adv & (16 * sa <= lastg)), sa);
      issue(ballot(adv & jump & (16 * (s + 1) <= lastg)), s + 1);
      segl = adv ? s : segl;
    }
    // Keep at most 40 in flight, so everything issued before J - 40 has
    // landed; wait further only for a half whose DMA may still be in flight.
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(40));
    jret = J > 40 ? (J - 40 > jret ? J - 40 : jret) : jret;
    const uint32_t e = ((u & ~3u) + 7) >> 8;
    const int32_t ja = (s & 1) ? jh1 : jh0, jb = (e & 1) ? jh1 : jh0;
    const int32_t jn = ja > jb ? ja : jb;
    const bool pend = act & (jn >= (int32_t)jret);
    if (ballot(pend)) {
      int32_t top = -1;
      for (uint64_t m = ballot(pend); m; m &= m - 1) {
        const int32_t v = (int32_t)lane_val((uint32_t)jn, (uint32_t)__builtin_ctzll(m));
        top = v > top ? v : top;
      }
      const uint32_t allow = J - 1 - (uint32_t)top;           // newer instructions that may stay
      if (allow >= 16) {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(16));
        jret = J - 16;
      } else if (allow >= 4) {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(4));
        jret = J - 4;
      } else {
        __builtin_amdgcn_s_waitcnt(0x0f70);                   // vmcnt(0)
        jret = J;
      }
    }
    // The tag (snappy.c:210-324; parse_tag's folded rejects).
    uint32_t x, y;
    rd(u, &x, &y);
    const uint32_t tag = x & 0xffu, kind = tag & 3u, m0 = tag >> 2;
    const uint32_t left = slen - pos;
    const uint32_t b1 = (x >> 8) | (y << 24);                   // bytes 1..4
    const bool lit = kind == 0;
    const uint32_t extra = m0 >= 60 ? m0 - 59 : 0u;
    const uint32_t emask = extra >= 4 ? 0xffffffffu : (1u << (8 * (extra & 3u))) - 1u;
    const uint32_t m = extra ? (b1 & emask) : m0;
    const uint32_t clen = kind == 1 ? 4 + (m0 & 7u) : m0 + 1;
    const uint32_t cdist = kind == 1 ? ((tag & 0xe0u) << 3) | (b1 & 0xffu)
                                     : (kind == 2 ? b1 & 0xffffu : b1);
    const uint32_t len = lit ? m + 1 : clen;
    const uint32_t hl = lit ? 1 + extra : (kind == 3 ? 5u : kind + 1);
    const bool bad = (hl > left) | (len > want - made) |
                     (lit ? (m >= 0x7fffffffu) | (hl + len > left) : (cdist - 1 >= made));
    const bool take = act & !bad & (k < kK);
    st = (act & bad) ? 0u : st;
    st = (act & !bad & (k >= kK)) ? 4u : st;
    const uint32_t r = lit ? ((len - 1) << 17) | (pos + hl)
                           : 0x80000000u | ((len - 1) << 17) | cdist;
    const uint32_t q = k & 3u;
    rb.x = (take & (q == 0)) ? r : rb.x;
    rb.y = (take & (q == 1)) ? r : rb.y;
    rb.z = (take & (q == 2)) ? r : rb.z;
    rb.w = (take & (q == 3)) ? r : rb.w;
    const bool full = take & (q == 3);
    if (ballot(full)) {
      if (full) rq[k >> 2] = rb;
      ++J;
    }
    k += take ? 1u : 0u;
    made += take ? len : 0u;
    pos += take ? hl + (lit ? len : 0u) : 0u;
  }
  if ((st == 1) & (made != want)) st = 0;                        // snappy.c:337
  const bool part = (st == 1) & ((k & 3u) != 0);
  if (part) rq[k >> 2] = rb;
  if (exists) {
    if (st == 1) {
      meta[slot] = uint2{kExec | k, want};
    } else if (st == 4) {
      meta[slot] = uint2{kSelf, 0};
    } else {
      meta[slot] = uint2{0, 0};
      status[i] = (uint8_t)st;
      out_len[i] = 0;
    }
  }
}

// Exact-size LDS writes of the first t < 16 bytes of v at p (exec-masked).
__device__ __forceinline__ void lds_exact(uint8_t* p, u32x4 v, uint32_t t) {
  typedef uint64_t u64_a1 __attribute__((aligned(1)));
  typedef uint32_t u32_a1 __attribute__((aligned(1)));
  typedef uint16_t u16_a1 __attribute__((aligned(1)));
  if (t & 8) {
    *(u64_a1*)p = ((uint64_t)v.y << 32) | v.x;
    v = u32x4{v.z, v.w, 0, 0};
    p += 8;
  }
  if (t & 4) {
    *(u32_a1*)p = v.x;
    v.x = v.y;
    p += 4;
  }
  if (t & 2) {
    *(u16_a1*)p = (uint16_t)v.x;
    v.x >>= 16;
    p += 2;
  }
  if (t & 1) *p = (uint8_t)v.x;
}

// Up to 64 bytes (c0..c3) at p: whole 16-byte pieces, then the exact tail.
__device__ __forceinline__ void lds_put64(uint8_t* p, uint32_t n, bool on, u32x4 c0, u32x4 c1,
                                          u32x4 c2, u32x4 c3) {
  if (on & (n >= 16)) lwr16(p, c0);
  if (on & (n >= 32)) lwr16(p + 16, c1);
  if (on & (n >= 48)) lwr16(p + 32, c2);
  if (on & (n >= 64)) lwr16(p + 48, c3);
  const uint32_t t = n >> 4;
  const u32x4 ct = t == 0 ? c0 : (t == 1 ? c1 : (t == 2 ? c2 : c3));
  if (on & ((n & 15u) != 0)) lds_exact(p + 16 * t, ct, n & 15u);
}

template <uint32_t OUT>
__global__ __launch_bounds__(64) void op_exec_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    const uint32_t* __restrict__ index, uint32_t n, const uint32_t* __restrict__ count,
    const uint32_t* __restrict__ rec, const uint2* __restrict__ meta) {
  using namespace ops;
  // The output image at its destination's alignment, + 64 bytes so that
  // 64-byte source reads at any offset stay inside.
  __shared__ __attribute__((aligned(16))) uint8_t s_img[OUT + 16 + 80];
  const uint32_t slot = blockIdx.x;
  if (slot >= (count ? uni(*count) : n)) return;
  const uint32_t mx = uni(meta[slot].x), want = uni(meta[slot].y);
  const uint32_t state = mx & 0xc0000000u, nops = mx & 0x3fffffffu;
  if (state == 0) return;                                  // pass 1 wrote its status
  const uint32_t i = uni(index ? index[slot] : slot);
  const uint32_t lane = lane_id();
  const gptr<uint8_t> dst = to_global(out) + uni64(out_off[i]);
  uint8_t* const o = s_img + ((uint32_t)reinterpret_cast<uintptr_t>(dst) & 15u);
  const gptr<const uint8_t> src = to_global(in) + uni64(in_off[i]);
  if (state == kSelf) {
    const uint32_t slen = uni(in_len[i]);
    const uint32_t cap = uni(out_cap[i] < OUT ? out_cap[i] : OUT);
    uint32_t w = 0;
    const uint32_t st = decode_stream(GlobalStream{src, slen}, slen, o, cap, &w);
    order();
    if (st == 1) flush_out(dst, s_img, w);
    if (lane == 0) {
      status[i] = (uint8_t)st;
      out_len[i] = st == 1 ? w : 0;
    }
    return;
  }
  const gptr<const uint32_t> rp = to_global(rec) + (size_t)slot * kK;
  uint32_t carry = 0;
  for (uint32_t b = 0; b < nops; b += kWave) {
    const bool valid = b + lane < nops;
    const uint32_t r = valid ? rp[b + lane] : 0u;
    const bool isc = valid & (r >> 31 != 0);
    const uint32_t len = valid ? ((r >> 17) & 0x3fffu) + 1 : 0u;
    const uint32_t x = r & 0x1ffffu;                       // literal: stream offset; copy: distance
    const uint32_t incl = wave_incl_sum(len);
    const uint32_t d = carry + incl - len;                 // output offset
    carry += lane_val(incl, kWave - 1);

    // 1. literals of <= 64 bytes, one per lane: five 16-byte loads in flight
    //    (clamped to the literal's first piece when past it), then writes.
    const bool lit = valid & !isc;
    const bool sl = lit & (len <= 64);
    {
      const uint32_t a = sl ? x : 0u, ln = sl ? len : 0u;
      const u32x4 c0 = ld16(src + a);
      const u32x4 c1 = ld16(src + a + (ln > 16 ? 16u : 0u));
      const u32x4 c2 = ld16(src + a + (ln > 32 ? 32u : 0u));
      const u32x4 c3 = ld16(src + a + (ln > 48 ? 48u : 0u));
      lds_put64(o + d, len, sl, c0, c1, c2, c3);
    }
    // 2. longer literals: the whole wave on one at a time.
    for (uint64_t big = ballot(lit & (len > 64)); big; big &= big - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(big);
      const uint32_t bx = lane_val(x, l), bl = lane_val(len, l), bd = lane_val(d, l);
      for (uint32_t t = 16 * lane; ballot(t < bl); t += 16 * kWave) {
        const u32x4 v = ld16(src + bx + (t < bl ? t : 0u));
        if (t + 16 <= bl) lwr16(o + bd + t, v);
        else if (t < bl) lds_exact(o + bd + t, v, bl - t);
      }
    }
    order();
    // 3. copies (snappy.c:326-331).  Parallel: those whose source starts at
    //    or after the end of the batch's previous copy, or ends before its
    //    first, and does not overlap the copy's own output -- no earlier
    //    copy of the batch writes a byte they read.
    const uint32_t pm = wave_shr1(wave_incl_max(isc ? d + len : 0u));
    const uint64_t cm = ballot(isc);
    const uint32_t first = cm ? lane_val(d, (uint32_t)__builtin_ctzll(cm)) : 0u;
    const uint32_t s0 = d - x;
    const bool indep = isc & (x >= len) & ((s0 >= pm) | (s0 + len <= first));
    if (ballot(indep)) {
      const uint32_t a = indep ? s0 : 0u;
      const u32x4 c0 = lrd16(o + a), c1 = lrd16(o + a + 16), c2 = lrd16(o + a + 32),
                  c3 = lrd16(o + a + 48);
      lds_put64(o + d, len, indep, c0, c1, c2, c3);
    }
    order();
    //    The rest in order, a byte per lane (an overlapping copy repeats its
    //    dist-byte pattern: the reference's forward byte loop).
    for (uint64_t dm = ballot(isc & !indep); dm; dm &= dm - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(dm);
      const uint32_t cd = lane_val(d, l), cl = lane_val(len, l), cx = lane_val(x, l);
      uint32_t from = cd - cx + lane;
      if (cx < cl) from = cd - cx + lane % cx;
      if (lane < cl) o[cd + lane] = o[from];
      order();
    }
  }
  order();
  flush_out(dst, s_img, want);
  if (lane == 0) {
    status[i] = 1;
    out_len[i] = want;
  }
}

hipError_t launch_decode_ops(const DecodeArgs& a, hipStream_t s) {
  using namespace ops;
  const size_t rec_bytes = (size_t)a.n * kK * sizeof(uint32_t);
  Scratch scratch(rec_bytes + (size_t)a.n * sizeof(uint2), s);
  hipError_t e = scratch.status();
  if (e != hipSuccess) return e;
  uint32_t* rec = (uint32_t*)scratch.get();
  uint2* meta = (uint2*)((uint8_t*)scratch.get() + rec_bytes);
  hipLaunchKernelGGL((tag_scan_kernel<kBL>), dim3((a.n + kBL - 1) / kBL), dim3(64), 0, s, a.in,
                     a.in_off, a.in_len, a.out_cap, a.out_len, a.status, a.index, a.n, a.count,
                     rec, meta);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((op_exec_kernel<kOut>), dim3(a.n), dim3(64), 0, s, a.in, a.in_off, a.in_len,
                     a.out, a.out_off, a.out_cap, a.out_len, a.status, a.index, a.n, a.count,
                     rec, meta);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return scratch.release();
}

}  // namespace lgs
