// lgs_encode_group.hip -- batched Snappy encoder, several blocks per wave.
//
// Same algorithm and output as encode_kernel (lgs_encode.hip, which
// documents the exact emulation of lcdb's snappy.c:104-195), restated so
// that one wave64 carries 64/G blocks, each owned by a group of G lanes.
//
// Why: with one block per wave, every per-block decision is a scalar (SALU)
// instruction and the CU has one scalar unit for all its waves -- encode_kernel
// spends ~14 K SALU + 3.4 K branch instructions per 4 KiB block.  Here the
// per-block state lives in VGPRs (uniform inside a group), the decisions are
// VALU instructions issued for all groups at once on the CU's four SIMDs, and
// only the shared control flow stays scalar.
//
// Per group, a literal-search batch holds G probes (probe index pi = G-1-gl,
// gl = lane in group), and a match-extension step compares G bytes.  Groups
// progress independently through a small state machine (SEARCH -> COPY ->
// SEARCH ... -> TAIL -> DONE); each pass over the loop runs one step for
// every group, masked by state.
//
// Items must be single chunks (<= 64 KiB, the launcher checks).
#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {

namespace {

// Probe schedule (snappy.c:138-143); a per-translation-unit copy.
__constant__ ProbeTable kProbeG = ProbeTable();

constexpr uint32_t kSinkG = kTableCap;   // sink slot past the 2048 real entries

enum : uint32_t { ST_SEARCH = 0, ST_COPY = 1, ST_TAIL = 2, ST_DONE = 3 };

template <uint32_t G>
struct Group {
  static constexpr uint64_t kMask = G == 64 ? ~0ull : ((1ull << G) - 1);
  uint32_t gl;      // lane within group
  uint32_t gbase;   // first lane of the group (0, G, 2G, ...)
  __device__ Group() : gl(lane_id() & (G - 1)), gbase(lane_id() & ~(G - 1)) {}
  // This group's slice of a wave ballot; bit gl <-> lane gbase + gl.
  __device__ uint64_t ballot(bool c) const {
    const uint64_t m = __ballot(c);
    return G == 64 ? m : ((m >> gbase) & kMask);
  }
  // Value held by lane `l` of this group.
  __device__ uint32_t from(uint32_t v, uint32_t l) const { return __shfl(v, gbase + l); }
};

}  // namespace

template <uint32_t G, uint32_t IN_CAP>
__global__ __launch_bounds__(64) void encode_group_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
    const uint32_t* __restrict__ index, uint32_t n) {
  constexpr uint32_t NG = 64 / G;
  __shared__ __attribute__((aligned(16))) uint8_t s_in[NG][IN_CAP + 48];
  __shared__ __attribute__((aligned(16))) uint16_t s_tab[NG][kTableCap + 8];
  __shared__ __attribute__((aligned(16))) uint8_t s_lid[NG][kTableCap + 16];

  const Group<G> grp;
  const uint32_t gl = grp.gl;
  const uint32_t pi = G - 1 - gl;                    // probe index in a batch
  const uint32_t g = lane_id() / G;
  const uint32_t slot = blockIdx.x * NG + g;
  const bool live = slot < n;
  const uint32_t item = live ? (index ? index[slot] : slot) : 0;

  const uint32_t len = live ? in_len[item] : 0;
  const gptr<const uint8_t> src = to_global(in) + (live ? in_off[item] : 0);
  const gptr<uint8_t> o = to_global(out) + (live ? out_off[item] : 0);
  uint16_t* const tab = &s_tab[g][0];
  uint8_t* const lid = &s_lid[g][0];

  // ---- stage the block in LDS (G lanes x 16 B per step; keeps src & 15).
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15u);
  {
    gptr<const u32x4> gs = (gptr<const u32x4>)(src - sh);
    u32x4* l = reinterpret_cast<u32x4*>(&s_in[g][0]);
    const uint32_t n16 = live ? (sh + len + 15u) >> 4 : 0;
    for (uint32_t c = gl; c < n16; c += G) l[c] = gs[c];
    if (gl == 0) l[n16] = u32x4{0, 0, 0, 0};
  }
  const uint8_t* const x = &s_in[g][sh];

  // ---- varint32 header (coding.h:140-167).
  uint32_t op = 0;
  {
    const uint32_t hv = len;
    const uint32_t hl = hv < (1u << 7) ? 1 : hv < (1u << 14) ? 2 : hv < (1u << 21) ? 3
                      : hv < (1u << 28) ? 4 : 5;
    if (live && gl < hl) {
      uint32_t b = (hv >> (7 * gl)) & 0x7fu;
      if (gl + 1 < hl) b |= 0x80u;
      o[gl] = (uint8_t)b;
    }
    op = hl;
  }

  // ---- per-block encoder state (group-uniform VGPRs).
  const uint32_t last = len - kMargin;               // snappy.c:106 (len >= 17)
  uint32_t tsize = 256, shift = 24;                  // snappy.c:108-125
  while (tsize < kTableCap && tsize < len) {
    tsize <<= 1;
    --shift;
  }
  uint32_t st = !live ? ST_DONE : (len >= kMinBlock ? ST_SEARCH : ST_TAIL);
  for (uint32_t e = gl; e < tsize; e += G) tab[e] = 0;   // snappy.c:129
  order();

  uint32_t lit = 0, at = 1, ref = 0;                 // snappy.c:110-112
  uint32_t start = 1, k = 0;                         // literal search: origin, probes done
  const uint32_t off0 = kProbeG.off[pi], off1 = kProbeG.off[pi + 1];

  // Literal [from, from+ll) (snappy.c:53-73) at o + op; group-parallel.
  auto emit_lit = [&](bool on, uint32_t from, uint32_t ll) {
    const uint32_t m = ll - 1;
    const uint32_t hl = m < 60 ? 1u : (m < 256 ? 2u : 3u);
    const uint32_t h0 = m < 60 ? (m << 2) : (m < 256 ? 0xf0u : 0xf4u);
    const uint32_t hdr = h0 | ((m & 0xffu) << 8) | ((m >> 8) << 16);
    const uint32_t total = on ? hl + ll : 0;
    const uint64_t more = __ballot(total > 0);
#pragma clang loop unroll(disable)
    for (uint32_t j0 = 0; more && __ballot(j0 < total); j0 += G) {
      const uint32_t j = j0 + gl;
      const uint32_t lb = x[from + (j >= hl && j < total ? j - hl : 0)];
      const uint32_t v = j < hl ? (hdr >> (8 * j)) : lb;
      if (j < total) o[op + j] = (uint8_t)v;
    }
    op += total;
  };

  for (;;) {
    const bool s_search = st == ST_SEARCH, s_copy = st == ST_COPY, s_tail = st == ST_TAIL;
    const uint64_t any_search = __ballot(s_search);
    const uint64_t any_copy = __ballot(s_copy);
    const uint64_t any_tail = __ballot(s_tail);
    if (!(any_search | any_copy | any_tail)) break;

    // ================= literal-search batch (snappy.c:133-154) =================
    if (any_search) {
      uint32_t o0 = off0, o1 = off1;
      bool in_tab = true;
      if (__ballot(s_search & (k != 0))) {                // some group is past probe 63
        const uint32_t kk = k + pi;
        const bool it = kk < kProbeTab;
        const uint32_t kc = it ? kk : kProbeTab - 1;
        const uint32_t t0 = kProbeG.off[kc], t1 = kProbeG.off[kc + 1];
        if (k != 0) {
          o0 = t0;
          o1 = t1;
          in_tab = it;
        }
      }
      const bool valid = s_search & in_tab & (start + o1 <= last);        // snappy.c:143
      const uint32_t nvalid = (uint32_t)__builtin_popcountll(grp.ballot(valid));
      const uint32_t p = valid ? start + o0 : 0;
      const uint32_t xv = lds_ld32(x, p);
      const uint32_t hh = valid ? hash32(xv, shift) : kSinkG;
      const uint32_t ct = tab[hh];                                        // snappy.c:146
      const uint32_t yt = lds_ld32(x, valid ? ct : 0);
      lid[hh] = (uint8_t)pi;
      order();
      const uint32_t w1 = lid[hh];
      const bool loser = valid & (w1 != pi);
      const uint64_t lmask = grp.ballot(loser);
      uint32_t ncut = G, w2 = 0xffu;
      bool exact2 = false;
      if (__ballot(lmask != 0)) {
        const bool disorder1 = grp.ballot(loser & (w1 > pi)) != 0;
        lid[loser ? hh : kSinkG] = (uint8_t)pi;
        order();
        const uint32_t r2 = lid[hh];
        w2 = r2 == w1 ? 0xffu : r2;
        const bool disorder = disorder1 | (grp.ballot(loser & (r2 > pi)) != 0);
        const uint64_t third = grp.ballot(loser & (w2 != pi));
        // earliest loser / third member, as probe indices (bit gl <-> pi = G-1-gl)
        const uint32_t first_loser = lmask ? (G - 1) - (63 - (uint32_t)__builtin_clzll(lmask)) : G;
        const uint32_t first_third = third ? (G - 1) - (63 - (uint32_t)__builtin_clzll(third)) : G;
        if (lmask != 0) {
          if (disorder) {
            ncut = first_loser > 1 ? first_loser : 1;
          } else {
            ncut = first_third;
            exact2 = true;
          }
        }
      }
      const uint32_t nproc = ncut < nvalid ? ncut : nvalid;
      const bool act = pi < nproc;
      const uint32_t src1 = (G - 1) - (w1 & (G - 1));                    // lane of w1's probe
      const uint32_t pfirst = grp.from(p, src1);
      const uint32_t xfirst = grp.from(xv, src1);
      const bool use_first = exact2 & loser;
      const uint32_t cand = use_first ? pfirst : ct;
      const uint32_t yv = use_first ? xfirst : yt;
      const uint64_t mm = grp.ballot(act & (xv == yv));                  // snappy.c:152
      const uint32_t mpi = mm ? (G - 1) - (63 - (uint32_t)__builtin_clzll(mm)) : G;
      const uint32_t ncommit = mm ? mpi + 1 : nproc;
      const bool shadowed = exact2 & !loser & (w2 < ncommit);
      tab[(valid & (pi < ncommit) & !shadowed) ? hh : kSinkG] = (uint16_t)p;   // snappy.c:148
      order();
      // Group outcome (all lanes of a group agree).
      const uint32_t msrc = (G - 1) - (mpi & (G - 1));
      const uint32_t mat = grp.from(p, msrc), mref = grp.from(cand, msrc);
      if (s_search) {
        if (nvalid == 0) {
          st = ST_TAIL;                                                  // first probe past limit
        } else if (mm) {
          at = mat;
          ref = mref;
          st = ST_COPY;
        } else if (nproc < ncut) {
          st = ST_TAIL;                                                  // next probe past limit
        } else {
          k += nproc;
        }
      }
      // Literal before the match (snappy.c:156).
      const bool emit = s_search & (mm != 0);
      emit_lit(emit, lit, at - lit);
    }

    // ================= one copy (snappy.c:158-187) =================
    if (any_copy) {
      uint32_t base = at, r = ref + 4, a2 = at + 4;
      bool ext = s_copy;
#pragma clang loop unroll(disable)
      while (__ballot(ext)) {                                            // snappy.c:163-164
        const uint32_t q = a2 + gl;
        const bool inr = ext & (q < len);
        const uint32_t qa = inr ? q : 0, ra = inr ? r + gl : 0;
        const bool same = inr & (x[ra] == x[qa]);
        const uint64_t diff = grp.ballot(!same);
        if (ext) {
          if (diff) {
            a2 += (uint32_t)__builtin_ctzll(diff);
            ext = false;
          } else {
            a2 += G;
            r += G;
          }
        }
      }
      if (s_copy) at = a2;
      // emit_copy (snappy.c:75-102), group lane b writes byte b.
      {
        const uint32_t dist = base - ref, cl = at - base;
        const uint32_t lo = dist & 0xffu, hi = (dist >> 8) & 0xffu;
        const uint32_t n64 = cl >= 68 ? (cl - 68) / 64 + 1 : 0;
        uint32_t rest = cl - 64 * n64;
        const uint32_t has60 = rest > 64 ? 1u : 0u;
        rest -= 60 * has60;
        const bool c1 = rest < 12 && dist < 2048;
        const uint32_t head = 3 * (n64 + has60);
        const uint32_t total = s_copy ? head + (c1 ? 2u : 3u) : 0;
        const uint32_t last0 = c1 ? (((dist >> 8) << 5) | ((rest - 4) << 2) | 1u)
                                  : (((rest - 1) << 2) | 2u);
#pragma clang loop unroll(disable)
        for (uint32_t b0 = 0; __ballot(b0 < total); b0 += G) {
          const uint32_t b = b0 + gl;
          if (b < total) {
            uint32_t v;
            if (b < head) {
              const uint32_t rr = b % 3;
              const bool is60 = has60 && b >= 3 * n64;
              v = rr == 0 ? (is60 ? 0xeeu : 0xfeu) : (rr == 1 ? lo : hi);
            } else {
              const uint32_t rr = b - head;
              v = rr == 0 ? last0 : (rr == 1 ? lo : hi);
            }
            o[op + b] = (uint8_t)v;
          }
        }
        op += total;
      }
      if (s_copy) lit = at;
      // Post-copy re-probe with lcdb's 64-bit compare (snappy.c:169-186).
      const bool go = s_copy & (at < last);
      const uint64_t w = lds_ld64(x, go ? at - 1 : 0);
      tab[go ? hash32((uint32_t)w, shift) : kSinkG] = (uint16_t)(at - 1);
      order();
      const uint32_t cur = go ? hash32((uint32_t)(w >> 8), shift) : kSinkG;
      const uint32_t nref = tab[cur];
      order();
      tab[cur] = (uint16_t)at;
      order();
      const uint32_t rv = lds_ld32(x, go ? nref : 0);
      if (s_copy) {
        if (!go) {
          st = ST_TAIL;                                                  // snappy.c:169
        } else if ((w >> 8) != (uint64_t)rv) {
          ++at;                                                          // snappy.c:182-185
          start = at;
          k = 0;
          st = ST_SEARCH;
        } else {
          ref = nref;                                                    // immediate re-match
        }
      }
    }

    // ================= tail literal (snappy.c:190-192) =================
    if (any_tail) {
      emit_lit(s_tail & (lit < len), lit, len - lit);
      if (s_tail) st = ST_DONE;
    }
  }

  if (live && gl == 0) out_len[item] = op;
}

template <uint32_t G, uint32_t IN_CAP>
static hipError_t launch_group(const EncodeArgs& a, hipStream_t s) {
  constexpr uint32_t NG = 64 / G;
  const uint32_t grid = (a.n + NG - 1) / NG;
  hipLaunchKernelGGL((encode_group_kernel<G, IN_CAP>), dim3(grid), dim3(64), 0, s, a.in, a.in_off,
                     a.in_len, a.out, a.out_off, a.out_len, a.index, a.n);
  return hipGetLastError();
}

// Group-per-block encode for whole blocks (no varint override) of <= 4608 B.
// Returns hipErrorNotSupported when the batch does not qualify.
hipError_t launch_encode_group(const EncodeArgs& a, uint32_t max_in, uint32_t lanes,
                               hipStream_t s) {
  if (a.hdr != nullptr || max_in > 4608) return hipErrorNotSupported;
  if (lanes == 32) return launch_group<32, 4608>(a, s);
  if (lanes == 16) return launch_group<16, 4608>(a, s);
  if (lanes == 64) return launch_group<64, 4608>(a, s);
  return hipErrorNotSupported;
}

}  // namespace lgs
