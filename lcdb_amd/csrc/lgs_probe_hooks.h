// lgs_probe_hooks.h -- measurement hooks of the codec kernels, one macro per
// site.  The product library defines no LGS_PROBE_* macro, so every hook
// below expands to nothing there; probe builds (tools/mk_variants.sh with
// -DLGS_PROBE_..., never loaded by lcdb or bench.py) turn one family on.
//
//   LGS_PROBE_RING_PHASES  decode_ring_kernel: shader-clock cycles per trip
//                          phase, summed per wave (tools/ring_phases.py)
//   LGS_PROBE_TRIPCOUNT    decode_ring_kernel: trips per wave (ring_trips.py)
//   LGS_PROBE_NOFAR / NOFLUSH  decode_ring_kernel: drop the far-copy loads /
//                          the flush stores (same control flow; traffic
//                          calibration)
#pragma once

#include <stdint.h>

// ---- decode_ring_kernel trip phases --------------------------------------
// RING_PH_DECL at the kernel's start, RING_PH(k) at the end of phase k
// (adds the cycles since the previous stamp to phase k), RING_PH_STORE(
// lane, slot_ok, dst32) at the end: lane k < 8 writes phase k's sum, lane 8
// the trip count, into its block's out_len entry.
#ifdef LGS_PROBE_RING_PHASES
#define LGS_RING_PH_DECL                                   \
  uint32_t ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0};               \
  uint32_t ph_trips_ = 0;                                   \
  uint64_t ph_t_ = __builtin_amdgcn_s_memtime()
#define LGS_RING_PH(k)                                     \
  do {                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();      \
    ph_[k] += (uint32_t)(t_ - ph_t_);                      \
    ph_t_ = t_;                                            \
  } while (0)
#define LGS_RING_PH_TRIP() (++ph_trips_)
#define LGS_RING_PH_VALUE(lane, dflt) lgs_ring_ph_value_(ph_, ph_trips_, (lane), (dflt))
#define LGS_RING_PH_ACTIVE 1
__device__ __forceinline__ uint32_t lgs_ring_ph_value_(const uint32_t* ph, uint32_t trips,
                                                       uint32_t lane, uint32_t dflt) {
  uint32_t v = lane == 8 ? trips : dflt;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) v = lane == k ? ph[k] : v;   // selects, no dynamic index
  return v;
}
#else
#define LGS_RING_PH_DECL do {} while (0)
#define LGS_RING_PH(k) do {} while (0)
#define LGS_RING_PH_TRIP() do {} while (0)
#define LGS_RING_PH_VALUE(lane, dflt) (dflt)
#define LGS_RING_PH_ACTIVE 0
#endif

#ifdef LGS_PROBE_TRIPCOUNT
#define LGS_RING_TRIPS_DECL uint32_t trips_ = 0
#define LGS_RING_TRIP() (++trips_)
#define LGS_RING_OUT_LEN(v) (trips_)
#else
#define LGS_RING_TRIPS_DECL do {} while (0)
#define LGS_RING_TRIP() do {} while (0)
#define LGS_RING_OUT_LEN(v) (v)
#endif

// ---- decode_ring_kernel traffic calibration -----------------
// LGS_RING_FAR_LD16(p): a far copy's 16-byte load; LGS_RING_FLUSH_ST(g, v, c):
// a flush job's store of c (<= 16) bytes.
#ifdef LGS_PROBE_NOFAR
#define LGS_RING_FAR_LD16(p) ((void)(p), u32x4{0, 0, 0, 0})
#else
#define LGS_RING_FAR_LD16(p) ld16(p)
#endif
#ifdef LGS_PROBE_NOFLUSH
// (never true: keeps v live, so the flush's LDS reads stay)
#define LGS_RING_FLUSH_ST(g, v, c) \
  do { if ((v).x == 0x12345678u && (c) == 77777u) st16((g), (v)); } while (0)
#else
#define LGS_RING_FLUSH_ST(g, v, c) \
  do { if ((c) >= 16) st16((g), (v)); else st_exact((g), (v), (c)); } while (0)
#endif

// ---- decode_kernel phases (tools/dec_phases.py) ---------------------------
// Shader-clock stamps of staging, the tag walk and the flush, and the 100 MHz
// real-time clock, stored by lane 0 at STORE_PTR (the tool gives every block
// 32 bytes of spare capacity).  The probe flushes inside the stamped region
// (FLUSH_STMT) and again after it; harmless.
#ifdef LGS_PROBE_DEC_TIMING
#define LGS_DEC_PH_DECL                                                   \
  const uint64_t dtp0_ = __builtin_amdgcn_s_memtime();                    \
  const uint64_t drt0_ = __builtin_amdgcn_s_memrealtime();                \
  uint64_t dtp1_ = dtp0_
#define LGS_DEC_PH_STAGED()                                               \
  do { __builtin_amdgcn_s_waitcnt(0); dtp1_ = __builtin_amdgcn_s_memtime(); } while (0)
#define LGS_DEC_PH_END(FLUSH_STMT, STORE_PTR)                             \
  do {                                                                    \
    __builtin_amdgcn_s_waitcnt(0);                                        \
    const uint64_t tp2_ = __builtin_amdgcn_s_memtime();                   \
    FLUSH_STMT;                                                           \
    __builtin_amdgcn_s_waitcnt(0);                                        \
    const uint64_t tp3_ = __builtin_amdgcn_s_memtime();                   \
    const uint64_t rt3_ = __builtin_amdgcn_s_memrealtime();               \
    if (lane_id() == 0) {                                                 \
      gptr<uint32_t> q_ = (STORE_PTR);                                    \
      q_[0] = (uint32_t)(dtp1_ - dtp0_);                                  \
      q_[1] = (uint32_t)(tp2_ - dtp1_);                                   \
      q_[2] = (uint32_t)(tp3_ - tp2_);                                    \
      q_[3] = (uint32_t)(rt3_ - drt0_);                                   \
    }                                                                     \
  } while (0)
#else
#define LGS_DEC_PH_DECL do {} while (0)
#define LGS_DEC_PH_STAGED() do {} while (0)
#define LGS_DEC_PH_END(FLUSH_STMT, STORE_PTR) do {} while (0)
#endif

// ---- encode_kernel ----------------------------------------------------------
// LGS_PROBE_FORCE_REPLAY: every search batch takes the lane-by-lane replay
// path (checked exact on C2), LGS_ENC_REPLAY(cond, vmask) its condition.
// LGS_PROBE_ENC_TIMING: shader-clock cycles of staging and the parse, stored
// by lane 0 in the last 16 bytes of the block's output slot
// (tools/enc_phases.py).
#ifdef LGS_PROBE_FORCE_REPLAY
#define LGS_ENC_REPLAY(cond, vmask) (vmask)
#else
#define LGS_ENC_REPLAY(cond, vmask) (ballot(cond) & (vmask))
#endif
#ifdef LGS_PROBE_ENC_TIMING
#define LGS_ENC_PH_DECL                                                   \
  const uint64_t etp0_ = __builtin_amdgcn_s_memtime();                    \
  uint64_t etp1_ = etp0_
#define LGS_ENC_PH_STAGED()                                               \
  do { __builtin_amdgcn_s_waitcnt(0); etp1_ = __builtin_amdgcn_s_memtime(); } while (0)
#define LGS_ENC_PH_END(SLOT, LEN)                                         \
  do {                                                                    \
    __builtin_amdgcn_s_waitcnt(0);                                        \
    const uint64_t tp2_ = __builtin_amdgcn_s_memtime();                   \
    if (lane_id() == 0) {                                                 \
      const uint32_t b_ = 32 + (LEN) + (LEN) / 6 - 16;                    \
      (SLOT).put4(0, b_, (uint32_t)(etp1_ - etp0_));                      \
      (SLOT).put4(0, b_ + 4, (uint32_t)(tp2_ - etp1_));                   \
      (SLOT).put4(0, b_ + 8, 0x7e57u);                                    \
    }                                                                     \
  } while (0)
#else
#define LGS_ENC_PH_DECL do {} while (0)
#define LGS_ENC_PH_STAGED() do {} while (0)
#define LGS_ENC_PH_END(SLOT, LEN) do {} while (0)
#endif
