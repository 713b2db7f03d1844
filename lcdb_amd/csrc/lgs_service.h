// lgs_service.h -- device side of the drop-in service (lgs_launch.h): the
// mailbox protocol shared by encode_service_kernel (lgs_encode.hip) and
// decode_service_kernel (lgs_decode.hip).
//
// Every access to a mailbox is a system-scope vector memory operation
// (global_load/store ... sc0 sc1, buffer_inv / buffer_wbl2): the mailboxes
// live in fine-grained pinned host memory that the host writes and polls.
// A request's input is read from the slot's arena (the same pinned memory),
// after the system-scope acquire of the request word: round 5 staged inputs
// in host-written fine-grained VRAM instead, and a wave read a request's
// bytes torn with its predecessor's (GPUTEST_r05: a valid stream rejected)
// -- host writes through the BAR land in HBM through the HDP, which nothing
// on this path flushes, while the request word arrives through host memory.
#pragma once

#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {

// One poll: {req, len} (one 8-byte atomic load, so a request's length is
// never torn from its number), the stop flag, the arena and the kernel's
// closing mark, each by its own lane in one instruction.
struct SvcPoll {
  uint32_t req, len, stop, closing;
  uint64_t arena;
};
__device__ __forceinline__ SvcPoll svc_poll(SvcMailbox* m, SvcControl* ctl) {
  const uint32_t lane = lane_id();
  uint64_t v = 0;
  if (lane < 4) {
    // +0 {req,len}, +8 {aux,stop}, +16 arena; lane 3: the closing mark.
    uint64_t* p = lane < 3 ? reinterpret_cast<uint64_t*>(m) + lane : &ctl->closing;
    v = __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  // (readlane returns int: each word goes through uint32_t, or the arena's
  // low word would be sign-extended into its high one.)
  SvcPoll r;
  r.req = (uint32_t)__builtin_amdgcn_readlane(lo, 0);
  r.len = (uint32_t)__builtin_amdgcn_readlane(hi, 0);
  r.stop = (uint32_t)__builtin_amdgcn_readlane(hi, 1);
  const uint32_t alo = (uint32_t)__builtin_amdgcn_readlane(lo, 2);
  const uint32_t ahi = (uint32_t)__builtin_amdgcn_readlane(hi, 2);
  r.arena = ((uint64_t)ahi << 32) | alo;
  r.closing = (uint32_t)__builtin_amdgcn_readlane(lo, 3);
  return r;
}

// Completion: the result words, then (release, system scope: every output
// store of the wave is performed first) the acknowledged sequence number.
__device__ __forceinline__ void svc_finish(SvcMailbox* m, uint32_t req, uint32_t status,
                                           uint32_t out_len) {
  __builtin_amdgcn_s_waitcnt(0);                        // every lane's output stores
  if (lane_id() == 0) {
    __hip_atomic_store(&m->status, status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&m->out_len, out_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(&m->ack, req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void svc_touch(SvcControl* ctl, uint64_t t) {
  if (lane_id() == 0)
    __hip_atomic_store(&ctl->activity, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The wave's loop: serve(len, input, arena, &status, &out_len) for every new
// request of mailbox m (input at arena + kSvcIn).
//
// Exit is collective: a wave that has seen no request anywhere in
// its kernel for `idle` ticks of the 100 MHz clock (ctl->activity, stamped
// when a request is picked up and when it is answered) sets ctl->closing,
// and every wave leaves at its next poll -- before taking a new request, so
// no wave outlives the others while requests wait on a wave that has gone.
// The host relaunches a kernel it finds finished (hipEventQuery) and clears
// the mark first; the new waves serve whatever is pending.
template <class Serve>
__device__ __forceinline__ void svc_loop(SvcMailbox* m, uint64_t idle, SvcControl* ctl,
                                         const Serve& serve) {
  uint32_t done =
      uni(__hip_atomic_load(&m->ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  svc_touch(ctl, last);
  for (;;) {
    const SvcPoll q = svc_poll(m, ctl);
    if (q.stop || q.closing) break;
    if (q.req != done && q.arena != 0) {
      svc_touch(ctl, __builtin_amdgcn_s_memrealtime());
      uint32_t status = 0, out_len = 0;
      serve(q.len, q.arena + kSvcIn, q.arena, &status, &out_len);
      svc_finish(m, q.req, status, out_len);
      done = q.req;
      last = __builtin_amdgcn_s_memrealtime();
      svc_touch(ctl, last);
      continue;
    }
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    // (Signed: another wave may have stamped activity after this one read
    // the clock.)
    if ((int64_t)(now - last) > (int64_t)idle) {
      const uint64_t a = uni64(__hip_atomic_load(&ctl->activity, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT));
      if ((int64_t)(now - a) > (int64_t)idle) {
        if (lane_id() == 0)
          __hip_atomic_store(&ctl->closing, (uint64_t)1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      last = a;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace lgs
