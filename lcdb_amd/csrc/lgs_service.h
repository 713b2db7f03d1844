// lgs_service.h -- device side of the drop-in service (lgs_launch.h): the
// mailbox protocol shared by encode_service_kernel (lgs_encode.hip) and
// decode_service_kernel (lgs_decode.hip).
//
// Every access to a mailbox is a system-scope vector memory operation
// (global_load/store ... sc0 sc1, buffer_inv / buffer_wbl2): the mailboxes
// live in fine-grained pinned host memory that the host writes and polls.
#pragma once

#include "lgs_device.h"
#include "lgs_launch.h"

namespace lgs {

// One poll: {req, len} (one 8-byte atomic load, so a request's length is
// never torn from its number), the stop flag, the arena and the inbox, each
// by its own lane in one instruction.
struct SvcPoll {
  uint32_t req, len, stop;
  uint64_t arena, inbox;
};
__device__ __forceinline__ SvcPoll svc_poll(SvcMailbox* m) {
  const uint32_t lane = lane_id();
  uint64_t v = 0;
  if (lane < 4) {
    uint64_t* p = reinterpret_cast<uint64_t*>(m) + lane;   // +0 {req,len}, +8 {-,stop}, +16 arena, +24 inbox
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
  const uint32_t ilo = (uint32_t)__builtin_amdgcn_readlane(lo, 3);
  const uint32_t ihi = (uint32_t)__builtin_amdgcn_readlane(hi, 3);
  r.inbox = ((uint64_t)ihi << 32) | ilo;
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

// The wave's loop: serve(len, input, arena, &status, &out_len) for every new
// request (input: the inbox when set, else arena + kSvcIn)
// of mailbox m; exits on the stop flag or once the whole kernel has seen no
// request for `idle` ticks of the 100 MHz clock (activity: the kernel's last
// request, device memory).
template <class Serve>
__device__ __forceinline__ void svc_loop(SvcMailbox* m, uint64_t idle, uint64_t* activity,
                                         const Serve& serve) {
  uint32_t done =
      uni(__hip_atomic_load(&m->ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  if (lane_id() == 0) __hip_atomic_store(activity, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const SvcPoll q = svc_poll(m);
    if (q.stop) break;
    if (q.req != done && q.arena != 0) {
      uint32_t status = 0, out_len = 0;
      serve(q.len, q.inbox ? q.inbox : q.arena + kSvcIn, q.arena, &status, &out_len);
      svc_finish(m, q.req, status, out_len);
      done = q.req;
      last = __builtin_amdgcn_s_memrealtime();
      if (lane_id() == 0)
        __hip_atomic_store(activity, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (now - last > idle) {
      // Idle here; exit only if the kernel as a whole is (the waves leave
      // within a poll of each other, so a request never waits on a wave that
      // has gone while its kernel lingers).
      const uint64_t a = uni64(__hip_atomic_load(activity, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT));
      if (now - a > idle) break;
      last = a;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace lgs
