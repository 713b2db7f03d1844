// tools/lds_atomic_probe.hip -- does one ds_mskor_rtn_b32 wave instruction
// whose lanes hit the same LDS dword serialise them in ascending lane order?
// The encoder's literal search (lgs_encode.hip, encode_chunk) relies on it:
// each lane swaps its probe position into the u16 hash-table entry of its
// hash and gets back what the serial loop of snappy.c:146-148 would have read
// (the previous probe of the batch with that hash, else the old entry).  The
// encoder checks every batch itself and falls back to one probe per batch if
// the order is ever violated; this probe measures how often that would be.
//   build: hipcc -O2 --offload-arch=gfx950 tools/lds_atomic_probe.hip -o tools/lds_atomic_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mskor_rtn(uint32_t addr, uint32_t mask, uint32_t val) {
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(old) : "v"(addr), "v"(mask), "v"(val) : "memory");
  return old;
}

// LDS byte address of a __shared__ pointer (32-bit, address space 3).
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}

// Each wave: T trials; per trial every lane takes a pseudo-random 11-bit hash
// (with a configurable number of distinct values, to force collisions), swaps
// (trial << 8 | lane) into entry hash of a 2048 x u16 table, and checks the
// returned value and the final table against a serial replay in lane order.
__global__ __launch_bounds__(256) void probe(uint32_t trials, uint32_t distinct, uint32_t* bad,
                                             uint32_t* total, uint32_t active_mod) {
  __shared__ uint32_t tab[4][1024];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* t = tab[wv];
  for (uint32_t i = lane; i < 1024; i += 64) t[i] = 0x80008000u | (i << 1) | ((i << 1 | 1) << 16);
  __syncthreads();
  uint32_t nbad = 0, n = 0;
  uint32_t seed = blockIdx.x * 977u + wv * 131u + 12345u;
  for (uint32_t tr = 0; tr < trials; ++tr) {
    seed = seed * 1664525u + 1013904223u;
    const uint32_t s2 = seed;
    // lane hash: a few distinct values drawn from the full 2048 range
    uint32_t x = (s2 ^ (lane * 0x9e3779b9u)) * 0x85ebca6bu;
    x ^= x >> 13;
    const uint32_t pick = x % distinct;
    const uint32_t h = ((pick * 0x2545f491u) ^ s2) & 2047u;
    const bool act = active_mod == 0 || ((lane * 7 + tr) % active_mod) != 0;
    const uint32_t val = ((tr & 0xffu) << 8) | lane;
    uint32_t old = 0;
    if (act) {
      const uint32_t sh = (h & 1u) * 16;
      old = (mskor_rtn((h >> 1) * 4 + lds_addr(t), 0xffffu << sh, val << sh) >> sh) &
            0xffffu;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    // serial replay in lane order: expected old for lane l = value of the
    // highest active lane j < l with the same hash, else the entry's value
    // before this trial (which the lowest such lane received).
    uint32_t exp = 0xffffffffu;
    for (uint32_t j = 0; j < 64; ++j) {
      const uint32_t hj = __shfl(h, j), aj = __shfl((uint32_t)act, j);
      if (j < lane && aj && hj == h) exp = ((tr & 0xffu) << 8) | j;
    }
    // lanes with no earlier member: compare against the value the first
    // member of the group received (all must see the same pre-trial entry).
    uint32_t first = 64;
    for (uint32_t j = 0; j < 64; ++j) {
      const uint32_t hj = __shfl(h, j), aj = __shfl((uint32_t)act, j);
      if (aj && hj == h && first == 64) first = j;
    }
    const uint32_t first_old = __shfl(old, first & 63);
    if (exp == 0xffffffffu) exp = first_old;
    if (act) {
      ++n;
      if (old != exp) ++nbad;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  atomicAdd(bad, nbad);
  atomicAdd(total, n);
}

int main() {
  uint32_t *bad, *total;
  if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&total, 8) != hipSuccess) return 1;
  const uint32_t dist[] = {1, 2, 4, 8, 16, 64, 2048};
  const uint32_t amod[] = {0, 3};
  int rc = 0;
  for (uint32_t am : amod)
    for (uint32_t d : dist) {
      hipMemset(bad, 0, 8);
      hipMemset(total, 0, 8);
      hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, 200u, d, bad, total, am);
      uint32_t hb = 0, ht = 0;
      hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
      hipMemcpy(&ht, total, 4, hipMemcpyDeviceToHost);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      printf("distinct %4u active_mod %u: %u lane results, %u not in ascending lane order\n", d, am,
             ht, hb);
      if (hb) rc = 3;
    }
  printf(rc ? "ORDER VIOLATED\n" : "ascending lane order held in every trial\n");
  return rc;
}
