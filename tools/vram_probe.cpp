// tools/vram_probe.cpp -- can the host write fine-grained device memory through its
// mapping, and does the GPU see it (the drop-in service inbox)?
// build: hipcc -O2 --offload-arch=gfx950 tools/vram_probe.cpp -o tools/vram_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <signal.h>
#include <setjmp.h>
static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }
__global__ void rd(const unsigned* p, unsigned* out) { out[0] = p[0]; }
int main() {
  signal(SIGSEGV, on_segv);
  struct { const char* name; unsigned flags; } kinds[] = {{"finegrained", hipDeviceMallocFinegrained}, {"uncached", hipDeviceMallocUncached}};
  for (auto k : kinds) {
    unsigned* p = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&p, 4096, k.flags);
    printf("%s alloc %d %p\n", k.name, (int)e, (void*)p);
    if (e != hipSuccess) continue;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) == hipSuccess) printf("  type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
    if (sigsetjmp(jb, 1) == 0) {
      volatile unsigned* q = p; q[0] = 0x1234; printf("  cpu write ok, read %x\n", q[0]);
      unsigned* o; hipMalloc(&o, 4); rd<<<1,1>>>(p, o); unsigned h = 0; hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost); printf("  gpu sees %x\n", h);
    } else printf("  cpu write SEGV\n");
  }
  return 0;
}
