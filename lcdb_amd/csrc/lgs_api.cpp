// lgs_api.cpp -- host runtime and C ABI of the gfx950 Snappy codec
// (declarations, and the reference interfaces they replace:
// include/lcdb_gpu_snappy.h).
//
// HIP resources live in contexts (a non-blocking stream on one device plus a
// device arena and a pinned host arena) that are pooled per device and
// leased for the length of one call, never tied to a thread: lcdb enters the
// codec concurrently from user threads (reads) and its compaction thread
// (writes) (db_impl.c:1614-1652), and a host may create and join threads
// freely without leaking pinned memory.  Two pools:
//   * the drop-in's (ldb_snappy_*): at most LGS_DROPIN_SLOTS contexts per
//     device (default 8), each with fixed arenas of LGS_DROPIN_MB (default 4)
//     MiB that never grow -- any input size is handled in bounded passes;
//   * the batched host API's (lgs_*_host): arenas grow to the largest batch
//     a context has served, at most 16 contexts per device.
// A caller waits when its device's contexts are all leased.
//
// No compression or decompression happens on the host.  The host only moves
// bytes (pageable <-> pinned <-> device), computes the size bound
// (snappy.c:347-362) and reads the varint32 size header (snappy.c:386-399),
// and rejects on the host the streams whose header the stream's length
// cannot satisfy (an arithmetic bound, below) -- the reference rejects them
// too, so the result is the same without a device round trip.

#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lcdb_gpu_snappy.h"

#include "lgs_launch.h"

namespace lgs {
namespace {

constexpr uint32_t kChunk = 65536;   // snappy.c:28

thread_local char t_err[512];

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof t_err, fmt, ap);
  va_end(ap);
  return code;
}

#define LGS_HIP(call)                                                              \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(LGS_EHIP, "%s failed: %s", #call, hipGetErrorString(e_));        \
  } while (0)

#define LGS_TRY(expr)              \
  do {                             \
    int r_ = (expr);               \
    if (r_ != LGS_OK) return r_;   \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) & ~(a - 1); }

size_t bound_of(size_t n) { return 32 + n + n / 6; }   // snappy.c:354

// Host staging copies (pageable caller buffers <-> the pinned arena) split
// over threads once a call moves more than 8 MB: one thread copies ~10 GB/s,
// slower than the transfers it feeds.  Threads are per call (no shared pool:
// callers enter from several threads at once).  LGS_HOST_THREADS overrides
// the count (default: the hardware threads, at most 16).
unsigned host_threads(size_t bytes) {
  static const unsigned hw = [] {
    const char* e = getenv("LGS_HOST_THREADS");
    int v = e ? atoi(e) : 0;
    if (v <= 0) v = (int)std::thread::hardware_concurrency();
    if (v > 16) v = 16;
    return v > 0 ? (unsigned)v : 1u;
  }();
  return bytes < (8u << 20) ? 1u : hw;
}

// Worker threads for the staging copies: created once, never destroyed
// (like the HIP resources below), shared by every calling thread.
class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool(host_threads(~(size_t)0));
    return *p;
  }
  // f(0 .. t-1): part 0 on the caller, the others on workers.
  void run(unsigned t, const std::function<void(unsigned)>& f) {
    std::mutex m;
    std::condition_variable cv;
    unsigned left = t - 1;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (unsigned k = 1; k < t; ++k)
        q_.push_back([&, k] {
          f(k);
          std::lock_guard<std::mutex> g2(m);      // the caller's stack frame outlives this
          if (--left == 0) cv.notify_one();
        });
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return left == 0; });
  }

 private:
  explicit Pool(unsigned n) {
    for (unsigned k = 1; k < n; ++k) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

// f(i0, i1) over [0, n) in contiguous ranges, on host_threads(bytes) threads.
template <class F>
void par_for(uint32_t n, size_t bytes, const F& f) {
  const unsigned t = host_threads(bytes);
  if (t <= 1 || n < 2 * t) {
    f(0u, n);
    return;
  }
  const uint32_t per = (n + t - 1) / t;
  Pool::get().run(t, [&](unsigned k) {
    const uint32_t a = k * per, b = a + per < n ? a + per : n;
    if (a < b) f(a, b);
  });
}

struct Ctx {
  int device = -1;          // device this context's resources live on
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;   // the chunk pipeline's second stream (lazily)
  hipEvent_t done[2] = {nullptr, nullptr};
  uint8_t* d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t* h_buf = nullptr; // pinned
  size_t h_cap = 0;
  uint8_t* h_dev = nullptr; // a drop-in slot's pinned arena as the device sees it
  bool fixed = false;       // a drop-in slot: arenas never grow
  uint32_t svc_idx = ~0u;   // a drop-in slot's service mailbox (kSvcMaxSlots: none)
  uint32_t svc_seq[2] = {0, 0};   // its last request per kind (encode, decode)
  bool retired = false;     // a service request timed out: never leased again
};

// lgs_set_device() choice of the calling thread (-1: its current device).
thread_local int t_want_device = -1;

int visible_devices() {
  static const int n = [] {
    int c = 0;
    return hipGetDeviceCount(&c) == hipSuccess ? c : 0;
  }();
  return n;
}

// The device a call from this thread runs on (made current for the thread).
int call_device(int* dev) {
  const int count = visible_devices();
  if (count <= 0) return fail(LGS_ENODEV, "no HIP device visible");
  if (t_want_device < 0) {
    LGS_HIP(hipGetDevice(dev));
  } else {
    if (t_want_device >= count)
      return fail(LGS_ENODEV, "device %d not present (%d visible)", t_want_device, count);
    *dev = t_want_device;
    LGS_HIP(hipSetDevice(*dev));
  }
  if (*dev < 0 || *dev >= 64) return fail(LGS_ENODEV, "device %d out of range", *dev);
  return LGS_OK;
}

constexpr size_t kSlotDev = 64 << 10;   // a drop-in slot's device arena

size_t env_size(const char* name, size_t dflt, size_t lo, size_t hi) {
  const char* e = getenv(name);
  long v = e ? atol(e) : 0;
  size_t r = v > 0 ? (size_t)v : dflt;
  return r < lo ? lo : (r > hi ? hi : r);
}

// Drop-in slot arenas (pinned and device, each): LGS_DROPIN_MB MiB, at least
// 1 (one 64 KiB chunk's input and bound-sized output fit with room to spare).
size_t dropin_cap() {
  static const size_t v = env_size("LGS_DROPIN_MB", 4, 1, 1024) << 20;
  return v;
}
unsigned dropin_max_slots() {
  static const unsigned v = (unsigned)env_size("LGS_DROPIN_SLOTS", 8, 1, 256);
  return v;
}

// Contexts of one kind, per device.  Created on demand up to `max` per
// device; HIP resources are never freed (freeing from static destructors can
// run after the runtime is torn down at process exit).
class CtxPool {
 public:
  CtxPool(unsigned max, size_t fixed_cap) : max_(max), fixed_cap_(fixed_cap) {}

  // Lease a context on the calling thread's device; waits while all of that
  // device's contexts are leased.
  int acquire(Ctx** out) {
    int dev = -1;
    LGS_TRY(call_device(&dev));
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      std::vector<Ctx*>& fl = free_[dev];
      if (!fl.empty()) {
        *out = fl.back();
        fl.pop_back();
        return LGS_OK;
      }
      if (live_[dev] < max_) break;
      cv_.wait(lk);
    }
    ++live_[dev];
    lk.unlock();
    Ctx* c = new Ctx;
    c->device = dev;
    const int rc = create(c);
    if (rc != LGS_OK) {
      destroy_partial(c);
      lk.lock();
      --live_[dev];
      const bool others = live_[dev] > 0;
      lk.unlock();
      cv_.notify_all();
      // Out of pinned or device memory while other contexts exist: wait for
      // one of them instead of failing the call.
      if (rc == LGS_ENOMEM && others) return acquire_existing(dev, out);
      return rc;
    }
    *out = c;
    return LGS_OK;
  }

  void release(Ctx* c) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (c->retired)
        --live_[c->device];               // leaked on purpose; a new one may be made
      else
        free_[c->device].push_back(c);
    }
    cv_.notify_one();
  }

  // Bytes of pinned / device memory held by this pool's contexts.
  void footprint(size_t* pinned, size_t* device, unsigned* count) {
    std::lock_guard<std::mutex> g(mu_);
    size_t p = 0, d = 0;
    unsigned n = 0;
    for (const Ctx* c : all_) {
      p += c->h_cap;
      d += c->d_cap;
      ++n;
    }
    *pinned = p;
    *device = d;
    *count = n;
  }

  size_t fixed_cap() const { return fixed_cap_; }

 private:
  int create(Ctx* c) {
    LGS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (fixed_cap_) {
      c->fixed = true;
      // Device memory only for the per-item arrays of an over-slot decode
      // (in-slot calls work in the mapped pinned arena).
      if (hipMalloc(&c->d_buf, kSlotDev) != hipSuccess)
        return fail(LGS_ENOMEM, "hipMalloc(%zu) failed", kSlotDev);
      c->d_cap = kSlotDev;
      // Mapped and coherent: the kernels of an in-slot call read their input
      // from it and write their output to it directly (no copies).
      if (hipHostMalloc(&c->h_buf, fixed_cap_, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess)
        return fail(LGS_ENOMEM, "hipHostMalloc(%zu) failed", fixed_cap_);
      c->h_cap = fixed_cap_;
      void* dp = nullptr;
      LGS_HIP(hipHostGetDevicePointer(&dp, c->h_buf, 0));
      c->h_dev = (uint8_t*)dp;
    }
    std::lock_guard<std::mutex> g(mu_);
    all_.push_back(c);
    if (fixed_cap_) c->svc_idx = next_idx_[c->device]++;
    return LGS_OK;
  }
  static void destroy_partial(Ctx* c) {
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->d_buf) (void)hipFree(c->d_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
  }
  int acquire_existing(int dev, Ctx** out) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !free_[dev].empty(); });
    *out = free_[dev].back();
    free_[dev].pop_back();
    return LGS_OK;
  }

  const unsigned max_;
  const size_t fixed_cap_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Ctx*> free_[64];
  unsigned live_[64] = {};
  std::vector<Ctx*> all_;
  uint32_t next_idx_[64] = {};
};

CtxPool& dropin_pool() {
  static CtxPool* p = new CtxPool(dropin_max_slots(), dropin_cap());
  return *p;
}
CtxPool& batch_pool() {
  static CtxPool* p = new CtxPool(16, 0);
  return *p;
}

// One context, leased for the length of a call.
class Lease {
 public:
  explicit Lease(CtxPool& p) : pool_(p) {}
  ~Lease() {
    if (c_) pool_.release(c_);
  }
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
  int acquire() { return pool_.acquire(&c_); }
  Ctx& ctx() { return *c_; }

 private:
  CtxPool& pool_;
  Ctx* c_ = nullptr;
};

int ctx_reserve(Ctx& c, size_t dev_bytes, size_t pin_bytes) {
  if (c.fixed) {
    (void)dev_bytes;                        // in-slot calls work in the pinned arena
    if (pin_bytes > c.h_cap)
      return fail(LGS_EINTERNAL, "drop-in slot of %zu bytes, %zu needed", c.h_cap, pin_bytes);
    return LGS_OK;
  }
  if (dev_bytes > c.d_cap) {
    if (c.d_buf) LGS_HIP(hipFree(c.d_buf));
    c.d_buf = nullptr;
    c.d_cap = 0;
    const size_t cap = align_up(dev_bytes + dev_bytes / 4, 1 << 20);
    if (hipMalloc(&c.d_buf, cap) != hipSuccess) return fail(LGS_ENOMEM, "hipMalloc(%zu) failed", cap);
    c.d_cap = cap;
  }
  if (pin_bytes > c.h_cap) {
    if (c.h_buf) LGS_HIP(hipHostFree(c.h_buf));
    c.h_buf = nullptr;
    c.h_cap = 0;
    const size_t cap = align_up(pin_bytes + pin_bytes / 4, 1 << 20);
    if (hipHostMalloc(&c.h_buf, cap, hipHostMallocDefault) != hipSuccess)
      return fail(LGS_ENOMEM, "hipHostMalloc(%zu) failed", cap);
    c.h_cap = cap;
  }
  return LGS_OK;
}

// Two streams and two events for the chunk pipeline below.
int ctx_pipeline(Ctx& c) {
  if (c.stream2 == nullptr) LGS_HIP(hipStreamCreateWithFlags(&c.stream2, hipStreamNonBlocking));
  for (hipEvent_t& e : c.done)
    if (e == nullptr) LGS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return LGS_OK;
}

// Runs `chunks` independent pieces of a host call through two streams:
// stage(k) fills chunk k's own part of the pinned arena, launch(k, stream)
// enqueues its uploads, kernels and downloads, finish(k) copies its results
// out once they have arrived.  Staging chunk k+1 and finishing chunk k-1 on
// the host overlap chunk k's transfers and kernels, and consecutive chunks'
// transfers overlap each other's kernels.  Chunks use disjoint parts of the
// arenas; a stream's scratch is reused only after that stream's previous
// chunk has finished.
template <class Stage, class Launch, class Finish>
int pipeline(Ctx& c, uint32_t chunks, const Stage& stage, const Launch& launch,
             const Finish& finish) {
  LGS_TRY(ctx_pipeline(c));
  const hipStream_t st[2] = {c.stream, c.stream2};
  for (uint32_t k = 0; k < chunks; ++k) {
    stage(k);
    LGS_TRY(launch(k, st[k & 1]));
    LGS_HIP(hipEventRecord(c.done[k & 1], st[k & 1]));
    if (k >= 1) {
      LGS_HIP(hipEventSynchronize(c.done[(k - 1) & 1]));
      LGS_TRY(finish(k - 1));
    }
  }
  LGS_HIP(hipEventSynchronize(c.done[(chunks - 1) & 1]));
  return finish(chunks - 1);
}

// Chunk boundaries: [first[k], first[k+1]) over n items of `bytes` in total,
// about LGS_HOST_CHUNK_MB (default 64; 0: no chunking) each; one chunk for
// small calls.
size_t chunk_bytes() {
  static const size_t v = [] {
    const char* e = getenv("LGS_HOST_CHUNK_MB");
    return (size_t)(e ? atoi(e) : 64) << 20;
  }();
  return v;
}

std::vector<uint32_t> chunk_bounds(uint32_t n, size_t bytes, const uint32_t* len) {
  const size_t kChunkBytes = chunk_bytes();
  std::vector<uint32_t> first{0};
  if (kChunkBytes > 0 && bytes >= 2 * kChunkBytes) {
    size_t acc = 0;
    for (uint32_t i = 0; i < n; ++i) {
      acc += len[i];
      if (acc >= kChunkBytes && i + 1 < n) {
        first.push_back(i + 1);
        acc = 0;
      }
    }
  }
  first.push_back(n);
  return first;
}

// Offsets into a staging area, 256-byte aligned.  The pinned arena and the
// device arena use the same layout, so an upload or a download is a single
// contiguous hipMemcpyAsync.
struct Layout {
  size_t at = 0;
  size_t take(size_t bytes) {
    const size_t o = at;
    at = align_up(at + bytes, 256);
    return o;
  }
};

// coding.h:169-204 on the host, for the size header only.  Returns the
// header's length in bytes (1-5), 0 if there is no valid header.
int read_varint32(uint32_t* v, const uint8_t* p, size_t n) {
  uint32_t acc = 0;
  unsigned sh = 0;
  for (size_t i = 0; sh <= 28 && i < n; sh += 7, ++i) {
    const uint32_t b = p[i];
    if ((b & 0x80u) == 0) {
      *v = acc | (b << sh);
      return (int)i + 1;
    }
    acc |= (b & 0x7fu) << sh;
  }
  *v = 0;
  return 0;
}

// LGS_DIE_EXIT=<code>: exit with that code instead of abort() (tests drive
// the failure paths in child processes without a SIGABRT on the GPU box).
[[noreturn]] void die(const char* what) {
  fprintf(stderr, "lcdb_gpu_snappy: %s failed: %s\n", what, t_err);
  fflush(stderr);
  const char* e = getenv("LGS_DIE_EXIT");
  if (e && atoi(e) > 0) _exit(atoi(e));
  abort();
}

// ---- the drop-in (ldb_snappy_encode / ldb_snappy_decode) ----
//
// Single blocks from lcdb's table builder and block reader.  Every call
// leases a drop-in slot (fixed arenas of dropin_cap() bytes), so a call
// never allocates: an input of any size goes through the slot in passes of
// whole 64 KiB chunks, which are independent (snappy.c:370-381), and the
// chunks' encodings are concatenated on the host as they come back.  The
// slot's pinned arena is mapped into the device: a pass copies the input
// into it, launches the kernel on it (input read and output written over
// PCIe, no hipMemcpy) and synchronises once.

// ---- the drop-in service (lgs_launch.h, lgs_service.h) ----
//
// One request at a time per slot: the input goes to the slot's arena at
// kSvcIn, {sequence, length} into its mailbox with one 8-byte store, and the
// call spins on the mailbox's ack (host memory) until the resident wave has
// written the output at kSvcOut.  The service kernels start on the first
// request; a request that finds its kernel gone (idle exit) relaunches it.
// LGS_DROPIN_SERVICE=0 (or lgs_set_option("service", "0")) sends every call
// through the launch path instead; so do items over kSvcMaxItem.
std::atomic<int> g_svc_enabled{[] {
  const char* e = getenv("LGS_DROPIN_SERVICE");
  return e && !strcmp(e, "0") ? 0 : 1;
}()};
std::atomic<bool> g_svc_shutdown{false};
// lgs_service_quiesce() .. lgs_service_resume(): calls take the launch path.
std::atomic<bool> g_svc_paused{false};
// svc_call's answer for a request taken back from a stopped service: the
// caller runs it through the launch path.
constexpr int kSvcWithdrawn = 1;

// Idle exit of the resident waves (LGS_SERVICE_IDLE_US, default 2 ms): a
// device-wide synchronisation waits at most this long after the last call.
uint64_t svc_idle_us() {
  static const uint64_t v = env_size("LGS_SERVICE_IDLE_US", 2000, 50, 10000000);
  return v;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Service {
  std::mutex mu;
  int state = 0;                      // 0 not set up, 1 ready, -1 unavailable
  SvcMailbox* mb = nullptr;           // host view: encode [0, S), decode [S, 2S)
  SvcMailbox* mb_dev = nullptr;
  SvcControl* ctl = nullptr;          // device, one per kind
  hipStream_t stream[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  std::atomic<bool> launched[2];
  std::atomic<int64_t> last_use[2];   // steady-clock ns of the last finished request
  uint32_t nslots = 0;

  SvcMailbox* box(int kind, uint32_t idx) { return mb + (size_t)kind * kSvcMaxSlots + idx; }

  int setup() {                       // under mu
    if (state) return state > 0 ? LGS_OK : LGS_EINTERNAL;
    state = -1;
    const size_t bytes = 2 * kSvcMaxSlots * sizeof(SvcMailbox);
    if (hipHostMalloc(&mb, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(LGS_ENOMEM, "service mailboxes: hipHostMalloc(%zu) failed", bytes);
    memset(mb, 0, bytes);
    void* dp = nullptr;
    LGS_HIP(hipHostGetDevicePointer(&dp, mb, 0));
    mb_dev = (SvcMailbox*)dp;
    if (hipMalloc(&ctl, 2 * sizeof(SvcControl)) != hipSuccess)
      return fail(LGS_ENOMEM, "service: hipMalloc failed");
    LGS_HIP(hipMemset(ctl, 0, 2 * sizeof(SvcControl)));
    // Each kind's resident kernel on a hardware queue of its own.  Streams
    // beyond GPU_MAX_HW_QUEUES share queues, and a queue runs its packets in
    // order: a relaunched encode service queued behind a decode service that
    // sustained traffic keeps alive would never start (found by
    // test_service_busy_slot_does_not_strand_another).  A stream with a CU
    // mask gets a new queue, never one from the shared pool; the mask here
    // is every CU.
    int dev = 0;
    hipDeviceProp_t prop{};
    LGS_HIP(hipGetDevice(&dev));
    LGS_HIP(hipGetDeviceProperties(&prop, dev));
    std::vector<uint32_t> cus((size_t)(prop.multiProcessorCount + 31) / 32, ~0u);
    for (int k = 0; k < 2; ++k) {
      LGS_HIP(hipExtStreamCreateWithCUMask(&stream[k], (uint32_t)cus.size(), cus.data()));
      LGS_HIP(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
      last_use[k] = 0;
      launched[k] = false;
    }
    const unsigned s = dropin_max_slots();
    nslots = s < kSvcMaxSlots ? s : kSvcMaxSlots;
    state = 1;
    return LGS_OK;
  }

  // Has the kernel of `kind` finished (or never run)?  Under mu.
  int finished(int kind, bool* gone) {
    *gone = true;
    if (!launched[kind]) return LGS_OK;
    const hipError_t q = hipEventQuery(done[kind]);
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      *gone = false;
      return LGS_OK;
    }
    if (q != hipSuccess) LGS_HIP(q);
    return LGS_OK;
  }

  // The kernel of `kind` running, or (re)launched -- unless the service is
  // paused (quiesce), when *gone reports whether it has finished.
  int ensure(int kind, bool* gone) {
    std::lock_guard<std::mutex> g(mu);
    *gone = false;
    if (g_svc_paused.load()) return finished(kind, gone);
    if (launched[kind]) {
      const hipError_t q = hipEventQuery(done[kind]);
      // (A pending query's hipErrorNotReady must not linger as this thread's
      // last error: the launchers return hipGetLastError().)
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        return LGS_OK;
      }
      if (q != hipSuccess) LGS_HIP(q);
    }
    const uint64_t idle = svc_idle_us() * 100;          // 100 MHz ticks
    // The previous kernel of this kind has finished (stream order): clear its
    // closing mark for the new waves.
    LGS_HIP(hipMemsetAsync(&ctl[kind].closing, 0, sizeof(uint64_t), stream[kind]));
    LGS_HIP(kind == 0 ? launch_encode_service(mb_dev, nslots, idle, ctl, stream[0])
                      : launch_decode_service(mb_dev + kSvcMaxSlots, nslots, idle, ctl + 1,
                                              stream[1]));
    LGS_HIP(hipEventRecord(done[kind], stream[kind]));
    launched[kind] = true;
    return LGS_OK;
  }
};

Service* g_services[64] = {};
std::mutex g_services_mu;

void svc_stop_all() {
  g_svc_shutdown = true;
  for (Service* sv : g_services)
    if (sv && sv->state > 0)
      for (uint32_t i = 0; i < 2 * kSvcMaxSlots; ++i)
        __atomic_store_n(&sv->mb[i].stop, 1u, __ATOMIC_RELEASE);
}

// lgs_service_quiesce(): every service kernel stopped and finished, and
// drop-in calls sent through the launch path until lgs_service_resume(), so
// an embedding application's device-wide synchronisation (hipFree,
// hipDeviceSynchronize) does not wait for resident waves under sustained
// traffic.  A call whose request the stopped waves left unanswered takes it
// back (svc_call) and runs it through the launch path.
int svc_quiesce() {
  g_svc_paused = true;
  for (Service* sv : g_services) {
    if (!sv) continue;
    std::lock_guard<std::mutex> g(sv->mu);
    if (sv->state <= 0) continue;
    for (uint32_t i = 0; i < 2 * kSvcMaxSlots; ++i)
      __atomic_store_n(&sv->mb[i].stop, 1u, __ATOMIC_RELEASE);
    int rc = LGS_OK;
    for (int k = 0; k < 2; ++k)
      if (sv->launched[k] && hipEventSynchronize(sv->done[k]) != hipSuccess)
        rc = fail(LGS_EINTERNAL, "service quiesce: %s", hipGetErrorString(hipGetLastError()));
    for (uint32_t i = 0; i < 2 * kSvcMaxSlots; ++i)
      __atomic_store_n(&sv->mb[i].stop, 0u, __ATOMIC_RELEASE);
    for (int k = 0; k < 2; ++k) sv->launched[k] = false;
    if (rc != LGS_OK) return rc;
  }
  return LGS_OK;
}

// The calling slot's service, ready, with its arena registered; nullptr
// when the call should take the launch path.
Service* svc_for(Ctx& c) {
  if (!g_svc_enabled.load(std::memory_order_relaxed) || g_svc_shutdown.load() ||
      g_svc_paused.load() || c.svc_idx >= kSvcMaxSlots || c.device < 0 || c.device >= 64)
    return nullptr;
  Service* sv;
  {
    std::lock_guard<std::mutex> g(g_services_mu);
    sv = g_services[c.device];
    if (!sv) {
      sv = g_services[c.device] = new Service;
      static std::once_flag once;
      std::call_once(once, [] { atexit(svc_stop_all); });
    }
  }
  std::lock_guard<std::mutex> g(sv->mu);
  if (sv->setup() != LGS_OK) return nullptr;
  if (c.svc_idx >= sv->nslots) return nullptr;
  for (int k = 0; k < 2; ++k) {
    SvcMailbox* m = sv->box(k, c.svc_idx);
    if (__atomic_load_n(&m->arena, __ATOMIC_RELAXED) == 0)
      __atomic_store_n(&m->arena, (uint64_t)(uintptr_t)c.h_dev, __ATOMIC_RELEASE);
  }
  return sv;
}

// A request's input goes to the arena at kSvcIn, 16 zero bytes after it
// (the decoder's read slack).  (Round 5 staged it in host-written
// fine-grained device memory for -0.8 us, and a wave read it torn with the
// previous request's bytes: lgs_service.h.)
void svc_stage(Ctx& c, const uint8_t* xp, uint32_t n) {
  uint8_t* in = c.h_buf + kSvcIn;
  memcpy(in, xp, n);
  memset(in + n, 0, 16);
}

// Post the request staged by svc_stage and wait for it: *status and
// *out_len as the wave reported them.  kSvcWithdrawn: the service was
// stopped (quiesce) before it answered; the request is withdrawn (its ack
// written by the host, so no later wave serves it) and the caller takes the
// launch path.
int svc_call(Service& sv, Ctx& c, int kind, uint32_t len, uint32_t* status, uint32_t* out_len) {
  SvcMailbox* m = sv.box(kind, c.svc_idx);
  uint32_t seq = c.svc_seq[kind] + 1;
  if (seq == 0) seq = 1;
  c.svc_seq[kind] = seq;
  __atomic_store_n(reinterpret_cast<uint64_t*>(m), (uint64_t)seq | ((uint64_t)len << 32),
                   __ATOMIC_RELEASE);
  const int64_t t_post = now_ns();
  // Not used for over half the idle time: its kernel has likely exited.
  bool gone = false;
  if (!sv.launched[kind] ||
      t_post - sv.last_use[kind].load(std::memory_order_relaxed) > (int64_t)svc_idle_us() * 500)
    LGS_TRY(sv.ensure(kind, &gone));
  int64_t t_check = t_post;
  for (uint32_t spin = 0; __atomic_load_n(&m->ack, __ATOMIC_ACQUIRE) != seq; ++spin) {
    __builtin_ia32_pause();
    if (gone || (spin & 255) == 255) {
      const int64_t t = now_ns();
      if (gone || t - t_check > 50000) {             // 50 us: is the kernel still there?
        if (!gone) LGS_TRY(sv.ensure(kind, &gone));
        if (gone) {
          // Paused and its kernel finished: answered before it left, or
          // withdrawn now (no wave is left to write the arena).
          if (__atomic_load_n(&m->ack, __ATOMIC_ACQUIRE) == seq) break;
          __atomic_store_n(&m->ack, seq, __ATOMIC_RELEASE);
          return kSvcWithdrawn;
        }
        t_check = t;
      }
      if (t - t_post > 20000000000ll) {
        // The wave may still answer later and write into the arena: stop it
        // and retire the slot, so no later lessee shares the arena with it.
        __atomic_store_n(&m->stop, 1u, __ATOMIC_RELEASE);
        c.retired = true;
        return fail(LGS_EINTERNAL, "drop-in service: no answer in 20 s");
      }
    }
  }
  *status = __atomic_load_n(&m->status, __ATOMIC_RELAXED);
  *out_len = __atomic_load_n(&m->out_len, __ATOMIC_RELAXED);
  sv.last_use[kind].store(now_ns(), std::memory_order_relaxed);
  return LGS_OK;
}

// Device bytes one 64 KiB-or-less chunk takes in a pass.
constexpr size_t kChunkIn = kChunk + 16;                         // its input
size_t chunk_out(uint32_t len) { return align_up(bound_of(len) + 8, 16); }

int encode_one(uint8_t* zp, const uint8_t* xp, size_t xn, size_t* written) {
  if (xn > 0x7fffffffu) return fail(LGS_EINVAL, "input of %zu bytes too large", xn);
  Lease lease(dropin_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  const uint32_t n = (uint32_t)xn;
  if (n <= kSvcMaxItem) {
    if (Service* sv = svc_for(c)) {                              // a resident wave
      svc_stage(c, xp, n);
      uint32_t st = 0, olen = 0;
      const int rc = svc_call(*sv, c, 0, n, &st, &olen);
      if (rc == LGS_OK) {
        if (st != 1 || olen > bound_of(n))
          return fail(LGS_EINTERNAL, "service encode: status %u, %u bytes", st, olen);
        memcpy(zp, c.h_buf + kSvcOut, olen);
        *written = olen;
        return LGS_OK;
      }
      if (rc != kSvcWithdrawn) return rc;
    }
  }
  // snappy.c:370-381: full 64 KiB chunks, then the remainder (if any);
  // a zero-length input is one empty item (just the varint header).
  const uint32_t nit = n <= kChunk ? 1u : (n + kChunk - 1) / kChunk;
  // Chunks per pass: per chunk its input, its output slot and 32 bytes of
  // per-item arrays, plus 7 x 256 of alignment slack.
  const size_t per = kChunkIn + chunk_out(kChunk) + 32 + 64;
  const uint32_t kmax = (uint32_t)((c.h_cap - 8 * 256) / per);
  if (kmax == 0) return fail(LGS_EINTERNAL, "drop-in slot of %zu bytes too small", c.h_cap);
  uint8_t* const h = c.h_buf;
  uint8_t* const hd = c.h_dev;
  size_t total = 0;
  for (uint32_t j0 = 0; j0 < nit; j0 += kmax) {
    const uint32_t k = nit - j0 < kmax ? nit - j0 : kmax;
    const size_t at = (size_t)j0 * kChunk;                      // input offset of the pass
    const size_t in_bytes = n - at < (size_t)k * kChunk ? n - at : (size_t)k * kChunk;
    Layout L;                                                    // upload | download
    const size_t o_in = L.take(in_bytes + 16);
    const size_t o_ioff = L.take(8 * (size_t)k);
    const size_t o_ilen = L.take(4 * (size_t)k);
    const size_t o_ooff = L.take(8 * (size_t)k);
    const size_t o_hdr = L.take(4 * (size_t)k);
    const size_t up_end = L.at;
    const size_t o_olen = L.take(4 * (size_t)k);
    size_t out_bytes = 0;
    for (uint32_t j = 0; j < k; ++j) {
      const size_t off = (size_t)j * kChunk;
      const uint32_t len = (uint32_t)(in_bytes - off < kChunk ? in_bytes - off : kChunk);
      out_bytes += chunk_out(len);
    }
    const size_t o_out = L.take(out_bytes);
    const size_t down_end = L.at;
    LGS_TRY(ctx_reserve(c, down_end, down_end));

    memcpy(h + o_in, xp + at, in_bytes);
    memset(h + o_in + in_bytes, 0, 16);
    uint64_t* ioff = (uint64_t*)(h + o_ioff);
    uint32_t* ilen = (uint32_t*)(h + o_ilen);
    uint64_t* ooff = (uint64_t*)(h + o_ooff);
    uint32_t* hdr = (uint32_t*)(h + o_hdr);
    size_t oa = o_out;
    for (uint32_t j = 0; j < k; ++j) {
      const size_t off = (size_t)j * kChunk;
      ilen[j] = (uint32_t)(in_bytes - off < kChunk ? in_bytes - off : kChunk);
      ioff[j] = o_in + off;
      ooff[j] = oa;
      oa += chunk_out(ilen[j]);
      hdr[j] = j0 + j == 0 ? n : 0xffffffffu;                    // snappy.c:368
    }
    (void)up_end;
    EncodeArgs a{hd, (const uint64_t*)(hd + o_ioff), (const uint32_t*)(hd + o_ilen), hd,
                 (const uint64_t*)(hd + o_ooff), (uint32_t*)(hd + o_olen),
                 (const uint32_t*)(hd + o_hdr), nullptr, k, nullptr};
    if (k == 1) a.one = Item1{ioff[0], ooff[0], ilen[0], hdr[0], 1};
    LGS_HIP(launch_encode(a, k == 1 ? ilen[0] : kChunk, c.stream));
    LGS_HIP(hipStreamSynchronize(c.stream));
    const uint32_t* olen = (const uint32_t*)(h + o_olen);
    for (uint32_t j = 0; j < k; ++j) {
      if (olen[j] > chunk_out(ilen[j]))
        return fail(LGS_EINTERNAL, "encoded chunk of %u bytes exceeds its bound", olen[j]);
      memcpy(zp + total, h + ooff[j], olen[j]);
      total += olen[j];
    }
  }
  if (total > bound_of(n)) return fail(LGS_EINTERNAL, "encoded length %zu exceeds bound", total);
  *written = total;
  return LGS_OK;
}

// The largest output an in-slot decode produces: the wave decoder's biggest
// LDS class (lgs_decode.hip kDecCap2).
constexpr uint32_t kInSlotDecodeMax = 66048;

// Host-side reference rejects, from the header and the stream length only
// (snappy.c:201-341): with m stream bytes after a header of `want`,
//   * want == 0: the reference accepts exactly when m == 0 (every tag either
//     produces >= 1 byte, failing len > zn, or is a copy failing :323);
//   * a COPY2 tag (3 bytes) yields at most 64 bytes, every other tag less
//     per byte, so 3 * want > 64 * m can never reach zn == 0 (:337);
//   * a tag consumes at most 6 bytes per byte it yields (a literal of one
//     byte with a 4-byte length: 1 + 4 + 1), so m > 6 * want must run out
//     of output first (:263, :323).
// Returns 1 (accept), 0 (reject) or -1 (the device decides).
int host_verdict(uint32_t want, size_t m) {
  if (want == 0) return m == 0 ? 1 : 0;
  if (3 * (uint64_t)want > 64 * (uint64_t)m) return 0;
  if ((uint64_t)m > 6 * (uint64_t)want) return 0;
  return -1;
}

// Device memory for an over-slot decode.  A valid stream must never come
// back as corrupt because memory is short for a moment (lcdb
// would turn that 0 into a lasting LDB_CORRUPTION background error), so a
// failed hipMalloc is tried 13 times, 12 sleeps from 0.5 ms doubling to a
// 256 ms cap between them (about 1 s in all), before the call fails -- and then ldb_snappy_decode aborts with a
// diagnostic, as on any other device failure.  Test hook:
// lgs_set_option("inject_alloc_failures", "N") makes the next N attempts
// fail as if the device were out of memory.
std::atomic<int> g_inject_alloc_failures{0};

// Stream-ordered (Scratch, lgs_launch.h): freed with hipFreeAsync on the
// slot's stream, never with hipFree, which synchronises the whole device and
// so would wait for resident service waves.
int big_alloc(std::unique_ptr<Scratch>* p, size_t bytes, uint32_t want, hipStream_t s) {
  unsigned wait_us = 500;
  for (int attempt = 0;; ++attempt) {
    int inj = g_inject_alloc_failures.load();
    bool injected = false;
    while (inj > 0 && !(injected = g_inject_alloc_failures.compare_exchange_weak(inj, inj - 1))) {
    }
    if (!injected) {
      p->reset(new Scratch(bytes, s));
      if ((*p)->status() == hipSuccess) return LGS_OK;
      p->reset();
      (void)hipGetLastError();
    }
    if (attempt == 12)
      return fail(LGS_ENOMEM, "hipMalloc(%zu) for a %u-byte block failed %d times", bytes, want,
                  attempt + 1);
    std::this_thread::sleep_for(std::chrono::microseconds(wait_us));
    wait_us = wait_us < 256000 ? 2 * wait_us : wait_us;
  }
}

// Decode one host block on the GPU.  *ok = reference decode result.
int decode_one(uint8_t* zp, const uint8_t* xp, size_t xn, int* ok) {
  *ok = 0;
  uint32_t want = 0;
  const int hl = read_varint32(&want, xp, xn);
  if (hl == 0 || want > 0x7fffffffu) return LGS_OK;            // snappy.c:405-409
  const int hv = host_verdict(want, xn - (size_t)hl);
  if (hv >= 0) {
    *ok = hv;
    return LGS_OK;
  }
  // Blocks are addressed with 32-bit lengths on the device.  A stream this
  // long passed host_verdict (want >= xn / 6 > 700 MB) and may be valid, so
  // it is not reported as corrupt: the call fails as unsupported.  (lcdb's
  // blocks are 4 KiB - a few MiB; format.c reads a block's bytes from the
  // file before decoding, so only a real multi-GiB block gets here.)
  if (xn > 0xffffffffu)
    return fail(LGS_EINVAL, "a %zu-byte stream exceeds the device decoder's 4 GiB limit", xn);
  const uint32_t n = (uint32_t)xn;
  Lease lease(dropin_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  uint8_t* const h = c.h_buf;
  if (want <= kSvcMaxItem && (size_t)n + 16 <= kSvcOut - kSvcIn) {
    if (Service* sv = svc_for(c)) {                              // a resident wave
      svc_stage(c, xp, n);
      uint32_t st = 0, olen = 0;
      const int rc = svc_call(*sv, c, 1, n, &st, &olen);
      if (rc == LGS_OK) {
        if (st == LGS_ST_OK && olen != want)
          return fail(LGS_EINTERNAL, "service decode: %u bytes for a %u-byte header", olen, want);
        if (st == LGS_ST_OK) memcpy(zp, h + kSvcOut, want);
        *ok = st == LGS_ST_OK;
        return LGS_OK;
      }
      if (rc != kSvcWithdrawn) return rc;
    }
  }

  Layout L;
  const size_t o_in = L.take((size_t)n + 16);
  const size_t o_ioff = L.take(8);
  const size_t o_ilen = L.take(4);
  const size_t o_ooff = L.take(8);
  const size_t o_ocap = L.take(4);
  const size_t up_end = L.at;
  const size_t o_st = L.take(4);
  const size_t o_olen = L.take(4);
  const size_t o_out = L.take((size_t)want + 16);
  const size_t down_end = L.at;
  if (down_end <= c.h_cap && want <= kInSlotDecodeMax) {
    // In the slot: the kernel reads the stream from the mapped pinned arena
    // and writes status, length and output there; one synchronisation.
    // (Outputs over the LDS classes decode straight against global memory,
    // one fenced round trip per copy: those take device memory below.)
    uint8_t* const hd = c.h_dev;
    (void)up_end;
    memcpy(h + o_in, xp, n);
    memset(h + o_in + n, 0, 16);
    *(uint64_t*)(h + o_ioff) = o_in;
    *(uint32_t*)(h + o_ilen) = n;
    *(uint64_t*)(h + o_ooff) = o_out;
    *(uint32_t*)(h + o_ocap) = want;
    DecodeArgs a{hd, (const uint64_t*)(hd + o_ioff), (const uint32_t*)(hd + o_ilen), hd,
                 (const uint64_t*)(hd + o_ooff), (const uint32_t*)(hd + o_ocap),
                 (uint32_t*)(hd + o_olen), hd + o_st, nullptr, 1, nullptr};
    a.one = Item1{o_in, o_out, n, want, 1};
    LGS_HIP(launch_decode(a, want, c.stream));
    LGS_HIP(hipStreamSynchronize(c.stream));
    const uint8_t st = h[o_st];
    if (st == LGS_ST_OK) memcpy(zp, h + o_out, want);
    *ok = st == LGS_ST_OK;
    return LGS_OK;
  }
  // Larger than the slot or than the LDS classes (multi-MiB index blocks):
  // device memory for this call only, the stream uploaded straight from the
  // caller's (pageable) buffer, and the output downloaded into zp only once
  // the status says ok.
  std::unique_ptr<Scratch> guard;
  const size_t big_bytes = align_up((size_t)n + 16, 256) + align_up((size_t)want + 16, 256);
  LGS_TRY(big_alloc(&guard, big_bytes, want, c.stream));
  uint8_t* const big = (uint8_t*)guard->get();
  uint8_t* const d_in = big;
  uint8_t* const d_out = big + align_up((size_t)n + 16, 256);
  Layout M;                                                      // per-item arrays, in the slot
  const size_t m_ioff = M.take(8), m_ilen = M.take(4), m_ooff = M.take(8), m_ocap = M.take(4);
  const size_t m_up = M.at;
  const size_t m_st = M.take(4), m_olen = M.take(4);
  const size_t m_down = M.at;
  uint8_t* const d = c.d_buf;
  *(uint64_t*)(h + m_ioff) = 0;
  *(uint32_t*)(h + m_ilen) = n;
  *(uint64_t*)(h + m_ooff) = 0;
  *(uint32_t*)(h + m_ocap) = want;
  LGS_HIP(hipMemcpyAsync(d_in, xp, n, hipMemcpyHostToDevice, c.stream));
  LGS_HIP(hipMemsetAsync(d_in + n, 0, 16, c.stream));
  LGS_HIP(hipMemcpyAsync(d, h, m_up, hipMemcpyHostToDevice, c.stream));
  DecodeArgs a{d_in, (const uint64_t*)(d + m_ioff), (const uint32_t*)(d + m_ilen), d_out,
               (const uint64_t*)(d + m_ooff), (const uint32_t*)(d + m_ocap),
               (uint32_t*)(d + m_olen), d + m_st, nullptr, 1, nullptr};
  LGS_HIP(launch_decode(a, want, c.stream));
  LGS_HIP(hipMemcpyAsync(h + m_st, d + m_st, m_down - m_st, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  if (h[m_st] == LGS_ST_OK) {
    LGS_HIP(hipMemcpyAsync(zp, d_out, want, hipMemcpyDeviceToHost, c.stream));
    LGS_HIP(hipStreamSynchronize(c.stream));
    *ok = 1;
  }
  return LGS_OK;
}

// Kernel options: lgs_set_option(), initial values from the environment.
Options& options_init() {
  static Options* o = [] {
    Options* v = new Options;
    const char* dk = getenv("LGS_DECODE_KERNEL");
    if (dk && !strcmp(dk, "ring")) v->decoder = kDecRing;
    if (dk && !strcmp(dk, "wave")) v->decoder = kDecWave;
#ifdef LGS_PROBE_DECODERS
    if (dk && !strcmp(dk, "chain")) v->decoder = kDecChain;
    if (dk && !strcmp(dk, "group")) v->decoder = kDecGroup;
    const char* wg = getenv("LGS_WIDE_DECODER");
    if (wg && !strcmp(wg, "group")) v->wide = kWideGroup;
    if (dk && !strcmp(dk, "quad")) v->decoder = kDecQuad;
    if (dk && !strcmp(dk, "ops")) v->decoder = kDecOps;
    const char* wd = getenv("LGS_WIDE_DECODER");
    if (wd && !strcmp(wd, "trips")) v->wide = kWideTrips;
#endif
#ifndef LGS_PROBE_DECODERS
    // The decoders that lost their A/B exist in the probe library only: say
    // so rather than silently measuring the default.
    const char* wd0 = getenv("LGS_WIDE_DECODER");
    if ((dk && (!strcmp(dk, "quad") || !strcmp(dk, "ops") || !strcmp(dk, "group") ||
                !strcmp(dk, "chain"))) ||
        (wd0 && (!strcmp(wd0, "trips") || !strcmp(wd0, "group"))))
      fprintf(stderr,
              "lcdb_gpu_snappy: LGS_DECODE_KERNEL=%s LGS_WIDE_DECODER=%s names a probe-library "
              "decoder; this library uses its default decoders\n",
              dk ? dk : "", wd0 ? wd0 : "");
#endif
    const char* vo = getenv("LGS_VERIFY_OVERLAP");
    if (vo && !strcmp(vo, "0")) v->verify_overlap = 0;
    const char* ns = getenv("LGS_NO_SPLIT");
    if (ns && *ns && strcmp(ns, "0")) v->split = 0;
    return v;
  }();
  return *o;
}

}  // namespace

int set_error(int code, const char* msg) { return fail(code, "%s", msg); }

Options& options() { return options_init(); }

// off[i] = i * stride (lgs_table.hip; declared here, not in lgs_launch.h,
// whose text keys the codec kernels' traffic figures).
hipError_t launch_fill_stride(uint64_t* off, uint64_t stride, uint32_t n, hipStream_t s);
// check_kernel's checks with one lane per handle, no CRC (lgs_table.hip;
// declared here for the same reason).
hipError_t launch_check_lane(const CheckArgs& a, hipStream_t s);

}  // namespace lgs

using namespace lgs;

extern "C" {

// ---- drop-in (src/util/snappy.h:28-38) ----

int ldb_snappy_encode_size(size_t* zn, size_t xn) {   // snappy.c:347-362
  if (xn > 0x7fffffff) return 0;
  const size_t n = bound_of(xn);
  if (n > 0x7fffffff) return 0;
  *zn = n;
  return 1;
}

size_t ldb_snappy_encode(uint8_t* zp, const uint8_t* xp, size_t xn) {
  // lcdb's encode path has no error return (table_builder.c:182-188): a
  // failure here is a lost device or a broken runtime, so abort loudly.
  size_t written = 0;
  if (encode_one(zp, xp, xn, &written) != LGS_OK) die("ldb_snappy_encode");
  return written;
}

int ldb_snappy_decode_size(size_t* zn, const uint8_t* xp, size_t xn) {   // snappy.c:386-399
  uint32_t v;
  if (!read_varint32(&v, xp, xn)) return 0;
  if (v > 0x7fffffffu) return 0;
  *zn = v;
  return 1;
}

int ldb_snappy_decode(uint8_t* zp, const uint8_t* xp, size_t xn) {
  // format.c:237-251 turns 0 into LDB_CORRUPTION, so 0 means exactly the
  // reference's 0.  A call that cannot run (device memory still short after
  // big_alloc's retries, a lost device, a stream beyond the device's 4 GiB
  // addressing) is not a corrupt block: it aborts with a diagnostic.
  int ok = 0;
  if (decode_one(zp, xp, xn, &ok) != LGS_OK) die("ldb_snappy_decode");
  return ok;
}

// ---- drop-in footprint and kernel options ----

int lgs_dropin_footprint(size_t* pinned, size_t* device, uint32_t* slots, size_t* slot_bytes) {
  if (!pinned || !device || !slots || !slot_bytes) return fail(LGS_EINVAL, "NULL argument");
  unsigned n = 0;
  dropin_pool().footprint(pinned, device, &n);
  *slots = n;
  *slot_bytes = dropin_pool().fixed_cap();
  return LGS_OK;
}

int lgs_service_quiesce(void) { return lgs::svc_quiesce(); }

int lgs_service_resume(void) {
  lgs::g_svc_paused = false;
  return LGS_OK;
}

int lgs_set_option(const char* name, const char* value) {
  if (!name || !value) return fail(LGS_EINVAL, "NULL argument");
  Options& o = options();
  if (!strcmp(name, "decoder")) {
    if (!strcmp(value, "auto") || !*value) o.decoder = kDecAuto;
    else if (!strcmp(value, "ring")) o.decoder = kDecRing;
    else if (!strcmp(value, "wave")) o.decoder = kDecWave;
#ifdef LGS_PROBE_DECODERS
    else if (!strcmp(value, "chain")) o.decoder = kDecChain;
    else if (!strcmp(value, "group")) o.decoder = kDecGroup;
    // The decoders that lost their A/B exist in the probe library only
    // (lgs_decode_probe.hip); the product rejects them.
    else if (!strcmp(value, "quad")) o.decoder = kDecQuad;
    else if (!strcmp(value, "ops")) o.decoder = kDecOps;
#endif
    else return fail(LGS_EINVAL, "decoder '%s' (auto, ring or wave)", value);
    return LGS_OK;
  }
  if (!strcmp(name, "inject_alloc_failures")) {   // test hook (big_alloc)
    char* end = nullptr;
    const long v = strtol(value, &end, 10);
    if (!*value || *end || v < 0 || v > 1000000)
      return fail(LGS_EINVAL, "inject_alloc_failures '%s' (0..1000000)", value);
    g_inject_alloc_failures = (int)v;
    return LGS_OK;
  }
  if (!strcmp(name, "wide")) {
    if (!strcmp(value, "walk") || !*value) o.wide = kWideWalk;
#ifdef LGS_PROBE_DECODERS
    else if (!strcmp(value, "group")) o.wide = kWideGroup;
    else if (!strcmp(value, "trips")) o.wide = kWideTrips;
#endif
    else return fail(LGS_EINVAL, "wide '%s' (walk)", value);
    return LGS_OK;
  }
  if (!strcmp(name, "service")) {   // the drop-in's resident waves (LGS_DROPIN_SERVICE)
    if (!strcmp(value, "1")) g_svc_enabled = 1;
    else if (!strcmp(value, "0")) g_svc_enabled = 0;
    else return fail(LGS_EINVAL, "service '%s' (0 or 1)", value);
    return LGS_OK;
  }
  if (!strcmp(name, "verify_overlap")) {   // table reads: CRC pass beside the decoder
    if (!strcmp(value, "1")) o.verify_overlap = 1;
    else if (!strcmp(value, "0")) o.verify_overlap = 0;
    else return fail(LGS_EINVAL, "verify_overlap '%s' (0 or 1)", value);
    return LGS_OK;
  }
  if (!strcmp(name, "split")) {
    if (!strcmp(value, "1")) o.split = 1;
    else if (!strcmp(value, "0")) o.split = 0;
    else return fail(LGS_EINVAL, "split '%s' (0 or 1)", value);
    return LGS_OK;
  }
  return fail(LGS_EINVAL, "unknown option '%s'", name);
}

// ---- batched API ----

size_t lgs_encode_bound(size_t n) { return bound_of(n); }

int lgs_encode_batch_dev(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                         uint8_t* d_out, const uint64_t* d_out_off, uint32_t* d_out_len,
                         uint32_t n, uint32_t max_in_len, void* stream) {
  if (n == 0) return LGS_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len)
    return fail(LGS_EINVAL, "NULL argument");
  if (max_in_len > 0x7fffffffu) return fail(LGS_EINVAL, "max_in_len %u too large", max_in_len);
  EncodeArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, nullptr, nullptr, n, nullptr};
  LGS_HIP(launch_encode(a, max_in_len, (hipStream_t)stream));
  return LGS_OK;
}

int lgs_decode_batch_dev(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                         uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                         uint32_t* d_out_len, uint8_t* d_status, uint32_t n,
                         uint32_t max_out_cap, void* stream) {
  if (n == 0) return LGS_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len ||
      !d_status)
    return fail(LGS_EINVAL, "NULL argument");
  DecodeArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_cap, d_out_len, d_status,
               nullptr, n, nullptr};
  LGS_HIP(launch_decode(a, max_out_cap, (hipStream_t)stream));
  return LGS_OK;
}

int lgs_encode_batch_host(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                          uint8_t* out, const uint64_t* out_off, uint32_t* out_len, uint32_t n) {
  if (n == 0) return LGS_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_len)
    return fail(LGS_EINVAL, "NULL argument");
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t in_total = 0, out_total = 0;
  uint32_t max_in = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (in_len[i] > 0x7fffffffu) return fail(LGS_EINVAL, "block %u too large", i);
    in_total += align_up(in_len[i], 16);
    out_total += align_up(bound_of(in_len[i]), 16);
    if (in_len[i] > max_in) max_in = in_len[i];
  }
  // The encodings land in bound-spaced device slots; a scan of their lengths
  // and a pack kernel then put them end to end, so only the compressed bytes
  // cross PCIe (C2: 153 MB instead of 316 MB of slots).  The packed region
  // comes back into the pinned slot region, which it never exceeds.
  Layout L;
  const size_t o_in = L.take(in_total + 16);
  const size_t o_ioff = L.take(8 * (size_t)n);
  const size_t o_ilen = L.take(4 * (size_t)n);
  const size_t o_ooff = L.take(8 * (size_t)n);
  const size_t up_end = L.at;
  const size_t o_olen = L.take(4 * (size_t)n);
  const size_t o_poff = L.take(8 * (size_t)n);
  const size_t o_pend = L.take(8);
  const size_t meta_end = L.at;
  const size_t o_out = L.take(out_total + 16);
  const size_t down_end = L.at;
  const size_t o_part = L.take(8 * scan_parts(n) + 8);          // device only
  const size_t o_pack = L.take(out_total + 16);                 // device only
  LGS_TRY(ctx_reserve(c, L.at, down_end));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  uint64_t* ioff = (uint64_t*)(h + o_ioff);
  uint32_t* ilen = (uint32_t*)(h + o_ilen);
  uint64_t* ooff = (uint64_t*)(h + o_ooff);
  size_t ia = o_in, oa = o_out;
  for (uint32_t i = 0; i < n; ++i) {
    ioff[i] = ia;
    ilen[i] = in_len[i];
    ooff[i] = oa;
    ia += align_up(in_len[i], 16);
    oa += align_up(bound_of(in_len[i]), 16);
  }
  par_for(n, in_total, [&](uint32_t i0, uint32_t i1) {
    for (uint32_t i = i0; i < i1; ++i) memcpy(h + ioff[i], in + in_off[i], in_len[i]);
  });
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  EncodeArgs a{d, (const uint64_t*)(d + o_ioff), (const uint32_t*)(d + o_ilen), d,
               (const uint64_t*)(d + o_ooff), (uint32_t*)(d + o_olen), nullptr, nullptr, n, nullptr};
  LGS_HIP(launch_encode(a, max_in, c.stream));
  LGS_HIP(launch_scan(2, nullptr, (const uint32_t*)(d + o_olen), (uint64_t*)(d + o_part), 0,
                      (uint64_t*)(d + o_poff), (uint64_t*)(d + o_pend), n, c.stream));
  LGS_HIP(launch_pack(d, (const uint64_t*)(d + o_ooff), (const uint32_t*)(d + o_olen),
                      d + o_pack, (const uint64_t*)(d + o_poff), n, c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_olen, d + o_olen, meta_end - o_olen, hipMemcpyDeviceToHost,
                         c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  const uint64_t packed = *(const uint64_t*)(h + o_pend);
  if (packed > out_total) return fail(LGS_EINTERNAL, "packed encodings exceed their slots");
  LGS_HIP(hipMemcpyAsync(h + o_out, d + o_pack, packed, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  const uint32_t* olen = (const uint32_t*)(h + o_olen);
  const uint64_t* poff = (const uint64_t*)(h + o_poff);
  par_for(n, packed, [&](uint32_t i0, uint32_t i1) {
    for (uint32_t i = i0; i < i1; ++i) {
      memcpy(out + out_off[i], h + o_out + poff[i], olen[i]);
      out_len[i] = olen[i];
    }
  });
  return LGS_OK;
}

int lgs_decode_batch_host(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                          uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                          uint32_t* out_len, uint8_t* status, uint32_t n) {
  if (n == 0) return LGS_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len || !status)
    return fail(LGS_EINVAL, "NULL argument");
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t in_total = 0, out_total = 0;
  uint32_t max_cap = 0;
  for (uint32_t i = 0; i < n; ++i) {
    in_total += align_up(in_len[i], 16);
    out_total += align_up(out_cap[i], 16);
    if (out_cap[i] > max_cap) max_cap = out_cap[i];
  }
  Layout L;
  const size_t o_in = L.take(in_total + 16);
  const size_t o_ioff = L.take(8 * (size_t)n);
  const size_t o_ilen = L.take(4 * (size_t)n);
  const size_t o_ooff = L.take(8 * (size_t)n);
  const size_t o_ocap = L.take(4 * (size_t)n);
  const size_t up_end = L.at;
  const size_t o_st = L.take((size_t)n);
  const size_t o_olen = L.take(4 * (size_t)n);
  const size_t o_out = L.take(out_total + 16);
  const size_t down_end = L.at;
  LGS_TRY(ctx_reserve(c, down_end, down_end));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  uint64_t* ioff = (uint64_t*)(h + o_ioff);
  uint32_t* ilen = (uint32_t*)(h + o_ilen);
  uint64_t* ooff = (uint64_t*)(h + o_ooff);
  uint32_t* ocap = (uint32_t*)(h + o_ocap);
  size_t ia = o_in, oa = o_out;
  for (uint32_t i = 0; i < n; ++i) {
    ioff[i] = ia;
    ilen[i] = in_len[i];
    ooff[i] = oa;
    ocap[i] = out_cap[i];
    ia += align_up(in_len[i], 16);
    oa += align_up(out_cap[i], 16);
  }
  par_for(n, in_total, [&](uint32_t i0, uint32_t i1) {
    for (uint32_t i = i0; i < i1; ++i) memcpy(h + ioff[i], in + in_off[i], in_len[i]);
  });
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  DecodeArgs a{d, (const uint64_t*)(d + o_ioff), (const uint32_t*)(d + o_ilen), d,
               (const uint64_t*)(d + o_ooff), (const uint32_t*)(d + o_ocap),
               (uint32_t*)(d + o_olen), d + o_st, nullptr, n, nullptr};
  LGS_HIP(launch_decode(a, max_cap, c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_st, d + o_st, down_end - o_st, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  const uint32_t* olen = (const uint32_t*)(h + o_olen);
  par_for(n, out_total, [&](uint32_t i0, uint32_t i1) {
    for (uint32_t i = i0; i < i1; ++i) {
      status[i] = h[o_st + i];
      out_len[i] = olen[i];
      if (status[i] == LGS_ST_OK) memcpy(out + out_off[i], h + ooff[i], olen[i]);
    }
  });
  return LGS_OK;
}

// ---- SSTable block framing (kernels: lgs_table.hip) ----

int lgs_crc32c_batch_dev(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                         const uint8_t* d_type, int masked, uint32_t* d_crc, uint32_t n,
                         void* stream) {
  if (n == 0) return LGS_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_crc) return fail(LGS_EINVAL, "NULL argument");
  LGS_HIP(launch_crc(d_in, d_in_off, d_in_len, d_type, masked, d_crc, n, (hipStream_t)stream));
  return LGS_OK;
}

int lgs_hbm_copy_dev(void* d_dst, const void* d_src, size_t bytes, void* stream) {
  if (bytes == 0) return LGS_OK;
  if (!d_dst || !d_src) return fail(LGS_EINVAL, "NULL argument");
  if (((uintptr_t)d_dst | (uintptr_t)d_src | bytes) & 15)
    return fail(LGS_EINVAL, "hbm copy needs 16-byte aligned pointers and length");
  LGS_HIP(launch_hbm_copy(d_dst, d_src, bytes, (hipStream_t)stream));
  return LGS_OK;
}

namespace {

// Device scratch of the write path (offsets from the scratch base).
struct WriteScratch {
  size_t enc_off, enc_len, part, foff, enc, enc_cap, total;
  WriteScratch(uint32_t n, uint64_t raw_total) {
    Layout L;
    enc_off = L.take(8 * (size_t)n);
    enc_len = L.take(4 * (size_t)n);
    part = L.take(8 * scan_parts(n) + 8);
    foff = L.take(8 * (size_t)n);
    // >= the sum of 16-aligned bounds, with 1/8 more so that near-uniform
    // blocks (lcdb's: every one within 1/8 of the mean) take one stride
    // (table_write: one fill kernel instead of a three-kernel scan).
    const uint64_t bounds = raw_total + raw_total / 6;
    enc_cap = 48 * (size_t)n + bounds + bounds / 8 + 64;
    enc = L.take(enc_cap);
    total = L.at;
  }
};

struct ReadScratch {
  size_t in_off, len, off, cap, olen, st, bad, dummy, total;
  explicit ReadScratch(uint32_t n) {
    Layout L;
    bad = L.take((size_t)n);
    in_off = L.take(8 * (size_t)n);
    len = L.take(4 * (size_t)n);
    off = L.take(8 * (size_t)n);
    cap = L.take(4 * (size_t)n);
    olen = L.take(4 * (size_t)n);
    st = L.take((size_t)n);
    dummy = L.take(64);
    total = L.at;
  }
};

static int table_write(const uint8_t* d_raw, const uint64_t* d_raw_off, const uint32_t* d_raw_len,
                uint32_t n, uint32_t max_raw_len, int compression, uint64_t base, uint8_t* d_file,
                uint64_t* d_handle_off, uint64_t* d_handle_size, uint64_t* d_end, uint8_t* scratch,
                const WriteScratch& W, hipStream_t s) {
  uint64_t* enc_off = (uint64_t*)(scratch + W.enc_off);
  uint32_t* enc_len = (uint32_t*)(scratch + W.enc_len);
  uint64_t* part = (uint64_t*)(scratch + W.part);
  uint64_t* foff = (uint64_t*)(scratch + W.foff);
  uint8_t* enc = scratch + W.enc;
  const bool snappy = compression == LGS_SNAPPY_COMPRESSION;
  if (snappy) {                       // table_builder.c:176-188, every block at once
    // Encode slots: one stride for all when n of the largest block's bound
    // fit (lcdb's near-uniform blocks: one fill instead of a three-kernel
    // scan), else the scan of every block's own bound.
    const uint64_t stride = (32 + (uint64_t)max_raw_len + max_raw_len / 6 + 15) & ~15ull;
    if (stride * n <= W.enc_cap)
      LGS_HIP(launch_fill_stride(enc_off, stride, n, s));
    else
      LGS_HIP(launch_scan(0, d_raw_len, nullptr, part, 0, enc_off, nullptr, n, s));
    EncodeArgs a{d_raw, d_raw_off, d_raw_len, enc, enc_off, enc_len, nullptr, nullptr, n, nullptr};
    LGS_HIP(launch_encode(a, max_raw_len, s));
  }
  // File offsets of the framed blocks (table_builder.c:150), then the blocks.
  LGS_HIP(launch_scan(1, d_raw_len, snappy ? enc_len : nullptr, part, base, foff, d_end, n, s));
  FrameArgs f{d_raw, d_raw_off, d_raw_len, enc, enc_off, snappy ? enc_len : nullptr,
              d_file, base, foff, d_handle_off, d_handle_size, n};
  LGS_HIP(launch_frame(f, s));
  return LGS_OK;
}

// A second stream per device and calling thread for the table reader's
// checksum pass (one per device for the whole process would serialise
// independent callers' passes on it).
static hipStream_t aux_stream() {
  thread_local hipStream_t s[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!s[dev] && hipStreamCreateWithFlags(&s[dev], hipStreamNonBlocking) != hipSuccess)
    s[dev] = nullptr;
  return s[dev];
}

struct EventPair {
  hipEvent_t e[2] = {nullptr, nullptr};
  ~EventPair() {
    for (hipEvent_t x : e)
      if (x) (void)hipEventDestroy(x);   // released once the work it marks completes
  }
};

static int table_read(const uint8_t* d_file, uint64_t file_len, const uint64_t* d_hoff,
               const uint64_t* d_hsize, uint32_t n, int verify, uint8_t* d_out,
               const uint64_t* d_out_off, const uint32_t* d_out_cap, uint32_t max_out_cap,
               uint32_t* d_out_len, uint8_t* d_status, uint8_t* scratch, const ReadScratch& R,
               hipStream_t s) {
  uint64_t* dec_in_off = (uint64_t*)(scratch + R.in_off);
  uint32_t* dec_len = (uint32_t*)(scratch + R.len);
  uint64_t* dec_off = (uint64_t*)(scratch + R.off);
  uint32_t* dec_cap = (uint32_t*)(scratch + R.cap);
  uint32_t* dec_olen = (uint32_t*)(scratch + R.olen);
  uint8_t* dec_st = scratch + R.st;
  uint8_t* bad = scratch + R.bad;
  // The dummy slot as an offset from d_out (two's complement wrap).
  const uint64_t dummy_off = (uint64_t)(uintptr_t)(scratch + R.dummy) - (uint64_t)(uintptr_t)d_out;
  // With checksums verified, the CRC pass (verify_kernel) runs on a second
  // stream beside the type dispatch and the decoder, which do not need its
  // result; the merge applies it first, as format.c:203-211 checks the
  // trailer before the type.  Outputs of a block that fails are unspecified.
  hipStream_t a = verify && options().verify_overlap.load() ? aux_stream() : nullptr;
  EventPair ev;
  CheckArgs c{d_file, file_len, d_hoff, d_hsize, verify && !a ? 1u : 0u, d_out, d_out_off, d_out_cap,
              d_out_len, d_status, dec_in_off, dec_len, dec_off, dec_cap, dummy_off, n};
  // (Without verification: one lane per handle; ahead of the verify pass the
  // wave-per-block check, lgs_table.hip.)
  LGS_HIP(verify ? launch_check(c, s) : launch_check_lane(c, s));
  if (a) {
    // After the type dispatch: queued with it, both ran slower (profiles/r6j),
    // and queued first but sleeping through it, its workgroups took the CUs
    // before the decoder's and left some without room for eight decoder
    // waves (365-493 us, profiles/r6r); the event costs ~8 us before the
    // decoder starts (profiles/r6i).
    LGS_HIP(hipEventCreateWithFlags(&ev.e[0], hipEventDisableTiming));
    LGS_HIP(hipEventCreateWithFlags(&ev.e[1], hipEventDisableTiming));
    LGS_HIP(hipEventRecord(ev.e[0], s));
    LGS_HIP(hipStreamWaitEvent(a, ev.e[0], 0));
    LGS_HIP(launch_verify(d_file, file_len, d_hoff, d_hsize, bad, n, a));
    LGS_HIP(hipEventRecord(ev.e[1], a));
  }
  DecodeArgs d{d_file, dec_in_off, dec_len, d_out, dec_off, dec_cap, dec_olen, dec_st, nullptr, n, nullptr};
  LGS_HIP(launch_decode(d, max_out_cap, s));
  if (a) LGS_HIP(hipStreamWaitEvent(s, ev.e[1], 0));
  LGS_HIP(launch_merge(d_status, d_out_len, dec_st, dec_olen, a ? bad : nullptr, n, s));
  return LGS_OK;
}

}  // namespace

size_t lgs_table_write_scratch(uint32_t n, uint64_t raw_total) {
  return WriteScratch(n, raw_total).total;
}

size_t lgs_table_read_scratch(uint32_t n) { return ReadScratch(n).total; }

int lgs_table_write_dev(const uint8_t* d_raw, const uint64_t* d_raw_off,
                        const uint32_t* d_raw_len, uint32_t n, uint32_t max_raw_len,
                        uint64_t raw_total, int compression, uint64_t base, uint8_t* d_file,
                        uint64_t* d_handle_off, uint64_t* d_handle_size, uint64_t* d_end,
                        void* d_scratch, size_t scratch_bytes, void* stream) {
  if (n == 0) return LGS_OK;
  if (!d_raw || !d_raw_off || !d_raw_len || !d_file || !d_handle_off || !d_handle_size ||
      !d_scratch)
    return fail(LGS_EINVAL, "NULL argument");
  if (compression != LGS_NO_COMPRESSION && compression != LGS_SNAPPY_COMPRESSION)
    return fail(LGS_EINVAL, "unknown compression type %d", compression);
  if (max_raw_len > 0x7fffffffu) return fail(LGS_EINVAL, "block of %u bytes too large", max_raw_len);
  const WriteScratch W(n, raw_total);
  if (scratch_bytes < W.total)
    return fail(LGS_EINVAL, "scratch of %zu bytes, %zu needed", scratch_bytes, W.total);
  return table_write(d_raw, d_raw_off, d_raw_len, n, max_raw_len, compression, base, d_file,
                     d_handle_off, d_handle_size, d_end, (uint8_t*)d_scratch, W,
                     (hipStream_t)stream);
}

int lgs_table_read_dev(const uint8_t* d_file, uint64_t file_len, const uint64_t* d_handle_off,
                       const uint64_t* d_handle_size, uint32_t n, int verify_checksums,
                       uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                       uint32_t max_out_cap, uint32_t* d_out_len, uint8_t* d_status,
                       void* d_scratch, size_t scratch_bytes, void* stream) {
  if (n == 0) return LGS_OK;
  if (!d_file || !d_handle_off || !d_handle_size || !d_out || !d_out_off || !d_out_cap ||
      !d_out_len || !d_status || !d_scratch)
    return fail(LGS_EINVAL, "NULL argument");
  const ReadScratch R(n);
  if (scratch_bytes < R.total)
    return fail(LGS_EINVAL, "scratch of %zu bytes, %zu needed", scratch_bytes, R.total);
  return table_read(d_file, file_len, d_handle_off, d_handle_size, n, verify_checksums, d_out,
                    d_out_off, d_out_cap, max_out_cap, d_out_len, d_status, (uint8_t*)d_scratch,
                    R, (hipStream_t)stream);
}

int lgs_table_write_host(const uint8_t* raw, const uint64_t* raw_off, const uint32_t* raw_len,
                         uint32_t n, int compression, uint64_t base, uint8_t* file,
                         size_t file_cap, uint64_t* handle_off, uint64_t* handle_size,
                         uint64_t* end) {
  if (!end) return fail(LGS_EINVAL, "NULL argument");
  if (n == 0) {
    *end = base;
    return LGS_OK;
  }
  if (!raw || !raw_off || !raw_len || !file || !handle_off || !handle_size)
    return fail(LGS_EINVAL, "NULL argument");
  if (compression != LGS_NO_COMPRESSION && compression != LGS_SNAPPY_COMPRESSION)
    return fail(LGS_EINVAL, "unknown compression type %d", compression);
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t in_total = 0;
  uint32_t max_in = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (raw_len[i] > 0x7fffffffu) return fail(LGS_EINVAL, "block %u too large", i);
    in_total += align_up(raw_len[i], 16);
    if (raw_len[i] > max_in) max_in = raw_len[i];
  }
  // Chunks of consecutive blocks are framed independently at file offset 0
  // (a block's framing does not depend on where it lands) and placed at
  // their running offset when they come back.  The staging is two slots,
  // each sized for the largest chunk, used by alternate chunks: the pinned
  // and device arenas stay bounded by the chunk size (LGS_HOST_CHUNK_MB),
  // not by the call, so a multi-GiB table does not pin its whole image.
  const std::vector<uint32_t> first = chunk_bounds(n, in_total, raw_len);
  const uint32_t chunks = (uint32_t)first.size() - 1;
  uint32_t max_n = 0;
  size_t max_inb = 0, max_fo = 0;
  uint64_t max_raw = 0;
  for (uint32_t k = 0; k < chunks; ++k) {
    uint64_t r = 0;
    size_t ib = 0;
    for (uint32_t i = first[k]; i < first[k + 1]; ++i) {
      r += raw_len[i];
      ib += align_up(raw_len[i], 16);
    }
    const uint32_t m = first[k + 1] - first[k];
    const size_t fo = align_up((size_t)r + LGS_TRAILER_SIZE * (size_t)m + 16, 256);
    if (m > max_n) max_n = m;
    if (r > max_raw) max_raw = r;
    if (ib > max_inb) max_inb = ib;
    if (fo > max_fo) max_fo = fo;
  }
  const WriteScratch W(max_n, max_raw + 16 * (uint64_t)max_n);
  Layout L;  // one slot: uploads | downloads | device-only
  const size_t o_in = L.take(max_inb + 16);
  const size_t o_ioff = L.take(8 * (size_t)max_n);
  const size_t o_ilen = L.take(4 * (size_t)max_n);
  const size_t o_hoff = L.take(8 * (size_t)max_n);
  const size_t o_hsize = L.take(8 * (size_t)max_n);
  const size_t o_end = L.take(8);
  const size_t o_file = L.take(max_fo);
  const size_t pin_slot = L.at;
  const size_t o_scr = L.take(W.total);
  const size_t dev_slot = L.at;
  const uint32_t nslot = chunks > 1 ? 2 : 1;
  LGS_TRY(ctx_reserve(c, nslot * dev_slot, nslot * pin_slot));
  uint64_t at = base;                      // file offset of the next chunk
  auto stage = [&](uint32_t k) {
    uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    uint64_t* ioff = (uint64_t*)(h + o_ioff);
    uint32_t* ilen = (uint32_t*)(h + o_ilen);
    size_t ia = o_in;
    for (uint32_t i = first[k]; i < first[k + 1]; ++i) {
      ioff[i - first[k]] = ia;
      ilen[i - first[k]] = raw_len[i];
      ia += align_up(raw_len[i], 16);
    }
    par_for(first[k + 1] - first[k], ia - o_in, [&](uint32_t j0, uint32_t j1) {
      for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t i = first[k] + j;
        memcpy(h + ioff[j], raw + raw_off[i], raw_len[i]);
      }
    });
  };
  auto launch = [&](uint32_t k, hipStream_t s) -> int {
    uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    uint8_t* d = c.d_buf + (k & 1) * dev_slot;
    const uint32_t m = first[k + 1] - first[k];
    const uint64_t* ioff = (const uint64_t*)(h + o_ioff);
    const size_t a1 = ioff[m - 1] + align_up(raw_len[first[k + 1] - 1], 16);
    LGS_HIP(hipMemcpyAsync(d + o_in, h + o_in, a1 - o_in, hipMemcpyHostToDevice, s));
    LGS_HIP(hipMemcpyAsync(d + o_ioff, h + o_ioff, 8 * (size_t)m, hipMemcpyHostToDevice, s));
    LGS_HIP(hipMemcpyAsync(d + o_ilen, h + o_ilen, 4 * (size_t)m, hipMemcpyHostToDevice, s));
    LGS_TRY(table_write(d, (const uint64_t*)(d + o_ioff), (const uint32_t*)(d + o_ilen), m, max_in,
                        compression, 0, d + o_file, (uint64_t*)(d + o_hoff),
                        (uint64_t*)(d + o_hsize), (uint64_t*)(d + o_end), d + o_scr, W, s));
    LGS_HIP(hipMemcpyAsync(h + o_hoff, d + o_hoff, 8 * (size_t)m, hipMemcpyDeviceToHost, s));
    LGS_HIP(hipMemcpyAsync(h + o_hsize, d + o_hsize, 8 * (size_t)m, hipMemcpyDeviceToHost, s));
    LGS_HIP(hipMemcpyAsync(h + o_end, d + o_end, 8, hipMemcpyDeviceToHost, s));
    // The region's size is known only on the device: its bound comes back.
    uint64_t r = 0;
    for (uint32_t i = first[k]; i < first[k + 1]; ++i) r += raw_len[i];
    const size_t fo = align_up((size_t)r + LGS_TRAILER_SIZE * (size_t)m + 16, 256);
    LGS_HIP(hipMemcpyAsync(h + o_file, d + o_file, fo, hipMemcpyDeviceToHost, s));
    return LGS_OK;
  };
  auto finish = [&](uint32_t k) -> int {
    const uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    const uint32_t i0 = first[k], m = first[k + 1] - i0;
    const uint64_t bytes = *(const uint64_t*)(h + o_end);
    if (at - base + bytes > file_cap)
      return fail(LGS_EINVAL, "file buffer of %zu bytes, %zu needed", file_cap,
                  (size_t)(at - base + bytes));
    const uint8_t* src = h + o_file;
    uint8_t* dst = file + (at - base);
    const uint32_t parts = 64;
    const size_t per = ((size_t)bytes + parts - 1) / parts;
    par_for(parts, (size_t)bytes, [&](uint32_t q0, uint32_t q1) {
      const size_t x0 = (size_t)q0 * per, x1 = (size_t)q1 * per < bytes ? (size_t)q1 * per : bytes;
      if (x0 < x1) memcpy(dst + x0, src + x0, x1 - x0);
    });
    const uint64_t* ho = (const uint64_t*)(h + o_hoff);
    const uint64_t* hs = (const uint64_t*)(h + o_hsize);
    for (uint32_t j = 0; j < m; ++j) {
      handle_off[i0 + j] = ho[j] + at;
      handle_size[i0 + j] = hs[j];
    }
    at += bytes;
    return LGS_OK;
  };
  LGS_TRY(pipeline(c, chunks, stage, launch, finish));
  *end = at;
  return LGS_OK;
}

int lgs_table_read_host(const uint8_t* file, uint64_t file_len, const uint64_t* handle_off,
                        const uint64_t* handle_size, uint32_t n, int verify_checksums,
                        uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                        uint32_t* out_len, uint8_t* status) {
  if (n == 0) return LGS_OK;
  if (!file || !handle_off || !handle_size || !out || !out_off || !out_cap || !out_len || !status)
    return fail(LGS_EINVAL, "NULL argument");
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  // Only each block's byte range (+ trailer) travels, packed 16-aligned into
  // its chunk's image; a range outside the file keeps an offset past that
  // image, so the device reports the truncated read itself (format.c:195-198).
  auto in_file = [&](uint32_t i) {
    const uint64_t o = handle_off[i], sz = handle_size[i];
    return sz <= ~0ull - LGS_TRAILER_SIZE && o <= file_len && file_len - o >= sz + LGS_TRAILER_SIZE;
  };
  size_t out_total = 0;
  uint32_t max_cap = 0;
  for (uint32_t i = 0; i < n; ++i) {
    out_total += align_up(out_cap[i], 16);
    if (out_cap[i] > max_cap) max_cap = out_cap[i];
  }
  // Chunks of consecutive handles through the two-stream pipeline (see
  // pipeline()), staged in two slots sized for the largest chunk (bounded
  // by LGS_HOST_CHUNK_MB, not by the call; see lgs_table_write_host).
  const std::vector<uint32_t> first = chunk_bounds(n, out_total, out_cap);
  const uint32_t chunks = (uint32_t)first.size() - 1;
  uint32_t max_n = 0;
  size_t max_blk = 0, max_out = 0;
  for (uint32_t k = 0; k < chunks; ++k) {
    size_t bb = 0, ob = 0;
    for (uint32_t i = first[k]; i < first[k + 1]; ++i) {
      if (in_file(i)) bb += align_up((size_t)handle_size[i] + LGS_TRAILER_SIZE, 16);
      ob += align_up(out_cap[i], 16);
    }
    if (first[k + 1] - first[k] > max_n) max_n = first[k + 1] - first[k];
    if (bb > max_blk) max_blk = bb;
    if (ob > max_out) max_out = ob;
  }
  const ReadScratch R(max_n);
  Layout L;  // one slot
  const size_t o_blk = L.take(max_blk + 16);
  const size_t o_hoff = L.take(8 * (size_t)max_n);
  const size_t o_hsize = L.take(8 * (size_t)max_n);
  const size_t o_ooff = L.take(8 * (size_t)max_n);
  const size_t o_ocap = L.take(4 * (size_t)max_n);
  const size_t o_st = L.take((size_t)max_n);
  const size_t o_olen = L.take(4 * (size_t)max_n);
  const size_t o_out = L.take(max_out + 16);
  const size_t pin_slot = L.at;
  const size_t o_scr = L.take(R.total);
  const size_t dev_slot = L.at;
  const uint32_t nslot = chunks > 1 ? 2 : 1;
  LGS_TRY(ctx_reserve(c, nslot * dev_slot, nslot * pin_slot));
  std::vector<size_t> blk_len(chunks, 0);   // each chunk's packed image length
  auto stage = [&](uint32_t k) {
    uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    uint64_t* hoff = (uint64_t*)(h + o_hoff);
    uint64_t* hsize = (uint64_t*)(h + o_hsize);
    uint64_t* ooff = (uint64_t*)(h + o_ooff);
    uint32_t* ocap = (uint32_t*)(h + o_ocap);
    size_t ba = 0, oa = o_out;
    const uint32_t i0 = first[k], m = first[k + 1] - i0;
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t i = i0 + j;
      hsize[j] = handle_size[i];
      hoff[j] = in_file(i) ? ba : ~0ull;
      if (in_file(i)) ba += align_up((size_t)handle_size[i] + LGS_TRAILER_SIZE, 16);
      ooff[j] = oa;
      ocap[j] = out_cap[i];
      oa += align_up(out_cap[i], 16);
    }
    blk_len[k] = ba;
    for (uint32_t j = 0; j < m; ++j)
      if (hoff[j] == ~0ull) hoff[j] = ba + 16 + 1;   // past the image: a truncated read
    par_for(m, ba, [&](uint32_t j0, uint32_t j1) {
      for (uint32_t j = j0; j < j1; ++j)
        if (hoff[j] <= ba)
          memcpy(h + o_blk + hoff[j], file + handle_off[i0 + j], (size_t)hsize[j] + LGS_TRAILER_SIZE);
    });
  };
  auto launch = [&](uint32_t k, hipStream_t s) -> int {
    uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    uint8_t* d = c.d_buf + (k & 1) * dev_slot;
    const uint32_t m = first[k + 1] - first[k];
    const uint64_t* ooff = (const uint64_t*)(h + o_ooff);
    if (blk_len[k] > 0)
      LGS_HIP(hipMemcpyAsync(d + o_blk, h + o_blk, blk_len[k], hipMemcpyHostToDevice, s));
    for (const size_t o : {o_hoff, o_hsize, o_ooff})
      LGS_HIP(hipMemcpyAsync(d + o, h + o, 8 * (size_t)m, hipMemcpyHostToDevice, s));
    LGS_HIP(hipMemcpyAsync(d + o_ocap, h + o_ocap, 4 * (size_t)m, hipMemcpyHostToDevice, s));
    LGS_TRY(table_read(d + o_blk, blk_len[k] + 16, (const uint64_t*)(d + o_hoff),
                       (const uint64_t*)(d + o_hsize), m, verify_checksums, d,
                       (const uint64_t*)(d + o_ooff), (const uint32_t*)(d + o_ocap), max_cap,
                       (uint32_t*)(d + o_olen), d + o_st, d + o_scr, R, s));
    LGS_HIP(hipMemcpyAsync(h + o_st, d + o_st, m, hipMemcpyDeviceToHost, s));
    LGS_HIP(hipMemcpyAsync(h + o_olen, d + o_olen, 4 * (size_t)m, hipMemcpyDeviceToHost, s));
    const size_t oe = ooff[m - 1] + align_up(out_cap[first[k + 1] - 1], 16);
    LGS_HIP(hipMemcpyAsync(h + o_out, d + o_out, oe - o_out, hipMemcpyDeviceToHost, s));
    return LGS_OK;
  };
  auto finish = [&](uint32_t k) -> int {
    const uint8_t* h = c.h_buf + (k & 1) * pin_slot;
    const uint32_t i0 = first[k], m = first[k + 1] - i0;
    const uint32_t* olen = (const uint32_t*)(h + o_olen);
    const uint64_t* ooff = (const uint64_t*)(h + o_ooff);
    const size_t bytes = ooff[m - 1] + out_cap[first[k + 1] - 1] - ooff[0];
    par_for(m, bytes, [&](uint32_t j0, uint32_t j1) {
      for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t i = i0 + j;
        status[i] = h[o_st + j];
        out_len[i] = olen[j];
        if (status[i] == LGS_ST_OK) memcpy(out + out_off[i], h + ooff[j], olen[j]);
      }
    });
    return LGS_OK;
  };
  LGS_TRY(pipeline(c, chunks, stage, launch, finish));
  return LGS_OK;
}

// ---- bloom filter (kernels: lgs_bloom.hip) ----

namespace {

static uint32_t bloom_k(int bpk) {                        // bloom.c:35-45
  size_t k = (size_t)(bpk * 0.69);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return (uint32_t)k;
}

static size_t bloom_bytes(uint64_t n, int bpk) {          // bloom.c:69-80
  uint64_t bits = n * (uint64_t)bpk;
  if (bits < 64) bits = 64;
  return (size_t)((bits + 7) / 8);
}

constexpr int kMaxBitsPerKey = 1 << 16;

}  // namespace

size_t lgs_bloom_filter_size(uint32_t nkeys, int bits_per_key) {
  if (nkeys == 0 || bits_per_key < 0) return 0;
  return bloom_bytes(nkeys, bits_per_key) + 1;
}

int lgs_bloom_build_dev(const uint8_t* d_keys, const uint64_t* d_key_off,
                        const uint32_t* d_key_len, const uint32_t* d_first, uint32_t nfilters,
                        int bits_per_key, uint8_t* d_out, const uint64_t* d_out_off,
                        void* stream) {
  if (nfilters == 0) return LGS_OK;
  if (!d_keys || !d_key_off || !d_key_len || !d_first || !d_out || !d_out_off)
    return fail(LGS_EINVAL, "NULL argument");
  if (bits_per_key < 0 || bits_per_key > kMaxBitsPerKey)
    return fail(LGS_EINVAL, "bits_per_key %d out of range", bits_per_key);
  LGS_HIP(launch_bloom_build(d_keys, d_key_off, d_key_len, d_first, nfilters,
                             (uint32_t)bits_per_key, bloom_k(bits_per_key), d_out, d_out_off,
                             0, (hipStream_t)stream));
  return LGS_OK;
}

int lgs_bloom_match_dev(const uint8_t* d_filters, const uint64_t* d_filter_off,
                        const uint32_t* d_filter_len, const uint32_t* d_query_filter,
                        const uint8_t* d_keys, const uint64_t* d_key_off,
                        const uint32_t* d_key_len, uint8_t* d_match, uint32_t nq, void* stream) {
  if (nq == 0) return LGS_OK;
  if (!d_filters || !d_filter_off || !d_filter_len || !d_query_filter || !d_keys || !d_key_off ||
      !d_key_len || !d_match)
    return fail(LGS_EINVAL, "NULL argument");
  LGS_HIP(launch_bloom_match(d_filters, d_filter_off, d_filter_len, d_query_filter, d_keys,
                             d_key_off, d_key_len, d_match, nq, (hipStream_t)stream));
  return LGS_OK;
}

int lgs_bloom_build_host(const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len,
                         const uint32_t* first, uint32_t nfilters, int bits_per_key,
                         uint8_t* out, const uint64_t* out_off) {
  if (nfilters == 0) return LGS_OK;
  if (!keys || !key_off || !key_len || !first || !out || !out_off)
    return fail(LGS_EINVAL, "NULL argument");
  if (bits_per_key < 0 || bits_per_key > kMaxBitsPerKey)
    return fail(LGS_EINVAL, "bits_per_key %d out of range", bits_per_key);
  for (uint32_t f = 0; f < nfilters; ++f)
    if (first[f + 1] < first[f]) return fail(LGS_EINVAL, "first[] decreases at filter %u", f);
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  const uint32_t nkeys = first[nfilters] - first[0];
  const uint32_t k0 = first[0];
  size_t key_bytes = 0, filt_bytes = 0;
  for (uint32_t i = k0; i < k0 + nkeys; ++i) key_bytes += key_len[i];
  for (uint32_t f = 0; f < nfilters; ++f)
    filt_bytes += lgs_bloom_filter_size(first[f + 1] - first[f], bits_per_key);
  Layout L;  // upload | download
  const size_t o_keys = L.take(key_bytes + 16);
  const size_t o_koff = L.take(8 * (size_t)nkeys);
  const size_t o_klen = L.take(4 * (size_t)nkeys);
  const size_t o_first = L.take(4 * ((size_t)nfilters + 1));
  const size_t o_foff = L.take(8 * (size_t)nfilters);
  const size_t up_end = L.at;
  const size_t o_filt = L.take(filt_bytes + 16);
  const size_t down_end = L.at;
  LGS_TRY(ctx_reserve(c, down_end, down_end));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  uint64_t* koff = (uint64_t*)(h + o_koff);
  uint32_t* klen = (uint32_t*)(h + o_klen);
  uint32_t* fst = (uint32_t*)(h + o_first);
  uint64_t* foff = (uint64_t*)(h + o_foff);
  size_t at = o_keys;
  for (uint32_t j = 0; j < nkeys; ++j) {
    memcpy(h + at, keys + key_off[k0 + j], key_len[k0 + j]);
    koff[j] = at;
    klen[j] = key_len[k0 + j];
    at += key_len[k0 + j];
  }
  memset(h + at, 0, 16);
  size_t fat = 0;
  for (uint32_t f = 0; f <= nfilters; ++f) fst[f] = first[f] - k0;
  for (uint32_t f = 0; f < nfilters; ++f) {
    foff[f] = fat;
    fat += lgs_bloom_filter_size(first[f + 1] - first[f], bits_per_key);
  }
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  LGS_HIP(launch_bloom_build(d, (const uint64_t*)(d + o_koff), (const uint32_t*)(d + o_klen),
                             (const uint32_t*)(d + o_first), nfilters, (uint32_t)bits_per_key,
                             bloom_k(bits_per_key), d + o_filt, (const uint64_t*)(d + o_foff),
                             0, c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_filt, d + o_filt, filt_bytes, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  for (uint32_t f = 0; f < nfilters; ++f)
    memcpy(out + out_off[f], h + o_filt + foff[f],
           lgs_bloom_filter_size(first[f + 1] - first[f], bits_per_key));
  return LGS_OK;
}

int lgs_bloom_match_host(const uint8_t* filters, const uint64_t* filter_off,
                         const uint32_t* filter_len, uint32_t nfilters,
                         const uint32_t* query_filter, const uint8_t* keys,
                         const uint64_t* key_off, const uint32_t* key_len, uint32_t nq,
                         uint8_t* match) {
  if (nq == 0) return LGS_OK;
  if (!filters || !filter_off || !filter_len || !query_filter || !keys || !key_off || !key_len ||
      !match)
    return fail(LGS_EINVAL, "NULL argument");
  for (uint32_t q = 0; q < nq; ++q)
    if (query_filter[q] >= nfilters)
      return fail(LGS_EINVAL, "query %u names filter %u of %u", q, query_filter[q], nfilters);
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t fb = 0, kb = 0;
  for (uint32_t f = 0; f < nfilters; ++f) fb += filter_len[f];
  for (uint32_t q = 0; q < nq; ++q) kb += key_len[q];
  Layout L;
  const size_t o_f = L.take(fb + 16);
  const size_t o_foff = L.take(8 * (size_t)nfilters);
  const size_t o_flen = L.take(4 * (size_t)nfilters);
  const size_t o_qf = L.take(4 * (size_t)nq);
  const size_t o_k = L.take(kb + 16);
  const size_t o_koff = L.take(8 * (size_t)nq);
  const size_t o_klen = L.take(4 * (size_t)nq);
  const size_t up_end = L.at;
  const size_t o_m = L.take(nq);
  const size_t down_end = L.at;
  LGS_TRY(ctx_reserve(c, down_end, down_end));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  uint64_t* foff = (uint64_t*)(h + o_foff);
  uint32_t* flen = (uint32_t*)(h + o_flen);
  uint64_t* koff = (uint64_t*)(h + o_koff);
  uint32_t* klen = (uint32_t*)(h + o_klen);
  size_t at = 0;
  for (uint32_t f = 0; f < nfilters; ++f) {
    memcpy(h + o_f + at, filters + filter_off[f], filter_len[f]);
    foff[f] = at;
    flen[f] = filter_len[f];
    at += filter_len[f];
  }
  memset(h + o_f + at, 0, 16);
  memcpy(h + o_qf, query_filter, 4 * (size_t)nq);
  at = 0;
  for (uint32_t q = 0; q < nq; ++q) {
    memcpy(h + o_k + at, keys + key_off[q], key_len[q]);
    koff[q] = at;
    klen[q] = key_len[q];
    at += key_len[q];
  }
  memset(h + o_k + at, 0, 16);
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  LGS_HIP(launch_bloom_match(d + o_f, (const uint64_t*)(d + o_foff), (const uint32_t*)(d + o_flen),
                             (const uint32_t*)(d + o_qf), d + o_k, (const uint64_t*)(d + o_koff),
                             (const uint32_t*)(d + o_klen), d + o_m, nq, c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_m, d + o_m, nq, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  memcpy(match, h + o_m, nq);
  return LGS_OK;
}

// ---- the filter block (filter_block.c; kernels: lgs_bloom.hip) ----

namespace {

constexpr uint64_t kMaxDataEnd = 1ull << 42;   // 2^31 filters: offsets fit the u32 array

struct FilterScratch {
  size_t kf, foff, part, meta, total;
  explicit FilterScratch(uint64_t data_end) {
    const size_t nf = (size_t)(data_end >> 11) + 2;
    Layout L;
    kf = L.take(4 * nf);
    foff = L.take(8 * nf);
    part = L.take(8 * filter_block_parts(data_end));
    meta = L.take(12);
    total = L.at;
  }
};

static int filter_args(uint32_t nblocks, uint64_t data_end, int bits_per_key, int internal_keys) {
  if (bits_per_key < 0 || bits_per_key > kMaxBitsPerKey)
    return fail(LGS_EINVAL, "bits_per_key %d out of range", bits_per_key);
  if (data_end >= kMaxDataEnd) return fail(LGS_EINVAL, "data_end %llu too large",
                                           (unsigned long long)data_end);
  if (internal_keys != 0 && internal_keys != 1)
    return fail(LGS_EINVAL, "internal_keys must be 0 or 1");
  (void)nblocks;
  return LGS_OK;
}

}  // namespace

size_t lgs_filter_block_bound(uint32_t nkeys, uint32_t nblocks, uint64_t data_end,
                              int bits_per_key) {
  if (bits_per_key < 0 || data_end >= kMaxDataEnd) return 0;
  // Nonempty filters <= nblocks, each <= n * bpk / 8 + 10 bytes; 4 bytes per
  // filter offset (<= data_end / 2048 + 1 of them), 5 trailing.
  return (size_t)(((uint64_t)nkeys * (uint64_t)bits_per_key + 7) / 8 + 10ull * nblocks +
                  4ull * ((data_end >> 11) + 1) + 5);
}

size_t lgs_filter_block_scratch(uint64_t data_end) {
  if (data_end >= kMaxDataEnd) return 0;
  return FilterScratch(data_end).total;
}

int lgs_filter_block_build_dev(const uint8_t* d_keys, const uint64_t* d_key_off,
                               const uint32_t* d_key_len, uint32_t nkeys,
                               const uint32_t* d_block_first, const uint64_t* d_block_off,
                               uint32_t nblocks, uint64_t data_end, int bits_per_key,
                               int internal_keys, uint8_t* d_out, size_t out_cap,
                               uint64_t* d_size, void* d_scratch, size_t scratch_bytes,
                               void* stream) {
  LGS_TRY(filter_args(nblocks, data_end, bits_per_key, internal_keys));
  if (!d_block_first || !d_out || !d_size || !d_scratch || (nblocks && !d_block_off) ||
      (nkeys && (!d_keys || !d_key_off || !d_key_len)))
    return fail(LGS_EINVAL, "NULL argument");
  const FilterScratch S(data_end);
  if (scratch_bytes < S.total)
    return fail(LGS_EINVAL, "scratch %zu < %zu (lgs_filter_block_scratch)", scratch_bytes,
                S.total);
  const size_t bound = lgs_filter_block_bound(nkeys, nblocks, data_end, bits_per_key);
  if (out_cap < bound)
    return fail(LGS_ENOSPC, "out_cap %zu < %zu (lgs_filter_block_bound)", out_cap, bound);
  uint8_t* sc = (uint8_t*)d_scratch;
  LGS_HIP(launch_filter_block_build(d_keys, d_key_off, d_key_len, d_block_first, d_block_off,
                                    nblocks, data_end, (uint32_t)bits_per_key,
                                    bloom_k(bits_per_key), internal_keys ? 8u : 0u, d_out,
                                    d_size, (uint32_t*)(sc + S.kf), (uint64_t*)(sc + S.foff),
                                    (uint64_t*)(sc + S.part), (uint32_t*)(sc + S.meta),
                                    (hipStream_t)stream));
  return LGS_OK;
}

int lgs_filter_block_build_host(const uint8_t* keys, const uint64_t* key_off,
                                const uint32_t* key_len, const uint32_t* block_first,
                                const uint64_t* block_off, uint32_t nblocks, uint64_t data_end,
                                int bits_per_key, int internal_keys, uint8_t* out,
                                size_t out_cap, size_t* size) {
  LGS_TRY(filter_args(nblocks, data_end, bits_per_key, internal_keys));
  if (!block_first || !out || !size || (nblocks && !block_off))
    return fail(LGS_EINVAL, "NULL argument");
  for (uint32_t b = 0; b < nblocks; ++b) {
    if (block_first[b + 1] < block_first[b])
      return fail(LGS_EINVAL, "block_first[] decreases at block %u", b);
    if ((b + 1 < nblocks ? block_off[b + 1] : data_end) < block_off[b])
      return fail(LGS_EINVAL, "block offsets decrease at block %u", b);
  }
  const uint32_t k0 = block_first[0], nkeys = block_first[nblocks] - k0;
  if (nkeys && (!keys || !key_off || !key_len)) return fail(LGS_EINVAL, "NULL argument");
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t key_bytes = 0;
  for (uint32_t i = k0; i < k0 + nkeys; ++i) key_bytes += key_len[i];
  const size_t bound = lgs_filter_block_bound(nkeys, nblocks, data_end, bits_per_key);
  const FilterScratch S(data_end);
  Layout L;  // upload | scratch | download
  const size_t o_keys = L.take(key_bytes + 16);
  const size_t o_koff = L.take(8 * (size_t)nkeys);
  const size_t o_klen = L.take(4 * (size_t)nkeys);
  const size_t o_bf = L.take(4 * ((size_t)nblocks + 1));
  const size_t o_bo = L.take(8 * (size_t)nblocks);
  const size_t up_end = L.at;
  const size_t o_scr = L.take(S.total);
  const size_t o_size = L.take(8);
  const size_t o_out = L.take(bound);
  const size_t down_end = o_out + bound;
  LGS_TRY(ctx_reserve(c, L.at, L.at));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  uint64_t* koff = (uint64_t*)(h + o_koff);
  uint32_t* klen = (uint32_t*)(h + o_klen);
  uint32_t* bf = (uint32_t*)(h + o_bf);
  size_t at = o_keys;
  for (uint32_t j = 0; j < nkeys; ++j) {
    memcpy(h + at, keys + key_off[k0 + j], key_len[k0 + j]);
    koff[j] = at;
    klen[j] = key_len[k0 + j];
    at += key_len[k0 + j];
  }
  memset(h + at, 0, 16);
  for (uint32_t b = 0; b <= nblocks; ++b) bf[b] = block_first[b] - k0;
  if (nblocks) memcpy(h + o_bo, block_off, 8 * (size_t)nblocks);
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  LGS_TRY(lgs_filter_block_build_dev(d, (const uint64_t*)(d + o_koff),
                                     (const uint32_t*)(d + o_klen), nkeys,
                                     (const uint32_t*)(d + o_bf), (const uint64_t*)(d + o_bo),
                                     nblocks, data_end, bits_per_key, internal_keys, d + o_out,
                                     bound, (uint64_t*)(d + o_size), d + o_scr, S.total,
                                     c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_size, d + o_size, down_end - o_size, hipMemcpyDeviceToHost,
                         c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  const uint64_t n = *(const uint64_t*)(h + o_size);
  if (n > bound) return fail(LGS_EINTERNAL, "filter block %llu > bound %zu",
                             (unsigned long long)n, bound);
  *size = (size_t)n;
  if (n > out_cap) return fail(LGS_ENOSPC, "filter block needs %llu bytes, out_cap %zu",
                               (unsigned long long)n, out_cap);
  memcpy(out, h + o_out, (size_t)n);
  return LGS_OK;
}

int lgs_filter_block_match_dev(const uint8_t* d_block, size_t block_len,
                               const uint64_t* d_block_offset, const uint8_t* d_keys,
                               const uint64_t* d_key_off, const uint32_t* d_key_len, uint32_t nq,
                               int internal_keys, uint8_t* d_match, void* stream) {
  if (nq == 0) return LGS_OK;
  if ((block_len && !d_block) || !d_block_offset || !d_keys || !d_key_off || !d_key_len ||
      !d_match)
    return fail(LGS_EINVAL, "NULL argument");
  if (internal_keys != 0 && internal_keys != 1)
    return fail(LGS_EINVAL, "internal_keys must be 0 or 1");
  LGS_HIP(launch_filter_block_match(d_block, block_len, d_block_offset, d_keys, d_key_off,
                                    d_key_len, internal_keys ? 8u : 0u, d_match, nq,
                                    (hipStream_t)stream));
  return LGS_OK;
}

int lgs_filter_block_match_host(const uint8_t* block, size_t block_len,
                                const uint64_t* block_offset, const uint8_t* keys,
                                const uint64_t* key_off, const uint32_t* key_len, uint32_t nq,
                                int internal_keys, uint8_t* match) {
  if (nq == 0) return LGS_OK;
  if ((block_len && !block) || !block_offset || !keys || !key_off || !key_len || !match)
    return fail(LGS_EINVAL, "NULL argument");
  Lease lease(batch_pool());
  LGS_TRY(lease.acquire());
  Ctx& c = lease.ctx();
  size_t kb = 0;
  for (uint32_t q = 0; q < nq; ++q) kb += key_len[q];
  Layout L;
  const size_t o_b = L.take(block_len + 16);
  const size_t o_qo = L.take(8 * (size_t)nq);
  const size_t o_k = L.take(kb + 16);
  const size_t o_koff = L.take(8 * (size_t)nq);
  const size_t o_klen = L.take(4 * (size_t)nq);
  const size_t up_end = L.at;
  const size_t o_m = L.take(nq);
  LGS_TRY(ctx_reserve(c, L.at, L.at));
  uint8_t* h = c.h_buf;
  uint8_t* d = c.d_buf;
  if (block_len) memcpy(h + o_b, block, block_len);
  memcpy(h + o_qo, block_offset, 8 * (size_t)nq);
  uint64_t* koff = (uint64_t*)(h + o_koff);
  uint32_t* klen = (uint32_t*)(h + o_klen);
  size_t at = 0;
  for (uint32_t q = 0; q < nq; ++q) {
    memcpy(h + o_k + at, keys + key_off[q], key_len[q]);
    koff[q] = at;
    klen[q] = key_len[q];
    at += key_len[q];
  }
  memset(h + o_k + at, 0, 16);
  LGS_HIP(hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, c.stream));
  LGS_TRY(lgs_filter_block_match_dev(d + o_b, block_len, (const uint64_t*)(d + o_qo), d + o_k,
                                     (const uint64_t*)(d + o_koff),
                                     (const uint32_t*)(d + o_klen), nq, internal_keys, d + o_m,
                                     c.stream));
  LGS_HIP(hipMemcpyAsync(h + o_m, d + o_m, nq, hipMemcpyDeviceToHost, c.stream));
  LGS_HIP(hipStreamSynchronize(c.stream));
  memcpy(match, h + o_m, nq);
  return LGS_OK;
}

int lgs_device_count(void) { return visible_devices(); }

int lgs_set_device(int device) {
  int count = lgs_device_count();
  if (device < 0 || device >= count)
    return fail(LGS_ENODEV, "device %d not present (%d visible)", device, count);
  t_want_device = device;
  return LGS_OK;
}

const char* lgs_last_error(void) { return t_err; }

const char* lgs_version(void) { return "lcdb_gpu_snappy 0.1 gfx950"; }

}  // extern "C"
