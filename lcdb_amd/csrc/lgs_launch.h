// lgs_launch.h -- host-side launch interface between the runtime
// (lgs_api.cpp) and the kernels (lgs_encode.hip, lgs_decode.hip,
// lgs_table.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>

namespace lgs {

// Process-wide kernel choices (lgs_set_option; the initial values come from
// LGS_DECODE_KERNEL / LGS_NO_SPLIT, read once at load -- nothing on the
// launch path reads the environment).
enum DecodeKernel {
  kDecAuto = 0, kDecRing = 1, kDecWave = 2, kDecQuad = 3, kDecOps = 4, kDecGroup = 5, kDecChain = 6
};
// Outputs over the 16 KiB class: the one-tag walk (default), or, in the
// probe library, the trip decoder or the workgroup decoder.
enum WideKernel { kWideWalk = 0, kWideTrips = 1, kWideGroup = 2 };
struct Options {
  std::atomic<int> decoder{kDecAuto};   // DecodeKernel
  std::atomic<int> split{1};            // size-class split of mixed batches
  std::atomic<int> wide{0};             // WideKernel: the decoder of the wide class
  std::atomic<int> verify_overlap{1};   // table reads: trailer CRCs beside the decoder
};
Options& options();

// One work item's offsets and lengths passed by value (the drop-in, whose
// per-item arrays sit in mapped host memory: reading them would cost the
// kernel a PCIe round trip before it can load the stream).  on == 0: the
// kernels read the arrays.  Kernels that do not take it read the arrays,
// which the drop-in fills as well.
struct Item1 {
  uint64_t in_off = 0, out_off = 0;
  uint32_t in_len = 0, aux = 0;   // aux: decode out_cap, encode hdr
  uint32_t on = 0;
};

struct DecodeArgs {
  const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
  uint8_t* out; const uint64_t* out_off; const uint32_t* out_cap;
  uint32_t* out_len; uint8_t* status; const uint32_t* index; uint32_t n;
  const uint32_t* count;   // device count of index[] entries (nullptr: n)
  Item1 one{};             // item 0 by value (decode_kernel)
};

struct EncodeArgs {
  const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
  uint8_t* out; const uint64_t* out_off; uint32_t* out_len;
  const uint32_t* hdr; const uint32_t* index; uint32_t n;
  const uint32_t* count;   // device count of index[] entries (nullptr: n)
  Item1 one{};             // item 0 by value (encode_kernel)
};

// max_out: largest out_cap in the launch (selects the LDS class).
hipError_t launch_decode(const DecodeArgs& a, uint32_t max_out, hipStream_t s);
#ifdef LGS_PROBE_DECODERS
// Probe library only (lgs_decode_probe.hip): the decoders that lost their
// A/B, selectable through lgs_set_option for tests and measurements.
hipError_t launch_decode_quad(const DecodeArgs& a, hipStream_t s);
hipError_t launch_decode_ops(const DecodeArgs& a, hipStream_t s);
hipError_t launch_decode_trips(const DecodeArgs& a, hipStream_t s);
#endif
// The ring decoder (lane per block, large batches), for the split launch.
hipError_t launch_decode_ring(const DecodeArgs& a, hipStream_t s);

#ifdef LGS_PROBE_DECODERS
// Probe library only: the workgroup (pointer-jumping) decoder of
// lgs_decode_group.hip, outputs up to kGroupMaxOut bytes, and the chain
// decoder of lgs_decode_chain.hip (a wave per block, the tag walk apart
// from the byte moves), outputs up to kChainMaxOut bytes.
constexpr uint32_t kGroupMaxOut = 66048;
hipError_t launch_decode_group(const DecodeArgs& a, uint32_t max_out, hipStream_t s);
constexpr uint32_t kChainMaxOut = 16896;
hipError_t launch_decode_chain(const DecodeArgs& a, uint32_t max_out, hipStream_t s);
#endif
// max_in: largest item length in the launch (<= 65536).
hipError_t launch_encode(const EncodeArgs& a, uint32_t max_in, hipStream_t s);
// Sort a mixed-size batch into size classes on the device: class c holds
// the items with len in (b[c-1], b[c]] (b[3] = infinity); list[c * n + k]
// is its k-th item (in no particular order), cnt[c] its size.  cnt must be
// zeroed beforehand.
// Below this many blocks a split gains nothing (each wave has a CU to
// itself whatever its LDS class) and would only add its fixed cost to
// latency-bound calls such as the drop-in's single blocks.
constexpr uint32_t kSplitMinBlocks = 512;
hipError_t launch_classify(const uint32_t* len, uint32_t n, uint32_t b0, uint32_t b1, uint32_t b2,
                           uint32_t* list, uint32_t* cnt, hipStream_t s);
// Stream-ordered scratch of a split launch, from a private memory pool of
// the current device (the process's default pool is left alone: this
// library is loaded into lcdb).  Freed on the stream when the guard leaves
// scope, on every path; release() frees it early and reports the error.
class Scratch {
 public:
  Scratch(size_t bytes, hipStream_t s);
  ~Scratch() { (void)release(); }
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  hipError_t status() const { return err_; }
  void* get() const { return p_; }
  hipError_t release() {
    void* p = p_;
    p_ = nullptr;
    return p ? hipFreeAsync(p, s_) : hipSuccess;
  }

 private:
  void* p_ = nullptr;
  hipStream_t s_;
  hipError_t err_;
};

// ---- the drop-in service: resident encode / decode waves ----
//
// A drop-in call of one small block spends ~17 us on a kernel launch and a
// stream synchronisation (profiles/r4z_dropin_breakdown.json).  The service
// keeps one wave per drop-in slot resident instead: wave k of the encode (or
// decode) service kernel polls mailbox k in the slot's mapped pinned memory,
// runs the ordinary single-block walk on the slot's arena when the host posts
// a request, and posts completion back.  The kernel's waves leave together
// after `idle` 100 MHz ticks without a request anywhere in it (so a
// device-wide synchronisation waits at most that long after the last call
// from any thread), and a wave leaves when the host sets its stop flag; the
// host relaunches the kernel when a request finds it gone.
constexpr uint32_t kSvcMaxSlots = 64;      // mailboxes per kind
constexpr uint32_t kSvcMaxItem = 4608;     // the 4 KiB LDS class (encode input / decode output)
constexpr uint32_t kSvcIn = 0;             // arena offset of the request's input
constexpr uint32_t kSvcOut = 8192;         // arena offset of its output (>= 16 + bound(4608))

struct alignas(128) SvcMailbox {
  // host -> device: one 16-byte group (read in one request) + the arena
  uint32_t req;      // sequence number of the posted request
  uint32_t len;      // input bytes at arena + kSvcIn
  uint32_t aux;      // encode: the varint header value; decode: the output capacity
  uint32_t stop;     // nonzero: the wave exits
  uint64_t arena;    // device address of the slot's mapped arena
  uint64_t pad0[5];
  // device -> host
  uint32_t ack;      // sequence number of the last finished request
  uint32_t status;   // decode: LGS_ST_*; encode: 1
  uint32_t out_len;  // bytes written at arena + kSvcOut
  uint32_t pad1[13];
};
static_assert(sizeof(SvcMailbox) == 128, "mailbox layout");

// Device memory shared by one service kernel's waves (lgs_service.h).
struct alignas(64) SvcControl {
  uint64_t activity;   // the kernel's last request picked up or answered, 100 MHz ticks
  uint64_t closing;    // nonzero: every wave leaves (set by the first idle wave; the host clears it)
  uint64_t pad[6];
};

// nslots waves polling mb[0 .. nslots).
hipError_t launch_encode_service(SvcMailbox* mb, uint32_t nslots, uint64_t idle,
                                 SvcControl* ctl, hipStream_t s);
hipError_t launch_decode_service(SvcMailbox* mb, uint32_t nslots, uint64_t idle,
                                 SvcControl* ctl, hipStream_t s);

// ---- SSTable block framing (lgs_table.hip) ----

// Per-block status codes (the LGS_ST_* values of include/lcdb_gpu_snappy.h).
constexpr uint32_t kStCorrupt = 0, kStOk = 1, kStNoSpace = 2, kStIoErr = 3, kStBadCrc = 4,
                   kStBadType = 5;

struct FrameArgs {
  const uint8_t* raw; const uint64_t* raw_off; const uint32_t* raw_len;
  // Encoder output; enc_len == nullptr: no compression (every block raw).
  const uint8_t* enc; const uint64_t* enc_off; const uint32_t* enc_len;
  uint8_t* file; uint64_t base; const uint64_t* foff;
  uint64_t* handle_off; uint64_t* handle_size; uint32_t n;
};

struct CheckArgs {
  const uint8_t* file; uint64_t file_len; const uint64_t* hoff; const uint64_t* hsize;
  uint32_t verify; uint8_t* out; const uint64_t* out_off; const uint32_t* out_cap;
  uint32_t* out_len; uint8_t* status;
  uint64_t* dec_in_off; uint32_t* dec_len; uint64_t* dec_off; uint32_t* dec_cap;
  uint64_t dummy_off; uint32_t n;
};

// CRC32C of each block (followed by its type byte when type != null),
// masked (crc32c.h:46-50) or not.
hipError_t launch_crc(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      const uint8_t* type, int masked, uint32_t* crc, uint32_t n, hipStream_t s);
// Exclusive scan of per-item region sizes (mode 0: 16-aligned encode bounds;
// mode 1: framed block sizes; mode 2: enc_len itself) into u64 offsets
// starting at base; *end = base + total when end != null.  part:
// scan_parts(n) u64 of device scratch.
size_t scan_parts(uint32_t n);
hipError_t launch_scan(int mode, const uint32_t* raw_len, const uint32_t* enc_len, uint64_t* part,
                       uint64_t base, uint64_t* off, uint64_t* end, uint32_t n, hipStream_t s);
hipError_t launch_frame(const FrameArgs& a, hipStream_t s);
// Item i's len[i] bytes from src + src_off[i] to dst + dst_off[i] (any
// alignment; the regions do not overlap).
hipError_t launch_pack(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                       uint8_t* dst, const uint64_t* dst_off, uint32_t n, hipStream_t s);
hipError_t launch_check(const CheckArgs& a, hipStream_t s);
hipError_t launch_merge(uint8_t* status, uint32_t* out_len, const uint8_t* dec_status,
                        const uint32_t* dec_out_len, const uint8_t* bad, uint32_t n,
                        hipStream_t s);
// The trailer CRC checks alone (bad[i] = 1 on a mismatch), sized to run
// beside the ring decoder.
hipError_t launch_verify(const uint8_t* file, uint64_t file_len, const uint64_t* hoff,
                         const uint64_t* hsize, uint8_t* bad, uint32_t n, hipStream_t s);

// ---- bloom filter (lgs_bloom.hip) ----

// Filters f = keys [first[f], first[f+1]) written at out + out_off[f]
// (bloom.c:102-119); bpk = bits per key, k = probes (bloom.c:35-45); each
// key hashed without its last `trim` bytes (8: the internal filter policy).
hipError_t launch_bloom_build(const uint8_t* keys, const uint64_t* key_off,
                              const uint32_t* key_len, const uint32_t* first, uint32_t nfilters,
                              uint32_t bpk, uint32_t k, uint8_t* out, const uint64_t* out_off,
                              uint32_t trim, hipStream_t s);
// match[q] = bloom_match(filter qfilter[q], key q) (bloom.c:121-165).
hipError_t launch_bloom_match(const uint8_t* filters, const uint64_t* filter_off,
                              const uint32_t* filter_len, const uint32_t* qfilter,
                              const uint8_t* keys, const uint64_t* key_off,
                              const uint32_t* key_len, uint8_t* match, uint32_t nq,
                              hipStream_t s);
// The filter block of one table (filter_block.c:79-150 as table_builder.c
// drives it): data block b = keys [block_first[b], block_first[b+1]) at file
// offset block_off[b]; data_end = offset after the last one.  Scratch: kf
// (fmax + 1 u32), foff (fmax + 1 u64), meta (1 u32), fmax = data_end/2048 + 1.
// out receives the block, size[0] its length.
hipError_t launch_filter_block_build(const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, const uint32_t* block_first,
                                     const uint64_t* block_off, uint32_t nblocks,
                                     uint64_t data_end, uint32_t bpk, uint32_t k, uint32_t trim,
                                     uint8_t* out, uint64_t* size, uint32_t* kf, uint64_t* foff,
                                     uint64_t* part, uint32_t* meta, hipStream_t s);
size_t filter_block_parts(uint64_t data_end);
// match[q] = ldb_filter_matches(block, qoff[q], key q) (filter_block.c:170-225).
hipError_t launch_filter_block_match(const uint8_t* blk, uint64_t n, const uint64_t* qoff,
                                     const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, uint32_t trim, uint8_t* match,
                                     uint32_t nq, hipStream_t s);

// ---- HBM copy probe (lgs_probe.hip; bench yardstick, not the codec) ----
// dst/src 16-byte aligned, bytes a multiple of 16.
hipError_t launch_hbm_copy(void* dst, const void* src, size_t bytes, hipStream_t s);

// Host runtime (lgs_api.cpp): record msg as lgs_last_error(); returns code.
int set_error(int code, const char* msg);

}  // namespace lgs
