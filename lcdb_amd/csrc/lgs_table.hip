// lgs_table.hip -- SSTable block framing on gfx950:
//
//  * CRC32C of a block and its type byte, masked: the 5-byte block trailer
//    of src/table/table_builder.c:134-147 (crc32c.c:643-750, crc32c.h:38-57);
//  * the batched data-block writer: snappy encode (lgs_encode.hip), the
//    12.5 % rule of table_builder.c:190, trailers, and the blocks packed at
//    their file offsets (table_builder.c:123-153), byte-identical to
//    ldb_tablegen_write_block called once per block;
//  * the batched block reader: format.c:162-270 per block handle -- the
//    truncation check, the trailer CRC check (verify_checksums), the type
//    dispatch, raw copy or snappy decode (lgs_decode.hip).
//
// CRC32C on a wave (lgs_crc.h; one block per wave by default, two with
// LGS_CRC_LANES=32).  CRC32C is linear over GF(2), so the lanes split a
// block into segments of kSeg bytes (48 by default), one per lane, and
// combine them:
//  * the block's bytes are taken where they lie, as the aligned 16-byte
//    granules that hold them (only those: never another page), extended by
//    t < 16 trailing zeros to the end of the last granule and by leading
//    zeros to a whole number of passes (a "pass" = lanes x kSeg bytes).
//    Leading zeros leave a register that is 0 at 0; the ~0
//    pre-conditioning is the start register of the lane holding byte 0
//    (the register that its leading zeros turn into ~0); the trailing
//    zeros are divided out at the end (a multiplication by x^(-8t));
//  * a lane folds its dwords with slice-by-8 tables (eight bytes per
//    dependent step; slice-by-4 in the verify pass's small image), then
//    multiplies its CRC by x^(8 kSeg (lanes - 1 - lane)) -- the zero bytes
//    after its segment -- with a table of its own (eight nibble lookups),
//    and one DPP xor-reduction gives the pass's CRC (the small image: a
//    butterfly of shifts instead).  The CRC of the passes before enters as
//    lane 0's start register.
// Copies to the destination (the file image on the write path, the output
// slot of a raw block on the read path) are a pass of their own over whole
// aligned destination granules (copy_bytes).
#include "lgs_device.h"
#include "lgs_launch.h"

#include "lgs_crc.h"

namespace lgs {
namespace {

// ---- row 1: masked (or plain) CRC32C per block -------------------------

template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void crc_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
    const uint32_t* __restrict__ in_len, const uint8_t* __restrict__ type,
    uint32_t masked, uint32_t* __restrict__ crc_out, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
  load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint32_t len = on ? in_len[i] : 0u;
    const uint32_t ty = type && on ? type[i] : 0u;
    const uint32_t c = half_crc(T, to_global(in) + (on ? in_off[i] : 0), len, type ? 1u : 0u, ty, on);
    if (on & (hl == 0)) crc_out[i] = masked ? crc_mask(c) : c;
  }
}

// ---- row 2: data-block framing ------------------------------------------

// Size of item i's region in one of three layouts:
//   MODE 0: encode slot, 16-byte aligned encode bound (snappy.c:354);
//   MODE 1: framed block in the file: contents (compressed only when that
//           saves more than 12.5 %, table_builder.c:190) + 5-byte trailer;
//   MODE 2: the encoded bytes alone, packed (lgs_encode_batch_host).
template <int MODE>
__device__ __forceinline__ uint64_t item_size(const uint32_t* raw_len, const uint32_t* enc_len,
                                              uint32_t i) {
  if (MODE == 2) return enc_len[i];
  const uint32_t L = raw_len[i];
  if (MODE == 0) return ((uint64_t)32 + L + L / 6 + 15) & ~15ull;
  const uint32_t e = enc_len ? enc_len[i] : 0xffffffffu;
  return (uint64_t)(e < L - L / 8 ? e : L) + kTrailer;
}

constexpr uint32_t kScanT = 256, kScanPer = 8, kScanItems = kScanT * kScanPer;

// Exclusive scan of u64 values inside one workgroup; returns the total.
__device__ __forceinline__ uint64_t wg_scan(uint64_t* s, uint64_t v, uint64_t* excl) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kScanT; d <<= 1) {
    const uint64_t t = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  *excl = s[threadIdx.x] - v;
  const uint64_t tot = s[kScanT - 1];
  __syncthreads();
  return tot;
}

template <int MODE>
__global__ __launch_bounds__(kScanT) void scan_part_kernel(const uint32_t* __restrict__ raw_len,
                                                           const uint32_t* __restrict__ enc_len,
                                                           uint64_t* __restrict__ part,
                                                           uint32_t n) {
  __shared__ uint64_t s[kScanT];
  const uint32_t i0 = blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  uint64_t sum = 0;
  for (uint32_t j = 0; j < kScanPer; ++j)
    if (i0 + j < n) sum += item_size<MODE>(raw_len, enc_len, i0 + j);
  uint64_t ex;
  const uint64_t tot = wg_scan(s, sum, &ex);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanT) void scan_top_kernel(uint64_t* __restrict__ part,
                                                          uint32_t nparts) {
  __shared__ uint64_t s[kScanT];
  const uint32_t per = (nparts + kScanT - 1) / kScanT;
  const uint32_t j0 = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) sum += part[j];
  uint64_t ex;
  wg_scan(s, sum, &ex);
  for (uint32_t j = j0; j < j0 + per && j < nparts; ++j) {
    const uint64_t v = part[j];
    part[j] = ex;
    ex += v;
  }
}

template <int MODE>
__global__ __launch_bounds__(kScanT) void scan_out_kernel(const uint32_t* __restrict__ raw_len,
                                                          const uint32_t* __restrict__ enc_len,
                                                          const uint64_t* __restrict__ part,
                                                          uint64_t base, uint64_t* __restrict__ off,
                                                          uint64_t* __restrict__ end, uint32_t n) {
  __shared__ uint64_t s[kScanT];
  const uint32_t i0 = blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  uint64_t v[kScanPer];
  uint64_t sum = 0;
  for (uint32_t j = 0; j < kScanPer; ++j) {
    v[j] = i0 + j < n ? item_size<MODE>(raw_len, enc_len, i0 + j) : 0;
    sum += v[j];
  }
  uint64_t ex;
  wg_scan(s, sum, &ex);
  uint64_t at = base + part[blockIdx.x] + ex;
  for (uint32_t j = 0; j < kScanPer; ++j) {
    if (i0 + j < n) {
      off[i0 + j] = at;
      if (end && i0 + j == n - 1) *end = at + v[j];
    }
    at += v[j];
  }
}

// One wave per block: pick the contents (table_builder.c:182-199), write
// them and the trailer (:123-153) at file offset off[i] (file[0] is offset
// `base`), record the handle.
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void frame_kernel(
    const uint8_t* __restrict__ raw, const uint64_t* __restrict__ raw_off,
    const uint32_t* __restrict__ raw_len, const uint8_t* __restrict__ enc,
    const uint64_t* __restrict__ enc_off, const uint32_t* __restrict__ enc_len,
    uint8_t* __restrict__ file, uint64_t base, const uint64_t* __restrict__ foff,
    uint64_t* __restrict__ handle_off, uint64_t* __restrict__ handle_size, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
  load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint32_t L = on ? raw_len[i] : 0u;
    const uint32_t e = enc_len && on ? enc_len[i] : 0xffffffffu;
    const bool comp = e < L - L / 8;                                  // :190
    const uint32_t size = comp ? e : L;
    const gptr<const uint8_t> src = !on ? to_global(raw)
                                  : comp ? to_global((const uint8_t*)enc) + enc_off[i]
                                         : to_global(raw) + raw_off[i];
    const uint64_t at = on ? foff[i] : base;
    const gptr<uint8_t> dst = to_global(file) + (at - base);
    const uint32_t c = half_crc(T, src, size, 1u, comp ? 1u : 0u, on);
    if (on) {
      copy_block(src, dst, size, hl);
      if (hl == 0) dst[size] = (uint8_t)(comp ? 1u : 0u);
      const uint32_t m = crc_mask(c);                                 // :142
      if (hl < 4) dst[size + 1 + hl] = (uint8_t)(m >> (8 * hl));
      if (hl == 0) {
        handle_off[i] = at;                                           // :128-129
        handle_size[i] = size;
      }
    }
  }
}

// ---- row 3: block reads --------------------------------------------------

constexpr uint8_t kPending = 0xff;   // snappy block: status decided by the decoder

// format.c:162-231, 263-267 per handle; snappy blocks (:233-261) are handed
// to the decoder through dec_in_off/dec_len/dec_off/dec_cap (others get an
// empty input at file offset 0 and a zero-capacity dummy slot, so the
// decoder cannot touch their output).  CRC: the trailer checks here
// (verify_checksums without the overlapped verify pass); without them this
// instance runs ahead of the decoder and verify_kernel (table_read), and
// check_lane_kernel below serves reads without verification.
template <uint32_t WAVES, bool CRC>
__global__ __launch_bounds__(64 * WAVES) void check_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint32_t verify, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    uint64_t* __restrict__ dec_in_off, uint32_t* __restrict__ dec_len,
    uint64_t* __restrict__ dec_off, uint32_t* __restrict__ dec_cap, uint64_t dummy_off,
    uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[CRC ? kTabWords : 4];
  if (CRC) load_tables<64 * WAVES, kTabWords>(s_tab);
  const Crc T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint64_t off = on ? hoff[i] : 0, size = on ? hsize[i] : 0;
    const uint32_t cap = on ? out_cap[i] : 0u;
    const uint64_t oo = on ? out_off[i] : 0;
    uint32_t st = kStCorrupt;
    uint32_t olen = 0;
    bool snappy = false;
    // The checks of format.c:174-198 first; the trailer CRC (:203-211) of
    // every block that passes them, by the whole wave (half_crc).
    const bool bad_size = size > ~0ull - kTrailer;                    // :174-175
    const bool io = !bad_size && (off > file_len || file_len - off < size + kTrailer);  // :195-198
    const bool big = !bad_size && !io && size > 0x7fffffffull;        // beyond this ABI
    const bool body = on && !bad_size && !io && !big;
    const gptr<const uint8_t> data = to_global(file) + (body ? off : 0);
    const uint32_t sz = body ? (uint32_t)size : 0u;
    const uint32_t ty = body ? (uint32_t)data[sz] : 0u;
    uint32_t c = 0;
    if (CRC) c = half_crc(T, data, sz, 1u, ty, body && verify);
    if (bad_size) {
      st = kStCorrupt;
    } else if (io) {
      st = kStIoErr;
    } else if (big) {
      st = kStNoSpace;
    } else if (on) {
      const bool raw_fits = ty == 0 && sz <= cap;
      bool ok = true;
      if (CRC && verify) {                                            // :203-211
        const uint32_t stored = (uint32_t)data[sz + 1] | ((uint32_t)data[sz + 2] << 8) |
                                ((uint32_t)data[sz + 3] << 16) | ((uint32_t)data[sz + 4] << 24);
        ok = crc_unmask(stored) == c;
      }
      if (raw_fits) copy_block(data, to_global(out) + oo, sz, hl);   // (unspecified if the CRC fails)
      if (!ok) {
        st = kStBadCrc;
      } else if (ty == 0) {                                           // :213-231
        st = raw_fits ? kStOk : kStNoSpace;
        olen = raw_fits ? sz : 0u;
      } else if (ty == 1) {                                           // :233-261
        st = kPending;
        snappy = true;
      } else {                                                        // :263-267
        st = kStBadType;
      }
    }
    if (on & (hl == 0)) {
      status[i] = (uint8_t)st;
      out_len[i] = olen;
      dec_in_off[i] = snappy ? off : 0u;   // never an out-of-range address
      dec_len[i] = snappy ? (uint32_t)size : 0u;
      dec_off[i] = snappy ? oo : dummy_off;
      dec_cap[i] = snappy ? cap : 0u;
    }
  }
}

// check_kernel for reads without verify_checksums (lcdb's default): one lane
// per handle -- the checks are a few loads and compares a block, and a wave
// per block spent 15.8 us on C2's 65 536 handles -- then the wave copies its
// raw blocks one after the other, every lane on each.  (Ahead of the
// overlapped verify pass it loses: 350 against 331 us on C2's verified read,
// profiles/r8e_check_lane_ab.txt -- the wave-per-block check's length is what
// lets the decoder's workgroups take their CUs before verify_kernel's.)
__global__ __launch_bounds__(256) void check_lane_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint8_t* __restrict__ out,
    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
    uint32_t* __restrict__ out_len, uint8_t* __restrict__ status,
    uint64_t* __restrict__ dec_in_off, uint32_t* __restrict__ dec_len,
    uint64_t* __restrict__ dec_off, uint32_t* __restrict__ dec_cap, uint64_t dummy_off,
    uint32_t n) {
  const uint32_t lane = lane_id();
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (uni(blockIdx.x * 256 + (threadIdx.x & ~63u)) >= n) return;   // a whole wave past n
  const bool on = i < n;
  const uint64_t off = on ? hoff[i] : 0, size = on ? hsize[i] : 0;
  const uint32_t cap = on ? out_cap[i] : 0u;
  const uint64_t oo = on ? out_off[i] : 0;
  // format.c:174-198, as check_kernel.
  const bool bad_size = size > ~0ull - kTrailer;                      // :174-175
  const bool io = !bad_size && (off > file_len || file_len - off < size + kTrailer);  // :195-198
  const bool big = !bad_size && !io && size > 0x7fffffffull;          // beyond this ABI
  const bool body = on && !bad_size && !io && !big;
  const uint32_t sz = body ? (uint32_t)size : 0u;
  const uint32_t ty = body ? (uint32_t)file[off + sz] : 0u;
  const bool raw_fits = body && ty == 0 && sz <= cap;
  uint32_t st = kStCorrupt, olen = 0;
  if (bad_size) st = kStCorrupt;
  else if (io) st = kStIoErr;
  else if (big) st = kStNoSpace;
  else if (ty == 0) { st = raw_fits ? kStOk : kStNoSpace; olen = raw_fits ? sz : 0u; }  // :213-231
  else if (ty == 1) st = kPending;                                    // :233-261
  else st = kStBadType;                                               // :263-267
  const bool snappy = body && ty == 1;
  if (on) {
    status[i] = (uint8_t)st;
    out_len[i] = olen;
    dec_in_off[i] = snappy ? off : 0u;   // never an out-of-range address
    dec_len[i] = snappy ? sz : 0u;
    dec_off[i] = snappy ? oo : dummy_off;
    dec_cap[i] = snappy ? cap : 0u;
  }
  // The raw blocks (format.c:213-231), a wave at a time.
  for (uint64_t m = ballot(raw_fits); m; m &= m - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    const uint64_t so = ((uint64_t)lane_val((uint32_t)(off >> 32), l) << 32) | lane_val((uint32_t)off, l);
    const uint64_t d = ((uint64_t)lane_val((uint32_t)(oo >> 32), l) << 32) | lane_val((uint32_t)oo, l);
    copy_block(to_global(file) + so, to_global(out) + d, lane_val(sz, l), lane);
  }
}

// The trailer checks of format.c:203-211 on their own (check_kernel then
// runs without them): bad[i] = 1 when block i's stored CRC does not match.
// Its 6.6 KB of tables let one workgroup sit on every CU beside the ring
// decoder's eight waves (151.5 of 160 KB of LDS), so it runs while the
// blocks decode (table_read).
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void verify_kernel(
    const uint8_t* __restrict__ file, uint64_t file_len, const uint64_t* __restrict__ hoff,
    const uint64_t* __restrict__ hsize, uint8_t* __restrict__ bad, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kSmallWords];
  load_tables<64 * WAVES, kSmallWords>(s_tab);
  const CrcSmall T{{s_tab}};
  const uint32_t wv = uni(threadIdx.x >> 6), hl = lane_id() & (kHalf - 1), half = lane_id() / kHalf;
  // kBpw blocks per wave (half_crc).
  for (uint32_t i0 = kBpw * (blockIdx.x * WAVES + wv); i0 < n; i0 += kBpw * gridDim.x * WAVES) {
    const uint32_t i = i0 + half;
    const bool on = i < n;
    const uint64_t off = on ? hoff[i] : 0, size = on ? hsize[i] : 0;
    const bool body = on && size <= ~0ull - kTrailer && off <= file_len &&
                      file_len - off >= size + kTrailer && size <= 0x7fffffffull;  // as check_kernel
    const gptr<const uint8_t> data = to_global(file) + (body ? off : 0);
    const uint32_t sz = body ? (uint32_t)size : 0u;
    const uint32_t ty = body ? (uint32_t)data[sz] : 0u;
    const uint32_t c = half_crc(T, data, sz, 1u, ty, body);
    uint32_t b = 0;
    if (body) {
      const uint32_t stored = (uint32_t)data[sz + 1] | ((uint32_t)data[sz + 2] << 8) |
                              ((uint32_t)data[sz + 3] << 16) | ((uint32_t)data[sz + 4] << 24);
      b = crc_unmask(stored) != c;
    }
    if (on & (hl == 0)) bad[i] = (uint8_t)b;
  }
}

__global__ __launch_bounds__(256) void merge_kernel(uint8_t* __restrict__ status,
                                                    uint32_t* __restrict__ out_len,
                                                    const uint8_t* __restrict__ dec_status,
                                                    const uint32_t* __restrict__ dec_out_len,
                                                    const uint8_t* __restrict__ bad, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (bad && bad[i]) {            // format.c:203-211 before the type dispatch
    status[i] = kStBadCrc;
    out_len[i] = 0;
    return;
  }
  if (status[i] != kPending) return;
  status[i] = dec_status[i];      // LGS_ST_CORRUPT / OK / NOSPACE, format.c:237-252
  out_len[i] = dec_out_len[i];
}

// Grid for the one-wave-per-block framing kernels: every workgroup
// resident at once (CUs x the occupancy the kernel's LDS allows), each
// loading the tables once and striding over blocks -- no second, partial
// round of workgroups.
constexpr uint32_t kFrameWaves = 8;
uint32_t g_res_crc = 0, g_res_pack = 0, g_res_frame = 0, g_res_check = 0, g_res_check_plain = 0;
template <class K>
uint32_t frame_grid(K kernel, uint32_t n, uint32_t& resident) {   // resident: per kernel,
  if (resident == 0) {                                              // same on every device
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64 * kFrameWaves, 0) !=
            hipSuccess ||
        cus <= 0 || per <= 0) {
      cus = 256;
      per = 4;
    }
    resident = (uint32_t)(cus * per);
  }
  // (Two blocks per wave: half_crc.)
  const uint32_t want = (n + kBpw * kFrameWaves - 1) / (kBpw * kFrameWaves);
  return want < resident ? (want ? want : 1u) : resident;
}

}  // namespace

hipError_t launch_crc(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      const uint8_t* type, int masked, uint32_t* crc, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(crc_kernel<kFrameWaves>, dim3(frame_grid(crc_kernel<kFrameWaves>, n, g_res_crc)), dim3(64 * kFrameWaves),
                     0, s, in, in_off, in_len, type, (uint32_t)(masked != 0), crc, n);
  return hipGetLastError();
}

size_t scan_parts(uint32_t n) { return (n + kScanItems - 1) / kScanItems; }

__global__ __launch_bounds__(256) void fill_stride_kernel(uint64_t* __restrict__ off,
                                                          uint64_t stride, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) off[i] = (uint64_t)i * stride;
}

hipError_t launch_fill_stride(uint64_t* off, uint64_t stride, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_stride_kernel, dim3((n + 255) / 256), dim3(256), 0, s, off, stride, n);
  return hipGetLastError();
}

hipError_t launch_scan(int mode, const uint32_t* raw_len, const uint32_t* enc_len, uint64_t* part,
                       uint64_t base, uint64_t* off, uint64_t* end, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t np = (uint32_t)scan_parts(n);
  if (mode == 0) {
    hipLaunchKernelGGL(scan_part_kernel<0>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  } else if (mode == 1) {
    hipLaunchKernelGGL(scan_part_kernel<1>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  } else {
    hipLaunchKernelGGL(scan_part_kernel<2>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part, n);
  }
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanT), 0, s, part, np);
  if (mode == 0) {
    hipLaunchKernelGGL(scan_out_kernel<0>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  } else if (mode == 1) {
    hipLaunchKernelGGL(scan_out_kernel<1>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  } else {
    hipLaunchKernelGGL(scan_out_kernel<2>, dim3(np), dim3(kScanT), 0, s, raw_len, enc_len, part,
                       base, off, end, n);
  }
  return hipGetLastError();
}

// Item i's len[i] bytes from src + src_off[i] to dst + dst_off[i], one wave
// per item: whole 16-byte destination granules with one (unaligned) 16-byte
// load and one aligned store, the ragged ends byte by byte.
template <uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void pack_kernel(const uint8_t* __restrict__ src,
                                                         const uint64_t* __restrict__ src_off,
                                                         const uint32_t* __restrict__ len,
                                                         uint8_t* __restrict__ dst,
                                                         const uint64_t* __restrict__ dst_off,
                                                         uint32_t n) {
  typedef u32x4 u32x4_g __attribute__((aligned(1)));
  for (uint32_t i = uni(blockIdx.x * WAVES + (threadIdx.x >> 6)); i < n;
       i += gridDim.x * WAVES) {
    const gptr<const uint8_t> s = to_global(src) + src_off[i];
    const gptr<uint8_t> d = to_global(dst) + dst_off[i];
    const uint32_t e = len[i];
    const uint64_t d0 = (uint64_t)(uintptr_t)d;
    const uint64_t g_lo = d0 & ~15ull, g_hi = (d0 + e + 15) & ~15ull;
    for (uint64_t g = g_lo + 16ull * lane_id(); g < g_hi; g += 16ull * kWave) {
      const int64_t k0 = (int64_t)(g - d0);
      if (g >= d0 && g + 16 <= d0 + e) {
        *(gptr<u32x4>)(d + k0) = *(gptr<const u32x4_g>)(s + k0);
      } else {
        for (uint32_t t = 0; t < 16; ++t) {
          const int64_t k = k0 + t;
          if (k >= 0 && k < (int64_t)e) d[k] = s[k];
        }
      }
    }
  }
}

hipError_t launch_pack(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                       uint8_t* dst, const uint64_t* dst_off, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pack_kernel<kFrameWaves>, dim3(frame_grid(pack_kernel<kFrameWaves>, n, g_res_pack)),
                     dim3(64 * kFrameWaves), 0, s, src, src_off, len, dst, dst_off, n);
  return hipGetLastError();
}

hipError_t launch_frame(const FrameArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(frame_kernel<kFrameWaves>, dim3(frame_grid(frame_kernel<kFrameWaves>, a.n, g_res_frame)), dim3(64 * kFrameWaves), 0,
                     s, a.raw, a.raw_off, a.raw_len, a.enc, a.enc_off, a.enc_len, a.file, a.base,
                     a.foff, a.handle_off, a.handle_size, a.n);
  return hipGetLastError();
}

hipError_t launch_check(const CheckArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (a.verify) {
    hipLaunchKernelGGL((check_kernel<kFrameWaves, true>),
                       dim3(frame_grid(check_kernel<kFrameWaves, true>, a.n, g_res_check)),
                       dim3(64 * kFrameWaves), 0, s, a.file, a.file_len, a.hoff, a.hsize, a.verify,
                       a.out, a.out_off, a.out_cap, a.out_len, a.status, a.dec_in_off, a.dec_len,
                       a.dec_off, a.dec_cap, a.dummy_off, a.n);
  } else {
    hipLaunchKernelGGL((check_kernel<kFrameWaves, false>),
                       dim3(frame_grid(check_kernel<kFrameWaves, false>, a.n, g_res_check_plain)),
                       dim3(64 * kFrameWaves), 0, s, a.file, a.file_len, a.hoff, a.hsize, a.verify,
                       a.out, a.out_off, a.out_cap, a.out_len, a.status, a.dec_in_off, a.dec_len,
                       a.dec_off, a.dec_cap, a.dummy_off, a.n);
  }
  return hipGetLastError();
}

hipError_t launch_check_lane(const CheckArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(check_lane_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a.file,
                     a.file_len, a.hoff, a.hsize, a.out, a.out_off, a.out_cap, a.out_len,
                     a.status, a.dec_in_off, a.dec_len, a.dec_off, a.dec_cap, a.dummy_off, a.n);
  return hipGetLastError();
}

hipError_t launch_merge(uint8_t* status, uint32_t* out_len, const uint8_t* dec_status,
                        const uint32_t* dec_out_len, const uint8_t* bad, uint32_t n,
                        hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(merge_kernel, dim3((n + 255) / 256), dim3(256), 0, s, status, out_len,
                     dec_status, dec_out_len, bad, n);
  return hipGetLastError();
}

// One workgroup of 8 waves per CU: the verify pass keeps to the LDS the ring
// decoder leaves free.
constexpr uint32_t kVerifyWaves = 8;
hipError_t launch_verify(const uint8_t* file, uint64_t file_len, const uint64_t* hoff,
                         const uint64_t* hsize, uint8_t* bad, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  static uint32_t cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
              ? (uint32_t)c : 256u;
  }
  const uint32_t want = (n + kBpw * kVerifyWaves - 1) / (kBpw * kVerifyWaves);
  hipLaunchKernelGGL(verify_kernel<kVerifyWaves>, dim3(want < cus ? want : cus),
                     dim3(64 * kVerifyWaves), 0, s, file, file_len, hoff, hsize, bad, n);
  return hipGetLastError();
}

}  // namespace lgs
