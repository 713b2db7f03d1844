/*
 * lcdb_gpu_snappy.h -- C ABI of the MI355X (gfx950) Snappy block codec.
 *
 * Two layers, both plain C (C89-compatible declarations, no HIP or torch
 * types; streams are passed as `void *` holding a hipStream_t):
 *
 * 1. The drop-in.  The four symbols lcdb's codec exports, with identical
 *    names, argument meaning and return values, so lcdb's src/table/ (*.c) and
 *    src/builder.c link against this library unchanged in place of
 *    src/util/snappy.c (CMakeLists.txt:209 / Makefile.am:86-87):
 *
 *      ldb_snappy_encode_size  replaces  src/util/snappy.c:347-362
 *                                        (declared snappy.h:28-29)
 *      ldb_snappy_encode       replaces  src/util/snappy.c:364-384
 *                                        (declared snappy.h:31-32)
 *      ldb_snappy_decode_size  replaces  src/util/snappy.c:386-399
 *                                        (declared snappy.h:34-35)
 *      ldb_snappy_decode       replaces  src/util/snappy.c:401-412
 *                                        (declared snappy.h:37-38)
 *
 *    Callers: src/table/table_builder.c:182,187 (encode) and
 *    src/table/format.c:237,247 (decode); both pass pageable host buffers.
 *    Both are thread-safe.  A call leases one of a bounded pool of staging
 *    slots (per device: at most LGS_DROPIN_SLOTS = 8 slots of LGS_DROPIN_MB =
 *    4 MiB pinned + 4 MiB device memory, created on first use; a caller waits
 *    while all are leased), so the drop-in's memory is bounded whatever the
 *    input: encode runs any input through its slot in passes of whole 64 KiB
 *    chunks (independent, snappy.c:370-381); decode rejects on the host every
 *    stream whose size header its length cannot satisfy (exactly the
 *    reference's result, no device work), and decodes a block larger than a
 *    slot in device memory taken for that call only.
 *    Compressed bytes are identical to the reference encoder's and decode
 *    accepts/rejects exactly what the reference does.  The *_size functions
 *    are header arithmetic (a bound, a varint32 read) and run on the host.
 *    Errors: lcdb's encode path has no error return (table_builder.c:182-
 *    188), so ldb_snappy_encode aborts with a diagnostic only when the device
 *    fails (or no slot at all can be created); ldb_snappy_decode returns 0
 *    (LDB_CORRUPTION at format.c:247-251) with a diagnostic when device
 *    memory for an over-slot block runs out, and aborts only when the device
 *    fails.  There is no CPU fallback.  On a decode failure the contents of
 *    zp are unspecified, as in the reference.
 *
 * 2. The batched API (lgs_*), new: tens of thousands of independent blocks
 *    per launch.  Blocks are addressed by byte offsets into one base buffer.
 *    Output per block is byte-identical to ldb_snappy_encode on that block
 *    alone (encode) / to ldb_snappy_decode (decode).
 *
 *    Return values: LGS_OK (0) or a negative LGS_E* code; lgs_last_error()
 *    gives a message for the calling thread.
 */
#ifndef LCDB_GPU_SNAPPY_H
#define LCDB_GPU_SNAPPY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- drop-in: src/util/snappy.h:28-38 ---- */
int ldb_snappy_encode_size(size_t *zn, size_t xn);
size_t ldb_snappy_encode(uint8_t *zp, const uint8_t *xp, size_t xn);
int ldb_snappy_decode_size(size_t *zn, const uint8_t *xp, size_t xn);
int ldb_snappy_decode(uint8_t *zp, const uint8_t *xp, size_t xn);

/* ---- batched API ---- */
#define LGS_OK          0
#define LGS_EINVAL     -1   /* bad argument (NULL, size out of range)   */
#define LGS_EHIP       -2   /* HIP runtime error                        */
#define LGS_ENODEV     -3   /* no usable gfx950 device                  */
#define LGS_ENOMEM     -4   /* device / pinned allocation failed        */
#define LGS_ENOSPC     -5   /* output buffer too small                  */
#define LGS_EINTERNAL  -6   /* a device result broke its own bound      */

/* Per-block decode status written by the decode calls. */
#define LGS_ST_CORRUPT  0   /* reference decode would return 0          */
#define LGS_ST_OK       1
#define LGS_ST_NOSPACE  2   /* decoded length > out_cap[i]              */

/* Worst-case encoded size (same formula as ldb_snappy_encode_size). */
size_t lgs_encode_bound(size_t n);

/* Device-resident encode.  All pointers are device pointers.  Block i is
   d_in[d_in_off[i] .. + d_in_len[i]) (any length < 2^31; blocks over
   64 KiB are encoded as consecutive 64 KiB chunks by one wave, exactly as
   snappy.c:370-381 does); its encoding is written at d_out + d_out_off[i]
   (room for lgs_encode_bound(d_in_len[i]) bytes) and its length to
   d_out_len[i].  max_in_len >= every d_in_len[i] (selects the LDS class).  Asynchronous on
   `stream` (a hipStream_t, NULL = default stream). */
int lgs_encode_batch_dev(const uint8_t *d_in, const uint64_t *d_in_off,
                         const uint32_t *d_in_len, uint8_t *d_out,
                         const uint64_t *d_out_off, uint32_t *d_out_len,
                         uint32_t n, uint32_t max_in_len, void *stream);

/* Device-resident decode.  Block i is d_in[d_in_off[i] .. + d_in_len[i]);
   it decodes into d_out + d_out_off[i] (capacity d_out_cap[i]);
   d_out_len[i] = decoded length (0 unless ok), d_status[i] = LGS_ST_*.
   max_out_cap >= every d_out_cap[i].  Asynchronous on `stream`.
   Read slack: the kernel may READ (never write) up to 16 bytes past the end
   of a block's input and past its output cursor, so both allocations must
   extend at least 16 bytes beyond the last block.
   Both _dev calls: a batch of >= 512 blocks whose largest block is over
   4 608 bytes is sorted into size classes on the device first, with up to
   16 bytes per block of stream-ordered scratch from a private memory pool
   of the device (hipMallocFromPoolAsync, freed on `stream`; the process's
   default pool is not touched); LGS_ENOMEM-class HIP errors are possible
   there.  lgs_set_option("split", "0") turns this off. */
int lgs_decode_batch_dev(const uint8_t *d_in, const uint64_t *d_in_off,
                         const uint32_t *d_in_len, uint8_t *d_out,
                         const uint64_t *d_out_off, const uint32_t *d_out_cap,
                         uint32_t *d_out_len, uint8_t *d_status, uint32_t n,
                         uint32_t max_out_cap, void *stream);

/* Host-buffer variants: same layout with host pointers (pageable is fine).
   Data moves through pinned staging with hipMemcpyAsync on a pooled
   context's stream (contexts are leased per call, never tied to a thread;
   their arenas grow to the largest batch served); the call returns when the
   results are in the caller's buffers. */
int lgs_encode_batch_host(const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t *out,
                          const uint64_t *out_off, uint32_t *out_len,
                          uint32_t n);
int lgs_decode_batch_host(const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t *out,
                          const uint64_t *out_off, const uint32_t *out_cap,
                          uint32_t *out_len, uint8_t *status, uint32_t n);

/* ---- SSTable block framing ----
 *
 * lcdb frames every table block as  contents | type (1 byte) | masked
 * crc32c of contents+type (fixed32)  (table_builder.c:123-153), and reads a
 * block back through format.c:162-270.  These calls do both for many blocks
 * per launch, byte-identical to the reference doing them one at a time. */

#define LGS_NO_COMPRESSION      0   /* enum ldb_compression (options.h)       */
#define LGS_SNAPPY_COMPRESSION  1
#define LGS_TRAILER_SIZE        5   /* LDB_TRAILER_SIZE (format.h:34)         */

/* Further per-block read statuses (besides LGS_ST_CORRUPT/OK/NOSPACE). */
#define LGS_ST_IOERR    3   /* truncated block read -> LDB_IOERR (format.c:195-198)     */
#define LGS_ST_BADCRC   4   /* checksum mismatch -> LDB_CORRUPTION (format.c:203-211)   */
#define LGS_ST_BADTYPE  5   /* bad block type -> LDB_CORRUPTION (format.c:263-267)      */

/* Row 1.  d_crc[i] = ldb_crc32c_value(block i) (crc32c.c:1147, crc32c.h:29),
   extended over the byte d_type[i] when d_type != NULL (table_builder.c:139-
   140), then ldb_crc32c_mask'ed (crc32c.h:46-50) when masked != 0.  With a
   type and masked = 1 this is the trailer's crc field.  Asynchronous. */
int lgs_crc32c_batch_dev(const uint8_t *d_in, const uint64_t *d_in_off,
                         const uint32_t *d_in_len, const uint8_t *d_type,
                         int masked, uint32_t *d_crc, uint32_t n, void *stream);

/* Row 2.  n finished data blocks (ldb_blockgen_finish output, raw bytes)
   written as ldb_tablegen_write_block writes them (table_builder.c:155-213):
   snappy-encoded when compression = LGS_SNAPPY_COMPRESSION and that saves
   more than 12.5 % (:190), else raw; each followed by its trailer; block i at
   file offset handle_off[i] with handle_size[i] content bytes (:128-129);
   the first block at offset `base`.  d_file[j] receives file offset base + j;
   *d_end = base + bytes written.  d_file needs sum(raw_len) + 5n bytes.
   raw_total = sum of the raw lengths (sizes the scratch);
   d_scratch: lgs_table_write_scratch(n, raw_total) device bytes.  Inputs
   must stay readable 16 bytes past each block.  Asynchronous. */
size_t lgs_table_write_scratch(uint32_t n, uint64_t raw_total);
int lgs_table_write_dev(const uint8_t *d_raw, const uint64_t *d_raw_off,
                        const uint32_t *d_raw_len, uint32_t n, uint32_t max_raw_len,
                        uint64_t raw_total, int compression, uint64_t base,
                        uint8_t *d_file, uint64_t *d_handle_off,
                        uint64_t *d_handle_size, uint64_t *d_end,
                        void *d_scratch, size_t scratch_bytes, void *stream);
/* Host buffers; returns when file/handles/end are written.  file_cap: room
   in `file` (sum(raw_len) + 5n always suffices). */
int lgs_table_write_host(const uint8_t *raw, const uint64_t *raw_off,
                         const uint32_t *raw_len, uint32_t n, int compression,
                         uint64_t base, uint8_t *file, size_t file_cap,
                         uint64_t *handle_off, uint64_t *handle_size,
                         uint64_t *end);

/* Row 3.  ldb_read_block (format.c:162-270) for n block handles of one
   table image (d_file[0 .. file_len) = file offsets 0 ..): truncation check,
   trailer check when verify_checksums, then raw copy or snappy decode into
   d_out + d_out_off[i] (capacity d_out_cap[i]; the decoded size of a snappy
   block is its varint32 header, ldb_snappy_decode_size).  d_status[i] =
   LGS_ST_OK or the reason the reference fails; d_out_len[i] = contents
   length when ok (the output bytes of a block that fails are unspecified).
   With verify_checksums the CRC checks run on a second stream of the
   library's own beside the decoder (lgs_set_option("verify_overlap", "0")
   or LGS_VERIFY_OVERLAP=0: inside the type dispatch); the call stays
   ordered on `stream`.  d_file must stay readable 16 bytes past file_len.
   d_scratch: lgs_table_read_scratch(n) device bytes.  Asynchronous. */
size_t lgs_table_read_scratch(uint32_t n);
int lgs_table_read_dev(const uint8_t *d_file, uint64_t file_len,
                       const uint64_t *d_handle_off, const uint64_t *d_handle_size,
                       uint32_t n, int verify_checksums, uint8_t *d_out,
                       const uint64_t *d_out_off, const uint32_t *d_out_cap,
                       uint32_t max_out_cap, uint32_t *d_out_len, uint8_t *d_status,
                       void *d_scratch, size_t scratch_bytes, void *stream);
/* Host buffers (e.g. an mmap'd .ldb); only the handles' byte ranges are
   uploaded.  Returns when out/out_len/status are written. */
int lgs_table_read_host(const uint8_t *file, uint64_t file_len,
                        const uint64_t *handle_off, const uint64_t *handle_size,
                        uint32_t n, int verify_checksums, uint8_t *out,
                        const uint64_t *out_off, const uint32_t *out_cap,
                        uint32_t *out_len, uint8_t *status);

/* Row 3, opening a table: ldb_table_open (table.c:120-180) and the index
   walk of its two-level iterator, for the batched read above.  From the
   footer (format.c:116-137) it reads the index block through
   lgs_table_read_host (checksums verified when paranoid_checks, as
   table.c:148-151) and returns, in index order, each entry's data-block
   handle (handle_off/handle_size, cap of them; *count written) and, if keys
   != NULL, its separator key (keys[key_off[i] .. key_off[i+1]), keys_cap
   bytes, key_off has cap + 1 entries).  internal_keys: index keys are
   internal keys (the DB's tables), so one under 8 bytes is a bad entry
   (block.c:270-273).  With filter_name (e.g.
   "filter.leveldb.BuiltinBloomFilter2") the metaindex is read too and
   *filter_off and *filter_size receive that entry's handle, or ~0 / 0 when
   there is none or the metaindex does not read (table.c:78-120 ignores
   those errors).  *status: LGS_ST_OK; LGS_ST_CORRUPT for a short file, a
   bad footer, a bad index block or entry (the walk stops there), or an
   entry whose value is no handle (skipped, as the two-level iterator skips
   it); the block read's own status (LGS_ST_IOERR, _BADCRC, _BADTYPE) when
   the index block does not read.  Returns LGS_ENOSPC when cap or keys_cap is
   too small. */
int lgs_table_index_host(const uint8_t *file, uint64_t file_len, int paranoid_checks,
                         int internal_keys, const char *filter_name, uint64_t *handle_off,
                         uint64_t *handle_size, uint32_t cap, uint32_t *count, uint8_t *keys,
                         size_t keys_cap, uint64_t *key_off, uint64_t *filter_off,
                         uint64_t *filter_size, uint8_t *status);

/* Row 4.  lcdb's builtin bloom filter (src/util/bloom.c, src/util/hash.c):
   filter f holds keys [first[f], first[f+1]) and is written at out +
   out_off[f] exactly as ldb_bloom_build appends it (bloom.c:102-119):
   lgs_bloom_filter_size(n, bits_per_key) bytes = the bit array
   (max(64, n * bits_per_key) bits, rounded up to bytes) + one byte k
   (bits_per_key * 0.69, clamped to [1, 30]); an empty filter has no bytes
   (filter_block.c:89-93).  match[q] = ldb_bloom_match(filter
   query_filter[q], key q) (bloom.c:121-165).  Keys must stay readable 16
   bytes past their end.  The _dev calls are asynchronous. */
size_t lgs_bloom_filter_size(uint32_t nkeys, int bits_per_key);
int lgs_bloom_build_dev(const uint8_t *d_keys, const uint64_t *d_key_off,
                        const uint32_t *d_key_len, const uint32_t *d_first,
                        uint32_t nfilters, int bits_per_key, uint8_t *d_out,
                        const uint64_t *d_out_off, void *stream);
int lgs_bloom_match_dev(const uint8_t *d_filters, const uint64_t *d_filter_off,
                        const uint32_t *d_filter_len, const uint32_t *d_query_filter,
                        const uint8_t *d_keys, const uint64_t *d_key_off,
                        const uint32_t *d_key_len, uint8_t *d_match, uint32_t nq,
                        void *stream);
int lgs_bloom_build_host(const uint8_t *keys, const uint64_t *key_off,
                         const uint32_t *key_len, const uint32_t *first,
                         uint32_t nfilters, int bits_per_key, uint8_t *out,
                         const uint64_t *out_off);
int lgs_bloom_match_host(const uint8_t *filters, const uint64_t *filter_off,
                         const uint32_t *filter_len, uint32_t nfilters,
                         const uint32_t *query_filter, const uint8_t *keys,
                         const uint64_t *key_off, const uint32_t *key_len, uint32_t nq,
                         uint8_t *match);

/* Row 4, the filter block of one table (src/table/filter_block.c), as
   lcdb's table builder makes it: data block b holds keys [block_first[b],
   block_first[b+1]) and sits at file offset block_off[b] (file order, the
   first at 0); data_end is the offset after the last one.  The builder adds
   each block's keys, writes the block, then calls
   ldb_filtergen_start_block(offset after it) (table_builder.c:242-243,
   276-277) and ldb_filtergen_finish at the end (:294): one bloom filter per
   started 2 KiB of data offsets (filter_block.c:79-121), then the u32
   offset array, its start and base_lg = 11 (:131-150).  internal_keys = 1
   is the DB's internal filter policy (dbformat.c:308-334): keys are internal
   keys and filters cover the user key, i.e. all but the last 8 bytes.
   Keys must stay readable 16 bytes past their end; block_first and
   block_off must not decrease, block_off[nblocks-1] <= data_end (checked by
   _host; the _dev caller's contract, as for handles from lgs_table_write_dev).
   Sizes: lgs_filter_block_bound(...) bytes of out suffice;
   lgs_filter_block_scratch(data_end) bytes of device scratch for _dev, whose
   block length lands in *d_size.  The _dev calls are asynchronous. */
size_t lgs_filter_block_bound(uint32_t nkeys, uint32_t nblocks, uint64_t data_end,
                              int bits_per_key);
size_t lgs_filter_block_scratch(uint64_t data_end);
int lgs_filter_block_build_dev(const uint8_t *d_keys, const uint64_t *d_key_off,
                               const uint32_t *d_key_len, uint32_t nkeys,
                               const uint32_t *d_block_first, const uint64_t *d_block_off,
                               uint32_t nblocks, uint64_t data_end, int bits_per_key,
                               int internal_keys, uint8_t *d_out, size_t out_cap,
                               uint64_t *d_size, void *d_scratch, size_t scratch_bytes,
                               void *stream);
int lgs_filter_block_build_host(const uint8_t *keys, const uint64_t *key_off,
                                const uint32_t *key_len, const uint32_t *block_first,
                                const uint64_t *block_off, uint32_t nblocks, uint64_t data_end,
                                int bits_per_key, int internal_keys, uint8_t *out,
                                size_t out_cap, size_t *size);
/* ldb_filter_matches (filter_block.c:170-225) of the filter block
   block[0 .. block_len) -- as ldb_filter_init parses it -- for query q =
   (key q, the data block at file offset block_offset[q]): 0 = the key is
   certainly absent from that block, 1 = it may be present (also for every
   malformed filter block or offset out of its range). */
int lgs_filter_block_match_dev(const uint8_t *d_block, size_t block_len,
                               const uint64_t *d_block_offset, const uint8_t *d_keys,
                               const uint64_t *d_key_off, const uint32_t *d_key_len, uint32_t nq,
                               int internal_keys, uint8_t *d_match, void *stream);
int lgs_filter_block_match_host(const uint8_t *block, size_t block_len,
                                const uint64_t *block_offset, const uint8_t *keys,
                                const uint64_t *key_off, const uint32_t *key_len, uint32_t nq,
                                int internal_keys, uint8_t *match);

/* Devices and diagnostics. */
/* The drop-in's current footprint: pinned and device bytes held by its
   staging slots, the number of slots created (all devices) and the bytes of
   one slot's arena.  The totals never exceed slots * slot_bytes. */
int lgs_dropin_footprint(size_t *pinned, size_t *device, uint32_t *slots,
                         size_t *slot_bytes);

/* Stop the drop-in's resident service waves (every device), wait until they
   have left, and send drop-in calls through the launch path (one kernel and
   one stream synchronisation per call) until lgs_service_resume().  The
   waves otherwise stay while calls keep coming and leave
   LGS_SERVICE_IDLE_US (default 2 ms) after the last call from any thread;
   an application that synchronises the whole device under sustained
   drop-in traffic (hipDeviceSynchronize, hipFree) brackets that with these
   two calls.  Calls in flight complete (through the launch path if the
   waves left first); results are the same either way. */
int lgs_service_quiesce(void);
int lgs_service_resume(void);

/* Process-wide kernel choices (A/B and tests; the defaults pick by batch):
     "decoder": "auto" | "ring" (lane-per-block) | "wave" (wave-per-block)
     "wide":    "walk"  (decoder of outputs over 16 KiB: the one-tag walk)
     "split":   "1" | "0"  (size-class split of mixed batches, see above)
     "service": "1" | "0"  (the drop-in's resident waves)
     "verify_overlap": "1" | "0"  (table reads: CRC pass beside the decoder)
   Initial values: LGS_DECODE_KERNEL, LGS_NO_SPLIT=1, LGS_DROPIN_SERVICE,
   LGS_VERIFY_OVERLAP=0, read once at load.
   LGS_EINVAL for an unknown name or value.  (The decoders that lost their
   A/B -- "decoder" "quad", "ops", "group" and "chain", "wide" "trips" and
   "group" --
   exist only in the test-only probe library; this library
   rejects them.) */
int lgs_set_option(const char *name, const char *value);

/* HBM yardstick, not part of the codec: copies `bytes` (a multiple of 16)
   from d_src to d_dst (both 16-byte aligned device pointers) with a
   16-bytes-per-lane streaming kernel, asynchronously on `stream`.  bench.py
   times it to report the device's achievable HBM rate beside the 8 TB/s
   spec peak. */
int lgs_hbm_copy_dev(void *d_dst, const void *d_src, size_t bytes, void *stream);

int lgs_device_count(void);
int lgs_set_device(int device);  /* device used by the calling thread */
const char *lgs_last_error(void);
const char *lgs_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LCDB_GPU_SNAPPY_H */
