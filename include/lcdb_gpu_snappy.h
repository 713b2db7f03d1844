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
 *    encode/decode stage through pinned memory on a per-thread HIP stream;
 *    both are thread-safe.  Compressed bytes are identical to the reference
 *    encoder's and decode accepts/rejects exactly what the reference does.
 *    The *_size functions are header arithmetic (a bound, a varint32 read)
 *    and run on the host.  Encode has no error path in lcdb, so a HIP
 *    failure inside ldb_snappy_encode prints a diagnostic and aborts (there
 *    is no silent CPU fallback).  On a decode failure the contents of zp are
 *    unspecified, as in the reference.
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
   extend at least 16 bytes beyond the last block. */
int lgs_decode_batch_dev(const uint8_t *d_in, const uint64_t *d_in_off,
                         const uint32_t *d_in_len, uint8_t *d_out,
                         const uint64_t *d_out_off, const uint32_t *d_out_cap,
                         uint32_t *d_out_len, uint8_t *d_status, uint32_t n,
                         uint32_t max_out_cap, void *stream);

/* Host-buffer variants: same layout with host pointers (pageable is fine).
   Data moves through pinned staging with hipMemcpyAsync on a per-thread
   stream; the call returns when the results are in the caller's buffers. */
int lgs_encode_batch_host(const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t *out,
                          const uint64_t *out_off, uint32_t *out_len,
                          uint32_t n);
int lgs_decode_batch_host(const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t *out,
                          const uint64_t *out_off, const uint32_t *out_cap,
                          uint32_t *out_len, uint8_t *status, uint32_t n);

/* Devices and diagnostics. */
int lgs_device_count(void);
int lgs_set_device(int device);  /* device used by the calling thread */
const char *lgs_last_error(void);
const char *lgs_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LCDB_GPU_SNAPPY_H */
