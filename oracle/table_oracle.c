/*
 * table_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker for the
 * SSTable block-framing rows of SURVEY.md §8(f): CRC32C trailers, batched
 * data-block writes, batched block reads).
 *
 * A plain-C89 restatement of
 *   - lcdb's CRC32C (src/util/crc32c.c:643-750, the portable path every
 *     accelerated path must agree with; mask/unmask src/util/crc32c.h:38-57);
 *   - the data-block write of src/table/table_builder.c:123-213
 *     (ldb_tablegen_write_raw_block + ldb_tablegen_write_block: the 12.5 %
 *     rule, the 1-byte type and masked-CRC trailer, file offsets);
 *   - the block read of src/table/format.c:162-270 (ldb_read_block: the
 *     truncation check, the trailer CRC check, the type dispatch and the
 *     snappy decode).
 * Nothing in lcdb_amd/ links, loads or calls this file.
 *
 * Parity pin: the CRC is checked against the known answers of
 * test/t-crc32c.c:39-54 (RFC 3720 B.4) and against the reference's own
 * crc32c.c compiled unmodified into oracle/_ref/ (tests/test_table_oracle.py);
 * the write/read restatements against .ldb files written and read by the
 * reference's own table code (oracle/harness/dump_blocks.c,
 * oracle/harness/build_table.c).
 */

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "snappy_oracle.h"
#include "table_oracle.h"

#define ORC_POLY        0x82f63b78u    /* CRC32C, reflected             */
#define ORC_CRC_XOR     0xffffffffu    /* crc32c.c:501                  */
#define ORC_MASK_DELTA  0xa282ead8u    /* crc32c.h:38                   */
#define ORC_TRAILER     5              /* format.h: type + fixed32 crc  */

static uint32_t orc_crc_tab[256];
static int orc_crc_ready = 0;

static void
orc_crc_init(void) {
  uint32_t b, k, c;
  for (b = 0; b < 256; b++) {
    c = b;
    for (k = 0; k < 8; k++)
      c = (c & 1) ? (c >> 1) ^ ORC_POLY : (c >> 1);
    orc_crc_tab[b] = c;
  }
  orc_crc_ready = 1;
}

/* crc32c.c:643-750 (crc32c_generic): pre- and post-conditioned by ~0; the
   byte step is crc32c.c:649-652.  The reference's 4-stride loop computes the
   same function; one byte at a time is the plain statement of it. */
uint32_t
oracle_crc32c_extend(uint32_t z, const uint8_t *xp, size_t xn) {
  uint32_t l = z ^ ORC_CRC_XOR;
  size_t i;
  if (!orc_crc_ready)
    orc_crc_init();
  for (i = 0; i < xn; i++)
    l = orc_crc_tab[(l ^ xp[i]) & 0xff] ^ (l >> 8);
  return l ^ ORC_CRC_XOR;
}

/* crc32c.h:46-50. */
uint32_t
oracle_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + ORC_MASK_DELTA;
}

/* crc32c.h:53-57. */
uint32_t
oracle_crc32c_unmask(uint32_t masked) {
  uint32_t rot = masked - ORC_MASK_DELTA;
  return (rot >> 17) | (rot << 15);
}

static void
orc_put32(uint8_t *p, uint32_t v) {   /* coding.h ldb_fixed32_write */
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

static uint32_t
orc_get32(const uint8_t *p) {         /* coding.h ldb_fixed32_decode */
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8)
       | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* table_builder.c:155-213 for n consecutive data blocks: block i's raw
   contents raw[off[i] .. +len[i]) are snappy-encoded when `compression` is
   1 (LDB_SNAPPY_COMPRESSION), kept only when they shrink by more than 12.5 %
   (:190), then written with their type byte and masked CRC trailer
   (:123-153) at file offset base + (bytes written so far).  `file` receives
   the bytes of file offsets [base, *end).  scratch must hold the largest
   encode bound.  Returns 0. */
int
oracle_table_write_blocks(const uint8_t *raw, const uint64_t *off, const uint32_t *len,
                          uint32_t n, int compression, uint64_t base, uint8_t *file,
                          uint64_t *handle_off, uint64_t *handle_size, uint64_t *end,
                          uint8_t *scratch) {
  uint64_t at = base;
  uint32_t i;
  for (i = 0; i < n; i++) {
    const uint8_t *x = raw + off[i];
    const uint8_t *contents = x;
    size_t size = len[i];
    uint8_t type = 0;
    uint32_t crc;
    uint8_t *dst = file + (at - base);
    if (compression == 1) {
      size_t zn = oracle_snappy_encode(scratch, x, len[i]);       /* :182-188 */
      if (zn < (size_t)len[i] - (size_t)len[i] / 8) {           /* :190     */
        contents = scratch;
        size = zn;
        type = 1;
      }
    }
    handle_off[i] = at;                                          /* :128-129 */
    handle_size[i] = size;
    memcpy(dst, contents, size);
    dst[size] = type;                                            /* :137     */
    crc = oracle_crc32c_extend(0, contents, size);               /* :139-140 */
    crc = oracle_crc32c_extend(crc, &type, 1);
    orc_put32(dst + size + 1, oracle_crc32c_mask(crc));          /* :142     */
    at += size + ORC_TRAILER;                                    /* :150     */
  }
  *end = at;
  return 0;
}

/* format.c:162-270 on an in-memory file image: the block at handle
   (off, size).  Returns an ORACLE_ST_* code; on ORACLE_ST_OK the block
   contents (decoded if snappy) are in out[0 .. *out_len) (out_cap bytes of
   room; ORACLE_ST_NOSPACE if they do not fit). */
int
oracle_table_read_block(const uint8_t *file, uint64_t file_len, uint64_t off,
                        uint64_t size, int verify, uint8_t *out, size_t out_cap,
                        size_t *out_len) {
  const uint8_t *data;
  size_t ulen;
  *out_len = 0;
  if (size > (uint64_t)-1 - ORC_TRAILER)                        /* :174-175 */
    return ORACLE_ST_CORRUPT;
  if (off > file_len || file_len - off < size + ORC_TRAILER)    /* :195-198 */
    return ORACLE_ST_IOERR;
  data = file + off;
  if (verify) {                                                  /* :203-211 */
    uint32_t crc = oracle_crc32c_unmask(orc_get32(data + size + 1));
    uint32_t actual = oracle_crc32c_extend(0, data, (size_t)size + 1);
    if (crc != actual)
      return ORACLE_ST_BADCRC;
  }
  switch (data[size]) {
    case 0:                                                      /* :213-231 */
      if (size > out_cap)
        return ORACLE_ST_NOSPACE;
      memcpy(out, data, (size_t)size);
      *out_len = (size_t)size;
      return ORACLE_ST_OK;
    case 1:                                                      /* :233-261 */
      if (!oracle_snappy_decode_size(&ulen, data, (size_t)size))
        return ORACLE_ST_CORRUPT;
      if (ulen > out_cap)
        return ORACLE_ST_NOSPACE;
      if (!oracle_snappy_decode(out, data, (size_t)size))
        return ORACLE_ST_CORRUPT;
      *out_len = ulen;
      return ORACLE_ST_OK;
    default:                                                     /* :263-267 */
      return ORACLE_ST_BADTYPE;
  }
}
