/*
 * table_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker for the block
 * framing rows, see table_oracle.c).  Status codes equal the product's
 * LGS_ST_* values (include/lcdb_gpu_snappy.h) so tests compare them directly.
 */
#ifndef LCDB_ORACLE_TABLE_H
#define LCDB_ORACLE_TABLE_H

#include <stddef.h>
#include <stdint.h>

#define ORACLE_ST_CORRUPT 0   /* LDB_CORRUPTION: snappy header/stream       */
#define ORACLE_ST_OK      1
#define ORACLE_ST_NOSPACE 2
#define ORACLE_ST_IOERR   3   /* LDB_IOERR: truncated block read            */
#define ORACLE_ST_BADCRC  4   /* LDB_CORRUPTION: block checksum mismatch    */
#define ORACLE_ST_BADTYPE 5   /* LDB_CORRUPTION: bad block type             */

uint32_t oracle_crc32c_extend(uint32_t z, const uint8_t *xp, size_t xn);
uint32_t oracle_crc32c_mask(uint32_t crc);
uint32_t oracle_crc32c_unmask(uint32_t masked);

int oracle_table_write_blocks(const uint8_t *raw, const uint64_t *off, const uint32_t *len,
                              uint32_t n, int compression, uint64_t base, uint8_t *file,
                              uint64_t *handle_off, uint64_t *handle_size, uint64_t *end,
                              uint8_t *scratch);

int oracle_table_read_block(const uint8_t *file, uint64_t file_len, uint64_t off,
                            uint64_t size, int verify, uint8_t *out, size_t out_cap,
                            size_t *out_len);

#endif
