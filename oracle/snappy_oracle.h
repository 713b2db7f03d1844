/*
 * snappy_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker, see
 * snappy_oracle.c).  Same argument meaning and return values as lcdb's
 * src/util/snappy.h:28-38, under distinct names so the oracle can never be
 * mistaken for (or linked in place of) the product's ldb_snappy_* symbols.
 */
#ifndef LCDB_ORACLE_SNAPPY_H
#define LCDB_ORACLE_SNAPPY_H

#include <stddef.h>
#include <stdint.h>

int oracle_snappy_encode_size(size_t *zn, size_t xn);
size_t oracle_snappy_encode(uint8_t *zp, const uint8_t *xp, size_t xn);
int oracle_snappy_decode_size(size_t *zn, const uint8_t *xp, size_t xn);
int oracle_snappy_decode(uint8_t *zp, const uint8_t *xp, size_t xn);

#endif
