/*
 * bloom_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker for the bloom
 * filter row, see bloom_oracle.c).
 */
#ifndef LCDB_ORACLE_BLOOM_H
#define LCDB_ORACLE_BLOOM_H

#include <stddef.h>
#include <stdint.h>

uint32_t oracle_hash(const uint8_t *data, size_t size, uint32_t seed);
uint32_t oracle_bloom_k(int bits_per_key);
size_t oracle_bloom_bytes(size_t n, int bits_per_key);
size_t oracle_bloom_build(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                          size_t n, int bits_per_key, uint8_t *out);
int oracle_bloom_match(const uint8_t *filter, size_t len, const uint8_t *key, size_t klen);

size_t oracle_filter_block_build(const uint8_t *base, const uint64_t *key_off,
                                 const uint32_t *key_len, const uint32_t *block_first,
                                 const uint64_t *block_off, uint32_t nblocks, uint64_t data_end,
                                 int bits_per_key, uint32_t trim, uint8_t *out,
                                 uint32_t *filter_offsets);
int oracle_filter_matches(const uint8_t *block, size_t n, uint64_t block_offset,
                          const uint8_t *key, size_t klen, uint32_t trim);

#endif
