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

#endif
