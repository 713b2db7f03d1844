/*
 * bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker for SURVEY.md
 * §8(f) row 4: lcdb's bloom filter).
 *
 * A plain-C89 restatement of
 *   - ldb_hash (src/util/hash.c:22-58), the murmur-like hash;
 *   - the builtin bloom policy (src/util/bloom.c:24-165): k from
 *     bits_per_key (:35-45), filter size (:69-80), the double-hashed probes
 *     of bloom_add (:82-100), bloom_build (:102-119: bits, then one byte k)
 *     and bloom_match (:121-165).
 * Nothing in lcdb_amd/ links, loads or calls this file.
 *
 * Parity pin: the known answers of test/t-hash.c:33-38, and filters built
 * and probed by the reference's own bloom.c + hash.c (oracle/harness/
 * bloom_ref.c, linked against lcdb's sources by oracle/lcdb.mk).
 */

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "bloom_oracle.h"

static uint32_t
orc_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8)
       | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* hash.c:22-58. */
uint32_t
oracle_hash(const uint8_t *data, size_t size, uint32_t seed) {
  const uint32_t m = 0xc6a4a793u;
  uint32_t h = seed ^ (uint32_t)(size * m);
  while (size >= 4) {
    h += orc_le32(data);
    h *= m;
    h ^= (h >> 16);
    data += 4;
    size -= 4;
  }
  switch (size) {
    case 3:
      h += (uint32_t)data[2] << 16;
      /* fallthrough */
    case 2:
      h += (uint32_t)data[1] << 8;
      /* fallthrough */
    case 1:
      h += data[0];
      h *= m;
      h ^= (h >> 24);
      break;
  }
  return h;
}

/* bloom.c:35-45 (k = bits_per_key * 0.69, truncated, clamped to [1, 30]). */
uint32_t
oracle_bloom_k(int bits_per_key) {
  size_t k = (size_t)(bits_per_key * 0.69);
  if (k < 1)
    k = 1;
  if (k > 30)
    k = 30;
  return (uint32_t)k;
}

/* bloom.c:69-80: bytes of filter bits for n keys (the k byte not included). */
size_t
oracle_bloom_bytes(size_t n, int bits_per_key) {
  size_t bits = n * (size_t)bits_per_key;
  if (bits < 64)
    bits = 64;
  return (bits + 7) / 8;
}

/* bloom.c:102-119 with bloom_add (:82-100) inlined: keys i = base[off[i] ..
   + len[i]).  Writes bytes + 1 bytes to out; returns that count. */
size_t
oracle_bloom_build(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                   size_t n, int bits_per_key, uint8_t *out) {
  size_t bytes = oracle_bloom_bytes(n, bits_per_key);
  size_t bits = bytes * 8;
  uint32_t k = oracle_bloom_k(bits_per_key);
  size_t i;
  uint32_t j;
  memset(out, 0, bytes);
  for (i = 0; i < n; i++) {
    uint32_t h = oracle_hash(base + off[i], len[i], 0xbc9f1d34u);   /* :64-67 */
    uint32_t delta = (h >> 17) | (h << 15);
    for (j = 0; j < k; j++) {
      uint32_t pos = (uint32_t)(h % bits);
      out[pos / 8] |= (uint8_t)(1u << (pos % 8));
      h += delta;
    }
  }
  out[bytes] = (uint8_t)k;
  return bytes + 1;
}

/* bloom.c:121-165. */
int
oracle_bloom_match(const uint8_t *filter, size_t len, const uint8_t *key, size_t klen) {
  size_t bits;
  uint32_t k, h, delta, j;
  if (len < 2)
    return 0;
  bits = (len - 1) * 8;
  k = filter[len - 1];
  if (k > 30)
    return 1;
  h = oracle_hash(key, klen, 0xbc9f1d34u);
  delta = (h >> 17) | (h << 15);
  for (j = 0; j < k; j++) {
    uint32_t pos = (uint32_t)(h % bits);
    if ((filter[pos / 8] & (1u << (pos % 8))) == 0)
      return 0;
    h += delta;
  }
  return 1;
}
