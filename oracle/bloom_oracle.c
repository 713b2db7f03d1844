/*
 * bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker for SURVEY.md
 * §8(f) row 4: lcdb's bloom filter).
 *
 * A plain-C89 restatement of
 *   - ldb_hash (src/util/hash.c:22-58), the murmur-like hash;
 *   - the builtin bloom policy (src/util/bloom.c:24-165): k from
 *     bits_per_key (:35-45), filter size (:69-80), the double-hashed probes
 *     of bloom_add (:82-100), bloom_build (:102-119: bits, then one byte k)
 *     and bloom_match (:121-165);
 *   - the filter block (src/table/filter_block.c:79-225): one filter per
 *     2 KiB of data-block offsets, built the way the table builder drives it
 *     (table_builder.c:242-243, 276-277, 294), and ldb_filter_matches.
 * Nothing in lcdb_amd/ links, loads or calls this file.
 *
 * Parity pin: the known answers of test/t-hash.c:33-38, and filters built
 * and probed by the reference's own bloom.c + hash.c (oracle/harness/
 * bloom_ref.c, linked against lcdb's sources by oracle/lcdb.mk).
 */

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
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

/* ---- the filter block (src/table/filter_block.c) ---- */

static void
orc_put32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

/* The filter block of one table, as lcdb's table builder makes it: for each
   data block b in file order, its keys [block_first[b], block_first[b + 1])
   go to ldb_filtergen_add_key (table_builder.c:242-243), then the block is
   written and ldb_filtergen_start_block(offset after the block) runs
   (table_builder.c:276-277); ldb_filtergen_finish (table_builder.c:294) at the
   end.  The offset after block b is block_off[b + 1] (data_end for the last).
   filter_block.c:79-150 restated: `generate` turns the pending keys into one
   filter (or an empty one) and records its offset; start_block generates
   until there is one filter per started 2 KiB (LDB_FILTER_BASE_LG = 11).
   trim = 8 restates the internal filter policy (dbformat.c:308-326: user key
   = key without its 8-byte trailer).  Writes to out (no bound check: size it
   with oracle_filter_block_bound) and returns the size. */
size_t
oracle_filter_block_build(const uint8_t *base, const uint64_t *key_off, const uint32_t *key_len,
                          const uint32_t *block_first, const uint64_t *block_off,
                          uint32_t nblocks, uint64_t data_end, int bits_per_key, uint32_t trim,
                          uint8_t *out, uint32_t *filter_offsets) {
  size_t result = 0;          /* bytes of filters so far */
  uint32_t nfilt = 0;         /* filter_offsets.length */
  uint32_t pend0 = 0, pend1 = 0;   /* pending keys [pend0, pend1) */
  uint32_t b, f;

  for (b = 0; b <= nblocks; b++) {
    uint64_t end, index;
    if (b < nblocks) {
      pend1 = block_first[b + 1];            /* add_key for the block's keys */
      end = b + 1 < nblocks ? block_off[b + 1] : data_end;
      index = end >> 11;                     /* start_block, :114-121 */
    } else {
      index = 0;                             /* finish, :131-150 */
      if (pend1 > pend0)
        index = (uint64_t)nfilt + 1;
    }
    while (index > nfilt) {                  /* generate, :79-112 */
      filter_offsets[nfilt++] = (uint32_t)result;
      if (pend1 > pend0) {
        size_t n = pend1 - pend0, i;
        uint64_t *o = (uint64_t *)malloc(n * sizeof(uint64_t));
        uint32_t *l = (uint32_t *)malloc(n * sizeof(uint32_t));
        for (i = 0; i < n; i++) {
          o[i] = key_off[pend0 + i];
          l[i] = key_len[pend0 + i] > trim ? key_len[pend0 + i] - trim : 0;
        }
        result += oracle_bloom_build(base, o, l, n, bits_per_key, out + result);
        free(o);
        free(l);
        pend0 = pend1;
      }
    }
  }
  for (f = 0; f < nfilt; f++)
    orc_put32(out + result + 4 * f, filter_offsets[f]);
  orc_put32(out + result + 4 * nfilt, (uint32_t)result);
  out[result + 4 * nfilt + 4] = 11;          /* LDB_FILTER_BASE_LG */
  return result + 4 * (size_t)nfilt + 5;
}

/* ldb_filter_init + ldb_filter_matches (filter_block.c:170-225) for the key
   of a data block at block_offset; trim as above (ldb_ifp_match,
   dbformat.c:328-334). */
int
oracle_filter_matches(const uint8_t *block, size_t n, uint64_t block_offset,
                      const uint8_t *key, size_t klen, uint32_t trim) {
  uint32_t base_lg, last_word, start, limit;
  uint64_t index, num;
  if (n < 5)
    return 1;                                /* num = 0 */
  base_lg = block[n - 1] & 63;
  last_word = orc_le32(block + n - 5);
  if (last_word > n - 5)
    return 1;
  num = (n - 5 - last_word) / 4;
  index = block_offset >> base_lg;
  if (index >= num)
    return 1;
  start = orc_le32(block + last_word + index * 4);
  limit = orc_le32(block + last_word + index * 4 + 4);
  if (start <= limit && limit <= last_word)
    return oracle_bloom_match(block + start, limit - start, key, klen > trim ? klen - trim : 0);
  if (start == limit)
    return 0;
  return 1;
}
