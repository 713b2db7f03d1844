/*
 * bloom_ref.c -- TEST INFRASTRUCTURE ONLY: a ctypes-callable face of the
 * REFERENCE's own bloom filter (src/util/bloom.c, src/util/hash.c), linked
 * against lcdb's sources by oracle/lcdb.mk into _ref/lcdb/libref_bloom.so.
 * and filter block (src/table/filter_block.c).  It pins the bloom and filter
 * block restatement (oracle/bloom_oracle.c) and checks the GPU kernels
 * (lgs_bloom_*, lgs_filter_block_*) against the reference itself.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "util/bloom.h"
#include "util/buffer.h"
#include "util/hash.h"
#include "util/slice.h"
#include "util/types.h"
#include "dbformat.h"
#include "table/filter_block.h"

uint32_t
ref_hash(const uint8_t *data, size_t size, uint32_t seed) {
  return ldb_hash(data, size, seed);
}

/* ldb_bloom_build over keys i = base[off[i] .. + len[i]) with a policy of
   bits_per_key (ldb_bloom_init).  Copies the filter to out (cap bytes) and
   returns its size, or 0 if it does not fit. */
size_t
ref_bloom_build(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                int bits_per_key, uint8_t *out, size_t cap) {
  ldb_bloom_t bloom;
  ldb_buffer_t dst;
  ldb_slice_t *keys = (ldb_slice_t *)malloc((n ? n : 1) * sizeof(ldb_slice_t));
  size_t i, size;
  ldb_bloom_init(&bloom, bits_per_key);
  ldb_buffer_init(&dst);
  for (i = 0; i < n; i++)
    ldb_slice_set(&keys[i], base + off[i], len[i]);
  ldb_bloom_build(&bloom, &dst, keys, n);
  size = dst.size;
  if (size <= cap)
    memcpy(out, dst.data, size);
  else
    size = 0;
  ldb_buffer_clear(&dst);
  free(keys);
  return size;
}

int
ref_bloom_match(const uint8_t *filter, size_t flen, const uint8_t *key, size_t klen) {
  ldb_slice_t f, k;
  ldb_slice_set(&f, filter, flen);
  ldb_slice_set(&k, key, klen);
  return ldb_bloom_match(ldb_bloom_default, &f, &k);
}

/* The filter block of one table through lcdb's own filter_block.c, driven the
   way its table builder drives it (table_builder.c:242-243, 276-277, 294):
   per data block b, add_key for keys [block_first[b], block_first[b+1]),
   then start_block(offset after the block = block_off[b+1], data_end for the
   last); finish.  internal != 0 uses the internal filter policy (dbformat.c
   ldb_ifp_*: filters over user keys = keys without their 8-byte trailer).
   Copies the block to out (cap bytes); returns its size, or 0 if it does not
   fit. */
size_t
ref_filter_block_build(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       const uint32_t *block_first, const uint64_t *block_off, uint32_t nblocks,
                       uint64_t data_end, int bits_per_key, int internal, uint8_t *out,
                       size_t cap) {
  ldb_bloom_t user, ifp;
  ldb_filtergen_t fb;
  ldb_slice_t res, key;
  uint32_t b, i;
  size_t size;
  ldb_bloom_init(&user, bits_per_key);
  ldb_ifp_init(&ifp, &user);
  ldb_filtergen_init(&fb, internal ? &ifp : &user);
  ldb_filtergen_start_block(&fb, 0);                 /* table_builder.c:92 */
  for (b = 0; b < nblocks; b++) {
    for (i = block_first[b]; i < block_first[b + 1]; i++) {
      ldb_slice_set(&key, base + off[i], len[i]);
      ldb_filtergen_add_key(&fb, &key);
    }
    ldb_filtergen_start_block(&fb, b + 1 < nblocks ? block_off[b + 1] : data_end);
  }
  res = ldb_filtergen_finish(&fb);
  size = res.size;
  if (size <= cap)
    memcpy(out, res.data, size);
  else
    size = 0;
  ldb_filtergen_clear(&fb);
  return size;
}

/* ldb_filter_init + ldb_filter_matches (filter_block.c:170-225). */
int
ref_filter_matches(const uint8_t *block, size_t n, uint64_t block_offset, const uint8_t *key,
                   size_t klen, int internal) {
  ldb_bloom_t ifp;
  ldb_filter_t fr;
  ldb_slice_t c, k;
  ldb_ifp_init(&ifp, ldb_bloom_default);
  ldb_slice_set(&c, block, n);
  ldb_slice_set(&k, key, klen);
  ldb_filter_init(&fr, internal ? &ifp : ldb_bloom_default, &c);
  return ldb_filter_matches(&fr, block_offset, &k);
}
