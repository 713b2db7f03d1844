/*
 * bloom_ref.c -- TEST INFRASTRUCTURE ONLY: a ctypes-callable face of the
 * REFERENCE's own bloom filter (src/util/bloom.c, src/util/hash.c), linked
 * against lcdb's sources by oracle/lcdb.mk into _ref/lcdb/libref_bloom.so.
 * It pins the bloom restatement (oracle/bloom_oracle.c) and checks the GPU
 * kernels (lgs_bloom_*) against the reference itself.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "util/bloom.h"
#include "util/buffer.h"
#include "util/hash.h"
#include "util/slice.h"

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
