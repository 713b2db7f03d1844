/*
 * corpus.c -- synthetic SSTable data blocks shaped like lcdb's db_bench
 * fillseq workload (bench / test input generator, host C).
 *
 * Restates, from the reference's behaviour:
 *   - value ring: Park-Miller RNG seeded 301 (src/util/random.c:22-55),
 *     ldb_compressible_string(ratio 0.5, len 100) pieces appended until the
 *     ring holds >= 1 MiB (bench/db_bench.c:206-227, src/util/testutil.c:76-103,
 *     random string = ' ' + uniform(95), testutil.c:37-51); values are
 *     consecutive 100-byte slices, wrapping to 0 (db_bench.c:235-246);
 *   - keys "%016d" (db_bench.c:253-257) as internal keys with the 8-byte
 *     little-endian tag (seq << 8) | 1, seq = k + 1;
 *   - block layout of src/table/block_builder.c:76-151 (restart interval 16,
 *     shared-prefix key deltas, restart array + count) flushed when the size
 *     estimate reaches block_size (src/table/table_builder.c:251-254).
 *
 * Also a splitmix64 random-bytes filler (seed 0x5eed in SURVEY §8d) for the
 * incompressible half of the mixed corpus.
 */

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define RING_MIN   1048576u
#define VALUE_LEN  100u
#define RESTART_K  16u

static uint8_t *g_ring;
static size_t g_ring_len;

static uint32_t
pm_next(uint32_t *seed) {
  uint64_t prod = (uint64_t)(*seed) * 16807u;
  uint32_t s = (uint32_t)((prod >> 31) + (prod & 0x7fffffffu));
  if (s > 0x7fffffffu)
    s -= 0x7fffffffu;
  *seed = s;
  return s;
}

static int
ring_build(void) {
  uint32_t seed = 301;
  size_t cap = RING_MIN + VALUE_LEN;
  uint8_t piece[VALUE_LEN];
  uint8_t chunk[VALUE_LEN];
  size_t chunklen = (size_t)(VALUE_LEN * 0.5);

  if (g_ring)
    return 0;

  g_ring = (uint8_t *)malloc(cap);
  if (!g_ring)
    return -1;

  g_ring_len = 0;
  while (g_ring_len < RING_MIN) {
    size_t i, filled = 0;
    for (i = 0; i < chunklen; i++)
      chunk[i] = (uint8_t)(' ' + pm_next(&seed) % 95u);
    while (filled < VALUE_LEN) {
      size_t take = chunklen;
      if (take > VALUE_LEN - filled)
        take = VALUE_LEN - filled;
      memcpy(piece + filled, chunk, take);
      filled += take;
    }
    memcpy(g_ring + g_ring_len, piece, VALUE_LEN);
    g_ring_len += VALUE_LEN;
  }
  return 0;
}

static uint8_t *
put_varint(uint8_t *p, uint32_t v) {
  while (v >= 0x80) {
    *p++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *p++ = (uint8_t)v;
  return p;
}

static void
make_ikey(uint8_t *k, uint32_t key) {
  uint64_t tag = ((uint64_t)key + 1) << 8 | 1u;
  char txt[32];
  int i;
  snprintf(txt, sizeof txt, "%016d", (int)key);
  memcpy(k, txt, 16);
  for (i = 0; i < 8; i++)
    k[16 + i] = (uint8_t)(tag >> (8 * i));
}

/* Build one data block into dst (cap bytes).  Returns its length, or 0 if
   cap is too small.  *key and *ring_pos advance past the entries used. */
static size_t
fill_block(uint8_t *dst, size_t cap, uint32_t block_size,
           uint32_t *key, uint32_t *ring_pos) {
  uint32_t restarts[4096];
  uint32_t nrestart = 1, counter = 0;
  uint8_t last[24];
  int have_last = 0;
  uint8_t *p = dst;

  restarts[0] = 0;

  for (;;) {
    uint8_t ik[24];
    size_t shared = 0, est;
    const uint8_t *val;

    make_ikey(ik, *key);

    if (*ring_pos + VALUE_LEN > g_ring_len)
      *ring_pos = 0;
    val = g_ring + *ring_pos;

    if (counter < RESTART_K) {
      if (have_last)
        while (shared < 24 && last[shared] == ik[shared])
          shared++;
    } else {
      if (nrestart >= 4096)
        return 0;
      restarts[nrestart++] = (uint32_t)(p - dst);
      counter = 0;
    }

    if ((size_t)(p - dst) + 15 + (24 - shared) + VALUE_LEN + 4 * (nrestart + 1) > cap)
      return 0;

    p = put_varint(p, (uint32_t)shared);
    p = put_varint(p, (uint32_t)(24 - shared));
    p = put_varint(p, VALUE_LEN);
    memcpy(p, ik + shared, 24 - shared);
    p += 24 - shared;
    memcpy(p, val, VALUE_LEN);
    p += VALUE_LEN;

    memcpy(last, ik, 24);
    have_last = 1;
    counter++;
    (*key)++;
    *ring_pos += VALUE_LEN;

    est = (size_t)(p - dst) + 4 * nrestart + 4;
    if (est >= block_size)
      break;
  }

  {
    uint32_t i;
    for (i = 0; i <= nrestart; i++) {
      uint32_t v = i < nrestart ? restarts[i] : nrestart;
      p[0] = (uint8_t)v;
      p[1] = (uint8_t)(v >> 8);
      p[2] = (uint8_t)(v >> 16);
      p[3] = (uint8_t)(v >> 24);
      p += 4;
    }
  }
  return (size_t)(p - dst);
}

/*
 * Round-robin shard of a fillseq stream: of the blocks the stream produces,
 * keep block g when g % stride == phase, until n are kept (block g of the
 * unsharded stream is the same block in every shard).  Kept block i starts
 * at off[i] (rounded up to `align`, a power of two) and is len[i] bytes.
 * key0 / ring0 give the generator state of block 0 (0 / 0 reproduces a fresh
 * db_bench run).  Returns total bytes used, or 0 on failure (cap too small).
 */
uint64_t
corpus_fillseq_shard(uint8_t *dst, uint64_t cap, uint64_t *off, uint32_t *len,
                     uint32_t n, uint32_t block_size, uint32_t align,
                     uint32_t key0, uint32_t ring0, uint32_t stride,
                     uint32_t phase) {
  uint64_t at = 0;
  uint32_t key = key0, ring = ring0, i = 0, g;
  uint8_t *skip = NULL;
  size_t skip_cap = (size_t)block_size * 2 + 8192;

  if (ring_build() != 0 || align == 0 || (align & (align - 1)) != 0 ||
      stride == 0 || phase >= stride)
    return 0;
  if (stride > 1 && (skip = (uint8_t *)malloc(skip_cap)) == NULL)
    return 0;

  for (g = 0; i < n; g++) {
    size_t got;
    if (g % stride != phase) {
      got = fill_block(skip, skip_cap, block_size, &key, &ring);
      if (got == 0)
        break;
      continue;
    }
    at = (at + align - 1) & ~(uint64_t)(align - 1);
    if (at >= cap)
      break;
    got = fill_block(dst + at, (size_t)(cap - at), block_size, &key, &ring);
    if (got == 0)
      break;
    off[i] = at;
    len[i] = (uint32_t)got;
    at += got;
    i++;
  }
  free(skip);
  return i == n ? at : 0;
}

/* The unsharded stream: n blocks from key0 / ring0. */
uint64_t
corpus_fillseq(uint8_t *dst, uint64_t cap, uint64_t *off, uint32_t *len,
               uint32_t n, uint32_t block_size, uint32_t align,
               uint32_t key0, uint32_t ring0) {
  return corpus_fillseq_shard(dst, cap, off, len, n, block_size, align, key0,
                              ring0, 1, 0);
}

/* splitmix64 byte stream. */
void
corpus_random(uint8_t *dst, uint64_t nbytes, uint64_t seed) {
  uint64_t s = seed, i = 0;
  while (i < nbytes) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    int k;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    for (k = 0; k < 8 && i < nbytes; k++, i++)
      dst[i] = (uint8_t)(z >> (8 * k));
  }
}

/* Return the value ring (for tests). */
const uint8_t *
corpus_ring(uint64_t *len) {
  if (ring_build() != 0)
    return NULL;
  *len = g_ring_len;
  return g_ring;
}
