/*
 * snappy_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A plain-C89 restatement of lcdb's raw Snappy block codec
 * (/root/reference/src/util/snappy.c, chjj/lcdb @ 2026-03-13).  It exists so
 * that tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg can
 * check the HIP path against an independent CPU statement of the algorithm.
 * Nothing in lcdb_amd/ links, loads or calls this file: the product path is
 * the HIP library, which fails loudly when it is absent.
 *
 * Parity pin: every function below is checked byte-for-byte against
 *   (1) the reference's own known answers (test/t-snappy.c:40 ramp size
 *       53203; t-snappy.c:90-96 golang .rawsnappy decode; t-snappy.c:47,74
 *       round trips), committed under tests/golden/, and
 *   (2) golden vectors produced by the reference snappy.c itself, compiled
 *       unmodified from /root/reference by oracle/Makefile into oracle/_ref/
 *       (tests/golden/make_golden.py).
 *
 * lcdb-specific behaviour restated here (and NOT golang/snappy's):
 *   - hash table capped at 2048 u16 entries (snappy.c:25);
 *   - the post-copy repeat test compares 7 input bytes, zero-extended,
 *     against a 4-byte load in 64-bit arithmetic (snappy.c:182).
 */

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "snappy_oracle.h"

/* Format constants: snappy.c:25-35. */
#define ORC_TABLE_CAP   2048u          /* MAX_TABLE_SIZE (1 << 11)       */
#define ORC_MARGIN      15u            /* INPUT_MARGIN (16 - 1)          */
#define ORC_MIN_BLOCK   17u            /* MIN_BLOCK_SIZE                 */
#define ORC_CHUNK       65536u         /* MAX_BLOCK_SIZE                 */
#define ORC_HASH_MUL    0x1e35a7bdu    /* snappy.c:46                    */

/* Little-endian loads: coding.h:33-63 (ldb_fixed32/64_decode). */
static uint32_t
orc_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8)
       | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint64_t
orc_le64(const uint8_t *p) {
  return (uint64_t)orc_le32(p) | ((uint64_t)orc_le32(p + 4) << 32);
}

/* snappy.c:44-47: multiply in 32 bits, keep the top bits. */
static uint32_t
orc_hash(uint32_t v, unsigned shift) {
  return (uint32_t)(v * ORC_HASH_MUL) >> shift;
}

/* coding.h:140-167: varint32 writer. */
static uint8_t *
orc_put_varint32(uint8_t *out, uint32_t v) {
  while (v >= 0x80) {
    *out++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *out++ = (uint8_t)v;
  return out;
}

/* coding.h:169-204: varint32 reader.  At most five bytes are consumed
   (shift 0..28); bits shifted past 32 are dropped; a fifth byte with the
   continuation bit set, or running out of input, is a failure. */
static int
orc_get_varint32(uint32_t *v, const uint8_t **pp, size_t *np) {
  uint32_t acc = 0;
  unsigned sh;

  for (sh = 0; sh <= 28 && *np > 0; sh += 7) {
    uint32_t b = **pp;

    (*pp)++;
    (*np)--;

    if ((b & 0x80) == 0) {
      *v = acc | (b << sh);
      return 1;
    }

    acc |= (b & 0x7f) << sh;
  }

  *v = 0;
  return 0;
}

/* snappy.c:53-73: literal header (1, 2 or 3 bytes) then the bytes. */
static uint8_t *
orc_literal(uint8_t *out, const uint8_t *src, size_t len) {
  size_t m = len - 1;

  if (m < 60) {
    *out++ = (uint8_t)(m << 2);
  } else if (m < 256) {
    *out++ = 0xf0;                      /* 60 << 2 */
    *out++ = (uint8_t)m;
  } else {
    *out++ = 0xf4;                      /* 61 << 2 */
    *out++ = (uint8_t)(m & 0xff);
    *out++ = (uint8_t)(m >> 8);
  }

  memcpy(out, src, len);
  return out + len;
}

/* snappy.c:75-102: copy pieces.  64-byte COPY2 pieces while len >= 68,
   one 60-byte COPY2 if len is then > 64, then a final COPY2 (len >= 12 or
   offset >= 2048) or COPY1.  COPY4 is never produced. */
static uint8_t *
orc_copy(uint8_t *out, uint32_t dist, uint32_t len) {
  uint8_t lo = (uint8_t)(dist & 0xff);
  uint8_t hi = (uint8_t)((dist >> 8) & 0xff);

  for (; len >= 68; len -= 64) {
    out[0] = 0xfe; out[1] = lo; out[2] = hi;  /* (63 << 2) | 2 */
    out += 3;
  }

  if (len > 64) {
    out[0] = 0xee; out[1] = lo; out[2] = hi;  /* (59 << 2) | 2 */
    out += 3;
    len -= 60;
  }

  if (len < 12 && dist < 2048) {
    out[0] = (uint8_t)(((dist >> 8) << 5) | ((len - 4) << 2) | 1);
    out[1] = lo;
    return out + 2;
  }

  out[0] = (uint8_t)(((len - 1) << 2) | 2);
  out[1] = lo;
  out[2] = hi;
  return out + 3;
}

/* snappy.c:104-195: greedy LZ77 over one chunk, 17 <= n <= 65536. */
static uint8_t *
orc_chunk(uint8_t *out, const uint8_t *in, size_t n) {
  uint16_t tab[ORC_TABLE_CAP];
  size_t tsize = 256;
  unsigned shift = 24;
  size_t last = n - ORC_MARGIN;     /* probes may not run past this */
  size_t lit = 0;                   /* start of pending literal bytes */
  size_t at = 1;                    /* current probe position */
  size_t ref = 0;                   /* candidate match position */
  uint32_t h;

  /* Table size: smallest power of two >= n, between 256 and 2048
     (snappy.c:122-125). */
  while (tsize < ORC_TABLE_CAP && tsize < n) {
    tsize <<= 1;
    shift--;
  }
  memset(tab, 0, tsize * sizeof(tab[0]));

  h = orc_hash(orc_le32(in + at), shift);

  for (;;) {
    /* Literal search with the skip heuristic (snappy.c:133-154). */
    uint32_t skip = 32;
    size_t ahead = at;

    for (;;) {
      at = ahead;
      ahead = at + (skip >> 5);
      skip += skip >> 5;

      if (ahead > last)
        goto tail;

      ref = tab[h];
      tab[h] = (uint16_t)at;
      h = orc_hash(orc_le32(in + ahead), shift);

      if (orc_le32(in + at) == orc_le32(in + ref))
        break;
    }

    out = orc_literal(out, in + lit, at - lit);

    /* Copies, including immediate re-matches (snappy.c:158-187). */
    for (;;) {
      size_t start = at;
      size_t r = ref + 4;
      uint64_t w;

      at += 4;
      while (at < n && in[r] == in[at]) {
        r++;
        at++;
      }

      out = orc_copy(out, (uint32_t)(start - ref), (uint32_t)(at - start));
      lit = at;

      if (at >= last)
        goto tail;

      w = orc_le64(in + at - 1);
      tab[orc_hash((uint32_t)w, shift)] = (uint16_t)(at - 1);

      h = orc_hash((uint32_t)(w >> 8), shift);
      ref = tab[h];
      tab[h] = (uint16_t)at;

      /* lcdb quirk (snappy.c:182): 64-bit compare of w >> 8 (bytes
         at..at+6) against a zero-extended 32-bit load. */
      if ((w >> 8) != (uint64_t)orc_le32(in + ref)) {
        h = orc_hash((uint32_t)(w >> 16), shift);
        at++;
        break;
      }
    }
  }

tail:
  if (lit < n)
    out = orc_literal(out, in + lit, n - lit);

  return out;
}

/* snappy.c:347-362 */
int
oracle_snappy_encode_size(size_t *zn, size_t xn) {
  size_t bound;

  if (xn > 0x7fffffff)
    return 0;

  bound = 32 + xn + xn / 6;

  if (bound > 0x7fffffff)
    return 0;

  *zn = bound;
  return 1;
}

/* snappy.c:364-384: header, 64 KiB chunks, short tail as a literal. */
size_t
oracle_snappy_encode(uint8_t *zp, const uint8_t *xp, size_t xn) {
  uint8_t *out = orc_put_varint32(zp, (uint32_t)xn);
  size_t done = 0;

  while (xn - done >= ORC_CHUNK) {
    out = orc_chunk(out, xp + done, ORC_CHUNK);
    done += ORC_CHUNK;
  }

  if (xn - done >= ORC_MIN_BLOCK)
    out = orc_chunk(out, xp + done, xn - done);
  else if (xn - done > 0)
    out = orc_literal(out, xp + done, xn - done);

  return (size_t)(out - zp);
}

/* snappy.c:386-399 */
int
oracle_snappy_decode_size(size_t *zn, const uint8_t *xp, size_t xn) {
  uint32_t v;

  if (!orc_get_varint32(&v, &xp, &xn))
    return 0;

  if (v > 0x7fffffff)
    return 0;

  *zn = v;
  return 1;
}

/* snappy.c:201-341: tag interpreter.  Returns 1 iff the stream fills
   exactly `want` bytes with every check passing. */
static int
orc_run_tags(uint8_t *dst, size_t want, const uint8_t *p, size_t left) {
  size_t made = 0;
  uint32_t len = 0, dist = 0;

  while (left > 0) {
    uint32_t tag = p[0];

    if ((tag & 3) == 0) {
      /* Literal: length-1 in the tag, or in 1..4 following bytes
         (snappy.c:210-273). */
      uint32_t m = tag >> 2;
      size_t extra = 0;

      p++;
      left--;

      if (m >= 60) {
        size_t k;

        extra = m - 59;
        if (left < extra)
          return 0;

        m = 0;
        for (k = 0; k < extra; k++)
          m |= (uint32_t)p[k] << (8 * k);

        p += extra;
        left -= extra;
      }

      if (m >= 0x7fffffff)
        return 0;

      len = m + 1;

      if (len > want - made || len > left)
        return 0;

      memcpy(dst + made, p, len);
      made += len;
      p += len;
      left -= len;
      continue;
    }

    if ((tag & 3) == 1) {
      /* COPY1: 3-bit length, 11-bit offset (snappy.c:276-287). */
      if (left < 2)
        return 0;

      len = 4 + ((tag >> 2) & 7);
      dist = ((tag & 0xe0) << 3) | p[1];
      p += 2;
      left -= 2;
    } else if ((tag & 3) == 2) {
      /* COPY2: 6-bit length, 16-bit offset (snappy.c:289-301). */
      if (left < 3)
        return 0;

      len = 1 + (tag >> 2);
      dist = (uint32_t)p[1] | ((uint32_t)p[2] << 8);
      p += 3;
      left -= 3;
    } else {
      /* COPY4: 6-bit length, 32-bit offset (snappy.c:303-317). */
      if (left < 5)
        return 0;

      len = 1 + (tag >> 2);
      dist = orc_le32(p + 1);
      p += 5;
      left -= 5;
    }

    /* snappy.c:320-324 */
    if (dist == 0 || dist >= 0x80000000u)
      return 0;

    if (made < dist || len > want - made)
      return 0;

    /* snappy.c:326-331: forward byte order gives run-length semantics
       when the source overlaps the destination. */
    {
      uint8_t *w = dst + made;
      const uint8_t *r = w - dist;
      uint32_t i;

      for (i = 0; i < len; i++)
        w[i] = r[i];
    }

    made += len;
  }

  return made == want;   /* snappy.c:337 */
}

/* snappy.c:401-412 */
int
oracle_snappy_decode(uint8_t *zp, const uint8_t *xp, size_t xn) {
  uint32_t want;

  if (!orc_get_varint32(&want, &xp, &xn))
    return 0;

  if (want > 0x7fffffff)
    return 0;

  return orc_run_tags(zp, want, xp, xn);
}
