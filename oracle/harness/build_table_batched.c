/*
 * build_table_batched.c -- BASELINE config 5 through the BATCHED entry points
 * (test infrastructure, and the worked example of INTEGRATION.md §3.1).
 *
 * Builds the same SSTable as build_table.c, whose every step is lcdb's own
 * (memtable -> ldb_build_table -> ldb_tablegen_*, one snappy call per block),
 * but the way a bulk writer would use the library:
 *   1. the data blocks are cut with lcdb's block builder under the boundary
 *      rule of ldb_tablegen_add (table_builder.c:204-230), keeping each
 *      block's index key (ldb_shortest_separator against the next block's
 *      first key, ldb_short_successor for the last, table_builder.c:213-223,
 *      332-340);
 *   2. ONE lgs_table_write_host call compresses, applies the 12.5 % rule,
 *      frames (type + masked crc32c) and packs every data block at its file
 *      offset (table_builder.c:155-213 for each block);
 *   3. the metaindex and index blocks and the footer are written as
 *      ldb_tablegen_finish writes them (table_builder.c:266-363), through the
 *      drop-in's ldb_snappy_encode;
 *   4. the file is written and synced (builder.c:85-89);
 *   5. every data block is read back with ONE lgs_table_read_host call
 *      (checksums verified, format.c:162-270 per block) and compared with the
 *      raw block it was built from.
 * The .ldb must equal build_table's byte for byte (its SHA-256 is pinned in
 * tests/golden/digests.json for config 5).  Linked only against the drop-in
 * library (oracle/lcdb.mk: build_table_batched.gpu).
 *
 * Entries: db_bench fillseq as in build_table.c (keys "%016d", sequence
 * k + 1, 100-byte values from the seed-301 compressible-string ring), with
 * the internal keys formed directly (dbformat.h ldb_ikey_set) instead of
 * through a memtable: the memtable iterates them in this same order.
 *
 * usage: build_table_batched DIR NUM_ENTRIES [BLOCK_SIZE]
 * prints: rc=0 file_size=N blocks=N raw_bytes=N cut_s=.. init_s=.. write_s=..
 *         write_warm_s=.. finish_s=.. io_s=.. read_s=.. read_bad=0
 * (init_s: HIP start-up; write_s: the first write call, which also grows the
 * pinned staging arena; write_warm_s: the same call again.)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "util/options.h"
#include "dbformat.h"
#include "table/block_builder.h"
#include "table/format.h"
#include "util/buffer.h"
#include "util/coding.h"
#include "util/comparator.h"
#include "util/crc32c.h"
#include "util/env.h"
#include "util/slice.h"
#include "util/status.h"
#include "util/testutil.h"
#include "util/random.h"

#include "lcdb_gpu_snappy.h"

static double
now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *
xrealloc(void *p, size_t n) {
  void *q = realloc(p, n);
  if (q == NULL) {
    fprintf(stderr, "out of memory (%lu bytes)\n", (unsigned long)n);
    exit(3);
  }
  return q;
}

/* ldb_tablegen_write_block + write_raw_block (table_builder.c:117-195) for
   one meta block, appended to the file image at *at. */
static void
put_block(uint8_t **file, size_t *cap, uint64_t *at, ldb_slice_t raw,
          ldb_handle_t *handle) {
  size_t max = 0, zn;
  uint8_t *z, trailer[LDB_TRAILER_SIZE];
  const uint8_t *body = raw.data;
  size_t n = raw.size;
  uint32_t crc;

  if (!ldb_snappy_encode_size(&max, raw.size))
    abort();
  z = xrealloc(NULL, max ? max : 1);
  zn = ldb_snappy_encode(z, raw.data, raw.size);
  trailer[0] = LDB_NO_COMPRESSION;
  if (zn < raw.size - raw.size / 8) {
    body = z;
    n = zn;
    trailer[0] = LDB_SNAPPY_COMPRESSION;
  }
  crc = ldb_crc32c_value(body, n);
  crc = ldb_crc32c_extend(crc, trailer, 1);
  ldb_fixed32_write(trailer + 1, ldb_crc32c_mask(crc));
  if (*at + n + LDB_TRAILER_SIZE > *cap) {
    *cap = (size_t)(*at + n + LDB_TRAILER_SIZE) * 2;
    *file = xrealloc(*file, *cap);
  }
  handle->offset = *at;
  handle->size = n;
  memcpy(*file + *at, body, n);
  memcpy(*file + *at + n, trailer, LDB_TRAILER_SIZE);
  *at += n + LDB_TRAILER_SIZE;
  free(z);
}

int
main(int argc, char **argv) {
  const char *dir;
  char path[4096];
  long num, k;
  ldb_comparator_t icmp;
  ldb_dbopt_t options, index_options;
  ldb_blockgen_t data, index, meta;
  ldb_buffer_t ring, piece, last_key, ikey;
  ldb_rand_t rnd;
  ldb_handle_t meta_handle, index_handle;
  ldb_footer_t footer;
  uint8_t footer_buf[LDB_FOOTER_SIZE];
  ldb_buffer_t footer_enc;
  uint8_t *raw = NULL, *file = NULL, *back = NULL, *status = NULL;
  uint64_t *raw_off = NULL, *hoff = NULL, *hsize = NULL, *keys_off = NULL;
  uint32_t *raw_len = NULL, *back_len = NULL;
  char *keys = NULL;
  size_t raw_cap = 0, raw_at = 0, keys_cap = 0, keys_at = 0, file_cap;
  uint32_t nb = 0, nb_cap = 0, i, bad = 0;
  uint64_t end = 0, at;
  size_t pos = 0;
  int pending = 0, rc;
  double t0, t1, ti, t2, t2w, t3, t4, t5;
  uint64_t end_warm = 0;
  FILE *f;

  if (argc < 3) {
    fprintf(stderr, "usage: %s DIR NUM_ENTRIES [BLOCK_SIZE]\n", argv[0]);
    return 2;
  }
  dir = argv[1];
  num = atol(argv[2]);

  ldb_ikc_init(&icmp, ldb_bytewise_comparator);
  options = *ldb_dbopt_default;
  options.comparator = &icmp;
  if (argc > 3)
    options.block_size = (size_t)atol(argv[3]);
  index_options = options;
  index_options.block_restart_interval = 1;   /* table_builder.c:86 */

  ldb_create_dir(dir);

  ldb_buffer_init(&ring);
  ldb_buffer_init(&piece);
  ldb_rand_init(&rnd, 301);
  while (ring.size < 1048576) {
    ldb_compressible_string(&piece, &rnd, 0.5, 100);
    ldb_buffer_concat(&ring, &piece);
  }

  /* 1. Cut the data blocks (ldb_tablegen_add's rule), keeping index keys. */
  t0 = now();
  ldb_blockgen_init(&data, &options);
  ldb_buffer_init(&last_key);
  ldb_ikey_init(&ikey);
  for (k = 0; k <= num; k++) {
    char kbuf[32];
    ldb_slice_t ukey, val, blk;

    if (k < num) {
      sprintf(kbuf, "%016d", (int)k);
      ukey = ldb_slice((uint8_t *)kbuf, 16);
      ldb_ikey_set(&ikey, &ukey, (ldb_seqnum_t)(k + 1), LDB_TYPE_VALUE);
    }
    if (pending) {
      /* the previous block's index key (table_builder.c:213-223, 332-340) */
      if (k < num)
        ldb_shortest_separator(&icmp, &last_key, &ikey);
      else
        ldb_short_successor(&icmp, &last_key);
      if (keys_at + last_key.size + 16 > keys_cap) {
        keys_cap = keys_cap ? 2 * keys_cap : (1 << 20);
        keys = xrealloc(keys, keys_cap);
      }
      keys_off[nb - 1] = keys_at;
      memcpy(keys + keys_at, last_key.data, last_key.size);
      keys_at += last_key.size;
      pending = 0;
    }
    if (k == num)
      break;
    ldb_buffer_copy(&last_key, &ikey);
    if (pos + 100 > ring.size)
      pos = 0;
    val = ldb_slice(ring.data + pos, 100);
    pos += 100;
    ldb_blockgen_add(&data, &ikey, &val);
    if (ldb_blockgen_size_estimate(&data) >= options.block_size || k == num - 1) {
      blk = ldb_blockgen_finish(&data);
      if (nb == nb_cap) {
        nb_cap = nb_cap ? 2 * nb_cap : 65536;
        raw_off = xrealloc(raw_off, (nb_cap + 1) * sizeof(*raw_off));
        raw_len = xrealloc(raw_len, nb_cap * sizeof(*raw_len));
        keys_off = xrealloc(keys_off, (nb_cap + 1) * sizeof(*keys_off));
      }
      if (raw_at + blk.size > raw_cap) {
        raw_cap = raw_cap ? 2 * raw_cap : (64u << 20);
        while (raw_at + blk.size > raw_cap)
          raw_cap *= 2;
        raw = xrealloc(raw, raw_cap);
      }
      raw_off[nb] = raw_at;
      raw_len[nb] = (uint32_t)blk.size;
      memcpy(raw + raw_at, blk.data, blk.size);
      raw_at += blk.size;
      nb++;
      ldb_blockgen_reset(&data);
      pending = 1;
    }
  }
  if (nb == 0)
    return 4;
  keys_off[nb] = keys_at;
  t1 = now();
  /* HIP runtime and device start-up, timed apart from the codec. */
  if (lgs_device_count() <= 0) {
    fprintf(stderr, "no device\n");
    return 5;
  }
  ti = now();

  /* 2. Every data block in one call: compress, 12.5 % rule, trailers, packing. */
  hoff = xrealloc(NULL, nb * sizeof(*hoff));
  hsize = xrealloc(NULL, nb * sizeof(*hsize));
  file_cap = raw_at + (size_t)nb * LDB_TRAILER_SIZE + (64u << 20);
  file = xrealloc(NULL, file_cap);
  rc = lgs_table_write_host(raw, raw_off, raw_len, nb, LGS_SNAPPY_COMPRESSION, 0, file, file_cap,
                            hoff, hsize, &end);
  if (rc != LGS_OK) {
    fprintf(stderr, "lgs_table_write_host: %d (%s)\n", rc, lgs_last_error());
    return 5;
  }
  t2 = now();
  /* The same call again: the first one also grew the library's pinned
     staging arena to this table's size; the second is the steady state a
     bulk writer sees from its second table on. */
  rc = lgs_table_write_host(raw, raw_off, raw_len, nb, LGS_SNAPPY_COMPRESSION, 0, file, file_cap,
                            hoff, hsize, &end_warm);
  if (rc != LGS_OK || end_warm != end) {
    fprintf(stderr, "lgs_table_write_host (warm): %d (%s)\n", rc, lgs_last_error());
    return 5;
  }
  t2w = now();

  /* 3. Metaindex, index, footer (table_builder.c:266-363; no filter policy). */
  at = end;
  ldb_blockgen_init(&meta, &options);
  put_block(&file, &file_cap, &at, ldb_blockgen_finish(&meta), &meta_handle);
  ldb_blockgen_clear(&meta);
  ldb_blockgen_init(&index, &index_options);
  for (i = 0; i < nb; i++) {
    uint8_t tmp[LDB_HANDLE_SIZE];
    ldb_buffer_t enc;
    ldb_handle_t h;
    ldb_slice_t key = ldb_slice((uint8_t *)keys + keys_off[i], keys_off[i + 1] - keys_off[i]);
    h.offset = hoff[i];
    h.size = hsize[i];
    ldb_buffer_rwset(&enc, tmp, sizeof(tmp));
    ldb_handle_export(&enc, &h);
    ldb_blockgen_add(&index, &key, &enc);
  }
  put_block(&file, &file_cap, &at, ldb_blockgen_finish(&index), &index_handle);
  ldb_blockgen_clear(&index);
  footer.metaindex_handle = meta_handle;
  footer.index_handle = index_handle;
  ldb_buffer_rwset(&footer_enc, footer_buf, sizeof(footer_buf));
  ldb_footer_export(&footer_enc, &footer);
  if (at + footer_enc.size > file_cap) {
    file_cap = at + footer_enc.size;
    file = xrealloc(file, file_cap);
  }
  memcpy(file + at, footer_enc.data, footer_enc.size);
  at += footer_enc.size;
  t3 = now();

  /* 4. The file (builder.c:85-89: sync, close). */
  sprintf(path, "%s/000001.ldb", dir);
  f = fopen(path, "wb");
  if (f == NULL || fwrite(file, 1, at, f) != at || fflush(f) != 0 || fsync(fileno(f)) != 0)
    return 6;
  fclose(f);
  t4 = now();

  /* 5. Every data block back in one call, checked against what was written. */
  back = xrealloc(NULL, raw_at + 16);
  back_len = xrealloc(NULL, nb * sizeof(*back_len));
  status = xrealloc(NULL, nb);
  {
    uint32_t *cap = xrealloc(NULL, nb * sizeof(*cap));
    for (i = 0; i < nb; i++)
      cap[i] = raw_len[i];
    rc = lgs_table_read_host(file, at, hoff, hsize, nb, 1, back, raw_off, cap, back_len, status);
    free(cap);
  }
  if (rc != LGS_OK) {
    fprintf(stderr, "lgs_table_read_host: %d (%s)\n", rc, lgs_last_error());
    return 7;
  }
  t5 = now();
  for (i = 0; i < nb; i++) {
    if (status[i] != LGS_ST_OK || back_len[i] != raw_len[i] ||
        memcmp(back + raw_off[i], raw + raw_off[i], raw_len[i]) != 0)
      bad++;
  }

  printf("rc=%d file_size=%lu blocks=%u raw_bytes=%lu cut_s=%.3f init_s=%.3f write_s=%.3f "
         "write_warm_s=%.3f finish_s=%.3f io_s=%.3f read_s=%.3f read_bad=%u\n",
         bad ? 1 : 0, (unsigned long)at, nb, (unsigned long)raw_at, t1 - t0, ti - t1, t2 - ti,
         t2w - t2, t3 - t2w, t4 - t3, t5 - t4, bad);

  ldb_blockgen_clear(&data);
  ldb_buffer_clear(&last_key);
  ldb_ikey_clear(&ikey);
  ldb_buffer_clear(&piece);
  ldb_buffer_clear(&ring);
  free(raw);
  free(raw_off);
  free(raw_len);
  free(keys);
  free(keys_off);
  free(hoff);
  free(hsize);
  free(file);
  free(back);
  free(back_len);
  free(status);
  return bad ? 1 : 0;
}
