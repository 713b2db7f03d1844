/*
 * build_table.c -- BASELINE config 5 harness (test infrastructure).
 *
 * Builds one SSTable with lcdb's own table path, unchanged:
 *   memtable (src/memtable.c) of db_bench fillseq entries
 *     -> ldb_build_table (src/builder.c:35-121)
 *        -> ldb_tablegen_* (src/table/table_builder.c) -> snappy_encode
 *        -> re-open + iterate through the table cache (builder.c:99,
 *           table_cache.c:151) -> ldb_read_block -> snappy_decode
 * Linked twice by oracle/lcdb.mk: with lcdb's src/util/snappy.c (CPU
 * reference) and with liblcdb_gpu_snappy.so (the drop-in).  The two .ldb
 * files must be byte-identical (tests/test_lcdb_integration.py).
 *
 * Entries follow bench/db_bench.c fillseq: keys "%016d" (db_bench.c:253-257),
 * sequence k + 1, 100-byte values from the db_bench value generator
 * (seed 301, ratio 0.5; db_bench.c:206-246 via src/util/testutil.c).
 *
 * With BLOOM_BITS > 0 the table also gets lcdb's filter block: the DB's
 * internal filter policy (dbformat.c:308-345) over ldb_bloom_init(BLOOM_BITS),
 * as db_impl.c:455-460 sets it up.
 *
 * usage: build_table DIR NUM_ENTRIES [BLOCK_SIZE [BLOOM_BITS]]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "builder.h"
#include "dbformat.h"
#include "memtable.h"
#include "table_cache.h"
#include "version_edit.h"
#include "table/iterator.h"
#include "util/bloom.h"
#include "util/buffer.h"
#include "util/comparator.h"
#include "util/env.h"
#include "util/options.h"
#include "util/random.h"
#include "util/slice.h"
#include "util/status.h"
#include "util/testutil.h"

int
main(int argc, char **argv) {
  const char *dir;
  long num, k;
  ldb_comparator_t icmp;
  ldb_dbopt_t options;
  ldb_memtable_t *mem;
  ldb_tables_t *tables;
  ldb_filemeta_t meta;
  ldb_iter_t *iter;
  ldb_buffer_t ring, piece;
  ldb_rand_t rnd;
  ldb_bloom_t user_bloom, ifp;
  size_t pos = 0;
  int rc;
  struct timespec ts0, ts1, ts2;

  if (argc < 3) {
    fprintf(stderr, "usage: %s DIR NUM_ENTRIES [BLOCK_SIZE [BLOOM_BITS]]\n", argv[0]);
    return 2;
  }

  dir = argv[1];
  num = atol(argv[2]);

  ldb_ikc_init(&icmp, ldb_bytewise_comparator);
  options = *ldb_dbopt_default;
  options.comparator = &icmp;
  if (argc > 3)
    options.block_size = (size_t)atol(argv[3]);
  if (argc > 4 && atoi(argv[4]) > 0) {
    ldb_bloom_init(&user_bloom, atoi(argv[4]));
    ldb_ifp_init(&ifp, &user_bloom);
    options.filter_policy = &ifp;
  }

  ldb_create_dir(dir);

  /* db_bench value ring: compressible 100-byte pieces, >= 1 MiB. */
  ldb_buffer_init(&ring);
  ldb_buffer_init(&piece);
  ldb_rand_init(&rnd, 301);
  while (ring.size < 1048576) {
    ldb_compressible_string(&piece, &rnd, 0.5, 100);
    ldb_buffer_concat(&ring, &piece);
  }

  clock_gettime(CLOCK_MONOTONIC, &ts0);
  mem = ldb_memtable_create(&icmp);
  ldb_memtable_ref(mem);

  for (k = 0; k < num; k++) {
    char kbuf[32];
    ldb_slice_t key, val;

    sprintf(kbuf, "%016d", (int)k);
    key = ldb_slice((uint8_t *)kbuf, 16);

    if (pos + 100 > ring.size)
      pos = 0;
    val = ldb_slice(ring.data + pos, 100);
    pos += 100;

    ldb_memtable_add(mem, (ldb_seqnum_t)(k + 1), LDB_TYPE_VALUE, &key, &val);
  }

  tables = ldb_tables_create(dir, &options, 100);

  ldb_filemeta_init(&meta);
  meta.number = 1;

  clock_gettime(CLOCK_MONOTONIC, &ts1);
  iter = ldb_memiter_create(mem);
  rc = ldb_build_table(dir, &options, tables, iter, &meta);
  ldb_iter_destroy(iter);
  clock_gettime(CLOCK_MONOTONIC, &ts2);

  /* fill_s: memtable inserts; build_s: ldb_build_table (write, sync, reopen) */
  printf("rc=%d (%s) file_size=%lu fill_s=%.3f build_s=%.3f\n", rc, ldb_strerror(rc),
         (unsigned long)meta.file_size,
         (ts1.tv_sec - ts0.tv_sec) + (ts1.tv_nsec - ts0.tv_nsec) * 1e-9,
         (ts2.tv_sec - ts1.tv_sec) + (ts2.tv_nsec - ts1.tv_nsec) * 1e-9);

  ldb_tables_destroy(tables);
  ldb_memtable_unref(mem);
  ldb_buffer_clear(&piece);
  ldb_buffer_clear(&ring);

  return rc == LDB_OK ? 0 : 1;
}
