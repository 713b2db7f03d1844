/*
 * dump_blocks.c -- TEST INFRASTRUCTURE ONLY: reads every block of an .ldb
 * with lcdb's own table code (src/table/format.c ldb_read_block, block.c
 * index iteration) and dumps what the reference returns, so the block
 * framing restatement (oracle/table_oracle.c) and the GPU batched read and
 * write paths (lgs_table_*) are checked against the reference itself.
 *
 * usage: dump_blocks FILE.ldb OUT VERIFY [HANDLES]
 *   Blocks: the data blocks named by the index block, then the metaindex
 *   and index blocks (footer, format.c:116-150).  With HANDLES (a file of
 *   u64 offset, u64 size pairs) those handles are read instead.
 *   OUT (host-endian): u64 file_size, u64 metaindex_off, u64 metaindex_size,
 *   u64 index_off, u64 index_size, u32 count, then per block
 *   u64 offset, u64 size, i32 rc (LDB_* status), u32 len, len content bytes.
 *   With DUMP_DIGEST=1 in the environment each block's content is replaced by
 *   a u64 digest of it (a word-wise multiply-xor hash; the same in the .cpu and
 *   .gpu builds), so a multi-GiB table's read-back compares as a small file.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "table/block.h"
#include "table/format.h"
#include "table/iterator.h"
#include "util/comparator.h"
#include "util/env.h"
#include "util/options.h"
#include "util/slice.h"
#include "util/status.h"

static void
put(FILE *f, const void *p, size_t n) {
  if (fwrite(p, 1, n, f) != n) {
    perror("fwrite");
    exit(2);
  }
}

static int digest_only = 0;

static uint64_t
digest(const uint8_t *p, size_t n) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)n, w;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    memcpy(&w, p + i, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdull;
    h ^= h >> 29;
  }
  for (; i < n; i++)
    h = (h ^ p[i]) * 0x100000001b3ull;
  return h ^ (h >> 32);
}

static void
dump_one(FILE *out, ldb_rfile_t *file, const ldb_readopt_t *opt, const ldb_handle_t *h) {
  ldb_contents_t c;
  int32_t rc = ldb_read_block(&c, file, opt, h);
  uint32_t len = rc == LDB_OK ? (uint32_t)c.data.size : 0;
  put(out, &h->offset, 8);
  put(out, &h->size, 8);
  put(out, &rc, 4);
  put(out, &len, 4);
  if (rc == LDB_OK) {
    if (digest_only) {
      uint64_t d = digest(c.data.data, len);
      put(out, &d, 8);
    } else {
      put(out, c.data.data, len);
    }
    if (c.heap_allocated)
      free(c.data.data);
  }
}

int
main(int argc, char **argv) {
  ldb_rfile_t *file;
  ldb_readopt_t opt;
  uint64_t size;
  uint8_t fbuf[LDB_FOOTER_SIZE];
  ldb_slice_t fs;
  ldb_footer_t footer;
  ldb_contents_t ic;
  ldb_block_t *index;
  ldb_iter_t *it;
  ldb_handle_t *hs = NULL;
  uint32_t count = 0, cap = 0, i;
  FILE *out;

  if (argc < 4) {
    fprintf(stderr, "usage: %s FILE.ldb OUT VERIFY [HANDLES]\n", argv[0]);
    return 2;
  }
  if (ldb_file_size(argv[1], &size) != LDB_OK || size < LDB_FOOTER_SIZE)
    return 3;
  if (ldb_randfile_create(argv[1], &file, 0) != LDB_OK)
    return 3;

  digest_only = getenv("DUMP_DIGEST") != NULL && atoi(getenv("DUMP_DIGEST")) != 0;
  opt = *ldb_readopt_default;
  opt.verify_checksums = atoi(argv[3]);

  if (ldb_rfile_pread(file, &fs, fbuf, LDB_FOOTER_SIZE, size - LDB_FOOTER_SIZE) != LDB_OK)
    return 4;
  if (!ldb_footer_import(&footer, &fs))
    return 4;

  if (argc > 4) {
    FILE *hf = fopen(argv[4], "rb");
    uint64_t pair[2];
    if (hf == NULL)
      return 5;
    while (fread(pair, 8, 2, hf) == 2) {
      if (count == cap) {
        cap = cap ? 2 * cap : 1024;
        hs = realloc(hs, cap * sizeof(*hs));
      }
      hs[count].offset = pair[0];
      hs[count].size = pair[1];
      count++;
    }
    fclose(hf);
  } else {
    /* The index block (read with checksums, as table.c:95-110 opens it). */
    ldb_readopt_t iopt = opt;
    iopt.verify_checksums = 1;
    if (ldb_read_block(&ic, file, &iopt, &footer.index_handle) != LDB_OK)
      return 6;
    index = ldb_block_create(&ic);
    it = ldb_blockiter_create(index, ldb_bytewise_comparator);
    for (ldb_iter_first(it); ldb_iter_valid(it); ldb_iter_next(it)) {
      ldb_slice_t v = ldb_iter_value(it);
      if (count == cap) {
        cap = cap ? 2 * cap : 1024;
        hs = realloc(hs, cap * sizeof(*hs));
      }
      if (!ldb_handle_import(&hs[count], &v))
        return 7;
      count++;
    }
    ldb_iter_destroy(it);
    ldb_block_destroy(index);
    hs = realloc(hs, (count + 2) * sizeof(*hs));
    hs[count++] = footer.metaindex_handle;
    hs[count++] = footer.index_handle;
  }

  out = fopen(argv[2], "wb");
  if (out == NULL)
    return 8;
  put(out, &size, 8);
  put(out, &footer.metaindex_handle.offset, 8);
  put(out, &footer.metaindex_handle.size, 8);
  put(out, &footer.index_handle.offset, 8);
  put(out, &footer.index_handle.size, 8);
  put(out, &count, 4);
  for (i = 0; i < count; i++)
    dump_one(out, file, &opt, &hs[i]);
  fclose(out);
  free(hs);
  ldb_rfile_destroy(file);
  return 0;
}
