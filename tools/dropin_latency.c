/* Per-call latency of the drop-in from C, the way lcdb calls it
 * (table_builder.c:182-188: ldb_snappy_encode_size + ldb_snappy_encode;
 * format.c:237-251: ldb_snappy_decode_size + ldb_snappy_decode) on 4 KiB
 * db_bench fillseq blocks -- no Python or ctypes in the timed region
 * (tools/bench_dropin_latency.py measures the same through ctypes).
 *
 * build: gcc -O2 -std=gnu99 tools/dropin_latency.c -Iinclude -Llcdb_amd \
 *          -llcdb_gpu_snappy -lcorpus -Wl,-rpath,$PWD/lcdb_amd -o tools/dropin_latency
 * usage: tools/dropin_latency [REPS]      prints one JSON line (microseconds) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lcdb_gpu_snappy.h"

uint64_t corpus_fillseq(uint8_t *dst, uint64_t cap, uint64_t *off, uint32_t *len, uint32_t n,
                        uint32_t block_size, uint32_t align, uint32_t key0, uint32_t ring0);

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

static void pct(const char *name, double *t, int n, int last) {
  qsort(t, n, sizeof *t, cmp);
  printf("\"%s\": {\"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f, \"calls\": %d}%s", name,
         t[n / 2], t[n * 9 / 10], t[n * 99 / 100], n, last ? "" : ", ");
}

int main(int argc, char **argv) {
  enum { NB = 256 };
  const int reps = argc > 1 ? atoi(argv[1]) : 4000;
  static uint8_t raw[NB * 4200 + 64];
  static uint64_t off[NB];
  static uint32_t len[NB];
  static uint8_t enc[NB][8192], out[8192];
  static size_t elen[NB];
  double *te = malloc(sizeof(double) * reps), *td = malloc(sizeof(double) * reps);
  size_t zn, i;
  int k;
  if (!corpus_fillseq(raw, sizeof raw, off, len, NB, 4096, 16, 0, 0)) return 1;
  for (i = 0; i < NB; i++) elen[i] = ldb_snappy_encode(enc[i], raw + off[i], len[i]);
  for (k = 0; k < 100; k++) {                                   /* warm-up */
    ldb_snappy_encode(out, raw + off[0], len[0]);
    if (!ldb_snappy_decode(out, enc[0], elen[0])) return 2;
  }
  for (k = 0; k < reps; k++) {
    const int b = k % NB;
    double t0 = now_us(), t1, t2;
    if (!ldb_snappy_encode_size(&zn, len[b])) return 3;
    if (ldb_snappy_encode(enc[b], raw + off[b], len[b]) != elen[b]) return 4;
    t1 = now_us();
    if (!ldb_snappy_decode_size(&zn, enc[b], elen[b]) || zn != len[b]) return 5;
    if (!ldb_snappy_decode(out, enc[b], elen[b])) return 6;
    t2 = now_us();
    if (memcmp(out, raw + off[b], len[b])) return 7;
    te[k] = t1 - t0;
    td[k] = t2 - t1;
  }
  printf("{\"caller\": \"C, lcdb's call sequence\", ");
  pct("encode_4KiB_us", te, reps, 0);
  pct("decode_4KiB_us", td, reps, 1);
  printf("}\n");
  return 0;
}
