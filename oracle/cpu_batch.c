/*
 * cpu_batch.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Drives a per-block CPU codec (the oracle restatement, or the reference
 * snappy.c compiled into oracle/_ref/) over a batch of blocks with a static
 * round-robin (or contiguous) block partition across T pthreads.  Used by tests/ to check
 * whole corpora and by bench.py's cpu_baseline leg (BASELINE.md "CPU-baseline
 * plan": 1 thread and N threads, round-robin).  The codec is passed in as
 * function pointers with the signatures of lcdb's src/util/snappy.h:31-38.
 */

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

int cpu_batch_run2(int mode, void *fn, int threads, int partition,
                   const uint8_t *in, const uint64_t *in_off,
                   const uint32_t *in_len, uint8_t *out,
                   const uint64_t *out_off, uint32_t *out_len,
                   uint8_t *status, uint32_t n);

typedef size_t (*cb_encode_fn)(uint8_t *, const uint8_t *, size_t);
typedef int (*cb_decode_fn)(uint8_t *, const uint8_t *, size_t);

typedef struct {
  int mode;                  /* 0 = encode, 1 = decode */
  cb_encode_fn enc;
  cb_decode_fn dec;
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *out_len;         /* encode: bytes written; decode: unused */
  uint8_t *status;           /* decode: 1 ok / 0 corrupt; may be NULL */
  uint32_t n;               /* blocks [first, n) with this stride */
  uint32_t stride;
  uint32_t first;
  uint32_t reps;            /* passes over the partition (timing: amortises thread start) */
} cb_job;

static void *
cb_worker(void *arg) {
  const cb_job *j = (const cb_job *)arg;
  uint32_t i, r;

  for (r = 0; r < j->reps; r++)
  for (i = j->first; i < j->n; i += j->stride) {
    const uint8_t *src = j->in + j->in_off[i];
    uint8_t *dst = j->out + j->out_off[i];

    if (j->mode == 0) {
      j->out_len[i] = (uint32_t)j->enc(dst, src, j->in_len[i]);
    } else {
      int ok = j->dec(dst, src, j->in_len[i]);
      if (j->status)
        j->status[i] = (uint8_t)(ok != 0);
    }
  }

  return NULL;
}

/* partition 0: static round-robin (thread t takes blocks t, t + T, ...);
 * partition 1: contiguous (thread t takes blocks [t n / T, (t + 1) n / T)),
 * so each thread's output pages are its own (first-touched by it when the
 * caller passes untouched buffers).  Returns 0 on success, -1 if a thread
 * could not be started. */
int
cpu_batch_run3(int mode, void *fn, int threads, int partition, uint32_t reps,
               const uint8_t *in, const uint64_t *in_off,
               const uint32_t *in_len, uint8_t *out,
               const uint64_t *out_off, uint32_t *out_len,
               uint8_t *status, uint32_t n) {
  pthread_t *tid;
  cb_job *jobs;
  int t, rc = 0;

  if (threads < 1)
    threads = 1;

  tid = (pthread_t *)calloc((size_t)threads, sizeof(*tid));
  jobs = (cb_job *)calloc((size_t)threads, sizeof(*jobs));

  if (tid == NULL || jobs == NULL) {
    free(tid);
    free(jobs);
    return -1;
  }

  for (t = 0; t < threads; t++) {
    cb_job *j = &jobs[t];
    j->mode = mode;
    j->enc = mode == 0 ? (cb_encode_fn)fn : NULL;
    j->dec = mode == 1 ? (cb_decode_fn)fn : NULL;
    j->in = in;
    j->in_off = in_off;
    j->in_len = in_len;
    j->out = out;
    j->out_off = out_off;
    j->out_len = out_len;
    j->status = status;
    j->reps = reps < 1 ? 1 : reps;
    if (partition == 1) {
      j->first = (uint32_t)((uint64_t)n * (uint64_t)t / (uint64_t)threads);
      j->n = (uint32_t)((uint64_t)n * (uint64_t)(t + 1) / (uint64_t)threads);
      j->stride = 1;
    } else {
      j->n = n;
      j->stride = (uint32_t)threads;
      j->first = (uint32_t)t;
    }
  }

  if (threads == 1) {
    cb_worker(&jobs[0]);
  } else {
    int started = 0;
    for (t = 0; t < threads; t++) {
      if (pthread_create(&tid[t], NULL, cb_worker, &jobs[t]) != 0) {
        rc = -1;
        break;
      }
      started++;
    }
    for (t = 0; t < started; t++)
      pthread_join(tid[t], NULL);
  }

  free(tid);
  free(jobs);
  return rc;
}

int
cpu_batch_run(int mode, void *fn, int threads,
              const uint8_t *in, const uint64_t *in_off,
              const uint32_t *in_len, uint8_t *out,
              const uint64_t *out_off, uint32_t *out_len,
              uint8_t *status, uint32_t n) {
  return cpu_batch_run2(mode, fn, threads, 0, in, in_off, in_len, out, out_off,
                        out_len, status, n);
}

int
cpu_batch_run2(int mode, void *fn, int threads, int partition,
               const uint8_t *in, const uint64_t *in_off,
               const uint32_t *in_len, uint8_t *out,
               const uint64_t *out_off, uint32_t *out_len,
               uint8_t *status, uint32_t n) {
  return cpu_batch_run3(mode, fn, threads, partition, 1, in, in_off, in_len, out,
                        out_off, out_len, status, n);
}
