/*
 * refarch.c — TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline
 * "refarch" figure and tests/test_refarch_cpu.py).  Never linked by the
 * product (libhpgq, the CLI).
 *
 * The reference's own CPU architecture for `stats` (+ filter), restated so
 * that it can be timed beside the GPU and beside the OpenMP dense-array port
 * (hpgq_oracle.c): per 10,000-read batch (src/stats_options.c:22,
 * batch_size) a worker thread computes each read's stats record and the
 * pass / fail decision (the stage() of src/stats_fastq.c:202-250; 2 workers,
 * src/stats_options.c:21, num_threads), and ONE consumer thread merges the
 * records in input order into hash maps, one kh_put per base and map
 * (fastq_stats_consumer, src/stats_fastq.c:257-417: kh_length_histogram,
 * kh_quality_histogram, kh_gc_histogram, kh_count_quality_per_nt,
 * kh_acc_quality_per_nt and kh_num_{A,T,C,G,N}s_per_nt).  The maps are an
 * open-addressing int -> int64 table of this file's own (khash, the
 * reference's, lives in the absent common-libs); the per-read rules are the
 * oracle's, so the dense counters it ends with equal
 * hpgq_oracle.c's on the exact-integer fields (hist_len, hist_gc, pos_qsum,
 * pos_base, the scalars), which tests/test_refarch_cpu.py checks.
 * Supports the options of configs C1 / C2: length and mean-quality filter.
 */
#include <pthread.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hpgq.h"

/* ---- int -> int64 map, open addressing (kh_put + value update) ---------- */
typedef struct {
  int32_t *key;
  int64_t *val;
  uint8_t *used;
  uint32_t cap, n;   /* cap a power of two */
} imap_t;

static int imap_init(imap_t *m, uint32_t cap) {
  m->cap = cap;
  m->n = 0;
  m->key = calloc(cap, sizeof(int32_t));
  m->val = calloc(cap, sizeof(int64_t));
  m->used = calloc(cap, 1);
  return m->key && m->val && m->used ? 0 : -1;
}

static void imap_free(imap_t *m) {
  free(m->key);
  free(m->val);
  free(m->used);
}

static int imap_grow(imap_t *m);

/* the slot of `k`, inserted with value 0 when absent (kh_put) */
static int64_t *imap_put(imap_t *m, int32_t k) {
  if (2 * (m->n + 1) > m->cap && imap_grow(m)) return NULL;
  uint32_t h = ((uint32_t)k * 2654435761u) & (m->cap - 1);
  while (m->used[h] && m->key[h] != k) h = (h + 1) & (m->cap - 1);
  if (!m->used[h]) {
    m->used[h] = 1;
    m->key[h] = k;
    m->val[h] = 0;
    m->n++;
  }
  return &m->val[h];
}

static int imap_grow(imap_t *m) {
  imap_t g;
  if (imap_init(&g, m->cap * 2)) return -1;
  for (uint32_t i = 0; i < m->cap; ++i)
    if (m->used[i]) *imap_put(&g, m->key[i]) = m->val[i];
  imap_free(m);
  *m = g;
  return 0;
}

/* ---- worker: per-read stats records (the stage() of the workflow) ------- */
typedef struct {
  int32_t length, sumq;   /* raw signed-char quality sum */
  int32_t num_A, num_C, num_G, num_T, num_N;
  uint8_t pass;
} read_stats_t;

typedef struct {
  const hpgq_params_t *p;
  const hpgq_batch_t *b;
  int batch_reads, nbatches;
  read_stats_t *recs;   /* one per read */
  int *done;            /* per batch */
  int next;             /* next batch to take */
  pthread_mutex_t mu;
  pthread_cond_t cv;
} ra_t;

static void stage(ra_t *R, int k) {
  const hpgq_params_t *p = R->p;
  const int64_t r0 = (int64_t)k * R->batch_reads;
  int64_t r1 = r0 + R->batch_reads;
  if (r1 > R->b->num_reads) r1 = R->b->num_reads;
  for (int64_t r = r0; r < r1; ++r) {
    const int32_t a = R->b->data_indices[r], n = R->b->data_indices[r + 1] - a;
    read_stats_t *s = &R->recs[r];
    memset(s, 0, sizeof(*s));
    s->length = n;
    for (int32_t j = 0; j < n; ++j) {
      s->sumq += (signed char)R->b->quality[a + j];
      switch (R->b->seq[a + j]) {
        case 'A': s->num_A++; break;
        case 'C': s->num_C++; break;
        case 'G': s->num_G++; break;
        case 'T': s->num_T++; break;
        case 'N': s->num_N++; break;
        default: break;
      }
    }
    /* the filter's length and mean-quality rules, exact */
    const int64_t q = (int64_t)s->sumq - (int64_t)p->phred * n;
    s->pass = !p->filter_on || (n >= p->min_read_length && n <= p->max_read_length &&
                                (int64_t)p->min_read_quality * n <= q && q <= (int64_t)p->max_read_quality * n);
  }
}

static void *worker(void *arg) {
  ra_t *R = arg;
  for (;;) {
    pthread_mutex_lock(&R->mu);
    const int k = R->next++;
    pthread_mutex_unlock(&R->mu);
    if (k >= R->nbatches) break;
    stage(R, k);
    pthread_mutex_lock(&R->mu);
    R->done[k] = 1;
    pthread_cond_broadcast(&R->cv);
    pthread_mutex_unlock(&R->mu);
  }
  return NULL;
}

/*
 * stats (+ filter) over one batch of reads the reference's way: `workers`
 * threads produce per-read records per `batch_reads` reads, the calling thread
 * merges them in order through the hash maps.  ctr (hpgq_counters_len(lmax)
 * u64, zeroed here) receives the maps as dense counters.  0, or -1 (out of
 * memory / unsupported options).
 */
int refarch_stats(const hpgq_params_t *p, const hpgq_batch_t *b, int batch_reads, int workers,
                  uint64_t *ctr) {
  if (p->edit_on || p->paired || batch_reads < 1 || workers < 1) return -1;
  if (p->filter_on && (p->max_N < HPGQ_MAX_VALUE || p->max_out_of_quality < HPGQ_MAX_VALUE || p->left_length > 0 ||
                       p->right_length > 0))
    return -1;
  ra_t R;
  memset(&R, 0, sizeof(R));
  R.p = p;
  R.b = b;
  R.batch_reads = batch_reads;
  R.nbatches = (int)((b->num_reads + batch_reads - 1) / batch_reads);
  R.recs = malloc((size_t)(b->num_reads > 0 ? b->num_reads : 1) * sizeof(read_stats_t));
  R.done = calloc((size_t)R.nbatches + 1, sizeof(int));
  enum { H_LEN, H_QUAL, H_GC, H_CNTQ, H_ACCQ, H_A, H_T, H_C, H_G, H_N, NMAPS };
  imap_t h[NMAPS];
  int rc = R.recs && R.done ? 0 : -1;
  for (int i = 0; i < NMAPS; ++i)
    if (imap_init(&h[i], 64)) rc = -1;
  if (rc) goto out;
  pthread_mutex_init(&R.mu, NULL);
  pthread_cond_init(&R.cv, NULL);
  pthread_t th[64];
  if (workers > 64) workers = 64;
  int started = 0;
  for (int t = 0; t < workers; ++t)
    if (pthread_create(&th[t], NULL, worker, &R) == 0) started++;
  if (!started) worker(&R);   /* (no thread could start: this one works) */
  uint64_t n_in = 0, n_pass = 0, n_fail = 0, n_stats = 0;
  /* the consumer: batches in input order, every passed read base by base */
  for (int k = 0; k < R.nbatches && rc == 0; ++k) {
    pthread_mutex_lock(&R.mu);
    while (!R.done[k]) pthread_cond_wait(&R.cv, &R.mu);
    pthread_mutex_unlock(&R.mu);
    const int64_t r0 = (int64_t)k * batch_reads;
    const int64_t r1 = r0 + batch_reads < b->num_reads ? r0 + batch_reads : b->num_reads;
    for (int64_t r = r0; r < r1 && rc == 0; ++r) {
      const read_stats_t *s = &R.recs[r];
      n_in++;
      if (!s->pass) {
        n_fail++;
        continue;
      }
      n_pass++;
      if (!p->stats_on) continue;
      n_stats++;
      const int32_t n = s->length, a = b->data_indices[r];
      int64_t *v = imap_put(&h[H_LEN], n);
      if (!v) { rc = -1; break; }
      ++*v;
      if (n == 0) continue;   /* (no mean or GC bin for an empty read, quirk Q8) */
      v = imap_put(&h[H_QUAL], (int32_t)lround((double)s->sumq / n) & 255);
      if (!v) { rc = -1; break; }
      ++*v;
      v = imap_put(&h[H_GC], 100 * (s->num_G + s->num_C) / n);
      if (!v) { rc = -1; break; }
      ++*v;
      for (int32_t j = 0; j < n; ++j) {
        if (!(v = imap_put(&h[H_CNTQ], j))) { rc = -1; break; }
        ++*v;
        if (!(v = imap_put(&h[H_ACCQ], j))) { rc = -1; break; }
        *v += (signed char)b->quality[a + j];
        int m = -1;
        switch (b->seq[a + j]) {
          case 'A': m = H_A; break;
          case 'T': m = H_T; break;
          case 'C': m = H_C; break;
          case 'G': m = H_G; break;
          case 'N': m = H_N; break;
          default: break;
        }
        if (m >= 0) {
          if (!(v = imap_put(&h[m], j))) { rc = -1; break; }
          ++*v;
        }
      }
    }
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&R.mu);
  pthread_cond_destroy(&R.cv);
  if (rc == 0) {   /* the maps as the dense counter set */
    const int lmax = p->lmax;
    memset(ctr, 0, hpgq_counters_len(lmax) * sizeof(uint64_t));
    ctr[HPGQ_S_NUM_INPUT] = n_in;
    ctr[HPGQ_S_NUM_PASSED] = n_pass;
    ctr[HPGQ_S_NUM_FAILED] = n_fail;
    ctr[HPGQ_S_NUM_STATS] = n_stats;
    static const int base_map[5] = {H_A, H_C, H_G, H_T, H_N};
    for (int i = 0; i < NMAPS; ++i)
      for (uint32_t s = 0; s < h[i].cap; ++s) {
        if (!h[i].used[s]) continue;
        const int32_t key = h[i].key[s];
        const uint64_t val = (uint64_t)h[i].val[s];
        if (i == H_LEN) {
          if (key <= lmax) ctr[hpgq_off_hist_len(lmax) + key] += val;
          else ctr[HPGQ_S_LONG_READS] += val;
        } else if (i == H_QUAL) {
          ctr[hpgq_off_hist_meanq(lmax) + key] += val;
        } else if (i == H_GC) {
          ctr[hpgq_off_hist_gc(lmax) + key] += val;
        } else if (i == H_ACCQ) {
          if (key < lmax) ctr[hpgq_off_pos_qsum(lmax) + key] += val;
        } else if (i != H_CNTQ) {
          for (int bb = 0; bb < 5; ++bb)
            if (base_map[bb] == i && key < lmax) ctr[hpgq_off_pos_base(lmax, bb) + key] += val;
        }
      }
  }
out:
  for (int i = 0; i < NMAPS; ++i) imap_free(&h[i]);
  free(R.recs);
  free(R.done);
  return rc;
}
