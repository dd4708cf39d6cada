/*
 * dropin_bench.c — INTEGRATION.md's stats worker on libhpgq, timed (a tool,
 * not product).  It reproduces the drop-in binding the way the reference
 * would run it:
 *   producer  a FASTQ file read into batches of --batch reads (default the
 *             reference's 10,000, src/stats_options.c:22) as AoS reads, one
 *             malloc'd sequence and quality per read, as fastq_fread_se fills
 *             its array_list_t (src/stats_fastq.c:183).  All batches are read
 *             before the clock starts: the reader is not what is measured.
 *   workers   --threads threads (default the reference's 2,
 *             src/stats_options.c:21), one hpgq ctx each (GPU t % ndev).  A
 *             worker takes the next batch, packs it into malloc'd SoA buffers,
 *             calls hpgq_run_host + hpgq_sync and frees the buffers --
 *             fastq_stats_worker of INTEGRATION.md (src/stats_fastq.c:202-250);
 *             the SoA buffers are the ctx's staging slot (hpgq_host_batch),
 *             or with --copy malloc'd ones that hpgq_run_host copies.
 *             --no-sync: the stats worker as the stats consumer needs it -- no
 *             mask (the engine merges the passed reads itself), so no
 *             hpgq_sync per batch: hpgq_host_batch waits for the slot's
 *             previous batch (two in flight per ctx), and each worker syncs
 *             its ctx once after its last batch (inside the clock).
 *   consumer  nothing per read; the ctxs' counters are summed at the end.
 * Prints one JSON line.  --counters F / --mask F write the summed u64 counter
 * set and the per-read masks (input order) for tests/test_dropin_gpu.py.
 *
 *   dropin_bench in.fq [--batch 10000] [--threads 2] [--lmax 1024] [--c2] [--copy]
 *                      [--no-sync] [--counters F] [--mask F] [--repeat R]
 * --c2: the C2 filter (--read-quality-range 20, --read-length-range 50,).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hpgq.h"

typedef struct {
  char *sequence, *quality;   /* fastq_read_t's two strings */
} read_t;

typedef struct {
  read_t *reads;
  size_t n;
  size_t first;   /* index of the batch's first read in the file */
} batch_t;

static batch_t *g_batches;
static size_t g_nbatches, g_total;
static size_t g_next;   /* next batch to take (atomic) */
static uint8_t *g_mask;
static hpgq_params_t g_params;
static int g_fail;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static char *dup_line(const char *s, size_t n) {
  char *p = malloc(n + 1);
  memcpy(p, s, n);
  p[n] = 0;
  return p;
}

static int load(const char *path, size_t batch) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  char *line[4] = {0};
  size_t cap[4] = {0};
  ssize_t len[4];
  size_t nb_cap = 1024;
  g_batches = calloc(nb_cap, sizeof(batch_t));
  batch_t *cur = NULL;
  for (;;) {
    int k;
    for (k = 0; k < 4; ++k) {
      len[k] = getline(&line[k], &cap[k], f);
      if (len[k] < 0) break;
      while (len[k] > 0 && (line[k][len[k] - 1] == '\n' || line[k][len[k] - 1] == '\r')) --len[k];
    }
    if (k < 4) break;
    if (!cur || cur->n == batch) {
      if (g_nbatches == nb_cap) {
        nb_cap *= 2;
        g_batches = realloc(g_batches, nb_cap * sizeof(batch_t));
      }
      cur = &g_batches[g_nbatches++];
      cur->reads = malloc(batch * sizeof(read_t));
      cur->n = 0;
      cur->first = g_total;
    }
    cur->reads[cur->n].sequence = dup_line(line[1], (size_t)len[1]);
    cur->reads[cur->n].quality = dup_line(line[3], (size_t)len[3]);
    cur->n++;
    g_total++;
  }
  for (int k = 0; k < 4; ++k) free(line[k]);
  fclose(f);
  return 0;
}

typedef struct {
  int id;
  hpgq_ctx_t *ctx;
} worker_t;

static int g_copy;     /* --copy: the malloc'd-batch worker (hpgq_run_host copies it) */
static int g_nosync;   /* --no-sync: no mask, one hpgq_sync per worker at the end */

/* INTEGRATION.md fastq_stats_worker, once per batch: the reads are packed
 * straight into the ctx's staging slot (hpgq_host_batch), or with --copy into
 * malloc'd buffers that hpgq_run_host copies into the slot */
static void *worker(void *arg) {
  worker_t *w = arg;
  for (;;) {
    const size_t bi = __atomic_fetch_add(&g_next, 1, __ATOMIC_RELAXED);
    if (bi >= g_nbatches) break;
    const batch_t *bt = &g_batches[bi];
    const size_t n = bt->n;
    int32_t *idx = malloc((n + 1) * sizeof(int32_t));   /* offsets first: one strlen per read */
    idx[0] = 0;
    for (size_t i = 0; i < n; i++) idx[i + 1] = idx[i] + (int32_t)strlen(bt->reads[i].sequence);
    hpgq_batch_t b;
    char *seq, *qual;
    int rc = HPGQ_OK;
    if (g_copy) {
      seq = malloc((size_t)idx[n] + 1);
      qual = malloc((size_t)idx[n] + 1);
      b = (hpgq_batch_t){(int64_t)n, seq, qual, idx};
    } else {
      rc = hpgq_host_batch(w->ctx, (int64_t)n, (size_t)idx[n], 0, &b, NULL);
      if (rc == HPGQ_OK) memcpy((int32_t *)b.data_indices, idx, (n + 1) * sizeof(int32_t));
      seq = (char *)b.seq;
      qual = (char *)b.quality;
    }
    if (rc == HPGQ_OK) {
      for (size_t i = 0; i < n; i++) {
        const size_t len = (size_t)(idx[i + 1] - idx[i]);
        memcpy(seq + idx[i], bt->reads[i].sequence, len);
        memcpy(qual + idx[i], bt->reads[i].quality, len);
      }
    }
    uint8_t *mask = g_nosync ? NULL : malloc(n);
    if (rc == HPGQ_OK) rc = hpgq_run_host(w->ctx, &b, NULL, mask, NULL);
    if (rc == HPGQ_OK && !g_nosync) rc = hpgq_sync(w->ctx);   /* mask valid, buffers reusable */
    if (rc != HPGQ_OK) {
      fprintf(stderr, "hpgq: %s\n", hpgq_strerror(rc));
      g_fail = 1;
    }
    if (g_mask && mask) memcpy(g_mask + bt->first, mask, n);
    free(mask);
    if (g_copy) {
      free(seq);
      free(qual);
    }
    free(idx);
  }
  if (g_nosync) {   /* the workflow's end: this worker's batches are done */
    const int rc = hpgq_sync(w->ctx);
    if (rc != HPGQ_OK) {
      fprintf(stderr, "hpgq: %s\n", hpgq_strerror(rc));
      g_fail = 1;
    }
  }
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: dropin_bench in.fq [--batch N] [--threads T] [--lmax L] [--c2] [--copy] "
                    "[--no-sync] [--counters F] [--mask F] [--repeat R]\n");
    return 2;
  }
  size_t batch = 10000;
  int threads = 2, lmax = 1024, c2 = 0, repeat = 1;
  const char *ctr_path = NULL, *mask_path = NULL;
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "--batch") && i + 1 < argc) batch = (size_t)atol(argv[++i]);
    else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--lmax") && i + 1 < argc) lmax = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--repeat") && i + 1 < argc) repeat = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--c2")) c2 = 1;
    else if (!strcmp(argv[i], "--copy")) g_copy = 1;
    else if (!strcmp(argv[i], "--no-sync")) g_nosync = 1;
    else if (!strcmp(argv[i], "--counters") && i + 1 < argc) ctr_path = argv[++i];
    else if (!strcmp(argv[i], "--mask") && i + 1 < argc) mask_path = argv[++i];
    else {
      fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  if (batch < 1 || threads < 1 || repeat < 1) return 2;
  if (g_nosync && mask_path) {
    fprintf(stderr, "--no-sync takes no mask (the stats consumer needs none)\n");
    return 2;
  }
  const double t_load = now();
  if (load(argv[1], batch)) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 1;
  }
  const double load_s = now() - t_load;
  hpgq_params_init(&g_params);
  g_params.lmax = lmax;
  g_params.stats_on = 1;
  if (c2) {   /* stats --read-quality-range 20, --read-length-range 50, */
    g_params.filter_on = 1;
    g_params.min_read_quality = 20;
    g_params.min_read_length = 50;
  }
  if (mask_path) g_mask = calloc(g_total ? g_total : 1, 1);
  const int ndev = hpgq_device_count();
  if (ndev < 1) {
    fprintf(stderr, "no HIP device\n");
    return 1;
  }
  worker_t *w = calloc((size_t)threads, sizeof(worker_t));
  for (int t = 0; t < threads; t++) {
    w[t].id = t;
    int rc = hpgq_open(&w[t].ctx, t % ndev, &g_params);
    if (rc) {
      fprintf(stderr, "hpgq_open: %s\n", hpgq_strerror(rc));
      return 1;
    }
  }
  pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
  double best = 1e30, sum = 0;
  for (int r = 0; r < repeat; r++) {
    for (int t = 0; t < threads; t++) hpgq_reset(w[t].ctx);
    g_next = 0;
    const double t0 = now();
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &w[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    const double el = now() - t0;
    sum += el;
    if (el < best) best = el;
  }
  if (g_fail) return 1;
  const size_t len = hpgq_counters_len(lmax);
  uint64_t *tot = calloc(len, sizeof(uint64_t)), *one = malloc(len * sizeof(uint64_t));
  for (int t = 0; t < threads; t++) {
    if (hpgq_read_counters(w[t].ctx, one, len)) return 1;
    for (size_t j = 0; j < len; j++) tot[j] += one[j];
    hpgq_close(w[t].ctx);
  }
  if (ctr_path) {
    FILE *f = fopen(ctr_path, "wb");
    if (!f || fwrite(tot, sizeof(uint64_t), len, f) != len) return 1;
    fclose(f);
  }
  if (mask_path) {
    FILE *f = fopen(mask_path, "wb");
    if (!f || fwrite(g_mask, 1, g_total, f) != g_total) return 1;
    fclose(f);
  }
  printf("{\"reads\": %zu, \"batches\": %zu, \"batch_reads\": %zu, \"threads\": %d, \"gpus\": %d, "
         "\"repeat\": %d, \"best_s\": %.6f, \"mean_s\": %.6f, \"mreads_s\": %.3f, \"mreads_s_mean\": %.3f, "
         "\"load_s\": %.3f, \"num_input\": %llu, \"num_passed\": %llu, \"staging\": \"%s\", "
         "\"sync\": \"%s\"}\n",
         g_total, g_nbatches, batch, threads, threads < ndev ? threads : ndev, repeat, best, sum / repeat,
         g_total / best / 1e6, g_total / (sum / repeat) / 1e6, load_s,
         (unsigned long long)tot[HPGQ_S_NUM_INPUT], (unsigned long long)tot[HPGQ_S_NUM_PASSED],
         g_copy ? "copy" : "in_place", g_nosync ? "once per worker at the end" : "per batch");
  return 0;
}
