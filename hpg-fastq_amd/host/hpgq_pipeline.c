/*
 * hpgq_pipeline.c — producer -> GPU worker -> consumer for hpg-fastq on libhpgq.
 *
 * The reference runs producer (fastq_fread_se into 10,000-read batches),
 * worker threads (bioinfo-libs filter / stats / edit) and an ordered consumer
 * (merge or write), src/stats_fastq.c:174-250, src/filter_fastq.c:106-174,
 * src/edit_fastq.c:113-206.  Here:
 *   reader     fills page-locked chunks of FASTQ text (--chunk-mb), with
 *              --num-threads parallel pread()s, cut at the last whole record
 *              (hpgq_fastq_complete_prefix); the partial record is carried
 *              into the next chunk.
 *   GPU        --gpu-workers threads per GPU (default 2: one copies a chunk
 *              in while the other's kernels run) on --gpus devices (default
 *              every visible one), chunk k on worker k mod G: hpgq_parse_host (H2D +
 *              parse into a device batch) and hpgq_run_device (filter / edit /
 *              stats fused) on the worker's ctx stream; for filter / edit the
 *              mask, trims and record offsets come back.  At the end the
 *              workers' device counters (k-mer tables, CGR tables) are summed
 *              on the host: the read-sharded merge of DESIGN.md §6.
 *   --cg       one chaos_game_fill_tables call per batch of --cg-batch-size
 *              bytes of FASTQ text (default 64,000,000, the old tool's
 *              batch_size, old/main_hpg_fastq_old.c:116): batch j holds the
 *              records ending in ((j-1)B, jB], so the calls (whose double
 *              state starts afresh, old/chaos_game.c:180-181) do not depend on
 *              --chunk-mb or --gpus; the reader then cuts every chunk at a
 *              batch end.
 *   outputs    (filter / edit) passed.fq / failed.fq / edit.fq in input
 *              order: filter copies whole input records; edit writes the
 *              header and '+' lines as read and the trimmed sequence /
 *              quality.  Regular output files are mapped shared, sized to the
 *              bound (each output is at most the input), and every chunk is
 *              placed in input order from its per-class byte counts and then
 *              copied into the maps by its worker's copy threads in parallel
 *              (one writer thread through write() capped filter at 18 and edit
 *              at 15-17 Mreads/s: a tmpfs or page-cache file takes one write()
 *              at a time, page stores from many threads at once); the files
 *              are truncated to their final sizes at the end.  Otherwise
 *              (--stream-writer, or a map that fails) one writer thread
 *              writes the chunks in order.
 * Stats never leave the device until the end (hpgq_read_counters).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include "hpgq_cli.h"
#include "hpgq_mapout.h"

#define MAX_WORKERS 16
#define MAX_SLOTS (2 * MAX_WORKERS + 2)
#define MAX_CARRY (64u << 20)   /* longest record the reader can carry over */
#define TRACE_MAX 1024

typedef struct {
  char *buf;          /* page-locked */
  size_t cap, len, use;
  int eof;
  int state;          /* 0 free, 1 filled (reader -> GPU), 2 processed (GPU -> writer) */
  int64_t chunk;      /* the chunk it holds */
  /* GPU results for the writer */
  int64_t nreads;
  uint8_t *mask;
  uint32_t *trim, *rec_start, *seq_start, *plus_start, *qual_start;
  int32_t *idx;
  size_t res_cap;
  /* edit: the chunk's output records per class (0 edit.fq / passed, 1 failed),
   * assembled by the GPU worker so the writer only writes them in order */
  char *out[2];
  size_t out_cap[2], out_len[2];
  uint64_t out_n[2];
  /* mapped outputs: this chunk's copy parts (copy_part_t[MAX_COPIERS]) and
   * how many are still being copied (state 3 until the last one is done) */
  void *parts;
  int parts_left;
} slot_t;

typedef struct {
  const cli_options_t *o;
  int fd;
  off_t size, pos;
  int nslots, nworkers;
  slot_t slot[MAX_SLOTS];
  char *carry;
  size_t carry_len;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  int reader_done, error;
  int64_t chunks;
  FILE *out_pass, *out_fail;
  uint64_t written_pass, written_fail;
  /* mapped outputs: [0] passed / edit.fq, [1] failed.fq (NULL: not written) */
  int mmap_out;
  mapout_t mo;           /* the mappings: reservation, prefault threads, SIGBUS guard */
  char *map[2];          /* (= mo.map) */
  size_t map_cap;
  uint64_t out_off[2];   /* bytes placed so far per output */
  int64_t placed;        /* chunks placed (in input order) */
  /* the copy pool: placed chunks' parts, copied into the maps by --num-threads
   * copier threads while the GPU workers go on with the next chunks */
  void **cq;             /* ring of copy_part_t * */
  int cq_cap, cq_head, cq_tail, cq_exit, ncopiers;
  pthread_mutex_t cq_mu;
  pthread_cond_t cq_cv;
  int copies_pending;    /* slots in state 3 (under mu) */
  pthread_t copier[64];
  int64_t cg_batch;   /* --cg: bytes of FASTQ text per chaos-game call (0: off) */
  /* HPGQ_TRACE=1: per chunk (the first TRACE_MAX) the reader's and the worker's
   * start / end times, printed to stderr at the end (diagnostics only) */
  int trace;
  double t0;
  /* read start, read end, worker start, sync start, worker end, parsed,
   * synced, placed */
  double tr[TRACE_MAX][8];
  int tw[TRACE_MAX];
} pipe_t;

static double now_s(void);
static void trace_at(pipe_t *P, int64_t k, int i, int w) {
  if (!P->trace || k >= TRACE_MAX) return;
  P->tr[k][i] = now_s() - P->t0;
  if (w >= 0) P->tw[k] = w;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* ---- NUMA placement --------------------------------------------------------- */

/* Run this process's threads (reader, GPU workers, writer -- created after
 * this call, so they inherit it) on the CPUs of the GPUs' NUMA node, within
 * the CPUs it may use, and so allocate the page-locked chunks there (first
 * touch): the reader's copies and the chunks' H2D stay on the GPU's side of
 * the socket link.  Skipped when the GPUs sit on different nodes, the node is
 * unknown, or it holds none of the allowed CPUs. */
static void bind_numa(const cli_options_t *o, int ngpus, int ndev) {
  int node = -2;
  for (int g = 0; g < ngpus && g < ndev; ++g) {
    const int nd = hpgq_device_numa_node((o->device + g) % ndev);
    if (nd < 0 || (node != -2 && nd != node)) return;
    node = nd;
  }
  if (node < 0) return;
  char path[96], list[4096];
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = fopen(path, "r");
  if (!f) return;
  const int ok = fgets(list, sizeof(list), f) != NULL;
  fclose(f);
  if (!ok) return;
  cpu_set_t allowed, want;
  if (sched_getaffinity(0, sizeof(allowed), &allowed)) return;
  CPU_ZERO(&want);
  for (char *p = list; *p && *p != '\n';) {   /* "a-b,c,d-e" */
    char *e;
    long a = strtol(p, &e, 10), b = a;
    if (e == p) break;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET((int)c, &allowed)) CPU_SET((int)c, &want);
    p = *e == ',' ? e + 1 : e;
  }
  if (CPU_COUNT(&want) == 0) return;
  if (sched_setaffinity(0, sizeof(want), &want) == 0 && getenv("HPGQ_TRACE"))
    fprintf(stderr, "hpg-fastq: threads on NUMA node %d (%d CPUs)\n", node, CPU_COUNT(&want));
}

/* ---- reader ------------------------------------------------------------- */

typedef struct {
  int fd;
  char *dst;
  size_t n;
  off_t off;
  ssize_t got;
} pread_job_t;

static void *pread_worker(void *arg) {
  pread_job_t *j = arg;
  size_t done = 0;
  while (done < j->n) {
    ssize_t r = pread(j->fd, j->dst + done, j->n - done, j->off + (off_t)done);
    if (r < 0 && errno == EINTR) continue;
    if (r < 0) {
      j->got = -1;
      return NULL;
    }
    if (r == 0) break;
    done += (size_t)r;
  }
  j->got = (ssize_t)done;
  return NULL;
}

/* read up to n bytes at P->pos with the reader threads */
static ssize_t read_parallel(pipe_t *P, char *dst, size_t n) {
  const int nt = P->o->num_threads;
  if (nt <= 1 || n < (4u << 20)) {
    pread_job_t j = {P->fd, dst, n, P->pos, 0};
    pread_worker(&j);
    return j.got;
  }
  pthread_t th[64];
  pread_job_t jobs[64];
  const int k = nt > 64 ? 64 : nt;
  const size_t per = (n + k - 1) / k;
  int started = 0;
  for (int i = 0; i < k; ++i) {
    const size_t a = (size_t)i * per;
    if (a >= n) break;
    jobs[i] = (pread_job_t){P->fd, dst + a, (a + per > n ? n - a : per), P->pos + (off_t)a, 0};
    pthread_create(&th[i], NULL, pread_worker, &jobs[i]);
    started++;
  }
  ssize_t total = 0;
  int short_read = 0, failed = 0;
  for (int i = 0; i < started; ++i) {
    pthread_join(th[i], NULL);
    if (jobs[i].got < 0) failed = 1;
    if (!short_read && jobs[i].got > 0) total += jobs[i].got;
    if (jobs[i].got < 0 || (size_t)jobs[i].got < jobs[i].n) short_read = 1;   /* EOF inside this piece */
  }
  return failed ? -1 : total;
}

static void reader_fail(pipe_t *P, int code) {
  pthread_mutex_lock(&P->mu);
  P->error = code;
  pthread_cond_broadcast(&P->cv);
  pthread_mutex_unlock(&P->mu);
}

static void *reader_main(void *arg) {
  pipe_t *P = arg;
  int64_t target = 0;   /* --cg: file offset of the current chaos-game batch end */
  for (int64_t k = 0;; ++k) {
    slot_t *s = &P->slot[k % P->nslots];
    pthread_mutex_lock(&P->mu);
    while (s->state != 0 && !P->error) pthread_cond_wait(&P->cv, &P->mu);
    const int err = P->error;
    pthread_mutex_unlock(&P->mu);
    if (err) break;
    trace_at(P, k, 0, -1);
    memcpy(s->buf, P->carry, P->carry_len);
    s->len = P->carry_len;
    const off_t g0 = P->pos - (off_t)P->carry_len;   /* file offset of buf[0] */
    int64_t use = 0;
    if (P->cg_batch > 0) {
      /* the next batch end(s): the last record ending at or before target */
      for (;;) {
        target += P->cg_batch;
        const size_t want = (size_t)(target - g0) < s->cap - 1 ? (size_t)(target - g0) : s->cap - 1;
        if (want > s->len) {
          const ssize_t got = read_parallel(P, s->buf + s->len, want - s->len);
          if (got < 0) {
            use = -1;   /* an I/O error, reported as such below */
            break;
          }
          P->pos += got;
          s->len += (size_t)got;
        }
        s->eof = P->pos >= P->size;
        if (s->eof) break;
        use = hpgq_fastq_complete_prefix(s->buf, (int64_t)s->len, 0);
        if (use > 0 || s->len >= s->cap - 1) break;
        /* no record ends in this batch (one longer than the batch): the next */
      }
    } else {
      const size_t room = s->cap - 1 - s->len;   /* 1 byte for a final newline */
      const ssize_t got = read_parallel(P, s->buf + s->len, room);
      if (got < 0) {
        reader_fail(P, HPGQ_E_IO);
        break;
      }
      P->pos += got;
      s->len += (size_t)got;
      s->eof = P->pos >= P->size;
    }
    if (use < 0) {
      reader_fail(P, HPGQ_E_IO);
      break;
    }
    if (s->eof && s->len > 0 && s->buf[s->len - 1] != '\n') s->buf[s->len++] = '\n';
    if (s->eof || P->cg_batch <= 0) use = hpgq_fastq_complete_prefix(s->buf, (int64_t)s->len, s->eof);
    if (use <= 0 && !s->eof) {
      fprintf(stderr, "hpg-fastq: a record longer than --chunk-mb, or not FASTQ\n");
      pthread_mutex_lock(&P->mu);
      P->error = HPGQ_E_FORMAT;
      pthread_cond_broadcast(&P->cv);
      pthread_mutex_unlock(&P->mu);
      break;
    }
    s->use = (size_t)(use > 0 ? use : 0);
    P->carry_len = s->len - s->use;
    if (P->carry_len > MAX_CARRY) {
      pthread_mutex_lock(&P->mu);
      P->error = HPGQ_E_FORMAT;
      pthread_cond_broadcast(&P->cv);
      pthread_mutex_unlock(&P->mu);
      break;
    }
    memcpy(P->carry, s->buf + s->use, P->carry_len);
    trace_at(P, k, 1, -1);
    pthread_mutex_lock(&P->mu);
    s->chunk = k;
    s->state = 1;
    P->chunks = k + 1;
    if (s->eof) P->reader_done = 1;
    pthread_cond_broadcast(&P->cv);
    pthread_mutex_unlock(&P->mu);
    if (s->eof) break;
  }
  pthread_mutex_lock(&P->mu);
  P->reader_done = 1;
  pthread_cond_broadcast(&P->cv);
  pthread_mutex_unlock(&P->mu);
  return NULL;
}

/* ---- writer ------------------------------------------------------------- */

static int write_span(FILE *f, const char *p, size_t n) { return fwrite(p, 1, n, f) == n ? 0 : -1; }

/* the spans of one output class, flushed by writev (the stream is drained
 * first: nothing of it is buffered in stdio across these calls) */
#define SPAN_IOV 1024
typedef struct {
  FILE *f;
  struct iovec v[SPAN_IOV];
  int n;
} spans_t;

static int spans_flush(spans_t *S) {
  int k = 0;
  while (k < S->n) {
    const int cnt = S->n - k;
    const ssize_t w = writev(fileno(S->f), S->v + k, cnt);
    if (w < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    size_t left = (size_t)w;   /* partial write: skip the whole iovecs, trim the next */
    while (k < S->n && left >= S->v[k].iov_len) left -= S->v[k++].iov_len;
    if (k < S->n) {
      S->v[k].iov_base = (char *)S->v[k].iov_base + left;
      S->v[k].iov_len -= left;
    }
  }
  S->n = 0;
  return 0;
}

static int spans_add(spans_t *S, const char *p, size_t n) {
  if (S->n && (const char *)S->v[S->n - 1].iov_base + S->v[S->n - 1].iov_len == p) {   /* contiguous */
    S->v[S->n - 1].iov_len += n;
    return 0;
  }
  if (S->n == SPAN_IOV && spans_flush(S)) return -1;
  S->v[S->n].iov_base = (void *)p;
  S->v[S->n].iov_len = n;
  S->n++;
  return 0;
}

static int write_slot(pipe_t *P, slot_t *s) {
  const int edit = P->o->command == CMD_EDIT;
  const int filter_on = P->o->filter_on;
  if (edit) {   /* the worker assembled the trimmed records (assemble_edit) */
    FILE *fc[2] = {P->out_pass, P->out_fail};
    for (int c = 0; c < 2; ++c)
      if (fc[c] && s->out_len[c] && write_span(fc[c], s->out[c], s->out_len[c])) return -1;
    P->written_pass += s->out_n[0];
    P->written_fail += s->out_n[1];
    return 0;
  }
  /* whole input records, consecutive records of one class as one span, the
   * spans of each class gathered into writev calls of up to SPAN_IOV spans
   * (one write per span -- ~5 KB at 6 % failed reads -- ran at 4 GB/s into
   * tmpfs, which takes 8.6 GB/s in 64 KB writes) */
  static __thread spans_t S[2];
  S[0].f = P->out_pass;
  S[1].f = P->out_fail;   /* (without a filter every record is class 0) */
  for (int c = 0; c < 2; ++c) {
    S[c].n = 0;
    if (S[c].f && fflush(S[c].f)) return -1;
  }
  for (int64_t i = 0; i < s->nreads; ++i) {
    const int pass = s->mask[i] != 0;
    spans_t *sp = &S[pass || !filter_on ? 0 : 1];
    int64_t j = i + 1;
    while (j < s->nreads && (s->mask[j] != 0) == pass) ++j;
    if (sp->f) {
      const uint32_t a = s->rec_start[i];
      const uint32_t ee = j < s->nreads ? s->rec_start[j] : (uint32_t)s->use;
      if (spans_add(sp, s->buf + a, ee - a)) return -1;
      if (pass) P->written_pass += (uint64_t)(j - i);
      else P->written_fail += (uint64_t)(j - i);
    }
    i = j - 1;
  }
  for (int c = 0; c < 2; ++c)
    if (S[c].f && S[c].n && spans_flush(&S[c])) return -1;
  return 0;
}

static void *writer_main(void *arg) {
  pipe_t *P = arg;
  for (int64_t k = 0;; ++k) {
    slot_t *s = &P->slot[k % P->nslots];
    pthread_mutex_lock(&P->mu);
    while (!(s->state == 2 && s->chunk == k) && !P->error && !(P->reader_done && k >= P->chunks))
      pthread_cond_wait(&P->cv, &P->mu);
    const int stop = P->error || !(s->state == 2 && s->chunk == k);
    pthread_mutex_unlock(&P->mu);
    if (stop) break;
    const int rc = write_slot(P, s);
    pthread_mutex_lock(&P->mu);
    if (rc) P->error = -1;
    s->state = 0;
    pthread_cond_broadcast(&P->cv);
    pthread_mutex_unlock(&P->mu);
    if (rc) break;
  }
  return NULL;
}

/* ---- GPU worker (this thread) -------------------------------------------- */

/* edit: a chunk's trimmed records per output class, in input order (header
 * line, seq[ts, len - te), '+' line, qual[ts, len - te); each at most its input
 * record's bytes), built on the worker thread: with the writer formatting them
 * read by read through stdio (6 calls per read) `edit` ran at 6.8 Mreads/s end
 * to end against 135 for `stats` */
static int assemble_edit(pipe_t *P, slot_t *s) {
  const int filter_on = P->o->filter_on;
  FILE *fc[2] = {P->out_pass, P->out_fail};
  for (int c = 0; c < 2; ++c) {
    s->out_len[c] = 0;
    s->out_n[c] = 0;
    if (fc[c] && s->out_cap[c] < s->use + 64) {
      free(s->out[c]);
      s->out_cap[c] = s->use + s->use / 8 + 64;
      s->out[c] = malloc(s->out_cap[c]);
      if (!s->out[c]) {
        s->out_cap[c] = 0;
        return HPGQ_E_NOMEM;
      }
    }
  }
  char *d[2] = {s->out[0], s->out[1]};
  for (int64_t i = 0; i < s->nreads; ++i) {
    const int c = s->mask[i] != 0 || !filter_on ? 0 : 1;
    if (!fc[c]) continue;
    const uint32_t a = s->rec_start[i];
    const uint32_t ts = s->trim[i] & 0xFFFFu, te = s->trim[i] >> 16;
    const uint32_t len = (uint32_t)(s->idx[i + 1] - s->idx[i]);
    const uint32_t keep = len - ts - te;
    const uint32_t hl = s->seq_start[i] - a, pl = s->qual_start[i] - s->plus_start[i];
    char *o = d[c];
    memcpy(o, s->buf + a, hl);                               /* header line */
    o += hl;
    memcpy(o, s->buf + s->seq_start[i] + ts, keep);
    o += keep;
    *o++ = '\n';
    memcpy(o, s->buf + s->plus_start[i], pl);                 /* '+' line */
    o += pl;
    memcpy(o, s->buf + s->qual_start[i] + ts, keep);
    o += keep;
    *o++ = '\n';
    d[c] = o;
    s->out_n[c]++;
  }
  for (int c = 0; c < 2; ++c) s->out_len[c] = fc[c] ? (size_t)(d[c] - s->out[c]) : 0;
  return 0;
}

/* the per-chunk results come back by DMA: page-locked buffers (pageable
 * destinations are staged through the runtime's bounce buffer, synchronously) */
static void free_results(slot_t *s) {
  void **b[7] = {(void **)&s->mask, (void **)&s->trim, (void **)&s->rec_start, (void **)&s->seq_start,
                 (void **)&s->plus_start, (void **)&s->qual_start, (void **)&s->idx};
  for (int i = 0; i < 7; ++i) {
    hpgq_host_free(*b[i]);
    *b[i] = NULL;
  }
  s->res_cap = 0;
}

static int ensure_results(slot_t *s, int64_t n) {
  if ((size_t)n <= s->res_cap) return 0;
  free_results(s);
  const size_t c = (size_t)n + (size_t)n / 4 + 1024;
  void **b[7] = {(void **)&s->mask, (void **)&s->trim, (void **)&s->rec_start, (void **)&s->seq_start,
                 (void **)&s->plus_start, (void **)&s->qual_start, (void **)&s->idx};
  const size_t sz[7] = {c, c * 4, c * 4, c * 4, c * 4, c * 4, (c + 1) * 4};
  for (int i = 0; i < 7; ++i)
    if (hpgq_host_alloc(b[i], sz[i])) {
      free_results(s);
      return -1;
    }
  s->res_cap = c;
  return 0;
}

/* ---- mapped outputs: placement in input order, parallel copy -------------- */

/* output class of record i (0: passed / edit.fq, 1: failed.fq) and its output
 * bytes: the whole input record (filter) or the trimmed one (edit) */
static inline int rec_class(const pipe_t *P, const slot_t *s, int64_t i) {
  return s->mask[i] != 0 || !P->o->filter_on ? 0 : 1;
}

static inline uint64_t rec_out_bytes(const pipe_t *P, const slot_t *s, int64_t i) {
  if (P->o->command != CMD_EDIT) {
    const uint32_t ee = i + 1 < s->nreads ? s->rec_start[i + 1] : (uint32_t)s->use;
    return ee - s->rec_start[i];
  }
  const uint32_t ts = s->trim[i] & 0xFFFFu, te = s->trim[i] >> 16;
  const uint32_t keep = (uint32_t)(s->idx[i + 1] - s->idx[i]) - ts - te;
  return (uint64_t)(s->seq_start[i] - s->rec_start[i]) + (s->qual_start[i] - s->plus_start[i]) + 2u * keep + 2u;
}

#define MAX_COPIERS 64
typedef struct {
  pipe_t *P;
  slot_t *s;
  int64_t i0, i1;      /* records of this part */
  uint64_t bytes[2];   /* its output bytes per class */
  char *dst[2];        /* where its records go */
  pthread_t th;
  int started;
} copy_part_t;

/* records [i0, i1) into the maps at dst[class] */
static void copy_records(pipe_t *P, slot_t *s, int64_t i0, int64_t i1, char *dst[2]) {
  const int edit = P->o->command == CMD_EDIT;
  for (int64_t i = i0; i < i1; ++i) {
    const int c = rec_class(P, s, i);
    if (!P->map[c]) continue;
    if (!edit) {   /* a run of same-class records is one contiguous span */
      int64_t j = i + 1;
      while (j < i1 && rec_class(P, s, j) == c) ++j;
      const uint32_t a = s->rec_start[i];
      const uint32_t ee = j < s->nreads ? s->rec_start[j] : (uint32_t)s->use;
      memcpy(dst[c], s->buf + a, ee - a);
      dst[c] += ee - a;
      i = j - 1;
      continue;
    }
    const uint32_t a = s->rec_start[i];
    const uint32_t ts = s->trim[i] & 0xFFFFu, te = s->trim[i] >> 16;
    const uint32_t keep = (uint32_t)(s->idx[i + 1] - s->idx[i]) - ts - te;
    const uint32_t hl = s->seq_start[i] - a, pl = s->qual_start[i] - s->plus_start[i];
    char *o = dst[c];
    memcpy(o, s->buf + a, hl);                              /* header line */
    o += hl;
    memcpy(o, s->buf + s->seq_start[i] + ts, keep);
    o += keep;
    *o++ = '\n';
    memcpy(o, s->buf + s->plus_start[i], pl);                /* '+' line */
    o += pl;
    memcpy(o, s->buf + s->qual_start[i] + ts, keep);
    o += keep;
    *o++ = '\n';
    dst[c] = o;
  }
}

static void *size_part(void *arg) {
  copy_part_t *cp = arg;
  cp->bytes[0] = cp->bytes[1] = 0;
  for (int64_t i = cp->i0; i < cp->i1; ++i) cp->bytes[rec_class(cp->P, cp->s, i)] += rec_out_bytes(cp->P, cp->s, i);
  return NULL;
}

/* fn over the parts: part 0 on this thread, the others on threads of their own
 * (a part whose thread cannot start runs here too) */
static void run_parts(void *(*fn)(void *), copy_part_t *part, int n) {
  for (int t = 1; t < n; ++t) part[t].started = pthread_create(&part[t].th, NULL, fn, &part[t]) == 0;
  fn(&part[0]);
  for (int t = 1; t < n; ++t) {
    if (part[t].started) pthread_join(part[t].th, NULL);
    else fn(&part[t]);
  }
}

static void copy_part_run(void *arg) {
  copy_part_t *cp = arg;
  copy_records(cp->P, cp->s, cp->i0, cp->i1, cp->dst);
}

/* copier thread: takes parts off the queue; the last part of a chunk frees its
 * slot for the reader */
static void *copier_main(void *arg) {
  pipe_t *P = arg;
  for (;;) {
    pthread_mutex_lock(&P->cq_mu);
    while (P->cq_head == P->cq_tail && !P->cq_exit) pthread_cond_wait(&P->cq_cv, &P->cq_mu);
    if (P->cq_head == P->cq_tail) {
      pthread_mutex_unlock(&P->cq_mu);
      break;
    }
    copy_part_t *cp = P->cq[P->cq_head % P->cq_cap];
    P->cq_head++;
    pthread_mutex_unlock(&P->cq_mu);
    /* a store the file system cannot back ends the copy with HPGQ_E_IO, not SIGBUS */
    const int e = mapout_guard(copy_part_run, cp);
    pthread_mutex_lock(&P->mu);
    if (e && !P->error) P->error = e;
    if (--cp->s->parts_left == 0) {
      cp->s->state = 0;
      P->copies_pending--;
      pthread_cond_broadcast(&P->cv);
    }
    pthread_mutex_unlock(&P->mu);
  }
  return NULL;
}

static int start_copiers(pipe_t *P) {
  int n = P->o->copy_threads > 0 ? P->o->copy_threads : P->o->num_threads;
  if (n > 64) n = 64;
  if (n < 1) n = 1;
  P->cq_cap = P->nslots * MAX_COPIERS;
  P->cq = calloc((size_t)P->cq_cap, sizeof(void *));
  if (!P->cq) return HPGQ_E_NOMEM;
  for (int i = 0; i < P->nslots; ++i) {
    P->slot[i].parts = calloc(MAX_COPIERS, sizeof(copy_part_t));
    if (!P->slot[i].parts) return HPGQ_E_NOMEM;
  }
  for (int t = 0; t < n; ++t) {
    if (pthread_create(&P->copier[t], NULL, copier_main, P)) break;
    P->ncopiers++;
  }
  return P->ncopiers ? 0 : HPGQ_E_NOMEM;
}

/* every placed chunk copied, then the copiers end */
static void stop_copiers(pipe_t *P) {
  pthread_mutex_lock(&P->mu);
  while (P->copies_pending > 0) pthread_cond_wait(&P->cv, &P->mu);
  pthread_mutex_unlock(&P->mu);
  pthread_mutex_lock(&P->cq_mu);
  P->cq_exit = 1;
  pthread_cond_broadcast(&P->cq_cv);
  pthread_mutex_unlock(&P->cq_mu);
  for (int t = 0; t < P->ncopiers; ++t) pthread_join(P->copier[t], NULL);
  P->ncopiers = 0;
}

/* a processed chunk into the mapped outputs: size its records per class (in
 * parallel), place it after chunk k-1 (which only needs k-1's sizes, not its
 * copies), queue its parts for the copier threads (the slot stays busy, state
 * 3, until they are copied) */
static int place_and_copy(pipe_t *P, slot_t *s, int *handed) {
  copy_part_t *part = s->parts;
  int n = P->ncopiers;   /* one part per copier thread (--copy-threads, default --num-threads) */
  const int64_t per_min = 16384;   /* records per copier at least */
  if (n > MAX_COPIERS) n = MAX_COPIERS;
  if ((int64_t)n > s->nreads / per_min + 1) n = (int)(s->nreads / per_min + 1);
  if (n < 1) n = 1;
  const int64_t per = (s->nreads + n - 1) / n;
  for (int t = 0; t < n; ++t) {
    copy_part_t *cp = &part[t];
    cp->P = P;
    cp->s = s;
    cp->i0 = (int64_t)t * per < s->nreads ? (int64_t)t * per : s->nreads;
    cp->i1 = cp->i0 + per < s->nreads ? cp->i0 + per : s->nreads;
  }
  run_parts(size_part, part, n);
  uint64_t sz[2] = {0, 0}, base[2] = {0, 0}, npass = 0, nfail = 0;
  for (int t = 0; t < n; ++t) {
    sz[0] += part[t].bytes[0];
    sz[1] += part[t].bytes[1];
  }
  int rc = 0;
  pthread_mutex_lock(&P->mu);
  while (P->placed != s->chunk && !P->error) pthread_cond_wait(&P->cv, &P->mu);
  if (P->error) {
    rc = P->error;   /* (stop; a copier's HPGQ_E_IO reaches the caller as is) */
  } else if (P->out_off[0] + sz[0] > P->map_cap || P->out_off[1] + sz[1] > P->map_cap) {
    rc = HPGQ_E_IO;   /* (cannot happen: each output is at most the input) */
  } else if ((rc = mapout_error(&P->mo)) == 0) {   /* (a window the prefault threads could not back) */
    for (int c = 0; c < 2; ++c) {
      base[c] = P->out_off[c];
      P->out_off[c] += sz[c];
      mapout_advance(&P->mo, c, P->out_off[c]);
    }
    P->placed++;
  }
  pthread_cond_broadcast(&P->cv);
  pthread_mutex_unlock(&P->mu);
  if (rc) return rc;
  trace_at(P, s->chunk, 7, -1);
  for (int t = 0; t < n; ++t) {
    for (int c = 0; c < 2; ++c) {
      part[t].dst[c] = P->map[c] ? P->map[c] + base[c] : NULL;
      base[c] += part[t].bytes[c];
    }
  }
  for (int64_t i = 0; i < s->nreads; ++i) {
    if (rec_class(P, s, i)) ++nfail;
    else ++npass;
  }
  const int queue = s->nreads > 0;
  pthread_mutex_lock(&P->mu);
  P->written_pass += npass;
  P->written_fail += nfail;
  if (queue) {   /* busy until copied (set before the parts can finish) */
    s->state = 3;
    s->parts_left = n;
    P->copies_pending++;
  }
  pthread_mutex_unlock(&P->mu);
  /* from here the copiers own the slot: the last part frees it and the reader
   * may refill it at once, so neither this function nor the worker touches s */
  *handed = queue;
  if (queue) {
    pthread_mutex_lock(&P->cq_mu);
    for (int t = 0; t < n; ++t) P->cq[P->cq_tail++ % P->cq_cap] = &part[t];
    pthread_cond_broadcast(&P->cq_cv);
    pthread_mutex_unlock(&P->cq_mu);
  }
  return 0;
}

/* map the outputs for the parallel writer (hpgq_mapout.h): each is at most
 * the input (+ the final newline the reader may add); 0 when mapped, 1: the
 * stream writer runs (files left empty), < 0 an error */
static int map_outputs(pipe_t *P) {
  const int fd[2] = {P->out_pass ? fileno(P->out_pass) : -1, P->out_fail ? fileno(P->out_fail) : -1};
  P->map_cap = (size_t)P->size + 4096;
  /* --prefault-threads N: populate two chunks ahead of the placed records on
   * N threads.  Default none past the reserved first window: on MI355X boxes
   * the prefault threads made stored `filter` slower (same box, alternating:
   * median 16 vs 24-26 Mreads/s with 2 threads vs none, profiles/
   * r05_writer_ab.json) -- they contend with the copiers for the one file's
   * page allocation; the SIGBUS guard covers what is not reserved */
  const size_t ahead = (size_t)2 * ((size_t)P->o->chunk_mb << 20);
  const int pft = P->o->prefault_threads < 0 ? 0 : P->o->prefault_threads;
  const int rc = mapout_open(&P->mo, fd, P->map_cap, ahead, pft, P->o->writer_hook);
  if (rc) return rc;
  P->map[0] = P->mo.map[0];
  P->map[1] = P->mo.map[1];
  P->mmap_out = 1;
  return 0;
}

static void unmap_outputs(pipe_t *P, int *rc) {
  const uint64_t size[2] = {P->out_off[0], P->out_off[1]};
  const int e = mapout_close(&P->mo, size);
  if (e && *rc == 0) *rc = e;
  P->map[0] = P->map[1] = NULL;
}

/* one GPU worker: its own ctx, parser, k-mer and CGR accumulators on one device */
typedef struct {
  pipe_t *P;
  const hpgq_params_t *p;
  int w, device;
  hpgq_ctx_t *ctx;
  hpgq_parser_t *ps;
  hpgq_kmers_t *km;
  hpgq_cgr_t *cg;
  uint8_t *d_mask;
  uint32_t *d_trim;
  size_t dcap;
  int rc;
  pthread_t th;
  uint64_t num_reads;
  int cg_exact_calls;
  double fastq_bytes;
} worker_t;

static int worker_open(worker_t *W) {
  const cli_options_t *o = W->P->o;
  int rc = hpgq_open(&W->ctx, W->device, W->p);
  if (rc == 0) rc = hpgq_parser_open(&W->ps, W->device, hpgq_stream(W->ctx));
  /* --kmers counts the reads the stats merge (passed ones when filtering,
   * src/stats_fastq.c:268-272,384-410) on the engine's stream, after it */
  if (rc == 0 && o->kmers_on) rc = hpgq_kmers_open(&W->km, W->device, W->p->lmax, hpgq_stream(W->ctx));
  /* --cg: chaos_game_fill_tables per batch (= chunk), the base quality from
   * --quality-encoding; with a filter only the passed reads (ONLY_VALID_READS
   * with the mask as read_status, old/chaos_game.c:188) */
  if (rc == 0 && o->cg_on) rc = hpgq_cgr_open(&W->cg, W->device, o->k_cg, W->p->phred);
  return rc;
}

static void worker_close(worker_t *W) {
  hpgq_device_free(W->d_mask);
  hpgq_device_free(W->d_trim);
  hpgq_parser_close(W->ps);
  hpgq_kmers_close(W->km);
  hpgq_cgr_close(W->cg);
  hpgq_close(W->ctx);
}

/* one chunk on the worker's GPU (parse, engine, k-mers, CGR; results for the writer) */
static int worker_chunk(worker_t *W, slot_t *s) {
  const cli_options_t *o = W->P->o;
  const int writes = o->command != CMD_STATS;
  const int edit = o->command == CMD_EDIT;
  const int need_mask = writes || ((W->km || W->cg) && o->filter_on);
  hpgq_batch_t b;
  int rc = hpgq_parse_host(W->ps, s->buf, (int64_t)s->use, &b);
  trace_at(W->P, s->chunk, 5, -1);
  if (rc || b.num_reads == 0) {
    s->nreads = 0;
    return rc;
  }
  if (need_mask && (size_t)b.num_reads > W->dcap) {
    hpgq_device_free(W->d_mask);
    hpgq_device_free(W->d_trim);
    W->d_mask = NULL;
    W->d_trim = NULL;
    W->dcap = (size_t)b.num_reads + (size_t)b.num_reads / 4 + 1024;
    rc = hpgq_device_alloc(W->device, (void **)&W->d_mask, W->dcap);
    if (rc == 0) rc = hpgq_device_alloc(W->device, (void **)&W->d_trim, W->dcap * 4);
  }
  if (rc == 0) {   /* the long-read tails for the unit's longest record: no second pass */
    const int64_t ml = hpgq_parser_max_length(W->ps);
    rc = hpgq_reserve_length(W->ctx, ml);
    if (rc == 0 && W->km) rc = hpgq_kmers_reserve_length(W->km, ml);
  }
  if (rc == 0) rc = hpgq_run_device(W->ctx, &b, NULL, need_mask ? W->d_mask : NULL, edit ? W->d_trim : NULL);
  if (rc == 0 && W->km) rc = hpgq_kmers_count_device(W->km, &b, o->filter_on ? W->d_mask : NULL);
  if (rc == 0 && writes) {
    s->nreads = b.num_reads;
    if (ensure_results(s, b.num_reads)) rc = HPGQ_E_NOMEM;
    if (rc == 0) rc = hpgq_copy_to_host(W->ctx, s->mask, W->d_mask, (size_t)b.num_reads);
    if (rc == 0 && edit) {
      rc = hpgq_copy_to_host(W->ctx, s->trim, W->d_trim, (size_t)b.num_reads * 4);
      if (rc == 0) rc = hpgq_copy_to_host(W->ctx, s->idx, b.data_indices, ((size_t)b.num_reads + 1) * 4);
    }
    if (rc == 0) rc = hpgq_parse_records(W->ps, s->rec_start, s->seq_start, s->plus_start, s->qual_start);
  }
  trace_at(W->P, s->chunk, 3, -1);
  if (rc == 0) rc = hpgq_sync(W->ctx);
  trace_at(W->P, s->chunk, 6, -1);
  if (rc == 0 && edit && !W->P->mmap_out) rc = assemble_edit(W->P, s);
  if (rc == 0 && W->cg) {   /* after the parse and the mask; settled before the next parse reuses b */
    rc = hpgq_cgr_fill_device(W->cg, &b, o->filter_on ? W->d_mask : NULL,
                              o->filter_on ? HPGQ_CGR_ONLY_VALID_READS : HPGQ_CGR_ALL_READS);
    if (rc == 0) rc = hpgq_cgr_sync(W->cg);
    if (rc == 0) W->cg_exact_calls += hpgq_cgr_last_exact(W->cg);
  }
  W->num_reads += (uint64_t)b.num_reads;
  return rc;
}

static void *worker_main(void *arg) {
  worker_t *W = arg;
  pipe_t *P = W->P;
  const int writes = P->o->command != CMD_STATS;
  for (int64_t k = W->w;; k += P->nworkers) {
    slot_t *s = &P->slot[k % P->nslots];
    pthread_mutex_lock(&P->mu);
    while (!(s->state == 1 && s->chunk == k) && !P->error && !(P->reader_done && k >= P->chunks))
      pthread_cond_wait(&P->cv, &P->mu);
    const int stop = P->error || !(s->state == 1 && s->chunk == k);
    pthread_mutex_unlock(&P->mu);
    if (stop) break;
    trace_at(P, k, 2, W->w);
    const size_t use = s->use;   /* (s is the copiers' once place_and_copy handed it over) */
    int handed = 0;
    int rc = worker_chunk(W, s);
    if (rc == 0 && writes && P->mmap_out) {
      rc = place_and_copy(P, s, &handed);   /* (an empty chunk is placed too: input order) */
    }
    trace_at(P, k, 4, -1);
    W->fastq_bytes += (double)use;
    pthread_mutex_lock(&P->mu);
    if (rc && !P->error) P->error = rc;
    if (!handed) s->state = writes && rc == 0 && !P->mmap_out ? 2 : 0;   /* (handed: the copiers free it) */
    pthread_cond_broadcast(&P->cv);
    pthread_mutex_unlock(&P->mu);
    if (rc) {
      W->rc = rc;
      break;
    }
  }
  return NULL;
}

/* dst (nm sets, layout of lmax ld) += src (nm sets, layout of lmax ls <= ld):
 * the workers' full-length counter sets (hpgq_read_counters_ext) */
static void add_relayout(uint64_t *dst, int ld, const uint64_t *src, int ls, int nm) {
  for (int m = 0; m < nm; ++m) {
    uint64_t *d = dst + (size_t)m * hpgq_counters_len(ld);
    const uint64_t *x = src + (size_t)m * hpgq_counters_len(ls);
    for (int i = 0; i < HPGQ_NUM_SCALARS; ++i) d[i] += x[i];
    for (int i = 0; i <= ls; ++i) d[hpgq_off_hist_len(ld) + i] += x[hpgq_off_hist_len(ls) + i];
    for (int i = 0; i < HPGQ_MEANQ_BINS; ++i) d[hpgq_off_hist_meanq(ld) + i] += x[hpgq_off_hist_meanq(ls) + i];
    for (int i = 0; i < HPGQ_GC_BINS; ++i) d[hpgq_off_hist_gc(ld) + i] += x[hpgq_off_hist_gc(ls) + i];
    for (int i = 0; i < ls; ++i) d[hpgq_off_pos_qsum(ld) + i] += x[hpgq_off_pos_qsum(ls) + i];
    for (int b = 0; b < 5; ++b)
      for (int i = 0; i < ls; ++i) d[hpgq_off_pos_base(ld, b) + i] += x[hpgq_off_pos_base(ls, b) + i];
  }
}

int cli_run(const cli_options_t *o, const hpgq_params_t *p, cli_result_t *res) {
  pipe_t P;
  memset(&P, 0, sizeof(P));
  P.trace = getenv("HPGQ_TRACE") != NULL;
  P.o = o;
  memset(res, 0, sizeof(*res));
  P.fd = open(o->in_filename, O_RDONLY);
  if (P.fd < 0) return HPGQ_E_INVALID;
  struct stat st;
  fstat(P.fd, &st);
  P.size = st.st_size;
  pthread_mutex_init(&P.mu, NULL);
  pthread_cond_init(&P.cv, NULL);
  pthread_mutex_init(&P.cq_mu, NULL);
  pthread_cond_init(&P.cq_cv, NULL);

  /* GPU workers: --gpu-workers per device on --gpus devices (0: every visible
   * one); worker w on device (gpu + w mod ngpus) mod ndev */
  const int ndev = hpgq_device_count();
  if (ndev <= 0) {
    close(P.fd);
    return HPGQ_E_NO_DEVICE;
  }
  const int ngpus = o->num_gpus > 0 ? o->num_gpus : ndev;
  int G = ngpus * (o->gpu_workers > 0 ? o->gpu_workers : 1);
  if (G > MAX_WORKERS) G = MAX_WORKERS;
  P.nworkers = G;
  /* one slot per worker + the reader's + the writer's + one to run ahead (a
   * bound that does not double with the worker count: 16 workers of 256 MB
   * chunks would otherwise pin 10 GB) */
  P.nslots = G + 3;
  if (P.nslots > MAX_SLOTS) P.nslots = MAX_SLOTS;
  bind_numa(o, ngpus, ndev);
  P.cg_batch = o->cg_on ? o->cg_batch_size : 0;
  worker_t W[MAX_WORKERS];
  memset(W, 0, sizeof(W));
  int rc = 0;
  for (int w = 0; w < G && rc == 0; ++w) {
    W[w].P = &P;
    W[w].p = p;
    W[w].w = w;
    W[w].device = (o->device + w % ngpus) % ndev;
    rc = worker_open(&W[w]);
  }
  /* a chunk holds --chunk-mb of text (with --cg: one chaos-game batch) */
  size_t chunk = (size_t)o->chunk_mb << 20;
  if (P.cg_batch > 0 && (size_t)P.cg_batch > chunk) chunk = (size_t)P.cg_batch;
  const double pinned_gb = (double)P.nslots * (double)(chunk + MAX_CARRY) / 1e9;
  if (pinned_gb > 4.0)
    fprintf(stderr, "hpg-fastq: %d chunks of %zu MB: %.1f GB of page-locked host memory\n", P.nslots,
            (chunk + MAX_CARRY) >> 20, pinned_gb);
  for (int i = 0; i < P.nslots && rc == 0; ++i) {
    P.slot[i].cap = chunk + MAX_CARRY;
    rc = hpgq_host_alloc((void **)&P.slot[i].buf, P.slot[i].cap);
  }
  P.carry = malloc(MAX_CARRY + 16);
  const int writes = o->command != CMD_STATS;
  const int edit = o->command == CMD_EDIT;
  if (rc == 0 && writes) {
    char path[4096];
    /* "w+": read + write, which a shared writable mapping needs (an O_WRONLY
     * descriptor cannot be mapped) */
    snprintf(path, sizeof(path), "%s/%s.fq", o->out_dirname, edit ? "edit" : "passed");
    P.out_pass = fopen(path, "w+");
    if (!edit || o->filter_on) {
      snprintf(path, sizeof(path), "%s/failed.fq", o->out_dirname);
      P.out_fail = fopen(path, "w+");
    }
    if (!P.out_pass || ((!edit || o->filter_on) && !P.out_fail)) rc = HPGQ_E_INVALID;
    if (P.out_pass) setvbuf(P.out_pass, NULL, _IOFBF, 16 << 20);
    if (P.out_fail) setvbuf(P.out_fail, NULL, _IOFBF, 16 << 20);
    if (rc == 0 && !o->stream_writer) {   /* not mappable (1): the writer thread */
      const int m = map_outputs(&P);
      if (m < 0) rc = m;
    }
    res->writer = P.mmap_out ? 1 : 2;
    if (P.trace && P.mmap_out)
      fprintf(stderr, "hpg-fastq: writer: mapped output files, parallel copy (windows reserved by %s)\n",
              mapout_mode_name[__atomic_load_n(&P.mo.mode, __ATOMIC_RELAXED)]);
    else if (P.trace)
      fprintf(stderr, "hpg-fastq: writer: one stream writer thread\n");
  }
  if (rc) goto done;

  const double t0 = now_s();
  P.t0 = t0;
  if (P.mmap_out && (rc = start_copiers(&P))) goto done;
  pthread_t reader, writer;
  pthread_create(&reader, NULL, reader_main, &P);
  const int writer_thread = writes && !P.mmap_out;
  if (writer_thread) pthread_create(&writer, NULL, writer_main, &P);
  for (int w = 0; w < G; ++w) pthread_create(&W[w].th, NULL, worker_main, &W[w]);
  for (int w = 0; w < G; ++w) pthread_join(W[w].th, NULL);
  /* (a worker that stopped on an error left P.error set: reader and writer end) */
  pthread_mutex_lock(&P.mu);
  pthread_cond_broadcast(&P.cv);
  pthread_mutex_unlock(&P.mu);
  pthread_join(reader, NULL);
  if (writer_thread) pthread_join(writer, NULL);
  if (P.mmap_out) stop_copiers(&P);   /* every placed chunk is in the maps */
  for (int w = 0; w < G && rc == 0; ++w) rc = W[w].rc;
  /* (the reader's and writer's generic -1 is HPGQ_E_INVALID; a copier's or the
   * prefault threads' HPGQ_E_IO stays what it is) */
  if (rc == 0 && P.error)
    rc = P.error < 0 && P.error != HPGQ_E_FORMAT && P.error != HPGQ_E_IO ? HPGQ_E_INVALID : P.error;

  /* the read-sharded merge: device counters, k-mer and CGR tables summed over
   * the workers (u64; CGR u32, which wraps like the reference's tables).  The
   * counters and k-mer tables come at full length (the long-read tails,
   * hpgq_read_counters_ext / hpgq_kmers_read_ext): each worker's in the
   * layout of its own longest read, summed into the longest one's */
  const int nm = p->paired ? 2 : 1;
  int L = p->lmax, KP = 0;
  for (int w = 0; w < G && rc == 0; ++w) {
    int32_t lw = 0;
    rc = hpgq_read_counters_ext(W[w].ctx, NULL, 0, &lw);
    if (lw > L) L = lw;
    if (rc == 0 && o->kmers_on) rc = hpgq_kmers_read_ext(W[w].km, NULL, 0, &lw);
    if (o->kmers_on && lw > KP) KP = lw;
  }
  res->lmax = L;
  res->counters = rc == 0 ? calloc(hpgq_counters_len(L) * nm, sizeof(uint64_t)) : NULL;
  if (rc == 0 && !res->counters) rc = HPGQ_E_NOMEM;
  for (int w = 0; w < G && rc == 0; ++w) {
    int32_t lw = 0;
    rc = hpgq_read_counters_ext(W[w].ctx, NULL, 0, &lw);
    uint64_t *part = rc == 0 ? calloc(hpgq_counters_len(lw) * nm, sizeof(uint64_t)) : NULL;
    if (rc == 0 && !part) rc = HPGQ_E_NOMEM;
    if (rc == 0) rc = hpgq_read_counters_ext(W[w].ctx, part, hpgq_counters_len(lw) * nm, &lw);
    if (rc == 0) add_relayout(res->counters, L, part, lw, nm);
    free(part);
    res->num_reads += W[w].num_reads;
    res->fastq_bytes += W[w].fastq_bytes;
    res->cg_exact_calls += W[w].cg_exact_calls;
  }
  if (rc == 0 && o->kmers_on) {
    res->kmers_npos = KP;
    res->kmers = calloc((size_t)HPGQ_NUM_KMERS * KP + 1, sizeof(uint64_t));
    if (!res->kmers) rc = HPGQ_E_NOMEM;
    for (int w = 0; w < G && rc == 0; ++w) {
      int32_t pw = 0;
      rc = hpgq_kmers_read_ext(W[w].km, NULL, 0, &pw);
      uint64_t *kp = rc == 0 ? calloc((size_t)HPGQ_NUM_KMERS * pw + 1, sizeof(uint64_t)) : NULL;
      if (rc == 0 && !kp) rc = HPGQ_E_NOMEM;
      if (rc == 0) rc = hpgq_kmers_read_ext(W[w].km, kp, (size_t)HPGQ_NUM_KMERS * pw, &pw);
      for (int id = 0; rc == 0 && id < HPGQ_NUM_KMERS; ++id)
        for (int j = 0; j < pw; ++j) res->kmers[(size_t)id * KP + j] += kp[(size_t)id * pw + j];
      free(kp);
    }
  }
  if (rc == 0 && o->cg_on) {
    const size_t cells = (size_t)1 << (2 * o->k_cg);
    res->cg_seq = calloc(cells, sizeof(uint32_t));
    res->cg_q = calloc(cells, sizeof(uint32_t));
    uint32_t *ts = calloc(cells, sizeof(uint32_t)), *tq = calloc(cells, sizeof(uint32_t));
    if (!res->cg_seq || !res->cg_q || !ts || !tq) rc = HPGQ_E_NOMEM;
    for (int w = 0; w < G && rc == 0; ++w) {
      uint32_t words = 0;
      rc = hpgq_cgr_read(W[w].cg, ts, tq, &words);
      for (size_t i = 0; rc == 0 && i < cells; ++i) {
        res->cg_seq[i] += ts[i];
        res->cg_q[i] += tq[i];
      }
      res->cg_words += words;
    }
    free(ts);
    free(tq);
  }
  if (P.mmap_out) unmap_outputs(&P, &rc);   /* the files at their final sizes (inside the clock) */
  res->seconds = now_s() - t0;
  res->num_gpus = G;
  for (int64_t k = 0; P.trace && k < P.chunks && k < TRACE_MAX; ++k)
    fprintf(stderr,
            "trace chunk %lld: read %.1f-%.1f ms, worker %d %.1f-%.1f (parsed %.1f, sync %.1f-%.1f, placed %.1f) ms\n",
            (long long)k, 1e3 * P.tr[k][0], 1e3 * P.tr[k][1], P.tw[k], 1e3 * P.tr[k][2], 1e3 * P.tr[k][4],
            1e3 * P.tr[k][5], 1e3 * P.tr[k][3], 1e3 * P.tr[k][6], 1e3 * P.tr[k][7]);
  if (rc == 0) {
    res->num_passed = res->counters[HPGQ_S_NUM_PASSED];
    res->num_failed = res->counters[HPGQ_S_NUM_FAILED];
    res->num_edited = res->counters[HPGQ_S_NUM_EDITED];
  }

done:
  if (P.ncopiers) stop_copiers(&P);
  if (P.mmap_out) unmap_outputs(&P, &rc);
  if (P.out_pass) fclose(P.out_pass);
  if (P.out_fail) fclose(P.out_fail);
  for (int i = 0; i < P.nslots; ++i) {
    hpgq_host_free(P.slot[i].buf);
    free_results(&P.slot[i]);
    free(P.slot[i].parts);
    free(P.slot[i].out[0]);
    free(P.slot[i].out[1]);
  }
  free(P.carry);
  free(P.cq);
  for (int w = 0; w < G; ++w) worker_close(&W[w]);
  close(P.fd);
  return rc;
}
