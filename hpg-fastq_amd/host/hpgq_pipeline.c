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
 *   GPU        hpgq_parse_host (H2D + parse into a device batch) and
 *              hpgq_run_device (filter / edit / stats fused) on one stream;
 *              for filter / edit the mask, trims and record offsets come back.
 *   writer     (filter / edit) passed.fq / failed.fq / edit.fq in input
 *              order: filter copies whole input records; edit writes the
 *              header and '+' lines as read and the trimmed sequence /
 *              quality.
 * Stats never leave the device until the end (hpgq_read_counters).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "hpgq_cli.h"

#define NSLOTS 3
#define MAX_CARRY (64u << 20)   /* longest record the reader can carry over */

typedef struct {
  char *buf;          /* page-locked */
  size_t cap, len, use;
  int eof;
  int state;          /* 0 free, 1 filled (reader -> GPU), 2 processed (GPU -> writer) */
  /* GPU results for the writer */
  int64_t nreads;
  uint8_t *mask;
  uint32_t *trim, *rec_start, *seq_start, *plus_start, *qual_start;
  int32_t *idx;
  size_t res_cap;
} slot_t;

typedef struct {
  const cli_options_t *o;
  int fd;
  off_t size, pos;
  slot_t slot[NSLOTS];
  char *carry;
  size_t carry_len;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  int reader_done, error;
  int64_t chunks;
  FILE *out_pass, *out_fail;
  uint64_t written_pass, written_fail;
} pipe_t;

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
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
    if (r <= 0) break;
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
  int short_read = 0;
  for (int i = 0; i < started; ++i) {
    pthread_join(th[i], NULL);
    if (!short_read) total += jobs[i].got;
    if ((size_t)jobs[i].got < jobs[i].n) short_read = 1;   /* EOF inside this piece */
  }
  return total;
}

static void *reader_main(void *arg) {
  pipe_t *P = arg;
  for (int64_t k = 0;; ++k) {
    slot_t *s = &P->slot[k % NSLOTS];
    pthread_mutex_lock(&P->mu);
    while (s->state != 0 && !P->error) pthread_cond_wait(&P->cv, &P->mu);
    const int err = P->error;
    pthread_mutex_unlock(&P->mu);
    if (err) break;
    memcpy(s->buf, P->carry, P->carry_len);
    s->len = P->carry_len;
    const size_t room = s->cap - 1 - s->len;   /* 1 byte for a final newline */
    const ssize_t got = read_parallel(P, s->buf + s->len, room);
    if (got < 0) {
      pthread_mutex_lock(&P->mu);
      P->error = -1;
      pthread_cond_broadcast(&P->cv);
      pthread_mutex_unlock(&P->mu);
      break;
    }
    P->pos += got;
    s->len += (size_t)got;
    s->eof = P->pos >= P->size;
    if (s->eof && s->len > 0 && s->buf[s->len - 1] != '\n') s->buf[s->len++] = '\n';
    const int64_t use = hpgq_fastq_complete_prefix(s->buf, (int64_t)s->len, s->eof);
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
    pthread_mutex_lock(&P->mu);
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

static int write_slot(pipe_t *P, slot_t *s) {
  const int edit = P->o->command == CMD_EDIT;
  const int filter_on = P->o->filter_on;
  for (int64_t i = 0; i < s->nreads; ++i) {
    const int pass = s->mask[i] != 0;
    FILE *f = pass || !filter_on ? P->out_pass : P->out_fail;
    if (!f) continue;
    const uint32_t a = s->rec_start[i];
    const uint32_t e = i + 1 < s->nreads ? s->rec_start[i + 1] : (uint32_t)s->use;
    if (!edit) {
      /* whole input record; consecutive records of one class as one span */
      int64_t j = i + 1;
      while (j < s->nreads && (s->mask[j] != 0) == pass) ++j;
      const uint32_t ee = j < s->nreads ? s->rec_start[j] : (uint32_t)s->use;
      if (write_span(f, s->buf + a, ee - a)) return -1;
      if (pass) P->written_pass += (uint64_t)(j - i);
      else P->written_fail += (uint64_t)(j - i);
      i = j - 1;
      continue;
    }
    (void)e;
    const uint32_t ts = s->trim[i] & 0xFFFFu, te = s->trim[i] >> 16;
    const uint32_t len = (uint32_t)(s->idx[i + 1] - s->idx[i]);
    const uint32_t keep = len - ts - te;
    if (write_span(f, s->buf + a, s->seq_start[i] - a) ||                          /* header line */
        write_span(f, s->buf + s->seq_start[i] + ts, keep) || fputc('\n', f) == EOF ||
        write_span(f, s->buf + s->plus_start[i], s->qual_start[i] - s->plus_start[i]) ||   /* '+' line */
        write_span(f, s->buf + s->qual_start[i] + ts, keep) || fputc('\n', f) == EOF)
      return -1;
    if (pass || !filter_on) P->written_pass++;
    else P->written_fail++;
  }
  return 0;
}

static void *writer_main(void *arg) {
  pipe_t *P = arg;
  for (int64_t k = 0;; ++k) {
    slot_t *s = &P->slot[k % NSLOTS];
    pthread_mutex_lock(&P->mu);
    while (s->state != 2 && !P->error && !(P->reader_done && k >= P->chunks))
      pthread_cond_wait(&P->cv, &P->mu);
    const int stop = P->error || (s->state != 2);
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

static int ensure_results(slot_t *s, int64_t n) {
  if ((size_t)n <= s->res_cap) return 0;
  free(s->mask);
  free(s->trim);
  free(s->rec_start);
  free(s->seq_start);
  free(s->plus_start);
  free(s->qual_start);
  free(s->idx);
  const size_t c = (size_t)n + (size_t)n / 4 + 1024;
  s->mask = malloc(c);
  s->trim = malloc(c * 4);
  s->rec_start = malloc(c * 4);
  s->seq_start = malloc(c * 4);
  s->plus_start = malloc(c * 4);
  s->qual_start = malloc(c * 4);
  s->idx = malloc((c + 1) * 4);
  s->res_cap = c;
  return s->mask && s->trim && s->rec_start && s->seq_start && s->plus_start && s->qual_start &&
                 s->idx
             ? 0
             : -1;
}

int cli_run(const cli_options_t *o, const hpgq_params_t *p, uint64_t *counters, cli_result_t *res) {
  pipe_t P;
  memset(&P, 0, sizeof(P));
  P.o = o;
  memset(res, 0, sizeof(*res));
  P.fd = open(o->in_filename, O_RDONLY);
  if (P.fd < 0) return HPGQ_E_INVALID;
  struct stat st;
  fstat(P.fd, &st);
  P.size = st.st_size;
  pthread_mutex_init(&P.mu, NULL);
  pthread_cond_init(&P.cv, NULL);

  hpgq_ctx_t *ctx = NULL;
  hpgq_parser_t *ps = NULL;
  hpgq_kmers_t *km = NULL;
  hpgq_cgr_t *cg = NULL;
  int rc = hpgq_open(&ctx, o->device, p);
  if (rc == 0) rc = hpgq_parser_open(&ps, o->device, hpgq_stream(ctx));
  /* --kmers counts the reads the stats merge (passed ones when filtering,
   * src/stats_fastq.c:268-272,384-410) on the engine's stream, after it */
  if (rc == 0 && o->kmers_on) rc = hpgq_kmers_open(&km, o->device, p->lmax, hpgq_stream(ctx));
  /* --cg: chaos_game_fill_tables per parsed chunk (one call = one chunk), the
   * base quality from --quality-encoding; with a filter only the passed reads
   * (ONLY_VALID_READS with the mask as read_status, old/chaos_game.c:188) */
  if (rc == 0 && o->cg_on) rc = hpgq_cgr_open(&cg, o->device, o->k_cg, p->phred);
  const size_t chunk = (size_t)o->chunk_mb << 20;
  for (int i = 0; i < NSLOTS && rc == 0; ++i) {
    P.slot[i].cap = chunk + MAX_CARRY;
    rc = hpgq_host_alloc((void **)&P.slot[i].buf, P.slot[i].cap);
  }
  P.carry = malloc(MAX_CARRY + 16);
  uint8_t *d_mask = NULL;
  uint32_t *d_trim = NULL;
  size_t dcap = 0;
  const int writes = o->command != CMD_STATS;
  const int edit = o->command == CMD_EDIT;
  const int need_mask = writes || ((km || cg) && o->filter_on);
  if (rc == 0 && writes) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/%s.fq", o->out_dirname, edit ? "edit" : "passed");
    P.out_pass = fopen(path, "w");
    if (!edit || o->filter_on) {
      snprintf(path, sizeof(path), "%s/failed.fq", o->out_dirname);
      P.out_fail = fopen(path, "w");
    }
    if (!P.out_pass || ((!edit || o->filter_on) && !P.out_fail)) rc = HPGQ_E_INVALID;
    if (P.out_pass) setvbuf(P.out_pass, NULL, _IOFBF, 16 << 20);
    if (P.out_fail) setvbuf(P.out_fail, NULL, _IOFBF, 16 << 20);
  }
  if (rc) goto done;

  const double t0 = now_s();
  pthread_t reader, writer;
  pthread_create(&reader, NULL, reader_main, &P);
  if (writes) pthread_create(&writer, NULL, writer_main, &P);
  for (int64_t k = 0;; ++k) {
    slot_t *s = &P.slot[k % NSLOTS];
    pthread_mutex_lock(&P.mu);
    while (s->state != 1 && !P.error && !(P.reader_done && k >= P.chunks))
      pthread_cond_wait(&P.cv, &P.mu);
    const int stop = P.error || s->state != 1;
    pthread_mutex_unlock(&P.mu);
    if (stop) break;
    hpgq_batch_t b;
    rc = hpgq_parse_host(ps, s->buf, (int64_t)s->use, &b);
    if (rc == 0 && b.num_reads > 0) {
      if (need_mask && (size_t)b.num_reads > dcap) {
        hpgq_device_free(d_mask);
        hpgq_device_free(d_trim);
        dcap = (size_t)b.num_reads + (size_t)b.num_reads / 4 + 1024;
        rc = hpgq_device_alloc(o->device, (void **)&d_mask, dcap);
        if (rc == 0) rc = hpgq_device_alloc(o->device, (void **)&d_trim, dcap * 4);
      }
      if (rc == 0) rc = hpgq_run_device(ctx, &b, NULL, need_mask ? d_mask : NULL, edit ? d_trim : NULL);
      if (rc == 0 && km) rc = hpgq_kmers_count_device(km, &b, o->filter_on ? d_mask : NULL);
      if (rc == 0 && writes) {
        s->nreads = b.num_reads;
        if (ensure_results(s, b.num_reads)) rc = HPGQ_E_NOMEM;
        if (rc == 0) rc = hpgq_copy_to_host(ctx, s->mask, d_mask, (size_t)b.num_reads);
        if (rc == 0 && edit) {
          rc = hpgq_copy_to_host(ctx, s->trim, d_trim, (size_t)b.num_reads * 4);
          if (rc == 0) rc = hpgq_copy_to_host(ctx, s->idx, b.data_indices, ((size_t)b.num_reads + 1) * 4);
        }
        if (rc == 0) rc = hpgq_parse_records(ps, s->rec_start, s->seq_start, s->plus_start, s->qual_start);
      }
      if (rc == 0) rc = hpgq_sync(ctx);
      if (rc == 0 && cg) {   /* after the parse and the mask; settled before the next parse reuses b */
        rc = hpgq_cgr_fill_device(cg, &b, o->filter_on ? d_mask : NULL,
                                  o->filter_on ? HPGQ_CGR_ONLY_VALID_READS : HPGQ_CGR_ALL_READS);
        if (rc == 0) rc = hpgq_cgr_sync(cg);
        if (rc == 0) res->cg_exact_calls += hpgq_cgr_last_exact(cg);
      }
      res->num_reads += (uint64_t)b.num_reads;
    } else if (rc == 0) {
      s->nreads = 0;
    }
    res->fastq_bytes += (double)s->use;
    pthread_mutex_lock(&P.mu);
    if (rc) P.error = rc;
    s->state = writes && rc == 0 ? 2 : 0;
    pthread_cond_broadcast(&P.cv);
    pthread_mutex_unlock(&P.mu);
    if (rc) break;
  }
  pthread_join(reader, NULL);
  if (writes) pthread_join(writer, NULL);
  if (rc == 0 && P.error) rc = P.error < 0 && P.error != HPGQ_E_FORMAT ? HPGQ_E_INVALID : P.error;
  if (rc == 0) rc = hpgq_sync(ctx);   /* surfaces HPGQ_E_READ_TOO_LONG */
  if (rc == 0) rc = hpgq_read_counters(ctx, counters, hpgq_counters_size(ctx));
  if (rc == 0 && km) {
    res->kmers_npos = p->lmax > HPGQ_KMER_K - 1 ? p->lmax - (HPGQ_KMER_K - 1) : 0;
    res->kmers = calloc(hpgq_kmers_size(km) + 1, sizeof(uint64_t));
    rc = res->kmers ? hpgq_kmers_read(km, res->kmers, hpgq_kmers_size(km)) : HPGQ_E_NOMEM;
  }
  if (rc == 0 && cg) {
    const size_t cells = (size_t)1 << (2 * o->k_cg);
    res->cg_seq = calloc(cells, sizeof(uint32_t));
    res->cg_q = calloc(cells, sizeof(uint32_t));
    rc = res->cg_seq && res->cg_q ? hpgq_cgr_read(cg, res->cg_seq, res->cg_q, &res->cg_words) : HPGQ_E_NOMEM;
  }
  res->seconds = now_s() - t0;
  if (rc == 0) {
    res->num_passed = counters[HPGQ_S_NUM_PASSED];
    res->num_failed = counters[HPGQ_S_NUM_FAILED];
    res->num_edited = counters[HPGQ_S_NUM_EDITED];
  }

done:
  if (P.out_pass) fclose(P.out_pass);
  if (P.out_fail) fclose(P.out_fail);
  hpgq_device_free(d_mask);
  hpgq_device_free(d_trim);
  for (int i = 0; i < NSLOTS; ++i) {
    hpgq_host_free(P.slot[i].buf);
    free(P.slot[i].mask);
    free(P.slot[i].trim);
    free(P.slot[i].rec_start);
    free(P.slot[i].seq_start);
    free(P.slot[i].plus_start);
    free(P.slot[i].qual_start);
    free(P.slot[i].idx);
  }
  free(P.carry);
  hpgq_parser_close(ps);
  hpgq_kmers_close(km);
  hpgq_cgr_close(cg);
  hpgq_close(ctx);
  close(P.fd);
  return rc;
}
