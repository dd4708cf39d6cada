/*
 * hpgq_oracle.c — CPU restatement of hpg-fastq's per-read QC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * engine in hpg-fastq_amd/ and the timed CPU baseline of bench.py
 * (cpu_baseline.kind = "port").  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * PARITY STATUS:
 *   - stats merge (A4): restates the consumer merge of the reference,
 *     src/stats_fastq.c:257-417, over dense u64 counters.
 *   - filter (A5), per-read stats (A3), edit/trim (A6): the reference calls
 *     fastq_filter / fastq_reads_stats / fastq_edit from the bioinfo-libs
 *     submodule, which is EMPTY in /root/reference (.gitmodules:1-6; pinned
 *     version unknown).  These follow the written spec in DESIGN.md §3,
 *     derived from the call sites and help texts cited inline.
 *     -> "parity unpinned": the reference holds no tests, fixtures or golden
 *        vectors for this path, and its CPU path cannot be built here.
 *   - --kmers (§8f rank 2): build-defined 5-mer counts;
 *     the per-read k-mer code is in the same absent bioinfo-libs -> unpinned.
 *   - CGR (A7): line-by-line restatement of chaos_game_fill_tables,
 *     old/chaos_game.c:165-267.  The reference file needs an absent header
 *     (qc_batch.h) so it is not built here -> also "parity unpinned".
 *   Every restated rule is cross-checked against an independent pure-Python
 *   restatement (oracle/pyref.py) on the hand-written fixtures in
 *   tests/golden/.
 *
 * Build: make -C oracle  ->  oracle/liboracle.so (gcc -O3 -fopenmp).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "../include/hpgq.h"

/* ------------------------------------------------------------------ */
/* synthetic generator (restated independently of the product copy;   */
/* SURVEY §8d input description)                                      */
/* ------------------------------------------------------------------ */

static inline uint64_t o_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static inline uint64_t o_read_key(const hpgq_synth_t *s, int64_t idx) {
  return o_mix64(s->seed * 0x9E3779B97F4A7C15ULL + (uint64_t)idx);
}

int32_t oracle_synth_length(const hpgq_synth_t *s, int64_t idx) {
  uint64_t r = o_read_key(s, idx);
  int32_t L = s->read_length;
  if (L >= 20 && (int32_t)(r % 100) < s->trunc_pct)
    L = 20 + (int32_t)(o_mix64(r ^ 1ULL) % (uint64_t)(s->read_length - 20 + 1));
  return L;
}

/* fills reads [first, first+n); idx gets n+1 offsets starting at 0 */
void oracle_synth(const hpgq_synth_t *s, int64_t first, int64_t n,
                  char *seq, char *qual, int32_t *idx) {
  static const char acgt[4] = {'A', 'C', 'G', 'T'};
  idx[0] = 0;
  for (int64_t i = 0; i < n; i++) idx[i + 1] = idx[i] + oracle_synth_length(s, first + i);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) {
    uint64_t r = o_read_key(s, first + i);
    uint64_t mk = s->mate ? o_mix64(r ^ 0x5EEDULL) : r;
    int bad = (int32_t)((mk >> 20) % 100) < s->bad_pct;
    int32_t L = idx[i + 1] - idx[i];
    for (int32_t j = 0; j < L; j++) {
      uint64_t h = o_mix64(mk + (uint64_t)(j + 1) * 0xD1B54A32D192ED03ULL);
      char b = ((int32_t)(h & 1023) < s->n_per_1024) ? 'N' : acgt[(h >> 10) & 3];
      int32_t noise = (int32_t)((h >> 12) % 13) - 6;
      int32_t q = bad ? 12 + noise : 40 - (20 * j) / L + noise;
      if (q < 2) q = 2;
      if (q > 41) q = 41;
      seq[idx[i] + j] = b;
      qual[idx[i] + j] = (char)(q + s->phred);
    }
  }
}

/* ------------------------------------------------------------------ */
/* per-read arithmetic                                                */
/* ------------------------------------------------------------------ */

/* A quality byte as the reference's `char`, signed on x86-64 gcc: the merge
 * adds fq_read->quality[j] into an int (src/stats_fastq.c:353-355), and the
 * CGR accumulator adds quality[qpos] the same way (old/chaos_game.c:253-259).
 * Every quality rule below (filter sums, trims, out-of-range counts, the
 * per-read mean) uses this value: DESIGN.md §2.3, quirk Q13. */
static inline int32_t o_q(unsigned char c) { return (int32_t)(signed char)c; }

/* floor(a / b) for b > 0 (C division truncates towards zero) */
static inline int64_t o_floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}

typedef struct {
  int32_t ts, te;     /* trim start / end (A6) */
  int     pass;
} o_read_result_t;

/* mean-Q window check: min*k <= sum(Q) <= max*k, exact integers
 * (equals min <= sum/k <= max for the float mean the help text implies,
 *  src/stats_options.c:276,278,280) */
static inline int o_mean_in(int64_t sumq, int64_t k, int64_t lo, int64_t hi) {
  return lo * k <= sumq && sumq <= hi * k;
}

/*
 * fastq_edit (A6), build-defined: within the first left_len bases drop the
 * leading run with Q outside [minL,maxL]; within the last right_len bases of
 * what is left drop the trailing run with Q outside [minR,maxR]
 * (src/edit_options.c:280-283 "leftmost nucleotides to take into account to
 *  trim"; old/README:48-49,81-82 "trim of the first or last nucleotides if
 *  the selected criteria is not accomplished").
 */
static void o_trim(const hpgq_params_t *p, const unsigned char *q, int32_t n,
                   int32_t *ts_out, int32_t *te_out) {
  int32_t ts = 0, te = 0;
  if (p->edit_left_length > 0) {
    int32_t lim = p->edit_left_length < n ? p->edit_left_length : n;
    while (ts < lim) {
      int32_t Q = o_q(q[ts]) - p->phred;
      if (Q >= p->edit_min_left_quality && Q <= p->edit_max_left_quality) break;
      ts++;
    }
  }
  if (p->edit_right_length > 0) {
    int32_t rem = n - ts;
    int32_t lim = p->edit_right_length < rem ? p->edit_right_length : rem;
    while (te < lim) {
      int32_t Q = o_q(q[n - 1 - te]) - p->phred;
      if (Q >= p->edit_min_right_quality && Q <= p->edit_max_right_quality) break;
      te++;
    }
  }
  *ts_out = ts;
  *te_out = te;
}

/*
 * fastq_filter (A5), build-defined from fastq_filter_options_new's 12
 * arguments (src/filter_fastq.c:140-145) and the option help texts
 * (src/stats_options.c:275-282).  Thresholds are Phred (Q = char - phred).
 */
static int o_filter(const hpgq_params_t *p, const unsigned char *s,
                    const unsigned char *q, int32_t n) {
  if (n < p->min_read_length || n > p->max_read_length) return 0;
  int64_t sumq = 0, nN = 0, oor = 0;
  for (int32_t j = 0; j < n; j++) {
    int32_t Q = o_q(q[j]) - p->phred;
    sumq += Q;
    if (s[j] == 'N') nN++;
    if (Q < p->min_read_quality || Q > p->max_read_quality) oor++;
  }
  if (nN > p->max_N) return 0;
  if (!o_mean_in(sumq, n, p->min_read_quality, p->max_read_quality)) return 0;
  if (oor > p->max_out_of_quality) return 0;
  if (p->left_length > 0) {
    int32_t k = p->left_length < n ? p->left_length : n;
    int64_t sl = 0;
    for (int32_t j = 0; j < k; j++) sl += o_q(q[j]) - p->phred;
    if (k > 0 && !o_mean_in(sl, k, p->min_left_quality, p->max_left_quality)) return 0;
  }
  if (p->right_length > 0) {
    int32_t k = p->right_length < n ? p->right_length : n;
    int64_t sr = 0;
    for (int32_t j = n - k; j < n; j++) sr += o_q(q[j]) - p->phred;
    if (k > 0 && !o_mean_in(sr, k, p->min_right_quality, p->max_right_quality)) return 0;
  }
  return 1;
}

/*
 * Per-read stats + the consumer merge (A3 + A4), src/stats_fastq.c:283-382:
 *   length histogram             :306-314 (key = read_length)
 *   quality histogram            :316-324 (key = round(quality_average), raw units;
 *                                 C round(): halves away from zero; bin = key & 255)
 *   GC histogram                 :326-334 (key = 100*(G+C)/read_length, integer division)
 *   per position j < read_length :338-382 (quality[j] raw, signed char :353-355;
 *                                 A/T/C/G/N exact uppercase)
 *   acc_quality (float, :297)    -> exact fixed point sum, HPGQ_S_ACC_MEANQ_FX16 =
 *                                 sum of floor(65536*S/n), two's complement
 * len 0 reads get no quality/GC bin (quirk Q8: the reference divides by zero).
 * The reference has no length cap (khash keyed by j < read_length).  This
 * dense set holds lengths <= lmax and positions < lmax: a read longer than
 * lmax counts in HPGQ_S_LONG_READS and merges everything but its length and
 * its positions >= lmax (what the engine keeps in its long-read tail; an lmax
 * of at least the longest read gives the full set, hpgq_read_counters_ext).
 */
static void o_merge(uint64_t *c, int lmax, const unsigned char *s,
                    const unsigned char *q, int32_t n) {
  c[HPGQ_S_NUM_STATS]++;
  if (n > lmax) c[HPGQ_S_LONG_READS]++;
  else c[hpgq_off_hist_len(lmax) + n]++;
  int64_t sraw = 0;
  uint64_t gc = 0;
  uint64_t *pq = c + hpgq_off_pos_qsum(lmax);
  for (int32_t j = 0; j < n; j++) {
    sraw += o_q(q[j]);
    if (s[j] == 'C' || s[j] == 'G') gc++;
    if (j >= lmax) continue;
    pq[j] += (uint64_t)(int64_t)o_q(q[j]);   /* u64 wrap = the int sum's two's complement */
    int b = -1;
    switch (s[j]) {
      case 'A': b = HPGQ_BASE_A; break;
      case 'C': b = HPGQ_BASE_C; break;
      case 'G': b = HPGQ_BASE_G; break;
      case 'T': b = HPGQ_BASE_T; break;
      case 'N': b = HPGQ_BASE_N; break;
      default: break;
    }
    if (b >= 0) c[hpgq_off_pos_base(lmax, b) + j]++;
  }
  if (n > 0) {
    int64_t key = sraw >= 0 ? (2 * sraw + n) / (2 * (int64_t)n)            /* round(sraw/n) */
                            : -((-2 * sraw + n) / (2 * (int64_t)n));
    c[hpgq_off_hist_meanq(lmax) + ((uint64_t)key & 255u)]++;
    c[hpgq_off_hist_gc(lmax) + (100 * gc) / (uint64_t)n]++;
    c[HPGQ_S_ACC_MEANQ_FX16] += (uint64_t)o_floor_div(sraw * 65536, n);
  }
}

static void o_read_eval(const hpgq_params_t *p, const hpgq_batch_t *b, int64_t i,
                        o_read_result_t *r) {
  int32_t a = b->data_indices[i], e = b->data_indices[i + 1];
  int32_t n = e - a;
  const unsigned char *q = (const unsigned char *)b->quality + a;
  const unsigned char *s = (const unsigned char *)b->seq + a;
  r->ts = r->te = 0;
  if (p->edit_on) o_trim(p, q, n, &r->ts, &r->te);
  int32_t m = n - r->ts - r->te;
  r->pass = p->filter_on ? o_filter(p, s + r->ts, q + r->ts, m) : 1;
}

static void o_account(const hpgq_params_t *p, const hpgq_batch_t *b, int64_t i,
                      const o_read_result_t *r, int pass, uint64_t *c) {
  int32_t a = b->data_indices[i], e = b->data_indices[i + 1];
  int32_t n = e - a;
  c[HPGQ_S_NUM_INPUT]++;
  if (pass) c[HPGQ_S_NUM_PASSED]++; else c[HPGQ_S_NUM_FAILED]++;
  if (r->ts + r->te > 0) c[HPGQ_S_NUM_EDITED]++;
  if (p->stats_on && pass)
    o_merge(c, p->lmax, (const unsigned char *)b->seq + a + r->ts,
            (const unsigned char *)b->quality + a + r->ts, n - r->ts - r->te);
}

/*
 * One engine call: edit -> filter -> stats over a host batch (and its mate
 * batch when p->paired).  counters: hpgq_counters_len(lmax) u64 per set
 * (2 sets when paired), ACCUMULATED into.  nthreads <= 0: OpenMP default.
 */
int oracle_run(const hpgq_params_t *p, const hpgq_batch_t *b, const hpgq_batch_t *b2,
               uint8_t *mask, uint32_t *trim, uint64_t *counters, int nthreads) {
  int lmax = p->lmax;
  size_t clen = hpgq_counters_len(lmax);
  int nsets = p->paired ? 2 : 1;
  if (p->paired && (!b2 || b2->num_reads != b->num_reads)) return HPGQ_E_INVALID;
  int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
  uint64_t *part = (uint64_t *)calloc((size_t)nt * nsets * clen, sizeof(uint64_t));
  if (!part) return HPGQ_E_NOMEM;
  int64_t nr = b->num_reads;
#pragma omp parallel num_threads(nt)
  {
    int t = omp_get_thread_num();
    uint64_t *c0 = part + (size_t)t * nsets * clen;
    uint64_t *c1 = c0 + clen;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < nr; i++) {
      o_read_result_t r1, r2;
      o_read_eval(p, b, i, &r1);
      int pass = r1.pass;
      if (p->paired) {
        o_read_eval(p, b2, i, &r2);
        pass = pass && r2.pass;   /* pair-consistent filter */
      }
      if (mask) mask[i] = (uint8_t)pass;
      if (trim) {
        trim[i] = (uint32_t)r1.ts | ((uint32_t)r1.te << 16);
        if (p->paired) trim[nr + i] = (uint32_t)r2.ts | ((uint32_t)r2.te << 16);
      }
      o_account(p, b, i, &r1, pass, c0);
      if (p->paired) o_account(p, b2, i, &r2, pass, c1);
    }
  }
  for (int t = 0; t < nt; t++) {
    const uint64_t *src = part + (size_t)t * nsets * clen;
    for (size_t k = 0; k < nsets * clen; k++) counters[k] += src[k];
  }
  free(part);
  return HPGQ_OK;
}

/* ------------------------------------------------------------------ */
/* chaos game: chaos_game_fill_tables, old/chaos_game.c:165-267       */
/* ------------------------------------------------------------------ */

#define O_EPSILON 0.00001          /* old/chaos_game.h:41 */

/*
 * One call = one batch.  f starts at dim/2 (:107-108 read back at :180-181;
 * the function never stores f back, so every call restarts there) and is
 * carried across the reads of the batch; the word counter and quality
 * accumulator reset per read (:263-264).  table_seq/table_q are dim*dim u32
 * row-major [co_x][co_y] and are accumulated into; *word_count is
 * fq_word_count (u32, wraps).
 */
int oracle_cgr_fill(int k, int base_quality, const hpgq_batch_t *b, const uint8_t *status,
                    int mode, uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count) {
  if (k < 1 || k > 12) return HPGQ_E_INVALID;
  int dim_n = 1 << k;
  int word_size = k;
  int word_quality_substract = base_quality * word_size;     /* :185 */
  int nt_word_count = 0;
  unsigned int acc_word_quality = 0;
  double f_x = (double)(dim_n * 0.5), f_y = f_x;            /* :107-108 */
  const char *seq = b->seq, *quality = b->quality;
  for (int64_t i = 0; i < b->num_reads; i++) {
    if (mode == HPGQ_CGR_ONLY_VALID_READS && (!status || status[i] != 1)) continue;  /* :188 */
    int read_position = b->data_indices[i];
    int read_length = b->data_indices[i + 1] - b->data_indices[i];
    int quality_position = read_position;
    for (int j = 0; j < read_length; j++) {
      char quality_character = quality[quality_position++];
      switch (seq[read_position++]) {
        case 65:   /* A :201-207 */
          f_x = f_x + ((dim_n - f_x) * 0.5);
          f_y = f_y * 0.5;
          nt_word_count++;
          acc_word_quality += quality_character;
          break;
        case 67:   /* C :208-214 */
          f_x = f_x * 0.5;
          f_y = f_y * 0.5;
          nt_word_count++;
          acc_word_quality += quality_character;
          break;
        case 71:   /* G :215-221 */
          f_x = f_x * 0.5;
          f_y = f_y + ((dim_n - f_y) * 0.5);
          nt_word_count++;
          acc_word_quality += quality_character;
          break;
        case 84:   /* T :222-228 */
          f_x = f_x + ((dim_n - f_x) * 0.5);
          f_y = f_y + ((dim_n - f_y) * 0.5);
          nt_word_count++;
          acc_word_quality += quality_character;
          break;
        case 78:   /* N :229-233 */
          nt_word_count = 0;
          acc_word_quality = 0;
          break;
        default:
          break;
      }
      if (nt_word_count == word_size) {                       /* :236-260 */
        int co_x = (int)f_x;
        int co_y = (int)f_y;
        if (co_x == dim_n) { co_x = dim_n - 1; f_x = f_x - O_EPSILON; }
        if (co_y == dim_n) { co_y = dim_n - 1; f_y = f_y - O_EPSILON; }
        table_seq[(size_t)co_x * dim_n + co_y]++;
        (*word_count)++;
        nt_word_count--;
        table_q[(size_t)co_x * dim_n + co_y] += (acc_word_quality - word_quality_substract);
        acc_word_quality = acc_word_quality - quality[quality_position - word_size];
      }
    }
    nt_word_count = 0;                                          /* :263-264 */
    acc_word_quality = 0;
  }
  return HPGQ_OK;
}

/* independent batches (each its own fill call) in parallel: the CPU baseline
 * for config C5 (state resets per call, so batches are independent). */
/* nb independent fill calls spread over nthreads (bench.py's CPU baseline);
 * status (may be NULL): one read_status[] per call, with mode as in
 * oracle_cgr_fill */
int oracle_cgr_fill_batches(int k, int base_quality, const hpgq_batch_t *bs, const uint8_t *const *status,
                            int mode, int nb, uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count,
                            int nthreads) {
  int dim = 1 << k;
  size_t cells = (size_t)dim * dim;
  int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
  uint32_t *ts = (uint32_t *)calloc((size_t)nt * cells * 2, sizeof(uint32_t));
  uint32_t *wc = (uint32_t *)calloc((size_t)nt, sizeof(uint32_t));
  if (!ts || !wc) { free(ts); free(wc); return HPGQ_E_NOMEM; }
  int err = 0;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
  for (int i = 0; i < nb; i++) {
    int t = omp_get_thread_num();
    int e = oracle_cgr_fill(k, base_quality, &bs[i], status ? status[i] : NULL, mode,
                            ts + (size_t)t * cells * 2, ts + (size_t)t * cells * 2 + cells, wc + t);
    if (e) err = e;
  }
  for (int t = 0; t < nt; t++) {
    for (size_t c = 0; c < cells; c++) {
      table_seq[c] += ts[(size_t)t * cells * 2 + c];
      table_q[c] += ts[(size_t)t * cells * 2 + cells + c];
    }
    *word_count += wc[t];
  }
  free(ts);
  free(wc);
  return err;
}

/* ------------------------------------------------------------------ */
/* stats --kmers: build-defined 5-mer counts (the      */
/* per-read kmers of fastq_reads_stats are in the absent bioinfo-libs, */
/* merged at src/stats_fastq.c:384-410) -> parity unpinned             */
/* ------------------------------------------------------------------ */

static inline int o_kcode(unsigned char c) {
  switch (c) {   /* exact uppercase only, like the per-position counts (:360-372) */
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
  }
}

/* by_pos[HPGQ_NUM_KMERS][lmax-4] += counts of b's reads with mask[i] == 1
 * (all reads when mask is NULL); starts p >= lmax-4 are left out (an lmax of
 * at least the longest read gives them all, hpgq_kmers_read_ext) */
int oracle_kmers(const hpgq_batch_t *b, const uint8_t *mask, int lmax, uint64_t *by_pos) {
  const int npos = lmax > HPGQ_KMER_K - 1 ? lmax - (HPGQ_KMER_K - 1) : 0;
  if (!b || b->num_reads < 0 || lmax < 1) return HPGQ_E_INVALID;
  for (int64_t r = 0; r < b->num_reads; ++r) {
    if (mask && mask[r] != 1) continue;
    const int32_t a = b->data_indices[r], n = b->data_indices[r + 1] - a;
    const unsigned char *s = (const unsigned char *)b->seq + a;
    for (int p = 0; p + HPGQ_KMER_K <= n && p < npos; ++p) {
      int id = 0, ok = 1;
      for (int i = 0; i < HPGQ_KMER_K; ++i) {
        const int c = o_kcode(s[p + i]);
        if (c < 0) ok = 0;
        id = id * 4 + (c < 0 ? 0 : c);
      }
      if (ok) by_pos[(size_t)id * npos + p]++;
    }
  }
  return HPGQ_OK;
}

int oracle_max_threads(void) { return omp_get_max_threads(); }
