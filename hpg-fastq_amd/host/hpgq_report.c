/*
 * hpgq_report.c — stats report files, after src/stats_report.c.
 *
 * <in>.summary.txt (report_summary :60-153), <in>.length.histogram.data
 * (:159-180), <in>.read.quality.histogram.data (:363-390),
 * <in>.GC.histogram.data (:215-232), <in>.GC.per.nt.data (:268-285),
 * <in>.quality.per.nt.data (final form, quirk Q6: :306-322),
 * <in>.nucleotides.data (:336-352), and with --kmers <in>.kmers.txt and
 * <in>.kmers.per.nt.data (:492-530) plus the summary's k-mer list (:144-150).  Values come from the dense device
 * counters: per-position maps are read by position, not by
 * khash bucket (quirk Q3); the mean quality comes from the exact fixed-point
 * sum of per-read means, converted to float once (quirk Q2).  The arithmetic is
 * the reference's: `1.0f * a / b` and `100.0f * a / b` in float, `%i` of a
 * size_t count prints its low 32 bits; empty runs print 0 where the reference
 * divides by zero (quirk Q14).  tests/test_cli_gpu.py compares every file byte
 * for byte with oracle/report_ref.py.  The gnuplot images are not produced
 * (gnuplot is absent).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpgq_cli.h"

#define NORM_Q(q, phred) ((int)round((q) - (phred)))   /* _normalize_quality, :26 */

/* `%i` of a size_t count (src/stats_report.c:176,229,385): its low 32 bits */
static int i32(uint64_t v) { return (int)(uint32_t)v; }

/* `1.0f * a / b` (0 when b = 0, Q14) for a per-position quality sum, which is
 * signed (Q13: two's complement in the u64 counter) */
static float fdiv_q(uint64_t a, uint64_t b) { return b ? 1.0f * (int64_t)a / b : 0.0f; }

static FILE *open_out(const cli_options_t *o, const char *base, const char *suffix) {
  char path[4096];
  snprintf(path, sizeof(path), "%s/%s.%s", o->out_dirname, base, suffix);
  return fopen(path, "w");
}

/* --kmers: k-mers ordered by count, descending; ties by id (kmers_sort in the
 * absent bioinfo-libs, src/stats_fastq.c:481 -> build-defined) */
typedef struct {
  uint64_t count;
  int id;
  int size;   /* 1 + last start position with a nonzero count (counter_by_pos_size) */
} kmer_row_t;

static int kmer_cmp(const void *a, const void *b) {
  const kmer_row_t *x = a, *y = b;
  if (x->count != y->count) return x->count > y->count ? -1 : 1;
  return x->id - y->id;
}

static void kmer_string(int id, char out[HPGQ_KMER_K + 1]) {   /* kmers_string, :479 */
  for (int i = 0; i < HPGQ_KMER_K; ++i) out[i] = "ACGT"[(id >> (2 * (HPGQ_KMER_K - 1 - i))) & 3];
  out[HPGQ_KMER_K] = 0;
}

static kmer_row_t *kmer_rows(const cli_result_t *res) {
  kmer_row_t *rows = calloc(HPGQ_NUM_KMERS, sizeof(kmer_row_t));
  if (!rows) return NULL;
  for (int id = 0; id < HPGQ_NUM_KMERS; ++id) {
    const uint64_t *bp = res->kmers + (size_t)id * res->kmers_npos;
    rows[id].id = id;
    for (int j = 0; j < res->kmers_npos; ++j) {
      rows[id].count += bp[j];
      if (bp[j]) rows[id].size = j + 1;
    }
  }
  qsort(rows, HPGQ_NUM_KMERS, sizeof(kmer_row_t), kmer_cmp);
  return rows;
}

/* report_kmers, src/stats_report.c:492-530: <in>.kmers.txt (all 1024 by
 * count) and <in>.kmers.per.nt.data (the top 5 per start position; rows past a
 * k-mer's size read 0 instead of the reference's index-`size` read, quirk Q10) */
static int report_kmers(const cli_options_t *o, const char *base, const cli_result_t *res,
                        const kmer_row_t *rows) {
  char ks[HPGQ_KMER_K + 1];
  FILE *f = open_out(o, base, "kmers.txt");
  if (!f) return -1;
  fprintf(f, "# Sequence\tCount\n");
  for (int i = 0; i < HPGQ_NUM_KMERS; i++) {
    kmer_string(rows[i].id, ks);
    fprintf(f, "%s\t%lu\n", ks, (unsigned long)rows[i].count);
  }
  fclose(f);
  if (!(f = open_out(o, base, "kmers.per.nt.data"))) return -1;
  int num_cols = 0;
  for (int i = 0; i < 5; i++)
    if (num_cols < rows[i].size) num_cols = rows[i].size;
  for (int i = 0; i < num_cols; i++) {
    fprintf(f, "%i", i + 1);
    for (int t = 0; t < 5; t++) {
      const uint64_t v = i < rows[t].size ? res->kmers[(size_t)rows[t].id * res->kmers_npos + i] : 0;
      fprintf(f, "\t%lu", (unsigned long)v);
    }
    fprintf(f, "\n");
  }
  fclose(f);
  return 0;
}

/* --cg: chaos_game_calculate_table_dif / validate / write_table_images
 * (old/chaos_game.c:320-472) on the device tables: <in>_k=<k>_FG.pgm,
 * _QQ.pgm, with --gs-filename _FG_dif.pgm, and <in>.chaos_game.txt with the
 * word count, norms and the difference table's range, mean and deviation */
static int report_cg(const cli_options_t *o, const char *base, const cli_result_t *res) {
  const int k = o->k_cg;
  const size_t cells = (size_t)1 << (2 * k);
  int32_t *dif = NULL, hi = 0, lo = 0;
  uint32_t *gs = NULL, ref_words = 0;
  double mean = 0.0, sd = 0.0;
  int rc = 0;
  if (o->gs_filename) {
    gs = calloc(cells, sizeof(uint32_t));
    dif = calloc(cells, sizeof(int32_t));
    rc = gs && dif ? hpgq_cgr_load_gs(o->gs_filename, k, gs, &ref_words) : HPGQ_E_NOMEM;
    if (rc == 0) rc = hpgq_cgr_table_dif(k, res->cg_seq, res->cg_words, gs, ref_words, dif, &hi, &lo);
    if (rc == 0) rc = hpgq_cgr_dif_stats(k, dif, &mean, &sd);
  }
  FILE *f = rc == 0 ? open_out(o, base, "chaos_game.txt") : NULL;
  if (f) {
    const double mem = (double)cells;
    fprintf(f, "Chaos game (genomic signature), k = %d, %dx%d\n", k, 1 << k, 1 << k);
    fprintf(f, "Words read in FastQ file: %u\n", res->cg_words);
    if (res->cg_words) fprintf(f, "Fastq file normalization ratio = %12.6f\n", 128.0 / (res->cg_words / mem));
    if (o->gs_filename) {
      fprintf(f, "Genomic signature file: %s (%u words)\n", o->gs_filename, ref_words);
      if (ref_words) fprintf(f, "Genomic signature normalization ratio = %12.6f\n", 128.0 / (ref_words / mem));
      fprintf(f, "Interval of variation of diff matrix values = [%d, %d]\n", hi, lo);
      fprintf(f, "Diff matrix mean = %f, standard deviation = %f\n", mean, sd);
    }
    fprintf(f, "Calls redone by the exact double simulation: %d\n", res->cg_exact_calls);
    fclose(f);
  } else if (rc == 0) {
    rc = HPGQ_E_IO;
  }
  if (rc == 0 && res->cg_words)
    rc = hpgq_cgr_write_images(o->out_dirname, o->in_filename, k, res->cg_seq, res->cg_q, res->cg_words, dif);
  free(gs);
  free(dif);
  return rc;
}

int cli_report(const cli_options_t *o, const hpgq_params_t *p, const cli_result_t *res) {
  /* the full-length set: every merged read at every position (res->lmax >= --lmax) */
  const uint64_t *c = res->counters;
  const int lmax = res->lmax, phred = p->phred;
  const char *slash = strrchr(o->in_filename, '/');
  const char *base = slash ? slash + 1 : o->in_filename;
  hpgq_summary_t s;
  if (hpgq_counters_summary(c, lmax, &s)) return -1;
  const uint64_t *hl = c + hpgq_off_hist_len(lmax), *hq = c + hpgq_off_hist_meanq(lmax);
  const uint64_t *hg = c + hpgq_off_hist_gc(lmax), *pq = c + hpgq_off_pos_qsum(lmax);
  const uint64_t *pA = c + hpgq_off_pos_base(lmax, 0), *pC = c + hpgq_off_pos_base(lmax, 1);
  const uint64_t *pG = c + hpgq_off_pos_base(lmax, 2), *pT = c + hpgq_off_pos_base(lmax, 3);
  const uint64_t *pN = c + hpgq_off_pos_base(lmax, 4);
  const int maxlen = s.num_reads ? s.max_length : 0;
  /* count per position = reads longer than it */
  uint64_t *cnt = calloc((size_t)lmax + 1, sizeof(uint64_t));
  for (int j = lmax - 1; j >= 0; --j) cnt[j] = cnt[j + 1] + hl[j + 1];

  FILE *f = open_out(o, base, "summary.txt");
  if (!f) { free(cnt); return -1; }
  const uint64_t nt = s.num_A + s.num_C + s.num_G + s.num_T + s.num_N;
  fprintf(f, "-----------------------------------\n");
  fprintf(f, "      FastQ quality report\n");
  fprintf(f, "-----------------------------------\n");
  fprintf(f, "FastQ filename: %s\n\n", base);
  if (p->filter_on) {
    fprintf(f, "Filter options:\n");
    if (o->read_length_range) fprintf(f, "\tRead length range   : %s\n", o->read_length_range);
    if (o->read_quality_range) fprintf(f, "\tRead quality range  : %s\n", o->read_quality_range);
    if (p->left_length != HPGQ_MIN_VALUE && o->left_quality_range) {
      fprintf(f, "\tLeft length         : %i nucleotides\n", p->left_length);
      fprintf(f, "\tLeft quality range  : %s\n", o->left_quality_range);
    }
    if (p->right_length != HPGQ_MIN_VALUE && o->right_quality_range) {
      fprintf(f, "\tRight length        : %i nucleotides\n", p->right_length);
      fprintf(f, "\tRight quality range : %s\n", o->right_quality_range);
    }
    if (p->max_N != HPGQ_MAX_VALUE) fprintf(f, "\tMax. number of Ns   : %i\n", p->max_N);
    if (p->max_out_of_quality != HPGQ_MAX_VALUE && o->read_quality_range)
      fprintf(f, "\tMax. out of quality : %i nucletotides\n", p->max_out_of_quality);
    fprintf(f, "\n");
    const uint64_t tot = s.num_passed + s.num_failed;
    fprintf(f, "Number of reads in file  : %lu\n", (unsigned long)tot);
    fprintf(f, "Number of processed reads: %lu (%0.2f %%)\n", (unsigned long)s.num_reads,
            tot ? 100.0f * s.num_reads / tot : 0.0f);
  } else {
    fprintf(f, "Filter         : Disabled\n");
    fprintf(f, "Number of reads: %lu\n", (unsigned long)s.num_reads);
  }
  fprintf(f, "\n");
  fprintf(f, "Read length (min., mean, max.): (%i, %0.2f, %i)\n", s.num_reads ? s.min_length : 0,
          s.num_reads ? 1.0f * s.acc_length / s.num_reads : 0.0f, maxlen);
  fprintf(f, "\n");
  /* acc_quality (float in the reference, :297): the exact sum of per-read raw
   * means (fixed point, two's complement), converted to float once (Q2) */
  const float acc_q = (float)((double)(int64_t)c[HPGQ_S_ACC_MEANQ_FX16] / 65536.0);
  int qual = NORM_Q(s.num_reads ? 1.0f * acc_q / s.num_reads : 0.0f, phred);
  fprintf(f, "Mean quality = %i [%c]\n", qual, qual + phred);
  fprintf(f, "\n");
  fprintf(f, "Nucleotide content (A, C, G, T, N)\n");
  fprintf(f, "\tA: %0.2f %%\n", nt ? 100.0f * s.num_A / nt : 0.0f);
  fprintf(f, "\tT: %0.2f %%\n", nt ? 100.0f * s.num_T / nt : 0.0f);
  fprintf(f, "\tG: %0.2f %%\n", nt ? 100.0f * s.num_G / nt : 0.0f);
  fprintf(f, "\tC: %0.2f %%\n", nt ? 100.0f * s.num_C / nt : 0.0f);
  fprintf(f, "\tN: %0.2f %%\n", nt ? 100.0f * s.num_N / nt : 0.0f);
  fprintf(f, "GC content\n");
  fprintf(f, "\tCG: %0.2f %%\n", nt ? 100.0f * (s.num_G + s.num_C) / nt : 0.0f);
  fprintf(f, "\n");
  fprintf(f, "Mean quality per nucleotide position\n");
  for (int k = 0; k < maxlen; k++) {
    qual = NORM_Q(fdiv_q(pq[k], cnt[k]), phred);
    fprintf(f, "\tpos. %i: %i [%c]\t", k + 1, qual, qual + phred);
    if ((k + 1) % 5 == 0) fprintf(f, "\n");
  }
  fprintf(f, "\n");
  kmer_row_t *krows = res && res->kmers ? kmer_rows(res) : NULL;
  if (krows) {   /* :144-150 (21 rows there; the header's 20 here, quirk Q10) */
    char ks[HPGQ_KMER_K + 1];
    fprintf(f, "K-mers (top 20)\n");
    fprintf(f, "\tSequence\tCount\n");
    for (int i = 0; i < 20; i++) {
      kmer_string(krows[i].id, ks);
      fprintf(f, "\t%s\t\t%lu\n", ks, (unsigned long)krows[i].count);
    }
  }
  fclose(f);
  if (krows && report_kmers(o, base, res, krows)) {
    free(krows);
    free(cnt);
    return -1;
  }
  free(krows);
  if (res && res->cg_seq && report_cg(o, base, res)) {
    free(cnt);
    return -1;
  }

  if ((f = open_out(o, base, "length.histogram.data"))) {
    for (int i = 1; i <= maxlen; i++) fprintf(f, "%i\t%i\n", i, i32(hl[i]));
    fclose(f);
  }
  if ((f = open_out(o, base, "read.quality.histogram.data"))) {
    /* keys are signed (bin = key & 255, Q13); rows min_qual..max_qual as
       src/stats_report.c:410-425, whose max_qual starts at 0: with every key
       negative the rows still run up to key 0 (the reference then reads its
       array at negative indices; here those rows print the negative keys'
       own bins) */
    int lo = 1000, hi = 0;
    for (int i = 0; i < HPGQ_MEANQ_BINS; i++)
      if (hq[i]) {
        const int key = i >= 128 ? i - 256 : i;
        if (key < lo) lo = key;
        if (key > hi) hi = key;
      }
    for (int key = lo; key <= hi; key++) fprintf(f, "%i\t%i\n", key - phred, i32(hq[key & 255]));
    fclose(f);
  }
  if ((f = open_out(o, base, "GC.histogram.data"))) {
    for (int i = 1; i < 100; i++)
      if (hg[i]) fprintf(f, "%i\t%i\n", i, i32(hg[i]));
    fclose(f);
  }
  if ((f = open_out(o, base, "GC.per.nt.data"))) {
    for (int k = 0; k < maxlen; k++) {
      const uint64_t t = pA[k] + pC[k] + pG[k] + pT[k] + pN[k];
      const float v = t ? 100.0f * (pG[k] + pC[k]) / t : 0.0f;
      if (v > 1.0f) fprintf(f, "%i\t%0.2f\n", k + 1, v);
    }
    fclose(f);
  }
  if ((f = open_out(o, base, "quality.per.nt.data"))) {
    for (int k = 0; k < maxlen; k++)
      fprintf(f, "%i\t%i\n", k, NORM_Q(fdiv_q(pq[k], cnt[k]), phred));
    fclose(f);
  }
  if ((f = open_out(o, base, "nucleotides.data"))) {
    for (int k = 0; k < maxlen; k++) {
      const uint64_t t = pA[k] + pC[k] + pG[k] + pT[k] + pN[k];
#define PCT(x) (t ? 100.0f * (x) / t : 0.0f)
      fprintf(f, "%i\t%0.2f\t%0.2f\t%0.2f\t%0.2f\t%0.2f\n", k + 1, PCT(pA[k]), PCT(pT[k]), PCT(pG[k]),
              PCT(pC[k]), PCT(pN[k]));
#undef PCT
    }
    fclose(f);
  }
  free(cnt);
  return 0;
}
