/*
 * oracle_main.c — exercises the CPU oracle (oracle/hpgq_oracle.c) on edge
 * cases under ASan/UBSan (tests/sanitize/Makefile): empty and length-0 reads,
 * reads longer than lmax, quality bytes >= 128, non-ACGTN bytes, paired-end,
 * every filter knob, edit windows longer than the reads, and the chaos-game
 * accumulator on homopolymer runs, k = 1..12.  Exit status 0 = every call
 * returned 0 (the sanitizers abort on any memory or UB error).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hpgq.h"

int oracle_run(const hpgq_params_t *p, const hpgq_batch_t *b, const hpgq_batch_t *b2, uint8_t *mask,
               uint32_t *trim, uint64_t *counters, int nthreads);
int oracle_cgr_fill(int k, int base_quality, const hpgq_batch_t *b, const uint8_t *status, int mode,
                    uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count);
void oracle_synth(const hpgq_synth_t *s, int64_t first, int64_t n, char *seq, char *qual, int32_t *idx);

static uint64_t rng = 88172645463325252ull;
static uint32_t next(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}

/* n reads of random lengths 0..maxlen with a mix of bytes */
static void make(int n, int maxlen, char **seq, char **qual, int32_t **idx) {
  *idx = malloc(sizeof(int32_t) * (n + 1));
  (*idx)[0] = 0;
  for (int i = 0; i < n; ++i) (*idx)[i + 1] = (*idx)[i] + (int32_t)(next() % (uint32_t)(maxlen + 1));
  const int tot = (*idx)[n];
  *seq = malloc(tot + 1);
  *qual = malloc(tot + 1);
  static const char bases[] = "ACGTNacgtRY";
  for (int j = 0; j < tot; ++j) {
    const uint32_t r = next();
    (*seq)[j] = (r & 7) < 6 ? "AAAAACGT"[r % 8] : bases[r % 11];
    (*qual)[j] = (char)((r >> 8) % 7 == 0 ? 128 + (r >> 16) % 128 : 33 + (r >> 16) % 45);
  }
}

int main(void) {
  int fails = 0;
  const int n = 3000;
  char *s1, *q1, *s2, *q2;
  int32_t *i1, *i2;
  make(n, 400, &s1, &q1, &i1);
  make(n, 400, &s2, &q2, &i2);
  hpgq_batch_t b1 = {n, s1, q1, i1}, b2 = {n, s2, q2, i2}, b0 = {0, s1, q1, i1};
  uint8_t *mask = malloc(n);
  uint32_t *trim = malloc(2 * sizeof(uint32_t) * n);
  for (int variant = 0; variant < 6; ++variant) {
    hpgq_params_t p;
    hpgq_params_init(&p);
    p.lmax = variant % 2 ? 150 : 1024;
    p.filter_on = variant >= 1;
    if (variant >= 1) {
      p.min_read_length = 10; p.max_read_length = 350;
      p.min_read_quality = 15; p.max_read_quality = 60;
      p.max_N = 4; p.max_out_of_quality = 30;
      p.left_length = 12; p.min_left_quality = 10;
      p.right_length = 500; p.max_right_quality = 50;
    }
    if (variant >= 3) {
      p.edit_on = 1;
      p.edit_left_length = 20; p.edit_min_left_quality = 20;
      p.edit_right_length = 600; p.edit_min_right_quality = 25;
      p.left_length = p.right_length = 0;
    }
    p.paired = variant == 5;
    const size_t clen = hpgq_counters_len(p.lmax) * (p.paired ? 2 : 1);
    uint64_t *ctr = calloc(clen, sizeof(uint64_t));
    fails += oracle_run(&p, &b1, p.paired ? &b2 : NULL, mask, trim, ctr, 2) != 0;
    fails += oracle_run(&p, &b0, NULL, mask, trim, ctr, 1) != 0 && !p.paired;
    free(ctr);
  }
  /* chaos game: random batch, then homopolymer runs, every k */
  for (int k = 1; k <= 12; ++k) {
    const size_t cells = (size_t)1 << (2 * k);
    uint32_t *ts = calloc(cells, 4), *tq = calloc(cells, 4), wc = 0;
    fails += oracle_cgr_fill(k, 33, &b1, NULL, HPGQ_CGR_ALL_READS, ts, tq, &wc) != 0;
    uint8_t *st = malloc(n);
    for (int i = 0; i < n; ++i) st[i] = (uint8_t)(next() & 1);
    fails += oracle_cgr_fill(k, 33, &b1, st, HPGQ_CGR_ONLY_VALID_READS, ts, tq, &wc) != 0;
    free(st);
    free(ts);
    free(tq);
  }
  {
    const int hn = 200, L = 300;
    char *hs = malloc(hn * L), *hq = malloc(hn * L);
    int32_t *hi = malloc(sizeof(int32_t) * (hn + 1));
    for (int i = 0; i <= hn; ++i) hi[i] = i * L;
    for (int j = 0; j < hn * L; ++j) {
      hs[j] = (j / L) % 2 ? 'T' : 'A';
      hq[j] = 'I';
    }
    hpgq_batch_t hb = {hn, hs, hq, hi};
    uint32_t *ts = calloc(1 << 14, 4), *tq = calloc(1 << 14, 4), wc = 0;
    fails += oracle_cgr_fill(7, 33, &hb, NULL, HPGQ_CGR_ALL_READS, ts, tq, &wc) != 0;
    free(ts); free(tq); free(hs); free(hq); free(hi);
  }
  {  /* the synthetic generator */
    hpgq_synth_t sy = {2, 150, 5, 5, 1, 33, 0};
    char *ss = malloc(150 * 1000), *sq = malloc(150 * 1000);
    int32_t *si = malloc(sizeof(int32_t) * 1001);
    oracle_synth(&sy, 12345, 1000, ss, sq, si);
    free(ss); free(sq); free(si);
  }
  free(mask); free(trim); free(s1); free(q1); free(i1); free(s2); free(q2); free(i2);
  printf("oracle_main: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
