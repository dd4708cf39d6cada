/*
 * report_main.c — drives the C host's report writer (hpg-fastq_amd/host/
 * hpgq_report.c) and option parser (hpgq_options.c) without a GPU, for the
 * ASan/UBSan build of the host code (tests/sanitize/Makefile) and the CPU
 * byte-parity test against oracle/report_ref.py (tests/test_sanitize_cpu.py).
 *
 *   report_main <counters.bin> <lmax> stats -f <in.fq> -o <outdir> [stats flags]
 *
 * counters.bin: one raw u64 counter set (hpg-fastq --counters-out layout).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpgq_cli.h"

int main(int argc, char **argv) {
  if (argc < 4 || strcmp(argv[3], "stats") != 0) {
    fprintf(stderr, "usage: %s <counters.bin> <lmax> stats -f <in.fq> -o <outdir> [flags]\n", argv[0]);
    return 2;
  }
  const int lmax = atoi(argv[2]);
  cli_options_t *o = cli_parse(CMD_STATS, "hpg-fastq", argc - 3, argv + 3);
  hpgq_params_t p;
  cli_params(o, &p);
  p.lmax = lmax;
  const size_t clen = hpgq_counters_len(lmax);
  uint64_t *c = calloc(clen, sizeof(uint64_t));
  FILE *f = fopen(argv[1], "rb");
  if (!c || !f || fread(c, sizeof(uint64_t), clen, f) != clen) {
    fprintf(stderr, "report_main: cannot read %zu counters from %s\n", clen, argv[1]);
    return 2;
  }
  fclose(f);
  cli_result_t res;
  memset(&res, 0, sizeof(res));
  res.counters = c;   /* (the layout of lmax: what the CLI's full-length merge hands over) */
  res.lmax = lmax;
  const int rc = cli_report(o, &p, &res);
  free(c);
  cli_free(o);
  return rc ? 1 : 0;
}
