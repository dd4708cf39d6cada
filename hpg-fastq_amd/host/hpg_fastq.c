/*
 * hpg_fastq.c — `hpg-fastq stats | filter | edit` on MI355X (libhpgq).
 *
 * Command dispatch and result printing after src/hpg-fastq.c and the
 * stats_fastq / filter_fastq / edit_fastq drivers (src/stats_fastq.c:424-500,
 * src/filter_fastq.c:180-250, src/edit_fastq.c:236-300).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpgq_cli.h"

static void usage(const char *exec_name) {
  printf("Program: %s (High-performance tools for handling FastQ files, MI355X build)\n", exec_name);
  printf("Version: 1.0.0 (%s)\n", hpgq_version());
  printf("\n");
  printf("Usage: %s <command> [options]\n", exec_name);
  printf("\n");
  printf("Command: stats\t\tstatistics summary\n");
  printf("         filter\t\tfilter a FastQ file by using advanced criteria\n");
  printf("         edit\t\tedit a FastQ file according the specified options\n");
  printf("\n");
  printf("For more information about a certain command, type %s <command> --help\n", exec_name);
  exit(-1);
}

int main(int argc, char **argv) {
  const char *exec_name = argv[0];
  if (argc == 1 || !strcmp(argv[1], "-h") || !strcmp(argv[1], "--help")) usage(exec_name);
  int cmd;
  if (!strcmp(argv[1], "stats")) cmd = CMD_STATS;
  else if (!strcmp(argv[1], "filter")) cmd = CMD_FILTER;
  else if (!strcmp(argv[1], "edit")) cmd = CMD_EDIT;
  else usage(exec_name);
  cli_options_t *o = cli_parse(cmd, exec_name, argc - 1, argv + 1);
  hpgq_params_t p;
  cli_params(o, &p);
  if (o->print_params) {
    cli_print_params(&p);
    cli_free(o);
    return 0;
  }
  if (!o->quiet) cli_display(o);

  cli_result_t r;
  int rc = cli_run(o, &p, &r);
  if (rc) {
    fprintf(stderr, "\nError: %s (%d)\n", hpgq_strerror(rc), rc);
    free(r.counters);
    cli_free(o);
    return 1;
  }
  /* (the full-length set: layout of r.lmax = max(--lmax, longest merged read)) */
  const uint64_t *counters = r.counters;
  const size_t clen = hpgq_counters_len(r.lmax) * (p.paired ? 2 : 1);
  if (o->counters_out) {
    FILE *f = fopen(o->counters_out, "wb");
    if (!f || fwrite(counters, sizeof(uint64_t), clen, f) != clen) rc = 1;
    if (f) fclose(f);
  }
  if (o->kmers_out && r.kmers) {
    const size_t kn = (size_t)HPGQ_NUM_KMERS * (size_t)r.kmers_npos;
    FILE *f = fopen(o->kmers_out, "wb");
    if (!f || fwrite(r.kmers, sizeof(uint64_t), kn, f) != kn) rc = 1;
    if (f) fclose(f);
  }
  if (o->cg_out && r.cg_seq) {   /* [table_seq | table_q | word count] u32 */
    const size_t cells = (size_t)1 << (2 * o->k_cg);
    FILE *f = fopen(o->cg_out, "wb");
    if (!f || fwrite(r.cg_seq, 4, cells, f) != cells || fwrite(r.cg_q, 4, cells, f) != cells ||
        fwrite(&r.cg_words, 4, 1, f) != 1)
      rc = 1;
    if (f) fclose(f);
  }
  if (cmd == CMD_STATS && cli_report(o, &p, &r)) rc = 1;

  if (!o->quiet) {
    printf("\n\nRESULTS\n");
    printf("=================================================\n");
    if (cmd == CMD_STATS) {
      printf("Report files were stored in '%s' directory\n", o->out_dirname);
      if (p.filter_on) {
        printf("\nFiltering: enabled\n");
        printf("\tSo, statistics were computed for %lu of %lu reads.\n",
               (unsigned long)r.num_passed, (unsigned long)(r.num_passed + r.num_failed));
      } else {
        printf("\nFiltering: disabled\n");
        printf("\tSo, statistics were computed for the whole input file.\n");
      }
    } else if (cmd == CMD_FILTER) {
      printf("Num. passed reads: %lu (%s/passed.fq)\n", (unsigned long)r.num_passed, o->out_dirname);
      printf("Num. failed reads: %lu (%s/failed.fq)\n", (unsigned long)r.num_failed, o->out_dirname);
    } else {
      printf("Num. edited reads : %lu\n", (unsigned long)r.num_edited);
      printf("Output file       : %s/edit.fq\n", o->out_dirname);
      if (p.filter_on) {
        printf("\nFiltering : Enabled\n");
        printf("\tNum. passed reads : %lu (%s/edit.fq)\n", (unsigned long)r.num_passed, o->out_dirname);
        printf("\tNum. failed reads : %lu (%s/failed.fq)\n", (unsigned long)r.num_failed, o->out_dirname);
      }
    }
    if (r.writer)
      printf("Output writer     : %s\n", r.writer == 1 ? "mapped files, parallel copy" : "one stream writer thread");
    printf("\nThroughput: %lu reads, %.3f GB of FastQ in %.3f s = %.2f Mreads/s (%d GPU worker%s)\n",
           (unsigned long)r.num_reads, r.fastq_bytes / 1e9, r.seconds,
           r.seconds > 0 ? r.num_reads / r.seconds / 1e6 : 0.0, r.num_gpus, r.num_gpus == 1 ? "" : "s");
    printf("=================================================\n");
  }
  free(r.counters);
  free(r.kmers);
  free(r.cg_seq);
  free(r.cg_q);
  cli_free(o);
  return rc;
}
