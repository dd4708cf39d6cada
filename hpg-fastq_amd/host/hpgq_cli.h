/*
 * hpgq_cli.h — the C host side of hpg-fastq on libhpgq (stats | filter | edit).
 *
 * Mirrors the reference's command line (src/hpg-fastq.c; options
 * src/stats_options.c:260-300, src/filter_options.c:235-258,
 * src/edit_options.c:267-290), its producer -> worker -> consumer pipeline
 * (src/stats_fastq.c:174-250, src/filter_fastq.c:106-174,
 * src/edit_fastq.c:113-206) and its outputs (passed.fq / failed.fq,
 * edit.fq, <in>.summary.txt + data files, src/stats_report.c), with the
 * worker's bioinfo-libs calls replaced by the libhpgq C-ABI (include/hpgq.h)
 * and the reader's parsing moved onto the GPU (hpgq_parse_*).
 */
#ifndef HPGQ_CLI_H
#define HPGQ_CLI_H

#include <stddef.h>
#include <stdint.h>

#include "hpgq.h"

enum { CMD_STATS = 0, CMD_FILTER = 1, CMD_EDIT = 2 };

typedef struct {
  int command;
  const char *command_name;
  const char *exec_name;
  char *in_filename;
  char *out_dirname;
  int num_threads;          /* reader threads */
  int batch_size;           /* accepted for compatibility; chunks are sized in bytes */
  char *quality_encoding_name;
  int quality_encoding_value;
  int kmers_on;
  /* chaos game (old/main_hpg_fastq_old.c:185-189: --cg | --chaos-game, --k, --gs-filename) */
  int cg_on, k_cg;
  char *gs_filename;
  /* filter / trim options, NO_VALUE (-1) when unset (src/stats_options.c:18-40) */
  char *read_length_range, *read_quality_range, *left_quality_range, *right_quality_range;
  int min_read_length, max_read_length, min_read_quality, max_read_quality;
  int left_length, min_left_quality, max_left_quality;
  int right_length, min_right_quality, max_right_quality;
  int max_N, max_out_of_quality;
  int filter_on;
  /* MI355X build options */
  int device;               /* first GPU */
  int num_gpus;             /* devices (0: every visible one) */
  int gpu_workers;          /* worker threads per device (2: copy-in beside compute) */
  int64_t cg_batch_size;    /* --cg: FASTQ text bytes per chaos-game call */
  int lmax;                 /* per-position arrays (longest read kept) */
  int chunk_mb;             /* FASTQ text per parse unit */
  int print_params;         /* print hpgq_params_t and exit (no device) */
  char *counters_out;       /* raw u64 counter dump (tests) */
  char *kmers_out;          /* raw u64 k-mer table dump (tests) */
  char *cg_out;             /* raw u32 chaos-game tables dump (tests) */
  int quiet;
  int stream_writer;        /* filter / edit: one writer thread instead of mapped outputs */
  int writer_hook;          /* tests only (--writer-test-hook): hpgq_mapout.h MAPOUT_HOOK_* */
  int copy_threads;         /* mapped writer: copier threads (0: --num-threads) */
  int prefault_threads;     /* mapped writer: prefault threads (-1: default, none past the first window) */
} cli_options_t;

/* parse + validate (exits with the reference's messages on errors) */
cli_options_t *cli_parse(int command, const char *exec_name, int argc, char **argv);
void cli_display(const cli_options_t *o);
void cli_free(cli_options_t *o);
/* NO_VALUE -> MIN/MAX defaults and the libhpgq params (src/filter_fastq.c:195-206) */
void cli_params(const cli_options_t *o, hpgq_params_t *p);
void cli_print_params(const hpgq_params_t *p);
/* src/commons_fastq.c:31-103 */
int cli_parse_range(int *min, int *max, const char *range, const char *msg);

/* pipeline: returns 0 or a negative HPGQ_E* code */
typedef struct {
  uint64_t *counters;       /* the merged counter set(s) at full length (malloc'd) */
  int lmax;                 /* their layout's lmax: max(--lmax, longest merged read) */
  uint64_t num_reads, num_passed, num_failed, num_edited;
  double seconds, fastq_bytes;
  uint64_t *kmers;          /* --kmers: by_pos [HPGQ_NUM_KMERS][kmers_npos] (malloc'd) */
  int kmers_npos;
  uint32_t *cg_seq, *cg_q;  /* --cg: table_seq / table_q [dim*dim] (malloc'd) */
  uint32_t cg_words;        /* fq_word_count */
  int cg_exact_calls;       /* chaos-game calls the exact simulation redid */
  int num_gpus;             /* GPU worker threads that ran */
  int writer;               /* filter / edit outputs: 1 mapped files (parallel copy), 2 stream writer */
} cli_result_t;

int cli_run(const cli_options_t *o, const hpgq_params_t *p, cli_result_t *res);

/* src/stats_report.c: summary + data files (+ k-mer files when res->kmers) */
int cli_report(const cli_options_t *o, const hpgq_params_t *p, const cli_result_t *res);

#endif
