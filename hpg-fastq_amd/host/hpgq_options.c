/*
 * hpgq_options.c — command-line options of hpg-fastq stats | filter | edit.
 *
 * Same flags, defaults, validation and messages as the reference:
 * src/stats_options.c:15-300, src/filter_options.c:15-258,
 * src/edit_options.c:15-290; parse_range src/commons_fastq.c:31-103.
 * Build-specific additions: --gpu, --lmax, --chunk-mb, --print-params,
 * --counters-out, --kmers-out, --quiet.  --quality-encoding is accepted by every command
 * (quirk Q11).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "hpgq_cli.h"

static const char *kCommandHelp[] = {"statistics summary",
                                     "filter a FastQ file by using advanced criteria",
                                     "edit a FastQ file according the specified options"};

int cli_parse_range(int *min, int *max, const char *range, const char *msg) {
  int lmin = HPGQ_NO_VALUE, lmax = HPGQ_NO_VALUE;
  if (range == NULL) {
    *min = HPGQ_NO_VALUE;
    *max = HPGQ_NO_VALUE;
    return 1;
  }
  const char *comma = strchr(range, ',');
  if (comma) {
    if (comma[1] != '\0' && sscanf(comma + 1, "%d", &lmax) != 1) {
      printf("\nError: Invalid maximum value in the %s (%s)\n", msg, range);
      return 0;
    }
    if (comma != range && sscanf(range, "%d", &lmin) != 1) {
      printf("\nError: Invalid minimum value in the %s (%s)\n", msg, range);
      return 0;
    }
  } else {
    if (sscanf(range, "%d", &lmin) != 1) {
      printf("\nError: Invalid minimum value in the %s (%s)\n", msg, range);
      return 0;
    }
    lmax = HPGQ_NO_VALUE;
  }
  if (lmin != HPGQ_NO_VALUE && lmin < 0) {
    printf("\nError: Invalid %s (%s). Minimum value (%i) must be greater than 0\n", msg, range, lmin);
    return 0;
  }
  if (lmax != HPGQ_NO_VALUE && lmax < 0) {
    printf("\nError: Invalid %s (%s). Maximum value (%i) must be greater than 0\n", msg, range, lmax);
    return 0;
  }
  if (lmin != HPGQ_NO_VALUE && lmax != HPGQ_NO_VALUE && lmin > lmax) {
    printf("\nError: Invalid %s (%s). Maximum value (%i) must be greater than minimum value (%i)\n",
           msg, range, lmax, lmin);
    return 0;
  }
  *min = lmin;
  *max = lmax;
  return 1;
}

static void usage(const cli_options_t *o) {
  printf("Usage: %s %s [options]   (%s)\n\n", o->exec_name, o->command_name,
         kCommandHelp[o->command]);
  printf("  -h, --help                      Help option\n");
  printf("  -f, --fastq-file=<file>         Input file name (FastQ format)\n");
  printf("  -o, --outdir=<file>             Output directory name\n");
  printf("  --num-threads=<int>             Number of threads (file readers)\n");
  printf("  --batch-size=<int>              Batch size (accepted; batches are --chunk-mb of text)\n");
  printf("  --quality-encoding=<string>     Encoding for quality scores: phred33, phred64\n");
  if (o->command == CMD_STATS) {
    printf("  --kmers                         Enable k-mers analysis (5-mer)\n");
    printf("  --cg, --chaos-game              Genomic signature (chaos game) tables and images\n");
    printf("  --k=<int>                       Chaos game word size (1-12, default 7)\n");
    printf("  --gs-filename=<file>            Reference genomic signature: difference table and image\n");
    printf("  --cg-batch-size=<int>           FastQ text bytes per chaos-game call (default 64000000)\n");
  }
  printf("  --read-length-range=<string>    Read length range, eg. 80,110\n");
  printf("  --read-quality-range=<string>   Read quality range, eg. 20,40\n");
  printf("  --left-length=<int>             Number of leftmost nucleotides to take into account to %s\n",
         o->command == CMD_EDIT ? "trim" : "filter or trim");
  printf("  --left-quality-range=<string>   Quality range for the leftmost nucleotides, eg. 15,45\n");
  printf("  --right-length=<int>            Number of rightmost nucleotides to take into account to %s\n",
         o->command == CMD_EDIT ? "trim" : "filter or trim");
  printf("  --right-quality-range=<string>  Quality range for the rightmost nucleotides, eg. 10,60\n");
  printf("  --max-N=<int>                   Maximum number of Ns in the sequences\n");
  printf("  --max-out-of-quality=<int>      Maximum number of nucleotides out of the read quality range\n");
  printf("\n  MI355X build:\n");
  printf("  --gpu=<int>                     First HIP device (default 0)\n");
  printf("  --gpus=<int>                    GPUs, chunks round-robin (default: every visible device)\n");
  printf("  --gpu-workers=<int>             Worker threads per GPU (default 2: copy-in beside compute)\n");
  printf("  --lmax=<int>                    Longest read kept per position (default %d)\n",
         HPGQ_LMAX_LIMIT);
  printf("  --chunk-mb=<int>                FastQ text per GPU parse unit (default 256)\n");
  printf("  --print-params                  Print the engine parameters and exit\n");
  printf("  --counters-out=<file>           Write the raw u64 counter set\n");
  if (o->command == CMD_STATS)
    printf("  --kmers-out=<file>              Write the raw u64 k-mer table [1024][lmax-4]\n");
  if (o->command == CMD_STATS)
    printf("  --cg-out=<file>                 Write the raw u32 chaos-game tables + word count\n");
  if (o->command != CMD_STATS)
    printf("  --stream-writer                 Write the FastQ outputs through one writer thread\n"
           "                                  (default: mapped output files filled in parallel)\n"
           "  --copy-threads=<int>            Mapped writer: copier threads (default --num-threads)\n"
           "  --prefault-threads=<int>        Mapped writer: threads populating the outputs ahead (default 0)\n");
  printf("  --quiet                         No parameter / result display\n");
  exit(-1);
}

static int exists(const char *path) {
  struct stat st;
  return path && stat(path, &st) == 0;
}

/* a whole-string decimal in [lo, hi], else the usage error (atoi
 * turned garbage into 0 or the default) */
static int count_arg(const cli_options_t *o, const char *flag, const char *s, int lo, int hi) {
  char *end = NULL;
  errno = 0;
  const long v = strtol(s, &end, 10);
  if (errno || end == s || *end != '\0' || v < lo || v > hi) {
    printf("\nError: --%s must be an integer in %d..%d (%s)\n", flag, lo, hi, s);
    usage(o);
  }
  return (int)v;
}

enum {
  O_THREADS = 1000, O_BATCH, O_QENC, O_KMERS, O_LRANGE, O_QRANGE, O_LLEN, O_LQRANGE, O_RLEN,
  O_RQRANGE, O_MAXN, O_MAXOOQ, O_GPU, O_LMAX, O_CHUNK, O_PRINT, O_COUNTERS, O_QUIET,
  O_KMERSOUT, O_CG, O_KCG, O_GS, O_GPUS, O_CGBATCH, O_CGOUT, O_GPUW, O_STREAMW, O_WHOOK, O_COPYT, O_PFT
};

cli_options_t *cli_parse(int command, const char *exec_name, int argc, char **argv) {
  static const char *names[] = {"stats", "filter", "edit"};
  cli_options_t *o = calloc(1, sizeof(*o));
  o->command = command;
  o->command_name = names[command];
  o->exec_name = exec_name;
  o->num_threads = 4;
  o->batch_size = 10000;
  o->min_read_length = o->max_read_length = HPGQ_NO_VALUE;
  o->min_read_quality = o->max_read_quality = HPGQ_NO_VALUE;
  o->left_length = o->min_left_quality = o->max_left_quality = HPGQ_NO_VALUE;
  o->right_length = o->min_right_quality = o->max_right_quality = HPGQ_NO_VALUE;
  o->max_N = o->max_out_of_quality = HPGQ_NO_VALUE;
  o->lmax = HPGQ_LMAX_LIMIT;
  o->chunk_mb = 256;
  o->k_cg = 7;   /* DEFAULT_K_IN_CHAOS_GAME */
  o->cg_batch_size = 64000000;   /* DEFAULT_BATCH_SIZE_MB * 1000000, old/main_hpg_fastq_old.c:116 */
  o->gpu_workers = 2;
  o->prefault_threads = -1;
  static const struct option longopts[] = {
      {"help", no_argument, 0, 'h'},
      {"fastq-file", required_argument, 0, 'f'},
      {"outdir", required_argument, 0, 'o'},
      {"num-threads", required_argument, 0, O_THREADS},
      {"batch-size", required_argument, 0, O_BATCH},
      {"quality-encoding", required_argument, 0, O_QENC},
      {"kmers", no_argument, 0, O_KMERS},
      {"cg", no_argument, 0, O_CG},
      {"chaos-game", no_argument, 0, O_CG},
      {"k", required_argument, 0, O_KCG},
      {"gs-filename", required_argument, 0, O_GS},
      {"read-length-range", required_argument, 0, O_LRANGE},
      {"read-quality-range", required_argument, 0, O_QRANGE},
      {"left-length", required_argument, 0, O_LLEN},
      {"left-quality-range", required_argument, 0, O_LQRANGE},
      {"right-length", required_argument, 0, O_RLEN},
      {"right-quality-range", required_argument, 0, O_RQRANGE},
      {"max-N", required_argument, 0, O_MAXN},
      {"max-out-of-quality", required_argument, 0, O_MAXOOQ},
      {"gpu", required_argument, 0, O_GPU},
      {"gpus", required_argument, 0, O_GPUS},
      {"gpu-workers", required_argument, 0, O_GPUW},
      {"cg-batch-size", required_argument, 0, O_CGBATCH},
      {"cg-out", required_argument, 0, O_CGOUT},
      {"lmax", required_argument, 0, O_LMAX},
      {"chunk-mb", required_argument, 0, O_CHUNK},
      {"print-params", no_argument, 0, O_PRINT},
      {"counters-out", required_argument, 0, O_COUNTERS},
      {"kmers-out", required_argument, 0, O_KMERSOUT},
      {"quiet", no_argument, 0, O_QUIET},
      {"stream-writer", no_argument, 0, O_STREAMW},
      {"writer-test-hook", required_argument, 0, O_WHOOK},
      {"copy-threads", required_argument, 0, O_COPYT},
      {"prefault-threads", required_argument, 0, O_PFT},
      {0, 0, 0, 0}};
  if (argc < 2) usage(o);
  optind = 1;
  int c;
  while ((c = getopt_long(argc, argv, "hf:o:", longopts, NULL)) != -1) {
    switch (c) {
      case 'h': usage(o); break;
      case 'f': o->in_filename = strdup(optarg); break;
      case 'o': o->out_dirname = strdup(optarg); break;
      case O_THREADS: o->num_threads = atoi(optarg); break;
      case O_BATCH: o->batch_size = atoi(optarg); break;
      case O_QENC: o->quality_encoding_name = strdup(optarg); break;
      case O_KMERS:
        if (command != CMD_STATS) usage(o);
        o->kmers_on = 1;
        break;
      case O_CG:
        if (command != CMD_STATS) usage(o);
        o->cg_on = 1;
        break;
      case O_KCG: o->k_cg = atoi(optarg); break;
      case O_GS: o->gs_filename = strdup(optarg); break;
      case O_LRANGE: o->read_length_range = strdup(optarg); break;
      case O_QRANGE: o->read_quality_range = strdup(optarg); break;
      case O_LLEN: o->left_length = atoi(optarg); break;
      case O_LQRANGE: o->left_quality_range = strdup(optarg); break;
      case O_RLEN: o->right_length = atoi(optarg); break;
      case O_RQRANGE: o->right_quality_range = strdup(optarg); break;
      case O_MAXN: o->max_N = atoi(optarg); break;
      case O_MAXOOQ: o->max_out_of_quality = atoi(optarg); break;
      case O_GPU: o->device = atoi(optarg); break;
      case O_GPUS: o->num_gpus = atoi(optarg); break;
      case O_GPUW: o->gpu_workers = atoi(optarg); break;
      case O_CGBATCH: o->cg_batch_size = atoll(optarg); break;
      case O_LMAX: o->lmax = atoi(optarg); break;
      case O_CHUNK: o->chunk_mb = atoi(optarg); break;
      case O_PRINT: o->print_params = 1; break;
      case O_COUNTERS: o->counters_out = strdup(optarg); break;
      case O_KMERSOUT: o->kmers_out = strdup(optarg); break;
      case O_CGOUT: o->cg_out = strdup(optarg); break;
      case O_QUIET: o->quiet = 1; break;
      case O_STREAMW: o->stream_writer = 1; break;
      case O_WHOOK:   /* tests only: hpgq_mapout.h MAPOUT_HOOK_* force the writer's failure paths */
        if (!getenv("HPGQ_WRITER_TEST_HOOKS")) {
          printf("\nError: --writer-test-hook is a test option (set HPGQ_WRITER_TEST_HOOKS=1)\n");
          usage(o);
        }
        o->writer_hook = count_arg(o, "writer-test-hook", optarg, 0, 7);
        break;
      case O_COPYT: o->copy_threads = count_arg(o, "copy-threads", optarg, 0, 64); break;
      case O_PFT: o->prefault_threads = count_arg(o, "prefault-threads", optarg, 0, 4); break;
      default: usage(o);
    }
  }
  /* validation, src/stats_options.c:108-160 */
  if (!o->print_params && !exists(o->in_filename)) {
    printf("\nError: Input file name not found !\n");
    usage(o);
  }
  if (!exists(o->out_dirname)) {
    free(o->out_dirname);
    o->out_dirname = strdup(".");
  }
  if (o->quality_encoding_name) {
    if (strcmp(o->quality_encoding_name, "phred33") == 0) {
      o->quality_encoding_value = HPGQ_PHRED33;
    } else if (strcmp(o->quality_encoding_name, "phred64") == 0) {
      o->quality_encoding_value = HPGQ_PHRED64;
    } else {
      printf("\nError: Invalid quality encoding value (%s). Valid values: %s, %s\n",
             o->quality_encoding_name, "phred33", "phred64");
      usage(o);
    }
  } else {
    o->quality_encoding_name = strdup("phred33");
    o->quality_encoding_value = HPGQ_PHRED33;
  }
  if (!cli_parse_range(&o->min_read_length, &o->max_read_length, o->read_length_range,
                       "read length range") ||
      !cli_parse_range(&o->min_read_quality, &o->max_read_quality, o->read_quality_range,
                       "read quality range") ||
      !cli_parse_range(&o->min_left_quality, &o->max_left_quality, o->left_quality_range,
                       "left quality range") ||
      !cli_parse_range(&o->min_right_quality, &o->max_right_quality, o->right_quality_range,
                       "right quality range"))
    usage(o);
  if (o->lmax < 1 || o->lmax > HPGQ_LMAX_LIMIT) {
    printf("\nError: --lmax must be in 1..%d\n", HPGQ_LMAX_LIMIT);
    exit(-1);
  }
  if (o->chunk_mb < 1 || o->chunk_mb > 1536) {
    printf("\nError: --chunk-mb must be in 1..1536\n");
    exit(-1);
  }
  if (o->num_threads < 1) o->num_threads = 1;
  if (o->num_gpus < 0) o->num_gpus = 0;
  if (o->gpu_workers < 1) o->gpu_workers = 1;
  /* the old tool's floor (old/main_hpg_fastq_old.c:474-477 takes 64 MB below 64) */
  if (o->cg_batch_size < 64) o->cg_batch_size = 64000000;
  if (o->cg_batch_size > ((int64_t)1536 << 20)) {
    printf("\nError: --cg-batch-size must be at most %lld\n", (long long)1536 << 20);
    exit(-1);
  }
  if (o->cg_on && (o->k_cg < 1 || o->k_cg > 12)) {
    printf("\nError: --k must be in 1..12\n");
    exit(-1);
  }
  if (o->gs_filename && !exists(o->gs_filename)) {
    printf("\nError: Genomic signature file not found !\n");
    usage(o);
  }
  /* filter_on (src/stats_options.c:177-213; edit's ignores left/right,
   * src/edit_options.c:190-215) */
  int n = 0;
  n += o->read_length_range != NULL;
  n += o->read_quality_range != NULL;
  if (command != CMD_EDIT) {
    n += o->left_length != HPGQ_NO_VALUE && o->left_quality_range != NULL;
    n += o->right_length != HPGQ_NO_VALUE && o->right_quality_range != NULL;
  }
  n += o->max_N != HPGQ_NO_VALUE;
  n += o->max_out_of_quality != HPGQ_NO_VALUE && o->read_quality_range != NULL;
  o->filter_on = n > 0;
  if (command == CMD_FILTER && !o->filter_on) {   /* src/filter_options.c:166-172 */
    printf("\nError: Nothing to filter, no filter options specified !\n");
    usage(o);
  }
  if (command == CMD_EDIT &&
      !((o->left_length != HPGQ_NO_VALUE && o->left_quality_range) ||
        (o->right_length != HPGQ_NO_VALUE && o->right_quality_range))) {   /* edit_options.c:228-231 */
    printf("\nError: Nothing to edit, no edit options specified !\n");
    usage(o);
  }
  /* trims are two 16-bit fields (libhpgq's trim_out): HPGQ_MAX_EDIT_LENGTH */
  if (command == CMD_EDIT && (o->left_length > HPGQ_MAX_EDIT_LENGTH || o->right_length > HPGQ_MAX_EDIT_LENGTH)) {
    printf("\nError: --left-length and --right-length must be at most %d\n", HPGQ_MAX_EDIT_LENGTH);
    exit(-1);
  }
  return o;
}

void cli_display(const cli_options_t *o) {
  printf("PARAMETERS CONFIGURATION\n");
  printf("=================================================\n");
  printf("Command name : %s\n", o->command_name);
  printf("\nMain options\n");
  printf("\tFastQ input filename : %s\n", o->in_filename ? o->in_filename : "(none)");
  printf("\tOutput dirname       : %s\n", o->out_dirname);
  printf("\tQuality encoding     : %s\n", o->quality_encoding_name);
  printf("\n%s options\n", o->command == CMD_EDIT ? "Edit and filter" : "Filter");
  int shown = 0;
  if (o->read_length_range) printf("\tRead length range   : %s\n", o->read_length_range), shown++;
  if (o->read_quality_range) printf("\tRead quality range  : %s\n", o->read_quality_range), shown++;
  if (o->left_length != HPGQ_NO_VALUE && o->left_quality_range) {
    printf("\tLeft length         : %i nucleotides\n", o->left_length);
    printf("\tLeft quality range  : %s\n", o->left_quality_range);
    shown++;
  }
  if (o->right_length != HPGQ_NO_VALUE && o->right_quality_range) {
    printf("\tRight length        : %i nucleotides\n", o->right_length);
    printf("\tRight quality range : %s\n", o->right_quality_range);
    shown++;
  }
  if (o->max_N != HPGQ_NO_VALUE) printf("\tMax. number of Ns   : %i\n", o->max_N), shown++;
  if (o->max_out_of_quality != HPGQ_NO_VALUE && o->read_quality_range)
    printf("\tMax. out of quality : %i nucletotides\n", o->max_out_of_quality), shown++;
  if (!shown) printf("\tNone.\n");
  if (o->cg_on) {
    printf("\nChaos game options\n");
    printf("\tWord size (k)       : %d\n", o->k_cg);
    printf("\tGenomic signature   : %s\n", o->gs_filename ? o->gs_filename : "(none)");
  }
  printf("\nArchitecture options\n");
  printf("\tGPU                 : %d (gfx950), %d worker%s per GPU on %s\n", o->device, o->gpu_workers,
         o->gpu_workers == 1 ? "" : "s", o->num_gpus > 0 ? "--gpus GPUs" : "every visible GPU");
  printf("\tReader threads      : %d\n", o->num_threads);
  printf("\tChunk size          : %d MB of FastQ text\n", o->chunk_mb);
  printf("=================================================\n");
}

static int dflt(int v, int d) { return v == HPGQ_NO_VALUE ? d : v; }

void cli_params(const cli_options_t *o, hpgq_params_t *p) {
  hpgq_params_init(p);
  p->phred = o->quality_encoding_value;
  p->lmax = o->lmax;
  p->stats_on = o->command == CMD_STATS;
  p->filter_on = o->filter_on;
  p->min_read_length = dflt(o->min_read_length, HPGQ_MIN_VALUE);
  p->max_read_length = dflt(o->max_read_length, HPGQ_MAX_VALUE);
  p->min_read_quality = dflt(o->min_read_quality, HPGQ_MIN_VALUE);
  p->max_read_quality = dflt(o->max_read_quality, HPGQ_MAX_VALUE);
  p->max_out_of_quality = dflt(o->max_out_of_quality, HPGQ_MAX_VALUE);
  p->max_N = dflt(o->max_N, HPGQ_MAX_VALUE);
  const int ll = dflt(o->left_length, HPGQ_MIN_VALUE), rl = dflt(o->right_length, HPGQ_MIN_VALUE);
  const int lq0 = dflt(o->min_left_quality, HPGQ_MIN_VALUE), lq1 = dflt(o->max_left_quality, HPGQ_MAX_VALUE);
  const int rq0 = dflt(o->min_right_quality, HPGQ_MIN_VALUE), rq1 = dflt(o->max_right_quality, HPGQ_MAX_VALUE);
  if (o->command == CMD_EDIT) {
    /* the trim takes the left/right options; the filter runs with them off
     * (src/edit_fastq.c:148-166) */
    p->edit_on = 1;
    p->edit_left_length = ll;
    p->edit_min_left_quality = lq0;
    p->edit_max_left_quality = lq1;
    p->edit_right_length = rl;
    p->edit_min_right_quality = rq0;
    p->edit_max_right_quality = rq1;
  } else {
    p->left_length = ll;
    p->min_left_quality = lq0;
    p->max_left_quality = lq1;
    p->right_length = rl;
    p->min_right_quality = rq0;
    p->max_right_quality = rq1;
  }
}

void cli_print_params(const hpgq_params_t *p) {
  printf("phred=%d lmax=%d stats_on=%d filter_on=%d edit_on=%d paired=%d\n", p->phred, p->lmax,
         p->stats_on, p->filter_on, p->edit_on, p->paired);
  printf("min_read_length=%d max_read_length=%d min_read_quality=%d max_read_quality=%d\n",
         p->min_read_length, p->max_read_length, p->min_read_quality, p->max_read_quality);
  printf("max_out_of_quality=%d left_length=%d min_left_quality=%d max_left_quality=%d\n",
         p->max_out_of_quality, p->left_length, p->min_left_quality, p->max_left_quality);
  printf("right_length=%d min_right_quality=%d max_right_quality=%d max_N=%d\n", p->right_length,
         p->min_right_quality, p->max_right_quality, p->max_N);
  printf("edit_left_length=%d edit_min_left_quality=%d edit_max_left_quality=%d\n",
         p->edit_left_length, p->edit_min_left_quality, p->edit_max_left_quality);
  printf("edit_right_length=%d edit_min_right_quality=%d edit_max_right_quality=%d\n",
         p->edit_right_length, p->edit_min_right_quality, p->edit_max_right_quality);
}

void cli_free(cli_options_t *o) {
  if (!o) return;
  free(o->in_filename);
  free(o->out_dirname);
  free(o->quality_encoding_name);
  free(o->read_length_range);
  free(o->read_quality_range);
  free(o->left_quality_range);
  free(o->right_quality_range);
  free(o->counters_out);
  free(o->kmers_out);
  free(o->cg_out);
  free(o->gs_filename);
  free(o);
}
