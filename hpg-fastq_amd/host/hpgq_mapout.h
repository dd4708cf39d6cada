/*
 * hpgq_mapout.h — the mapped output files of filter / edit (host side).
 *
 * The reference's consumer writes passed / failed records through stdio in
 * input order (src/filter_fastq.c:161-174, src/edit_fastq.c:184-206).  Here
 * each regular output file is extended to a bound, mapped shared, and filled
 * by many copier threads at once (hpgq_pipeline.c); this module owns the
 * mapping and its failure modes:
 *   - not on file systems whose extended files are not sparse (FAT, exFAT,
 *     NTFS, HFS): there extending both outputs to the input's size would
 *     allocate twice the input before a record is written;
 *   - the first window of each output is reserved (populated) before the
 *     mapping is used, else the stream writer runs;
 *   - by default nothing past that first window is reserved: the copiers
 *     fault the pages in, and every copy runs under the SIGBUS guard below;
 *   - optional prefault threads (--prefault-threads N, default none: they
 *     measured slower than none on the GPU boxes) populate the
 *     outputs (MADV_POPULATE_WRITE, or fallocate where that is missing, or
 *     nothing where neither is supported) a window ahead of the records
 *     placed so far, so a file system that cannot back a page makes that call
 *     fail (HPGQ_E_IO) instead of a store raising SIGBUS;
 *   - every copy runs under a SIGBUS guard (mapout_guard): a store the file
 *     system cannot back (no room; another writer filled it after the check)
 *     ends that copy with HPGQ_E_IO instead of killing the process.  The
 *     guard's handler is re-installed at any copy that finds another SIGBUS
 *     handler in its place.
 */
#ifndef HPGQ_MAPOUT_H
#define HPGQ_MAPOUT_H

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#define MAPOUT_MAX_PF 4

/* test hooks (cli_options_t.writer_hook, CLI --writer-test-hook N; tests only) */
enum {
  MAPOUT_HOOK_RESERVE_FAIL = 1,    /* the first-window reservation fails: the stream writer runs */
  MAPOUT_HOOK_POPULATE_FAIL = 2,   /* every prefault window after the first fails: HPGQ_E_IO */
  MAPOUT_HOOK_SIGBUS = 4           /* output 0 shrinks to 0 bytes behind its mapping: stores fault */
};

typedef struct {
  int fd[2];              /* -1: no such output */
  char *map[2];
  size_t cap;             /* bytes mapped per output */
  size_t window, ahead;   /* prefault window, and how far past the placed bytes */
  int hook;
  /* prefault threads: populate [next, want) of each output in windows */
  pthread_t th[MAPOUT_MAX_PF];
  int nth;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  size_t want[2], next[2];
  int stop, err;
  int live;               /* mu / cv initialised (a successful mapout_open) */
  int mode;               /* how windows are reserved: MAPOUT_POPULATE / _FALLOCATE / _UNRESERVED */
} mapout_t;

enum { MAPOUT_POPULATE = 0, MAPOUT_FALLOCATE = 1, MAPOUT_UNRESERVED = 2 };
extern const char *const mapout_mode_name[3];

/* Map the outputs fd[c] (-1: none) at `cap` bytes each.  0: mapped, the
 * prefault threads running; 1: not mapped (not a regular file, a file system
 * whose extended files are not sparse, not enough room, or the first-window
 * reservation failed), the files left empty -- the caller runs the stream
 * writer; < 0: HPGQ_E_NOMEM. */
int mapout_open(mapout_t *m, const int fd[2], size_t cap, size_t ahead, int threads, int hook);
/* output c holds `placed` bytes of records (placed, maybe not yet copied):
 * keep it populated up to placed + ahead */
void mapout_advance(mapout_t *m, int c, size_t placed);
/* a prefault failure so far (HPGQ_E_IO) or 0 */
int mapout_error(mapout_t *m);
/* fn(arg) with SIGBUS turned into a return of HPGQ_E_IO (any thread) */
int mapout_guard(void (*fn)(void *), void *arg);
/* stop prefaulting, unmap, truncate output c to size[c]; 0 or the first
 * error (a prefault failure or a failed truncate: HPGQ_E_IO) */
int mapout_close(mapout_t *m, const uint64_t size[2]);

#endif
