// How fast can threads fill a fresh mapped tmpfs file (the mapped writer's
// output, host/hpgq_pipeline.c)?  Each mode: create DIR/hpgq_fill.tmp, size it
// to BYTES, map it shared, and let T threads fill disjoint contiguous ranges
// of it with memset in 256 MB chunks:
//   fault     page faults on first touch (the writer today)
//   populate  madvise(MADV_POPULATE_WRITE) of each chunk, then the memset
//   falloc    fallocate() of each chunk, then the memset (faults map
//             pages already in the page cache)
//   huge      madvise(MADV_HUGEPAGE) on the mapping, then first-touch faults
//             (2 MB tmpfs pages where shmem_enabled allows "advise")
// One JSON line per (mode, threads).
//   gcc -O2 -pthread tmpfs_fill.c -o tmpfs_fill && ./tmpfs_fill /dev/shm 3000000000
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

enum { FAULT, POPULATE, FALLOC, HUGE };
static const char *names[] = {"fault", "populate", "falloc", "huge"};

typedef struct {
  char *map;
  int fd, mode, err;
  size_t lo, hi;
} job_t;

static const size_t kChunk = (size_t)256 << 20;

static void *run(void *p) {
  job_t *j = p;
  for (size_t o = j->lo; o < j->hi; o += kChunk) {
    const size_t n = o + kChunk < j->hi ? kChunk : j->hi - o;
    if (j->mode == POPULATE && madvise(j->map + o, n, MADV_POPULATE_WRITE)) j->err = 1;
    if (j->mode == FALLOC && fallocate(j->fd, 0, (off_t)o, (off_t)n)) j->err = 1;
    memset(j->map + o, 0x41, n);
  }
  return NULL;
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
  const char *dir = argc > 1 ? argv[1] : "/dev/shm";
  const size_t bytes = argc > 2 ? strtoull(argv[2], NULL, 10) : (size_t)3000000000ull;
  char path[4096];
  snprintf(path, sizeof path, "%s/hpgq_fill.tmp", dir);
  const int tlist[] = {1, 4, 8, 16};
  char thp[256] = "?";
  FILE *f = fopen("/sys/kernel/mm/transparent_hugepage/shmem_enabled", "r");
  if (f) {
    if (!fgets(thp, sizeof thp, f)) thp[0] = 0;
    fclose(f);
    thp[strcspn(thp, "\n")] = 0;
  }
  printf("{\"shmem_enabled\": \"%s\"}\n", thp);
  for (int mode = 0; mode < 4; ++mode) {
    for (int ti = 0; ti < 4; ++ti) {
      const int T = tlist[ti];
      unlink(path);
      const int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
      if (fd < 0 || ftruncate(fd, (off_t)bytes)) return 1;
      char *map = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (map == MAP_FAILED) return 1;
      if (mode == HUGE && madvise(map, bytes, MADV_HUGEPAGE)) printf("{\"madv_hugepage\": \"failed\"}\n");
      pthread_t th[16];
      job_t jobs[16];
      const size_t per = (bytes / T + 4095) & ~(size_t)4095;
      const double t0 = now();
      for (int t = 0; t < T; ++t) {
        jobs[t] = (job_t){map, fd, mode, 0, per * t, per * (t + 1) < bytes ? per * (t + 1) : bytes};
        pthread_create(&th[t], NULL, run, &jobs[t]);
      }
      int err = 0;
      for (int t = 0; t < T; ++t) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
      }
      const double dt = now() - t0;
      printf("{\"mode\": \"%s\", \"threads\": %d, \"GB_s\": %.2f, \"err\": %d}\n", names[mode], T, bytes / dt / 1e9, err);
      fflush(stdout);
      munmap(map, bytes);
      close(fd);
      unlink(path);
    }
  }
  return 0;
}
