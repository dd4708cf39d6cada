/* The mapped output files' failure modes (hpg-fastq_amd/host/hpgq_mapout.c)
 * without a GPU: test infrastructure, run by tests/test_sanitize_cpu.py.
 *   mapout_main normal   DIR   windows prefaulted ahead, guarded copies, files truncated to size
 *   mapout_main reserve  DIR   the first-window reservation fails: 1 (stream writer), files empty
 *   mapout_main populate DIR   a later prefault window fails: HPGQ_E_IO from mapout_close
 *   mapout_main sigbus   DIR   a store past the file's end: the guard returns HPGQ_E_IO
 * Prints "mapout_main: ok <mode>" and exits 0 when the behaviour is the expected one. */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "hpgq.h"
#include "hpgq_mapout.h"

static int fail(const char *what) {
  printf("mapout_main: FAIL %s\n", what);
  return 1;
}

typedef struct {
  char *dst;
  const char *src;
  size_t n;
} copy_t;

static void do_copy(void *arg) {
  copy_t *c = arg;
  memcpy(c->dst, c->src, c->n);
}

static int open_pair(const char *dir, int fd[2]) {
  char path[4096];
  for (int c = 0; c < 2; ++c) {
    snprintf(path, sizeof(path), "%s/out%d.fq", dir, c);
    fd[c] = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (fd[c] < 0) return -1;
  }
  return 0;
}

static off_t fsize(int fd) {
  struct stat st;
  return fstat(fd, &st) ? -1 : st.st_size;
}

int main(int argc, char **argv) {
  if (argc != 3) return fail("usage");
  const char *mode = argv[1], *dir = argv[2];
  int fd[2];
  if (open_pair(dir, fd)) return fail("open");
  const size_t cap = (size_t)100 << 20, ahead = (size_t)48 << 20;
  mapout_t m;
  if (!strcmp(mode, "normal")) {
    if (mapout_open(&m, fd, cap, ahead, 2, 0) != 0) return fail("mapped");
    /* place + copy 7 MB pieces alternately into both outputs, as the pipeline does */
    const size_t piece = (size_t)7 << 20;
    char *src = malloc(piece);
    if (!src) return fail("malloc");
    uint64_t off[2] = {0, 0};
    char letters[2][16];
    int np[2] = {0, 0};
    for (int k = 0; k < 12; ++k) {
      const int c = k % 3 == 2;   /* two pieces to output 0, one to output 1 */
      memset(src, 'A' + k, piece);
      mapout_advance(&m, c, off[c] + piece);
      copy_t cp = {m.map[c] + off[c], src, piece};
      if (mapout_guard(do_copy, &cp)) return fail("guarded copy");
      off[c] += piece;
      letters[c][np[c]++] = (char)('A' + k);
    }
    free(src);
    if (mapout_error(&m)) return fail("prefault error");
    if (mapout_close(&m, off)) return fail("close");
    for (int c = 0; c < 2; ++c) {
      if ((uint64_t)fsize(fd[c]) != off[c]) return fail("final size");
      for (int i = 0; i < np[c]; ++i) {   /* first and last byte of each piece */
        char a, b;
        if (pread(fd[c], &a, 1, (off_t)(i * piece)) != 1 || pread(fd[c], &b, 1, (off_t)((i + 1) * piece - 1)) != 1 ||
            a != letters[c][i] || b != letters[c][i])
          return fail("content");
      }
    }
  } else if (!strcmp(mode, "reserve")) {
    if (mapout_open(&m, fd, cap, ahead, 2, MAPOUT_HOOK_RESERVE_FAIL) != 1) return fail("stream writer");
    if (fsize(fd[0]) != 0 || fsize(fd[1]) != 0) return fail("files left empty");
  } else if (!strcmp(mode, "populate")) {
    if (mapout_open(&m, fd, cap, ahead, 2, MAPOUT_HOOK_POPULATE_FAIL) != 0) return fail("mapped");
    mapout_advance(&m, 0, (size_t)40 << 20);   /* past the reserved first window */
    for (int t = 0; t < 2000 && !mapout_error(&m); ++t) {
      struct timespec ts = {0, 1000000};
      nanosleep(&ts, NULL);
    }
    if (mapout_error(&m) != HPGQ_E_IO) return fail("prefault error");
    const uint64_t z[2] = {0, 0};
    if (mapout_close(&m, z) != HPGQ_E_IO) return fail("close returns HPGQ_E_IO");
  } else if (!strcmp(mode, "sigbus")) {
    if (mapout_open(&m, fd, cap, ahead, 1, MAPOUT_HOOK_SIGBUS) != 0) return fail("mapped");
    char src[4096];
    memset(src, 'x', sizeof(src));
    copy_t cp = {m.map[0] + 8192, src, sizeof(src)};
    if (mapout_guard(do_copy, &cp) != HPGQ_E_IO) return fail("guard returns HPGQ_E_IO");
    copy_t ok = {m.map[1], src, sizeof(src)};   /* the other output still works */
    if (mapout_guard(do_copy, &ok) != 0) return fail("unaffected output");
    const uint64_t z[2] = {0, sizeof(src)};
    mapout_close(&m, z);
    if (fsize(fd[1]) != (off_t)sizeof(src)) return fail("other output size");
  } else {
    return fail("mode");
  }
  close(fd[0]);
  close(fd[1]);
  printf("mapout_main: ok %s\n", mode);
  return 0;
}
