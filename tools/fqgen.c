/*
 * fqgen.c — synthetic FASTQ file for the end-to-end benchmark (tool, not product).
 * Same counter-based generator as bench.py / the oracle: seed,
 * read length L, 5 % truncated, 5 % bad, 'N' at 1/1024, phred33.
 *   gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen && /tmp/fqgen out.fq 20000000 150 2 [cpus]
 * cpus: optional comma-separated CPU ids the generator pins itself to before
 * its threads start (bench.py: the GPU's NUMA node, so the file's pages land
 * there), instead of the parent pinning the child between fork and exec.
 */
#define _GNU_SOURCE
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: fqgen out.fq nreads L seed\n");
    return 1;
  }
  const int64_t n = atoll(argv[2]);
  const int L0 = atoi(argv[3]);
  const uint64_t seed = strtoull(argv[4], 0, 10);
  if (argc > 5 && argv[5][0]) {
    cpu_set_t set;
    CPU_ZERO(&set);
    for (char *t = argv[5]; *t;) {
      const long c = strtol(t, &t, 10);
      if (c >= 0 && c < CPU_SETSIZE) CPU_SET((int)c, &set);
      if (*t == ',') ++t;
      else if (*t) break;
    }
    if (CPU_COUNT(&set) && sched_setaffinity(0, sizeof(set), &set) != 0) perror("fqgen: sched_setaffinity");
  }
  FILE *f = fopen(argv[1], "wb");
  if (!f) return 1;
  const int64_t block = 1 << 16;
  const size_t rec_max = 32 + 2 * (size_t)L0 + 8;
  char *buf = malloc((size_t)block * rec_max);
  size_t *len = malloc(sizeof(size_t) * block);
  for (int64_t b0 = 0; b0 < n; b0 += block) {
    const int64_t nb = b0 + block > n ? n - b0 : block;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t i = b0 + k;
      const uint64_t r = mix64(seed * 0x9E3779B97F4A7C15ULL + (uint64_t)i);
      int L = L0;
      if (L0 >= 20 && (int)(r % 100) < 5) L = 20 + (int)(mix64(r ^ 1ULL) % (uint64_t)(L0 - 20 + 1));
      const int bad = (int)((r >> 20) % 100) < 5;
      char *o = buf + (size_t)k * rec_max;
      int p = sprintf(o, "@read_%lld\n", (long long)i);
      char *s = o + p, *q = s + L + 3;
      for (int j = 0; j < L; ++j) {
        const uint64_t h = mix64(r + (uint64_t)(j + 1) * 0xD1B54A32D192ED03ULL);
        s[j] = ((int)(h & 1023) < 1) ? 'N' : "ACGT"[(h >> 10) & 3];
        const int noise = (int)((h >> 12) % 13) - 6;
        int qq = bad ? 12 + noise : 40 - (20 * j) / L + noise;
        if (qq < 2) qq = 2;
        if (qq > 41) qq = 41;
        q[j] = (char)(qq + 33);
      }
      s[L] = '\n';
      s[L + 1] = '+';
      s[L + 2] = '\n';
      q[L] = '\n';
      len[k] = (size_t)p + 2 * (size_t)L + 4;
    }
    for (int64_t k = 0; k < nb; ++k) fwrite(buf + (size_t)k * rec_max, 1, len[k], f);
  }
  fclose(f);
  free(buf);
  free(len);
  return 0;
}
