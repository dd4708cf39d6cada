/*
 * hpgq_mapout.c — mapped output files with reservation, prefaulting and a
 * SIGBUS guard (see hpgq_mapout.h).
 */
#define _GNU_SOURCE
#include "hpgq_mapout.h"

#include <errno.h>
#include <fcntl.h>
#include <setjmp.h>
#include <signal.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include "hpgq.h"

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

const char *const mapout_mode_name[3] = {"MADV_POPULATE_WRITE", "fallocate", "none (first-touch faults)"};

/* file systems on which an extended (ftruncate'd) file is NOT sparse: there
 * extending both outputs to the input's size allocates (or zero-fills) twice
 * the input before a record is written */
static int dense_fs(int fd) {
  struct statfs sf;
  if (fstatfs(fd, &sf)) return 1;
  switch ((unsigned long)sf.f_type) {
    case 0x4D44UL:       /* msdos / vfat */
    case 0x2011BAB0UL:   /* exfat */
    case 0x5346544EUL:   /* ntfs */
    case 0x4244UL:       /* hfs */
      return 1;
    default:
      return 0;
  }
}

/* back [a, a + n) of output c with pages: 0, or -1 when the file system
 * cannot.  MADV_POPULATE_WRITE (allocates and maps the pages), else
 * fallocate (allocates them); where neither exists nothing is reserved and
 * the SIGBUS guard is what remains. */
static int populate(mapout_t *m, int c, size_t a, size_t n) {
  /* (mode is shared by the prefault threads: atomic loads and stores) */
  if (__atomic_load_n(&m->mode, __ATOMIC_RELAXED) == MAPOUT_POPULATE) {
    for (;;) {
      if (madvise(m->map[c] + a, n, MADV_POPULATE_WRITE) == 0) return 0;
      if (errno == EINTR || errno == EAGAIN) continue;
      if (errno != EINVAL) return -1;
      __atomic_store_n(&m->mode, MAPOUT_FALLOCATE, __ATOMIC_RELAXED);   /* (a kernel without MADV_POPULATE_WRITE) */
      break;
    }
  }
  if (__atomic_load_n(&m->mode, __ATOMIC_RELAXED) == MAPOUT_FALLOCATE) {
    for (;;) {
      const int e = posix_fallocate(m->fd[c], (off_t)a, (off_t)n);
      if (e == 0) return 0;
      if (e == EINTR) continue;
      if (e != EOPNOTSUPP && e != EINVAL) return -1;
      __atomic_store_n(&m->mode, MAPOUT_UNRESERVED, __ATOMIC_RELAXED);   /* (neither: first-touch faults, SIGBUS guard) */
      break;
    }
  }
  return 0;
}

static void *pf_main(void *arg) {
  mapout_t *m = arg;
  pthread_mutex_lock(&m->mu);
  for (;;) {
    int c = -1;
    for (int k = 0; k < 2; ++k)   /* the output furthest behind its target */
      if (m->map[k] && m->next[k] < m->want[k] &&
          (c < 0 || m->want[k] - m->next[k] > m->want[c] - m->next[c]))
        c = k;
    if (c < 0 || m->err) {
      if (m->stop) break;
      pthread_cond_wait(&m->cv, &m->mu);
      continue;
    }
    const size_t a = m->next[c];
    const size_t n = a + m->window < m->cap ? m->window : m->cap - a;
    m->next[c] = a + n;
    pthread_mutex_unlock(&m->mu);
    const int bad = (m->hook & MAPOUT_HOOK_POPULATE_FAIL) || populate(m, c, a, n);
    pthread_mutex_lock(&m->mu);
    if (bad && !m->err) m->err = HPGQ_E_IO;
  }
  pthread_mutex_unlock(&m->mu);
  return NULL;
}

static void unmap_all(mapout_t *m) {
  for (int c = 0; c < 2; ++c) {
    if (m->map[c]) munmap(m->map[c], m->cap);
    m->map[c] = NULL;
  }
}

int mapout_open(mapout_t *m, const int fd[2], size_t cap, size_t ahead, int threads, int hook) {
  memset(m, 0, sizeof(*m));
  m->fd[0] = fd[0];
  m->fd[1] = fd[1];
  m->cap = cap;
  m->window = (size_t)32 << 20;
  m->ahead = ahead > m->window ? ahead : m->window;
  m->hook = hook;
  int nout = 0;
  for (int c = 0; c < 2; ++c) {
    if (fd[c] < 0) continue;
    struct stat st;
    if (fstat(fd[c], &st) || !S_ISREG(st.st_mode) || dense_fs(fd[c])) return 1;
    nout++;
  }
  if (!nout) return 1;
  /* room for the outputs together (at most the input) plus slack; the
   * reservation below and the prefault threads check the rest as they go */
  struct statvfs vs;
  const int f0 = fd[0] >= 0 ? fd[0] : fd[1];
  if (fstatvfs(f0, &vs) || (unsigned long long)vs.f_bavail * vs.f_frsize < (unsigned long long)cap + (64ull << 20))
    return 1;
  int rc = 0;
  for (int c = 0; c < 2 && rc == 0; ++c) {
    if (fd[c] < 0) continue;
    if (ftruncate(fd[c], (off_t)cap)) rc = 1;
    void *p = rc ? MAP_FAILED : mmap(NULL, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd[c], 0);
    if (p == MAP_FAILED) rc = 1;
    else m->map[c] = p;
  }
  /* reserve the first window of each output now: a file system that cannot
   * back it sends the caller to the stream writer before anything is copied */
  for (int c = 0; c < 2 && rc == 0; ++c) {
    if (!m->map[c]) continue;
    const size_t n = m->window < cap ? m->window : cap;
    if ((hook & MAPOUT_HOOK_RESERVE_FAIL) || populate(m, c, 0, n)) rc = 1;
    m->next[c] = m->want[c] = n;
  }
  if (rc == 0 && (hook & MAPOUT_HOOK_SIGBUS) && m->map[0] && ftruncate(fd[0], 0)) rc = 1;
  if (rc) {
    unmap_all(m);
    for (int c = 0; c < 2; ++c)
      if (fd[c] >= 0 && ftruncate(fd[c], 0)) return HPGQ_E_IO;
    return 1;
  }
  pthread_mutex_init(&m->mu, NULL);
  pthread_cond_init(&m->cv, NULL);
  m->live = 1;
  if (threads < 0) threads = 0;   /* (0: only the reserved first window; copies fault the rest in) */
  if (threads > MAPOUT_MAX_PF) threads = MAPOUT_MAX_PF;
  for (int t = 0; t < threads; ++t) {
    if (pthread_create(&m->th[t], NULL, pf_main, m)) break;
    m->nth++;
  }
  return 0;
}

void mapout_advance(mapout_t *m, int c, size_t placed) {
  if (!m->map[c]) return;
  size_t w = placed + m->ahead;
  if (w > m->cap) w = m->cap;
  pthread_mutex_lock(&m->mu);
  if (w > m->want[c]) {
    m->want[c] = w;
    pthread_cond_broadcast(&m->cv);
  }
  pthread_mutex_unlock(&m->mu);
}

int mapout_error(mapout_t *m) {
  pthread_mutex_lock(&m->mu);
  const int e = m->err;
  pthread_mutex_unlock(&m->mu);
  return e;
}

/* ---- SIGBUS guard ---------------------------------------------------------- */

static __thread sigjmp_buf *g_jb;   /* the guarded call on this thread, if any */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static struct sigaction g_prev;

static void on_sigbus(int sig, siginfo_t *si, void *uc) {
  if (g_jb) siglongjmp(*g_jb, 1);
  /* not a guarded store: whatever was installed before (default: terminate) */
  if (g_prev.sa_flags & SA_SIGINFO) {
    if (g_prev.sa_sigaction) g_prev.sa_sigaction(sig, si, uc);
    return;
  }
  if (g_prev.sa_handler != SIG_IGN && g_prev.sa_handler != SIG_DFL && g_prev.sa_handler) {
    g_prev.sa_handler(sig);
    return;
  }
  signal(SIGBUS, SIG_DFL);
  raise(SIGBUS);
}

static int is_ours(const struct sigaction *a) { return (a->sa_flags & SA_SIGINFO) && a->sa_sigaction == on_sigbus; }

/* on_sigbus is the SIGBUS handler at every guarded copy: installed at the
 * first one, and again whenever a runtime or library installed its own since
 *  -- that one then becomes the handler unguarded faults chain to */
static void ensure_installed(void) {
  struct sigaction cur;
  if (sigaction(SIGBUS, NULL, &cur) == 0 && is_ours(&cur)) return;
  pthread_mutex_lock(&g_mu);
  if (sigaction(SIGBUS, NULL, &cur) != 0 || !is_ours(&cur)) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_sigbus;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGBUS, &sa, &g_prev);
  }
  pthread_mutex_unlock(&g_mu);
}

int mapout_guard(void (*fn)(void *), void *arg) {
  ensure_installed();
  sigjmp_buf jb;
  if (sigsetjmp(jb, 1)) {   /* (the mask is restored: SIGBUS unblocked again) */
    g_jb = NULL;
    return HPGQ_E_IO;
  }
  g_jb = &jb;
  fn(arg);
  g_jb = NULL;
  return 0;
}

int mapout_close(mapout_t *m, const uint64_t size[2]) {
  int rc = 0;
  if (m->live) {
    pthread_mutex_lock(&m->mu);
    m->stop = 1;
    pthread_cond_broadcast(&m->cv);
    pthread_mutex_unlock(&m->mu);
    for (int t = 0; t < m->nth; ++t) pthread_join(m->th[t], NULL);
    m->nth = 0;
    rc = m->err;
    pthread_mutex_destroy(&m->mu);
    pthread_cond_destroy(&m->cv);
    m->live = 0;
  }
  const int mapped = m->map[0] || m->map[1];
  unmap_all(m);
  for (int c = 0; c < 2 && mapped; ++c)
    if (m->fd[c] >= 0 && ftruncate(m->fd[c], (off_t)size[c]) && rc == 0) rc = HPGQ_E_IO;
  return rc;
}
