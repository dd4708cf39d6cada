// hpgq_host.cpp — the host-only part of the libhpgq C-ABI (no HIP): parameter
// defaults, error strings and the derived summary of a counter set.  Built
// with the host compiler into libhpgq.so, and on its own into the sanitizer
// builds of the host code (tests/sanitize/).
#include <cstdint>
#include <cstring>

#include "hpgq.h"

extern "C" {

void hpgq_params_init(hpgq_params_t *p) {
  std::memset(p, 0, sizeof(*p));
  p->phred = HPGQ_PHRED33;
  p->lmax = 256;
  p->stats_on = 1;
  p->min_read_length = HPGQ_MIN_VALUE;
  p->max_read_length = HPGQ_MAX_VALUE;
  p->min_read_quality = HPGQ_MIN_VALUE;
  p->max_read_quality = HPGQ_MAX_VALUE;
  p->max_out_of_quality = HPGQ_MAX_VALUE;
  p->left_length = HPGQ_MIN_VALUE;
  p->min_left_quality = HPGQ_MIN_VALUE;
  p->max_left_quality = HPGQ_MAX_VALUE;
  p->right_length = HPGQ_MIN_VALUE;
  p->min_right_quality = HPGQ_MIN_VALUE;
  p->max_right_quality = HPGQ_MAX_VALUE;
  p->max_N = HPGQ_MAX_VALUE;
  p->edit_left_length = HPGQ_MIN_VALUE;
  p->edit_min_left_quality = HPGQ_MIN_VALUE;
  p->edit_max_left_quality = HPGQ_MAX_VALUE;
  p->edit_right_length = HPGQ_MIN_VALUE;
  p->edit_min_right_quality = HPGQ_MIN_VALUE;
  p->edit_max_right_quality = HPGQ_MAX_VALUE;
}

const char *hpgq_strerror(int code) {
  switch (code) {
    case HPGQ_OK: return "ok";
    case HPGQ_E_INVALID: return "invalid argument";
    case HPGQ_E_HIP: return "HIP runtime error";
    case HPGQ_E_NOMEM: return "out of memory";
    case HPGQ_E_READ_TOO_LONG: return "read longer than lmax";
    case HPGQ_E_NO_DEVICE: return "no HIP device";
    case HPGQ_E_RCCL: return "RCCL error";
    case HPGQ_E_STATE: return "invalid ctx state";
    case HPGQ_E_FORMAT: return "malformed FASTQ text";
    case HPGQ_E_IO: return "file i/o error";
    default: return "unknown error";
  }
}

const char *hpgq_version(void) { return "hpgq 0.2 (gfx950)"; }


// ---------------------------------------------------------------------------
// derived summary (stats_counters_t view)
// ---------------------------------------------------------------------------

int hpgq_counters_summary(const uint64_t *set, int lmax, hpgq_summary_t *o) {
  if (!set || !o || lmax < 1) return HPGQ_E_INVALID;
  std::memset(o, 0, sizeof(*o));
  o->num_input = set[HPGQ_S_NUM_INPUT];
  o->num_passed = set[HPGQ_S_NUM_PASSED];
  o->num_failed = set[HPGQ_S_NUM_FAILED];
  o->num_edited = set[HPGQ_S_NUM_EDITED];
  o->num_reads = set[HPGQ_S_NUM_STATS];
  o->min_length = 100000;   // stats_counters_new, src/stats_fastq.c:108-109
  o->max_length = 0;
  const uint64_t *hl = set + hpgq_off_hist_len(lmax);
  for (int L = 0; L <= lmax; ++L) {
    if (!hl[L]) continue;
    if (L < o->min_length) o->min_length = L;
    if (L > o->max_length) o->max_length = L;
    o->acc_length += (uint64_t)L * hl[L];
  }
  uint64_t *tot[5] = {&o->num_A, &o->num_C, &o->num_G, &o->num_T, &o->num_N};
  for (int b = 0; b < 5; ++b) {
    const uint64_t *pb = set + hpgq_off_pos_base(lmax, b);
    for (int j = 0; j < lmax; ++j) *tot[b] += pb[j];
  }
  if (o->num_reads) {
    o->mean_length = (double)o->acc_length / (double)o->num_reads;
    o->mean_quality_raw = (double)(int64_t)set[HPGQ_S_ACC_MEANQ_FX16] / 65536.0 / (double)o->num_reads;
  }
  return HPGQ_OK;
}

}  // extern "C"
