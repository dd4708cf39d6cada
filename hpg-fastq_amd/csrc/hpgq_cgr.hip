// hpgq_cgr.hip — chaos-game accumulator (placeholder until the kernel lands)
#include "hpgq_common.h"
struct hpgq_cgr { int dummy; };
extern "C" {
int hpgq_cgr_open(hpgq_cgr_t **cg, int, int, int) { if (cg) *cg = nullptr; return HPGQ_E_STATE; }
void hpgq_cgr_close(hpgq_cgr_t *) {}
int hpgq_cgr_fill_device(hpgq_cgr_t *, const hpgq_batch_t *, const uint8_t *, int) { return HPGQ_E_STATE; }
int hpgq_cgr_sync(hpgq_cgr_t *) { return HPGQ_E_STATE; }
int hpgq_cgr_reset(hpgq_cgr_t *) { return HPGQ_E_STATE; }
int hpgq_cgr_read(hpgq_cgr_t *, uint32_t *, uint32_t *, uint32_t *) { return HPGQ_E_STATE; }
void *hpgq_cgr_stream(hpgq_cgr_t *) { return nullptr; }
int64_t hpgq_cgr_last_replays(hpgq_cgr_t *) { return 0; }
}
