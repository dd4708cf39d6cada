// hpgq_synth.hip — deterministic synthetic FASTQ batches, generated in HBM.
//
// Bench/test input only: counter-based (splitmix64 of the seed
// and the read index), so any rank regenerates its own shard without moving
// bytes, and the CPU oracle regenerates exactly the same reads.
//   length : L, or U[20, L] for trunc_pct % of reads
//   base   : 'N' with p = n_per_1024/1024, else uniform A/C/G/T
//   quality: clamp(40 - 20*j/L + U[-6,6], 2, 41) + phred; bad_pct % of reads
//            centred at 12 instead
// One wave per read: lane j writes base j (coalesced byte stores).

#include "hpgq_common.h"
#include <vector>

namespace hpgq {

__global__ void __launch_bounds__(256) synth_kernel(hpgq_synth_t s, int64_t first, int64_t n,
                                                    char *seq, char *qual, const int32_t *idx) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const char acgt[4] = {'A', 'C', 'G', 'T'};
  for (int64_t i = wave0; i < n; i += nwaves) {
    const uint64_t r = synth_read_key(s.seed, first + i);
    const uint64_t mk = s.mate ? mix64(r ^ 0x5EEDULL) : r;
    const bool bad = (int32_t)((mk >> 20) % 100) < s.bad_pct;
    const int32_t a = idx[i], L = idx[i + 1] - idx[i];
    for (int32_t j = lane; j < L; j += 64) {
      const uint64_t h = mix64(mk + (uint64_t)(j + 1) * 0xD1B54A32D192ED03ULL);
      const char b = ((int32_t)(h & 1023) < s.n_per_1024) ? 'N' : acgt[(h >> 10) & 3];
      const int32_t noise = (int32_t)((h >> 12) % 13) - 6;
      int32_t q = bad ? 12 + noise : 40 - (20 * j) / L + noise;
      q = q < 2 ? 2 : (q > 41 ? 41 : q);
      seq[a + j] = b;
      qual[a + j] = (char)(q + s.phred);
    }
  }
}

}  // namespace hpgq

extern "C" {

int32_t hpgq_synth_length(const hpgq_synth_t *s, int64_t idx) {
  return hpgq::synth_length(s->seed, s->read_length, s->trunc_pct, idx);
}

int hpgq_synth_indices_host(const hpgq_synth_t *s, int64_t first, int64_t n, int32_t *idx) {
  if (!s || !idx || n < 0) return HPGQ_E_INVALID;
  int64_t acc = 0;
  idx[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    acc += hpgq::synth_length(s->seed, s->read_length, s->trunc_pct, first + i);
    if (acc > INT32_MAX) return HPGQ_E_INVALID;   // batch must stay < 2 GiB (int offsets)
    idx[i + 1] = (int32_t)acc;
  }
  return HPGQ_OK;
}

int hpgq_synth_device(const hpgq_synth_t *s, int64_t first, int64_t n, char *seq_dev,
                      char *qual_dev, const int32_t *idx_dev, void *stream) {
  if (!s || n < 0 || !seq_dev || !qual_dev || !idx_dev) return HPGQ_E_INVALID;
  if (n == 0) return HPGQ_OK;
  const int64_t waves = n < 65536 ? n : 65536;
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL(hpgq::synth_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *s,
                     first, n, seq_dev, qual_dev, idx_dev);
  HPGQ_HIP_TRY(hipGetLastError());
  return HPGQ_OK;
}

}  // extern "C"
