// hpgq_common.h — internal helpers shared by the libhpgq translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../include/hpgq.h"

#define HPGQ_HIP_TRY(expr)                                                     \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      std::fprintf(stderr, "hpgq: %s failed: %s (%s:%d)\n", #expr,             \
                   hipGetErrorString(_e), __FILE__, __LINE__);                 \
      return HPGQ_E_HIP;                                                       \
    }                                                                          \
  } while (0)

namespace hpgq {

// splitmix64 finalizer; the synthetic generator is counter based so any
// shard / GPU regenerates its slice.
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__host__ __device__ inline uint64_t synth_read_key(uint64_t seed, int64_t idx) {
  return mix64(seed * 0x9E3779B97F4A7C15ULL + (uint64_t)idx);
}

__host__ __device__ inline int32_t synth_length(uint64_t seed, int32_t L0, int32_t trunc_pct,
                                                int64_t idx) {
  uint64_t r = synth_read_key(seed, idx);
  int32_t L = L0;
  if (L0 >= 20 && (int32_t)(r % 100) < trunc_pct)
    L = 20 + (int32_t)(mix64(r ^ 1ULL) % (uint64_t)(L0 - 20 + 1));
  return L;
}

}  // namespace hpgq
