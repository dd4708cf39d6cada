// Window-gather probe for the --kmers tile kernel's access shapes on gfx950:
// every read (150 bytes, packed back to back, unaligned) is visited once per
// 32-position tile, and each visit needs the 36 bytes [a + 32t, a + 32t + 36).
// How fast can a persistent grid gather those windows when
//   lane1   one lane per read: two 16-byte loads and one 4-byte load
//   lane2   two lanes per read: a 16-byte and a 4-byte load each (20 bytes)
//   lane4   four lanes per read: one 16-byte load each (48 bytes, 12 wasted)
//   dword9  nine lanes per read, one 4-byte load each (7 reads per wave load)
//   flat    the whole batch as contiguous 16-byte lane loads, once per tile
//           (150 bytes per read and tile: what staging whole reads costs)
//   lane1_68x3  one lane per read, 64-position tiles: 68-byte windows, 3 tiles
//           (window_TB_s still counts 5 x 36 bytes per read: the same work)
//   lane2_same, lane2_aligned  k_lanes<2> again, and with dword-aligned loads
//           (b128 + b64 from the dword below, v_alignbyte into place)
//   lane2_68x3, lane2_68x2_36  two lanes per read, 64-position tiles (36
//           bytes per lane), three of them / two and a 32-position tail
// Each lane XOR-folds what it loads (kept alive through one store per lane).
// The tiles of a read are visited back to back, so tiles 1..4 hit the cache:
// the time is the load path (TA, L1/L2), not HBM.
//   hipcc --offload-arch=gfx950 -O3 window_rates.hip -o window_rates && ./window_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kWG = 1024;
constexpr int kL = 150;
constexpr int kTiles = 5;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n, 0x00020000);
}

// LPR lanes per read; lane part k loads bytes [a + 32t + 16k, ...)
template <int LPR>
__global__ void __launch_bounds__(kWG) k_lanes(const char *s, uint32_t nreads, uint32_t *out) {
  const auto rs = rsrc(s, nreads * kL + 64);
  constexpr int kRpw = 64 / LPR;
  const int lane = threadIdx.x & 63, part = lane % LPR;
  uint32_t x = 0;
  const uint32_t nw = gridDim.x * (kWG / 64);
  for (uint32_t g = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6); g * kRpw < nreads; g += nw) {
    const uint32_t r = g * kRpw + lane / LPR;
    const uint32_t a = (r < nreads ? r : 0) * kL;
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
      const uint32_t o = a + 32 * t;
      if (LPR == 1) {
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
        const v4u q = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, 0);
        x ^= p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w ^ __builtin_amdgcn_raw_buffer_load_b32(rs, o + 32, 0, 0);
      } else if (LPR == 2) {
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16 * part, 0, 0);
        x ^= p.x ^ p.y ^ p.z ^ p.w ^ __builtin_amdgcn_raw_buffer_load_b32(rs, o + 16 * part + 16, 0, 0);
      } else {
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16 * part, 0, 0);
        x ^= p.x ^ p.y ^ p.z ^ p.w;
      }
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// one lane per read, 64-position tiles (68-byte windows: four 16-byte and
// one 4-byte load), three tiles per 150 bp read
__global__ void __launch_bounds__(kWG) k_lane1_68(const char *s, uint32_t nreads, uint32_t *out) {
  const auto rs = rsrc(s, nreads * kL + 128);
  const int lane = threadIdx.x & 63;
  uint32_t x = 0;
  const uint32_t nw = gridDim.x * (kWG / 64);
  for (uint32_t g = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6); g * 64 < nreads; g += nw) {
    const uint32_t r = g * 64 + lane;
    const uint32_t a = (r < nreads ? r : 0) * kL;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const uint32_t o = a + 64 * t;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16 * k, 0, 0);
        x ^= p.x ^ p.y ^ p.z ^ p.w;
      }
      x ^= __builtin_amdgcn_raw_buffer_load_b32(rs, o + 64, 0, 0);
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// two lanes per read, 64-position tiles (round 4): lane k of a read takes
// starts 32k..32k+31 of a tile, a 36-byte window (two 16-byte loads and one
// 4-byte load); TAIL: the 150 bp read's third visit is a 32-position tile
// (a 16-byte and a 4-byte load per lane, as k_lanes<2>) instead of a third
// 64-position one
template <bool TAIL>
__global__ void __launch_bounds__(kWG) k_lane2_64(const char *s, uint32_t nreads, uint32_t *out) {
  const auto rs = rsrc(s, nreads * kL + 128);
  const int lane = threadIdx.x & 63, part = lane & 1;
  uint32_t x = 0;
  const uint32_t nw = gridDim.x * (kWG / 64);
  for (uint32_t g = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6); g * 32 < nreads; g += nw) {
    const uint32_t r = g * 32 + (lane >> 1);
    const uint32_t a = (r < nreads ? r : 0) * kL;
#pragma unroll
    for (int t = 0; t < (TAIL ? 2 : 3); ++t) {
      const uint32_t o = a + 64 * t + 32 * part;
      const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
      const v4u q = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, 0);
      x ^= p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w ^ __builtin_amdgcn_raw_buffer_load_b32(rs, o + 32, 0, 0);
    }
    if (TAIL) {
      const uint32_t o = a + 128 + 16 * part;
      const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
      x ^= p.x ^ p.y ^ p.z ^ p.w ^ __builtin_amdgcn_raw_buffer_load_b32(rs, o + 16, 0, 0);
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// k_lanes<2> with dword-aligned loads: the 150-byte reads start at even
// offsets only, so a window's 16-byte load is misaligned by 2 bytes half the
// time; ALIGN loads the 24 bytes from the dword below instead (a b128 and a
// b64) and shifts them into place with v_alignbyte (what the kernel would do)
template <bool ALIGN>
__global__ void __launch_bounds__(kWG) k_lane2_al(const char *s, uint32_t nreads, uint32_t *out) {
  const auto rs = rsrc(s, nreads * kL + 64);
  const int lane = threadIdx.x & 63, part = lane & 1;
  uint32_t x = 0;
  const uint32_t nw = gridDim.x * (kWG / 64);
  for (uint32_t g = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6); g * 32 < nreads; g += nw) {
    const uint32_t r = g * 32 + (lane >> 1);
    const uint32_t a = (r < nreads ? r : 0) * kL;
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
      const uint32_t o = a + 32 * t + 16 * part;
      if (ALIGN) {
        const uint32_t sh = o & 3u;
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o & ~3u, 0, 0);
        const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rs, (o & ~3u) + 16, 0, 0);
        const uint32_t w[6] = {p.x, p.y, p.z, p.w, q.x, q.y};
#pragma unroll
        for (int i = 0; i < 5; ++i) x ^= __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
      } else {
        const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
        x ^= p.x ^ p.y ^ p.z ^ p.w ^ __builtin_amdgcn_raw_buffer_load_b32(rs, o + 16, 0, 0);
      }
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// nine lanes per read (lanes 63 idle), one dword each
__global__ void __launch_bounds__(kWG) k_dword9(const char *s, uint32_t nreads, uint32_t *out) {
  const auto rs = rsrc(s, nreads * kL + 64);
  const int lane = threadIdx.x & 63, part = lane % 9;
  uint32_t x = 0;
  const uint32_t nw = gridDim.x * (kWG / 64);
  for (uint32_t g = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6); g * 7 < nreads; g += nw) {
    const uint32_t r = g * 7 + lane / 9;
    const uint32_t a = (r < nreads && lane < 63 ? r : 0) * kL;
#pragma unroll
    for (int t = 0; t < kTiles; ++t) x ^= __builtin_amdgcn_raw_buffer_load_b32(rs, a + 32 * t + 4 * part, 0, 0);
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

__global__ void __launch_bounds__(kWG) k_flat(const char *s, uint32_t nreads, uint32_t *out) {
  const uint32_t n = nreads * kL;
  const auto rs = rsrc(s, n + 64);
  uint32_t x = 0;
  const uint32_t step = gridDim.x * kWG * 16;
  for (uint32_t o = (blockIdx.x * kWG + threadIdx.x) * 16; o < n; o += step) {
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
      uint32_t oo = o;
      asm volatile("" : "+v"(oo));   // a fresh load per tile (the same bytes: cache hits)
      const v4u p = __builtin_amdgcn_raw_buffer_load_b128(rs, oo, 0, 0);
      x ^= p.x ^ p.y ^ p.z ^ p.w;
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

int main() {
  const uint32_t nreads = 10000000;
  char *d;
  uint32_t *o;
  hipMalloc(&d, (size_t)nreads * kL + 128);
  hipMemset(d, 0x41, (size_t)nreads * kL + 128);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus;
  hipMalloc(&o, (size_t)grid * kWG * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    hipEventRecord(e0);
    const int it = 5;
    for (int i = 0; i < it; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / it;
    // "window bytes": 36 per read and tile
    printf("{\"shape\": \"%s\", \"us\": %.1f, \"window_TB_s\": %.3f}\n", name, us,
           36.0 * kTiles * nreads / (us * 1e-6) / 1e12);
  };
  run("lane1", [&] { hipLaunchKernelGGL(k_lanes<1>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane2", [&] { hipLaunchKernelGGL(k_lanes<2>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane4", [&] { hipLaunchKernelGGL(k_lanes<4>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("dword9", [&] { hipLaunchKernelGGL(k_dword9, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("flat", [&] { hipLaunchKernelGGL(k_flat, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane1_68x3", [&] { hipLaunchKernelGGL(k_lane1_68, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane2_68x3", [&] { hipLaunchKernelGGL(k_lane2_64<false>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane2_same", [&] { hipLaunchKernelGGL(k_lane2_al<false>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane2_aligned", [&] { hipLaunchKernelGGL(k_lane2_al<true>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  run("lane2_68x2_36", [&] { hipLaunchKernelGGL(k_lane2_64<true>, dim3(grid), dim3(kWG), 0, 0, d, nreads, o); });
  hipFree(d);
  hipFree(o);
  return 0;
}
