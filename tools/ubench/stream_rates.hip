// Streaming-read probe for the engine's access shapes on gfx950: how fast can
// a persistent grid read two byte buffers (seq + quality) when each lane takes
//   x4     16 contiguous bytes per load (fully coalesced 1 KB per wave-load)
//   x2      8 contiguous bytes per load
//   tri    the three-read kernel's shape: 3 reads per wave step, 20 lanes x 8 B
//          of a 150-byte read starting at its (unaligned, dword-rounded) offset
//   hex    6 reads per step, 10 lanes x 16 B of a 150-byte read
// Each lane XOR-folds what it loads (kept alive through one store per lane).
//   hipcc --offload-arch=gfx950 -O3 stream_rates.hip -o stream_rates && ./stream_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kWG = 256;
constexpr int kL = 150;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n, 0x00020000);
}

template <int W>   // bytes per lane per load: 8 or 16
__global__ void __launch_bounds__(kWG) k_flat(const char *a, const char *b, uint32_t n, uint32_t *out, int unroll) {
  const auto ra = rsrc(a, n), rb = rsrc(b, n);
  uint32_t x = 0;
  const uint32_t step = gridDim.x * kWG * W;
  for (uint32_t o = (blockIdx.x * kWG + threadIdx.x) * W; o < n; o += step) {
    if (W == 16) {
      const v4u p = __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, 0);
      const v4u q = __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, 0);
      x ^= p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w;
    } else {
      const v2u p = __builtin_amdgcn_raw_buffer_load_b64(ra, o, 0, 0);
      const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rb, o, 0, 0);
      x ^= p.x ^ p.y ^ q.x ^ q.y;
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// lane owns 32 contiguous bytes: two 16-byte loads at stride 32 (each wave
// load touches twice the cache lines of a contiguous one); U tiles in flight
template <int U>
__global__ void __launch_bounds__(kWG) k_s32(const char *a, const char *b, uint32_t n, uint32_t *out) {
  const auto ra = rsrc(a, n), rb = rsrc(b, n);
  uint32_t x = 0;
  const uint32_t step = gridDim.x * kWG * 32;
  for (uint32_t o = (blockIdx.x * kWG + threadIdx.x) * 32; o < n; o += U * step) {
    v4u p[U][2], q[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      p[u][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, o + u * step, 0, 0);
      p[u][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, o + u * step + 16, 0, 0);
      q[u][0] = __builtin_amdgcn_raw_buffer_load_b128(rb, o + u * step, 0, 0);
      q[u][1] = __builtin_amdgcn_raw_buffer_load_b128(rb, o + u * step + 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      for (int h = 0; h < 2; ++h) x ^= p[u][h].x ^ p[u][h].y ^ p[u][h].z ^ p[u][h].w ^ q[u][h].x ^ q[u][h].y ^ q[u][h].z ^ q[u][h].w;
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// contiguous 16-byte lanes, two wave loads 1 KB apart (same bytes per lane as k_s32)
template <int U>
__global__ void __launch_bounds__(kWG) k_c16(const char *a, const char *b, uint32_t n, uint32_t *out) {
  const auto ra = rsrc(a, n), rb = rsrc(b, n);
  uint32_t x = 0;
  const uint32_t step = gridDim.x * kWG * 32;
  const int lane = threadIdx.x & 63;
  for (uint32_t o = (blockIdx.x * kWG + (threadIdx.x & ~63)) * 32 + 16 * lane; o < n; o += U * step) {
    v4u p[U][2], q[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      p[u][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, o + u * step, 0, 0);
      p[u][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, o + u * step + 1024, 0, 0);
      q[u][0] = __builtin_amdgcn_raw_buffer_load_b128(rb, o + u * step, 0, 0);
      q[u][1] = __builtin_amdgcn_raw_buffer_load_b128(rb, o + u * step + 1024, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      for (int h = 0; h < 2; ++h) x ^= p[u][h].x ^ p[u][h].y ^ p[u][h].z ^ p[u][h].w ^ q[u][h].x ^ q[u][h].y ^ q[u][h].z ^ q[u][h].w;
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

// R reads per wave step, S lanes per read, W bytes per lane
template <int R, int S, int W>
__global__ void __launch_bounds__(kWG) k_reads(const char *a, const char *b, uint32_t n, const int32_t *idx,
                                              int64_t nreads, uint32_t *out) {
  const auto ra = rsrc(a, n + 64), rb = rsrc(b, n + 64);
  const int lane = threadIdx.x & 63;
  const int seg = lane / S, ls = lane - seg * S;
  const bool own = seg < R;
  uint32_t x = 0;
  const int64_t wave = (int64_t)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (kWG / 64);
  const int64_t nsteps = (nreads + R - 1) / R;
  for (int64_t st = wave; st < nsteps; st += nw) {
    const int64_t r = st * R + (own ? seg : 0);
    const int32_t off = r < nreads ? idx[r] : 0;
    const uint32_t o = (uint32_t)(off & ~3) + (uint32_t)(W * ls);
    if (W == 16) {
      const v4u p = __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, 0);
      const v4u q = __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, 0);
      x ^= p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w;
    } else {
      const v2u p = __builtin_amdgcn_raw_buffer_load_b64(ra, o, 0, 0);
      const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rb, o, 0, 0);
      x ^= p.x ^ p.y ^ q.x ^ q.y;
    }
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

int main() {
  const int64_t nreads = 10000000;
  const uint32_t n = (uint32_t)(nreads * kL);
  char *a, *b;
  int32_t *idx;
  uint32_t *out;
  hipMalloc(&a, n + 256);
  hipMalloc(&b, n + 256);
  hipMalloc(&idx, (nreads + 1) * 4);
  hipMemset(a, 1, n + 256);
  hipMemset(b, 2, n + 256);
  std::vector<int32_t> h(nreads + 1);
  for (int64_t i = 0; i <= nreads; ++i) h[i] = (int32_t)(i * kL);
  hipMemcpy(idx, h.data(), (nreads + 1) * 4, hipMemcpyHostToDevice);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipMalloc(&out, (size_t)cus * 64 * kWG * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, auto launch) {
    for (int occ : {4, 8, 16}) {
      const int grid = cus * occ;
      launch(grid);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 5; ++i) launch(grid);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double tbs = 2.0 * n * 5 / (ms * 1e-3) / 1e12;
      std::printf("%-5s grid %5d (%2d WG/CU): %.3f ms/pass  %.2f TB/s\n", name, grid, occ, ms / 5, tbs);
    }
  };
  run("x4", [&](int g) { k_flat<16><<<g, kWG>>>(a, b, n, out, 1); });
  run("x2", [&](int g) { k_flat<8><<<g, kWG>>>(a, b, n, out, 1); });
  run("s32u1", [&](int g) { k_s32<1><<<g, kWG>>>(a, b, n, out); });
  run("s32u2", [&](int g) { k_s32<2><<<g, kWG>>>(a, b, n, out); });
  run("c16u1", [&](int g) { k_c16<1><<<g, kWG>>>(a, b, n, out); });
  run("c16u2", [&](int g) { k_c16<2><<<g, kWG>>>(a, b, n, out); });
  run("tri", [&](int g) { k_reads<3, 21, 8><<<g, kWG>>>(a, b, n, idx, nreads, out); });
  run("hex", [&](int g) { k_reads<6, 10, 16><<<g, kWG>>>(a, b, n, idx, nreads, out); });
  return 0;
}
