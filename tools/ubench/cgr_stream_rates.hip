// Streaming probe for cgr_stream_kernel's access shape on gfx950 (round 4,
// VERDICT r3 item 3): one 1024-thread workgroup per CU (a 136 KB LDS
// allocation, as the 128 KB k = 7 table forces), wave g walks 16 KB spans
// g, g + W, ... as 2 KB tiles, a lane 32 contiguous bytes of seq and of
// quality per tile (two 16-byte loads each).  How fast can that read the
// C5 call's 2 x 1.25 GB when
//   D      tiles fetched ahead of the one being counted (1: the product's
//          double buffer; 2: HPGQ_C5_DEPTH 3; 3, 4: deeper)
//   work   dependent full-rate VALU pairs per lane and tile (v_alignbit +
//          v_add) between a tile's arrival and the next (0: pure streaming;
//          165: the product's ~330 VALU per tile)
//   lds    0: no LDS allocation (the same grid at up to 2 workgroups per CU)
// Each lane XOR-folds what it loads (kept alive through one store per lane).
//   hipcc --offload-arch=gfx950 -O3 cgr_stream_rates.hip -o cgr_stream_rates && ./cgr_stream_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kWG = 1024;
constexpr int kSpan = 16384, kTile = 2048;
constexpr uint32_t kN = 1250000000u;   // 5 M x 250 bytes per buffer

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n, 0x00020000);
}

struct Buf { v4u s0, s1, q0, q1; };

__device__ __forceinline__ Buf load_tile(__amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rq, uint32_t o) {
  Buf b;
  b.s0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
  b.s1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, 0);
  b.q0 = __builtin_amdgcn_raw_buffer_load_b128(rq, o, 0, 0);
  b.q1 = __builtin_amdgcn_raw_buffer_load_b128(rq, o + 16, 0, 0);
  return b;
}

template <int D, bool LDS>
__global__ void __launch_bounds__(kWG) k_stream(const char *a, const char *b, uint32_t *out, int work) {
  __shared__ uint32_t pad[LDS ? 34 * 1024 : 1];
  const auto rs = rsrc(a, kN), rq = rsrc(b, kN);
  const int lane = threadIdx.x & 63;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (kWG / 64) + (threadIdx.x >> 6));
  const int nw = gridDim.x * (kWG / 64);
  const int ns = (kN + kSpan - 1) / kSpan;
  const int tiles_per_span = kSpan / kTile;
  // the wave's tile stream: tile i = span gw + (i / 8) * nw, tile i % 8
  const int nspan_w = gw < ns ? (ns - gw + nw - 1) / nw : 0;
  const int nt = nspan_w * tiles_per_span;
  auto off = [&](int i) -> uint32_t {
    if (i >= nt) return kN;   // past the range: zeros, no traffic
    const int64_t s = gw + (int64_t)(i / tiles_per_span) * nw;
    return (uint32_t)(s * kSpan + (i % tiles_per_span) * kTile + 32 * lane);
  };
  uint32_t x = threadIdx.x;
  Buf buf[D];
#pragma unroll
  for (int d = 0; d < D; ++d) buf[d] = load_tile(rs, rq, off(d));
  for (int i = 0; i < nt; i += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const Buf c = buf[d];
      buf[d] = load_tile(rs, rq, off(i + d + D));
      uint32_t y = c.s0.x ^ c.s0.y ^ c.s0.z ^ c.s0.w ^ c.s1.x ^ c.s1.y ^ c.s1.z ^ c.s1.w ^
                   c.q0.x ^ c.q0.y ^ c.q0.z ^ c.q0.w ^ c.q1.x ^ c.q1.y ^ c.q1.z ^ c.q1.w;
      for (int k = 0; k < work; ++k) y = __builtin_amdgcn_alignbit(y, y, 7) + 0x9E3779B1u;
      x ^= y;
    }
  }
  if (LDS) {
    pad[threadIdx.x] = x;
    __syncthreads();
    x ^= pad[(threadIdx.x + 64) & (kWG - 1)];
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

template <int D, bool LDS>
static void run(const char *a, const char *b, uint32_t *out, int grid, int work) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 2; ++w) k_stream<D, LDS><<<grid, kWG>>>(a, b, out, work);
  const int it = 10;
  hipEventRecord(e0);
  for (int w = 0; w < it; ++w) k_stream<D, LDS><<<grid, kWG>>>(a, b, out, work);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1e3 * ms / it;
  printf("{\"D\": %d, \"lds\": %d, \"grid\": %d, \"work\": %d, \"us\": %.1f, \"TB_s\": %.3f}\n", D, (int)LDS, grid,
         work, us, 2.0 * kN / (us * 1e-6) / 1e12);
  fflush(stdout);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main(int argc, char **argv) {
  char *a, *b;
  uint32_t *out;
  if (hipMalloc(&a, kN + 4096) || hipMalloc(&b, kN + 4096) || hipMalloc(&out, 4096 * kWG * 4)) return 1;
  hipMemset(a, 0x41, kN);
  hipMemset(b, 0x28, kN);
  hipDeviceSynchronize();
  // work values (dependent VALU pairs per lane and tile) from the command line
  // (round 6: pricing VALU cuts per byte for C5)
  std::vector<int> works = {0, 80, 165, 250};
  if (argc > 1) {
    works.clear();
    for (int i = 1; i < argc; ++i) works.push_back(atoi(argv[i]));
  }
  for (int work : works) {
    run<1, true>(a, b, out, 256, work);
    run<2, true>(a, b, out, 256, work);
    run<3, true>(a, b, out, 256, work);
    run<4, true>(a, b, out, 256, work);
  }
  run<2, false>(a, b, out, 512, 0);
  run<4, false>(a, b, out, 512, 0);
  hipFree(a);
  hipFree(b);
  hipFree(out);
  return 0;
}
