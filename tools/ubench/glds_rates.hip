// Streaming-read probe: the hex segment shape (6 reads of 150 B per wave step,
// 10 lanes x 16 B each, dword-rounded offsets) with
//   reg<U>   a rolling two-group register pipeline, U steps per group (the
//            engine kernel's load pattern without its arithmetic)
//   glds<D>  LDS-DMA (buffer_load_dwordx4 ... lds) into a ring of D step slots
//            per wave, counted vmcnt, ds_read_b128 out of the oldest slot
// at 4 workgroups of 256 per CU (the engine's occupancy) and 8.  Offsets are
// r * 150 (no index loads).  Each lane XOR-folds what it reads.
//   hipcc --offload-arch=gfx950 -O3 glds_rates.hip -o glds_rates && ./glds_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kWG = 256;
constexpr int kL = 150;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n, 0x00020000);
}

__device__ __forceinline__ uint32_t hex_off(int64_t st, int64_t nreads, int seg, int ls) {
  const int64_t r = st * 6 + (seg < 6 ? seg : 0);
  return r < nreads ? (uint32_t)((r * kL) & ~3ll) + 16u * (uint32_t)ls : 0x80000000u;
}

template <int U>
__global__ void __launch_bounds__(kWG) k_reg(const char *a, const char *b, uint32_t n, int64_t nreads,
                                            uint32_t *out) {
  const auto ra = rsrc(a, n + 64), rb = rsrc(b, n + 64);
  const int lane = threadIdx.x & 63, seg = lane / 10, ls = lane - seg * 10;
  const int64_t wave = (int64_t)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (kWG / 64);
  const int64_t nsteps = (nreads + 5) / 6;
  const int64_t mine = wave < nsteps ? (nsteps - wave + nw - 1) / nw : 0;
  const int64_t ngroups = ((mine + U - 1) / U + 1) & ~1ll;
  v4u p[2][U], q[2][U];
  uint32_t x = 0;
  auto load = [&](int64_t g, int s) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = g * U + u;
      const uint32_t o = k < mine ? hex_off(wave + k * nw, nreads, seg, ls) : 0x80000000u;
      p[s][u] = __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, 0);
      q[s][u] = __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, 0);
    }
  };
  auto use = [&](int s) {
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= p[s][u].x ^ p[s][u].y ^ p[s][u].z ^ p[s][u].w ^ q[s][u].x ^ q[s][u].y ^ q[s][u].z ^ q[s][u].w;
  };
  load(0, 0);
  for (int64_t g = 0; g < ngroups; g += 2) {
    load(g + 1, 1);
    use(0);
    load(g + 2, 0);
    use(1);
  }
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

#define WAIT_VM(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")

template <int D, int AUX>
__global__ void __launch_bounds__(kWG) k_glds(const char *a, const char *b, uint32_t n, int64_t nreads,
                                             uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const auto ra = rsrc(a, n + 64), rb = rsrc(b, n + 64);
  const int lane = threadIdx.x & 63, seg = lane / 10, ls = lane - seg * 10;
  const int wv = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * (kWG / 64) + wv;
  const int64_t nw = (int64_t)gridDim.x * (kWG / 64);
  const int64_t nsteps = (nreads + 5) / 6;
  const int64_t mine = wave < nsteps ? (nsteps - wave + nw - 1) / nw : 0;
  uint8_t *wl = lds + wv * D * 2048;
  uint32_t x = 0;
  auto issue = [&](int64_t k, int slot) {
    const uint32_t o = k < mine ? hex_off(wave + k * nw, nreads, seg, ls) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void *)(wl + slot * 2048), 16, o, 0, 0, AUX);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void *)(wl + slot * 2048 + 1024), 16, o, 0, 0, AUX);
  };
#pragma unroll
  for (int k = 0; k < D; ++k) issue(k, k);
  int slot = 0;
  for (int64_t k = 0; k < mine; ++k) {
    WAIT_VM(2 * (D - 1));
    v4u p, q;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(p), "=v"(q)
                 : "v"((uint32_t)(uintptr_t)(wl + slot * 2048 + 16 * lane))
                 : "memory");
    x ^= p.x ^ p.y ^ p.z ^ p.w ^ q.x ^ q.y ^ q.z ^ q.w;
    issue(k + D, slot);
    slot = slot + 1 == D ? 0 : slot + 1;
  }
  WAIT_VM(0);
  out[blockIdx.x * kWG + threadIdx.x] = x;
}

int main() {
  const int64_t nreads = 10000000;
  const uint32_t n = (uint32_t)(nreads * kL);
  char *a, *b;
  uint32_t *out;
  hipMalloc(&a, n + 256);
  hipMalloc(&b, n + 256);
  hipMemset(a, 1, n + 256);
  hipMemset(b, 2, n + 256);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipMalloc(&out, (size_t)cus * 16 * kWG * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, size_t lds, auto launch) {
    for (int occ : {4, 5, 8}) {
      if (lds * occ > 160 * 1024) continue;
      const int grid = cus * occ;
      launch(grid, lds);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 10; ++i) launch(grid, lds);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double tbs = 2.0 * n * 10 / (ms * 1e-3) / 1e12;
      std::printf("%-10s grid %5d (%d WG/CU, %6zu B LDS): %.1f us/pass  %.2f TB/s\n", name, grid, occ, lds,
                  ms * 100, tbs);
    }
  };
  run("reg1", 0, [&](int g, size_t l) { k_reg<1><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("reg2", 0, [&](int g, size_t l) { k_reg<2><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("reg3", 0, [&](int g, size_t l) { k_reg<3><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("reg4", 0, [&](int g, size_t l) { k_reg<4><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds2", 4 * 2 * 2048, [&](int g, size_t l) { k_glds<2, 0><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds3", 4 * 3 * 2048, [&](int g, size_t l) { k_glds<3, 0><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds4", 4 * 4 * 2048, [&](int g, size_t l) { k_glds<4, 0><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds6", 4 * 6 * 2048, [&](int g, size_t l) { k_glds<6, 0><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds3nt", 4 * 3 * 2048, [&](int g, size_t l) { k_glds<3, 2><<<g, kWG, l>>>(a, b, n, nreads, out); });
  run("glds4nt", 4 * 4 * 2048, [&](int g, size_t l) { k_glds<4, 2><<<g, kWG, l>>>(a, b, n, nreads, out); });
  return 0;
}
