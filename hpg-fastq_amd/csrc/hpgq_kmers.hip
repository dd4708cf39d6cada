// hpgq_kmers.hip — `stats --kmers`: 5-mer counts, global and per position.
//
// Replaces the per-read kmer fields of fastq_reads_stats (bioinfo-libs,
// absent) and their merge in the stats consumer, src/stats_fastq.c:384-410
// (kmer_out->counter += ..., counter_by_pos[k] += ...).  Semantics are
// build-defined: 5-mers of exact uppercase A/C/G/T, id =
// sum code_i * 4^(4-i) with A=0 C=1 G=2 T=3 (first base most significant),
// counted at every start position p <= len-5 of every merged read.  Output:
// by_pos[1024][lmax-4] u64; the global counter of a k-mer is its row sum.
//
// Kernel: position tiles.  A workgroup owns kP start positions and an LDS
// table [1024 kmers][kP] (64 KB, u32: one read adds at most 1 per cell), and
// walks a stride of reads, each lane one read at a time: one 16-byte and one
// 4-byte buffer load cover the 20 bytes the tile's 5-mers span, codes come from
// a v_perm lookup with an exact byte check, and a 5-bit validity register
// gates the LDS adds.  Nonzero cells are flushed with global atomics.
#include "hpgq_common.h"

#include <algorithm>

namespace hpgq {
namespace kmers {

constexpr int kK = 5;
constexpr int kNum = 1 << (2 * kK);   // 1024
constexpr int kP = 16;                // start positions per tile
constexpr int kWG = 1024;

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// byte & 7 is one-to-one on A(1) C(3) T(4) G(7); the expected byte per code
// (0x01 never matches) and the 2-bit code per code
constexpr uint32_t kExLo = 0x43014101u;   // codes 0..3: -, A, -, C
constexpr uint32_t kExHi = 0x47010154u;   // codes 4..7: T, -, -, G
constexpr uint32_t kValLo = 0x01000000u;  // C = 1 at code 3
constexpr uint32_t kValHi = 0x02000003u;  // T = 3 at code 4, G = 2 at code 7

// 4 bytes -> 2-bit codes (byte lanes) and a valid bit per byte (bit 8*i)
__device__ __forceinline__ void codes4(uint32_t w, uint32_t &val, uint32_t &ok) {
  const uint32_t code = w & 0x07070707u;
  const uint32_t d = w ^ __builtin_amdgcn_perm(kExHi, kExLo, code);
  const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;   // inexact bytes
  ok = ~(nz >> 7) & 0x01010101u;
  val = __builtin_amdgcn_perm(kValHi, kValLo, code);
}

__global__ void __launch_bounds__(kWG) kmer_kernel(const char *seq, const int32_t *idx, int64_t n,
                                                   const uint8_t *mask, int npos,
                                                   unsigned long long *out) {
  __shared__ uint32_t t[kNum * kP];
  for (int i = threadIdx.x; i < kNum * kP; i += kWG) t[i] = 0;
  __syncthreads();
  const int p0 = blockIdx.x * kP;
  const int32_t data_end = __builtin_amdgcn_readfirstlane(idx[n]);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)seq, (short)0, data_end + HPGQ_DEVICE_SLACK, 0x00020000);
  for (int64_t r = (int64_t)blockIdx.y * kWG + threadIdx.x; r < n; r += (int64_t)gridDim.y * kWG) {
    if (mask && mask[r] != 1) continue;
    const int a = idx[r];
    const int last = min(idx[r + 1] - a - kK, npos - 1);   // last start position counted
    if (last < p0) continue;
    const v4u w = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(a + p0), 0, 0);
    const uint32_t w4 = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(a + p0 + 16), 0, 0);
    uint32_t val[5], ok[5];
#pragma unroll
    for (int i = 0; i < 4; ++i) codes4(w[i], val[i], ok[i]);
    codes4(w4, val[4], ok[4]);
    uint32_t id = 0, vb = 0;
#pragma unroll
    for (int i = 0; i < kP + kK - 1; ++i) {
      const uint32_t c = (val[i >> 2] >> (8 * (i & 3))) & 3u;
      const uint32_t v = (ok[i >> 2] >> (8 * (i & 3))) & 1u;
      id = ((id << 2) | c) & (kNum - 1);
      vb = ((vb << 1) | v) & 31u;
      const int j = i - (kK - 1);   // the 5-mer ending at byte i starts at p0 + j
      if (j >= 0 && vb == 31u && j <= last - p0) atomicAdd(&t[id * kP + j], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kNum * kP; i += kWG) {
    const uint32_t v = t[i];
    const int p = p0 + (i % kP);
    if (v && p < npos) atomicAdd(&out[(size_t)(i / kP) * npos + p], (unsigned long long)v);
  }
}

}  // namespace kmers
}  // namespace hpgq

struct hpgq_kmers {
  int device = 0;
  int lmax = 0, npos = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  unsigned long long *d_out = nullptr;
  int cus = 0;
};

extern "C" {

int hpgq_kmers_open(hpgq_kmers_t **km, int device, int lmax, void *stream) {
  if (!km || lmax < 1 || lmax > HPGQ_LMAX_LIMIT) return HPGQ_E_INVALID;
  *km = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return HPGQ_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(device));
  hpgq_kmers *k = new hpgq_kmers;
  k->device = device;
  k->lmax = lmax;
  k->npos = lmax > hpgq::kmers::kK - 1 ? lmax - (hpgq::kmers::kK - 1) : 0;
  if (stream) {
    k->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking) != hipSuccess) {
      delete k;
      return HPGQ_E_HIP;
    }
    k->own_stream = true;
  }
  const size_t bytes = (size_t)hpgq::kmers::kNum * (size_t)(k->npos > 0 ? k->npos : 1) * 8;
  if (hipMalloc(&k->d_out, bytes) != hipSuccess) {
    hpgq_kmers_close(k);
    return HPGQ_E_NOMEM;
  }
  if (hipMemsetAsync(k->d_out, 0, bytes, k->stream) != hipSuccess ||
      hipDeviceGetAttribute(&k->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    hpgq_kmers_close(k);
    return HPGQ_E_HIP;
  }
  *km = k;
  return HPGQ_OK;
}

void hpgq_kmers_close(hpgq_kmers_t *k) {
  if (!k) return;
  (void)hipSetDevice(k->device);
  if (k->stream) (void)hipStreamSynchronize(k->stream);
  (void)hipFree(k->d_out);
  if (k->own_stream) (void)hipStreamDestroy(k->stream);
  delete k;
}

int hpgq_kmers_count_device(hpgq_kmers_t *k, const hpgq_batch_t *b, const uint8_t *mask) {
  if (!k || !b || b->num_reads < 0) return HPGQ_E_INVALID;
  if (b->num_reads == 0 || k->npos == 0) return HPGQ_OK;
  if (!b->seq || !b->data_indices) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  using namespace hpgq::kmers;
  const int tiles = (k->npos + kP - 1) / kP;
  const int64_t need = (b->num_reads + kWG - 1) / kWG;
  // about two resident workgroups per CU over all tiles
  const int64_t ny = std::max<int64_t>(1, std::min<int64_t>(need, (2 * k->cus + tiles - 1) / tiles));
  hipLaunchKernelGGL(kmer_kernel, dim3(tiles, (unsigned)ny), dim3(kWG), 0, k->stream, b->seq,
                     b->data_indices, (int64_t)b->num_reads, mask, k->npos, k->d_out);
  HPGQ_HIP_TRY(hipGetLastError());
  return HPGQ_OK;
}

int hpgq_kmers_sync(hpgq_kmers_t *k) {
  if (!k) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  return HPGQ_OK;
}

int hpgq_kmers_reset(hpgq_kmers_t *k) {
  if (!k) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  HPGQ_HIP_TRY(hipMemsetAsync(k->d_out, 0, hpgq_kmers_size(k) * 8, k->stream));
  return HPGQ_OK;
}

size_t hpgq_kmers_size(const hpgq_kmers_t *k) {
  return k ? (size_t)hpgq::kmers::kNum * (size_t)k->npos : 0;
}

int hpgq_kmers_read(hpgq_kmers_t *k, uint64_t *by_pos, size_t n) {
  if (!k || (!by_pos && n) || n < hpgq_kmers_size(k)) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  if (hpgq_kmers_size(k))
    HPGQ_HIP_TRY(hipMemcpy(by_pos, k->d_out, hpgq_kmers_size(k) * 8, hipMemcpyDeviceToHost));
  return HPGQ_OK;
}

uint64_t *hpgq_kmers_device(hpgq_kmers_t *k) { return k ? (uint64_t *)k->d_out : nullptr; }

}  // extern "C"
