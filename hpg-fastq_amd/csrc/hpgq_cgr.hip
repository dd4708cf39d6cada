// hpgq_cgr.hip — chaos-game (CGR) k-mer accumulator, old/chaos_game.c:165-267.
//
// The reference walks every base of a batch with ONE double-precision state
// (f_x, f_y) that is carried across reads and clamped at `dim` with an
// EPSILON nudge (:236-251); counters (word count, quality sum) reset per read
// and on 'N'.  The tables are u32 sums, so only the cell sequence must be
// reproduced — but the cell comes from (int)f of that carried double state,
// which an integer k-mer index matches only away from long homopolymer runs
// (SURVEY §8a A7 probe).  So this path simulates the reference's double
// recurrence itself, bit for bit, and gets its parallelism by speculation:
//
//   cgr_fill_kernel   one lane per read.  The lane GUESSES its read's entry
//                     state by replaying the f/count/clamp logic over the
//                     kWarm bytes of context before the read (from a fixed
//                     start state; two double states that differ converge
//                     to the same bits within ~60-110 moving bases), then
//                     runs the read with full accounting into LDS tables
//                     (k <= 7; global atomics above) and stores the guess g_r
//                     and its exit state e_r.  A read whose context reaches
//                     the batch start gets the exact state (same operations
//                     in the same order as the serial loop).
//   cgr_check_kernel  flags r where g_r != e_{r-1} (bitwise) in a two-level
//                     bitmap.  No flags => every guess was exact (induction
//                     from read 0) and the tables are final.
//   cgr_fix_kernel    one lane walks the flagged reads in order: it takes the
//                     read's speculative contributions back out (u32
//                     arithmetic is a group, so subtraction undoes exactly),
//                     adds the ones from the true entry state e_{r-1}, and
//                     continues down the chain until an exit state meets the
//                     next read's guess again.
// Random reads never flag; homopolymer-heavy batches can (the double state
// keeps the relative history through a run of halvings) and then pay a serial
// replay for those reads only.  The word count does not depend on f, so it is
// exact from the first kernel.
#include "hpgq_common.h"

#include <algorithm>

namespace hpgq {
namespace cgr {

constexpr double kEps = 0.00001;   // old/chaos_game.h:41
constexpr int kWG = 1024;       // 16 waves share one set of LDS tables (128 KB at k = 7)
constexpr int kWarm = 128;         // bytes of context replayed to guess a read's entry state
constexpr int kLdsMaxK = 7;        // 2 x 4^7 x 4 B = 128 KB of LDS tables

typedef unsigned v2u __attribute__((ext_vector_type(2)));

struct Args {
  const char *seq, *qual;
  const int32_t *idx;
  const uint8_t *status;     // read_status[] (device) or null
  int mode;                  // HPGQ_CGR_ONLY_VALID_READS: skip status != 1 (:188)
  int64_t num_reads;
  uint32_t base_quality;
  uint32_t *ts, *tq;         // global tables [dim][dim]
  unsigned long long *words; // fq_word_count (u64 here, u32 on read-out)
  double2 *g, *e;            // per read: guessed entry state, exit state
  unsigned long long *flags; // [ceil(n/64)] one bit per read
  unsigned long long *sum;   // [ceil(n/4096)] one bit per nonzero flags word
  unsigned long long *replays;
};

struct Src {
  __amdgpu_buffer_rsrc_t rs, rq;
};

__device__ __forceinline__ Src make_src(const Args &A) {
  Src s;
  // reads end at data_end; 8-byte loads may touch HPGQ_DEVICE_SLACK more bytes
  const int32_t data_end = __builtin_amdgcn_readfirstlane(A.idx[A.num_reads]);
  s.rs = __builtin_amdgcn_make_buffer_rsrc((void *)A.seq, (short)0, data_end + HPGQ_DEVICE_SLACK,
                                           0x00020000);
  s.rq = __builtin_amdgcn_make_buffer_rsrc((void *)A.qual, (short)0, data_end + HPGQ_DEVICE_SLACK,
                                           0x00020000);
  return s;
}

__device__ __forceinline__ bool valid_read(const Args &A, int64_t r) {
  return A.mode != HPGQ_CGR_ONLY_VALID_READS || (A.status && A.status[r] == 1);
}

__device__ __forceinline__ uint32_t byte_of(v2u v, int u) { return (v[u >> 2] >> (8 * (u & 3))) & 0xFFu; }
__device__ __forceinline__ uint32_t sbyte_of(v2u v, int u) {   // signed char, as the u32 it adds
  return (uint32_t)(int32_t)(int8_t)byte_of(v, u);
}

struct State {
  double fx, fy;
};

// One base of chaos_game_fill_tables (:197-260).  FULL adds the word to the
// tables (sign = 1 adds, 0xFFFFFFFF takes it back out); !FULL only advances
// f, the word counter and the boundary clamp (context replay).
template <int K, bool FULL>
__device__ __forceinline__ void step(uint32_t sb, uint32_t qb, uint32_t qold, State &st, int &cnt,
                                     uint32_t &acc, uint32_t *ts, uint32_t *tq, uint32_t sign,
                                     uint32_t sub, uint32_t &words) {
  constexpr int dim = 1 << K;
  const bool isA = sb == 65u, isC = sb == 67u, isG = sb == 71u, isT = sb == 84u;
  if (sb == 78u) {   // 'N' (:229-233)
    cnt = 0;
    acc = 0;
  }
  if (isA | isC | isG | isT) {
    const bool bx = isA | isT, by = isG | isT;
    st.fx = bx ? st.fx + (((double)dim - st.fx) * 0.5) : st.fx * 0.5;
    st.fy = by ? st.fy + (((double)dim - st.fy) * 0.5) : st.fy * 0.5;
    ++cnt;
    if (FULL) acc += qb;
  }
  if (cnt == K) {   // :236-260
    int cx = (int)st.fx, cy = (int)st.fy;
    if (cx == dim) {
      cx = dim - 1;
      st.fx = st.fx - kEps;
    }
    if (cy == dim) {
      cy = dim - 1;
      st.fy = st.fy - kEps;
    }
    --cnt;
    if (FULL) {
      const int cell = cx * dim + cy;
      atomicAdd(&ts[cell], sign);
      atomicAdd(&tq[cell], sign * (acc - sub));
      ++words;
      acc -= qold;   // quality[quality_position - word_size] (:259), raw position
    }
  }
}

// word counter at byte p of a read: moving bases since the last reset
// (read start or 'N'), capped at K-1 (a completed word drops it to K-1)
template <int K>
__device__ int count_before(const char *seq, int a, int p) {
  int m = 0;
  for (int i = p - 1; i >= 0 && m < K - 1; --i) {
    const char c = seq[a + i];
    if (c == 'N') break;
    if (c == 'A' || c == 'C' || c == 'G' || c == 'T') ++m;
  }
  return m;
}

// Run read r from byte p0 (word counter cnt0) with state st.
template <int K, bool FULL>
__device__ void run_read(const Args &A, const Src &S, int64_t r, int p0, int cnt0, State &st,
                         uint32_t *ts, uint32_t *tq, uint32_t sign, uint32_t &words) {
  const int a = A.idx[r], n = A.idx[r + 1] - a;
  const uint32_t sub = A.base_quality * (uint32_t)K;
  int cnt = cnt0;
  uint32_t acc = 0;
  v2u q1 = {0u, 0u}, q2 = {0u, 0u};   // the two previous quality chunks
  for (int c = p0; c < n; c += 8) {
    const v2u sv = __builtin_amdgcn_raw_buffer_load_b64(S.rs, (uint32_t)(a + c), 0, 0);
    v2u qv = {0u, 0u};
    if (FULL) qv = __builtin_amdgcn_raw_buffer_load_b64(S.rq, (uint32_t)(a + c), 0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (c + u < n) {
        uint32_t qold = 0;
        if (FULL) {
          const int o = u + 1 - K;   // raw byte j+1-K relative to this chunk
          qold = o >= 0 ? sbyte_of(qv, o) : (o >= -8 ? sbyte_of(q1, o + 8) : sbyte_of(q2, o + 16));
        }
        step<K, FULL>(byte_of(sv, u), FULL ? sbyte_of(qv, u) : 0u, qold, st, cnt, acc, ts, tq, sign,
                      sub, words);
      }
    }
    q2 = q1;
    q1 = qv;
  }
}

// the entry state guess for read r: replay the kWarm bytes of (valid) context
// before it from the fixed start state; exact when the context reaches the
// batch start
template <int K>
__device__ State guess_entry(const Args &A, const Src &S, int64_t r) {
  constexpr double half = (double)(1 << K) * 0.5;   // :107-108
  State st = {half, half};
  int need = kWarm;
  int64_t t = r;
  int p = 0;
  while (need > 0 && t > 0) {
    --t;
    if (!valid_read(A, t)) continue;
    const int L = A.idx[t + 1] - A.idx[t];
    if (L >= need) {
      p = L - need;
      need = 0;
    } else {
      need -= L;
      p = 0;
    }
  }
  if (need > 0) {   // context reaches the batch start: replay it all, exactly
    t = 0;
    p = 0;
  }
  uint32_t w = 0;
  for (; t < r; ++t) {
    if (!valid_read(A, t)) continue;
    const int cnt0 = p > 0 ? count_before<K>(A.seq, A.idx[t], p) : 0;
    run_read<K, false>(A, S, t, p, cnt0, st, nullptr, nullptr, 0u, w);
    p = 0;
  }
  return st;
}

template <int K>
__global__ void __launch_bounds__(kWG) cgr_fill_kernel(Args A) {
  constexpr int dim = 1 << K;
  constexpr bool kLds = K <= kLdsMaxK;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *ts = kLds ? lds : A.ts;
  uint32_t *tq = kLds ? lds + dim * dim : A.tq;
  if (kLds) {
    for (int i = threadIdx.x; i < 2 * dim * dim; i += kWG) lds[i] = 0;
    __syncthreads();
  }
  const Src S = make_src(A);
  uint32_t words = 0;
  const int64_t stride = (int64_t)gridDim.x * kWG;
  for (int64_t r = (int64_t)blockIdx.x * kWG + threadIdx.x; r < A.num_reads; r += stride) {
    State st = guess_entry<K>(A, S, r);
    A.g[r] = make_double2(st.fx, st.fy);
    if (valid_read(A, r)) run_read<K, true>(A, S, r, 0, 0, st, ts, tq, 1u, words);
    A.e[r] = make_double2(st.fx, st.fy);
  }
  // fq_word_count: wave sum, one atomic per wave
  uint64_t w = words;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(A.words, (unsigned long long)w);
  if (kLds) {
    __syncthreads();
    for (int i = threadIdx.x; i < dim * dim; i += kWG) {
      if (lds[i]) atomicAdd(&A.ts[i], lds[i]);
      if (lds[dim * dim + i]) atomicAdd(&A.tq[i], lds[dim * dim + i]);
    }
  }
}

__device__ __forceinline__ bool same(double2 a, double2 b) {
  return __double_as_longlong(a.x) == __double_as_longlong(b.x) &&
         __double_as_longlong(a.y) == __double_as_longlong(b.y);
}

// flag r iff its guessed entry state differs (bitwise) from e_{r-1}
__global__ void __launch_bounds__(256) cgr_check_kernel(Args A) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool f = r > 0 && r < A.num_reads && !same(A.g[r], A.e[r - 1]);
  const unsigned long long b = __ballot(f);
  if ((threadIdx.x & 63) == 0 && r < A.num_reads) {
    const int64_t wi = r >> 6;
    A.flags[wi] = b;
    if (b) atomicOr(&A.sum[wi >> 6], 1ull << (wi & 63));
  }
}

// one lane: replay flagged reads in order with their true entry states
template <int K>
__global__ void __launch_bounds__(64) cgr_fix_kernel(Args A) {
  if (threadIdx.x != 0) return;
  const Src S = make_src(A);
  const int64_t nw = (A.num_reads + 63) >> 6;
  const int64_t ns = (nw + 63) >> 6;
  int64_t last = 0;   // reads <= last are final
  unsigned long long replays = 0;
  uint32_t dummy = 0;
  for (int64_t si = 0; si < ns; ++si) {
    unsigned long long sw = A.sum[si];
    while (sw) {
      const int64_t wi = si * 64 + __builtin_ctzll(sw);
      sw &= sw - 1;
      unsigned long long fw = A.flags[wi];
      while (fw) {
        int64_t r = wi * 64 + __builtin_ctzll(fw);
        fw &= fw - 1;
        if (r <= last) continue;
        double2 entry = A.e[r - 1];
        for (;;) {
          if (valid_read(A, r)) {
            const double2 g = A.g[r];
            State s1 = {g.x, g.y};
            run_read<K, true>(A, S, r, 0, 0, s1, A.ts, A.tq, 0xFFFFFFFFu, dummy);   // undo
          }
          State s2 = {entry.x, entry.y};
          if (valid_read(A, r)) run_read<K, true>(A, S, r, 0, 0, s2, A.ts, A.tq, 1u, dummy);
          const double2 ex = make_double2(s2.fx, s2.fy);
          A.e[r] = ex;
          ++replays;
          last = r;
          if (r + 1 >= A.num_reads || same(ex, A.g[r + 1])) break;
          entry = ex;
          ++r;
        }
      }
    }
  }
  *A.replays = replays;
}

template <int K>
struct Kernels {
  static const void *fill() { return (const void *)cgr_fill_kernel<K>; }
  static const void *fix() { return (const void *)cgr_fix_kernel<K>; }
};

static const void *fill_for(int k) {
  switch (k) {
    case 1: return Kernels<1>::fill();
    case 2: return Kernels<2>::fill();
    case 3: return Kernels<3>::fill();
    case 4: return Kernels<4>::fill();
    case 5: return Kernels<5>::fill();
    case 6: return Kernels<6>::fill();
    case 7: return Kernels<7>::fill();
    case 8: return Kernels<8>::fill();
    case 9: return Kernels<9>::fill();
    case 10: return Kernels<10>::fill();
    case 11: return Kernels<11>::fill();
    default: return Kernels<12>::fill();
  }
}

static const void *fix_for(int k) {
  switch (k) {
    case 1: return Kernels<1>::fix();
    case 2: return Kernels<2>::fix();
    case 3: return Kernels<3>::fix();
    case 4: return Kernels<4>::fix();
    case 5: return Kernels<5>::fix();
    case 6: return Kernels<6>::fix();
    case 7: return Kernels<7>::fix();
    case 8: return Kernels<8>::fix();
    case 9: return Kernels<9>::fix();
    case 10: return Kernels<10>::fix();
    case 11: return Kernels<11>::fix();
    default: return Kernels<12>::fix();
  }
}

}  // namespace cgr
}  // namespace hpgq

struct hpgq_cgr {
  int device = 0, k = 7, dim = 128;
  uint32_t base_quality = 33;
  hipStream_t stream = nullptr;
  uint32_t *d_ts = nullptr, *d_tq = nullptr;
  unsigned long long *d_words = nullptr, *d_replays = nullptr;
  double2 *d_g = nullptr, *d_e = nullptr;
  unsigned long long *d_flags = nullptr, *d_sum = nullptr;
  int64_t cap = 0;            // reads the per-read buffers hold
  size_t lds = 0;
  int grid = 0;
  int64_t last_replays = 0;
  bool pending = false;       // a fill whose replay count was not read back yet
};

static int cgr_ensure(hpgq_cgr *c, int64_t n) {
  if (n <= c->cap) return HPGQ_OK;
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_g);
  (void)hipFree(c->d_e);
  (void)hipFree(c->d_flags);
  (void)hipFree(c->d_sum);
  c->d_g = c->d_e = nullptr;
  c->d_flags = c->d_sum = nullptr;
  c->cap = 0;
  const int64_t cap = n + n / 4 + 1024;
  const int64_t nw = (cap + 63) / 64, ns = (nw + 63) / 64;
  if (hipMalloc(&c->d_g, cap * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->d_e, cap * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->d_flags, nw * 8) != hipSuccess || hipMalloc(&c->d_sum, ns * 8) != hipSuccess)
    return HPGQ_E_NOMEM;
  c->cap = cap;
  return HPGQ_OK;
}

extern "C" {

int hpgq_cgr_open(hpgq_cgr_t **cg, int device, int k, int base_quality) {
  if (!cg) return HPGQ_E_INVALID;
  *cg = nullptr;
  if (k < 1 || k > 12) return HPGQ_E_INVALID;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return HPGQ_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return HPGQ_E_INVALID;
  hpgq_cgr *c = new hpgq_cgr();
  c->device = device;
  c->k = k;
  c->dim = 1 << k;
  c->base_quality = (uint32_t)base_quality;
  const size_t cells = (size_t)c->dim * c->dim;
  HPGQ_HIP_TRY(hipSetDevice(device));
  HPGQ_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HPGQ_HIP_TRY(hipMalloc(&c->d_ts, cells * 4));
  HPGQ_HIP_TRY(hipMalloc(&c->d_tq, cells * 4));
  HPGQ_HIP_TRY(hipMalloc(&c->d_words, 8));
  HPGQ_HIP_TRY(hipMalloc(&c->d_replays, 8));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_ts, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_tq, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_words, 0, 8, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_replays, 0, 8, c->stream));
  c->lds = k <= hpgq::cgr::kLdsMaxK ? 2 * cells * 4 : 0;
  const void *kfn = hpgq::cgr::fill_for(k);
  if (c->lds > 64 * 1024)
    HPGQ_HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds));
  int per_cu = 0, cus = 0;
  HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, hpgq::cgr::kWG, c->lds));
  HPGQ_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  c->grid = std::max(1, per_cu) * cus;
  *cg = c;
  return HPGQ_OK;
}

void hpgq_cgr_close(hpgq_cgr_t *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_ts);
  (void)hipFree(c->d_tq);
  (void)hipFree(c->d_words);
  (void)hipFree(c->d_replays);
  (void)hipFree(c->d_g);
  (void)hipFree(c->d_e);
  (void)hipFree(c->d_flags);
  (void)hipFree(c->d_sum);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int hpgq_cgr_fill_device(hpgq_cgr_t *c, const hpgq_batch_t *b, const uint8_t *status, int mode) {
  if (!c || !b || b->num_reads < 0) return HPGQ_E_INVALID;
  if (mode != HPGQ_CGR_ALL_READS && mode != HPGQ_CGR_ONLY_VALID_READS) return HPGQ_E_INVALID;
  if (b->num_reads == 0) return HPGQ_OK;
  if (!b->seq || !b->quality || !b->data_indices) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  int rc = cgr_ensure(c, b->num_reads);
  if (rc) return rc;
  const int64_t n = b->num_reads;
  const int64_t nw = (n + 63) / 64, ns = (nw + 63) / 64;
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_sum, 0, ns * 8, c->stream));
  hpgq::cgr::Args A;
  A.seq = b->seq;
  A.qual = b->quality;
  A.idx = b->data_indices;
  A.status = status;
  A.mode = mode;
  A.num_reads = n;
  A.base_quality = c->base_quality;
  A.ts = c->d_ts;
  A.tq = c->d_tq;
  A.words = c->d_words;
  A.g = c->d_g;
  A.e = c->d_e;
  A.flags = c->d_flags;
  A.sum = c->d_sum;
  A.replays = c->d_replays;
  void *args[] = {&A};
  const int64_t need = (n + hpgq::cgr::kWG - 1) / hpgq::cgr::kWG;
  const int grid = (int)std::min<int64_t>(need, c->grid);
  HPGQ_HIP_TRY(hipLaunchKernel(hpgq::cgr::fill_for(c->k), dim3(grid), dim3(hpgq::cgr::kWG), args,
                               c->lds, c->stream));
  HPGQ_HIP_TRY(hipLaunchKernel((const void *)hpgq::cgr::cgr_check_kernel, dim3((unsigned)((n + 255) / 256)),
                               dim3(256), args, 0, c->stream));
  HPGQ_HIP_TRY(hipLaunchKernel(hpgq::cgr::fix_for(c->k), dim3(1), dim3(64), args, 0, c->stream));
  c->pending = true;
  return HPGQ_OK;
}

int hpgq_cgr_sync(hpgq_cgr_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->pending) {
    unsigned long long r = 0;
    HPGQ_HIP_TRY(hipMemcpy(&r, c->d_replays, 8, hipMemcpyDeviceToHost));
    c->last_replays = (int64_t)r;
    c->pending = false;
  }
  return HPGQ_OK;
}

int hpgq_cgr_reset(hpgq_cgr_t *c) {
  if (!c) return HPGQ_E_INVALID;
  const size_t cells = (size_t)c->dim * c->dim;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_ts, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_tq, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_words, 0, 8, c->stream));
  return HPGQ_OK;
}

int hpgq_cgr_read(hpgq_cgr_t *c, uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count) {
  if (!c) return HPGQ_E_INVALID;
  int rc = hpgq_cgr_sync(c);
  if (rc) return rc;
  const size_t cells = (size_t)c->dim * c->dim;
  if (table_seq) HPGQ_HIP_TRY(hipMemcpy(table_seq, c->d_ts, cells * 4, hipMemcpyDeviceToHost));
  if (table_q) HPGQ_HIP_TRY(hipMemcpy(table_q, c->d_tq, cells * 4, hipMemcpyDeviceToHost));
  if (word_count) {
    unsigned long long w = 0;
    HPGQ_HIP_TRY(hipMemcpy(&w, c->d_words, 8, hipMemcpyDeviceToHost));
    *word_count = (uint32_t)w;   // fq_word_count is a u32 (wraps)
  }
  return HPGQ_OK;
}

void *hpgq_cgr_stream(hpgq_cgr_t *c) { return c ? (void *)c->stream : nullptr; }

int64_t hpgq_cgr_last_replays(hpgq_cgr_t *c) { return c ? c->last_replays : 0; }

}  // extern "C"
