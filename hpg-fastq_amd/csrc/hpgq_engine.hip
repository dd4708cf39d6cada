// hpgq_engine.hip — fused edit -> filter -> stats kernel for gfx950 (MI355X).
//
// Replaces, for one SoA batch resident in HBM:
//   fastq_edit          src/edit_fastq.c:154            (5'/3' trim)
//   fastq_filter        src/stats_fastq.c:224, src/filter_fastq.c:148, src/edit_fastq.c:166
//   fastq_reads_stats   src/stats_fastq.c:230,244
//   the consumer merge  src/stats_fastq.c:257-417       (per-read + per-base counters)
//
// Data flow per workgroup (256 threads = 4 waves), grid-stride over tiles of
// `slots` reads per mate:
//   1. stage   : the tile's seq and quality bytes (one contiguous range per
//                buffer) are copied HBM -> LDS with 16-byte loads.
//   2. pass 1  : one lane per read: trim, then SWAR word loops over the read
//                window (v_sad_u8 quality sum, zero-byte tests for N and G/C,
//                byte compares for out-of-range qualities) -> pass/fail, the
//                per-read histogram keys (LDS atomics) and the mask/trim
//                outputs (coalesced stores).
//   3. pass 2  : one wave per read, lane l owns positions 4l..4l+3 (+256c):
//                per-position base counters as 5 six-bit fields per u32
//                (v_perm_b32 maps base byte -> field shift), quality sums as
//                16-bit pairs; flushed to u32 registers every 63 reads.  No
//                atomics on the per-base path.
//   4. end     : waves reduce through LDS, one u64 global atomic per counter
//                per workgroup.
// Everything is integer arithmetic; results are bit-identical to the CPU
// oracle by construction (order-independent sums).

#include "hpgq_common.h"

namespace hpgq {

constexpr int kWG = 256;
constexpr int kFlushEvery = 63;   // 6-bit base fields

struct EngineArgs {
  const char *seq[2];
  const char *qual[2];
  const int32_t *idx[2];
  int64_t num_reads;
  uint8_t *mask;
  uint32_t *trim;
  uint64_t *counters;
  int32_t *err;
  int lmax;
  int clen;
  int nm;          // mates (1 or 2)
  int slots;       // reads per mate per tile, multiple of 64
  int cap;         // LDS bytes per tile buffer (multiple of 16)
  int hwords;      // LDS histogram words per mate (multiple of 4)
  int phred;
  int filter_on, edit_on, stats_on;
  int min_len, max_len;
  int min_q, max_q;
  int check_oor, max_oor;
  uint32_t oor_lo4, oor_hi4;   // replicated raw thresholds (lo, hi+1)
  int oor_lo_none, oor_hi_none, oor_all;
  int max_n;
  int left_len, min_left, max_left;
  int right_len, min_right, max_right;
  int e_left_len, e_min_left, e_max_left;
  int e_right_len, e_min_right, e_max_right;
};

// ---------------------------------------------------------------------------
// SWAR helpers (4 bytes per u32)
// ---------------------------------------------------------------------------

// 0x80 in every byte of v that is zero, 0 elsewhere (exact, no borrow leak)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

// 0x80 in every byte where x >= c (unsigned), 0 elsewhere
__device__ __forceinline__ uint32_t ge_bytes(uint32_t x, uint32_t c4) {
  uint32_t d = (x | 0x80808080u) - (c4 & 0x7F7F7F7Fu);
  return ((x & ~c4) | (~(x ^ c4) & d)) & 0x80808080u;
}

// mask of the bytes of aligned word at byte address wb that fall in [lo, hi)
__device__ __forceinline__ uint32_t range_mask(int wb, int lo, int hi) {
  uint32_t m = 0xFFFFFFFFu;
  if (wb < lo) m &= 0xFFFFFFFFu << (8 * (lo - wb));
  if (wb + 4 > hi) m &= 0xFFFFFFFFu >> (8 * (wb + 4 - hi));
  return m;
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *lds, int wi) {
  return reinterpret_cast<const uint32_t *>(lds)[wi];
}

// 4 bytes at an unaligned LDS byte offset (off & 3 is wave uniform in pass 2)
__device__ __forceinline__ uint32_t lds_word(const uint8_t *lds, int off) {
  const int wi = off >> 2;
  const uint32_t lo = lds_u32(lds, wi), hi = lds_u32(lds, wi + 1);
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}

// raw quality sum of LDS bytes [lo, hi)
__device__ __forceinline__ uint32_t qsum_range(const uint8_t *lds, int lo, int hi) {
  uint32_t s = 0;
  for (int wb = lo & ~3; wb < hi; wb += 4)
    s = __builtin_amdgcn_sad_u8(lds_u32(lds, wb >> 2) & range_mask(wb, lo, hi), 0u, s);
  return s;
}

__device__ __forceinline__ bool mean_in(int64_t sumq, int64_t k, int lo, int hi) {
  return (int64_t)lo * k <= sumq && sumq <= (int64_t)hi * k;
}

// field shift per base code; code = (byte >> 1) & 7:
//   'A'->0 'C'->1 'T'->2 'G'->3 pad(0x08)->4 5,6 unused 'N'->7
// fields: A bits 0-5, C 6-11, G 12-17, T 18-23, N 24-29, 30-31 = garbage
constexpr uint32_t kExpLo = 0x47544341u;   // expected byte for codes 0..3
constexpr uint32_t kExpHi = 0x4E000008u;   // codes 4..7
constexpr uint32_t kShLo = 0x0C120600u;    // shifts for codes 0..3: 0, 6, 18, 12
constexpr uint32_t kShHi = 0x181E1E1Eu;    // codes 4..7: 30, 30, 30, 24

struct ReadInfo {
  int os, oq;        // LDS byte offset of the (trimmed) window start
  int wn;            // window length
  int ts, te;        // trim
  bool valid, pass, longread;
};

// pass 1: edit -> filter for one read held in LDS
__device__ __forceinline__ void pass1_read(const EngineArgs &A, const uint8_t *lds, int os0,
                                           int oq0, int n, ReadInfo &ri, uint32_t &sum_raw,
                                           uint32_t &ngc) {
  int ts = 0, te = 0;
  if (A.edit_on) {
    if (A.e_left_len > 0) {
      const int lim = min(A.e_left_len, n);
      while (ts < lim) {
        const int Q = (int)lds[oq0 + ts] - A.phred;
        if (Q >= A.e_min_left && Q <= A.e_max_left) break;
        ++ts;
      }
    }
    if (A.e_right_len > 0) {
      const int lim = min(A.e_right_len, n - ts);
      while (te < lim) {
        const int Q = (int)lds[oq0 + n - 1 - te] - A.phred;
        if (Q >= A.e_min_right && Q <= A.e_max_right) break;
        ++te;
      }
    }
  }
  const int wn = n - ts - te;
  const int os = os0 + ts, oq = oq0 + ts;
  ri.os = os; ri.oq = oq; ri.wn = wn; ri.ts = ts; ri.te = te;

  // quality window: raw sum (+ out-of-range count)
  uint32_t sq = 0, oor = 0;
  {
    const int lo = oq, hi = oq + wn;
    for (int wb = lo & ~3; wb < hi; wb += 4) {
      const uint32_t m = range_mask(wb, lo, hi);
      const uint32_t w = lds_u32(lds, wb >> 2);
      sq = __builtin_amdgcn_sad_u8(w & m, 0u, sq);
      if (A.check_oor) {
        uint32_t bad;
        if (A.oor_all) {
          bad = 0x80808080u;
        } else {
          bad = 0;
          if (!A.oor_lo_none) bad |= ~ge_bytes(w, A.oor_lo4) & 0x80808080u;
          if (!A.oor_hi_none) bad |= ge_bytes(w, A.oor_hi4);
        }
        oor += __builtin_popcount(bad & m & 0x80808080u);
      }
    }
  }
  // sequence window: N and G/C counts
  uint32_t nn = 0, gc = 0;
  {
    const int lo = os, hi = os + wn;
    for (int wb = lo & ~3; wb < hi; wb += 4) {
      const uint32_t m = range_mask(wb, lo, hi) & 0x80808080u;
      const uint32_t w = lds_u32(lds, wb >> 2);
      nn += __builtin_popcount(zero_bytes(w ^ 0x4E4E4E4Eu) & m);
      gc += __builtin_popcount(zero_bytes((w | 0x04040404u) ^ 0x47474747u) & m);
    }
  }
  sum_raw = sq;
  ngc = gc;

  bool pass = true;
  if (A.filter_on) {
    if (wn < A.min_len || wn > A.max_len) pass = false;
    if ((int)nn > A.max_n) pass = false;
    const int64_t sQ = (int64_t)sq - (int64_t)A.phred * wn;
    if (!mean_in(sQ, wn, A.min_q, A.max_q)) pass = false;
    if (A.check_oor && (int)oor > A.max_oor) pass = false;
    if (A.left_len > 0) {
      const int k = min(A.left_len, wn);
      if (k > 0) {
        const int64_t s = (int64_t)qsum_range(lds, oq, oq + k) - (int64_t)A.phred * k;
        if (!mean_in(s, k, A.min_left, A.max_left)) pass = false;
      }
    }
    if (A.right_len > 0) {
      const int k = min(A.right_len, wn);
      if (k > 0) {
        const int64_t s =
            (int64_t)qsum_range(lds, oq + wn - k, oq + wn) - (int64_t)A.phred * k;
        if (!mean_in(s, k, A.min_right, A.max_right)) pass = false;
      }
    }
  }
  ri.pass = pass;
}

template <int NCH>
struct PosAcc {
  uint32_t pk[NCH][4];      // packed 6-bit base fields per position
  uint32_t q02[NCH], q13[NCH];
  uint32_t wb[NCH][4][5];   // flushed base counts
  uint32_t wq[NCH][4];      // flushed quality sums

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      q02[c] = q13[c] = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pk[c][i] = 0;
        wq[c][i] = 0;
#pragma unroll
        for (int b = 0; b < 5; ++b) wb[c][i][b] = 0;
      }
    }
  }

  __device__ __forceinline__ void flush() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int b = 0; b < 5; ++b) wb[c][i][b] += (pk[c][i] >> (6 * b)) & 63u;
        pk[c][i] = 0;
      }
      wq[c][0] += q02[c] & 0xFFFFu;
      wq[c][2] += q02[c] >> 16;
      wq[c][1] += q13[c] & 0xFFFFu;
      wq[c][3] += q13[c] >> 16;
      q02[c] = q13[c] = 0;
    }
  }
};

template <int NCH>
__global__ void __launch_bounds__(kWG) engine_kernel(EngineArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int nm = A.nm, S = A.slots, cap = A.cap, lmax = A.lmax;
  const int nslots = nm * S;

  uint32_t *hist = reinterpret_cast<uint32_t *>(lds + nm * 2 * cap);
  unsigned long long *sc =
      reinterpret_cast<unsigned long long *>(lds + nm * 2 * cap + nm * A.hwords * 4);
  uint8_t *xch = reinterpret_cast<uint8_t *>(sc + nm * HPGQ_NUM_SCALARS);

  for (int i = tid; i < nm * A.hwords; i += kWG) hist[i] = 0;
  for (int i = tid; i < nm * HPGQ_NUM_SCALARS; i += kWG) sc[i] = 0;

  PosAcc<NCH> acc;
  acc.zero();
  int since_flush = 0;
  const bool p2_wave = A.stats_on && (64 * wave < nslots);
  const int p2_mate = p2_wave ? (64 * wave) / S : 0;

  const int64_t ntiles = (A.num_reads + S - 1) / S;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * S;
    const int nr = (int)min((int64_t)S, A.num_reads - r0);
    __syncthreads();   // previous tile's pass 2 is done with LDS

    // ---- 1. stage HBM -> LDS ------------------------------------------------
    int a0[2], shs[2], shq[2];
    bool fits = true;
    for (int m = 0; m < nm; ++m) {
      a0[m] = A.idx[m][r0];
      const int bytes = A.idx[m][r0 + nr] - a0[m];
      const uintptr_t ps = reinterpret_cast<uintptr_t>(A.seq[m] + a0[m]);
      const uintptr_t pq = reinterpret_cast<uintptr_t>(A.qual[m] + a0[m]);
      shs[m] = (int)(ps & 15);
      shq[m] = (int)(pq & 15);
      if (bytes + 32 > cap) fits = false;
      if (!fits) break;
      const int nvs = (shs[m] + bytes + 15) >> 4;
      const int nvq = (shq[m] + bytes + 15) >> 4;
      const uint4 *gs = reinterpret_cast<const uint4 *>(ps & ~(uintptr_t)15);
      const uint4 *gq = reinterpret_cast<const uint4 *>(pq & ~(uintptr_t)15);
      uint4 *ls = reinterpret_cast<uint4 *>(lds + m * 2 * cap);
      uint4 *lq = reinterpret_cast<uint4 *>(lds + m * 2 * cap + cap);
      int v = tid;
      for (; v + 3 * kWG < nvs; v += 4 * kWG) {
        const uint4 x0 = gs[v], x1 = gs[v + kWG], x2 = gs[v + 2 * kWG], x3 = gs[v + 3 * kWG];
        ls[v] = x0; ls[v + kWG] = x1; ls[v + 2 * kWG] = x2; ls[v + 3 * kWG] = x3;
      }
      for (; v < nvs; v += kWG) ls[v] = gs[v];
      v = tid;
      for (; v + 3 * kWG < nvq; v += 4 * kWG) {
        const uint4 x0 = gq[v], x1 = gq[v + kWG], x2 = gq[v + 2 * kWG], x3 = gq[v + 3 * kWG];
        lq[v] = x0; lq[v + kWG] = x1; lq[v + 2 * kWG] = x2; lq[v + 3 * kWG] = x3;
      }
      for (; v < nvq; v += kWG) lq[v] = gq[v];
    }
    if (!fits) {
      // a read longer than lmax made the tile overflow LDS: the call fails
      if (tid == 0) {
        atomicOr(A.err, 1);
        atomicAdd(&sc[HPGQ_S_LONG_READS], (unsigned long long)nr);
      }
      continue;
    }
    __syncthreads();

    // ---- 2. pass 1: one lane per read ---------------------------------------
    ReadInfo ri;
    ri.valid = false; ri.pass = false; ri.longread = false;
    ri.os = ri.oq = ri.wn = ri.ts = ri.te = 0;
    uint32_t sum_raw = 0, ngc = 0;
    const int mate = (tid < nslots) ? tid / S : 0;
    const int s = tid - mate * S;
    const int64_t r = r0 + s;
    if (tid < nslots && s < nr) {
      ri.valid = true;
      const int a = A.idx[mate][r], e = A.idx[mate][r + 1];
      const int n = e - a;
      const int base = mate * 2 * cap;
      pass1_read(A, lds, base + shs[mate] + (a - a0[mate]), base + cap + shq[mate] + (a - a0[mate]),
                 n, ri, sum_raw, ngc);
      ri.longread = ri.wn > lmax;
    }
    bool pass = ri.pass;
    if (nm == 2) {
      if (tid < nslots) xch[tid] = (uint8_t)ri.pass;
      __syncthreads();
      if (ri.valid) pass = xch[s] && xch[S + s];   // pair passes iff both mates pass
    }
    if (ri.valid) {
      if (mate == 0 && A.mask) A.mask[r] = (uint8_t)pass;
      if (A.trim) A.trim[(int64_t)mate * A.num_reads + r] = (uint32_t)ri.ts | ((uint32_t)ri.te << 16);
      unsigned long long *scm = sc + mate * HPGQ_NUM_SCALARS;
      uint32_t *hm = hist + mate * A.hwords;
      atomicAdd(&scm[HPGQ_S_NUM_INPUT], 1ull);
      atomicAdd(&scm[pass ? HPGQ_S_NUM_PASSED : HPGQ_S_NUM_FAILED], 1ull);
      if (ri.ts + ri.te > 0) atomicAdd(&scm[HPGQ_S_NUM_EDITED], 1ull);
      if (A.stats_on && pass) {
        atomicAdd(&scm[HPGQ_S_NUM_STATS], 1ull);
        if (ri.longread) {
          atomicAdd(&scm[HPGQ_S_LONG_READS], 1ull);
          atomicOr(A.err, 1);
        } else {
          const uint32_t wn = (uint32_t)ri.wn;
          atomicAdd(&hm[wn], 1u);
          if (wn > 0) {
            atomicAdd(&hm[lmax + 1 + (2 * sum_raw + wn) / (2 * wn)], 1u);
            atomicAdd(&hm[lmax + 1 + HPGQ_MEANQ_BINS + (100 * ngc) / wn], 1u);
            atomicAdd(&scm[HPGQ_S_ACC_MEANQ_FX16], ((unsigned long long)sum_raw << 16) / wn);
          }
        }
      }
    }
    const int st_flag = (A.stats_on && ri.valid && pass && !ri.longread) ? 1 : 0;

    // ---- 3. pass 2: one wave per read, lanes own positions ------------------
    if (p2_wave) {
#pragma unroll 1
      for (int j = 0; j < 64; ++j) {
        if (!__builtin_amdgcn_readlane(st_flag, j)) continue;
        const int os = __builtin_amdgcn_readlane(ri.os, j);
        const int oq = __builtin_amdgcn_readlane(ri.oq, j);
        const int wn = __builtin_amdgcn_readlane(ri.wn, j);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int p0 = 256 * c + 4 * lane;
          const int nv = wn - p0;
          if (nv > 0) {
            const uint32_t m = nv >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nv)) - 1u);
            uint32_t sw = lds_word(lds, os + p0);
            const uint32_t qw = lds_word(lds, oq + p0) & m;
            sw = (sw & m) | (0x08080808u & ~m);
            const uint32_t codes = (sw >> 1) & 0x07070707u;
            uint32_t sh = __builtin_amdgcn_perm(kShHi, kShLo, codes);
            const uint32_t ex = __builtin_amdgcn_perm(kExpHi, kExpLo, codes);
            if (sw != ex) {
              // bytes that are not exactly A/C/G/T/N (lowercase, IUPAC, ...)
              const uint32_t d = sw ^ ex;
              const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
              const uint32_t ff = (nz >> 7) * 0xFFu;
              sh = (sh & ~ff) | (0x1E1E1E1Eu & ff);
            }
            acc.pk[c][0] += 1u << (sh & 0xFFu);
            acc.pk[c][1] += 1u << ((sh >> 8) & 0xFFu);
            acc.pk[c][2] += 1u << ((sh >> 16) & 0xFFu);
            acc.pk[c][3] += 1u << (sh >> 24);
            acc.q02[c] += qw & 0x00FF00FFu;
            acc.q13[c] += (qw >> 8) & 0x00FF00FFu;
          }
        }
        if (++since_flush == kFlushEvery) {
          acc.flush();
          since_flush = 0;
        }
      }
    }
  }

  // ---- 4. workgroup reduction -> global -------------------------------------
  __syncthreads();
  uint32_t *red = reinterpret_cast<uint32_t *>(lds);   // nm * 6 * lmax words
  for (int i = tid; i < nm * 6 * lmax; i += kWG) red[i] = 0;
  __syncthreads();
  if (p2_wave) {
    acc.flush();
    uint32_t *rm = red + p2_mate * 6 * lmax;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = 256 * c + 4 * lane + i;
        if (pos < lmax) {
          if (acc.wq[c][i]) atomicAdd(&rm[pos], acc.wq[c][i]);
#pragma unroll
          for (int b = 0; b < 5; ++b)
            if (acc.wb[c][i][b]) atomicAdd(&rm[(1 + b) * lmax + pos], acc.wb[c][i][b]);
        }
      }
    }
  }
  __syncthreads();
  const size_t off_pos = HPGQ_NUM_SCALARS + (size_t)lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  for (int i = tid; i < nm * 6 * lmax; i += kWG) {
    const uint32_t v = red[i];
    if (v) {
      const int m = i / (6 * lmax), k = i - m * 6 * lmax;
      atomicAdd(reinterpret_cast<unsigned long long *>(A.counters + (size_t)m * A.clen + off_pos + k),
                (unsigned long long)v);
    }
  }
  const int hlen = lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  for (int i = tid; i < nm * hlen; i += kWG) {
    const int m = i / hlen, k = i - m * hlen;
    const uint32_t v = hist[m * A.hwords + k];
    if (v)
      atomicAdd(reinterpret_cast<unsigned long long *>(A.counters + (size_t)m * A.clen +
                                                       HPGQ_NUM_SCALARS + k),
                (unsigned long long)v);
  }
  if (tid < nm * HPGQ_NUM_SCALARS) {
    const unsigned long long v = sc[tid];
    const int m = tid / HPGQ_NUM_SCALARS, k = tid - m * HPGQ_NUM_SCALARS;
    if (v) atomicAdd(reinterpret_cast<unsigned long long *>(A.counters + (size_t)m * A.clen + k), v);
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

struct EngineGeom {
  int nch, slots, cap, hwords;
  size_t lds_bytes;
};

static EngineGeom engine_geom(int lmax, int nm) {
  EngineGeom g;
  g.nch = (lmax + 255) / 256;
  // reads per mate per tile: keep the two tile buffers near 80 KB so two
  // workgroups share a CU (160 KB LDS)
  int slots = 256 / nm;
  while (slots > 64 && (size_t)nm * 2 * ((size_t)slots * lmax + 32) > 80 * 1024) slots -= 64;
  g.slots = slots;
  g.cap = ((slots * lmax + 32) + 15) & ~15;
  g.hwords = ((lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS) + 3) & ~3;
  g.lds_bytes = (size_t)nm * 2 * g.cap + (size_t)nm * g.hwords * 4 +
                (size_t)nm * HPGQ_NUM_SCALARS * 8 + 256;
  // the end-of-kernel reduction reuses the tile region
  const size_t red = (size_t)nm * 6 * lmax * 4;
  if (red > (size_t)nm * 2 * g.cap) g.lds_bytes += red;   // never with slots >= 64
  return g;
}

}  // namespace hpgq

// ===========================================================================
// C-ABI
// ===========================================================================

#include <cstdlib>
#include <cstring>
#include <rccl/rccl.h>

struct hpgq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hpgq_params_t p{};
  int nm = 1;
  size_t clen = 0;
  uint64_t *d_counters = nullptr;
  int32_t *d_err = nullptr;
  hpgq::EngineGeom geom{};
  int grid = 0;
  // host-path device staging
  char *d_buf = nullptr;
  size_t d_buf_cap = 0;
  uint8_t *d_mask = nullptr;
  uint32_t *d_trim = nullptr;
  size_t d_out_cap = 0;
  ncclComm_t comm = nullptr;
};

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
    default: return "unknown error";
  }
}

const char *hpgq_version(void) { return "hpgq 0.1 (gfx950)"; }

int hpgq_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static int validate_params(const hpgq_params_t *p) {
  if (!p) return HPGQ_E_INVALID;
  if (p->lmax < 1 || p->lmax > HPGQ_LMAX_LIMIT) return HPGQ_E_INVALID;
  if (p->phred < 0 || p->phred > 255) return HPGQ_E_INVALID;
  return HPGQ_OK;
}

int hpgq_open(hpgq_ctx_t **out, int device, const hpgq_params_t *p) {
  if (!out) return HPGQ_E_INVALID;
  *out = nullptr;
  int rc = validate_params(p);
  if (rc) return rc;
  int ndev = 0;
  const hipError_t de = hipGetDeviceCount(&ndev);
  if (de != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "hpgq_open: hipGetDeviceCount -> %s, %d devices\n", hipGetErrorString(de), ndev);
    return HPGQ_E_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) return HPGQ_E_INVALID;
  hpgq_ctx *c = new hpgq_ctx();
  c->device = device;
  c->p = *p;
  c->nm = p->paired ? 2 : 1;
  c->clen = hpgq_counters_len(p->lmax);
  c->geom = hpgq::engine_geom(p->lmax, c->nm);
  HPGQ_HIP_TRY(hipSetDevice(device));
  HPGQ_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HPGQ_HIP_TRY(hipMalloc(&c->d_counters, c->clen * c->nm * sizeof(uint64_t)));
  HPGQ_HIP_TRY(hipMalloc(&c->d_err, sizeof(int32_t)));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_counters, 0, c->clen * c->nm * sizeof(uint64_t), c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
  int cus = 0;
  HPGQ_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  int per_cu = 0;
  const void *kfn = nullptr;
  switch (c->geom.nch) {
    case 1: kfn = (const void *)hpgq::engine_kernel<1>; break;
    case 2: kfn = (const void *)hpgq::engine_kernel<2>; break;
    case 3: kfn = (const void *)hpgq::engine_kernel<3>; break;
    default: kfn = (const void *)hpgq::engine_kernel<4>; break;
  }
  if (c->geom.lds_bytes > 64 * 1024)
    HPGQ_HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)c->geom.lds_bytes));
  HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, hpgq::kWG,
                                                            c->geom.lds_bytes));
  if (per_cu < 1) per_cu = 1;
  c->grid = cus * per_cu * 4;   // a few waves of tiles per slot keeps the tail short
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  *out = c;
  return HPGQ_OK;
}

void hpgq_close(hpgq_ctx_t *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  (void)hipFree(c->d_counters);
  (void)hipFree(c->d_err);
  (void)hipFree(c->d_buf);
  (void)hipFree(c->d_mask);
  (void)hipFree(c->d_trim);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static void fill_args(const hpgq_ctx *c, hpgq::EngineArgs &A) {
  const hpgq_params_t &p = c->p;
  A.lmax = p.lmax;
  A.clen = (int)c->clen;
  A.nm = c->nm;
  A.slots = c->geom.slots;
  A.cap = c->geom.cap;
  A.hwords = c->geom.hwords;
  A.phred = p.phred;
  A.filter_on = p.filter_on;
  A.edit_on = p.edit_on;
  A.stats_on = p.stats_on;
  A.min_len = p.min_read_length;
  A.max_len = p.max_read_length;
  A.min_q = p.min_read_quality;
  A.max_q = p.max_read_quality;
  A.max_oor = p.max_out_of_quality;
  A.check_oor = p.filter_on && p.max_out_of_quality < HPGQ_LMAX_LIMIT;
  // out of range  <=>  raw < phred + min_q  or  raw > phred + max_q
  const int64_t lo = (int64_t)p.phred + p.min_read_quality;
  const int64_t hi1 = (int64_t)p.phred + p.max_read_quality + 1;
  A.oor_lo_none = lo <= 0;
  A.oor_all = lo > 255 || hi1 <= 0;
  A.oor_hi_none = hi1 > 255;
  const uint32_t lob = (uint32_t)(lo < 0 ? 0 : lo > 255 ? 255 : lo);
  const uint32_t hib = (uint32_t)(hi1 < 0 ? 0 : hi1 > 255 ? 255 : hi1);
  A.oor_lo4 = lob * 0x01010101u;
  A.oor_hi4 = hib * 0x01010101u;
  A.max_n = p.max_N;
  A.left_len = p.left_length;
  A.min_left = p.min_left_quality;
  A.max_left = p.max_left_quality;
  A.right_len = p.right_length;
  A.min_right = p.min_right_quality;
  A.max_right = p.max_right_quality;
  A.e_left_len = p.edit_left_length;
  A.e_min_left = p.edit_min_left_quality;
  A.e_max_left = p.edit_max_left_quality;
  A.e_right_len = p.edit_right_length;
  A.e_min_right = p.edit_min_right_quality;
  A.e_max_right = p.edit_max_right_quality;
}

static int launch(hpgq_ctx *c, hpgq::EngineArgs &A) {
  if (A.num_reads <= 0) return HPGQ_OK;
  A.counters = c->d_counters;
  A.err = c->d_err;
  const int64_t ntiles = (A.num_reads + A.slots - 1) / A.slots;
  const int grid = (int)std::min<int64_t>(ntiles, c->grid);
  const dim3 g(grid), b(hpgq::kWG);
  const size_t lds = c->geom.lds_bytes;
  switch (c->geom.nch) {
    case 1: hipLaunchKernelGGL(hpgq::engine_kernel<1>, g, b, lds, c->stream, A); break;
    case 2: hipLaunchKernelGGL(hpgq::engine_kernel<2>, g, b, lds, c->stream, A); break;
    case 3: hipLaunchKernelGGL(hpgq::engine_kernel<3>, g, b, lds, c->stream, A); break;
    default: hipLaunchKernelGGL(hpgq::engine_kernel<4>, g, b, lds, c->stream, A); break;
  }
  HPGQ_HIP_TRY(hipGetLastError());
  return HPGQ_OK;
}

int hpgq_run_device(hpgq_ctx_t *c, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                    uint8_t *mask_out, uint32_t *trim_out) {
  if (!c || !b) return HPGQ_E_INVALID;
  if (c->nm == 2 && (!b2 || b2->num_reads != b->num_reads)) return HPGQ_E_INVALID;
  if (c->nm == 1 && b2) return HPGQ_E_INVALID;
  if (b->num_reads < 0) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  hpgq::EngineArgs A{};
  fill_args(c, A);
  A.num_reads = b->num_reads;
  A.seq[0] = b->seq; A.qual[0] = b->quality; A.idx[0] = b->data_indices;
  if (b2) { A.seq[1] = b2->seq; A.qual[1] = b2->quality; A.idx[1] = b2->data_indices; }
  A.mask = mask_out;
  A.trim = trim_out;
  return launch(c, A);
}

static int ensure_dev(hpgq_ctx *c, size_t bytes, size_t nreads) {
  if (bytes > c->d_buf_cap) {
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_buf);
    c->d_buf = nullptr;
    size_t cap = bytes + bytes / 4 + 4096;
    if (hipMalloc(&c->d_buf, cap) != hipSuccess) { c->d_buf_cap = 0; return HPGQ_E_NOMEM; }
    c->d_buf_cap = cap;
  }
  if (nreads > c->d_out_cap) {
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_mask);
    (void)hipFree(c->d_trim);
    size_t cap = nreads + nreads / 4 + 64;
    if (hipMalloc(&c->d_mask, cap) != hipSuccess) return HPGQ_E_NOMEM;
    if (hipMalloc(&c->d_trim, cap * 2 * sizeof(uint32_t)) != hipSuccess) return HPGQ_E_NOMEM;
    c->d_out_cap = cap;
  }
  return HPGQ_OK;
}

int hpgq_run_host(hpgq_ctx_t *c, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                  uint8_t *mask_out, uint32_t *trim_out) {
  if (!c || !b) return HPGQ_E_INVALID;
  if (c->nm == 2 && (!b2 || b2->num_reads != b->num_reads)) return HPGQ_E_INVALID;
  if (c->nm == 1 && b2) return HPGQ_E_INVALID;
  const int64_t n = b->num_reads;
  if (n < 0) return HPGQ_E_INVALID;
  if (n == 0) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  const hpgq_batch_t *bs[2] = {b, b2};
  size_t bytes[2] = {0, 0}, off[2][4];
  size_t total = 0;
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    bytes[m] = (size_t)(ix[n] - ix[0]);
    off[m][0] = total; total += (bytes[m] + 255) & ~(size_t)255;   // seq
    off[m][1] = total; total += (bytes[m] + 255) & ~(size_t)255;   // quality
    off[m][2] = total; total += ((size_t)(n + 1) * 4 + 255) & ~(size_t)255;
  }
  int rc = ensure_dev(c, total, (size_t)n);
  if (rc) return rc;
  hpgq::EngineArgs A{};
  fill_args(c, A);
  A.num_reads = n;
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    char *ds = c->d_buf + off[m][0], *dq = c->d_buf + off[m][1];
    int32_t *di = reinterpret_cast<int32_t *>(c->d_buf + off[m][2]);
    HPGQ_HIP_TRY(hipMemcpyAsync(ds, bs[m]->seq + ix[0], bytes[m], hipMemcpyHostToDevice, c->stream));
    HPGQ_HIP_TRY(hipMemcpyAsync(dq, bs[m]->quality + ix[0], bytes[m], hipMemcpyHostToDevice, c->stream));
    HPGQ_HIP_TRY(hipMemcpyAsync(di, ix, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    // absolute indices: shift the base pointers so data_indices need no rewrite
    A.seq[m] = ds - ix[0];
    A.qual[m] = dq - ix[0];
    A.idx[m] = di;
  }
  A.mask = mask_out ? c->d_mask : nullptr;
  A.trim = trim_out ? c->d_trim : nullptr;
  rc = launch(c, A);
  if (rc) return rc;
  if (mask_out) HPGQ_HIP_TRY(hipMemcpyAsync(mask_out, c->d_mask, (size_t)n, hipMemcpyDeviceToHost, c->stream));
  if (trim_out)
    HPGQ_HIP_TRY(hipMemcpyAsync(trim_out, c->d_trim, (size_t)n * c->nm * 4, hipMemcpyDeviceToHost,
                                c->stream));
  return HPGQ_OK;
}

int hpgq_sync(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  int32_t err = 0;
  HPGQ_HIP_TRY(hipMemcpy(&err, c->d_err, sizeof(err), hipMemcpyDeviceToHost));
  return err ? HPGQ_E_READ_TOO_LONG : HPGQ_OK;
}

int hpgq_reset(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_counters, 0, c->clen * c->nm * sizeof(uint64_t), c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
  return HPGQ_OK;
}

size_t hpgq_counters_size(const hpgq_ctx_t *c) { return c ? c->clen * c->nm : 0; }

int hpgq_read_counters(hpgq_ctx_t *c, uint64_t *out, size_t n) {
  if (!c || !out || n < c->clen * c->nm) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemcpyAsync(out, c->d_counters, c->clen * c->nm * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  return HPGQ_OK;
}

uint64_t *hpgq_counters_device(hpgq_ctx_t *c) { return c ? c->d_counters : nullptr; }
void *hpgq_stream(hpgq_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

// ---------------------------------------------------------------------------
// RCCL (one process per GPU): one in-place sum of the packed counters
// ---------------------------------------------------------------------------

static_assert(sizeof(ncclUniqueId) <= HPGQ_COMM_ID_BYTES, "nccl id size");

int hpgq_comm_unique_id(char id[HPGQ_COMM_ID_BYTES]) {
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return HPGQ_E_RCCL;
  std::memset(id, 0, HPGQ_COMM_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return HPGQ_OK;
}

int hpgq_comm_init(hpgq_ctx_t *c, int nranks, int rank, const char id[HPGQ_COMM_ID_BYTES]) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks) return HPGQ_E_INVALID;
  if (c->comm) return HPGQ_E_STATE;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  if (ncclCommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
    c->comm = nullptr;
    return HPGQ_E_RCCL;
  }
  return HPGQ_OK;
}

int hpgq_allreduce(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  if (!c->comm) return HPGQ_E_STATE;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  if (ncclAllReduce(c->d_counters, c->d_counters, c->clen * c->nm, ncclUint64, ncclSum, c->comm,
                    c->stream) != ncclSuccess)
    return HPGQ_E_RCCL;
  return HPGQ_OK;
}

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
    o->mean_quality_raw = (double)set[HPGQ_S_ACC_MEANQ_FX16] / 65536.0 / (double)o->num_reads;
  }
  return HPGQ_OK;
}

}  // extern "C"
