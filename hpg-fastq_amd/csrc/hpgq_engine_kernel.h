// hpgq_engine_kernel.h — the fused edit -> filter -> stats kernel (gfx950).
//
// Replaces, for one SoA batch resident in HBM:
//   fastq_edit          src/edit_fastq.c:154            (5'/3' trim)
//   fastq_filter        src/stats_fastq.c:224, src/filter_fastq.c:148, src/edit_fastq.c:166
//   fastq_reads_stats   src/stats_fastq.c:230,244
//   the consumer merge  src/stats_fastq.c:257-417       (per-read + per-base counters)
//
// Mapping: ONE WAVE PER READ, streaming straight from HBM (no LDS staging).
//   * reads are taken 64 at a time (a "block"); the block prologue loads the
//     64 read offsets coalesced (lane j <-> read j) and precomputes, per lane,
//     the aligned byte offset and alignment of read j in both buffers.
//   * per read, v_readlane puts those in SGPRs; lane l then loads ONE dword per
//     buffer with a buffer_load (SRD bounds check instead of per-lane clamps;
//     offset = SGPR read offset + lane*4) and takes its right neighbour's
//     dword by DPP wave_shl:1; v_alignbyte realigns the window so lane l < 63
//     holds positions 4l..4l+3 (+252c for chunk c).  Lane 63 only donates its
//     word.
//   * per-read sums (raw quality via v_sad_u8, G/C, N, out-of-range counts by
//     SWAR zero-byte / byte-compare tests) are packed into one or two u32 and
//     reduced with DPP row_shr + row_bcast; the pass/fail decision is then
//     wave-uniform 32-bit scalar arithmetic.
//   * per-position base counters: v_perm_b32 maps each base byte to a field
//     shift; 5 six-bit fields (A,C,G,T,N) per position in one u32, quality
//     sums as 16-bit pairs; every 63 reads flushed into per-workgroup LDS u32
//     arrays (ds_add), no global atomics on the per-base path.
//   * per-read results go to lane j of three VGPRs (v_writelane); the block
//     epilogue does the histogram-key divisions, the LDS histogram atomics and
//     the coalesced mask / trim stores vectorised over lanes.
//   * loads are register-pipelined: group g+1 (kU reads) is in flight while
//     group g is processed, across block boundaries; every group issue has a
//     fixed load count so the compiler counts vmcnt statically.
//   * at kernel end each workgroup adds its LDS partials into its own row of a
//     u64 slab (plain RMW); a reduce kernel folds the rows when counters are read.
// FAST instances (template GEN = false) handle the common filter (length and
// mean-quality bounds) with stats; GEN = true adds N / out-of-range /
// left/right windows / edit, selected at run time.
// All arithmetic is integer; results are bit-identical to the oracle.
#pragma once
#include "hpgq_common.h"

namespace hpgq {

constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;
constexpr int kFlushEvery = 63;   // 6-bit base fields
constexpr int kChunk = 252;       // positions per chunk (63 lanes x 4)

// flags (EngineArgs::flags)
constexpr int F_FILTER = 1, F_EDIT = 2, F_STATS = 4, F_NEED_N = 8, F_NEED_OOR = 16, F_NEED_LR = 32,
              F_OOR_LO_NONE = 64, F_OOR_HI_NONE = 128, F_OOR_ALL = 256;

// parameters only the rarer (GEN) paths read; copied into LDS at kernel start
struct ColdParams {
  int left_len, min_left, max_left;
  int right_len, min_right, max_right;
  int e_left_len, e_right_len;
  uint32_t el_lo4, el_hi4, er_lo4, er_hi4;     // edit in-range raw bounds (lo, hi+1)
  int el_lo_none, el_hi_none, el_none_in, er_lo_none, er_hi_none, er_none_in;
  uint32_t oor_lo4, oor_hi4;
  int max_n, max_oor;
};

struct EngineArgs {
  const char *seq[2];
  const char *qual[2];
  const int32_t *idx[2];
  uint8_t *mask;
  uint32_t *trim;
  uint64_t *slab;        // [gridDim.x][nm * clen]
  int32_t *err;
  const ColdParams *cold;
  int64_t num_reads;
  int lmax, clen, phred, flags;
  // pass iff min_len <= wn <= max_len and min_q*wn <= S - phred*wn <= max_q*wn
  int min_len, max_len, min_q, max_q;   // min_q/max_q clamped so that *1260 fits int32
};

// ---------------------------------------------------------------------------
// SWAR + wave helpers
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {   // 0x80 per zero byte
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

__device__ __forceinline__ uint32_t ge_bytes(uint32_t x, uint32_t c4) {   // 0x80 where x >= c
  const uint32_t d = (x | 0x80808080u) - (c4 & 0x7F7F7F7Fu);
  return ((x & ~c4) | (~(x ^ c4) & d)) & 0x80808080u;
}

// bytes of a lane word holding positions < nv (nv relative to the lane's first
// byte): branch-free, 64-bit shift so that nv >= 4 gives all ones
__device__ __forceinline__ uint32_t byte_mask(int nv) {
  const int t = min(max(nv, 0), 4);
  return ~(uint32_t)(0xFFFFFFFFFFFFFFFFull << (8 * t));
}

__device__ __forceinline__ uint32_t in_range(uint32_t w, uint32_t lo4, uint32_t hi4, int lo_none,
                                             int hi_none, int none_in) {
  if (none_in) return 0u;
  uint32_t r = 0x80808080u;
  if (!lo_none) r &= ge_bytes(w, lo4);
  if (!hi_none) r &= ~ge_bytes(w, hi4);
  return r;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);    // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);    // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);    // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);    // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);   // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_min(int v) {
  const int big = 0x7FFFFFFF;
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x111, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x112, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x114, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x118, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x142, 0xA, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(big, v, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_max(int v) {
  const int small = -0x7FFFFFFF;
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x111, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x112, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x114, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x118, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x142, 0xA, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(small, v, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(v, 63);
}

// lane i <- lane i+1 (wave_shl:1); lane 63 gets 0
__device__ __forceinline__ uint32_t next_lane(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// v[lane j] = val (val, j wave-uniform).  v_writelane takes the lane from M0:
// two SGPR operands would break the constant-bus limit.
__device__ __forceinline__ uint32_t put_lane(uint32_t v, uint32_t val, int j) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tv_writelane_b32 %0, %1, m0"
               : "+v"(v) : "s"(val), "s"(j) : "m0");
  return v;
}

// field shift per base code; code = byte & 7 is one-to-one on A,C,G,T,N:
//   pad(0x08)->0 'A'->1 'C'->3 'T'->4 'N'->6 'G'->7, codes 2 and 5 unused
// fields: A bits 0-5, C 6-11, G 12-17, T 18-23, N 24-29, bits 30-31 garbage.
// A byte whose code matches but whose value does not (lowercase, IUPAC, ...)
// fails the `expected byte` check and is sent to the garbage field.
constexpr uint32_t kExpLo = 0x43004108u;   // expected byte for codes 0..3
constexpr uint32_t kExpHi = 0x474E0054u;   // codes 4..7
constexpr uint32_t kShLo = 0x061E001Eu;    // shifts for codes 0..3: 30, 0, 30, 6
constexpr uint32_t kShHi = 0x0C181E12u;    // codes 4..7: 18, 30, 24, 12

// ---------------------------------------------------------------------------
// per-mate buffers
// ---------------------------------------------------------------------------

struct MateBuf {
  __amdgpu_buffer_rsrc_t rs, rq;   // SRDs over the 4-byte aligned-down bases
  int bs, bq;                      // base misalignment (ptr & 3)
};

__device__ __forceinline__ MateBuf make_mate(const char *seq, const char *qual, int data_end) {
  MateBuf b;
  const uintptr_t ps = reinterpret_cast<uintptr_t>(seq), pq = reinterpret_cast<uintptr_t>(qual);
  b.bs = (int)(ps & 3);
  b.bq = (int)(pq & 3);
  // bounds: every byte up to data_end, rounded up to a whole dword (same page)
  const int ns = (b.bs + data_end + 3) & ~3, nq = (b.bq + data_end + 3) & ~3;
  b.rs = __builtin_amdgcn_make_buffer_rsrc((void *)(ps - b.bs), (short)0, ns, 0x00020000);
  b.rq = __builtin_amdgcn_make_buffer_rsrc((void *)(pq - b.bq), (short)0, nq, 0x00020000);
  return b;
}

template <int NCH>
struct Pending {            // issued loads for one read of one mate
  uint32_t s[NCH], q[NCH];
};

// wave-uniform read descriptor, unpacked from the block prologue's lane j
struct ReadRef {
  uint32_t os, oq;   // aligned byte offsets (dword) into the SRDs
  int als, alq;      // byte alignment of the read start
  int n;             // length
};

// loads: lane l, chunk c reads the dword at os + 4*(63c + l); reads past the
// data end return 0 (SRD bound), past the read end they are garbage we mask
template <int NCH>
__device__ __forceinline__ void issue(const MateBuf &b, const ReadRef &r, uint32_t lane4,
                                      Pending<NCH> &p) {
  // readfirstlane: the offsets are uniform, say so (else hipcc may waterfall)
  const uint32_t os = (uint32_t)uni((int)r.os), oq = (uint32_t)uni((int)r.oq);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    p.s[c] = __builtin_amdgcn_raw_buffer_load_b32(b.rs, lane4 + 252 * c, os, 0);
    p.q[c] = __builtin_amdgcn_raw_buffer_load_b32(b.rq, lane4 + 252 * c, oq, 0);
  }
}

// window-aligned words: lane bytes = positions p0..p0+3
template <int NCH>
__device__ __forceinline__ void finish(const ReadRef &r, const Pending<NCH> &p,
                                       uint32_t (&sw)[NCH], uint32_t (&qw)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    sw[c] = __builtin_amdgcn_alignbyte(next_lane(p.s[c]), p.s[c], (uint32_t)r.als);
    qw[c] = __builtin_amdgcn_alignbyte(next_lane(p.q[c]), p.q[c], (uint32_t)r.alq);
  }
}

template <int NCH>
struct PosAcc {
  uint32_t pk[NCH][4];
  uint32_t q02[NCH], q13[NCH];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      q02[c] = q13[c] = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) pk[c][i] = 0;
    }
  }
  // pos_acc: [6][lmax] u32 in LDS (qsum, A, C, G, T, N); pos0 = lane's first position
  __device__ __forceinline__ void flush(uint32_t *pos_acc, int lmax, int pos0) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t qv[4] = {q02[c] & 0xFFFFu, q13[c] & 0xFFFFu, q02[c] >> 16, q13[c] >> 16};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = pos0 + kChunk * c + i;
        if (pos < lmax) {
          atomicAdd(&pos_acc[pos], qv[i]);
#pragma unroll
          for (int b = 0; b < 5; ++b)
            atomicAdd(&pos_acc[(1 + b) * lmax + pos], (pk[c][i] >> (6 * b)) & 63u);
        }
        pk[c][i] = 0;
      }
      q02[c] = q13[c] = 0;
    }
  }
  __device__ __forceinline__ void add(const uint32_t (&sw)[NCH], const uint32_t (&qw)[NCH],
                                      const uint32_t (&m)[NCH]) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t s = (sw[c] & m[c]) | (0x08080808u & ~m[c]);   // pad -> garbage field
      const uint32_t q = qw[c] & m[c];
      const uint32_t codes = s & 0x07070707u;
      uint32_t sh = __builtin_amdgcn_perm(kShHi, kShLo, codes);
      const uint32_t ex = __builtin_amdgcn_perm(kExpHi, kExpLo, codes);
      if (__builtin_expect(s != ex, 0)) {   // bytes that are not exactly A/C/G/T/N
        const uint32_t d = s ^ ex;
        const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
        const uint32_t ff = (nz >> 7) * 0xFFu;
        sh = (sh & ~ff) | (0x1E1E1E1Eu & ff);
      }
      pk[c][0] += 1u << (sh & 31u);
      pk[c][1] += 1u << ((sh >> 8) & 31u);
      pk[c][2] += 1u << ((sh >> 16) & 31u);
      pk[c][3] += 1u << ((sh >> 24) & 31u);
      q02[c] += q & 0x00FF00FFu;
      q13[c] += (q >> 8) & 0x00FF00FFu;
    }
  }
};

// per-read outcome (wave-uniform)
struct ReadOut {
  uint32_t r1;   // raw quality sum | GC << 18
  int wn, ts, te;
  bool pass;
};

template <bool GEN, int NCH>
__device__ __forceinline__ ReadOut evaluate(const EngineArgs &A, const ColdParams &C,
                                            const uint32_t (&sw)[NCH], const uint32_t (&qw)[NCH],
                                            const uint32_t (&m)[NCH], int wn, int lane_p0) {
  uint32_t p1 = 0, p2 = 0, pl = 0, pr = 0;
  int kl = 0, kr = 0;
  if (GEN && (A.flags & F_NEED_LR)) {
    kl = min(C.left_len, wn);
    kr = min(C.right_len, wn);
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int p0 = lane_p0 + kChunk * c;
    const uint32_t m80 = m[c] & 0x80808080u;
    const uint32_t q = qw[c] & m[c];
    p1 += __builtin_amdgcn_sad_u8(q, 0u, 0u);
    p1 += (uint32_t)__builtin_popcount(zero_bytes((sw[c] | 0x04040404u) ^ 0x47474747u) & m80) << 18;
    if (GEN) {
      if (A.flags & (F_NEED_N | F_NEED_OOR)) {
        uint32_t x = 0;
        if (A.flags & F_NEED_N) x = __builtin_popcount(zero_bytes(sw[c] ^ 0x4E4E4E4Eu) & m80);
        if (A.flags & F_NEED_OOR) {
          uint32_t bad;
          if (A.flags & F_OOR_ALL) {
            bad = 0x80808080u;
          } else {
            bad = 0;
            if (!(A.flags & F_OOR_LO_NONE)) bad |= ~ge_bytes(qw[c], C.oor_lo4) & 0x80808080u;
            if (!(A.flags & F_OOR_HI_NONE)) bad |= ge_bytes(qw[c], C.oor_hi4);
          }
          x += (uint32_t)__builtin_popcount(bad & m80) << 16;
        }
        p2 += x;
      }
      if (A.flags & F_NEED_LR) {
        if (kl > 0) pl += __builtin_amdgcn_sad_u8(q & byte_mask(kl - p0), 0u, 0u);
        if (kr > 0) pr += __builtin_amdgcn_sad_u8(q & ~byte_mask(wn - kr - p0), 0u, 0u);
      }
    }
  }
  ReadOut o;
  o.r1 = wave_sum(p1);
  o.wn = wn;
  o.ts = o.te = 0;
  bool pass = true;
  if (A.flags & F_FILTER) {
    const int sq = (int)(o.r1 & 0x3FFFFu) - A.phred * wn;
    pass = (wn >= A.min_len) & (wn <= A.max_len) & (A.min_q * wn <= sq) & (sq <= A.max_q * wn);
    if (GEN) {
      if (A.flags & (F_NEED_N | F_NEED_OOR)) {
        const uint32_t r2 = wave_sum(p2);
        if ((A.flags & F_NEED_N) && (int)(r2 & 0xFFFFu) > C.max_n) pass = false;
        if ((A.flags & F_NEED_OOR) && (int)(r2 >> 16) > C.max_oor) pass = false;
      }
      if (A.flags & F_NEED_LR) {
        if (kl > 0) {
          const int64_t s = (int64_t)wave_sum(pl) - (int64_t)A.phred * kl;
          if (!((int64_t)C.min_left * kl <= s && s <= (int64_t)C.max_left * kl)) pass = false;
        }
        if (kr > 0) {
          const int64_t s = (int64_t)wave_sum(pr) - (int64_t)A.phred * kr;
          if (!((int64_t)C.min_right * kr <= s && s <= (int64_t)C.max_right * kr)) pass = false;
        }
      }
    }
  }
  o.pass = pass;
  return o;
}

// edit (A6): trim lengths from the raw, read-aligned quality words
template <int NCH>
__device__ __forceinline__ void trim_read(const ColdParams &C, const uint32_t (&qw)[NCH], int n,
                                          int lane_p0, int &ts, int &te) {
  ts = 0;
  te = 0;
  if (C.e_left_len > 0) {
    const int lim = min(C.e_left_len, n);
    int cand = 0x7FFFFFFF;
#pragma unroll
    for (int c = NCH - 1; c >= 0; --c) {
      const int p0 = lane_p0 + kChunk * c;
      const uint32_t ok = in_range(qw[c], C.el_lo4, C.el_hi4, C.el_lo_none, C.el_hi_none,
                                   C.el_none_in) & byte_mask(lim - p0);
      if (ok) cand = p0 + (__builtin_ctz(ok) >> 3);
    }
    ts = min(wave_min(cand), lim);
  }
  if (C.e_right_len > 0) {
    const int lim = min(C.e_right_len, n - ts);
    if (lim > 0) {
      int cand = -1;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int p0 = lane_p0 + kChunk * c;
        const uint32_t ok = in_range(qw[c], C.er_lo4, C.er_hi4, C.er_lo_none, C.er_hi_none,
                                     C.er_none_in) & byte_mask(n - p0) & ~byte_mask(n - lim - p0);
        if (ok) cand = p0 + ((31 - __builtin_clz(ok)) >> 3);
      }
      const int last = wave_max(cand);
      te = last < 0 ? lim : (n - 1 - last);
    }
  }
}

template <int NM, int NCH, bool GEN>
__global__ void __launch_bounds__(kWG) engine_kernel(EngineArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int lmax = A.lmax;
  const int hlen = lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  // lane l < 63 owns positions 4l.. of every chunk; lane 63 none
  const int lane_p0 = lane < 63 ? 4 * lane : 0x40000000;
  const uint32_t lane4 = 4u * (uint32_t)lane;

  // LDS: pos_acc [NM][6][lmax] u32 | hist [NM][hlen] u32 | sc [NM][8] u64 | cold
  uint32_t *pos_acc = reinterpret_cast<uint32_t *>(lds);
  uint32_t *hist = pos_acc + NM * 6 * lmax;
  const int hist_words = (NM * hlen + 1) & ~1;
  unsigned long long *sc = reinterpret_cast<unsigned long long *>(hist + hist_words);
  ColdParams *cold = reinterpret_cast<ColdParams *>(sc + NM * HPGQ_NUM_SCALARS);
  for (int i = tid; i < NM * 6 * lmax + hist_words; i += kWG) pos_acc[i] = 0;
  for (int i = tid; i < NM * HPGQ_NUM_SCALARS; i += kWG) sc[i] = 0;
  if (GEN && tid < (int)(sizeof(ColdParams) / 4))
    reinterpret_cast<uint32_t *>(cold)[tid] = reinterpret_cast<const uint32_t *>(A.cold)[tid];
  __syncthreads();

  MateBuf mb[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m)
    mb[m] = make_mate(A.seq[m], A.qual[m], uni(A.idx[m][A.num_reads]));

  PosAcc<NCH> acc[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m].zero();
  int since_flush = 0;
  uint64_t fx16[NM];
  uint32_t cnt[NM][7];   // input, passed, failed, edited, stats, long, any-long (wave-uniform)
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    fx16[m] = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) cnt[m][k] = 0;
  }

  // reads per pipeline group (two groups of registers in flight)
  constexpr int kU = ((NM == 1 ? 8 : 4) / NCH) > 0 ? ((NM == 1 ? 8 : 4) / NCH) : 1;
  const int64_t nblocks = (A.num_reads + 63) / 64;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kWaves;

  // block prologue: lane j describes read r0 + j of mate m
  //   off_s/off_q: aligned byte offsets; info: n | als << 16 | alq << 20
  auto load_block = [&](int64_t blk, uint32_t (&off_s)[NM], uint32_t (&off_q)[NM],
                        uint32_t (&info)[NM]) {
    const int64_t r0 = blk * 64;
    const int nr = (int)min((int64_t)64, A.num_reads - r0);
    const int l = min(lane, nr - 1);
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int a = A.idx[m][r0 + l], e = A.idx[m][r0 + l + 1];
      const uint32_t xs = (uint32_t)(mb[m].bs + a), xq = (uint32_t)(mb[m].bq + a);
      off_s[m] = xs & ~3u;
      off_q[m] = xq & ~3u;
      info[m] = (uint32_t)(e - a) | ((xs & 3u) << 16) | ((xq & 3u) << 20);
    }
  };
  auto ref_of = [&](const uint32_t (&off_s)[NM], const uint32_t (&off_q)[NM],
                    const uint32_t (&info)[NM], int m, int j) {
    ReadRef r;
    r.os = __builtin_amdgcn_readlane(off_s[m], j);
    r.oq = __builtin_amdgcn_readlane(off_q[m], j);
    const uint32_t inf = __builtin_amdgcn_readlane(info[m], j);
    r.n = (int)(inf & 0xFFFFu);
    r.als = (int)((inf >> 16) & 3u);
    r.alq = (int)((inf >> 20) & 3u);
    return r;
  };

  Pending<NCH> grp[2][kU][NM];
  auto load_group = [&](const uint32_t (&os)[NM], const uint32_t (&oq)[NM],
                        const uint32_t (&inf)[NM], int nr, int g, int slot) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int j = min(g * kU + u, nr - 1);   // past the block end: reload the last read
#pragma unroll
      for (int m = 0; m < NM; ++m) issue<NCH>(mb[m], ref_of(os, oq, inf, m, j), lane4, grp[slot][u][m]);
    }
  };

  uint32_t os[NM], oq[NM], inf[NM], osn[NM], oqn[NM], infn[NM];
  int64_t blk = gw;
  if (blk < nblocks) {
    load_block(blk, os, oq, inf);
    load_group(os, oq, inf, (int)min((int64_t)64, A.num_reads - blk * 64), 0, 0);
  }
  for (; blk < nblocks; blk += nw) {
    const int64_t r0 = blk * 64;
    const int nr = (int)min((int64_t)64, A.num_reads - r0);
    const int64_t nblk = blk + nw < nblocks ? blk + nw : blk;   // next block (or self)
    const int nnr = (int)min((int64_t)64, A.num_reads - nblk * 64);
    load_block(nblk, osn, oqn, infn);
    // per-read results, lane j <-> read r0 + j
    uint32_t res_r1[NM], res_info[NM], res_trim[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) res_r1[m] = res_info[m] = res_trim[m] = 0;

    auto process_group = [&](int g, int slot) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int j = g * kU + u;
        if (j >= nr) break;
        ReadOut out[NM];
        uint32_t sw[NM][NCH], qw[NM][NCH], mk[NM][NCH];
        bool lng[NM];
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const ReadRef rr = ref_of(os, oq, inf, m, j);
          finish<NCH>(rr, grp[slot][u][m], sw[m], qw[m]);
          int ts = 0, te = 0;
          if (GEN && (A.flags & F_EDIT) && rr.n <= kChunk * NCH) {
            trim_read<NCH>(*cold, qw[m], rr.n, lane_p0, ts, te);
            if (ts > 0) {   // window no longer starts at the read start: realign
              ReadRef r2 = rr;
              const uint32_t xs = rr.os + (uint32_t)(rr.als + ts), xq = rr.oq + (uint32_t)(rr.alq + ts);
              r2.os = xs & ~3u;
              r2.oq = xq & ~3u;
              r2.als = (int)(xs & 3u);
              r2.alq = (int)(xq & 3u);
              Pending<NCH> p2;
              issue<NCH>(mb[m], r2, lane4, p2);
              finish<NCH>(r2, p2, sw[m], qw[m]);
            }
          }
          const int wn = rr.n - ts - te;
#pragma unroll
          for (int c = 0; c < NCH; ++c) mk[m][c] = byte_mask(wn - lane_p0 - kChunk * c);
          out[m] = evaluate<GEN, NCH>(A, *cold, sw[m], qw[m], mk[m], wn, lane_p0);
          out[m].ts = ts;
          out[m].te = te;
          lng[m] = rr.n > lmax;
        }
        bool pass = out[0].pass;
        if (NM == 2) pass = pass && out[NM - 1].pass;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          if ((A.flags & F_STATS) && pass && !lng[m]) acc[m].add(sw[m], qw[m], mk[m]);
          const uint32_t info = (uint32_t)out[m].wn | ((uint32_t)pass << 16) |
                                ((uint32_t)lng[m] << 17) |
                                ((uint32_t)(out[m].ts + out[m].te > 0) << 18);
          res_r1[m] = put_lane(res_r1[m], out[m].r1, j);
          res_info[m] = put_lane(res_info[m], info, j);
          if (GEN) res_trim[m] = put_lane(res_trim[m], (uint32_t)out[m].ts | ((uint32_t)out[m].te << 16), j);
        }
        if ((A.flags & F_STATS) && pass && ++since_flush == kFlushEvery) {
#pragma unroll
          for (int m = 0; m < NM; ++m) acc[m].flush(pos_acc + m * 6 * lmax, lmax, lane_p0);
          since_flush = 0;
        }
      }
    };

    // group g of this block sits in slot g & 1; the group after the last one
    // is the next block's group 0 (full blocks have an even group count, so it
    // lands in slot 0, where the next block expects it)
    const int ngroups = (nr + kU - 1) / kU;
    for (int g = 0; g < ngroups; g += 2) {
      if (g + 1 < ngroups) load_group(os, oq, inf, nr, g + 1, 1);
      else load_group(osn, oqn, infn, nnr, 0, 1);
      process_group(g, 0);
      if (g + 1 < ngroups) {
        if (g + 2 < ngroups) load_group(os, oq, inf, nr, g + 2, 0);
        else load_group(osn, oqn, infn, nnr, 0, 0);
        process_group(g + 1, 1);
      }
    }

    // ---- block epilogue, vectorised over lanes (lane j = read r0 + j) ------
    const bool valid = lane < nr;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const uint32_t info = res_info[m];
      const int wn = (int)(info & 0xFFFFu);
      const bool pass = valid && ((info >> 16) & 1u);
      const bool lg = valid && ((info >> 17) & 1u);
      const bool edited = valid && ((info >> 18) & 1u);
      if (valid) {
        if (m == 0 && A.mask) A.mask[r0 + lane] = (uint8_t)pass;
        if (A.trim) A.trim[(int64_t)m * A.num_reads + r0 + lane] = res_trim[m];
      }
      cnt[m][0] += (uint32_t)nr;
      cnt[m][1] += (uint32_t)__builtin_popcountll(__ballot(pass));
      cnt[m][2] += (uint32_t)__builtin_popcountll(__ballot(valid && !pass));
      cnt[m][3] += (uint32_t)__builtin_popcountll(__ballot(edited));
      cnt[m][6] += (uint32_t)__builtin_popcountll(__ballot(lg));
      if (A.flags & F_STATS) {
        cnt[m][4] += (uint32_t)__builtin_popcountll(__ballot(pass));
        cnt[m][5] += (uint32_t)__builtin_popcountll(__ballot(pass && lg));
        if (pass && !lg) {
          uint32_t *hm = hist + m * hlen;
          const uint32_t r1 = res_r1[m];
          const uint32_t s = r1 & 0x3FFFFu, gc = r1 >> 18, n = (uint32_t)wn;
          atomicAdd(&hm[n], 1u);
          if (n > 0) {
            atomicAdd(&hm[lmax + 1 + (2 * s + n) / (2 * n)], 1u);
            atomicAdd(&hm[lmax + 1 + HPGQ_MEANQ_BINS + (100 * gc) / n], 1u);
            const uint32_t q = s / n, rem = s - q * n;
            fx16[m] += ((uint64_t)q << 16) + (((uint32_t)rem << 16) / n);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      os[m] = osn[m];
      oq[m] = oqn[m];
      inf[m] = infn[m];
    }
  }

  // ---- workgroup epilogue ---------------------------------------------------
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m].flush(pos_acc + m * 6 * lmax, lmax, lane_p0);
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    // fx16: u64 per lane -> wave sum in 16-bit slices (no overflow)
    const uint32_t lo = (uint32_t)fx16[m], hi = (uint32_t)(fx16[m] >> 32);
    const uint64_t tot = (uint64_t)wave_sum(lo & 0xFFFFu) + ((uint64_t)wave_sum(lo >> 16) << 16) +
                         ((uint64_t)wave_sum(hi) << 32);
    if (lane == 0) {
      unsigned long long *scm = sc + m * HPGQ_NUM_SCALARS;
      if (cnt[m][0]) atomicAdd(&scm[HPGQ_S_NUM_INPUT], (unsigned long long)cnt[m][0]);
      if (cnt[m][1]) atomicAdd(&scm[HPGQ_S_NUM_PASSED], (unsigned long long)cnt[m][1]);
      if (cnt[m][2]) atomicAdd(&scm[HPGQ_S_NUM_FAILED], (unsigned long long)cnt[m][2]);
      if (cnt[m][3]) atomicAdd(&scm[HPGQ_S_NUM_EDITED], (unsigned long long)cnt[m][3]);
      if (cnt[m][4]) atomicAdd(&scm[HPGQ_S_NUM_STATS], (unsigned long long)cnt[m][4]);
      if (cnt[m][5]) atomicAdd(&scm[HPGQ_S_LONG_READS], (unsigned long long)cnt[m][5]);
      if (tot) atomicAdd(&scm[HPGQ_S_ACC_MEANQ_FX16], (unsigned long long)tot);
      if (cnt[m][6] && A.err) atomicOr(A.err, 1);
    }
  }
  __syncthreads();
  // add this workgroup's partials into its slab row (no other block touches it)
  uint64_t *row = A.slab + (size_t)blockIdx.x * NM * A.clen;
  const int off_pos = HPGQ_NUM_SCALARS + hlen;
  for (int m = 0; m < NM; ++m) {
    uint64_t *rm = row + (size_t)m * A.clen;
    for (int i = tid; i < HPGQ_NUM_SCALARS; i += kWG) rm[i] += sc[m * HPGQ_NUM_SCALARS + i];
    for (int i = tid; i < hlen; i += kWG) rm[HPGQ_NUM_SCALARS + i] += hist[m * hlen + i];
    for (int i = tid; i < 6 * lmax; i += kWG) rm[off_pos + i] += pos_acc[m * 6 * lmax + i];
  }
}

// fold the slab rows into the counters and clear them:
//   counters[k] += sum_rows slab[row][k]; slab[row][k] = 0
__global__ void __launch_bounds__(256) slab_reduce_kernel(uint64_t *slab, int rows, int len,
                                                          uint64_t *counters) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= len) return;
  uint64_t s = 0;
  for (int r = 0; r < rows; ++r) {
    s += slab[(size_t)r * len + k];
    slab[(size_t)r * len + k] = 0;
  }
  counters[k] += s;
}

}  // namespace hpgq
