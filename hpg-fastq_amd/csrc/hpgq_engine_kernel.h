// hpgq_engine_kernel.h — the fused edit -> filter -> stats kernels (gfx950):
// shared arguments, read routing and the catch-all one-wave-per-read kernel.
//
// Replaces, for one SoA batch resident in HBM:
//   fastq_edit          src/edit_fastq.c:154            (5'/3' trim)
//   fastq_filter        src/stats_fastq.c:224, src/filter_fastq.c:148, src/edit_fastq.c:166
//   fastq_reads_stats   src/stats_fastq.c:230,244
//   the consumer merge  src/stats_fastq.c:257-417       (per-read + per-base counters)
//
// Read routing.  A batch runs through a short chain of
// kernels on the ctx stream.  The first (the segmented kernel of
// hpgq_engine_tri.h) takes every read whose length fits its geometry and
// DEFERS the others: per unit (one of its read blocks) it stores a 64-bit mask
// of the deferred reads and counts them.  The next kernel in the chain walks
// those masks instead of the batch (a "follow-up" stage); it exits at once when
// the count is zero, which is the usual case.  The last stage is engine_kernel
// below, which takes any read of any length, so every read is processed by
// exactly one stage and the counters of all stages add up.
//
// engine_kernel mapping: ONE WAVE PER READ, streaming straight from HBM.
//   * reads are taken per unit (64 reads, or the deferred reads of an earlier
//     stage's unit, compacted); the unit prologue loads the read offsets (lane
//     j <-> read j) and precomputes the aligned byte offsets and alignments.
//   * per read, v_readlane puts those in SGPRs; lane l then loads ONE dword per
//     buffer and 252-position chunk with a buffer_load (SRD bounds check, offset
//     = SGPR read offset + lane*4) and takes its right neighbour's dword by DPP
//     wave_shl:1; v_alignbyte realigns so lane l < 63 holds positions 4l..4l+3.
//   * per-read sums (biased quality via v_sad_u8, G/C, N, out-of-range counts) are
//     reduced with DPP row_shr + row_bcast; the pass/fail decision is then
//     wave-uniform scalar arithmetic.
//   * per-position base counters: v_perm_b32 maps each base byte to a field
//     shift; 5 six-bit fields (A,C,G,T,N) per position in one u32, quality
//     sums as 16-bit pairs; every 63 reads flushed into per-workgroup LDS.
//   * reads longer than the NCH chunks the pipeline holds take a chunk loop
//     (long_trim / long_eval): filter and edit for any length; a merged
//     window longer than lmax is merged by long_merge (positions < lmax on
//     chip, the rest into the ctx's long-read tail).
//   * the workgroup epilogue adds its LDS partials into the ctx counters with
//     one no-return u64 global atomic per nonzero entry (no slab, no fold).
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
              F_OOR_LO_NONE = 64, F_OOR_HI_NONE = 128, F_OOR_ALL = 256,
              F_TAIL_ONLY = 512;   // the long-read tail's second pass (hpgq_sync): tail entries only

// One edit side's in-range test on RAW quality dwords w (biased b = w ^ 0x80,
// range [lo, hi1) biased), branch-free: with x = w ^ 0x80 the SWAR "x >= c"
// of bit 7 per byte is (~w & cq) | (~(w ^ cq) & ((w | 0x80) - c7)), cq = c ^
// 0x80, c7 = c & 0x7F (trim_side_ok).  lq / l7 and hq / h7 are those of lo4
// and hi4.  No upper bound: hq = 0, h7 = 0x80 (the formula is then 0 for
// every byte); no lower bound: lo4 = 0 (always >=); an empty range: lo4 = hi4
// = 0 (every byte >= both: none in range).
struct TrimSide {
  uint32_t lq, l7, hq, h7;
};

// parameters only the rarer paths read
struct ColdParams {
  int left_len, min_left, max_left;
  int right_len, min_right, max_right;
  int e_left_len, e_right_len;
  uint32_t el_lo4, el_hi4, er_lo4, er_hi4;     // edit in-range raw bounds (lo, hi+1)
  int el_lo_none, el_hi_none, el_none_in, er_lo_none, er_hi_none, er_none_in;
  uint32_t oor_lo4, oor_hi4;
  int max_n, max_oor;
  TrimSide tl, tr;   // the edit windows' in-range tests (segmented kernels' trim_finish)
  TrimSide to;       // the filter's quality range (segmented kernels' out-of-range count)
};

struct EngineArgs {
  const char *seq[2];
  const char *qual[2];
  const int32_t *idx[2];
  uint8_t *mask;
  uint32_t *trim;
  uint64_t *counters;    // [nm][clen], accumulated with global atomics
  int32_t *err;
  const ColdParams *cold;
  int64_t num_reads;     // of the batch (data end, paired trim offset)
  int lmax, clen, phred, flags;
  // pass iff min_len <= wn <= max_len and min_q*wn <= S - phred*wn <= max_q*wn
  int min_len, max_len, min_q, max_q;   // min_q/max_q clamped so that *1260 fits int32
  // ---- read routing (see the header comment) ----
  // follow-up stage: unit u holds the reads u*unit_reads + b for the set bits b
  // of unit_bits[u] & unit_and[u] (unit_and may be null); nullptr: this kernel
  // takes the whole batch in units of its own block size
  const uint64_t *unit_bits;
  const uint64_t *unit_and;
  int64_t nunits;
  int unit_reads;
  const uint32_t *pending;    // follow-up: reads deferred to this stage (0: exit at once)
  uint32_t *pending_clear;    // follow-up: the same counter of the next call, zeroed here
  uint32_t *pending_clear2;   // (a chain without stage 2: the next call's stage-2 counter too)
  // deferral out (segmented kernels): reads longer than defer_len go to the next
  // stage: bits per unit (every unit this kernel visits stores its word) + count
  uint64_t *defer_bits;
  uint32_t *defer_count;
  int defer_len;
  // follow-up: host-mapped words [deferred reads, batch reads, call sequence
  // number] for the host's choice of the next call's first stage (may be null)
  uint32_t *report;
  uint32_t report_seq;
  // ---- the long-read tail (merged windows longer than lmax; long_merge) ----
  // [cap][NM][8] u64 from position lmax on: entry (i, m) holds 0: mate m's
  // reads of length lmax + 1 + i, 1: its quality sum at position lmax + i,
  // 2..6: A C G T N there (7: unused)
  uint64_t *tail;
  int tail_lo, tail_hi;   // positions [lo, hi) go to the tail, lengths in (lo, hi]
  uint32_t *maxlen;       // atomicMax: the longest merged window longer than lmax
  uint32_t *need;         // atomicMax: a window longer than tail_hi (the tail was short)
  uint32_t *ovf;          // set to 1 when this call has such a window (nullptr: host path)
};

// ---------------------------------------------------------------------------
// quality bytes
// ---------------------------------------------------------------------------
// A quality byte is the reference's `char`, signed on x86-64 gcc: the merge
// adds fq_read->quality[j] into an int (src/stats_fastq.c:353-355), the CGR
// accumulator likewise (old/chaos_game.c:253-259); DESIGN.md §2.3, quirk Q13.
// The kernels work on BIASED bytes b ^ 0x80 = (signed char)b + 128, which
// v_sad_u8, the SWAR compares and the 16-bit pair counters take as unsigned:
// the host hands them phred + 128 as `phred` and biased thresholds, and the
// workgroup epilogues take the 128 per merged base back out (pos_fix).
constexpr uint32_t kQFlip = 0x80808080u;
constexpr int kQBias = 128;

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

// wave sum of per-lane u64 values (each < 2^58), in 16-bit slices
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return (uint64_t)wave_sum(lo & 0xFFFFu) + ((uint64_t)wave_sum(lo >> 16) << 16) +
         ((uint64_t)wave_sum(hi) << 32);
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

// inclusive prefix sum over the wave (row scans + row broadcasts)
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
  return v;
}

// lane i <- lane i+1 (wave_shl:1); lane 63 gets 0
__device__ __forceinline__ uint32_t next_lane(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return (uint64_t)(uint32_t)uni((int)(uint32_t)x) | ((uint64_t)(uint32_t)uni((int)(uint32_t)(x >> 32)) << 32);
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return (1ull << lane) - 1ull; }

// v[lane j] = val (j wave-uniform): a compare + select, no inline asm (the old
// v_writelane form needed M0, which an asm clobber list cannot reserve)
__device__ __forceinline__ uint32_t put_lane(uint32_t v, uint32_t val, int j) {
  return (int)(threadIdx.x & 63) == j ? val : v;
}

// ---------------------------------------------------------------------------
// units: the blocks of reads a wave takes in turn
// ---------------------------------------------------------------------------

// One unit: reads base + pos for the positions pos of `bits`, base = u *
// (reads per unit); direct units have contiguous bits 0..nr-1 (bits unused).
// u < 0: no unit (the pipeline's dummy).  32-bit: batches hold < 2^31 reads.
struct Unit {
  int u;
  int nr;
  uint64_t bits;
};

// Unit source of one wave: units u = gw, gw + nw, ... of BLOCK reads each.
// Follow-up (FOLLOW): the same sequence over the earlier stage's units,
// skipping those without deferred reads; each candidate's mask is one scalar
// load (lgkmcnt: it never waits behind the wave's vector loads in flight; a
// ballot over a vector-loaded window of masks cost the segmented kernel ~40
// VGPRs and its occupancy).
template <bool FOLLOW, int BLOCK>
struct UnitIter {
  int nw, nunits, num_reads, next_u;
  const uint64_t *bits1, *bits2;
  uint64_t held;   // positions a unit can hold (follow: the earlier stage's block)

  __device__ __forceinline__ void init(const EngineArgs &A, int gw, int nw_) {
    nw = nw_;
    num_reads = (int)A.num_reads;
    nunits = FOLLOW ? (int)A.nunits : (num_reads + BLOCK - 1) / BLOCK;
    next_u = gw;
    bits1 = A.unit_bits;
    bits2 = A.unit_and;
    held = FOLLOW && A.unit_reads < 64 ? (1ull << A.unit_reads) - 1ull : ~0ull;
  }
  __device__ __forceinline__ Unit next() {
    for (;;) {
      const int u = next_u;
      if (u >= nunits) return Unit{-1, 0, 0};
      next_u = u + nw;
      if (!FOLLOW) return Unit{u, min(BLOCK, num_reads - u * BLOCK), 0ull};
      uint64_t v = bits1[u] & held;
      if (bits2) v &= bits2[u];
      if (v) return Unit{u, __builtin_popcountll(v), v};
    }
  }
};

// read id of lane j (< U.nr) of unit U (first read `base`); scratch: 64 u32 of
// per-wave LDS
template <bool FOLLOW>
__device__ __forceinline__ int unit_read(const Unit &U, int base, uint32_t *scratch) {
  const int lane = threadIdx.x & 63;
  if (!FOLLOW) return base + lane;
  // compaction: the lane of each set bit writes its position to slot rank
  if ((U.bits >> lane) & 1ull) scratch[__builtin_popcountll(U.bits & lanes_below(lane))] = (uint32_t)lane;
  __builtin_amdgcn_wave_barrier();
  const int pos = lane < U.nr ? (int)scratch[lane] : 0;
  __builtin_amdgcn_wave_barrier();
  return base + pos;
}

// a follow-up stage with nothing deferred to it exits at once (grid-uniform)
__device__ __forceinline__ bool follow_up_idle(const EngineArgs &A) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (A.pending_clear) *A.pending_clear = 0u;
    if (A.pending_clear2) *A.pending_clear2 = 0u;
    if (A.report)   // ONE 8-byte store over PCIe into pinned host memory: the host never
                    // sees a count next to another call's sequence number
      *reinterpret_cast<volatile uint64_t *>(A.report) = (uint64_t)*A.pending | (uint64_t)A.report_seq << 32;
  }
  return A.unit_bits != nullptr && uni((int)*A.pending) == 0;
}

// ---------------------------------------------------------------------------
// base fields
// ---------------------------------------------------------------------------

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

// wave-uniform read descriptor, unpacked from the unit prologue's lane j
struct ReadRef {
  uint32_t os, oq;   // aligned byte offsets (dword) into the SRDs
  int als, alq;      // byte alignment of the read start
  int n;             // length (full 32 bits)
};

// loads: lane l, chunk c reads the dword at os + 4*(63c + l) + c0; reads past
// the data end return 0, past the read end they are garbage we mask.  The
// whole offset goes in the VGPR operand: the SRD range check covers the vector
// offset only (not soffset), and it is what keeps every load inside
// [base, base + data end) -- the base of a batch with absolute offsets lies
// before its allocation, so an unchecked offset below data_indices[0] would
// read unmapped memory.
template <int NCH>
__device__ __forceinline__ void issue(const MateBuf &b, const ReadRef &r, uint32_t lane4,
                                      Pending<NCH> &p, int c0 = 0) {
  // readfirstlane: the offsets are uniform, say so (else hipcc may waterfall)
  const uint32_t os = (uint32_t)uni((int)r.os), oq = (uint32_t)uni((int)r.oq);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    p.s[c] = __builtin_amdgcn_raw_buffer_load_b32(b.rs, os + lane4 + kChunk * c + c0, 0, 0);
    p.q[c] = __builtin_amdgcn_raw_buffer_load_b32(b.rq, oq + lane4 + kChunk * c + c0, 0, 0);
  }
}

// window-aligned words: lane bytes = positions p0..p0+3 (quality biased)
template <int NCH>
__device__ __forceinline__ void finish(const ReadRef &r, const Pending<NCH> &p,
                                       uint32_t (&sw)[NCH], uint32_t (&qw)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    sw[c] = __builtin_amdgcn_alignbyte(next_lane(p.s[c]), p.s[c], (uint32_t)r.als);
    qw[c] = __builtin_amdgcn_alignbyte(next_lane(p.q[c]), p.q[c], (uint32_t)r.alq) ^ kQFlip;   // biased
  }
}

// the read's window starting `ts` bases in
__device__ __forceinline__ ReadRef shift_ref(const ReadRef &rr, int ts) {
  ReadRef r2 = rr;
  const uint32_t xs = rr.os + (uint32_t)(rr.als + ts), xq = rr.oq + (uint32_t)(rr.alq + ts);
  r2.os = xs & ~3u;
  r2.oq = xq & ~3u;
  r2.als = (int)(xs & 3u);
  r2.alq = (int)(xq & 3u);
  r2.n = rr.n - ts;
  return r2;
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
  uint32_t r1;   // biased quality sum | GC << 19 (reads <= NCH chunks: 1260 x 255 < 2^19)
  int wn, ts, te;
  bool pass;
};

// mean-quality window test min*k <= S - phred*k <= max*k in 64-bit arithmetic
__device__ __forceinline__ bool mean_in(int64_t sraw, int64_t k, int phred, int lo, int hi) {
  const int64_t s = sraw - (int64_t)phred * k;
  return (int64_t)lo * k <= s && s <= (int64_t)hi * k;
}

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
    p1 += (uint32_t)__builtin_popcount(zero_bytes((sw[c] | 0x04040404u) ^ 0x47474747u) & m80) << 19;
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
    const int sq = (int)(o.r1 & 0x7FFFFu) - A.phred * wn;
    pass = (wn >= A.min_len) & (wn <= A.max_len) & (A.min_q * wn <= sq) & (sq <= A.max_q * wn);
    if (GEN) {
      if (A.flags & (F_NEED_N | F_NEED_OOR)) {
        const uint32_t r2 = wave_sum(p2);
        if ((A.flags & F_NEED_N) && (int)(r2 & 0xFFFFu) > C.max_n) pass = false;
        if ((A.flags & F_NEED_OOR) && (int)(r2 >> 16) > C.max_oor) pass = false;
      }
      if (A.flags & F_NEED_LR) {
        if (kl > 0 && !mean_in(wave_sum(pl), kl, A.phred, C.min_left, C.max_left)) pass = false;
        if (kr > 0 && !mean_in(wave_sum(pr), kr, A.phred, C.min_right, C.max_right)) pass = false;
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

// ---- reads longer than the pipeline's NCH chunks: one chunk at a time -------

// one 252-position chunk [c0, c0 + 252) of read r (words of positions c0 + 4 lane ..)
__device__ __forceinline__ void chunk_words(const MateBuf &b, const ReadRef &r, uint32_t lane4, int c0,
                                            uint32_t &sw, uint32_t &qw) {
  Pending<1> p;
  issue<1>(b, r, lane4, p, c0);
  sw = __builtin_amdgcn_alignbyte(next_lane(p.s[0]), p.s[0], (uint32_t)r.als);
  qw = __builtin_amdgcn_alignbyte(next_lane(p.q[0]), p.q[0], (uint32_t)r.alq) ^ kQFlip;   // biased
}

// edit (A6) trims of a read of any length (same rule as trim_read)
__device__ __forceinline__ void long_trim(const ColdParams &C, const MateBuf &b, const ReadRef &r,
                                       uint32_t lane4, int lane_p0, int &ts, int &te) {
  const int n = r.n;
  ts = 0;
  te = 0;
  uint32_t sw, qw;
  if (C.e_left_len > 0) {
    const int lim = min(C.e_left_len, n);
    ts = lim;
    for (int c0 = 0; c0 < lim; c0 += kChunk) {
      chunk_words(b, r, lane4, c0, sw, qw);
      const int p0 = c0 + lane_p0;
      const uint32_t ok = in_range(qw, C.el_lo4, C.el_hi4, C.el_lo_none, C.el_hi_none, C.el_none_in) &
                          byte_mask(lim - p0);
      const int first = wave_min(ok ? p0 + (__builtin_ctz(ok) >> 3) : 0x7FFFFFFF);
      if (first < lim) {
        ts = first;
        break;
      }
    }
  }
  if (C.e_right_len > 0) {
    const int lim = min(C.e_right_len, n - ts);
    const int lo = n - lim;
    te = lim;
    for (int c0 = ((n - 1) / kChunk) * kChunk; lim > 0 && c0 >= 0 && c0 + kChunk > lo; c0 -= kChunk) {
      chunk_words(b, r, lane4, c0, sw, qw);
      const int p0 = c0 + lane_p0;
      const uint32_t ok = in_range(qw, C.er_lo4, C.er_hi4, C.er_lo_none, C.er_hi_none, C.er_none_in) &
                          byte_mask(n - p0) & ~byte_mask(lo - p0);
      const int last = wave_max(ok ? p0 + ((31 - __builtin_clz(ok)) >> 3) : -1);
      if (last >= 0) {
        te = n - 1 - last;
        break;
      }
    }
  }
}

// filter (A5) of the window r (its n = the window length) of any length
__device__ __forceinline__ bool long_eval(const EngineArgs &A, const ColdParams &C, const MateBuf &b,
                                       const ReadRef &r, uint32_t lane4, int lane_p0) {
  if (!(A.flags & F_FILTER)) return true;
  const int wn = r.n;
  if (wn < A.min_len || wn > A.max_len) return false;
  const bool lr = A.flags & F_NEED_LR;
  const int kl = lr ? min(C.left_len, wn) : 0, kr = lr ? min(C.right_len, wn) : 0;
  uint64_t sq = 0, sl = 0, sr = 0, nn = 0, oo = 0;
  for (int c0 = 0; c0 < wn; c0 += kChunk) {
    uint32_t sw, qw;
    chunk_words(b, r, lane4, c0, sw, qw);
    const int p0 = c0 + lane_p0;
    const uint32_t m = byte_mask(wn - p0), m80 = m & 0x80808080u, q = qw & m;
    sq += __builtin_amdgcn_sad_u8(q, 0u, 0u);
    if (A.flags & F_NEED_N) nn += __builtin_popcount(zero_bytes(sw ^ 0x4E4E4E4Eu) & m80);
    if (A.flags & F_NEED_OOR) {
      uint32_t bad;
      if (A.flags & F_OOR_ALL) {
        bad = 0x80808080u;
      } else {
        bad = 0;
        if (!(A.flags & F_OOR_LO_NONE)) bad |= ~ge_bytes(qw, C.oor_lo4) & 0x80808080u;
        if (!(A.flags & F_OOR_HI_NONE)) bad |= ge_bytes(qw, C.oor_hi4);
      }
      oo += __builtin_popcount(bad & m80);
    }
    if (kl > 0) sl += __builtin_amdgcn_sad_u8(q & byte_mask(kl - p0), 0u, 0u);
    if (kr > 0) sr += __builtin_amdgcn_sad_u8(q & ~byte_mask(wn - kr - p0), 0u, 0u);
  }
  bool pass = mean_in((int64_t)wave_sum64(sq), wn, A.phred, A.min_q, A.max_q);
  if ((A.flags & F_NEED_N) && (int64_t)wave_sum64(nn) > C.max_n) pass = false;
  if ((A.flags & F_NEED_OOR) && (int64_t)wave_sum64(oo) > C.max_oor) pass = false;
  if (kl > 0 && !mean_in((int64_t)wave_sum64(sl), kl, A.phred, C.min_left, C.max_left)) pass = false;
  if (kr > 0 && !mean_in((int64_t)wave_sum64(sr), kr, A.phred, C.min_right, C.max_right)) pass = false;
  return pass;
}

// ---- a merged window longer than lmax ----------------------------------------
// The reference merges every position of every read (src/stats_fastq.c:338-382:
// khash keyed by j < read_length, no cap).  One wave, chunk by chunk:
// positions < lmax into the workgroup's LDS partials pa ([6][lmax]; the quality
// added SIGNED and unbiased -- pos_fix removes the bias only for the length
// histogram's reads -- and the A/C/G/T/N rows, :353-372), the mean-quality and
// GC bins into the LDS histogram hm (key = round(S / n), :316-324; 100 (G + C) /
// n, :326-334), the acc_quality term floor(65536 S / n) into fx (lane 0), and
// positions >= lmax plus the length into the tail with global u64 atomics
// (positions [tail_lo, tail_hi), lengths in (tail_lo, tail_hi]).  A window
// longer than tail_hi (a device batch beyond the tail reserved so far) flags
// the call; hpgq_sync grows the tail and merges the rest with TAIL_ONLY.
template <int NM>
__device__ void long_merge(const EngineArgs &A, const MateBuf &b, const ReadRef &rw, uint32_t lane4,
                           int lane_p0, int m, uint32_t *pa, uint32_t *hm, uint64_t &fx) {
  const int n = rw.n, lmax = A.lmax, lo = A.tail_lo, hi = A.tail_hi;
  const bool tail_only = A.flags & F_TAIL_ONLY;
  const int lane = threadIdx.x & 63;
  uint64_t sq = 0, gc = 0;
  const int cend = tail_only ? min(n, hi) : n;
  for (int c0 = tail_only ? (lo / kChunk) * kChunk : 0; c0 < cend; c0 += kChunk) {
    uint32_t sw, qw;
    chunk_words(b, rw, lane4, c0, sw, qw);
    const int p0 = c0 + lane_p0;
    const uint32_t mk = byte_mask(n - p0);
    sq += __builtin_amdgcn_sad_u8(qw & mk, 0u, 0u);
    gc += (uint32_t)__builtin_popcount(zero_bytes((sw | 0x04040404u) ^ 0x47474747u) & mk & 0x80808080u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = p0 + i;
      if (p >= n) break;
      const uint32_t sb = (sw >> (8 * i)) & 0xFFu;
      const int q = (int)((qw >> (8 * i)) & 0xFFu) - kQBias;   // the signed char (Q13)
      const int bi = sb == 'A' ? 0 : sb == 'C' ? 1 : sb == 'G' ? 2 : sb == 'T' ? 3 : sb == 'N' ? 4 : -1;
      if (p < lmax) {
        if (!tail_only) {
          atomicAdd(&pa[p], (uint32_t)q);
          if (bi >= 0) atomicAdd(&pa[(1 + bi) * lmax + p], 1u);
        }
      } else if (p >= lo && p < hi) {
        unsigned long long *t =
            reinterpret_cast<unsigned long long *>(A.tail + ((size_t)(p - lmax) * NM + m) * 8);
        atomicAdd(t + 1, (unsigned long long)(long long)q);
        if (bi >= 0) atomicAdd(t + 2 + bi, 1ull);
      }
    }
  }
  if (!tail_only) {
    const int64_t S = (int64_t)wave_sum64(sq) - (int64_t)kQBias * n;   // the signed quality sum
    const uint64_t g = wave_sum64(gc);
    if (lane == 0) {
      const int64_t n2 = 2 * (int64_t)n;
      const int64_t key = S >= 0 ? (2 * S + n) / n2 : -((-2 * S + n) / n2);   // C round()
      atomicAdd(&hm[lmax + 1 + (uint32_t)(key & 255)], 1u);
      atomicAdd(&hm[lmax + 1 + HPGQ_MEANQ_BINS + (uint32_t)((100 * g) / (uint64_t)n)], 1u);
      const int64_t t = S * 65536;
      fx += (uint64_t)(t / n - ((t % n != 0 && t < 0) ? 1 : 0));   // floor
      atomicMax(A.maxlen, (uint32_t)n);
    }
  }
  if (lane == 0) {
    if (lo < n && n <= hi) {
      atomicAdd(reinterpret_cast<unsigned long long *>(A.tail + ((size_t)(n - lmax - 1) * NM + m) * 8), 1ull);
    } else if (n > hi) {
      atomicMax(A.need, (uint32_t)n);
      if (A.ovf) *A.ovf = 1u;
    }
  }
}

// one merged read's quality-histogram bin and acc_quality term from its biased
// quality sum sb = S + 128 n (n > 0, n <= 1024, sb < 2^19): key = round(S / n) as C's
// round() (halves away from zero; src/stats_fastq.c:317), bin = key & 255
// (negative keys need quality bytes >= 128: bins 128..255); fx = floor(65536
// S / n) in two's complement (the acc_quality term, HPGQ_S_ACC_MEANQ_FX16)
__device__ __forceinline__ void meanq_terms(uint32_t sb, uint32_t n, uint32_t &bin, uint64_t &fx) {
  const uint32_t off = (uint32_t)kQBias * n;
  if (__builtin_expect(sb >= off, 1)) {
    bin = (2 * sb + n) / (2 * n) - (uint32_t)kQBias;
  } else {
    const uint32_t t = off - sb;
    bin = (256u - (2 * t + n) / (2 * n)) & 255u;
  }
  const uint32_t q = sb / n, rem = sb - q * n;
  fx = ((uint64_t)q << 16) + (((uint32_t)rem << 16) / n) - ((uint64_t)kQBias << 16);
}

// Per-position fix-ups of a workgroup's partial set in LDS, from the read
// count c[p] = sum_{L > p} hist_len[L] of its merged reads (a chunked suffix
// scan in O(lmax): thread t owns positions [4t, 4t + 4), lmax <= 1024 = 4 x
// kWG): the quality row loses the bias (128 c[p]); DERIVE_N: row 5 holds the
// "other" counts and becomes N = c[p] - A - C - G - T - other.  wtot: kWaves
// words of free LDS.  Ends with a barrier.
template <bool DERIVE_N>
__device__ __forceinline__ void pos_fix(uint32_t *pa, const uint32_t *h, int lmax, int tid, uint32_t *wtot) {
  static_assert(4 * kWG >= HPGQ_LMAX_LIMIT, "one 4-position chunk per thread");
  const int p0 = 4 * tid;
  uint32_t hv[4], s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int L = p0 + i + 1;
    hv[i] = L <= lmax ? h[L] : 0u;
    s += hv[i];
  }
  const uint32_t incl = wave_scan(s);   // reads of lengths (.., p0 + 4] within the wave
  if ((tid & 63) == 63) wtot[tid >> 6] = incl;
  __syncthreads();
  uint32_t total = 0, before = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const uint32_t t = wtot[w];
    total += t;
    if (w < (tid >> 6)) before += t;
  }
  uint32_t c = total - before - incl;   // reads longer than p0 + 4
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    const int p = p0 + i;
    c += hv[i];   // c[p] = h[p + 1] + c[p + 1]
    if (p < lmax) {
      pa[p] -= (uint32_t)kQBias * c;
      if (DERIVE_N)
        pa[5 * lmax + p] = c - pa[lmax + p] - pa[2 * lmax + p] - pa[3 * lmax + p] - pa[4 * lmax + p] -
                           pa[5 * lmax + p];
    }
  }
  __syncthreads();
}

// add one workgroup's partial counter set into the global counters: one
// no-return u64 atomic per nonzero entry (set layout: include/hpgq.h); the
// quality row (pos[0, lmax)) is a signed sum: sign-extended
__device__ __forceinline__ void add_partials(uint64_t *dst, const unsigned long long *sc,
                                             const uint32_t *hist, int hlen, const uint32_t *pos,
                                             int lmax, int tid, int nthreads) {
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += nthreads)
    if (sc[i]) atomicAdd(reinterpret_cast<unsigned long long *>(dst + i), sc[i]);
  for (int i = tid; i < hlen; i += nthreads)
    if (hist[i]) atomicAdd(reinterpret_cast<unsigned long long *>(dst + HPGQ_NUM_SCALARS + i),
                           (unsigned long long)hist[i]);
  uint64_t *dp = dst + HPGQ_NUM_SCALARS + hlen;
  for (int i = tid; i < 6 * lmax; i += nthreads)
    if (pos[i])
      atomicAdd(reinterpret_cast<unsigned long long *>(dp + i),
                i < lmax ? (unsigned long long)(long long)(int32_t)pos[i] : (unsigned long long)pos[i]);
}

// the same from an LDS set sized for lp <= lmax positions (the segmented
// kernels: their reads are at most a geometry's kPos long): hist [lp + 1 +
// MEANQ + GC], pos [6][lp], added at the global layout's lmax offsets
__device__ __forceinline__ void add_partials_lp(uint64_t *dst, const unsigned long long *sc,
                                                const uint32_t *hist, const uint32_t *pos, int lmax, int lp,
                                                int tid, int nthreads) {
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += nthreads)
    if (sc[i]) atomicAdd(reinterpret_cast<unsigned long long *>(dst + i), sc[i]);
  const int hl = lp + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  for (int i = tid; i < hl; i += nthreads)
    if (hist[i]) {
      const int gi = i <= lp ? i : i + (lmax - lp);   // mean-Q / GC bins follow the lmax + 1 length bins
      atomicAdd(reinterpret_cast<unsigned long long *>(dst + HPGQ_NUM_SCALARS + gi), (unsigned long long)hist[i]);
    }
  uint64_t *dp = dst + HPGQ_NUM_SCALARS + lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  for (int i = tid; i < 6 * lp; i += nthreads)
    if (pos[i]) {
      const int r = i / lp, j = i - r * lp;
      atomicAdd(reinterpret_cast<unsigned long long *>(dp + r * lmax + j),
                r == 0 ? (unsigned long long)(long long)(int32_t)pos[i] : (unsigned long long)pos[i]);
    }
}

template <int NM, int NCH, bool GEN, bool FOLLOW>
__global__ void __launch_bounds__(kWG) engine_kernel(EngineArgs A) {
  if (FOLLOW && follow_up_idle(A)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int lmax = A.lmax;
  const int hlen = lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  constexpr int kCap = kChunk * NCH;   // positions the pipelined loads hold
  // lane l < 63 owns positions 4l.. of every chunk; lane 63 none
  const int lane_p0 = lane < 63 ? 4 * lane : 0x40000000;
  const uint32_t lane4 = 4u * (uint32_t)lane;
  const int ublock = FOLLOW ? A.unit_reads : 64;   // reads per unit

  // LDS: pos_acc [NM][6][lmax] u32 | hist [NM][hlen] u32 | sc [NM][8] u64 | cold |
  //      per wave: compaction scratch [64] u32
  uint32_t *pos_acc = reinterpret_cast<uint32_t *>(lds);
  uint32_t *hist = pos_acc + NM * 6 * lmax;
  const int hist_words = (NM * hlen + 1) & ~1;
  unsigned long long *sc = reinterpret_cast<unsigned long long *>(hist + hist_words);
  ColdParams *cold = reinterpret_cast<ColdParams *>(sc + NM * HPGQ_NUM_SCALARS);
  uint32_t *scratch = reinterpret_cast<uint32_t *>(cold + 1) + wave * 64;
  for (int i = tid; i < NM * 6 * lmax + hist_words; i += kWG) pos_acc[i] = 0;
  for (int i = tid; i < NM * HPGQ_NUM_SCALARS; i += kWG) sc[i] = 0;
  if (tid < (int)(sizeof(ColdParams) / 4))
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
  uint32_t cnt[NM][6];   // input, passed, failed, edited, stats, long (wave-uniform)
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    fx16[m] = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) cnt[m][k] = 0;
  }

  // reads per pipeline group (two groups of registers in flight)
  constexpr int kU = ((NM == 1 ? 8 : 4) / NCH) > 0 ? ((NM == 1 ? 8 : 4) / NCH) : 1;
  UnitIter<FOLLOW, 64> it;
  it.init(A, (int)blockIdx.x * kWaves + wave, (int)gridDim.x * kWaves);

  // unit prologue: lane j describes read j of unit U for mate m
  //   off_s/off_q: aligned byte offsets; al: als | alq << 2; len: length; rid: read id
  auto load_block = [&](const Unit &U, uint32_t (&off_s)[NM], uint32_t (&off_q)[NM],
                        uint32_t (&al)[NM], int32_t (&len)[NM], int &rid) __attribute__((always_inline)) {
    rid = U.nr > 0 ? unit_read<FOLLOW>(U, U.u * ublock, scratch) : 0;
    const bool on = lane < U.nr;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int a = on ? A.idx[m][rid] : 0, e = on ? A.idx[m][rid + 1] : 0;
      // absent reads (the pipeline's dummy unit): offsets past the SRD range
      const uint32_t xs = on ? (uint32_t)(mb[m].bs + a) : 0x80000000u;
      const uint32_t xq = on ? (uint32_t)(mb[m].bq + a) : 0x80000000u;
      off_s[m] = xs & ~3u;
      off_q[m] = xq & ~3u;
      al[m] = (xs & 3u) | ((xq & 3u) << 2);
      len[m] = e - a;
    }
  };
  auto ref_of = [&](const uint32_t (&off_s)[NM], const uint32_t (&off_q)[NM], const uint32_t (&al)[NM],
                    const int32_t (&len)[NM], int m, int j) __attribute__((always_inline)) {
    ReadRef r;
    r.os = __builtin_amdgcn_readlane(off_s[m], j);
    r.oq = __builtin_amdgcn_readlane(off_q[m], j);
    const uint32_t a = __builtin_amdgcn_readlane(al[m], j);
    r.n = __builtin_amdgcn_readlane(len[m], j);
    r.als = (int)(a & 3u);
    r.alq = (int)((a >> 2) & 3u);
    return r;
  };

  Pending<NCH> grp[2][kU][NM];
  auto load_group = [&](const uint32_t (&os)[NM], const uint32_t (&oq)[NM], const uint32_t (&al)[NM],
                        const int32_t (&len)[NM], int nr, int g, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int j = max(min(g * kU + u, nr - 1), 0);   // past the unit end: reload the last read
#pragma unroll
      for (int m = 0; m < NM; ++m) issue<NCH>(mb[m], ref_of(os, oq, al, len, m, j), lane4, grp[slot][u][m]);
    }
  };

  uint32_t os[NM], oq[NM], al[NM], osn[NM], oqn[NM], aln[NM];
  int32_t ln[NM], lnn[NM];
  int rid = 0, ridn = 0;
  Unit cur = it.next();
  if (cur.u >= 0) {
    load_block(cur, os, oq, al, ln, rid);
    load_group(os, oq, al, ln, cur.nr, 0, 0);
  }
  while (cur.u >= 0) {
    const int nr = cur.nr;
    const Unit nxt = it.next();
    load_block(nxt, osn, oqn, aln, lnn, ridn);
    // per-read results, lane j <-> read j of the unit
    uint32_t res_r1[NM], res_info[NM], res_trim[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) res_r1[m] = res_info[m] = res_trim[m] = 0;

    auto process_group = [&](int g, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int j = g * kU + u;
        if (j >= nr) break;
        ReadOut out[NM];
        uint32_t sw[NM][NCH], qw[NM][NCH], mk[NM][NCH];
        bool lng[NM];
        ReadRef rrs[NM];
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const ReadRef rr = ref_of(os, oq, al, ln, m, j);
          rrs[m] = rr;
          finish<NCH>(rr, grp[slot][u][m], sw[m], qw[m]);
          int ts = 0, te = 0;
          if (GEN && (A.flags & F_EDIT)) {
            if (rr.n <= kCap) trim_read<NCH>(*cold, qw[m], rr.n, lane_p0, ts, te);
            else long_trim(*cold, mb[m], rr, lane4, lane_p0, ts, te);
            if (ts > 0 && rr.n - ts - te <= kCap) {   // window no longer starts at the read start: realign
              const ReadRef r2 = shift_ref(rr, ts);
              Pending<NCH> p2;
              issue<NCH>(mb[m], r2, lane4, p2);
              finish<NCH>(r2, p2, sw[m], qw[m]);
            }
          }
          const int wn = rr.n - ts - te;
          if (wn <= kCap) {
#pragma unroll
            for (int c = 0; c < NCH; ++c) mk[m][c] = byte_mask(wn - lane_p0 - kChunk * c);
            out[m] = evaluate<GEN, NCH>(A, *cold, sw[m], qw[m], mk[m], wn, lane_p0);
          } else {   // longer than the pipelined chunks (and than lmax): filter by chunk loop
            ReadRef rw = shift_ref(rr, ts);
            rw.n = wn;
            out[m].r1 = 0;
            out[m].wn = wn;
            out[m].pass = long_eval(A, *cold, mb[m], rw, lane4, lane_p0);
          }
          out[m].ts = ts;
          out[m].te = te;
          lng[m] = wn > lmax;
        }
        bool pass = out[0].pass;
        if (NM == 2) pass = pass && out[NM - 1].pass;
        const bool tail_only = A.flags & F_TAIL_ONLY;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          if ((A.flags & F_STATS) && pass && !lng[m] && !tail_only) acc[m].add(sw[m], qw[m], mk[m]);
          if ((A.flags & F_STATS) && pass && lng[m]) {   // longer than lmax: merged by its own chunk loop
            ReadRef rw = shift_ref(rrs[m], out[m].ts);
            rw.n = out[m].wn;
            long_merge<NM>(A, mb[m], rw, lane4, lane_p0, m, pos_acc + m * 6 * lmax, hist + m * hlen, fx16[m]);
          }
          // wn only feeds the histograms of reads <= lmax, so 16 bits suffice
          const uint32_t info = (uint32_t)min(out[m].wn, 0xFFFF) | ((uint32_t)pass << 16) |
                                ((uint32_t)lng[m] << 17) | ((uint32_t)(out[m].ts + out[m].te > 0) << 18);
          res_r1[m] = put_lane(res_r1[m], out[m].r1, j);
          res_info[m] = put_lane(res_info[m], info, j);
          if (GEN)
            res_trim[m] = put_lane(res_trim[m], (uint32_t)out[m].ts | ((uint32_t)out[m].te << 16), j);
        }
        if ((A.flags & F_STATS) && pass && ++since_flush == kFlushEvery) {
#pragma unroll
          for (int m = 0; m < NM; ++m) acc[m].flush(pos_acc + m * 6 * lmax, lmax, lane_p0);
          since_flush = 0;
        }
      }
    };

    // group g of this unit sits in slot g & 1; the group after the last one
    // is the next unit's group 0 (full units have an even group count, so it
    // lands in slot 0, where the next unit expects it)
    const int ngroups = (nr + kU - 1) / kU;
    for (int g = 0; g < ngroups; g += 2) {
      if (g + 1 < ngroups) load_group(os, oq, al, ln, nr, g + 1, 1);
      else load_group(osn, oqn, aln, lnn, nxt.nr, 0, 1);
      process_group(g, 0);
      if (g + 1 < ngroups) {
        if (g + 2 < ngroups) load_group(os, oq, al, ln, nr, g + 2, 0);
        else load_group(osn, oqn, aln, lnn, nxt.nr, 0, 0);
        process_group(g + 1, 1);
      }
    }

    // ---- unit epilogue, vectorised over lanes (lane j = read j) -------------
    // (the tail's second pass counts nothing here: the first pass did)
    const bool valid = lane < nr && !(A.flags & F_TAIL_ONLY);
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const uint32_t info = res_info[m];
      const int wn = (int)(info & 0xFFFFu);
      const bool pass = valid && ((info >> 16) & 1u);
      const bool lg = valid && ((info >> 17) & 1u);
      const bool edited = valid && ((info >> 18) & 1u);
      if (valid) {
        if (m == 0 && A.mask) A.mask[rid] = (uint8_t)pass;
        if (A.trim) A.trim[(int64_t)m * A.num_reads + rid] = res_trim[m];
      }
      cnt[m][0] += (A.flags & F_TAIL_ONLY) ? 0u : (uint32_t)nr;
      cnt[m][1] += (uint32_t)__builtin_popcountll(__ballot(pass));
      cnt[m][2] += (uint32_t)__builtin_popcountll(__ballot(valid && !pass));
      cnt[m][3] += (uint32_t)__builtin_popcountll(__ballot(edited));
      if (A.flags & F_STATS) {
        cnt[m][4] += (uint32_t)__builtin_popcountll(__ballot(pass));
        cnt[m][5] += (uint32_t)__builtin_popcountll(__ballot(pass && lg));
        if (pass && !lg) {
          uint32_t *hm = hist + m * hlen;
          const uint32_t r1 = res_r1[m];
          const uint32_t s = r1 & 0x7FFFFu, gc = r1 >> 19, n = (uint32_t)wn;
          atomicAdd(&hm[n], 1u);
          if (n > 0) {
            uint32_t bin;
            uint64_t fx;
            meanq_terms(s, n, bin, fx);
            atomicAdd(&hm[lmax + 1 + bin], 1u);
            atomicAdd(&hm[lmax + 1 + HPGQ_MEANQ_BINS + (100 * gc) / n], 1u);
            fx16[m] += fx;
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      os[m] = osn[m];
      oq[m] = oqn[m];
      al[m] = aln[m];
      ln[m] = lnn[m];
    }
    rid = ridn;
    cur = nxt;
  }

  // ---- workgroup epilogue ---------------------------------------------------
  if (A.flags & F_TAIL_ONLY) return;   // (grid-uniform: nothing on chip to add)
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m].flush(pos_acc + m * 6 * lmax, lmax, lane_p0);
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const uint64_t tot = wave_sum64(fx16[m]);
    if (lane == 0) {
      unsigned long long *scm = sc + m * HPGQ_NUM_SCALARS;
      if (cnt[m][0]) atomicAdd(&scm[HPGQ_S_NUM_INPUT], (unsigned long long)cnt[m][0]);
      if (cnt[m][1]) atomicAdd(&scm[HPGQ_S_NUM_PASSED], (unsigned long long)cnt[m][1]);
      if (cnt[m][2]) atomicAdd(&scm[HPGQ_S_NUM_FAILED], (unsigned long long)cnt[m][2]);
      if (cnt[m][3]) atomicAdd(&scm[HPGQ_S_NUM_EDITED], (unsigned long long)cnt[m][3]);
      if (cnt[m][4]) atomicAdd(&scm[HPGQ_S_NUM_STATS], (unsigned long long)cnt[m][4]);
      if (cnt[m][5]) atomicAdd(&scm[HPGQ_S_LONG_READS], (unsigned long long)cnt[m][5]);
      if (tot) atomicAdd(&scm[HPGQ_S_ACC_MEANQ_FX16], (unsigned long long)tot);
    }
  }
  __syncthreads();
  // (the compaction scratch is free now: pos_fix's wave totals)
  uint32_t *wtot = reinterpret_cast<uint32_t *>(cold + 1);
  for (int m = 0; m < NM; ++m) pos_fix<false>(pos_acc + m * 6 * lmax, hist + m * hlen, lmax, tid, wtot);
  for (int m = 0; m < NM; ++m)
    add_partials(A.counters + (size_t)m * A.clen, sc + m * HPGQ_NUM_SCALARS, hist + m * hlen, hlen,
                 pos_acc + m * 6 * lmax, lmax, tid, kWG);
}

}  // namespace hpgq
