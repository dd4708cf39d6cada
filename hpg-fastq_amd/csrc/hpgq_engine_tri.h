// hpgq_engine_tri.h — the FAST segmented stats/filter/edit kernel: several
// reads per wave step.
//
// Same contract and outputs as engine_kernel (hpgq_engine_kernel.h) for the
// reads whose length fits the geometry; longer reads are DEFERRED to the next
// stage of the chain (unit masks + a count, see hpgq_engine_kernel.h), so the
// kernel can run first on any batch.  The per-read fixed cost (the DPP scan,
// the pass/fail decision, bookkeeping) is shared by the reads of a step.  The
// kernel is close to VALU-issue bound, so everything below counts VALU
// instructions.
//
// Geometries (Geo<G>): a wave step holds kSegs reads, each owning a segment of
// kSegW lanes; a lane of a segment owns 4*NW consecutive positions.
//   tri  (G 0): 3 x 21 lanes x  8 B, reads <= 160, 54-read blocks
//   hex  (G 1): 6 x 10 lanes x 16 B, reads <= 156, 48-read blocks (1 KB per
//               wave-load: ~10 % more streaming rate than tri,
//               tools/ubench/stream_rates.hip)
//   wide (G 2): 4 x 16 lanes x 16 B, reads <= 252, 60-read blocks (250 bp
//               reads fill 98 % of the lanes)
//   * the unit prologue writes one 16-byte record per read (dword-aligned seq
//     and qual offsets, length | alignments) into a per-wave LDS table; each
//     lane fetches its segment's record with ONE ds_read_b128, issues ONE
//     buffer load per buffer and realigns with DPP wave_shl:1 + v_alignbyte
//     (the last lane of a segment borrows from the next segment, which only
//     reaches positions >= kPos).  Deferred and absent reads get offsets past
//     the SRD range, so their loads cost no memory traffic.
//   * base classification: code = byte & 7 (one-to-one on A,C,G,T,N; masked
//     bytes -> 0), then three v_perm_b32 LUTs: the expected byte (exact-match
//     check; lowercase / IUPAC / other bytes take a rare path and count as
//     "other"), C|G<<4 and A|T<<4 nibble one-hots.  G+C per read = popcount of
//     the C|G word.  N is not counted: the workgroup epilogue derives it as
//     count - A - C - G - T - other, count from the length histogram.
//   * nibble counters (<= 15 steps) are widened into 8-bit per-base counters
//     (<= 255 steps) and those flushed to LDS u32 arrays (ds_add); quality
//     sums are 16-bit pairs of biased bytes (b ^ 0x80, hpgq_engine_kernel.h).
//   * per-read sums (biased quality | G+C << 18) use ONE inclusive DPP prefix scan
//     for the wave; the last lane of each segment stores its segment end to
//     LDS (no wait) and the block epilogue takes differences.  (Per wave at
//     most 64 x 16 x 255 < 2^18 quality units: the fields never carry.)
//   * every read is accumulated; the epilogue decides pass/fail for the block
//     vectorised over lanes and takes the failed reads back out.
// The stats layout, histogram rules and counter epilogue are those of
// engine_kernel, so all kernels of a chain add into one counter set.
#pragma once
#include "hpgq_engine_kernel.h"

namespace hpgq {

constexpr int kTriSlack = 8;    // readable bytes past the data end the loads may touch

// The unit epilogue reads each read's length and trim word back from the read
// table (LDS) instead of holding them in VGPRs across the unit's steps (4 per
// mate: current and next unit), which the paired-end edit kernel spilled
// (TABLEN below; the follow-up stages keep them in registers).  The exact
// mean-quality sum (u64 per lane and mate) accumulates in per-lane LDS slots
// (one no-return ds_add_u64 per unit) instead of a VGPR pair held across the
// loop: the paired-end edit kernel spilled exactly those pairs, a scratch
// load + store per unit and mate (~200 MB of scratch writes per 10 M pairs).
// (32 slots, lane & 31, since round 6: two lanes add into each, which frees
// the LDS the reciprocal table takes without costing the paired-end edit
// kernel its third workgroup per CU)
constexpr int kFxSlots = 32;
constexpr int kFxWords = 2 * kFxSlots;   // per wave and mate: kFxSlots u64

constexpr int GEO_TRI = 0, GEO_HEX = 1, GEO_WIDE = 2;
constexpr int X_NOOR = 1, X_LR = 2;   // extra filter scans (engine_tri_x_kernel)
constexpr int X_ST = 4;               // single-end edit, trims applied at the step (tri_body ST)
// ST: per wave, the step's raw seq and quality dwords of every lane (64 x 16 B
// each, + 32 B read past the last lane), read back from a per-lane byte offset
constexpr int kStWords = 2 * (64 * 4 + 8);

// kBlock reads (<= 64: lane j <-> read j in the epilogue) in steps of kSegs
// reads, kU steps per pipeline group, an even number of groups per block.
template <int G>
struct Geo;
template <>
struct Geo<GEO_TRI> {
  static constexpr int kNW = 2, kSegs = 3, kSegW = 21, kOwn = 20, kBlock = 54, kU = 3, kPos = 160;
};
template <>
struct Geo<GEO_HEX> {
  static constexpr int kNW = 4, kSegs = 6, kSegW = 10, kOwn = 10, kBlock = 48, kU = 2, kPos = 156;
};
template <>
struct Geo<GEO_WIDE> {   // 60-read blocks: read-table entry 63 stays empty (the padding steps' source)
  static constexpr int kNW = 4, kSegs = 4, kSegW = 16, kOwn = 16, kBlock = 60, kU = 2, kPos = 252;
};

template <int G>
constexpr uint64_t not_seg_first_mask() {   // lanes j with j % kSegs != 0
  uint64_t m = 0;
  for (int j = 0; j < 64; ++j)
    if (j % Geo<G>::kSegs) m |= 1ull << j;
  return m;
}
constexpr int kNibbleEvery = 15;   // 4-bit counters
constexpr int kByteEvery = 255;    // 8-bit counters

// code = byte & 7: pad(masked)->0 'A'->1 'C'->3 'T'->4 'N'->6 'G'->7
constexpr uint32_t kX7Lo = 0x43004101u;   // expected byte, codes 0..3 (0x01: no code-0 byte matches)
constexpr uint32_t kX7Hi = 0x474E0054u;   // codes 4..7
constexpr uint32_t kCGLo = 0x01000000u;   // C -> 0x01
constexpr uint32_t kCGHi = 0x10000000u;   // G -> 0x10
constexpr uint32_t kATLo = 0x00000100u;   // A -> 0x01
constexpr uint32_t kATHi = 0x00000010u;   // T -> 0x10

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int NW>
struct TriPending {
  uint32_t s[NW], q[NW];   // the lane's 4*NW bytes of seq / quality (raw dwords)
  uint32_t n;              // its read's length | als << 16 | alq << 20
};

__device__ __forceinline__ uint32_t next_lane0(uint32_t v) {   // lane i <- lane i+1, lane 63 <- 0
  return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true);
}

// 0xFF in every byte of d that is non-zero
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t d) {
  const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
  return (nz >> 7) * 0xFFu;
}

template <int NW>
struct TriAcc {
  uint32_t n4[NW][2];   // [word][C|G<<4, A|T<<4]: nibble per position
  uint32_t c8[NW][4];   // [word][A, C, G, T]: byte per position
  uint32_t q02[NW], q13[NW];   // quality 16-bit pairs (positions 0,2 / 1,3 of the word)
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      n4[w][0] = n4[w][1] = 0;
      c8[w][0] = c8[w][1] = c8[w][2] = c8[w][3] = 0;
      q02[w] = q13[w] = 0;
    }
  }
  // nibbles -> bytes (every <= 15 steps and before any subtraction)
  __device__ __forceinline__ void widen() {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      c8[w][1] += n4[w][0] & 0x0F0F0F0Fu;
      c8[w][2] += (n4[w][0] >> 4) & 0x0F0F0F0Fu;
      c8[w][0] += n4[w][1] & 0x0F0F0F0Fu;
      c8[w][3] += (n4[w][1] >> 4) & 0x0F0F0F0Fu;
      n4[w][0] = n4[w][1] = 0;
    }
  }
  // bytes -> LDS (pos_acc [6][lmax]: qsum, A, C, G, T, N/other); nibbles empty
  __device__ __forceinline__ void flush(uint32_t *pos_acc, int lmax, int p0) {
    // rare (every <= 255 steps): keep its 40 LDS addresses out of the hot
    // loop's registers (hipcc would hoist them as loop invariants and spill).
    // Only the indices pass through the asm: a pointer that does comes out of
    // it generic, so these adds became FLAT atomics (round 5), and a FLAT
    // operation that may be in flight makes the wait-count pass wait for
    // every load at each use of a streamed group, all through the unit loop.
    // (C2's share of that coarse waiting is now an explicit wait, tri_body)
    asm volatile("" : "+v"(p0), "+s"(lmax));
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t qv[4] = {q02[w] & 0xFFFFu, q13[w] & 0xFFFFu, q02[w] >> 16, q13[w] >> 16};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = p0 + 4 * w + i;
        if (pos < lmax) {
          atomicAdd(&pos_acc[pos], qv[i]);
#pragma unroll
          for (int b = 0; b < 4; ++b)
            atomicAdd(&pos_acc[(1 + b) * lmax + pos], (c8[w][b] >> (8 * i)) & 0xFFu);
        }
      }
      c8[w][0] = c8[w][1] = c8[w][2] = c8[w][3] = 0;
      q02[w] = q13[w] = 0;
    }
  }
};

// codes of a masked word; marks bytes that are not exactly A/C/G/T/N
__device__ __forceinline__ uint32_t tri_codes(uint32_t s, uint32_t m, uint32_t &bad) {
  const uint32_t codes = s & m & 0x07070707u;
  const uint32_t ex = __builtin_amdgcn_perm(kX7Hi, kX7Lo, codes);
  bad |= (s ^ ex) & m;
  return codes;
}

// rare path: bytes that are not exactly A/C/G/T/N get code 0 (counted nowhere)
// and one "other" count per position (sign: +1 add, -1 subtract)
__device__ __forceinline__ uint32_t tri_fix(uint32_t s, uint32_t m, uint32_t codes, uint32_t *other,
                                            int lmax, int pos0, uint32_t sign) {
  // rare path: no hoisted addresses (see TriAcc::flush)
  asm volatile("" : "+v"(pos0), "+s"(lmax));
  const uint32_t ex = __builtin_amdgcn_perm(kX7Hi, kX7Lo, codes);
  const uint32_t ff = nonzero_bytes((s ^ ex) & m);
  if (ff) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (((ff >> (8 * i)) & 1u) && pos0 + i < lmax) atomicAdd(&other[pos0 + i], sign);
  }
  return codes & ~ff;
}

template <int V>
struct TriTag {
  static constexpr int value = V;
};
using AddTag = TriTag<0>;    // add the step's reads
using SubTag = TriTag<1>;    // take reads out of the widened byte counters (unit epilogue)
using UndoTag = TriTag<2>;   // take back what the same step just added (nibble counters)

// ---- edit (A6) on the segmented kernel ---------------------------------------
// The trim of one read: the leading run of out-of-range qualities within the
// first min(edit_left_length, n) bases and the trailing run within the last
// min(edit_right_length, n - ts) with the SWAR in_range
// test, from three 16-byte loads issued together for windows up to 16 / 32
// bytes (trim_issue + trim_finish; else 8 bytes at a time, trim_word); quality
// bytes [off, off + n) of rq; ts | te << 16 is the edit output.  Run by the
// unit prologue, one lane per read.

// the trim windows' quality bytes for the usual windows (left <= 16, right <=
// 32): three 16-byte loads issued together: the first 16 bytes of the read and
// the 32 bytes ENDING at its end (from off + n - 32, even for a read shorter
// than 32: the bytes before the read are the previous read's and lie before
// any right window, so trim_finish needs no mask).  Only where that start
// falls below the buffer (the first reads of a batch) do the loads start at 0
// and hi = off + n < 32 marks the window's end (trim_finish masks past it).
// Lanes without a read pass a negative offset (0xC0000000): out of range.
struct TrimLoads {
  v4u wl, wr0, wr1;
  int hi;   // the right window ends at byte hi of the 32 loaded (32 but at the buffer start)
};

__device__ __forceinline__ bool trim_usual(const ColdParams &C) { return C.e_left_len <= 16 && C.e_right_len <= 32; }

__device__ __forceinline__ TrimLoads trim_issue(const ColdParams &C, __amdgpu_buffer_rsrc_t rq, int off, int n) {
  TrimLoads T;
  T.wl = C.e_left_len > 0 ? __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)off, 0, 0) : v4u{0u, 0u, 0u, 0u};
  T.wr0 = T.wr1 = v4u{0u, 0u, 0u, 0u};
  int pa = off + n - 32;
  if (pa < 0 && off >= 0) pa = 0;
  T.hi = off + n - pa;
  if (C.e_right_len > 0) {
    T.wr0 = __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)pa, 0, 0);
    T.wr1 = __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)(pa + 16), 0, 0);
  }
  return T;
}

// v_ffbl / v_ffbh with the hardware's all-ones result for 0 (the builtins'
// defined-at-zero forms add a compare and a select per dword)
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t ffbh_raw(uint32_t x) {
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// 0x80 per in-range byte of the raw quality dword w (TrimSide): >= the lower
// bound and not >= the upper one, six VALU (w | 0x80 shared)
// (each compare is ONE v_bitop3 of (w, c ^ 0x80, (w | 0x80) - (c & 0x7F)):
// truth table 0x8E = (~w & c') | (~(w ^ c') & d); hipcc left to itself spends
// three instructions on it; the combine ge_lo & ~ge_hi & 0x80 is bitop3 0x20)
// HINONE (no upper bound, TrimSide::hq = 0 and h7 = 0x80808080, for which
// "≥ hi" never holds): the lower compare alone, four VALU
template <bool HINONE = false>
__device__ __forceinline__ uint32_t trim_side_ok(uint32_t w, const TrimSide &S) {
  const uint32_t wh = w | kQFlip;
  const uint32_t ge_lo = __builtin_amdgcn_bitop3_b32(w, S.lq, wh - S.l7, 0x8E);
  if (HINONE) return ge_lo & kQFlip;
  const uint32_t ge_hi = __builtin_amdgcn_bitop3_b32(w, S.hq, wh - S.h7, 0x8E);
  return __builtin_amdgcn_bitop3_b32(ge_lo, ge_hi, kQFlip, 0x20);
}
__device__ __forceinline__ bool trim_hi_none(const TrimSide &S) { return S.hq == 0u && S.h7 == kQFlip; }

// the trims of a read of length n from its usual-window loads: ts | te << 16.
// Branch-free (round 5): ts = min(first in-range index of the left window,
// min(left_len, n)); te = min(min(right_len, n - ts), hi - 1 - last in-range
// index of the 32 bytes ending at the read's end).  A dword with no in-range
// byte gives ffbl / ffbh = ~0, i.e. an index far past any window.
__device__ __forceinline__ uint32_t trim_finish(const ColdParams &C, const TrimLoads &T, int n) {
  const uint32_t wl[4] = {T.wl.x, T.wl.y, T.wl.z, T.wl.w};
  const uint32_t wr[8] = {T.wr0.x, T.wr0.y, T.wr0.z, T.wr0.w, T.wr1.x, T.wr1.y, T.wr1.z, T.wr1.w};
  // (a side without an upper bound -- the usual `--left-quality-range 20,` --
  // takes the four-VALU compare: a uniform branch per side; a left length of
  // at most 12 leaves the window's last dword out: an in-range byte there
  // would give ts >= 12 > left_len, which the min below makes left_len anyway)
  uint32_t first = ~0u;
  const int nl = C.e_left_len <= 12 ? 3 : 4;
  auto left = [&](auto hn) __attribute__((always_inline)) {
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (w < nl) first = min(first, (ffbl_raw(trim_side_ok<decltype(hn)::value>(wl[w], C.tl)) >> 3) + 4u * w);
  };
  if (trim_hi_none(C.tl)) left(std::true_type{});
  else left(std::false_type{});
  uint32_t okr[8];
  if (trim_hi_none(C.tr)) {
#pragma unroll
    for (int k = 0; k < 8; ++k) okr[k] = trim_side_ok<true>(wr[k], C.tr);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) okr[k] = trim_side_ok<false>(wr[k], C.tr);
  }
  if (__builtin_expect(T.hi < 32, 0)) {   // a read at the buffer start: bytes >= hi are the next read's
#pragma unroll
    for (int k = 0; k < 8; ++k) okr[k] &= byte_mask(T.hi - 4 * k);
  }
  int last = -1;
#pragma unroll
  for (int k = 0; k < 8; ++k) last = max(last, 4 * k + 3 - (int)(ffbh_raw(okr[k]) >> 3));
  const int ts = (int)min(first, (uint32_t)min(C.e_left_len, n));
  const int te = min(min(C.e_right_len, n - ts), T.hi - 1 - last);
  return (uint32_t)ts | ((uint32_t)te << 16);
}


// 16 bytes per lane from a buffer straight into LDS (buffer_load_dwordx4 ...
// lds: lane l writes at lds + 16 l; no VGPR destination).  Inline asm, so the
// compiler neither sees the LDS write (it would make every later LDS read of
// the kernel wait for it: one exposed HBM round trip per unit again) nor
// counts it: the reader waits for it explicitly (s_waitcnt vmcnt, in order).
// M0 (the LDS base: lds + OFF bytes, added in the asm so only `lds` is held in
// an SGPR across the loop, not one hoisted address per row) is saved and
// restored around it.
template <int OFF>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(lds), "n"(OFF)
               : "memory", "scc");
}

// 0x80 per in-range byte of raw quality words x, y (bytes 0-3, 4-7)
__device__ __forceinline__ uint64_t trim_ok(const ColdParams &C, uint32_t x, uint32_t y, bool right) {
  const TrimSide &S = right ? C.tr : C.tl;
  return (uint64_t)trim_side_ok(x, S) | ((uint64_t)trim_side_ok(y, S) << 32);
}

__device__ __forceinline__ uint64_t trim_low_bytes(int k) { return k >= 8 ? ~0ull : ((1ull << (8 * max(k, 0))) - 1); }

// any window: the usual ones by trim_finish, else 8 bytes at a time
__device__ __forceinline__ uint32_t trim_word(const ColdParams &C, __amdgpu_buffer_rsrc_t rq,
                                              int off, int n) {
  auto ok8 = [&](int pos, bool right) __attribute__((always_inline)) -> uint64_t {
    const v2u w = __builtin_amdgcn_raw_buffer_load_b64(rq, (uint32_t)(off + pos), 0, 0);
    return trim_ok(C, w.x, w.y, right);
  };
  auto low_bytes = [](int k) -> uint64_t { return trim_low_bytes(k); };
  if (trim_usual(C)) return trim_finish(C, trim_issue(C, rq, off, n), n);
  int ts = 0, te = 0;
  if (C.e_left_len > 0) {
    const int lim = min(C.e_left_len, n);
    ts = lim;
    for (int c = 0; c < lim; c += 8) {
      const uint64_t ok = ok8(c, false) & low_bytes(lim - c);
      if (ok) {
        ts = c + (__builtin_ctzll(ok) >> 3);
        break;
      }
    }
  }
  if (C.e_right_len > 0) {
    const int lim = min(C.e_right_len, n - ts);
    const int lo = n - lim;
    te = lim;
    for (int e = n; e > lo; e -= 8) {
      const int st = max(e - 8, lo);
      const uint64_t ok = ok8(st, true) & low_bytes(e - st);
      if (ok) {
        te = n - 1 - (st + ((63 - __builtin_clzll(ok)) >> 3));
        break;
      }
    }
  }
  return (uint32_t)ts | ((uint32_t)te << 16);
}

// floor(x / n) for a read length 1 <= n <= 252 from rc = ceil(2^32 / n) (the
// kernel's rtab; n = 1 has rc = 0 and one1 = 1): q = mulhi(x, rc) is exact
// while x * (n - 1) < 2^32 (the error of rc times x stays below one unit of
// 1 / n), which holds for every numerator of the unit epilogue (biased
// quality sums < 2^16, 100 x G+C, remainders << 16 < n 2^16)
__device__ __forceinline__ uint32_t div_len(uint32_t x, uint32_t rc, uint32_t one1) {
  return __umulhi(x, rc) + __umul24(x, one1);
}

// meanq_terms (hpgq_engine_kernel.h) for the segmented kernels' reads (n <=
// 252) by div_len: one multiply-high per quotient instead of a 32-bit division
// (round 6: ~65 VALU per unit epilogue and mate)
__device__ __forceinline__ void meanq_terms_rc(uint32_t sb, uint32_t n, uint32_t rc, uint32_t one1, uint32_t &bin,
                                               uint64_t &fx) {
  const uint32_t off = (uint32_t)kQBias * n;
  const uint32_t q = div_len(sb, rc, one1), rem = sb - __umul24(q, n);
  if (__builtin_expect(sb >= off, 1)) {
    bin = q + (2 * rem >= n ? 1u : 0u) - (uint32_t)kQBias;   // (2 sb + n) / (2 n) - 128
  } else {
    const uint32_t t = off - sb, qt = div_len(t, rc, one1), rt = t - __umul24(qt, n);
    bin = (256u - (qt + (2 * rt >= n ? 1u : 0u))) & 255u;
  }
  fx = ((uint64_t)q << 16) + div_len(rem << 16, rc, one1) - ((uint64_t)kQBias << 16);
}

template <int M>
struct MateTag {
  static constexpr int value = M;
};

// MINW: minimum waves per SIMD the register allocation must allow (occupancy).
// NM = 2: paired-end.  A block is one block's worth of pairs; the wave runs
// mate 1's steps, then mate 2's, each mate with its own accumulators / LDS
// partials / counter set; the epilogue takes the pair decision (both mates
// pass) and subtracts failed pairs from both sets.
// EDIT: the unit prologue trims each read (each mate; trim_word, written to
// A.trim when the caller wants it: mate 2 at num_reads + i) and describes it
// by its window [ts, n - te) (offset + ts, length n - ts - te): stats and the
// filter (with any extra scans) see the trimmed read.
// XM (extra filter scans; the plain kernels have none):
//   X_NOOR: the filter also counts N bases and out-of-range qualities per read
//     (max_N, max_out_of_quality; src/filter_fastq.c:140-145): a second
//     per-step scan of (N | out-of-range << 16), its segment ends in a second
//     LDS list;
//   X_LR: the 5'/3' window filters (left/right length + quality range,
//     src/filter_fastq.c:140-145 args 6-11): a per-step scan of the window
//     quality sums (left | right << 16; each < 255 x 252 < 2^16, and the
//     segment sums come out exact as differences mod 2^32), the windows cut
//     by two more rows of the byte-mask table.
// FOLLOW: a follow-up stage (reads deferred by the stage before, by unit masks).
template <int MINW, int NM, bool EDIT, int G, int XM, bool FOLLOW>
__device__ __forceinline__ void tri_body(const EngineArgs &A) {
  constexpr bool NX = XM & X_NOOR, LR = XM & X_LR;
  // PASS FIRST (single-end, no extra scans): each step decides its reads'
  // pass/fail from the step's own scan (segment totals by two ds_bpermute)
  // BEFORE accumulating, so failed reads are never added and never re-read to
  // be taken out (that re-read missed L2: +8 % HBM traffic and +3.5 % time at
  // C2's ~6 % failures).  Paired-end, edit and the follow-up stages still add
  // every read and subtract the failed ones in the unit epilogue.
  // (edit, follow-up: their registers would spill; the window variant alone
  // fails few reads and ran 4 % slower with it: 692 vs 665 us per 10 M reads)
  constexpr bool PF = NM == 1 && !EDIT && !FOLLOW && XM != X_LR;
  // ST (single-end edit, hex, first stage, usual windows with a left length <=
  // 12 -- the host picks it, plan_chain): the stream loads each read
  // UNTRIMMED, so no load waits for a trim; the group's trim windows are
  // gathered right after its stream loads (the same lines: no re-fetch) and
  // the trims are finished when the group is counted, each step shifting its
  // reads' bytes by their ts (a register shuffle, only in steps holding a
  // read with ts > 0) and counting n - ts - te of them; the finished trims
  // patch the read table for the unit epilogue (lengths, trim words, the
  // failed reads' re-gather).  See st_trims.
  constexpr bool ST = (XM & X_ST) != 0;
  static_assert(!ST || (XM == X_ST && NM == 1 && EDIT && !FOLLOW && G == GEO_HEX), "ST: single-end edit, hex");
  constexpr bool LATE = EDIT && !ST;   // the unit prologue's place (see the unit loop)
  constexpr bool TABLEN = !FOLLOW;   // epilogue lengths / trims from the read table
  // PEU (paired-end): a group is ONE step of both mates (grp[slot][m]); both
  // are added, the pair is decided from both scans at once (ds_bpermute), and
  // a failed pair is taken back out of the nibble counters from the registers
  // still holding it -- no re-read (the epilogue's re-gather of failed pairs
  // missed L2 and cost 15 % of C3).  Holding both mates' step values for a
  // pass-first decision instead needed 215 VGPRs (2 waves/SIMD: no faster).
  constexpr bool PEU = NM == 2 && !FOLLOW && XM == 0 && Geo<G>::kU >= 2;
  using GG = Geo<G>;
  constexpr int NW = GG::kNW, kSegs = GG::kSegs, kSegW = GG::kSegW, kBlock = GG::kBlock, kU = GG::kU;
  static_assert(4 * kU <= kNibbleEvery && kBlock / kSegs - 4 * kU <= kNibbleEvery, "nibble widening");
  static_assert(kSegs * kSegW <= 64 && kBlock < 64 && kBlock % kSegs == 0, "geometry");
  constexpr bool kMidWiden = kBlock / kSegs > 4 * kU;   // more steps per unit than 4 groups
  // TDMA (paired-end edit, first stage, no extra scans -- whose LDS would not
  // fit at 3 workgroups per CU): a unit's trim windows come from LDS, DMA'd
  // there during the unit before's last group pair, instead of gathers whose
  // round trip the unit prologue waited for.  Round 5, one
  // box: c4_pe 1578 -> 1500 us; single-end measured no faster (its lines,
  // fetched earlier, are evicted before the stream comes back for them: HBM
  // traffic 1.34 -> 1.40x, C4 824 -> 840 us), so single-end keeps the gathers.
  constexpr bool TDMA = EDIT && !FOLLOW && NM == 2 && XM == 0;
  // EG (single-end edit, first stage, no extra scans; 3 waves per SIMD, which
  // leave the registers): the next unit's trim windows gathered into VGPRs at
  // the top of this unit's last group pair -- a group of work before the
  // prologue that finishes them, instead of a round trip the prologue waits
  // for.  Round 6, one box, 3 alternating rounds: C4 844 us against 850 (the
  // same at 4 waves per SIMD spilled 7 VGPRs and ran slower, round 5; the
  // extra-scan kernels, c4_noor, ran 2.9 % slower with it and keep 4 waves)
  constexpr bool EG = EDIT && !FOLLOW && NM == 1 && XM == 0;
  if (FOLLOW && follow_up_idle(A)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int lmax = A.lmax;
  // the LDS partials cover lp positions: every read this kernel merges is at
  // most min(lmax, kPos) long (longer ones are deferred), so the counter set
  // on chip does not grow with lmax (at lmax 1024 it would cut the residency)
  const int lp = min(lmax, Geo<G>::kPos);
  const int hlen = lp + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  const int seg = min(lane / kSegW, kSegs);     // kSegs: idle lanes
  const int ls = lane - seg * kSegW;
  const bool owner = seg < kSegs && ls < GG::kOwn;
  const int p0 = owner ? 4 * NW * ls : (1 << 26);   // first position of this lane (8*p0 fits int32)
  const uint32_t lane8 = 4u * NW * (uint32_t)ls;   // byte offset of this lane's window
  const bool stats = A.flags & F_STATS, filter = A.flags & F_FILTER;
  // NX: the filter's extra limits, read once (not from *A.cold inside the loop,
  // where each scalar reload would wait for the outstanding LDS operations too)
  // (the quality range as the trims' TrimSide constants: no flags to branch on per word)
  const TrimSide xr = NX ? TrimSide{(uint32_t)uni((int)A.cold->to.lq), (uint32_t)uni((int)A.cold->to.l7),
                                    (uint32_t)uni((int)A.cold->to.hq), (uint32_t)uni((int)A.cold->to.h7)}
                         : TrimSide{0u, 0u, 0u, 0u};
  const bool x_hin = NX && trim_hi_none(xr);
  const int x_maxn = NX ? uni(A.cold->max_n) : 0, x_maxo = NX ? uni(A.cold->max_oor) : 0;
  const bool x_n = NX && (A.flags & F_NEED_N), x_o = NX && (A.flags & F_NEED_OOR);
  // LR: the window filters, read once (see NX above); length 0 = off
  const int w_ll = LR ? max(uni(A.cold->left_len), 0) : 0, w_rl = LR ? max(uni(A.cold->right_len), 0) : 0;
  // (window means lie in [-383, 127] Phred: bounds clamped to +-512 keep k * bound in int32)
  auto clampq = [](int q) { return min(max(q, -512), 512); };
  const int w_lmin = LR ? clampq(uni(A.cold->min_left)) : 0, w_lmax = LR ? clampq(uni(A.cold->max_left)) : 0;
  const int w_rmin = LR ? clampq(uni(A.cold->min_right)) : 0, w_rmax = LR ? clampq(uni(A.cold->max_right)) : 0;
  // mean-quality window test in 32-bit: min*k <= S - phred*k <= max*k (S < 2^16, k <= 252)
  auto win_in = [&](int sb, int k, int lo, int hi) __attribute__((always_inline)) {
    const int q = sb - A.phred * k;
    return lo * k <= q && q <= hi * k;
  };
  // a left window within a lane's positions and no right window: no scan (the
  // segment's first lane stores its sum)
  const bool w_direct = LR && w_rl == 0 && w_ll <= 4 * NW;
  // EDIT: the trim bounds, read once (see NX above)
  // (held across the loop: re-reading them per unit prologue cut the
  // single-end SGPR spills 90 -> 71 but cost 5 % of C4, and paired-end
  // spilled more VGPRs that way)
  ColdParams cold_all{};
  if (EDIT) cold_all = *A.cold;
  // biased-sum bounds (A.phred is phred + 128): pass iff min_len <= n <= max_len and lo_r*n <= S <= hi_r*n
  const int lo_r = A.min_q + A.phred, hi_r = A.max_q + A.phred;
  const int dlim = A.defer_len;   // longer reads go to the next stage

  // LDS per mate: pos_acc [6][lmax] u32 | hist [hlen] u32 | sc [8] u64, then
  // per wave: per mate two read tables [64] x 16 B (seq offset, qual offset,
  // length | alignments, -) alternating between blocks, and segment ends [64]
  // (+ [64] NX, + [64] LR), then a compaction scratch [64] u32 and a deferral word (u64,
  // disjoint from the scratch: no type-punned aliasing); then the byte-mask table.
  // (pos_acc row 5 holds "other" counts until the epilogue turns it into N)
  const int hist_words = (hlen + 1) & ~1;
  const int mate_words = 6 * lp + hist_words + 2 * HPGQ_NUM_SCALARS;   // even: sc 8-B aligned
  uint32_t *base = reinterpret_cast<uint32_t *>(lds);
  auto pos_acc = [&](int m) __attribute__((always_inline)) { return base + m * mate_words; };
  auto other = [&](int m) __attribute__((always_inline)) { return base + m * mate_words + 5 * lp; };
  auto hist = [&](int m) __attribute__((always_inline)) { return base + m * mate_words + 6 * lp; };
  auto sc = [&](int m) __attribute__((always_inline)) {
    return reinterpret_cast<unsigned long long *>(base + m * mate_words + 6 * lp + hist_words);
  };
  constexpr int kMateWaveWords = 2 * 256 + 64 * (1 + (NX ? 1 : 0) + (LR ? 1 : 0));
  // TDMA: the next unit's trim windows, DMA'd one unit ahead (see dma_windows):
  // per mate three rows (left, right 0, right 1) of kBlock x 16 B
  constexpr int kDmaWords = TDMA ? NM * 3 * kBlock * 4 : 0;
  constexpr int kWaveWords = NM * kMateWaveWords + 64 + 4 + NM * kFxWords + kDmaWords +
                             (ST ? kStWords : 0);   // (multiple of 4: 16 B tables)
  const int tab_words = (NM * mate_words + 3) & ~3;   // 16 B aligned (host: + 16 B)
  // (ST: the shift buffers first in the wave's region, so their reads' offsets
  // fit the ds_read2 offset fields)
  uint32_t *wst = base + tab_words + wave * kWaveWords;
  uint32_t *wtab = wst + (ST ? kStWords : 0);
  auto tab = [&](int m, int tb) __attribute__((always_inline)) { return wtab + m * kMateWaveWords + tb * 256; };
  auto wends = [&](int m) __attribute__((always_inline)) { return wtab + m * kMateWaveWords + 2 * 256; };
  auto wends2 = [&](int m) __attribute__((always_inline)) { return wtab + m * kMateWaveWords + 2 * 256 + 64; };   // NX only
  auto wends3 = [&](int m) __attribute__((always_inline)) {   // LR only
    return wtab + m * kMateWaveWords + 2 * 256 + (NX ? 128 : 64);
  };
  uint32_t *scratch = wtab + NM * kMateWaveWords;
  unsigned long long *dword = reinterpret_cast<unsigned long long *>(scratch + 64);   // 8 B aligned
  // the DMA rows of mate m, window w (16 B aligned)
  auto dma_row = [&](int m, int w) __attribute__((always_inline)) {
    return scratch + 64 + 4 + NM * kFxWords + (m * 3 + w) * kBlock * 4;
  };
  // per-lane exact mean-quality sums, 8 B aligned
  // ST: the wave's shift buffers (b = 0 seq, 1 quality; 16 B aligned)
  auto stbuf = [&](int b) __attribute__((always_inline)) {
    return wst + b * (kStWords / 2);
  };
  auto fxs = [&](int m) __attribute__((always_inline)) {
    return reinterpret_cast<unsigned long long *>(scratch + 64 + 4 + m * kFxWords);
  };
#pragma unroll
  for (int m = 0; m < NM; ++m)
    if (lane < kFxSlots) fxs(m)[lane] = 0ull;
  // byte masks by valid-byte count c = clamp(n - p0, 0, 4 NW): mtab[c][w]
  // (one LDS read per step instead of a clamp and a 64-bit shift per word)
  uint32_t *mtab = base + tab_words + kWaves * kWaveWords;   // 16 B aligned
  for (int i = tid; i < (4 * NW + 1) * NW; i += kWG) {
    const int nb = min(max(i / NW - 4 * (i % NW), 0), 4);
    mtab[i] = nb == 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1u;
  }
  // the epilogue's divisions by a read's length n <= kPos as multiply-highs:
  // rtab[n] = ceil(2^32 / n) (0 for n = 1, see div_len)
  uint32_t *rtab = mtab + 17 * 4;
  for (int i = tid; i <= GG::kPos; i += kWG) rtab[i] = i <= 1 ? 0u : 0xFFFFFFFFu / (uint32_t)i + 1u;
  for (int i = tid; i < NM * mate_words; i += kWG) base[i] = 0;
  __syncthreads();

  // SRDs: the read bytes plus the load slack
  __amdgpu_buffer_rsrc_t rs[NM], rq[NM];
  int bs[NM], bq[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int data_end = uni(A.idx[m][A.num_reads]);
    const uintptr_t ps = reinterpret_cast<uintptr_t>(A.seq[m]), pq = reinterpret_cast<uintptr_t>(A.qual[m]);
    bs[m] = (int)(ps & 3);
    bq[m] = (int)(pq & 3);
    rs[m] = __builtin_amdgcn_make_buffer_rsrc((void *)(ps - bs[m]), (short)0,
                                              bs[m] + data_end + kTriSlack, 0x00020000);
    rq[m] = __builtin_amdgcn_make_buffer_rsrc((void *)(pq - bq[m]), (short)0,
                                              bq[m] + data_end + kTriSlack, 0x00020000);
  }
  TriAcc<NW> acc[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m].zero();
  int since_flush = 0;   // steps per mate added since the last LDS flush (a byte grows <= 1 per step)
  // per-wave counts: input and passed reads (pairs) are the same for both
  // mates and failed = input - passed (a pass is valid), stats = passed when
  // stats are on; only the edited count is per mate (SGPRs are short in the
  // paired-end kernels: five counters per mate spilled into VGPR lanes)
  uint32_t cnt_in = 0, cnt_pass = 0, cnt_ed[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) cnt_ed[m] = 0;
  uint32_t ndefer = 0;   // reads this wave handed to the next stage

  const int ublock = FOLLOW ? A.unit_reads : kBlock;   // reads per unit
  UnitIter<FOLLOW, kBlock> it;
  it.init(A, (int)blockIdx.x * kWaves + wave, (int)gridDim.x * kWaves);

  // a unit's read offsets (lane j: read j), fetched one unit ahead of the
  // prologue that describes it, so the prologue does not wait for them
  // (FOLLOW: the compaction leaves the unit's read positions in `scratch` for
  // the prologue, so no register carries them across the iteration)
  auto fetch_idx = [&](const Unit &U, int32_t (&ia)[NM], int32_t (&ie)[NM]) __attribute__((always_inline)) {
    const int r = U.nr > 0 ? unit_read<FOLLOW>(U, U.u * ublock, scratch) : 0;
    const bool on = lane < U.nr;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      ia[m] = on ? A.idx[m][r] : 0;
      ie[m] = on ? A.idx[m][r + 1] : 0;
    }
  };
  // unit prologue: lane j describes read (pair) j in read table `tb`; absent
  // and deferred reads get length 0 and out-of-range offsets.  Returns this
  // lane's lengths (the epilogue needs them) and the deferred-lane mask.
  auto load_block = [&](const Unit &U, int tb, uint32_t (&len)[NM], uint32_t (&tw)[NM], uint64_t &dm,
                        const int32_t (&ia)[NM], const int32_t (&ie)[NM], bool dma,
                        const TrimLoads *pre = nullptr) __attribute__((always_inline)) {
    const bool on = lane < U.nr;
    const uint32_t rid = (uint32_t)(U.u * ublock) + (FOLLOW ? scratch[lane] : (uint32_t)lane);
    bool dfr = false;
#pragma unroll
    for (int m = 0; m < NM; ++m) dfr = dfr || (ie[m] - ia[m] > dlim);
    dfr = dfr && on;
    dm = __ballot(dfr);
    const bool live = on && !dfr;
    if (U.u >= 0) {
      uint64_t pbits = dm;   // deferred reads by position in the unit
      if (FOLLOW && dm) {
        if (lane == 0) *dword = 0ull;
        __builtin_amdgcn_wave_barrier();
        if (dfr) atomicOr(dword, 1ull << (rid - (uint32_t)(U.u * ublock)));
        __builtin_amdgcn_wave_barrier();
        pbits = uni64(*dword);
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) A.defer_bits[U.u] = pbits;
      ndefer += (uint32_t)__builtin_popcountll(dm);
    }
    // EDIT, usual windows: from the DMA rows (dma: the windows were DMA'd
    // during the unit before, and waited for by the caller), else (the first
    // unit; paired-end kernels without TDMA) both mates' trim loads in flight
    // before the first is finished (one exposed round trip per unit, not one
    // per mate; single-end without TDMA keeps trim_word)
    TrimLoads tl[NM];
    const ColdParams &cold = cold_all;
    const bool fromdma = TDMA && dma && trim_usual(cold);
    const bool usual = EDIT && (fromdma || (NM == 2 && trim_usual(cold)));
    if (fromdma) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int off = live ? bq[m] + ia[m] : (int)0xC0000000, n = ie[m] - ia[m];
        tl[m].wl = *reinterpret_cast<const v4u *>(dma_row(m, 0) + 4 * lane);
        tl[m].wr0 = *reinterpret_cast<const v4u *>(dma_row(m, 1) + 4 * lane);
        tl[m].wr1 = *reinterpret_cast<const v4u *>(dma_row(m, 2) + 4 * lane);
        int pa = off + n - 32;
        if (pa < 0 && off >= 0) pa = 0;
        tl[m].hi = off + n - pa;
      }
    } else if (usual) {
#pragma unroll
      for (int m = 0; m < NM; ++m)
        tl[m] = trim_issue(cold, rq[m], live ? bq[m] + ia[m] : (int)0xC0000000, ie[m] - ia[m]);
    }
    const bool pre_ok = EG && pre != nullptr && trim_usual(cold);   // EG: issued by gather_next
    // (ST: described untrimmed; the group's trims patch the records later)
    if (pre_ok) tl[0] = *pre;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      int a = ia[m], e = ie[m];
      tw[m] = 0;
      if (EDIT) {   // trim here, then describe the trimmed window
        tw[m] = !live || ST ? 0u : (usual || pre_ok) ? trim_finish(cold, tl[m], e - a) : trim_word(cold, rq[m], bq[m] + a, e - a);
        if (A.trim && live && !ST) A.trim[(size_t)m * (size_t)A.num_reads + rid] = tw[m];
        a += (int)(tw[m] & 0xFFFFu);
        e -= (int)(tw[m] >> 16);
        if (e < a) e = a;
      }
      const uint32_t n = live ? (uint32_t)(e - a) : 0u;
      const uint32_t xs = live ? (uint32_t)(bs[m] + a) : 0x80000000u;
      const uint32_t xq = live ? (uint32_t)(bq[m] + a) : 0x80000000u;
      // (FOLLOW: the read id rides in the record's spare dword, for the
      // epilogue; else the trim word, when the epilogue reads it back)
      const uint32_t spare = FOLLOW ? rid : tw[m];
      const v4u rec = v4u{xs & ~3u, xq & ~3u, n | ((xs & 3u) << 16) | ((xq & 3u) << 20), spare};
      *reinterpret_cast<v4u *>(tab(m, tb) + 4 * lane) = rec;
      len[m] = n;
    }
    __builtin_amdgcn_wave_barrier();   // other lanes read them (LDS is in order per wave)
  };
  // steps holding the unit's non-deferred reads (0: nothing to stream)
  auto steps_of = [&](const Unit &U, uint64_t dm) __attribute__((always_inline)) {
    return __builtin_popcountll(dm) == U.nr ? 0 : (U.nr + kSegs - 1) / kSegs;
  };
  // lane -> its segment's read (the entry `eoff` bytes into mate m's read table tb)
  // the stream loads' cache policy: non-temporal (nt) for the PF kernels (C2
  // and its N / out-of-range variants: round 6, one box, 3 alternating rounds,
  // C2 528.6 -> 523.5 us); the others re-read lines the stream brought in
  // (trim windows, step-boundary lines) and ran 3-4 % slower with nt
  // (C3 1107 -> 1147, C4 815 -> 840; profiles/r06_nt_ab.json)
  constexpr int kAux = PF ? 2 : 0;
  auto gather_at = [&](int m, int tb, uint32_t eoff, TriPending<NW> &pd) __attribute__((always_inline)) {
    const v4u rec = *reinterpret_cast<const v4u *>(reinterpret_cast<const uint8_t *>(tab(m, tb)) + eoff);
    pd.n = rec.z;
    if (NW == 2) {
      const v2u a = __builtin_amdgcn_raw_buffer_load_b64(rs[m], rec.x + lane8, 0, kAux);
      const v2u b = __builtin_amdgcn_raw_buffer_load_b64(rq[m], rec.y + lane8, 0, kAux);
      pd.s[0] = a.x; pd.s[1] = a.y; pd.q[0] = b.x; pd.q[1] = b.y;
    } else {
      const v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs[m], rec.x + lane8, 0, kAux);
      const v4u b = __builtin_amdgcn_raw_buffer_load_b128(rq[m], rec.y + lane8, 0, kAux);
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        pd.s[w] = a[w & 3];
        pd.q[w] = b[w & 3];
      }
    }
  };
  auto gather = [&](int m, int tb, int src, TriPending<NW> &pd) __attribute__((always_inline)) {
    gather_at(m, tb, 16u * (uint32_t)src, pd);
  };
  // step t's entry of this lane: kSegs t + seg (< kBlock + kSegs <= 64 for every
  // lane, idle ones included); a step past the unit end (t >= nt) reads entry
  // kBlock + seg, which no read of a unit fills (length 0, offsets out of
  // range: it adds nothing and loads nothing; a follow-up unit -- wide, 60 --
  // holds at most the 54 reads of a tri / hex unit, plan_chain).  The step part is uniform, so
  // the address is one VALU add (round 6; a clamp and a select were 5)
  const uint32_t seg16 = 16u * (uint32_t)seg;
  // segment end of step t -> list[kSegs t + seg] (the step part uniform: one
  // VALU add for the address, not a 64-bit multiply-add)
  // (the empty asm keeps hipcc from folding the two into a v_mad_u64_u32)
  auto put_end = [&](uint32_t *list, int t, uint32_t v) __attribute__((always_inline)) {
    uint32_t so = (uint32_t)(4 * kSegs * t);
    asm volatile("" : "+s"(so));
    *reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(list) + (seg16 >> 2) + so) = v;
  };
  auto step_off = [&](int t, int ntt) __attribute__((always_inline)) {
    return seg16 + (t < ntt ? (uint32_t)(16 * kSegs * t) : (uint32_t)(16 * kBlock));
  };

  TriPending<NW> grp[2][kU];
  // ST: the trim windows of a group PAIR (g, g + 1: the unit's reads 12 g ..
  // 12 g + 23), two lanes per read (lane 2r + h): h = 0 the first 16 quality
  // bytes (w0) and the first half of the 32 ending at the read's end (w1),
  // h = 1 its second half (w0)
  v4u stw0 = v4u{0u, 0u, 0u, 0u}, stw1 = v4u{0u, 0u, 0u, 0u};
  // issue group g (kU steps) of mate m; steps past the unit end gather an
  // entry no read fills (step_off), so they add nothing
  auto load_group = [&](int m, int tb, int nt, int g, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      gather_at(m, tb, step_off(g * kU + u, nt), grp[slot][u]);
    }
    if (ST && slot == 0) {   // (the pair's windows, after group g's stream loads: the same lines)
      const int r = lane >> 1, h = lane & 1, idx = kSegs * kU * g + r;
      uint32_t a0 = 0xC0000000u, a1 = 0xC0000000u;   // (out of range: zeros, no traffic)
      if (r < 2 * kSegs * kU && g * kU < nt) {
        const v4u rec = *reinterpret_cast<const v4u *>(tab(0, tb) + 4 * idx);
        const int n = (int)(rec.z & 0xFFFFu), off = (int)(rec.y | ((rec.z >> 20) & 3u));
        const int pa = max(off + n - 32, 0);
        if (n > 0 && !(rec.y & 0x80000000u)) {
          if (h == 0) {
            if (cold_all.e_left_len > 0) a0 = (uint32_t)off;
            if (cold_all.e_right_len > 0) a1 = (uint32_t)pa;
          } else if (cold_all.e_right_len > 0) {
            a0 = (uint32_t)(pa + 16);
          }
        }
      }
      stw0 = __builtin_amdgcn_raw_buffer_load_b128(rq[0], a0, 0, 0);
      stw1 = __builtin_amdgcn_raw_buffer_load_b128(rq[0], a1, 0, 0);
    }
  };
  // ST: the trims of the group pair from g (even, unit ubase); lane 2r returns
  // read r's ts | te << 16 (0 for a read without one or not live) and patches
  // its read-table record to the trimmed window (offsets + ts, length n - ts -
  // te, the trim word) -- after the groups' loads took the untrimmed records.
  // trim_finish's arithmetic over two lanes per read (the right window's
  // halves combined by one DPP).
  auto st_trims = [&](int tbx, int g, size_t ubase) __attribute__((always_inline)) -> uint32_t {
    const int r = lane >> 1, h = lane & 1, idx = kSegs * kU * g + r;
    const bool act = r < 2 * kSegs * kU;
    v4u rec = v4u{0x80000000u, 0x80000000u, 0u, 0u};
    if (act) rec = *reinterpret_cast<const v4u *>(tab(0, tbx) + 4 * idx);
    const int n = (int)(rec.z & 0xFFFFu), off = (int)(rec.y | ((rec.z >> 20) & 3u));
    const int pa = max(off + n - 32, 0), hi = off + n - pa;   // hi: 32 but at the buffer's start
    const TrimSide &L = cold_all.tl, &R = cold_all.tr;
    const uint32_t a[4] = {stw0.x, stw0.y, stw0.z, stw0.w}, b[4] = {stw1.x, stw1.y, stw1.z, stw1.w};
    uint32_t oka[4], okb[4];   // w0 on the lane's side (h = 0 left, 1 right), w1 right
    if (trim_hi_none(L) && trim_hi_none(R)) {
      const TrimSide S{h ? R.lq : L.lq, h ? R.l7 : L.l7, 0u, kQFlip};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        oka[k] = trim_side_ok<true>(a[k], S);
        okb[k] = trim_side_ok<true>(b[k], R);
      }
    } else {
      const TrimSide S{h ? R.lq : L.lq, h ? R.l7 : L.l7, h ? R.hq : L.hq, h ? R.h7 : L.h7};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        oka[k] = trim_side_ok<false>(a[k], S);
        okb[k] = trim_side_ok<false>(b[k], R);
      }
    }
    if (__builtin_expect(hi < 32, 0)) {   // a read at the buffer's start: bytes >= hi are the next read's
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        okb[k] &= byte_mask(hi - 4 * k);        // (h = 0: tail bytes 0..15)
        if (h) oka[k] &= byte_mask(hi - 16 - 4 * k);   // (h = 1: tail bytes 16..31)
      }
    }
    // h = 0: first in-range index of the left window; both: last in-range
    // index of their tail half (h = 1's from w0, at +16; negative when none)
    uint32_t f = ~0u;
    int vr = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f = min(f, (ffbl_raw(oka[k]) >> 3) + 4u * k);   // (h = 1: unused)
      const uint32_t y = h ? oka[k] : okb[k];
      vr = max(vr, 4 * k + 3 - (int)(ffbh_raw(y) >> 3));
    }
    if (h && vr >= 0) vr += 16;
    const int vr1 = __builtin_amdgcn_mov_dpp(vr, 0xF5, 0xF, 0xF, false);   // quad_perm [1,1,3,3]: lane 2r + 1
    const bool live = act && !(rec.y & 0x80000000u);
    uint32_t t = 0;
    if (h == 0 && live) {
      const int ts = min((int)min(f, 0x3FFFFFFFu), min(cold_all.e_left_len, n));
      const int te = max(min(min(cold_all.e_right_len, n - ts), hi - 1 - max(vr, vr1)), 0);
      t = (uint32_t)ts | ((uint32_t)te << 16);
      if (t) {
        const uint32_t xs = (rec.x | ((rec.z >> 16) & 3u)) + (uint32_t)ts;
        const uint32_t xq = (uint32_t)off + (uint32_t)ts, nn = (uint32_t)(n - ts - te);
        *reinterpret_cast<v4u *>(tab(0, tbx) + 4 * idx) =
            v4u{xs & ~3u, xq & ~3u, nn | ((xs & 3u) << 16) | ((xq & 3u) << 20), t};
      }
      if (A.trim) A.trim[ubase + (size_t)idx] = t;
    }
    return t;
  };

  // PEU: group g = step g of both mates
  auto load_group_pe = [&](int tbx, int ntx, int g, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < NM; ++m) gather_at(m, tbx, step_off(g, ntx), grp[slot][m]);
  };

  // byte masks of the lane's words for the positions < p0 + c (c clamped to [0, 4 NW])
  auto mask_row = [&](int c, uint32_t (&mk)[NW]) __attribute__((always_inline)) {
    c = min(max(c, 0), 4 * NW);
    if (NW == 4) {
      const v4u t = *reinterpret_cast<const v4u *>(mtab + 4 * c);
#pragma unroll
      for (int w = 0; w < NW; ++w) mk[w] = t[w & 3];
    } else {
      const v2u t = *reinterpret_cast<const v2u *>(mtab + 2 * c);
#pragma unroll
      for (int w = 0; w < NW; ++w) mk[w] = t[w & 1];
    }
  };

  // a step's per-lane values kept between its sums and its accumulation (PF)
  struct StepVals {
    uint32_t cd[NW], qm[NW], cg[NW];
    uint32_t bad;
  };
  // one step: per-lane partial (biased quality | G+C << 18); adds (SUB = false)
  // or removes (SUB = true) the lane's positions from mate m's counters
  // (count = false: sums only, the values left in sv); NX: x2 = N |
  // out-of-range << 16; LR: x3 = left | right window sums
  // (trim, ST only: the read's ts | te << 16 -- its bytes start ts later and
  // it counts n - ts - te of them)
  auto account = [&](auto mtag, const TriPending<NW> &pd, bool count, auto sub_tag, uint32_t &x2,
                     uint32_t &x3, StepVals &sv, uint32_t trim = 0u) __attribute__((always_inline)) -> uint32_t {
    constexpr int m = decltype(mtag)::value;
    constexpr bool SUB = decltype(sub_tag)::value != 0, UNDO = decltype(sub_tag)::value == 2;
    uint32_t sw[NW], qw[NW];
    const uint32_t als = (pd.n >> 16) & 3u, alq = (pd.n >> 20) & 3u;
    int nlen = (int)(pd.n & 0xFFFFu);
    const uint32_t ts = ST ? trim & 0xFFFFu : 0u;
    // (no clamp: te <= n - ts for a read, and a lane without one masks all
    // its bytes whatever the count -- mask_row clamps)
    if (ST) nlen -= (int)ts + (int)(trim >> 16);
    if (ST && __builtin_expect(__ballot(ts != 0u) != 0, 1)) {
      // the lane's bytes start al + ts bytes into its raw words (the rest from
      // lane + 1's): every lane's raw words go to the wave's LDS buffer and
      // come back from that byte offset -- as cheap in VALU as the DPP realign
      // (register shuffles by a per-lane whole-dword count cost 44 VALU per
      // step and were needed in most steps)
      auto via_lds = [&](uint32_t *buf, const uint32_t (&r)[NW], uint32_t S, uint32_t (&out)[NW])
                         __attribute__((always_inline)) {
        // (the memory clobbers: lane + 1's words are written by ANOTHER lane, so
        // hipcc, reasoning per lane, would hoist the read of them above the
        // write -- or sink a read below the next step's write; LDS itself runs
        // a wave's operations in order)
        *reinterpret_cast<v4u *>(buf + 4 * lane) = v4u{r[0], r[1], r[2], r[3]};
        asm volatile("" ::: "memory");
        const uint32_t *src = buf + 4 * lane + (S >> 2);
        uint32_t d[NW + 1];
#pragma unroll
        for (int k = 0; k <= NW; ++k) d[k] = src[k];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int w = 0; w < NW; ++w) out[w] = __builtin_amdgcn_alignbyte(d[w + 1], d[w], S & 3u);
      };
      via_lds(stbuf(0), pd.s, als + ts, sw);
      via_lds(stbuf(1), pd.q, alq + ts, qw);
    } else {   // realign: word w = bytes [al, al+4) of raw words w, w+1 (the last from lane+1)
      const uint32_t ns = next_lane0(pd.s[0]), nq = next_lane0(pd.q[0]);
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        sw[w] = __builtin_amdgcn_alignbyte(w + 1 < NW ? pd.s[(w + 1) % NW] : ns, pd.s[w], als);
        qw[w] = __builtin_amdgcn_alignbyte(w + 1 < NW ? pd.q[(w + 1) % NW] : nq, pd.q[w], alq);
      }
    }
    uint32_t mk[NW];
    mask_row(nlen - p0, mk);
    uint32_t qm[NW], cd[NW];
    uint32_t bad = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      qm[w] = __builtin_amdgcn_bitop3_b32(qw[w], kQFlip, mk[w], 0x28);   // (qw ^ 0x80..) & mk: biased quality bytes
      cd[w] = tri_codes(sw[w], mk[w], bad);
    }
    if (__builtin_expect(bad != 0, 0)) {
      const uint32_t sign = SUB ? 0xFFFFFFFFu : 1u;
#pragma unroll
      for (int w = 0; w < NW; ++w) cd[w] = tri_fix(sw[w], mk[w], cd[w], other(m), count ? lp : 0, p0 + 4 * w, sign);
    }
    uint32_t cg[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) cg[w] = __builtin_amdgcn_perm(kCGHi, kCGLo, cd[w]);
    sv.bad = bad;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      sv.cd[w] = cd[w];
      sv.qm[w] = qm[w];
      sv.cg[w] = cg[w];
    }
    if (count) {
      TriAcc<NW> &ac = acc[m];
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const uint32_t at = __builtin_amdgcn_perm(kATHi, kATLo, cd[w]);
        const uint32_t h = __builtin_amdgcn_perm(0u, qm[w], 0x0C030C01u);   // bytes 1, 3
        if (UNDO) {   // the same values this step added: no nibble can underflow
          ac.n4[w][0] -= cg[w];
          ac.n4[w][1] -= at;
          ac.q02[w] -= qm[w] & 0x00FF00FFu;
          ac.q13[w] -= h;
        } else if (SUB) {
          ac.c8[w][1] -= cg[w] & 0x0F0F0F0Fu;
          ac.c8[w][2] -= (cg[w] >> 4) & 0x0F0F0F0Fu;
          ac.c8[w][0] -= at & 0x0F0F0F0Fu;
          ac.c8[w][3] -= (at >> 4) & 0x0F0F0F0Fu;
          ac.q02[w] -= qm[w] & 0x00FF00FFu;
          ac.q13[w] -= h;
        } else {
          ac.n4[w][0] += cg[w];
          ac.n4[w][1] += at;
          ac.q02[w] += qm[w] & 0x00FF00FFu;
          ac.q13[w] += h;
        }
      }
    }
    uint32_t gc = 0, qs = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      gc += (uint32_t)__builtin_popcount(cg[w]);
      qs = __builtin_amdgcn_sad_u8(qm[w], 0u, qs);
    }
    if (NX && !SUB) {   // N | out-of-range << 16 over the lane's valid bytes (as engine_kernel)
      // Round 5: one uniform branch per count, not five per word (the flags
      // of the range's shape cost c4_noor 4x C4's branches and 1.6x its VALU):
      // N bytes by the SWAR zero test folded into one v_bitop3 (~t & ~v & m80);
      // out of range = valid and not (>= lo and not >= hi) from the raw bytes
      // with the TrimSide constants (a missing bound or an empty range is in
      // the constants), one v_bitop3 per bound and one for the combine
      uint32_t m80[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) m80[w] = mk[w] & 0x80808080u;
      uint32_t nn = 0, oo = 0;
      if (x_n) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const uint32_t v = sw[w] ^ 0x4E4E4E4Eu, t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
          nn += (uint32_t)__builtin_popcount(__builtin_amdgcn_bitop3_b32(t, v, m80[w], 0x02));
        }
      }
      if (x_o) {
        if (x_hin) {
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const uint32_t ge_lo = __builtin_amdgcn_bitop3_b32(qw[w], xr.lq, (qw[w] | kQFlip) - xr.l7, 0x8E);
            oo += (uint32_t)__builtin_popcount(__builtin_amdgcn_bitop3_b32(ge_lo, m80[w], 0u, 0x04));   // m80 & ~ge_lo
          }
        } else {
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const uint32_t wh = qw[w] | kQFlip;
            const uint32_t ge_lo = __builtin_amdgcn_bitop3_b32(qw[w], xr.lq, wh - xr.l7, 0x8E);
            const uint32_t ge_hi = __builtin_amdgcn_bitop3_b32(qw[w], xr.hq, wh - xr.h7, 0x8E);
            oo += (uint32_t)__builtin_popcount(__builtin_amdgcn_bitop3_b32(ge_lo, ge_hi, m80[w], 0x8A));   // m80 & (~ge_lo | ge_hi)
          }
        }
      }
      x2 = nn | (oo << 16);
    }
    if (LR && !SUB) {   // window sums: positions < min(left, n) and >= n - min(right, n)
      const int n = (int)(pd.n & 0xFFFFu);
      uint32_t sl = 0, sr = 0;
      if (w_ll > 0) {   // (uniform: scalar branches)
        uint32_t ml[NW];
        mask_row(min(w_ll, n) - p0, ml);
#pragma unroll
        for (int w = 0; w < NW; ++w) sl = __builtin_amdgcn_sad_u8(qm[w] & ml[w], 0u, sl);
      }
      if (w_rl > 0) {
        uint32_t mr[NW];
        mask_row(n - min(w_rl, n) - p0, mr);
#pragma unroll
        for (int w = 0; w < NW; ++w)
          sr = __builtin_amdgcn_sad_u8(__builtin_amdgcn_bitop3_b32(qm[w], mr[w], 0u, 0x30), 0u, sr);   // qm & ~mr
      }
      x3 = sl | (sr << 16);
    }
    return qs + (gc << 18);
  };

  // PF: the accumulation of a step whose values account() left in sv
  auto account_add = [&](auto mtag, const StepVals &sv) __attribute__((always_inline)) {
    TriAcc<NW> &ac = acc[decltype(mtag)::value];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      ac.n4[w][0] += sv.cg[w];
      ac.n4[w][1] += __builtin_amdgcn_perm(kATHi, kATLo, sv.cd[w]);
      ac.q02[w] += sv.qm[w] & 0x00FF00FFu;
      ac.q13[w] += __builtin_amdgcn_perm(0u, sv.qm[w], 0x0C030C01u);   // bytes 1, 3
    }
  };

  uint32_t len[NM], lenn[NM];
  uint32_t tw[NM], twn[NM];   // EDIT: trim words of the lane's read (pair)
  uint64_t dm = 0, dmn = 0;   // deferred lanes of the current / next unit
  int tb = 0;   // read table of the current unit
  int32_t ia[NM], ie[NM];   // offsets of the unit after the next one to be described
  Unit cur = it.next(), nxt = Unit{-1, 0, 0};
  for (int m = 0; m < NM; ++m) len[m] = lenn[m] = tw[m] = twn[m] = 0;
  // TDMA: unit U's trim windows (lane j: read j's first 16 quality bytes and
  // the 32 ending at its end, as trim_issue) into the wave's DMA rows, issued
  // at the top of the unit before it, so they land while that unit streams
  // (the offsets ia / ie of U were fetched a unit ahead).  Deferred and absent
  // reads load from past the descriptor's range: no traffic.
  auto dma_windows = [&](const Unit &U) __attribute__((always_inline)) {
    if (lane >= kBlock) return;
    const bool on = lane < U.nr;
    bool dfr = false;
#pragma unroll
    for (int m = 0; m < NM; ++m) dfr = dfr || (ie[m] - ia[m] > dlim);
    const bool live = on && !dfr;
    const uint32_t sb = (uint32_t)(uintptr_t)scratch;   // (the rows sit at constant offsets from it)
    auto mate = [&](auto mtag) __attribute__((always_inline)) {
      constexpr int m = decltype(mtag)::value;
      constexpr int kRow0 = 4 * (64 + 4 + NM * kFxWords + m * 3 * kBlock * 4), kRowB = 4 * kBlock * 4;
      const int off = bq[m] + ia[m], n = ie[m] - ia[m];
      int pa = off + n - 32;
      if (pa < 0) pa = 0;
      const uint32_t kOut = 0x80000000u;
      if (cold_all.e_left_len > 0) dma16<kRow0>(rq[m], live ? (uint32_t)off : kOut, sb);
      if (cold_all.e_right_len > 0) {
        dma16<kRow0 + kRowB>(rq[m], live ? (uint32_t)pa : kOut, sb);
        dma16<kRow0 + 2 * kRowB>(rq[m], live ? (uint32_t)pa + 16u : kOut, sb);
      }
    };
    mate(MateTag<0>{});
    if (NM == 2) mate(MateTag<NM - 1>{});
  };
  auto ngroups_of = [&](int nts) __attribute__((always_inline)) { return ((nts + kU - 1) / kU + 1) & ~1; };
  if (cur.u >= 0) {
    fetch_idx(cur, ia, ie);
    load_block(cur, tb, len, tw, dm, ia, ie, false);
    nxt = it.next();
    fetch_idx(nxt, ia, ie);
    if (PEU) load_group_pe(tb, steps_of(cur, dm), 0, 0);
    else load_group(0, tb, steps_of(cur, dm), 0, 0);
  }
  constexpr uint64_t not_seg_first = not_seg_first_mask<G>();   // lanes j with j % kSegs != 0
  while (cur.u >= 0) {
    const int nr = cur.nr;
    const int nt = steps_of(cur, dm);
    // the next unit's prologue (read table, deferral mask; for edit the trims,
    // which read the quality ends).  LATE (edit): just before the next unit's
    // first loads, so the lines the trims bring in are still in L2 when that
    // unit streams them (one unit ahead they were evicted: HBM traffic 1.5x
    // the algorithmic bytes); else at the unit start, a unit ahead.
    Unit nn2 = Unit{-1, 0, 0};
    int nnt = 0;
    // TDMA: the DMA rows are filled during this unit's last group pair
    // (issue_dma, inside its first process_pair: part of a group of work
    // before the next unit's prologue reads them; a unit earlier their lines
    // left L2 before the stream came back for them, +0.5 GB of HBM traffic
    // per C4 launch; at the pair's top hipcc's own vmcnt(0) drained it)
    const bool tdma = TDMA && trim_usual(cold_all);
    auto issue_dma = [&]() __attribute__((always_inline)) {
      if (tdma && nxt.u >= 0) dma_windows(nxt);
    };
    TrimLoads pre_tl;   // EG: the next unit's trim windows, issued a group early
    auto gather_next = [&]() __attribute__((always_inline)) {
      if (!EG || !trim_usual(cold_all)) return;
      const bool on = lane < nxt.nr;
      const bool live = on && !(ie[0] - ia[0] > dlim);
      pre_tl = trim_issue(cold_all, rq[0], live ? bq[0] + ia[0] : (int)0xC0000000, ie[0] - ia[0]);
    };
    auto describe_next = [&]() __attribute__((always_inline)) {
      // (the DMA is the youngest VMEM operation here: issued inside the pair's
      // first process_pair after its loads were waited for, or -- a wholly
      // deferred unit -- just before)
      if (tdma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      load_block(nxt, tb ^ 1, lenn, twn, dmn, ia, ie, true, EG ? &pre_tl : nullptr);
      nn2 = it.next();
      fetch_idx(nn2, ia, ie);
      nnt = steps_of(nxt, dmn);
    };
    if (!LATE) describe_next();
    if (stats && since_flush > kByteEvery - kBlock / kSegs) {   // keep every byte <= 255
#pragma unroll
      for (int m = 0; m < NM; ++m) acc[m].flush(pos_acc(m), lp, p0);
      since_flush = 0;
    }
    // an even number of groups per mate, so every mate (and unit) starts in
    // slot 0 (the padding group gathers length-0 reads)
    const int ngroups = ngroups_of(nt);

    uint32_t st_t = 0;   // ST: lane 2r: the current group pair's read r's trims
    auto run_mate = [&](auto mtag) __attribute__((always_inline)) {
      constexpr int m = decltype(mtag)::value;
      auto process_group = [&](int g, int slot) __attribute__((always_inline)) {
        // ST: the pair's trims when its first group is counted (st_t lives on
        // to the second)
        if (ST && slot == 0) {
          st_t = g * kU < nt ? st_trims(tb, g, (size_t)cur.u * kBlock) : 0u;
          __builtin_amdgcn_wave_barrier();   // (the patched records: LDS is in order per wave)
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int t = g * kU + u;
          uint32_t x2 = 0, x3 = 0;
          StepVals sv;
          // ST: this lane's read's trim, from lane 4r of its group's read r
          const uint32_t trim =
              ST ? (uint32_t)__builtin_amdgcn_ds_bpermute(8 * (kSegs * kU * slot + kSegs * u + min(seg, kSegs - 1)),
                                                          (int)st_t)
                 : 0u;
          // PF: sums first, the decision, then only passing reads are added;
          // else every read is added and failed ones are taken out in the unit epilogue
          const uint32_t x = account(MateTag<m>{}, grp[slot][u], stats && !PF, AddTag{}, x2, x3, sv, trim);
          const uint32_t P = wave_scan(x);
          // segment ends (the last lane of each segment) -> wends[kSegs t + seg], no wait needed
          if (ls == kSegW - 1 && seg < kSegs && t < nt) put_end(wends(m), t, P);
          uint32_t P2 = 0, P3 = 0;
          if (NX) {
            P2 = wave_scan(x2);
            if (ls == kSegW - 1 && seg < kSegs && t < nt) put_end(wends2(m), t, P2);
          }
          if (LR) {
            if (w_direct) {   // the segment's first lane holds the whole window sum
              if (ls == 0 && seg < kSegs && t < nt) put_end(wends3(m), t, x3);
            } else {
              P3 = wave_scan(x3);
              if (ls == kSegW - 1 && seg < kSegs && t < nt) put_end(wends3(m), t, P3);
            }
          }
          if (PF && stats) {
            bool pass = true;
            if (filter) {   // this read's totals: the segment's last inclusive prefix minus its first exclusive one
              const int sg = min(seg, kSegs - 1) * kSegW;
              auto seg_total = [&](uint32_t Pi, uint32_t xi) __attribute__((always_inline)) {
                return (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (sg + kSegW - 1), (int)Pi) -
                       (uint32_t)__builtin_amdgcn_ds_bpermute(4 * sg, (int)(Pi - xi));
              };
              const int n = (int)(grp[slot][u].n & 0xFFFFu), sraw = (int)(seg_total(P, x) & 0x3FFFFu);
              pass = n >= A.min_len && n <= A.max_len && lo_r * n <= sraw && sraw <= hi_r * n;
              if (NX) {
                const uint32_t r2 = seg_total(P2, x2);
                if (x_n && (int)(r2 & 0xFFFFu) > x_maxn) pass = false;
                if (x_o && (int)(r2 >> 16) > x_maxo) pass = false;
              }
              if (LR) {
                const uint32_t r3 = w_direct ? (uint32_t)__builtin_amdgcn_ds_bpermute(4 * sg, (int)x3) : seg_total(P3, x3);
                const int kl = min(w_ll, n), kr = min(w_rl, n);
                if (kl > 0 && !win_in((int)(r3 & 0xFFFFu), kl, w_lmin, w_lmax)) pass = false;
                if (kr > 0 && !win_in((int)(r3 >> 16), kr, w_rmin, w_rmax)) pass = false;
              }
            }
            if (__builtin_expect(__ballot(sv.bad != 0) != 0, 0)) {   // rare: non-ACGTN bytes ("other" counts)
              uint32_t d2, d3;
              StepVals d;
              if (pass) (void)account(MateTag<m>{}, grp[slot][u], true, AddTag{}, d2, d3, d);
            } else if (pass) {
              account_add(MateTag<m>{}, sv);
            }
          }
        }
      };
      // after this mate's last group: the next mate's first group, or the next unit's
      auto load_next_unit = [&](int slot) __attribute__((always_inline)) {
        if (m + 1 < NM) {
          load_group(m + 1 < NM ? m + 1 : 0, tb, nt, 0, slot);
        } else {
          if (LATE) describe_next();
          load_group(0, tb ^ 1, nnt, 0, slot);
        }
      };
      for (int g = 0; g < ngroups; g += 2) {
        const bool last = g + 2 >= ngroups;
        if (m == NM - 1 && last) issue_dma();   // (the unit's last group pair)
        if (EG && last) gather_next();
        load_group(m, tb, nt, g + 1, 1);
        process_group(g, 0);
        // PF (C2 and its N / out-of-range variants): every load waited for
        // before the next group's are issued, so a wave holds one group in
        // flight while it counts the other -- the coarse waits that round 5's
        // FLAT atomics induced by accident (ISA: a vmcnt(0) before this
        // table read), now stated: same box, 4 alternating rounds, 537 us
        // against 546 with the compiler's exact waits and 541 with the FLAT
        // ones (profiles/r06_c2_waits_ab.json); the edit, paired-end and
        // window kernels run faster with exact waits (round 5)
        if (PF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (NM == 1 && LATE) {
          // edit: ONE load site for slot 0, this unit's next group or the next
          // unit's first, behind the next unit's prologue (round 5: C4 811 ->
          // 806 us; C2, whose else-branch is a plain load, ran 1.5 % slower
          // this way and keeps the if / else)
          if (last) describe_next();
          load_group(0, last ? tb ^ 1 : tb, last ? nnt : nt, last ? 0 : g + 2, 0);
        } else if (!last) {
          load_group(m, tb, nt, g + 2, 0);
        } else {
          load_next_unit(0);
        }
        process_group(g + 1, 1);
        // nibbles hold at most 15 steps: widen after groups 0-3 and at the end
        // (a unit of at most 4 groups -- hex -- only at the end: round 6, the
        // second widen of zero nibbles was 48 VALU per unit)
        if (kMidWiden && stats && g == 2) acc[m].widen();
      }
      if (stats) acc[m].widen();
    };
    // PEU: step g of both mates added, the pair decided, a failed pair undone
    auto process_pair = [&](int g, int slot, bool dma_after) __attribute__((always_inline)) {
      constexpr int m1 = NM - 1;
      const int t = g;
      StepVals dsv;
      uint32_t d2 = 0, d3 = 0;
      const bool dec = stats && filter;
      const int sg = min(seg, kSegs - 1) * kSegW;
      auto read_ok = [&](uint32_t Pi, uint32_t xi, uint32_t ni) __attribute__((always_inline)) {
        const uint32_t tot = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (sg + kSegW - 1), (int)Pi) -
                             (uint32_t)__builtin_amdgcn_ds_bpermute(4 * sg, (int)(Pi - xi));
        const int n = (int)(ni & 0xFFFFu), sraw = (int)(tot & 0x3FFFFu);
        return n >= A.min_len && n <= A.max_len && lo_r * n <= sraw && sraw <= hi_r * n;
      };
      const uint32_t x0 = account(MateTag<0>{}, grp[slot][0], stats, AddTag{}, d2, d3, dsv);
      const uint32_t P0 = wave_scan(x0);
      if (ls == kSegW - 1 && seg < kSegs && t < nt) put_end(wends(0), t, P0);
      const bool pass0 = !dec || read_ok(P0, x0, grp[slot][0].n);   // (only a bool lives on)
      const uint32_t x1 = account(MateTag<m1>{}, grp[slot][m1], stats, AddTag{}, d2, d3, dsv);
      // TDMA: the next unit's windows, issued once this group's loads have been
      // waited for: the DMA is invisible to hipCC's wait counts, so a
      // compiler wait for any load after it (the loop top's, or this group's)
      // would drain it on the spot (vmcnt counts in order)
      if (dma_after) issue_dma();
      const uint32_t P1 = wave_scan(x1);
      if (ls == kSegW - 1 && seg < kSegs && t < nt) put_end(wends(m1), t, P1);
      if (!dec) return;
      const bool pass = pass0 && read_ok(P1, x1, grp[slot][m1].n);
      if (__builtin_expect(__ballot(!pass) != 0, 0) && !pass) {   // (lanes of a failed pair only)
        (void)account(MateTag<0>{}, grp[slot][0], true, UndoTag{}, d2, d3, dsv);
        (void)account(MateTag<m1>{}, grp[slot][m1], true, UndoTag{}, d2, d3, dsv);
      }
    };
    if (PEU && ngroups > 0) {
      const int ng = (nt + 1) & ~1;   // one step per group, an even count
      for (int g = 0; g < ng; g += 2) {
        load_group_pe(tb, nt, g + 1, 1);
        process_pair(g, 0, g + 2 >= ng);   // (the unit's last group pair: the DMA inside)
        const bool last = g + 2 >= ng;   // (one load site for slot 0, as in run_mate)
        if (LATE && last) describe_next();
        load_group_pe(last ? tb ^ 1 : tb, last ? nnt : nt, last ? 0 : g + 2, 0);
        process_pair(g + 1, 1, false);
        if (stats && ((g + 2) & 7) == 0 && g + 2 < ng)   // nibbles hold at most 15 steps (the end widens too)
          for (int m = 0; m < NM; ++m) acc[m].widen();
      }
      if (stats)
        for (int m = 0; m < NM; ++m) acc[m].widen();
    } else if (ngroups > 0) {
      run_mate(MateTag<0>{});
      if (NM == 2) run_mate(MateTag<NM - 1>{});
    } else if (PEU) {
      issue_dma();
      if (LATE) describe_next();
      load_group_pe(tb ^ 1, nnt, 0, 0);   // a wholly deferred unit: straight to the next
    } else {
      issue_dma();
      gather_next();
      if (LATE) describe_next();
      load_group(0, tb ^ 1, nnt, 0, 0);   // a wholly deferred unit: straight to the next
    }
    since_flush += nt;

    // ---- unit epilogue (lane j = read / pair j) ----------------------------
    // (a deferred read still has a segment end: its neighbour's sum is a difference of ends)
    const bool inb = lane < nr;
    const bool valid = inb && !((dm >> lane) & 1ull);
    const int my_read = FOLLOW ? (int)tab(0, tb)[4 * lane + 3] : cur.u * ublock + lane;
    if (TABLEN) {   // this unit's lengths and trim words from its read table
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const v2u r = *reinterpret_cast<const v2u *>(tab(m, tb) + 4 * lane + 2);
        len[m] = r.x & 0xFFFFu;
        tw[m] = EDIT ? r.y : 0u;
      }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t r1[NM];
    bool pass = valid;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      // per-read sums: difference of consecutive segment ends within a step
      // (wends[kSegs t + k] = inclusive wave prefix at the end of segment k)
      const uint32_t ends = inb ? wends(m)[lane] : 0u;
      const uint32_t prev = __builtin_amdgcn_mov_dpp(ends, 0x138, 0xF, 0xF, true);   // lane j-1
      r1[m] = ends - (((not_seg_first >> lane) & 1u) ? prev : 0u);
      const int n = (int)len[m];
      const int sraw = (int)(r1[m] & 0x3FFFFu);
      if (filter)
        pass = pass && n >= A.min_len && n <= A.max_len && lo_r * n <= sraw && sraw <= hi_r * n;
      if (NX && filter) {
        const uint32_t e2 = inb ? wends2(m)[lane] : 0u;
        const uint32_t p2 = __builtin_amdgcn_mov_dpp(e2, 0x138, 0xF, 0xF, true);   // lane j-1
        const uint32_t r2 = e2 - (((not_seg_first >> lane) & 1u) ? p2 : 0u);
        if (x_n && (int)(r2 & 0xFFFFu) > x_maxn) pass = false;
        if (x_o && (int)(r2 >> 16) > x_maxo) pass = false;
      }
      if (LR && filter) {   // min*k <= S - phred*k <= max*k over each window (k = min(len, n))
        const uint32_t e3 = inb ? wends3(m)[lane] : 0u;
        const uint32_t p3 = __builtin_amdgcn_mov_dpp(e3, 0x138, 0xF, 0xF, true);   // lane j-1
        const uint32_t r3 = w_direct ? e3 : e3 - (((not_seg_first >> lane) & 1u) ? p3 : 0u);
        const int kl = min(w_ll, n), kr = min(w_rl, n);
        if (kl > 0 && !win_in((int)(r3 & 0xFFFFu), kl, w_lmin, w_lmax)) pass = false;
        if (kr > 0 && !win_in((int)(r3 >> 16), kr, w_rmin, w_rmax)) pass = false;
      }
    }
    if (valid && A.mask) A.mask[my_read] = (uint8_t)pass;
    const uint64_t failed = __ballot(valid && !pass);
    const uint32_t npass = (uint32_t)__builtin_popcountll(__ballot(pass));
    const uint32_t nvalid = (uint32_t)(nr - __builtin_popcountll(dm));
    cnt_in += nvalid;
    cnt_pass += npass;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int n = (int)len[m];
      if (EDIT) cnt_ed[m] += (uint32_t)__builtin_popcountll(__ballot(valid && tw[m] != 0u));
      if (stats) {
        if (pass) {   // (reads longer than lmax were deferred: every pass merges)
          const uint32_t gc = r1[m] >> 18, wn = (uint32_t)n, s = r1[m] & 0x3FFFFu;
          uint32_t *h = hist(m);
          atomicAdd(&h[wn], 1u);
          if (wn > 0) {
            uint32_t bin;
            uint64_t fx;
            const uint32_t rc = rtab[wn], one1 = wn == 1u ? 1u : 0u;
            meanq_terms_rc(s, wn, rc, one1, bin, fx);
            atomicAdd(&h[lp + 1 + bin], 1u);
            atomicAdd(&h[lp + 1 + HPGQ_MEANQ_BINS + div_len(100 * gc, rc, one1)], 1u);
            atomicAdd(&fxs(m)[lane & (kFxSlots - 1)], (unsigned long long)fx);   // (no return: ds_add_u64)
          }
        }
      }
    }
    if (!PF && !PEU && stats && failed) {
      // take the failed reads (pairs: both mates) back out.  A read must leave
      // through the segment it entered by (its lanes' byte counters hold it;
      // another segment's could borrow), so the failed reads of each segment
      // class (j % kSegs) are listed by rank and step k takes the k-th of every
      // class at once: max-per-class steps instead of one per step holding a
      // failure.  The segment ends are consumed: mate 0's wends holds the list.
      uint32_t *flist = wends(0);
      constexpr uint64_t cls0 = ~not_seg_first;   // lanes j with j % kSegs == 0
      const int cls = lane % kSegs;
      const int rank = __builtin_popcountll(failed & (cls0 << cls) & lanes_below(lane));
      __builtin_amdgcn_wave_barrier();
      if (valid && !pass) flist[min(rank * kSegs + cls, 63)] = (uint32_t)lane;
      __builtin_amdgcn_wave_barrier();
      int nsub = 0, mycnt = 0;
#pragma unroll
      for (int c = 0; c < kSegs; ++c) {
        const int n = __builtin_popcountll(failed & (cls0 << c));
        nsub = max(nsub, n);
        if (c == seg) mycnt = n;
      }
      uint32_t sub_x2 = 0, sub_x3 = 0;   // (unused: failed reads leave the counters only)
      StepVals sub_sv;
      for (int k = 0; k < nsub; ++k) {
        const int src = seg < kSegs && k < mycnt ? (int)flist[min(k * kSegs + seg, 63)] : 63;
        TriPending<NW> pd;
        gather(0, tb, src, pd);
        (void)account(MateTag<0>{}, pd, true, SubTag{}, sub_x2, sub_x3, sub_sv);
        if (NM == 2) {
          gather(NM - 1, tb, src, pd);
          (void)account(MateTag<NM - 1>{}, pd, true, SubTag{}, sub_x2, sub_x3, sub_sv);
        }
      }
    }
    if (!TABLEN) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        len[m] = lenn[m];
        tw[m] = twn[m];
      }
    }
    dm = dmn;
    tb ^= 1;
    cur = nxt;
    nxt = nn2;
  }

  // ---- workgroup epilogue ---------------------------------------------------
  if (lane == 0 && ndefer) atomicAdd(A.defer_count, ndefer);
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    acc[m].widen();
    acc[m].flush(pos_acc(m), lp, p0);
    const uint64_t tot = wave_sum64(lane < kFxSlots ? (uint64_t)fxs(m)[lane] : 0ull);   // (LDS: in order per wave)
    if (lane == 0) {
      unsigned long long *s = sc(m);
      if (cnt_in) atomicAdd(&s[HPGQ_S_NUM_INPUT], (unsigned long long)cnt_in);
      if (cnt_pass) atomicAdd(&s[HPGQ_S_NUM_PASSED], (unsigned long long)cnt_pass);
      if (cnt_in - cnt_pass) atomicAdd(&s[HPGQ_S_NUM_FAILED], (unsigned long long)(cnt_in - cnt_pass));
      if (cnt_ed[m]) atomicAdd(&s[HPGQ_S_NUM_EDITED], (unsigned long long)cnt_ed[m]);
      if (stats && cnt_pass) atomicAdd(&s[HPGQ_S_NUM_STATS], (unsigned long long)cnt_pass);
      if (tot) atomicAdd(&s[HPGQ_S_ACC_MEANQ_FX16], (unsigned long long)tot);
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < NM; ++m) pos_fix<true>(pos_acc(m), hist(m), lp, tid, mtab);   // (mtab is free now)
#pragma unroll
  for (int m = 0; m < NM; ++m)
    add_partials_lp(A.counters + (size_t)m * A.clen, sc(m), hist(m), pos_acc(m), lmax, lp, tid, kWG);
}

template <int MINW, int NM, bool EDIT, int G, bool FOLLOW>
__global__ void __launch_bounds__(kWG, MINW) engine_tri_kernel(EngineArgs A) {
  tri_body<MINW, NM, EDIT, G, 0, FOLLOW>(A);
}

// the segmented kernel with extra filter scans (XM: X_NOOR | X_LR)
template <int MINW, int NM, int G, bool FOLLOW, int XM, bool EDIT>
__global__ void __launch_bounds__(kWG, MINW) engine_tri_x_kernel(EngineArgs A) {
  tri_body<MINW, NM, EDIT, G, XM, FOLLOW>(A);
}

// kernel selection (one translation unit per geometry, hpgq_engine_geo.hip):
// the instance for (NM, edit, xm, follow) or nullptr; name gets its signature
struct SegChoice {
  const void *fn;
  int min_waves;
};
SegChoice seg_kernel_tri(int nm, bool edit, int xm, bool follow, char *name, size_t cap);
SegChoice seg_kernel_hex(int nm, bool edit, int xm, bool follow, char *name, size_t cap);
SegChoice seg_kernel_wide(int nm, bool edit, int xm, bool follow, char *name, size_t cap);

}  // namespace hpgq
