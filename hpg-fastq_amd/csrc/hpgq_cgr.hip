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
#include <rccl/rccl.h>
#include <climits>
#include <cstring>
#include "hpgq_common.h"

#include <algorithm>
#include <vector>

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

// Byte classes (exact byte match, as the reference's switch, :197-233), kept
// in a 256-entry LDS table: bit0 moves f (A/C/G/T), bit1 x half (A/T), bit2
// y half (G/T), bit3 'N'.  Every other byte — and the zero bytes the loads
// mask in past a read's end — is class 0, an exact no-op of `step`.
constexpr uint32_t F_MV = 1, F_BX = 2, F_BY = 4, F_N = 8;
// the same classes in registers, 4 bytes at a time: code = byte & 7 is
// one-to-one on A(1) C(3) T(4) N(6) G(7); v_perm_b32 looks up the class and
// the expected byte per code, and bytes that are not exactly that byte
// (lowercase, IUPAC, anything else) get class 0
constexpr uint32_t kClsLo = 0x01000300u;   // codes 0..3: -, A, -, C
constexpr uint32_t kClsHi = 0x05080007u;   // codes 4..7: T, -, N, G
constexpr uint32_t kExLo = 0x43004101u;    // expected byte per code (code 0: 0x01 never matches)
constexpr uint32_t kExHi = 0x474E0054u;

__device__ __forceinline__ uint32_t classes4(uint32_t w) {
  const uint32_t code = w & 0x07070707u;
  const uint32_t d = w ^ __builtin_amdgcn_perm(kExHi, kExLo, code);
  const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;   // inexact bytes
  return __builtin_amdgcn_perm(kClsHi, kClsLo, code) & ~((nz >> 7) * 0xFFu);
}

__device__ __forceinline__ void fill_classes(uint8_t *cls, int tid, int nthreads) {
  for (int i = tid; i < 256; i += nthreads) {
    uint32_t f = 0;
    if (i == 'A') f = F_MV | F_BX;
    if (i == 'C') f = F_MV;
    if (i == 'G') f = F_MV | F_BY;
    if (i == 'T') f = F_MV | F_BX | F_BY;
    if (i == 'N') f = F_N;
    cls[i] = (uint8_t)f;
  }
}

// One base of chaos_game_fill_tables (:197-260), branch-free.  FULL adds the
// word to the tables (sign = 1 adds, 0xFFFFFFFF takes it back out); !FULL only
// advances f, the word counter and the boundary clamp (context replay).
//
// f moves as the reference's
//     A/T (axis bit 1): f = f + (dim - f) * 0.5       C/G (bit 0): f = f * 0.5
// computed as  D = fma(f, S, C);  f = fma(D, 0.5, f)  with S = -1 (moving
// base) / 0, C = dim (bit 1) / 0: D = round(dim - f) exactly as the
// subtraction, and D * 0.5 is exact, so fma(D, 0.5, f) rounds f + (dim - f) *
// 0.5 once as the reference does; bit 0 gives fma(-f, 0.5, f) = f / 2 exactly
// (= f * 0.5); a non-moving byte gives fma(0, 0.5, f) = f.  Two FP64 ops per
// axis and no selects.
//
// UNCOND (LDS tables, sign = 1): one 64-bit LDS add per base into an
// interleaved table — count in the low half (<= 2^32 words per workgroup
// launch, so it never carries), the raw quality accumulator in the high half
// (mod 2^32; the flush takes count * sub back out, so the table holds
// sum(acc - sub) as the reference's unsigned int does) — a base that
// completes no word adds to the spare cell dim*dim instead.
//
// CLAMP: the boundary clamp (:241-251) can fire in this step.  f reaches dim
// only after ~50 A/T (x) or G/T (y) in a row; run_chunk proves per 8 bases
// that it cannot (see kHot) and runs the clamp-free steps.
// f's move for byte class fl (see above)
template <int K>
__device__ __forceinline__ void move(uint32_t fl, State &st) {
  constexpr uint32_t kDimHi = (uint32_t)(1023 + K) << 20;   // high word of (double)dim
  const uint32_t mvm = (uint32_t)((int32_t)(fl << 31) >> 31);
  const uint32_t bxm = (uint32_t)((int32_t)(fl << 30) >> 31);
  const uint32_t bym = (uint32_t)((int32_t)(fl << 29) >> 31);
  const double S = __hiloint2double((int)(mvm & 0xBFF00000u), 0);
  const double Cx = __hiloint2double((int)(bxm & kDimHi), 0);
  const double Cy = __hiloint2double((int)(bym & kDimHi), 0);
  st.fx = __builtin_fma(__builtin_fma(st.fx, S, Cx), 0.5, st.fx);
  st.fy = __builtin_fma(__builtin_fma(st.fy, S, Cy), 0.5, st.fy);
}

template <int K, bool FULL, bool UNCOND, bool CLAMP>
__device__ __forceinline__ void step(uint32_t fl, uint32_t qb, uint32_t qold, State &st, int &cnt,
                                     uint32_t &acc, uint32_t *ts, uint32_t *tq, uint32_t sign,
                                     uint32_t sub, uint32_t &words) {
  constexpr int dim = 1 << K;
  const uint32_t mvm = (uint32_t)((int32_t)(fl << 31) >> 31);   // all ones when moving
  const uint32_t nm = (uint32_t)((int32_t)(fl << 28) >> 31);    // 'N'
  move<K>(fl, st);
  cnt = (int)(((uint32_t)cnt + (fl & F_MV)) & ~nm);
  if (FULL) acc = (acc + (qb & mvm)) & ~nm;
  const bool word = cnt == K;
  int cx = (int)st.fx, cy = (int)st.fy;
  if (CLAMP) {
    if (word && cx == dim) {
      cx = dim - 1;
      st.fx = st.fx - kEps;
    }
    if (word && cy == dim) {
      cy = dim - 1;
      st.fy = st.fy - kEps;
    }
  }
  cnt = word ? K - 1 : cnt;
  if (FULL) {
    if (UNCOND) {
      const uint32_t cell = word ? (uint32_t)(cx * dim + cy) : (uint32_t)(dim * dim);
      const uint64_t inc = ((uint64_t)acc << 32) | 1u;
      atomicAdd(reinterpret_cast<unsigned long long *>(ts) + cell, (unsigned long long)inc);
    } else if (word) {
      const int cell = cx * dim + cy;
      atomicAdd(&ts[cell], sign);
      atomicAdd(&tq[cell], sign * (acc - sub));
    }
    if (!UNCOND) words += word ? 1u : 0u;   // LDS tables: the flush sums the counts
    acc -= word ? qold : 0u;   // quality[quality_position - word_size] (:259), raw position
  }
}

// word counter at byte p of a read: moving bases since the last reset
// (read start or 'N'), capped at K-1 (a completed word drops it to K-1).
// The 16 bytes before p are scanned in registers; only when they hold fewer
// than K-1 A/C/G/T and no 'N' (other bytes in between) does it walk further.
template <int K>
__device__ int count_before(const Args &A, const Src &S, const uint8_t *cls, int a, int p) {
  const int lo = p >= 16 ? p - 16 : 0;
  const v2u w0 = __builtin_amdgcn_raw_buffer_load_b64(S.rs, (uint32_t)(a + lo), 0, 0);
  const v2u w1 = __builtin_amdgcn_raw_buffer_load_b64(S.rs, (uint32_t)(a + lo + 8), 0, 0);
  const v2u c0 = {classes4(w0.x), classes4(w0.y)}, c1 = {classes4(w1.x), classes4(w1.y)};
  int m = 0;
  bool alive = true;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    const int pos = lo + i;
    const uint32_t f = i >= 8 ? byte_of(c1, i - 8) : byte_of(c0, i);
    const bool in = pos < p;
    alive = alive && !(in && (f & F_N));
    m += (alive && in && (f & F_MV)) ? 1 : 0;
  }
  if (m >= K - 1) return K - 1;
  if (!alive || lo == 0) return m;
  for (int i = lo - 1; i >= 0 && m < K - 1; --i) {   // rare: other bytes in the window
    const uint32_t f = cls[(uint8_t)A.seq[a + i]];
    if (f & F_N) break;
    if (f & F_MV) ++m;
  }
  return m;
}

// A step moves f at most halfway towards dim (d' >= d/2 - ulp/2 for d = dim
// - f, ulp = dim * 2^-53; 'C'/'G' and the kEps nudge leave d >= 1e-5), so
// from d >= dim * 2^-30 at a chunk start f stays below dim for 8 steps and
// the clamp cannot fire: kHot is the wave-uniform test for the CLAMP steps.
template <int K>
__device__ __forceinline__ bool hot(const State &st) {
  constexpr double kHot = (double)(1 << K) * (1.0 - 0x1p-30);
  return __ballot(st.fx > kHot || st.fy > kHot) != 0ull;
}

__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Quality bytes around an 8-byte chunk at c: m = [c-8, c+8) and, for K > 9
// (quality[qpos - K] up to 11 bytes back), lo = [c-16, c-8); cut from the
// block registers (run_block) rather than rotated through registers: a
// loop-carried copy of the newest load makes the loop head wait for it.
typedef unsigned v4u __attribute__((ext_vector_type(4)));
struct QWin {
  v4u m;
  v2u lo;
};

template <int K>
__device__ __forceinline__ uint32_t qbyte(const QWin &q, int o) {   // o in [-16, 8)
  if (o >= -8) {
    const int i = o + 8;
    return (uint32_t)(int32_t)(int8_t)((q.m[i >> 2] >> (8 * (i & 3))) & 0xFFu);
  }
  return sbyte_of(q.lo, o + 16);
}

// One 8-byte chunk of a read (classes cl, qualities q).
template <int K, bool FULL, bool UNCOND, bool CLAMP>
__device__ __forceinline__ void run_chunk_steps(v2u cl, const QWin &q, State &st, int &cnt,
                                                uint32_t &acc, uint32_t *ts, uint32_t *tq,
                                                uint32_t sign, uint32_t sub, uint32_t &words) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    // quality[j + 1 - K], raw position (the reference's quality_position - word_size)
    const uint32_t qold = FULL ? qbyte<K>(q, u + 1 - K) : 0u;
    step<K, FULL, UNCOND, CLAMP>(byte_of(cl, u), FULL ? qbyte<K>(q, u) : 0u, qold, st, cnt, acc,
                                 ts, tq, sign, sub, words);
  }
}

template <int K, bool FULL, bool UNCOND>
__device__ __forceinline__ void run_chunk(v2u sv, const QWin &q, int left, State &st, int &cnt,
                                          uint32_t &acc, uint32_t *ts, uint32_t *tq, uint32_t sign,
                                          uint32_t sub, uint32_t &words) {
  // bytes past the read end -> 0 (class 0: no-op); left <= 0 masks all
  const uint64_t m = left >= 8 ? ~0ull : ((1ull << (8 * max(left, 0))) - 1);
  sv.x &= (uint32_t)m;
  sv.y &= (uint32_t)(m >> 32);
  const v2u cl = {classes4(sv.x), classes4(sv.y)};
  if (__builtin_expect(hot<K>(st), 0))
    run_chunk_steps<K, FULL, UNCOND, true>(cl, q, st, cnt, acc, ts, tq, sign, sub, words);
  else
    run_chunk_steps<K, FULL, UNCOND, false>(cl, q, st, cnt, acc, ts, tq, sign, sub, words);
}

// Run read [a, a+n) from byte p0 (word counter cnt0) with state st, 64 bytes
// at a time: a lane's block is seq [c, c+64) and quality [c-16, c+64) in
// 16-byte loads (the first quality piece [c-8, c) for K <= 9), two blocks in
// flight.  Taking a whole block per visit keeps
// the lanes' lines from being evicted between 8-byte visits (1024 lanes per
// CU x 2 streams of 128-byte lines overflow the L2) and quarters the
// address work per byte.  The [c-16, c) piece is a load of its own: before
// offset 0 it reads 0, and it then covers only bytes before the read.
struct Blk {
  v4u s[4];
  v4u q[5];
};

template <int K, bool FULL, bool UNCOND>
__device__ __forceinline__ void run_block(const Blk &B, int left, State &st, int &cnt,
                                          uint32_t &acc, uint32_t *ts, uint32_t *tq, uint32_t sign,
                                          uint32_t sub, uint32_t &words) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (__builtin_expect(__ballot(left - 8 * i > 0) == 0ull, 0)) return;   // the wave is done
    const v2u sv = {B.s[i >> 1][2 * (i & 1)], B.s[i >> 1][2 * (i & 1) + 1]};
    QWin q;   // dwords 2i+2 .. 2i+5 of quality [c-16, c+64): [c+8i-8, c+8i+8)
    const int d = 2 * i + 2;
    q.m = v4u{B.q[d >> 2][d & 3], B.q[(d + 1) >> 2][(d + 1) & 3], B.q[(d + 2) >> 2][(d + 2) & 3],
              B.q[(d + 3) >> 2][(d + 3) & 3]};
    q.lo = v2u{B.q[(d - 2) >> 2][(d - 2) & 3], B.q[(d - 1) >> 2][(d - 1) & 3]};
    run_chunk<K, FULL, UNCOND>(sv, q, left - 8 * i, st, cnt, acc, ts, tq, sign, sub, words);
  }
}

template <int K, bool FULL, bool UNCOND>
__device__ void run_read(const Args &A, const Src &S, int a, int n, int p0, int cnt0, State &st,
                         uint32_t *ts, uint32_t *tq, uint32_t sign, uint32_t &words) {
  const uint32_t sub = A.base_quality * (uint32_t)K;
  int cnt = cnt0;
  uint32_t acc = 0;
  auto load = [&](int c) {
    Blk B;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      B.s[i] = __builtin_amdgcn_raw_buffer_load_b128(S.rs, (uint32_t)(a + c + 16 * i), 0, 0);
#pragma unroll
    for (int i = 1; i < 5; ++i)
      B.q[i] = FULL ? __builtin_amdgcn_raw_buffer_load_b128(S.rq, (uint32_t)(a + c - 16 + 16 * i), 0, 0)
                    : v4u{0u, 0u, 0u, 0u};
    // [c-16, c-8) only for K > 9: a loaded dword that is never read is still
    // written by its load, and reusing its register makes the wave wait for it
    if (FULL && K > 9) {
      B.q[0] = __builtin_amdgcn_raw_buffer_load_b128(S.rq, (uint32_t)(a + c - 16), 0, 0);
    } else if (FULL) {
      const v2u h = __builtin_amdgcn_raw_buffer_load_b64(S.rq, (uint32_t)(a + c - 8), 0, 0);
      B.q[0] = v4u{0u, 0u, h.x, h.y};
    } else {
      B.q[0] = v4u{0u, 0u, 0u, 0u};
    }
    return B;
  };
  Blk B0 = load(p0), B1 = load(opaque(p0 + 64));
  for (int c = p0; c < n; c += 128) {
    run_block<K, FULL, UNCOND>(B0, n - c, st, cnt, acc, ts, tq, sign, sub, words);
    B0 = load(c + 128);
    run_block<K, FULL, UNCOND>(B1, n - c - 64, st, cnt, acc, ts, tq, sign, sub, words);
    B1 = load(c + 192);
  }
}

// Context replay, all reads valid: the context of read r is the kWarm bytes
// [c, ar) before it in seq (reads are contiguous), loaded in one visit (eight
// 16-byte loads) and replayed in the same 16 chunks by every lane.  Away from the clamp, f does not depend on the word
// counter, so a chunk only moves f (4 FP64 ops per base); a chunk kHot flags
// replays byte by byte with the counter rebuilt at its first byte and reset
// at every read start (warm_exact).
template <int K>
__device__ __noinline__ State warm_exact(const Args &A, const Src &S, const uint8_t *cls,
                                         int64_t r, int c, int end, State st) {
  int64_t t = r - 1;
  while (A.idx[t] > c) --t;   // the read holding byte c
  int cnt = count_before<K>(A, S, cls, A.idx[t], c - A.idx[t]);
  int nxt = A.idx[t + 1];
  uint32_t acc = 0, words = 0;
  for (int j = c; j < end; ++j) {
    while (j == nxt) {   // read start: the counter resets (empty reads included)
      cnt = 0;
      ++t;
      nxt = A.idx[t + 1];
    }
    step<K, false, false, true>(cls[(uint8_t)A.seq[j]], 0u, 0u, st, cnt, acc, nullptr, nullptr, 0u,
                                0u, words);
  }
  return st;   // by value: a State behind a reference to a call would live in scratch
}

template <int K>
__device__ __forceinline__ void warm_chunk(const Args &A, const Src &S, const uint8_t *cls,
                                           int64_t r, v2u sv, int c, int end, State &st) {
  const int left = end - c;
  const uint64_t m = left >= 8 ? ~0ull : ((1ull << (8 * max(left, 0))) - 1);
  if (__builtin_expect(hot<K>(st), 0)) {
    if (left > 0) st = warm_exact<K>(A, S, cls, r, c, min(c + 8, end), st);
    return;
  }
  const v2u cl = {classes4(sv.x & (uint32_t)m), classes4(sv.y & (uint32_t)(m >> 32))};
#pragma unroll
  for (int u = 0; u < 8; ++u) move<K>(byte_of(cl, u), st);
}

template <int K>
__device__ State warm_contiguous(const Args &A, const Src &S, const uint8_t *cls, int64_t r) {
  constexpr double half = (double)(1 << K) * 0.5;   // :107-108
  State st = {half, half};
  const int ar = A.idx[r];
  const int c0 = max(A.idx[0], ar - kWarm);   // at the batch start: exact
  static_assert(kWarm == 128, "the context is loaded as 8 x 16 bytes");
  v4u w[8];   // the whole context in one visit (see run_read)
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = __builtin_amdgcn_raw_buffer_load_b128(S.rs, (uint32_t)(c0 + 16 * i), 0, 0);
#pragma unroll
  for (int j = 0; j < 16; ++j)
    warm_chunk<K>(A, S, cls, r, v2u{w[j >> 1][2 * (j & 1)], w[j >> 1][2 * (j & 1) + 1]}, c0 + 8 * j, ar, st);
  return st;
}

// the entry state guess for read r: replay the kWarm bytes of (valid) context
// before it from the fixed start state; exact when the context reaches the
// batch start
template <int K>
__device__ State guess_entry(const Args &A, const Src &S, const uint8_t *cls, int64_t r) {
  constexpr double half = (double)(1 << K) * 0.5;   // :107-108
  State st = {half, half};
  if (r == 0) return st;
  if (A.mode != HPGQ_CGR_ONLY_VALID_READS) return warm_contiguous<K>(A, S, cls, r);
  // common case: the previous read alone holds kWarm bytes
  const int ap = A.idx[r - 1], ar = A.idx[r];
  int64_t t;
  int p, need;
  if (ar - ap >= kWarm && valid_read(A, r - 1)) {
    t = r - 1;
    p = ar - ap - kWarm;
    need = 0;
  } else {
    need = kWarm;
    t = r;
    p = 0;
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
  }
  if (need > 0) {   // context reaches the batch start: replay it all, exactly
    t = 0;
    p = 0;
  }
  uint32_t w = 0;
  for (; t < r; ++t) {
    if (!valid_read(A, t)) continue;
    const int a = A.idx[t], n = A.idx[t + 1] - a;
    const int cnt0 = p > 0 ? count_before<K>(A, S, cls, a, p) : 0;
    run_read<K, false, false>(A, S, a, n, p, cnt0, st, nullptr, nullptr, 0u, w);
    p = 0;
  }
  return st;
}

template <int K>
__global__ void __launch_bounds__(kWG) cgr_fill_kernel(Args A) {
  constexpr int dim = 1 << K;
  constexpr bool kLds = K <= kLdsMaxK;
  constexpr int cells = dim * dim + 1;   // + the spare cell of the unconditional adds
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint8_t cls[256];
  // LDS: one u64 per cell, count | quality sum << 32 (see step)
  uint32_t *ts = kLds ? lds : A.ts;
  uint32_t *tq = kLds ? nullptr : A.tq;
  if (kLds)
    for (int i = threadIdx.x; i < 2 * cells; i += kWG) lds[i] = 0;
  fill_classes(cls, threadIdx.x, kWG);
  __syncthreads();
  const Src S = make_src(A);
  uint32_t words = 0;
  const int64_t stride = (int64_t)gridDim.x * kWG;
  for (int64_t r = (int64_t)blockIdx.x * kWG + threadIdx.x; r < A.num_reads; r += stride) {
    State st = guess_entry<K>(A, S, cls, r);
    A.g[r] = make_double2(st.fx, st.fy);
    if (valid_read(A, r)) {
      const int a = A.idx[r];
      run_read<K, true, kLds>(A, S, a, A.idx[r + 1] - a, 0, 0, st, ts, tq, 1u, words);
    }
    A.e[r] = make_double2(st.fx, st.fy);
  }
  if (kLds) {
    __syncthreads();
    for (int i = threadIdx.x; i < dim * dim; i += kWG) {
      const uint32_t c = lds[2 * i];
      if (c) {
        atomicAdd(&A.ts[i], c);
        atomicAdd(&A.tq[i], lds[2 * i + 1] - c * A.base_quality * (uint32_t)K);
      }
      words += c;   // every completed word added 1 to one real cell
    }
  }
  // fq_word_count: wave sum, one atomic per wave
  uint64_t w = words;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(A.words, (unsigned long long)w);
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
  __shared__ uint8_t cls[256];
  fill_classes(cls, threadIdx.x, 64);
  __syncthreads();
  const int lane = threadIdx.x;
  const Src S = make_src(A);
  const int64_t nw = (A.num_reads + 63) >> 6;
  const int64_t ns = (nw + 63) >> 6;
  int64_t last = 0;   // reads <= last are final (lane 0)
  unsigned long long replays = 0;
  uint32_t dummy = 0;
  // the wave scans 64 summary words at a time; lane 0 replays in read order
  for (int64_t sb = 0; sb < ns; sb += 64) {
    const unsigned long long v = sb + lane < ns ? A.sum[sb + lane] : 0ull;
    unsigned long long nz = __ballot(v != 0ull);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      unsigned long long sw = __shfl(v, l);
      if (lane != 0) continue;
      const int64_t si = sb + l;
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
              run_read<K, true, false>(A, S, A.idx[r], A.idx[r + 1] - A.idx[r], 0, 0, s1, A.ts,
                                       A.tq, 0xFFFFFFFFu, dummy);   // undo
            }
            State s2 = {entry.x, entry.y};
            if (valid_read(A, r))
              run_read<K, true, false>(A, S, A.idx[r], A.idx[r + 1] - A.idx[r], 0, 0, s2, A.ts,
                                       A.tq, 1u, dummy);
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
  }
  if (lane == 0) *A.replays = replays;
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

#include "hpgq_cgr_stream.h"

namespace hpgq {
namespace cgr {
namespace stream {

template <bool VALID>
static const void *stream_for_mode(int k) {
  switch (k) {
    case 1: return (const void *)cgr_stream_kernel<1, VALID>;
    case 2: return (const void *)cgr_stream_kernel<2, VALID>;
    case 3: return (const void *)cgr_stream_kernel<3, VALID>;
    case 4: return (const void *)cgr_stream_kernel<4, VALID>;
    case 5: return (const void *)cgr_stream_kernel<5, VALID>;
    case 6: return (const void *)cgr_stream_kernel<6, VALID>;
    default: return (const void *)cgr_stream_kernel<7, VALID>;
  }
}

// valid: the ONLY_VALID_READS instance (reads with status != 1 skipped, :188)
static const void *stream_for(int k, bool valid) {
  return valid ? stream_for_mode<true>(k) : stream_for_mode<false>(k);
}

}  // namespace stream
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
  // stream path (k <= 7, either mode; hpgq_cgr_stream.h).  Each streamed fill
  // gets a gate/done slot; the exact simulation of a fill whose gate is set
  // runs at the next sync (the batch and its status array must stay valid
  // until then, as for any asynchronous fill).
  int path = HPGQ_CGR_PATH_AUTO;
  int32_t *d_span_first = nullptr;
  unsigned long long *d_toggles = nullptr;   // ONLY_VALID_READS: validity toggle bits per read
  int64_t toggles_cap = 0;                   // words
  unsigned long long *d_scratch = nullptr;
  uint32_t *d_slots = nullptr;            // [kSlots][2]: gate, done
  struct Fill {
    hpgq_batch_t b;
    const uint8_t *status;
    int mode;
  };
  std::vector<Fill> pending;              // streamed fills not synced yet (slot = index)
  bool ran_exact = false;                 // an exact simulation ran since the last sync
  int last_exact = 0;
  int s_grid[2] = {0, 0};   // stream grid: all reads, ONLY_VALID_READS
  // RCCL (hpgq_cgr_allreduce): [table_seq | table_q | word count] u32, packed
  // and summed out of place; reads return the sum until the next fill / reset
  ncclComm_t comm = nullptr;
  uint32_t *d_pack = nullptr, *d_global = nullptr;
  bool reduced = false;
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

// the exact double simulation of one call (cgr_fill / check / fix)
static int cgr_exact(hpgq_cgr *c, const hpgq_batch_t *b, const uint8_t *status, int mode) {
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
  c->ran_exact = true;
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
  c->lds = k <= hpgq::cgr::kLdsMaxK ? 2 * (cells + 1) * 4 : 0;   // u64 per cell + spare
  const void *kfn = hpgq::cgr::fill_for(k);
  if (c->lds > 64 * 1024)
    HPGQ_HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds));
  int per_cu = 0, cus = 0;
  HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, hpgq::cgr::kWG, c->lds));
  HPGQ_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  c->grid = std::max(1, per_cu) * cus;
  if (k <= hpgq::cgr::stream::kMaxK) {
    namespace S = hpgq::cgr::stream;
    HPGQ_HIP_TRY(hipMalloc(&c->d_span_first, S::kMaxSpans * sizeof(int32_t)));
    HPGQ_HIP_TRY(hipMalloc(&c->d_scratch, cells * 8));
    HPGQ_HIP_TRY(hipMemsetAsync(c->d_scratch, 0, cells * 8, c->stream));
    HPGQ_HIP_TRY(hipMalloc(&c->d_slots, S::kSlots * 2 * sizeof(uint32_t)));
    HPGQ_HIP_TRY(hipMemsetAsync(c->d_slots, 0, S::kSlots * 2 * sizeof(uint32_t), c->stream));
    for (int v = 0; v < 2; ++v) {
      int spc = 0;
      HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&spc, S::stream_for(k, v != 0), S::kWG, 0));
      c->s_grid[v] = std::max(1, spc) * cus;
    }
    c->pending.reserve(S::kSlots);
  }
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
  (void)hipFree(c->d_span_first);
  (void)hipFree(c->d_toggles);
  (void)hipFree(c->d_scratch);
  (void)hipFree(c->d_slots);
  (void)hipFree(c->d_pack);
  (void)hipFree(c->d_global);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int hpgq_cgr_fill_device(hpgq_cgr_t *c, const hpgq_batch_t *b, const uint8_t *status, int mode) {
  if (!c || !b || b->num_reads < 0) return HPGQ_E_INVALID;
  if (mode != HPGQ_CGR_ALL_READS && mode != HPGQ_CGR_ONLY_VALID_READS) return HPGQ_E_INVALID;
  if (b->num_reads == 0) return HPGQ_OK;
  if (!b->seq || !b->quality || !b->data_indices) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  c->reduced = false;
  const bool valid = mode == HPGQ_CGR_ONLY_VALID_READS;
  if (valid && !status) return HPGQ_OK;   // no status array: every read is skipped (:188)
  const bool streamed = c->path == HPGQ_CGR_PATH_AUTO && c->k <= hpgq::cgr::stream::kMaxK &&
                        b->num_reads < INT32_MAX;   // (32-bit read cursors)
  if (!streamed) return cgr_exact(c, b, status, mode);
  namespace S = hpgq::cgr::stream;
  if ((int)c->pending.size() == S::kSlots) {   // out of slots: settle the ones in flight
    int rc = hpgq_cgr_sync(c);
    if (rc) return rc;
  }
  const int64_t words = b->num_reads / 64 + 1;   // span_first_kernel's toggle words
  if (valid && words > c->toggles_cap) {
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));   // (fills in flight may still read the old words)
    (void)hipFree(c->d_toggles);
    c->d_toggles = nullptr;
    c->toggles_cap = 0;
    const int64_t cap = words + words / 4 + 64;
    if (hipMalloc(&c->d_toggles, cap * 8) != hipSuccess) return HPGQ_E_NOMEM;
    c->toggles_cap = cap;
  }
  const int slot = (int)c->pending.size();
  S::SArgs SA;
  SA.seq = b->seq;
  SA.qual = b->quality;
  SA.idx = b->data_indices;
  SA.status = valid ? status : nullptr;
  SA.toggles = valid ? c->d_toggles : nullptr;
  SA.num_reads = b->num_reads;
  SA.base_quality = c->base_quality;
  SA.span_first = c->d_span_first;
  SA.scratch = c->d_scratch;
  SA.gate = c->d_slots + 2 * slot;
  SA.done = c->d_slots + 2 * slot + 1;
  SA.ts = c->d_ts;
  SA.tq = c->d_tq;
  SA.words = c->d_words;
  void *sargs[] = {&SA};
  HPGQ_HIP_TRY(hipLaunchKernel((const void *)S::span_first_kernel,
                               dim3((unsigned)std::min<int64_t>((b->num_reads + 1 + 255) / 256, S::kSpanFirstGrid)),
                               dim3(256), sargs, 0, c->stream));
  HPGQ_HIP_TRY(hipLaunchKernel(S::stream_for(c->k, valid), dim3(c->s_grid[valid ? 1 : 0]), dim3(S::kWG), sargs, 0, c->stream));
  c->pending.push_back(hpgq_cgr::Fill{*b, status, mode});
  return HPGQ_OK;
}

int hpgq_cgr_sync(hpgq_cgr_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  if (!c->pending.empty()) {
    // streamed fills whose gate is set: the exact simulation, in fill order
    std::vector<uint32_t> slots(2 * c->pending.size());
    HPGQ_HIP_TRY(hipMemcpy(slots.data(), c->d_slots, slots.size() * 4, hipMemcpyDeviceToHost));
    std::vector<hpgq_cgr::Fill> todo;
    todo.swap(c->pending);
    for (size_t i = 0; i < todo.size(); ++i)
      if (slots[2 * i] & hpgq::cgr::stream::GATE_EXACT) {
        int rc = cgr_exact(c, &todo[i].b, todo[i].status, todo[i].mode);
        if (rc) return rc;
      }
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  }
  if (c->ran_exact) {
    unsigned long long r = 0;
    HPGQ_HIP_TRY(hipMemcpy(&r, c->d_replays, 8, hipMemcpyDeviceToHost));
    c->last_replays = (int64_t)r;
  } else {
    c->last_replays = 0;
  }
  c->last_exact = c->ran_exact ? 1 : 0;
  c->ran_exact = false;
  return HPGQ_OK;
}

int hpgq_cgr_reset(hpgq_cgr_t *c) {
  if (!c) return HPGQ_E_INVALID;
  int rc = hpgq_cgr_sync(c);   // fills before the reset settle first
  if (rc) return rc;
  const size_t cells = (size_t)c->dim * c->dim;
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_ts, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_tq, 0, cells * 4, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_words, 0, 8, c->stream));
  c->reduced = false;
  return HPGQ_OK;
}

int hpgq_cgr_read(hpgq_cgr_t *c, uint32_t *table_seq, uint32_t *table_q, uint32_t *word_count) {
  if (!c) return HPGQ_E_INVALID;
  int rc = hpgq_cgr_sync(c);
  if (rc) return rc;
  const size_t cells = (size_t)c->dim * c->dim;
  if (c->reduced) {   // the all-reduced tables (hpgq_cgr_allreduce)
    if (table_seq) HPGQ_HIP_TRY(hipMemcpy(table_seq, c->d_global, cells * 4, hipMemcpyDeviceToHost));
    if (table_q) HPGQ_HIP_TRY(hipMemcpy(table_q, c->d_global + cells, cells * 4, hipMemcpyDeviceToHost));
    if (word_count) HPGQ_HIP_TRY(hipMemcpy(word_count, c->d_global + 2 * cells, 4, hipMemcpyDeviceToHost));
    return HPGQ_OK;
  }
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

int hpgq_cgr_set_path(hpgq_cgr_t *c, int path) {
  if (!c || (path != HPGQ_CGR_PATH_AUTO && path != HPGQ_CGR_PATH_EXACT)) return HPGQ_E_INVALID;
  c->path = path;
  return HPGQ_OK;
}

int hpgq_cgr_last_exact(hpgq_cgr_t *c) { return c ? c->last_exact : HPGQ_E_INVALID; }

// ---------------------------------------------------------------------------
// RCCL (one process per GPU): the table sum of read-sharded fills
// ---------------------------------------------------------------------------

int hpgq_cgr_comm_init(hpgq_cgr_t *c, int nranks, int rank, const char id[HPGQ_COMM_ID_BYTES]) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return HPGQ_E_INVALID;
  if (c->comm) return HPGQ_E_STATE;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  const size_t words = 2 * (size_t)c->dim * c->dim + 1;
  if (!c->d_pack) HPGQ_HIP_TRY(hipMalloc(&c->d_pack, words * 4));
  if (!c->d_global) HPGQ_HIP_TRY(hipMalloc(&c->d_global, words * 4));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  if (ncclCommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
    c->comm = nullptr;
    return HPGQ_E_RCCL;
  }
  return HPGQ_OK;
}

// Sum of every rank's tables and word count as u32, so the sum wraps like the
// reference's unsigned tables and fq_word_count (old/chaos_game.c:253-258).
// Settles this rank's fills first (a gated fill's exact simulation runs in
// the sync); the result stays on the device for hpgq_cgr_read.
int hpgq_cgr_allreduce(hpgq_cgr_t *c) {
  if (!c) return HPGQ_E_INVALID;
  if (!c->comm) return HPGQ_E_STATE;
  int rc = hpgq_cgr_sync(c);
  if (rc) return rc;
  const size_t cells = (size_t)c->dim * c->dim;
  HPGQ_HIP_TRY(hipMemcpyAsync(c->d_pack, c->d_ts, cells * 4, hipMemcpyDeviceToDevice, c->stream));
  HPGQ_HIP_TRY(hipMemcpyAsync(c->d_pack + cells, c->d_tq, cells * 4, hipMemcpyDeviceToDevice, c->stream));
  // the u64 device word count's low half (little endian) is the u32 fq_word_count
  HPGQ_HIP_TRY(hipMemcpyAsync(c->d_pack + 2 * cells, c->d_words, 4, hipMemcpyDeviceToDevice, c->stream));
  if (ncclAllReduce(c->d_pack, c->d_global, 2 * cells + 1, ncclUint32, ncclSum, c->comm, c->stream) != ncclSuccess)
    return HPGQ_E_RCCL;
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  c->reduced = true;
  return HPGQ_OK;
}

uint32_t *hpgq_cgr_global_device(hpgq_cgr_t *c) { return c ? c->d_global : nullptr; }

int hpgq_cgr_comm_count(hpgq_cgr_t *c, int *count) {
  if (!c || !count) return HPGQ_E_INVALID;
  *count = 0;
  if (!c->comm) return HPGQ_E_STATE;
  return ncclCommCount(c->comm, count) == ncclSuccess ? HPGQ_OK : HPGQ_E_RCCL;
}

}  // extern "C"
