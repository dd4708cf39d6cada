// hpgq_cgr_stream.h — the coalesced CGR path (included by hpgq_cgr.hip).
//
// chaos_game_fill_tables (old/chaos_game.c:165-267) takes the cell of a word
// from (int) of a double state f that is carried across the whole call.  This
// path computes every cell from the word's own K bases instead, position-
// parallel over the batch's bytes, and is used only where that is provably
// the same cell; otherwise the exact simulation (cgr_fill/check/fix) runs.
//
// Why the cell is the word's own bases.  Per axis, with dim = 2^K, write a
// base's move as Z (f*0.5: C/G on x, A/C on y; exact) or D (f + (dim-f)*0.5:
// A/T on x, G/T on y; two roundings, each result within dim*2^-53 of the real
// value).  N and other bytes do not move f.  Let a word end at time t and let
// L = the integer whose bits are the word's K moves (D = 1, newest = MSB); the
// floor trajectory (start 0 at t-K) and the ceiling trajectory (start dim) of
// those K moves are exactly representable and end at L and L+1.  Both moves
// are monotone up to rounding that never crosses a representable point of
// those trajectories (checked per case: Z is exact; D's two roundings together
// stay within half an ulp of the result grid), so f_{t-K} in [0, dim] gives
// f_t in [L, L+1]: the cell is L unless f_t == L+1 exactly (L+1 = dim is the
// clamp, whose cell is dim-1 = L as well).  Hitting L+1 < dim needs the gap
// dim - f_{t-K} <= dim*2^(K-52): after a Z, f <= dim/2, and each D at most
// halves the gap less dim*2^-53, so the gap after a run of r D-moves is >=
// dim*(2^-(r+1) - 2^-52), which rules the hit out while r <= 49-K.  The same
// bound keeps f < dim, so no EPSILON nudge (:241-251) ever fires either.
//
// So a batch (one call) is exact on this path iff no axis has a run of >= kRun
// (= 48-K, a margin of 2) D-moves without a Z in between — counted over the
// moving bases of the whole call in order (f is carried across reads and
// across N) from f0 = dim/2 (a gap of dim/2, as after a Z) — and it holds no
// byte other than A/C/G/T/N (they would shift the raw-position quality
// subtraction of :259) and no quality byte >= 128 (signed char adds).  With
// those, a word at byte p is emitted iff bytes [p-K+1, p] are A/C/G/T in one
// read (the counter rule :234-236, reset at read starts and N), and its
// quality accumulator is the sum of those K quality bytes.  Random reads
// never violate this; a batch that does (poly-A/T/G runs, lowercase, IUPAC)
// sets the gate and the exact kernels redo the whole call.
//
// ONLY_VALID_READS (VALID): a read whose status is not VALID_READ is skipped
// before any state update (:188), so f passes through it unchanged and it
// emits no word: its bytes act exactly like 'N' bytes (no move, no word) and
// its quality bytes like zeros, and that is how the kernel treats them.  Read
// starts whose validity differs from the read before are scattered into a
// second per-wave bitmap (XOR, so empty reads at one offset cancel); a
// byte's "skipped" bit is the tile's entry state XOR a prefix parity of those
// toggles (within the lane by shifts, across lanes by one ballot), and a tile
// holding skipped bytes masks them before anything else looks at its bytes.
// The run bound and the exact run scan then see the moves of the valid reads
// only, across skipped reads, as the reference's carried f does.
//
// Layout: the bytes [idx[0], idx[n]) are cut into spans of kSpan bytes; wave
// g takes spans g, g + W, ... (W waves in the grid) as one stream of 2 KB
// tiles, a lane 32 contiguous bytes of seq and of quality per tile (16-byte
// loads; the next tile -- across span boundaries too, with its span's
// context and cursor -- in flight while this one is counted).  The K-1
// bytes of context come from the neighbouring lane by DPP (lane 0: the last
// lane of the previous tile, or a broadcast load at a span start).  The
// lane's bytes become a packed 2-bit code stream (v_dot4), so a word's cell
// is one v_alignbit and a mask.  Read starts inside a tile are scattered into
// a per-wave LDS bitmap from the read offsets the wave walks with a cursor.
// Words go to the workgroup's LDS table (u64 per cell: count | quality sum
// << 32, one ds_add_u64 per byte; a byte that ends no word adds to its lane's
// spare cell), flushed to a global u64 scratch table; the last workgroup to
// finish moves it into the reference layout (or discards it when the gate is
// set).  A run of >= kRun (>= 41) D-moves spans at least three aligned 16-byte
// chunks, and a chunk wholly inside it holds no Z on that axis; so only tiles
// with a Z-free chunk (a tile holding skipped bytes: see run_candidate) or
// entered with a long open run are scanned exactly (one segmented DPP scan
// per axis, tile_runs); the run open at such a tile's start is walked back
// for only when its bound would decide.
#pragma once

// (The round-4 timing-only ablations of the per-byte loop are a patch,
// tools/probes/c5_ablation.patch, applied by tools/probes/build_src_variant.sh:
// the tables they leave are wrong, so they are not in the product source.)

namespace hpgq {
namespace cgr {
namespace stream {

constexpr int kWaves = 16;
constexpr int kWG = kWaves * 64;
constexpr int kLaneBytes = 32;               // the packed code stream assumes it
constexpr int kNdw = kLaneBytes / 4;
constexpr int kTile = 64 * kLaneBytes;       // bytes per wave tile (2 KB)
constexpr int kSpanLog = 14;
constexpr int kSpan = 1 << kSpanLog;         // bytes per span (16 KB, 8 tiles)
constexpr int kSpanFirstGrid = 2048;
constexpr int kMaxK = 7;                     // 4^7 u64 cells = 128 KB of LDS
constexpr int64_t kMaxSpans = ((int64_t)1 << 31) / kSpan + 2;
constexpr int kSlots = 256;                  // fills in flight between two syncs

constexpr uint32_t GATE_EXACT = 1;   // the exact kernels must run

// byte & 7 -> per-byte LUTs (v_perm_b32, codes A=1 C=3 T=4 N=6 G=7)
constexpr uint32_t kCdLo = 0x00000100u;   // code = x | y << 1: A 1, C 0
constexpr uint32_t kCdHi = 0x02030003u;   //                    T 3, G 2, N 3 (N emits no word;
                                          // as 3 it has no Z bit in ~code below)
constexpr uint32_t kV1Lo = 0x01000100u;   // 1 for A/C/G/T, 0 for N
constexpr uint32_t kV1Hi = 0x01000001u;
constexpr uint32_t kDLo = 0x00000100u;    // D moves x | y << 1: A 1, C 0
constexpr uint32_t kDHi = 0x02000003u;    //                     T 3, G 2, N 0

struct SArgs {   // (read indices fit 31 bits: the host sends larger batches to the exact path)
  const char *seq, *qual;
  const int32_t *idx;
  const uint8_t *status;            // VALID: read_status[] (1 = VALID_READ)
  unsigned long long *toggles;      // VALID: bit r: read r's validity differs from read r-1's
                                    // (valid before read 0); written by span_first_kernel
  int64_t num_reads;
  uint32_t base_quality;
  int32_t *span_first;              // [kMaxSpans] first read with idx[r] >= span start - 32
  unsigned long long *scratch;      // [4^K] count | quality sum << 32
  uint32_t *gate;                   // this fill's slot: GATE_EXACT when it needs the exact path
  uint32_t *done;                   // this fill's slot: workgroups finished
  uint32_t *ts, *tq;                // final tables [dim][dim]
  unsigned long long *words;
};

// spans start at a0 = idx[0] rounded down to 16 bytes
__device__ __forceinline__ int64_t nspans(int32_t a0, int32_t b1) {
  return b1 > a0 ? ((int64_t)b1 - a0 + kSpan - 1) >> kSpanLog : 0;
}

// span_first[s] = the first read r with idx[r] >= a0 + s*kSpan - 32: thread r
// writes the spans whose (start - 32) lies in (idx[r-1], idx[r]]; thread 0
// also clears this fill's gate and done slots.  VALID: each wave also stores
// the validity toggles of its 64 reads as one word (ballot), words 0 ..
// num_reads / 64 (the stream kernel reads them through a range-checked
// descriptor: past them, 0).
// (grid-stride: a few thousand workgroups walk the whole idx array; one
// thread per read made the launch dispatch-bound at ~17 us per 5 M reads)
__global__ void __launch_bounds__(256) span_first_kernel(SArgs A) {
  const int32_t b0 = A.idx[0], b1 = A.idx[A.num_reads];
  const int32_t a0 = b0 & ~15;
  const int64_t ns = nspans(a0, b1);
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int lane = threadIdx.x & 63;
  for (int64_t r0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); r0 <= A.num_reads; r0 += stride) {
    const int64_t r = r0 + lane;
    if (r <= A.num_reads) {
      if (r == 0) {
        *A.gate = 0u;
        *A.done = 0u;
      }
      const int64_t hi = (int64_t)A.idx[r] + 32 - a0;   // s*kSpan <= hi
      const int64_t lo = r == 0 ? -1 : (int64_t)A.idx[r - 1] + 32 - a0;   // s*kSpan > lo
      const int64_t s0 = lo < 0 ? 0 : (lo >> kSpanLog) + 1;
      const int64_t s1 = r == A.num_reads ? ns - 1 : (hi >> kSpanLog);   // past the last start: the end sentinel
      for (int64_t s = s0; s <= s1 && s < ns; ++s) A.span_first[s] = (int32_t)r;
    }
    if (A.status) {
      const bool t = r < A.num_reads && (A.status[r] == 1) != (r == 0 || A.status[r - 1] == 1);
      const unsigned long long m = __ballot(t);
      if (lane == 0) A.toggles[r0 >> 6] = m;
    }
  }
}

// a lane's word of a bitmap, cleared for its next use
__device__ __forceinline__ uint32_t take_bits(uint32_t *p) {
  const uint32_t v = *p;
  *p = 0u;
  return v;
}

__device__ __forceinline__ uint32_t dpp_ror1(uint32_t v) {   // lane l <- lane l-1, lane 0 <- lane 63
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {   // lane l <- lane l-1
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// a lane's bytes of seq: LUT lookups, exactness and per-lane summaries
struct Cls {
  uint32_t cd[kNdw];   // per byte: its code x | y << 1
  uint32_t p0, p1;     // the 32 codes packed, byte j at bits 2j of the 64-bit p1:p0
  uint32_t v;          // bit j: byte j is A/C/G/T
  uint32_t zlo, zhi;   // OR of per-byte Z bits (bit0 x, bit1 y) over the first / last 16 bytes
  uint32_t bad;        // nonzero: a byte that is not exactly A/C/G/T/N
};

__device__ __forceinline__ Cls classify(const uint32_t s[kNdw]) {
  static_assert(kNdw == 8, "the packed code stream assumes 32 bytes per lane");
  Cls c;
  uint32_t bad = 0, zl = 0, zh = 0, vp[kNdw / 2], g[kNdw];
#pragma unroll
  for (int d = 0; d < kNdw; ++d) {
    const uint32_t code = s[d] & 0x07070707u;
    // bad |= s ^ expected (v_bitop3: one op, no compare per dword)
    bad = __builtin_amdgcn_bitop3_b32(bad, s[d], __builtin_amdgcn_perm(hpgq::cgr::kExHi, hpgq::cgr::kExLo, code), 0xF6);
    c.cd[d] = __builtin_amdgcn_perm(kCdHi, kCdLo, code);
    g[d] = __builtin_amdgcn_udot4(c.cd[d], 0x40100401u, 0u, false);   // 4 codes -> 8 bits
    // Z bits: a Z move on x is x = 0 (C/G), on y is y = 0 (A/C): ~code & 3
    if (d < 4) zl = __builtin_amdgcn_bitop3_b32(zl, c.cd[d], 0x03030303u, 0xF2);   // zl | (~cd & 3s)
    if (d >= kNdw - 4) zh = __builtin_amdgcn_bitop3_b32(zh, c.cd[d], 0x03030303u, 0xF2);
    // the V bit of byte j to bit j: byte weights 1,2,4,8 (<< 4 for odd dwords) by v_dot4
    const uint32_t v1 = __builtin_amdgcn_perm(kV1Hi, kV1Lo, code);
    vp[d >> 1] = (d & 1) ? __builtin_amdgcn_udot4(v1, 0x80402010u, vp[d >> 1], false)
                         : __builtin_amdgcn_udot4(v1, 0x08040201u, 0u, false);
  }
  c.p0 = g[0] | (g[1] << 8) | (g[2] << 16) | (g[3] << 24);
  c.p1 = g[4] | (g[5] << 8) | (g[6] << 16) | (g[7] << 24);
  c.v = 0;
#pragma unroll
  for (int d = 0; d < kNdw / 2; ++d) c.v |= vp[d] << (8 * d);
  c.zlo = zl;
  c.zhi = zh;
  c.bad = bad;
  return c;
}

// ---- which tiles could hold a run -----------------------------------------
// All reads: a tile with a Z-free 16-byte chunk (on either axis).  A run of
// >= kRun >= 41 D moves spans >= 3 aligned chunks: its first and last chunk
// hold <= 15 of its D moves each, so the chunks wholly inside it (Z-free)
// hold >= 11.  Skipped reads make many partly masked chunks Z-free, so a tile
// holding skipped bytes uses a sharper test that the same count still
// guarantees: a Z-free chunk with >= 6 D moves, or a lane whose two chunks
// are Z-free and hold a D move.  (Inside chunks with <= 5 D moves each mean
// >= 3 inside chunks holding D moves; at most two of them lie outside the
// lanes wholly inside the run, so a wholly inside lane holds one.)  A tile
// passing the cheap all-reads test in either case runs that sharper one.

// bit j <- byte j's bit 0, from per-byte 0/1 values (v_dot4 with byte weights)
__device__ __forceinline__ uint32_t byte_bits(const uint32_t (&b)[kNdw]);

__device__ __forceinline__ bool run_candidate(const Cls &c) {
  bool cand = false;
#pragma unroll
  for (int ax = 0; ax < 2; ++ax) {
    uint32_t xb[kNdw];
#pragma unroll
    for (int d = 0; d < kNdw; ++d) xb[d] = (c.cd[d] >> ax) & 0x01010101u;
    const uint32_t bits = byte_bits(xb);
    const uint32_t D = c.v & bits, Z = c.v & ~bits;
    const bool z0 = (Z & 0xFFFFu) != 0u, z1 = (Z >> 16) != 0u;
    const int d0 = __builtin_popcount(D & 0xFFFFu), d1 = __builtin_popcount(D >> 16);
    cand = cand || (!z0 && d0 >= 6) || (!z1 && d1 >= 6) || (!z0 && !z1 && D != 0u);
  }
  return __ballot(cand) != 0ull;
}

// ---- exact run scan of one tile (rare path: tiles that could hold a run) ----
// Runs within one lane's 32 bytes are < 41 <= kRun (a run needs no Z for
// kRun D moves), so only runs across lanes matter.  Per lane and axis: hz
// (the lane holds a Z), cnt (its D moves), pfx / sfx (D moves before its
// first / after its last Z); then one segmented inclusive scan over the wave
// (DPP row_shr + row_bcast, as wave_scan) of (hz, hz ? sfx : cnt): each lane
// learns the run open at its start.

__device__ __forceinline__ uint32_t byte_bits(const uint32_t (&b)[kNdw]) {
  uint32_t vp[kNdw / 2];
#pragma unroll
  for (int d = 0; d < kNdw; ++d)
    vp[d >> 1] = (d & 1) ? __builtin_amdgcn_udot4(b[d], 0x80402010u, vp[d >> 1], false)
                         : __builtin_amdgcn_udot4(b[d], 0x08040201u, 0u, false);
  return vp[0] | (vp[1] << 8) | (vp[2] << 16) | (vp[3] << 24);
}

// one step of the segmented scan: (f, v) <- (f_nb | f, f ? v : v_nb + v)
template <int CTRL, int RM, bool BC>
__device__ __forceinline__ void seg_step(uint32_t &f, uint32_t &v) {
  const uint32_t nv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, BC);
  const uint32_t nf = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, CTRL, RM, 0xF, BC);
  v = f ? v : v + nv;
  f |= nf;
}

struct TileRuns {
  bool risky;      // a run >= run_max that does not involve the entering run
  bool risky_in;   // the entering run e plus the tile's leading D moves reach run_max
  bool anyz;       // the tile holds a Z on this axis
  uint32_t out;    // D moves after the tile's last Z (anyz), else the tile's D moves
};

template <int AX>
__device__ __forceinline__ TileRuns tile_runs(const Cls &c, uint32_t e, uint32_t run_max) {
  uint32_t xb[kNdw];
#pragma unroll
  for (int d = 0; d < kNdw; ++d) xb[d] = (c.cd[d] >> AX) & 0x01010101u;
  const uint32_t bits = byte_bits(xb);
  const uint32_t D = c.v & bits, Z = c.v & ~bits;
  const uint32_t cnt = (uint32_t)__builtin_popcount(D);
  const uint32_t pfx = (uint32_t)__builtin_popcount(D & ((Z & (0u - Z)) - 1u));   // Z = 0: all of D
  const uint32_t top = Z ? (0xFFFFFFFFu >> __builtin_clz(Z)) : 0u;               // bits up to the last Z
  const uint32_t sfx = (uint32_t)__builtin_popcount(D & ~top);
  uint32_t f = Z ? 1u : 0u, v = Z ? sfx : cnt;
  seg_step<0x111, 0xF, true>(f, v);
  seg_step<0x112, 0xF, true>(f, v);
  seg_step<0x114, 0xF, true>(f, v);
  seg_step<0x118, 0xF, true>(f, v);
  seg_step<0x142, 0xA, false>(f, v);
  seg_step<0x143, 0xC, false>(f, v);
  // exclusive: lane l - 1's inclusive (lane 0: nothing before)
  const uint32_t ev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
  const uint32_t ef = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x138, 0xF, 0xF, false);
  TileRuns t;
  t.risky = __ballot(ef && ev + pfx >= run_max) != 0ull;
  t.risky_in = __ballot(!ef && e + ev + pfx >= run_max) != 0ull;
  t.anyz = __builtin_amdgcn_readlane(f, 63) != 0u;
  t.out = __builtin_amdgcn_readlane(v, 63);
  return t;
}

__device__ __forceinline__ bool moving_byte(uint8_t ch) { return ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T'; }

template <int AX>
__device__ __forceinline__ bool d_move(uint8_t ch) {
  return AX == 0 ? (ch == 'A' || ch == 'T') : (ch == 'G' || ch == 'T');
}

// the run open at byte `at` on axis AX (capped at run_max), walking back from
// it; rare: only for tiles that need the exact scan
template <int AX>
__device__ uint32_t run_before(const SArgs &A, int32_t b0, int32_t at, uint32_t run_max) {
  uint32_t run = 0;
  for (int32_t p = at - 1; p >= b0 && run < run_max; --p) {
    const uint8_t ch = (uint8_t)A.seq[p];
    if (!moving_byte(ch)) continue;   // N (other bytes set the gate in their own tile)
    if (!d_move<AX>(ch)) break;
    ++run;
  }
  return run;
}

// VALID: the same, skipping the reads that are not valid; t is the read that
// holds byte at - 1 (-1: none)
template <int AX>
__device__ uint32_t run_before_valid(const SArgs &A, int32_t at, int32_t t, uint32_t run_max) {
  uint32_t run = 0;
  int32_t p = at - 1;
  for (; t >= 0 && run < run_max; --t) {
    const int32_t lo = A.idx[t];
    if (A.status[t] == 1) {
      for (; p >= lo && run < run_max; --p) {
        const uint8_t ch = (uint8_t)A.seq[p];
        if (!moving_byte(ch)) continue;
        if (!d_move<AX>(ch)) return run;
        ++run;
      }
    }
    p = lo - 1;
  }
  return run;
}

template <int AX>
struct AxisTag {
  static constexpr int value = AX;
};

// the idx window a wave walks: lane j holds idx[r + j] (0x7FFFFFFF past the
// end); the load is unconditional (clamped index) so that no branch splits the
// compiler's view of the loads in flight.  VALID: tg = 1 when read r + j's
// validity differs from read r + j - 1's (the state before read 0 is valid):
// bit r + j of span_first_kernel's toggle words, one dword load per lane
// (rt: their descriptor; past the words, 0)
template <bool VALID>
__device__ __forceinline__ int32_t idx_window(const SArgs &A, __amdgpu_buffer_rsrc_t rt, int32_t r, int lane,
                                              uint32_t &tg) {
  const int32_t j = r + lane, n = (int32_t)A.num_reads;
  const int32_t v = A.idx[j <= n ? j : n];
  if (VALID) tg = __builtin_amdgcn_ubfe(__builtin_amdgcn_raw_buffer_load_b32(rt, ((uint32_t)j >> 5) * 4u, 0, 0), j & 31, 1);
  return j <= n ? v : 0x7FFFFFFF;
}

// the same loads, raw: the value and the toggle word as loaded, made into the
// window (idx_at, tog_at) only where scatter_starts uses them.  The window is
// loop-carried; any operation on a loaded value at the loop's merge point (the
// select above) makes the wave wait there for that load and, vmcnt being in
// order, for every load issued before it -- the tile bytes prefetched for the
// tiles after this one (round 4: a vmcnt(0) per tile removed).
template <bool VALID>
__device__ __forceinline__ int32_t idx_window_raw(const SArgs &A, __amdgpu_buffer_rsrc_t rt, int32_t r, int lane,
                                                  uint32_t &tw) {
  const int32_t j = r + lane, n = (int32_t)A.num_reads;
  const int32_t v = A.idx[j <= n ? j : n];
  if (VALID) tw = __builtin_amdgcn_raw_buffer_load_b32(rt, ((uint32_t)j >> 5) * 4u, 0, 0);
  return v;
}
__device__ __forceinline__ int32_t idx_at(const SArgs &A, int32_t r, int lane, int32_t v) {
  return r + lane <= (int32_t)A.num_reads ? v : 0x7FFFFFFF;
}
__device__ __forceinline__ uint32_t tog_at(int32_t r, int lane, uint32_t tw) {
  return __builtin_amdgcn_ubfe(tw, (uint32_t)(r + lane) & 31u, 1);
}

// read starts in [base, limit) (limit - base <= 64 * kLaneBytes): bits into
// the wave's LDS bitmap sc[64] (TOG: the validity toggles into tc[64]),
// advancing the cursor r past them.  iw / itg are the window at r (loaded
// ahead by the caller, raw: see idx_window_raw); they come
// back as the window at the new r, its load in flight.  hop: the tile is its span's last, so the cursor moves on to rn
// (the next span's first read) instead.
template <bool VALID, bool TOG>
__device__ __forceinline__ void scatter_starts(const SArgs &A, __amdgpu_buffer_rsrc_t rt, uint32_t *sc, uint32_t *tc,
                                               int32_t &r, int32_t &iw, uint32_t &itg, int32_t base, int32_t limit,
                                               int lane, bool hop = false, int32_t rn = 0) {
  auto put = [&](int32_t x, uint32_t tg) {
    const bool in = x < limit;
    const uint32_t o = (uint32_t)(x - base);
    if (in && o < 64u * kLaneBytes) {   // o in range unless idx is unsorted
      atomicOr(&sc[o / kLaneBytes], 1u << (o % kLaneBytes));
      if (TOG && tg) atomicXor(&tc[o / kLaneBytes], 1u << (o % kLaneBytes));
    }
    const int c = __popcll(__ballot(in));
    r += c;
    return c;
  };
  const int32_t x0 = idx_at(A, r, lane, iw);
  const uint32_t tg0 = VALID ? tog_at(r, lane, itg) : itg;
  if (__builtin_expect(put(x0, tg0) == 64, 0)) {   // rare: more than 64 starts in the tile
    int c;
    do {
      uint32_t tg = 0;
      const int32_t x = idx_window<VALID>(A, rt, r, lane, tg);
      c = put(x, tg);
    } while (c == 64);
  }
  if (hop) r = rn;
  iw = idx_window_raw<VALID>(A, rt, r, lane, itg);
}

// a lane's bytes at o (o >= 0) from a buffer descriptor; bytes past the end read 0
__device__ __forceinline__ void load32(__amdgpu_buffer_rsrc_t rsrc, uint32_t o, uint32_t w[kNdw]) {
#pragma unroll
  for (int h = 0; h < kNdw / 4; ++h) {
    const v4u a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o + 16u * h, 0, 0);
    w[4 * h] = a[0]; w[4 * h + 1] = a[1]; w[4 * h + 2] = a[2]; w[4 * h + 3] = a[3];
  }
}

// bytes outside [lo, hi) -> 'N' (no move, no word) and quality 0
__device__ __forceinline__ void mask_range(int32_t o, int32_t lo, int32_t hi, uint32_t sw[kNdw], uint32_t qw[kNdw]) {
#pragma unroll
  for (int j = 0; j < kLaneBytes; ++j) {
    const int32_t p = o + j;
    if (p >= lo && p < hi) continue;
    const uint32_t sh = 8 * (j & 3);
    sw[j >> 2] = (sw[j >> 2] & ~(0xFFu << sh)) | (0x4Eu << sh);
    qw[j >> 2] &= ~(0xFFu << sh);
  }
}

// VALID: bytes whose bit is set in skip (bit j = byte j) -> 'N' and quality 0
__device__ __forceinline__ void mask_skipped(uint32_t skip, uint32_t sw[kNdw], uint32_t qw[kNdw]) {
#pragma unroll
  for (int d = 0; d < kNdw; ++d) {
    // 4 bits -> 4 byte masks (the products land on distinct bits: no carries)
    const uint32_t bm = ((((skip >> (4 * d)) & 0xFu) * 0x00204081u) & 0x01010101u) * 0xFFu;
    sw[d] = __builtin_amdgcn_bitop3_b32(sw[d], bm, 0x4E4E4E4Eu, 0xB8);   // bm ? 'N' : sw
    qw[d] &= ~bm;
  }
}

// the chunk-and-axis pairs (4 bits: chunk 0 x, y, chunk 1 x, y) of a lane
// whose bytes hold a bit of u (per byte bits 0-1, lo: bytes 0..15, hi: 16..31)
__device__ __forceinline__ uint32_t chunk_bits(uint32_t lo, uint32_t hi) {
  const uint32_t u = lo | (hi << 2);
  return (u | (u >> 8) | (u >> 16) | (u >> 24)) & 0xFu;
}

// the same for D moves (A/T on x, G/T on y) of a lane's seq bytes
__device__ __forceinline__ uint32_t chunk_bits_d(const uint32_t (&s)[kNdw]) {
  uint32_t dl = 0, dh = 0;
#pragma unroll
  for (int d = 0; d < kNdw; ++d) {
    const uint32_t dm = __builtin_amdgcn_perm(kDHi, kDLo, s[d] & 0x07070707u);
    if (d < 4) dl |= dm;
    else dh |= dm;
  }
  return chunk_bits(dl, dh);
}

template <int K, bool VALID>
__global__ void __launch_bounds__(kWG) cgr_stream_kernel(SArgs A) {
  static_assert(K >= 1 && K <= kMaxK, "LDS table");
  constexpr int cells = 1 << (2 * K);
  constexpr uint32_t M = (uint32_t)(cells - 1) << 3;   // cell byte address mask
  constexpr uint32_t SPARE = (uint32_t)cells << 3;      // the spare cells (one per lane: bytes
                                                        // that end no word do not collide)
  constexpr uint32_t kRun = 48 - K;
  // (VALID: the third tile's registers spill; it stays at 2)
  // tiles of bytes in flight per wave: 3 (the next two tiles fetched while
  // this one is counted); the VALID kernel spills at 3 and keeps 2
  constexpr int kDepth = !VALID ? 3 : 2;
  // per wave: start bitmaps of two tiles (this, next) + context; VALID: the
  // validity toggles of the two tiles
  constexpr int kBm = VALID ? 5 : 3;
  __shared__ unsigned long long tab[cells + 64];
  __shared__ uint32_t scb[kWaves * kBm * 64];
  __shared__ uint32_t last;
  for (int i = threadIdx.x; i < cells + 64; i += kWG) tab[i] = 0ull;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: spans, tiles and buffer descriptors stay scalar
  const uint32_t spare = SPARE + 8u * (uint32_t)lane;
  uint32_t *sc = scb + kBm * 64 * wid;
#pragma unroll
  for (int b = 0; b < kBm; ++b) sc[64 * b + lane] = 0u;
  __syncthreads();

  const int32_t b0 = __builtin_amdgcn_readfirstlane(A.idx[0]);
  const int32_t b1 = __builtin_amdgcn_readfirstlane(A.idx[A.num_reads]);
  const int32_t a0 = b0 & ~15;
  const int32_t ns = (int32_t)nspans(a0, b1);
  const int32_t gw = (int32_t)blockIdx.x * kWaves + wid, nwav = (int32_t)gridDim.x * kWaves;
  bool risky = false;

  // one descriptor pair per call: offsets past b1 + slack read zeros without
  // memory traffic (the context loads of tiles that enter no span, the
  // prefetch past a wave's last span); a tile crossing b1 is masked.  The
  // range check is per dword, so a dword straddling b1 still loads
  // (HPGQ_DEVICE_SLACK readable bytes).
  const uint32_t nrec = (uint32_t)b1 + HPGQ_DEVICE_SLACK;
  const uint32_t kPast = nrec;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)A.seq, (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)A.qual, (short)0, nrec, 0x00020000);
  // VALID: span_first_kernel's toggle words 0 .. num_reads / 64
  const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
      (void *)A.toggles, (short)0, VALID ? (uint32_t)((A.num_reads / 64 + 1) * 8) : 0u, 0x00020000);
  // span cursors through the scalar cache (read-only here)
  const __attribute__((address_space(4))) int32_t *sfirst =
      (const __attribute__((address_space(4))) int32_t *)A.span_first;
  uint32_t *scx = sc + 128;   // the context bitmap: starts in the 32 bytes before a span
  uint32_t *tcb = sc + 192;   // VALID: the toggle bitmaps of the two tiles

  // The wave's spans s = gw, gw + nwav, ... form one tile stream: the next
  // tile's bytes, read-start bits and (entering a span) context are fetched
  // while this tile is counted, across span boundaries too, so a span start
  // costs no memory round trip.  The cursor of the next span (rn) is read at
  // span entry and taken over when the span's last tile is scattered.
  if (gw < ns) {
    int32_t s = gw;
    // lane 0 of each: the previous tile's last lane (packed codes 16..31, last
    // quality dwords, V and starts), the "old" operand of wave_shr:1
    uint32_t pp1, pq6, pq7, pv, pS;
    // the run open at the tile start per axis: exact when ekx / eky, else at
    // most 16 (a tile without a candidate chunk) or 15 (a span context
    // whose last 16 bytes hold a Z on both axes), walked back for only when
    // that bound would decide a run
    uint32_t einx = 15, einy = 15;
    bool ekx = false, eky = false;
    // span entry: the 16 bytes before t0 (all 'N' before the batch) and the
    // read starts among the 32 before it; VALID: rv = the read holding byte
    // t0 - 1 (-1: none), the entry state skip_in (1: that read is skipped)
    auto enter = [&](const uint32_t (&cs)[4], const uint32_t (&cq)[2], const uint32_t ps, const int32_t t0,
                     const int32_t rv, uint32_t &skip_in) {
      uint32_t sw[kNdw];
#pragma unroll
      for (int d = 0; d < kNdw; ++d) sw[d] = d < kNdw - 4 ? 0x4E4E4E4Eu : cs[d - (kNdw - 4)];
      const Cls c = classify(sw);
      pp1 = __builtin_amdgcn_readfirstlane(c.p1);
      pq6 = __builtin_amdgcn_readfirstlane(cq[0]);
      pq7 = __builtin_amdgcn_readfirstlane(cq[1]);
      pv = __builtin_amdgcn_readfirstlane(c.v);
      pS = ps;
      einx = einy = 15;
      ekx = eky = false;
      if (!VALID) {
        if (!(c.zhi & 0x01010101u) || !(c.zhi & 0x02020202u)) {
          einx = run_before<0>(A, b0, t0, kRun);
          einy = run_before<1>(A, b0, t0, kRun);
          ekx = eky = true;
        }
        return;
      }
      // VALID: the bound of 15 holds when read rv is valid and its bytes among
      // the 16 hold a Z on both axes (they are the bytes after its start)
      const bool vrd = rv >= 0 && __builtin_amdgcn_readfirstlane(A.status[rv]) == 1;
      skip_in = rv >= 0 && !vrd ? 1u : 0u;
      const uint32_t st = ps >> 16;   // starts among the 16 bytes
      const uint32_t own = st ? (0xFFFFu << (31 - __builtin_clz(st))) & 0xFFFFu : 0xFFFFu;
      uint32_t xb[kNdw], yb[kNdw];
#pragma unroll
      for (int d = 0; d < kNdw; ++d) {
        xb[d] = c.cd[d] & 0x01010101u;
        yb[d] = (c.cd[d] >> 1) & 0x01010101u;
      }
      const uint32_t zx = (c.v & ~byte_bits(xb)) >> 16, zy = (c.v & ~byte_bits(yb)) >> 16;   // Z moves among the 16
      if (!vrd || !(zx & own) || !(zy & own)) {
        einx = run_before_valid<0>(A, t0, rv, kRun);
        einy = run_before_valid<1>(A, t0, rv, kRun);
        ekx = eky = true;
      }
    };
    auto ctx_starts = [&](int32_t &r, int32_t &iw, uint32_t &itg, const int32_t t0) {
      scatter_starts<VALID, false>(A, rt, scx, nullptr, r, iw, itg, t0 - kLaneBytes, t0, lane);
      __builtin_amdgcn_wave_barrier();
      const uint32_t ps = __builtin_amdgcn_readfirstlane(scx[0]);
      __builtin_amdgcn_wave_barrier();
      scx[0] = 0u;
      return ps;
    };
    // mid: runs between the tile's set-up and its table adds (the next tile's
    // start scatter: its LDS read then waits behind the previous tile's adds,
    // long drained, rather than behind this one's).  VALID: sk = the skip
    // state at the tile start, tg = the lane's toggle word, rf = the first read
    // starting in the tile; returns the toggles' parity (the next tile's state
    // is sk ^ parity).
    auto tile = [&](const int32_t t, const int32_t tend, uint32_t (&sw)[kNdw], uint32_t (&qw)[kNdw],
                    const uint32_t so, const uint32_t sk, const uint32_t tg, const int32_t rf, auto &&mid) {
      const int32_t o = t + kLaneBytes * lane;
      if (t < b0 || t + kTile > tend) mask_range(o, b0, tend, sw, qw);   // edge tiles
      uint32_t par = 0;
      bool masked = false;   // VALID: the tile holds skipped bytes
      if (VALID && (sk || __ballot(tg != 0u))) {
        // skip bit of byte j = sk ^ (toggles of the lanes below) ^ (toggles of bytes <= j)
        uint32_t px = tg;
        px ^= px << 1;
        px ^= px << 2;
        px ^= px << 4;
        px ^= px << 8;
        px ^= px << 16;
        const uint64_t bal = __ballot(__builtin_popcount(tg) & 1);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        const uint32_t skip = px ^ (0u - ((below ^ sk) & 1u));
        par = (uint32_t)__popcll(bal) & 1u;
        masked = __ballot(skip != 0u) != 0ull;
        if (masked) mask_skipped(skip, sw, qw);
      }
      const Cls c = classify(sw);
      uint32_t qor = 0;
#pragma unroll
      for (int d = 0; d < kNdw; ++d) qor |= qw[d];
      // flags: unsupported bytes
      if (__ballot(c.bad != 0u || (qor & 0x80808080u) != 0u)) risky = true;
      // runs: a 16-byte chunk without a Z on an axis (VALID: that holds a D
      // move there), or a long run entering the tile
      // (a tile without skipped bytes: any Z-free chunk, as for all reads; with
      // them, only Z-free chunks holding a D move, so that wholly skipped
      // chunks do not trigger)
      const uint32_t zc = chunk_bits(c.zlo, c.zhi);
      bool zfree = zc != 0xFu;
      if (VALID && masked && zfree && __ballot((chunk_bits_d(sw) & ~zc) != 0u)) zfree = run_candidate(c);
      else if (VALID && masked) zfree = false;
      if (__builtin_expect(__ballot(zfree) != 0ull || einx > 16 || einy > 16, 0)) {
        // exact scan; an entering run known only by its bound is walked back
        // for only when the bound would decide (>= kRun - 16 leading D moves)
        auto axis = [&](auto ax, uint32_t &ein, bool &ek) __attribute__((always_inline)) {
          constexpr int AX = decltype(ax)::value;
          const TileRuns tr = tile_runs<AX>(c, ein, kRun);
          if (tr.risky) risky = true;
          if (tr.risky_in) {
            if (!ek) {
              ein = VALID ? run_before_valid<AX>(A, t, rf - 1, kRun) : run_before<AX>(A, b0, t, kRun);
              ek = true;
              if (tile_runs<AX>(c, ein, kRun).risky_in) risky = true;
            } else {
              risky = true;
            }
          }
          if (tr.anyz) {
            ein = tr.out;
            ek = true;
          } else {
            ein = min(ein + tr.out, 1u << 20);
          }
        };
        axis(AxisTag<0>{}, einx, ekx);
        axis(AxisTag<1>{}, einy, eky);
      } else {
        einx = einy = 16;   // (see the header: a tile without a candidate chunk leaves <= 16)
        ekx = eky = false;
      }
      // neighbours (lane 0: the previous tile's last lane / the span context)
      const uint32_t np1 = dpp_shr1(pp1, c.p1);   // the code stream below byte 0
      const uint32_t nq6 = dpp_shr1(pq6, qw[kNdw - 2]), nq7 = dpp_shr1(pq7, qw[kNdw - 1]);
      const uint32_t nv = dpp_shr1(pv, c.v), nS = dpp_shr1(pS, so);
      // emission: bytes [i-K+1, i] all A/C/G/T and no read start in (i-K+1, i]
      uint32_t E;
      {
        // 64-bit frames, high word = this lane's bytes, low word = the
        // previous lane's: V (A/C/G/T) and W = V without read starts.  E bit j
        // = AND over a < K-1 of (W << a) and (V << (K-1)), high words only:
        // hi(X << a) = v_alignbit(Xh, Xl, 32 - a)
        const uint32_t wh = c.v & ~so, wl = nv & ~nS;
        E = K == 1 ? c.v : wh & __builtin_amdgcn_alignbit(c.v, nv, 32 - (K - 1));
#pragma unroll
        for (int a = 1; a < K - 1; ++a) E &= __builtin_amdgcn_alignbit(wh, wl, 32 - a);
      }
      // the quality sum at the previous lane's last byte
      uint32_t acc = 0;
      // (v_sad_u8 sums the previous lane's last K quality bytes, 4 per op)
      if (K > 4)
        acc = __builtin_amdgcn_sad_u8(nq7, 0u, __builtin_amdgcn_sad_u8(nq6 & (0xFFFFFFFFu << (8 * (8 - K))), 0u, 0u));
      else
        acc = __builtin_amdgcn_sad_u8(nq7 & (0xFFFFFFFFu << (8 * (4 - K))), 0u, 0u);
      mid();
      // one ds_add_u64 per byte: count | quality sum << 32 (spare cell: no word)
      // the word ending at byte j: codes of bytes j-K+1..j (oldest at bits 0-1)
      // from the 96-bit stream np1:p0:p1 (byte i at bit 2(i + 16)), cut out by
      // one v_alignbit at the cell's byte offset (x 8), then masked
#pragma unroll
      for (int j = 0; j < kLaneBytes; ++j) {
        const int sh = 2 * j + 29 - 2 * (K - 1);   // stream bit of byte j-K+1, less 3
        const uint32_t win = sh < 32 ? __builtin_amdgcn_alignbit(c.p0, np1, sh)
                           : sh < 64 ? __builtin_amdgcn_alignbit(c.p1, c.p0, sh - 32)
                                     : c.p1 >> (sh - 64);
        const uint32_t w = win & M;   // M: the cell byte-address mask
        const int jo = j - K;   // the byte leaving the quality window
        {
          const uint32_t qold = jo >= 0 ? __builtin_amdgcn_ubfe(qw[jo >> 2], 8 * (jo & 3), 8)
                                        : __builtin_amdgcn_ubfe(jo + kLaneBytes < kLaneBytes - 4 ? nq6 : nq7, 8 * (jo & 3), 8);
          acc = acc + __builtin_amdgcn_ubfe(qw[j >> 2], 8 * (j & 3), 8) - qold;
        }
        // addr = E bit j ? w : spare (v_bfe_i32 + v_bitop3; left to itself the
        // compiler spends three instructions on it)
        const uint32_t e = (uint32_t)__builtin_amdgcn_sbfe((int)E, j, 1);
        const uint32_t addr = __builtin_amdgcn_bitop3_b32(e, w, spare, 0xCA);   // e ? w : spare
        const unsigned long long inc = ((unsigned long long)acc << 32) | 1ull;
        atomicAdd(reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(tab) + addr), inc);
      }
      // carry the last lane to the next tile's lane 0
      // (rotated by one lane: lane 0 holds lane 63's, the "old" operand of
      // the next tile's wave_shr:1)
      pp1 = dpp_ror1(c.p1);
      pq6 = dpp_ror1(qw[kNdw - 2]);
      pq7 = dpp_ror1(qw[kNdw - 1]);
      pv = dpp_ror1(c.v);
      pS = dpp_ror1(so);
      return par;
    };
    int32_t tA = (int32_t)(a0 + ((int64_t)s << kSpanLog)), tB;
    int32_t eA = (int32_t)min((int64_t)tA + kSpan, (int64_t)b1), eB;
    int32_t r = sfirst[s];
    int32_t rn = sfirst[min(s + nwav, ns - 1)];
    uint32_t itg = 0;
    int32_t iw = idx_window_raw<VALID>(A, rt, r, lane, itg);
    uint32_t skA = 0, skB = 0;   // VALID: skip state at the tile starts
    {
      uint32_t cs[4] = {0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu}, cq[2] = {0u, 0u};
      if (s != 0) {   // spans after the first start >= 16 KB past b0
        const v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)tA - 16u, 0, 0);
        const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rq, (uint32_t)tA - 8u, 0, 0);
        cs[0] = a[0]; cs[1] = a[1]; cs[2] = a[2]; cs[3] = a[3];
        cq[0] = q[0]; cq[1] = q[1];
      }
      const uint32_t ps = ctx_starts(r, iw, itg, tA);
      enter(cs, cq, ps, tA, r - 1, skA);
    }
    uint32_t sA[kNdw], qA[kNdw], sB[kNdw], qB[kNdw], soA, soB, tgA = 0, tgB = 0;
    int32_t rfA = r, rfB = 0;   // VALID: the first read starting in the tile
    scatter_starts<VALID, VALID>(A, rt, sc, tcb, r, iw, itg, tA, tA + kTile, lane, tA + kTile >= eA, rn);
    soA = take_bits(&sc[lane]);
    if (VALID) tgA = take_bits(&tcb[lane]);
    load32(rs, (uint32_t)(tA + kLaneBytes * lane), sA);
    load32(rq, (uint32_t)(tA + kLaneBytes * lane), qA);
    // the load cursor (wave-uniform) walks the same tile stream one tile
    // ahead of the start cursor: tile z = y's successor is fetched while x is
    // counted, so a tile's bytes have two tiles' work to arrive
    int32_t ls = s, lt = tA, le = eA;
    bool lfin = false;
    auto lnext = [&] {
      if (lfin) return;
      lt += kTile;
      if (lt >= le) {
        ls += nwav;
        if (ls < ns) {
          lt = (int32_t)(a0 + ((int64_t)ls << kSpanLog));
          le = (int32_t)min((int64_t)lt + kSpan, (int64_t)b1);
        } else {
          lfin = true;
        }
      }
    };
    uint32_t sC[kNdw], qC[kNdw], soC, tgC = 0, skC = 0;
    int32_t tC, eC, rfC = 0;
    if constexpr (kDepth == 3) {
      lnext();
      load32(rs, lfin ? kPast : (uint32_t)(lt + kLaneBytes * lane), sB);
      load32(rq, lfin ? kPast : (uint32_t)(lt + kLaneBytes * lane), qB);
    }
    // count tile x while fetching tile y (straight-line: the loads are
    // unconditional, so the compiler counts the loads in flight exactly and
    // a tile waits only for its own bytes); false past the wave's last tile.
    // (kDepth 3: y's bytes are in flight already; the loads go to z)
    auto half = [&](const int32_t tx, const int32_t ex, uint32_t (&sx)[kNdw], uint32_t (&qx)[kNdw], const uint32_t sox,
                    const uint32_t skx, const uint32_t tgx, const int32_t rfx, uint32_t *scpy, uint32_t *tcpy,
                    int32_t &ty, int32_t &ey, uint32_t (&sy)[kNdw], uint32_t (&qy)[kNdw], uint32_t &soy,
                    uint32_t &sky, uint32_t &tgy, int32_t &rfy, uint32_t (&sz)[kNdw], uint32_t (&qz)[kNdw]) {
      ty = tx + kTile;
      ey = ex;
      bool entering = false, fin = false;
      uint32_t psn = 0;
      if (ty >= ex) {   // x is its span's last tile: y is the next span's first
        s += nwav;
        if (s < ns) {
          ty = (int32_t)(a0 + ((int64_t)s << kSpanLog));
          ey = (int32_t)min((int64_t)ty + kSpan, (int64_t)b1);
          entering = true;
          rn = sfirst[min(s + nwav, ns - 1)];
          psn = ctx_starts(r, iw, itg, ty);
        } else {
          fin = true;
        }
      }
      const int32_t rv = r - 1;   // entering: the read holding byte ty - 1
      const v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs, entering ? (uint32_t)ty - 16u : kPast, 0, 0);
      const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rq, entering ? (uint32_t)ty - 8u : kPast, 0, 0);
      if constexpr (kDepth == 3) {
        lnext();
        const uint32_t oz = lfin ? kPast : (uint32_t)(lt + kLaneBytes * lane);
        load32(rs, oz, sz);
        load32(rq, oz, qz);
      } else {
        const uint32_t oy = fin ? kPast : (uint32_t)(ty + kLaneBytes * lane);
        load32(rs, oy, sy);
        load32(rq, oy, qy);
      }
      const uint32_t par = tile(tx, ex, sx, qx, sox, skx, tgx, rfx, [&] {
        rfy = r;
        scatter_starts<VALID, VALID>(A, rt, scpy, tcpy, r, iw, itg, ty, fin ? INT32_MIN : ty + kTile, lane,
                                     ty + kTile >= ey, rn);
        soy = take_bits(&scpy[lane]);
        if (VALID) tgy = take_bits(&tcpy[lane]);
      });
      if (fin) return false;
      sky = skx ^ par;
      if (entering) {
        const uint32_t cs[4] = {a[0], a[1], a[2], a[3]}, cq[2] = {q[0], q[1]};
        enter(cs, cq, psn, ty, rv, sky);
      }
      return true;
    };
    if constexpr (kDepth == 3) {
    // (the start bitmaps alternate between the two halves of sc / tcb: tile x
    // reads its own before scattering y's into the other)
    for (;;) {
      if (!half(tA, eA, sA, qA, soA, skA, tgA, rfA, sc + 64, tcb + 64, tB, eB, sB, qB, soB, skB, tgB, rfB, sC, qC)) break;
      if (!half(tB, eB, sB, qB, soB, skB, tgB, rfB, sc, tcb, tC, eC, sC, qC, soC, skC, tgC, rfC, sA, qA)) break;
      if (!half(tC, eC, sC, qC, soC, skC, tgC, rfC, sc + 64, tcb + 64, tA, eA, sA, qA, soA, skA, tgA, rfA, sB, qB)) break;
      if (!half(tA, eA, sA, qA, soA, skA, tgA, rfA, sc, tcb, tB, eB, sB, qB, soB, skB, tgB, rfB, sC, qC)) break;
      if (!half(tB, eB, sB, qB, soB, skB, tgB, rfB, sc + 64, tcb + 64, tC, eC, sC, qC, soC, skC, tgC, rfC, sA, qA)) break;
      if (!half(tC, eC, sC, qC, soC, skC, tgC, rfC, sc, tcb, tA, eA, sA, qA, soA, skA, tgA, rfA, sB, qB)) break;
    }
    } else {
    for (;;) {
      if (!half(tA, eA, sA, qA, soA, skA, tgA, rfA, sc + 64, tcb + 64, tB, eB, sB, qB, soB, skB, tgB, rfB, sA, qA)) break;
      if (!half(tB, eB, sB, qB, soB, skB, tgB, rfB, sc, tcb, tA, eA, sA, qA, soA, skA, tgA, rfA, sB, qB)) break;
    }
    }
  }
  if (__ballot(risky) && lane == 0) atomicOr(A.gate, GATE_EXACT);
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += kWG) {
    const unsigned long long v = tab[i];
    if (v) atomicAdd(&A.scratch[i], v);
  }
  // the last workgroup moves the scratch table into the reference layout
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(A.done, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  // acquire: this CU's L1 is invalidated, the loads below see the other
  // workgroups' adds (performed at L2) and independent loads stay pipelined
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const bool exact = (__hip_atomic_load(A.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GATE_EXACT) != 0u;
  unsigned long long cnt = 0;
  constexpr int kPer = (cells + kWG - 1) / kWG;
  unsigned long long vals[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x + u * kWG;
    vals[u] = i < cells ? A.scratch[i] : 0ull;
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x + u * kWG;
    const unsigned long long v = vals[u];
    if (!v) continue;
    A.scratch[i] = 0ull;
    if (exact) continue;
    // code bits 2b / 2b+1 = x / y of the base K-1-b steps back (the oldest at
    // b = 0); the newest is the MSB of co_x / co_y, so bit b of co_x is x of b
    uint32_t cx = 0, cy = 0;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      cx |= ((uint32_t)(i >> (2 * b)) & 1u) << b;
      cy |= ((uint32_t)(i >> (2 * b + 1)) & 1u) << b;
    }
    const uint32_t cn = (uint32_t)v, q = (uint32_t)(v >> 32);
    const uint32_t cell = (cx << K) | cy;
    A.ts[cell] += cn;
    A.tq[cell] += q - cn * A.base_quality * (uint32_t)K;
    cnt += cn;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0 && cnt) atomicAdd(A.words, cnt);
}

}  // namespace stream
}  // namespace cgr
}  // namespace hpgq
