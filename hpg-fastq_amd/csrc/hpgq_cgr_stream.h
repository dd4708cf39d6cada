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
// Layout: the bytes [idx[0], idx[n]) are cut into spans of kSpan bytes; a
// wave takes a span as 16 tiles of 1 KB, a lane 16 contiguous bytes of seq
// and of quality per tile (one 16-byte load each, fully coalesced).  The K-1
// bytes of context come from the neighbouring lane by DPP (lane 0: the last
// lane of the previous tile, or a broadcast load at the span start).  Read
// starts inside a tile are scattered into a per-wave LDS bitmap from the
// read offsets the wave walks with a cursor.  Words go to the workgroup's
// LDS table (u64 per cell: count | quality sum << 32, one ds_add_u64 per
// byte; a byte that ends no word adds to a spare cell), flushed to a global
// u64 scratch table that the finalize kernel moves into the reference
// layout.  A run of >= kRun D-moves covers >= 32 whole bytes, so it contains
// a 16-byte lane with no Z on that axis: only tiles holding such a lane (or
// entered with a long open run) are scanned exactly, lane by lane.
#pragma once

namespace hpgq {
namespace cgr {
namespace stream {

constexpr int kWaves = 16;
constexpr int kWG = kWaves * 64;
constexpr int kTile = 1024;                  // bytes per wave tile: 64 lanes x 16
constexpr int kSpanTiles = 16;
constexpr int kSpan = kTile * kSpanTiles;    // bytes per span (16 KB)
constexpr int kMaxK = 7;                     // 4^7 u64 cells = 128 KB of LDS
constexpr int64_t kMaxSpans = ((int64_t)1 << 31) / kSpan + 2;

constexpr uint32_t GATE_EXACT = 1;   // the exact kernels must run

// byte & 7 -> per-byte LUTs (v_perm_b32, codes A=1 C=3 T=4 N=6 G=7)
constexpr uint32_t kXYLo = 0x00000800u;   // code << 3, code = x | y << 1: A 1, C 0
constexpr uint32_t kXYHi = 0x10000018u;   //                               T 3, G 2
constexpr uint32_t kVLo = 0xFF00FF00u;    // 0xFF for A/C/G/T, 0 for N
constexpr uint32_t kVHi = 0xFF0000FFu;
constexpr uint32_t kZLo = 0x03000200u;    // bit0: a Z move on x (C/G), bit1: on y (A/C)
constexpr uint32_t kZHi = 0x01000000u;

struct SArgs {
  const char *seq, *qual;
  const int32_t *idx;
  int64_t num_reads;
  uint32_t base_quality;
  int32_t *span_first;              // [kMaxSpans] first read with idx[r] >= span start - 16
  unsigned long long *scratch;      // [4^K] count | quality sum << 32
  uint32_t *gate;                   // GATE_EXACT when the batch needs the exact path
  uint32_t *ts, *tq;                // final tables [dim][dim]
  unsigned long long *words;
};

__device__ __forceinline__ int32_t batch_lo(const SArgs &A) {
  return __builtin_amdgcn_readfirstlane(A.idx[0]);
}
__device__ __forceinline__ int32_t batch_hi(const SArgs &A) {
  return __builtin_amdgcn_readfirstlane(A.idx[A.num_reads]);
}

// spans start at a0 = idx[0] rounded down to 16 bytes
__device__ __forceinline__ int64_t nspans(int32_t a0, int32_t b1) {
  return b1 > a0 ? ((int64_t)b1 - a0 + kSpan - 1) / kSpan : 0;
}

// span_first[s] = the first read r with idx[r] >= a0 + s*kSpan - 16: thread r
// writes the spans whose (start - 16) lies in (idx[r-1], idx[r]]
__global__ void __launch_bounds__(256) span_first_kernel(SArgs A) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r > A.num_reads) return;
  const int32_t b0 = A.idx[0], b1 = A.idx[A.num_reads];
  const int32_t a0 = b0 & ~15;
  const int64_t ns = nspans(a0, b1);
  const int64_t hi = (int64_t)A.idx[r] + 16 - a0;   // s*kSpan <= hi
  const int64_t lo = r == 0 ? -1 : (int64_t)A.idx[r - 1] + 16 - a0;   // s*kSpan > lo
  int64_t s0 = lo < 0 ? 0 : lo / kSpan + 1;
  int64_t s1 = hi < 0 ? -1 : hi / kSpan;
  if (r == A.num_reads) s1 = ns - 1;   // spans past the last start: the end sentinel
  for (int64_t s = s0; s <= s1 && s < ns; ++s) A.span_first[s] = (int32_t)r;
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {   // lane l <- lane l-1
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// sum of the 4 bytes of x (v_sad_u8 against 0) plus c
__device__ __forceinline__ uint32_t sad4(uint32_t x, uint32_t c) {
  return __builtin_amdgcn_sad_u8(x, 0u, c);
}

// 16 bytes of seq: LUT lookups, exactness and per-lane summaries
struct Cls {
  uint32_t xy[4];   // per byte: (x | y << 1) << 3
  uint32_t v;       // bit j: byte j is A/C/G/T
  uint32_t zany;    // OR of per-byte Z bits (bit0 x, bit1 y) over the bytes
  uint32_t bad;     // nonzero: a byte that is not exactly A/C/G/T/N
};

__device__ __forceinline__ Cls classify(const uint32_t s[4]) {
  Cls c;
  uint32_t bad = 0, z = 0, v0 = 0, v1 = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t code = s[d] & 0x07070707u;
    bad |= s[d] ^ __builtin_amdgcn_perm(hpgq::cgr::kExHi, hpgq::cgr::kExLo, code);
    c.xy[d] = __builtin_amdgcn_perm(kXYHi, kXYLo, code);
    z |= __builtin_amdgcn_perm(kZHi, kZLo, code);
    // gather the V bit of byte j to bit j: byte values 1,2,4,8 (<< 4 for the odd dword), summed
    const uint32_t vb = __builtin_amdgcn_perm(kVHi, kVLo, code) & ((d & 1) ? 0x80402010u : 0x08040201u);
    if (d < 2) v0 = sad4(vb, v0);
    else v1 = sad4(vb, v1);
  }
  c.v = v0 | (v1 << 8);
  c.zany = z;
  c.bad = bad;
  return c;
}

// per-lane run summary of one axis over its 16 bytes (rare path)
struct RunSum {
  uint32_t pfx, sfx, cnt, hz;
};

template <int AX>
__device__ __forceinline__ RunSum run_sum(const Cls &c) {
  RunSum r = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (!((c.v >> j) & 1u)) continue;
    const uint32_t d = (c.xy[j >> 2] >> (8 * (j & 3) + 3 + AX)) & 1u;
    if (d) {
      ++r.cnt;
      ++r.sfx;
      if (!r.hz) ++r.pfx;
    } else {
      r.hz = 1;
      r.sfx = 0;
    }
  }
  return r;
}

// exact run scan of one tile on one axis: runs enter with ein, returns the
// run open at the tile end; risky |= a run >= run_max
template <int AX>
__device__ uint32_t scan_tile(const Cls &c, uint32_t ein, uint32_t run_max, bool &risky) {
  const RunSum rs = run_sum<AX>(c);
  const uint32_t packed = rs.pfx | (rs.sfx << 8) | (rs.cnt << 16) | (rs.hz << 24);
  uint32_t run = ein;
  for (int l = 0; l < 64; ++l) {
    const uint32_t p = __builtin_amdgcn_readlane(packed, l);
    const uint32_t pfx = p & 0xFF, sfx = (p >> 8) & 0xFF, cnt = (p >> 16) & 0xFF;
    if (p >> 24) {
      if (run + pfx >= run_max) risky = true;
      run = sfx;
    } else {
      run += cnt;
    }
    if (run >= run_max) risky = true;
    run = min(run, 1u << 20);
  }
  return run;
}

// the run open at byte `at` on axis AX (capped at run_max), walking back from
// it; rare: only for tiles that need the exact scan
template <int AX>
__device__ uint32_t run_before(const SArgs &A, int32_t b0, int32_t at, uint32_t run_max) {
  uint32_t run = 0;
  for (int32_t p = at - 1; p >= b0 && run < run_max; --p) {
    const uint8_t ch = (uint8_t)A.seq[p];
    const bool mv = ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T';
    if (!mv) continue;   // N (other bytes set the gate in their own tile)
    const bool d = AX == 0 ? (ch == 'A' || ch == 'T') : (ch == 'G' || ch == 'T');
    if (!d) break;
    ++run;
  }
  return run;
}

// read starts in [base, base + 16*64): bits into the wave's LDS bitmap sc[64],
// advancing the cursor r past them
__device__ __forceinline__ void scatter_starts(const SArgs &A, uint32_t *sc, int64_t &r,
                                               int32_t base, int32_t limit, int lane) {
  for (;;) {
    const int64_t j = r + lane;
    const int32_t iw = j <= A.num_reads ? A.idx[j] : 0x7FFFFFFF;
    const bool in = iw < limit;
    const unsigned long long b = __ballot(in);
    const uint32_t o = (uint32_t)(iw - base);
    if (in && o < 16u * 64u) atomicOr(&sc[o >> 4], 1u << (o & 15));   // o < 1024 unless idx is unsorted
    const int c = __popcll(b);
    r += c;
    if (c < 64) break;
  }
}

template <int K>
__global__ void __launch_bounds__(kWG) cgr_stream_kernel(SArgs A) {
  static_assert(K >= 1 && K <= kMaxK, "LDS table");
  constexpr int cells = 1 << (2 * K);
  constexpr uint32_t M = (uint32_t)(cells - 1) << 3;   // cell byte address mask
  constexpr uint32_t SPARE = (uint32_t)cells << 3;      // the spare cell
  constexpr uint32_t kRun = 48 - K;
  extern __shared__ __attribute__((aligned(16))) unsigned long long tab[];   // cells + 1, then sc
  uint32_t *scb = reinterpret_cast<uint32_t *>(tab + cells + 1);
  for (int i = threadIdx.x; i < cells + 1; i += kWG) tab[i] = 0ull;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t *sc = scb + 64 * wid;
  sc[lane] = 0u;
  __syncthreads();

  const int32_t b0 = batch_lo(A), b1 = batch_hi(A);
  const int32_t a0 = b0 & ~15;
  const int64_t ns = nspans(a0, b1);
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wid, nwav = (int64_t)gridDim.x * kWaves;
  // the range check is per dword: a dword that straddles b1 must still load
  // (HPGQ_DEVICE_SLACK readable bytes past the data; bytes >= b1 are masked)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)A.seq, (short)0, b1 + HPGQ_DEVICE_SLACK, 0x00020000);
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc((void *)A.qual, (short)0, b1 + HPGQ_DEVICE_SLACK, 0x00020000);
  bool risky = false;

  for (int64_t s = gw; s < ns; s += nwav) {
    const int32_t t0 = a0 + (int32_t)(s * kSpan);
    const int32_t tend = (int32_t)min((int64_t)t0 + kSpan, (int64_t)b1);
    int64_t r = A.span_first[s];
    // ---- context: the 16 bytes before the span, the same on every lane
    uint32_t pxy2, pxy3, pq2, pq3, pv, pS;
    // the run open at the tile start per axis: exact when eknown, else at
    // most 15 (the last 16 bytes hold a Z on both axes) and walked back for
    // only when a tile needs the exact scan
    uint32_t einx = 15, einy = 15;
    bool eknown = false;
    {
      const int32_t c0 = t0 - 16;
      v4u sv = {0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu};   // 'N': no move, no word
      v4u qv = {0u, 0u, 0u, 0u};
      if (c0 >= b0) {
        sv = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)c0, 0, 0);
        qv = __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)c0, 0, 0);
      } else if (t0 > b0) {   // partly before the batch: byte-wise
        uint32_t w[4] = {0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu}, q[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int32_t p = c0 + j;
          if (p < b0) continue;
          const uint32_t sh = 8 * (j & 3);
          w[j >> 2] = (w[j >> 2] & ~(0xFFu << sh)) | ((uint32_t)(uint8_t)A.seq[p] << sh);
          q[j >> 2] |= (uint32_t)(uint8_t)A.qual[p] << sh;
        }
        sv = v4u{w[0], w[1], w[2], w[3]};
        qv = v4u{q[0], q[1], q[2], q[3]};
      }
      const uint32_t sa[4] = {sv[0], sv[1], sv[2], sv[3]};
      const Cls c = classify(sa);
      pxy2 = c.xy[2];
      pxy3 = c.xy[3];
      pq2 = qv[2];
      pq3 = qv[3];
      pv = c.v;
      if (c.bad || ((qv[0] | qv[1] | qv[2] | qv[3]) & 0x80808080u)) risky = true;
      // read starts in [c0, t0)
      scatter_starts(A, sc, r, c0, t0, lane);
      __builtin_amdgcn_wave_barrier();
      pS = __builtin_amdgcn_readfirstlane(sc[0]);
      __builtin_amdgcn_wave_barrier();
      sc[0] = 0u;
      if (!(c.zany & 0x01010101u) || !(c.zany & 0x02020202u)) {
        einx = run_before<0>(A, b0, t0, kRun);
        einy = run_before<1>(A, b0, t0, kRun);
        eknown = true;
      }
    }
    // ---- tiles
    for (int32_t t = t0; t < tend; t += kTile) {
      const int32_t o = t + 16 * lane;
      v4u sv = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)o, 0, 0);
      v4u qv = __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)o, 0, 0);
      scatter_starts(A, sc, r, t, t + kTile, lane);
      uint32_t sw[4] = {sv[0], sv[1], sv[2], sv[3]};
      uint32_t qw[4] = {qv[0], qv[1], qv[2], qv[3]};
      if (t < b0 || t + kTile > tend) {   // edge tile: bytes outside [b0, b1) -> 'N', quality 0
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int32_t p = o + j;
          if (p >= b0 && p < b1 && p < tend) continue;
          const uint32_t sh = 8 * (j & 3);
          sw[j >> 2] = (sw[j >> 2] & ~(0xFFu << sh)) | (0x4Eu << sh);
          qw[j >> 2] &= ~(0xFFu << sh);
        }
      }
      const Cls c = classify(sw);
      __builtin_amdgcn_wave_barrier();
      const uint32_t so = sc[lane];
      __builtin_amdgcn_wave_barrier();
      sc[lane] = 0u;
      // flags: unsupported bytes
      if (__ballot(c.bad != 0u || ((qw[0] | qw[1] | qw[2] | qw[3]) & 0x80808080u) != 0u)) risky = true;
      // runs: a lane without a Z on an axis, or a long run entering the tile
      const bool zfree = !(c.zany & 0x01010101u) || !(c.zany & 0x02020202u);
      if (__builtin_expect(__ballot(zfree) != 0ull || einx > 16 || einy > 16, 0)) {
        if (!eknown) {
          einx = run_before<0>(A, b0, t, kRun);
          einy = run_before<1>(A, b0, t, kRun);
        }
        einx = scan_tile<0>(c, einx, kRun, risky);
        einy = scan_tile<1>(c, einy, kRun, risky);
        eknown = true;
      } else {
        einx = einy = 15;
        eknown = false;
      }
      // neighbours (lane 0: the previous tile's last lane / the span context)
      const uint32_t nxy2 = dpp_shr1(pxy2, c.xy[2]), nxy3 = dpp_shr1(pxy3, c.xy[3]);
      const uint32_t nq2 = dpp_shr1(pq2, qw[2]), nq3 = dpp_shr1(pq3, qw[3]);
      const uint32_t nv = dpp_shr1(pv, c.v), nS = dpp_shr1(pS, so);
      // emission: bytes [i-K+1, i] all A/C/G/T and no read start in (i-K+1, i]
      const uint32_t V32 = nv | (c.v << 16), S32 = nS | (so << 16);
      uint32_t E;
      {
        const uint32_t W = V32 & ~S32;
        uint32_t R = W;
        int have = 1;
#pragma unroll
        for (int step = 0; step < 4; ++step) {
          if (have < K - 1) {
            const int sh = have < K - 1 - have ? have : K - 1 - have;
            R &= R << sh;
            have += sh;
          }
        }
        E = (K == 1 ? V32 : R & (V32 << (K - 1))) >> 16;
      }
      // the code window and the quality sum at byte 15 of the previous lane
      uint32_t w = 0, acc = 0;
#pragma unroll
      for (int j = 16 - (K - 1); j < 16; ++j) {
        const uint32_t xw = j < 12 ? nxy2 : nxy3;
        w = (w << 2) | __builtin_amdgcn_ubfe(xw, 8 * (j & 3), 5);
      }
#pragma unroll
      for (int j = 16 - K; j < 16; ++j) {
        const uint32_t qx = j < 12 ? nq2 : nq3;
        acc += __builtin_amdgcn_ubfe(qx, 8 * (j & 3), 8);
      }
      // one ds_add_u64 per byte: count | quality sum << 32 (spare cell: no word)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        w = (w << 2) | __builtin_amdgcn_ubfe(c.xy[j >> 2], 8 * (j & 3), 5);
        const int jo = j - K;   // the byte leaving the quality window
        const uint32_t qold = jo >= 0 ? __builtin_amdgcn_ubfe(qw[jo >> 2], 8 * (jo & 3), 8)
                                      : __builtin_amdgcn_ubfe(jo + 16 < 12 ? nq2 : nq3, 8 * ((jo + 16) & 3), 8);
        acc = acc + __builtin_amdgcn_ubfe(qw[j >> 2], 8 * (j & 3), 8) - qold;
        const uint32_t e = (uint32_t)__builtin_amdgcn_sbfe((int)E, j, 1);
        const uint32_t addr = (e & w & M) | (~e & SPARE);
        const unsigned long long inc = ((unsigned long long)acc << 32) | 1ull;
        atomicAdd(reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(tab) + addr), inc);
      }
      // carry the last lane to the next tile's lane 0
      pxy2 = __builtin_amdgcn_readlane(c.xy[2], 63);
      pxy3 = __builtin_amdgcn_readlane(c.xy[3], 63);
      pq2 = __builtin_amdgcn_readlane(qw[2], 63);
      pq3 = __builtin_amdgcn_readlane(qw[3], 63);
      pv = __builtin_amdgcn_readlane(c.v, 63);
      pS = __builtin_amdgcn_readlane(so, 63);
    }
  }
  if (__ballot(risky) && lane == 0) atomicOr(A.gate, GATE_EXACT);
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += kWG) {
    const unsigned long long v = tab[i];
    if (v) atomicAdd(&A.scratch[i], v);
  }
}

// scratch (code order) -> the reference's tables [co_x][co_y], or just clear
// it when the gate sends the batch to the exact path
template <int K>
__global__ void __launch_bounds__(256) cgr_stream_finalize_kernel(SArgs A) {
  constexpr int cells = 1 << (2 * K);
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool exact = (*A.gate & GATE_EXACT) != 0u;
  unsigned long long cnt = 0;
  if (i < cells) {
    const unsigned long long v = A.scratch[i];
    A.scratch[i] = 0ull;
    if (!exact && v) {
      // code bits 2a / 2a+1 = x / y of the base `a` steps back; the newest is
      // the MSB of co_x / co_y
      uint32_t cx = 0, cy = 0;
#pragma unroll
      for (int a = 0; a < K; ++a) {
        cx |= ((uint32_t)(i >> (2 * a)) & 1u) << (K - 1 - a);
        cy |= ((uint32_t)(i >> (2 * a + 1)) & 1u) << (K - 1 - a);
      }
      const uint32_t c = (uint32_t)v, q = (uint32_t)(v >> 32);
      const uint32_t cell = (cx << K) | cy;
      A.ts[cell] += c;
      A.tq[cell] += q - c * A.base_quality * (uint32_t)K;
      cnt = c;
    }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(A.words, cnt);
}

}  // namespace stream
}  // namespace cgr
}  // namespace hpgq
