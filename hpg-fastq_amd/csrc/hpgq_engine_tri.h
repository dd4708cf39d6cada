// hpgq_engine_tri.h — FAST single-end stats/filter kernel, three reads per wave.
//
// Same contract and outputs as engine_kernel<1, *, false> (hpgq_engine_kernel.h)
// for batches whose reads are at most 160 bases: the per-read fixed cost (the
// DPP reduction, the pass/fail decision, bookkeeping) is shared by three reads
// and lane utilisation goes from 38/64 to 57/64 at 150 bp.  The kernel is
// VALU-issue bound (PMC: ~80% VALU busy at 13.9 Greads/s with the previous
// per-position field scheme), so everything below counts VALU instructions
// (15.3 Greads/s with this one at 5 waves/SIMD).
//
//   * the wave is cut into 3 segments of 21 lanes (lanes 20, 41, 62, 63 own no
//     positions); segment k works on read 3t + k of the block and lane ls < 20
//     of a segment owns positions 8ls..8ls+7 (160 per read).
//   * the block prologue writes one 16-byte record per read (dword-aligned seq
//     and qual offsets, length | alignments) into a per-wave LDS table; each
//     lane fetches its segment's record with ONE ds_read_b128, issues ONE
//     buffer_load_dwordx2 per buffer and realigns with DPP wave_shl:1 +
//     v_alignbyte (UNAL = true loads unaligned windows instead: fewer VALU,
//     but measured ~15% slower in the address/data path).  The SRDs cover
//     data_end + 8 bytes (the slack the C-ABI requires of device buffers).
//   * base classification: code = byte & 7 (one-to-one on A,C,G,T,N; masked
//     bytes -> 0), then three v_perm_b32 LUTs: the expected byte (exact-match
//     check; lowercase / IUPAC / other bytes take a rare path and count as
//     "other"), C|G<<4 and A|T<<4 nibble one-hots.  G+C per read = popcount of
//     the C|G word.  N is not counted: the workgroup epilogue derives it as
//     count - A - C - G - T - other, count from the length histogram.
//   * nibble counters (<= 15 triples) are widened into 8-bit per-base counters
//     (<= 255 triples) and those flushed to LDS u32 arrays (ds_add); quality
//     sums are 16-bit pairs.
//   * per-read sums (raw quality | G+C << 18) use ONE inclusive DPP prefix scan
//     for the three segments; lanes 20, 41, 62 store the segment ends to LDS
//     (no wait) and the block epilogue takes differences.
//   * every read is accumulated; the epilogue decides pass/fail for the block
//     vectorised over lanes and takes the failed reads back out.
// The stats layout, histogram rules and workgroup epilogue are identical, so
// the two kernels are interchangeable (the tests run both against the oracle).
#pragma once
#include "hpgq_engine_kernel.h"

namespace hpgq {

constexpr int kTriW = 21;       // lanes per segment
constexpr int kTriPos = 160;    // positions per segment (20 owning lanes x 8)
constexpr int kTriBlock = 54;   // reads per block (18 triples)
constexpr int kTriU = 3;        // triples per pipeline group (6 groups per full block)
constexpr int kTriSlack = 8;    // readable bytes past the data end the loads may touch
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

struct TriPending {
  v2u s, q;        // the lane's 8 bytes of seq / quality (raw dwords if aligned loads)
  uint32_t n;      // its read's length (| als << 16 | alq << 20 if aligned loads)
};

__device__ __forceinline__ uint32_t next_lane0(uint32_t v) {   // lane i <- lane i+1, lane 63 <- 0
  return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true);
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

// masks of the lane's two words: bytes at positions < n (nv = n - p0)
__device__ __forceinline__ void tri_masks(int nv, uint32_t &m0, uint32_t &m1) {
  const int e = 32 - 8 * nv;   // right shift of 0x00000000FFFFFFFF giving m0
  const uint64_t ones = 0xFFFFFFFFull;
  m0 = (uint32_t)(ones >> min(max(e, 0), 32));
  m1 = (uint32_t)(ones >> min(max(e + 32, 0), 32));
}

// 0xFF in every byte of d that is non-zero
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t d) {
  const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
  return (nz >> 7) * 0xFFu;
}

struct TriAcc {
  uint32_t n4[2][2];   // [word][C|G<<4, A|T<<4]: nibble per position
  uint32_t c8[2][4];   // [word][A, C, G, T]: byte per position
  uint32_t q02[2], q13[2];   // quality 16-bit pairs (positions 0,2 / 1,3 of the word)
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      n4[w][0] = n4[w][1] = 0;
      c8[w][0] = c8[w][1] = c8[w][2] = c8[w][3] = 0;
      q02[w] = q13[w] = 0;
    }
  }
  // nibbles -> bytes (every <= 15 triples and before any subtraction)
  __device__ __forceinline__ void widen() {
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      c8[w][1] += n4[w][0] & 0x0F0F0F0Fu;
      c8[w][2] += (n4[w][0] >> 4) & 0x0F0F0F0Fu;
      c8[w][0] += n4[w][1] & 0x0F0F0F0Fu;
      c8[w][3] += (n4[w][1] >> 4) & 0x0F0F0F0Fu;
      n4[w][0] = n4[w][1] = 0;
    }
  }
  // bytes -> LDS (pos_acc [6][lmax]: qsum, A, C, G, T, N/other); nibbles empty
  __device__ __forceinline__ void flush(uint32_t *pos_acc, int lmax, int p0) {
#pragma unroll
    for (int w = 0; w < 2; ++w) {
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
  const uint32_t ex = __builtin_amdgcn_perm(kX7Hi, kX7Lo, codes);
  const uint32_t ff = nonzero_bytes((s ^ ex) & m);
  if (ff) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (((ff >> (8 * i)) & 1u) && pos0 + i < lmax) atomicAdd(&other[pos0 + i], sign);
  }
  return codes & ~ff;
}

template <bool B>
struct TriTag {
  static constexpr bool value = B;
};
using AddTag = TriTag<false>;
using SubTag = TriTag<true>;

// MINW: minimum waves per SIMD the register allocation must allow (occupancy)
// UNAL: unaligned 8-byte loads at the read's byte offset; else dword-aligned
// loads realigned with DPP wave_shl:1 + v_alignbyte
template <int MINW, bool UNAL>
__global__ void __launch_bounds__(kWG, MINW) engine_tri_kernel(EngineArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int lmax = A.lmax;
  const int hlen = lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  const int seg = lane / kTriW;                 // 0..2, lane 63 -> 3 (idle)
  const int ls = lane - seg * kTriW;            // 0..20
  const bool owner = seg < 3 && ls < 20;
  const int p0 = owner ? 8 * ls : (1 << 26);   // first position of this lane (8*p0 fits int32)
  const uint32_t lane8 = 8u * (uint32_t)ls;
  const bool stats = A.flags & F_STATS, filter = A.flags & F_FILTER;
  // raw-sum bounds: pass iff min_len <= n <= max_len and lo_r*n <= S <= hi_r*n
  const int lo_r = A.min_q + A.phred, hi_r = A.max_q + A.phred;

  // LDS: pos_acc [6][lmax] u32 | hist [hlen] u32 | sc [8] u64 | per-wave tables
  // (pos_acc row 5 holds "other" counts until the epilogue turns it into N)
  uint32_t *pos_acc = reinterpret_cast<uint32_t *>(lds);
  uint32_t *other = pos_acc + 5 * lmax;
  uint32_t *hist = pos_acc + 6 * lmax;
  const int hist_words = (hlen + 1) & ~1;
  unsigned long long *sc = reinterpret_cast<unsigned long long *>(hist + hist_words);
  // per wave: two read tables [64] x 16 B (seq offset, qual offset, length, -)
  // alternating between consecutive blocks, and the segment ends [64] u32
  const int tab_words = (6 * lmax + hist_words + 2 * HPGQ_NUM_SCALARS + 3) & ~3;   // 16 B aligned
  uint32_t *wtab = pos_acc + tab_words + wave * (2 * 256 + 64);
  uint32_t *wends = wtab + 2 * 256;
  for (int i = tid; i < 6 * lmax + hist_words; i += kWG) pos_acc[i] = 0;
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += kWG) sc[i] = 0;
  __syncthreads();

  // SRDs: the read bytes plus the load slack (unaligned 8-byte windows)
  const int data_end = uni(A.idx[0][A.num_reads]);
  const uintptr_t ps = reinterpret_cast<uintptr_t>(A.seq[0]), pq = reinterpret_cast<uintptr_t>(A.qual[0]);
  const int bs = UNAL ? 0 : (int)(ps & 3), bq = UNAL ? 0 : (int)(pq & 3);   // base misalignment
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(ps - bs), (short)0, bs + data_end + kTriSlack, 0x00020000);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(pq - bq), (short)0, bq + data_end + kTriSlack, 0x00020000);
  TriAcc acc;
  acc.zero();
  int since_flush = 0;   // triples added since the last LDS flush (a byte grows <= 1 per triple)
  uint64_t fx16 = 0;
  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};   // input, passed, failed, edited, stats, long, any-long

  const int64_t nblocks = (A.num_reads + kTriBlock - 1) / kTriBlock;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kWaves;

  // block prologue: lane j describes read r0 + j in read table `tb`; lanes >=
  // nr get length 0, so whatever gathers them contributes nothing.  Returns
  // this lane's length (the epilogue needs it).
  auto load_block = [&](int64_t blk, int tb) -> uint32_t {
    const int64_t r0 = blk * kTriBlock;
    const int nr = (int)min((int64_t)kTriBlock, A.num_reads - r0);
    const int l = min(lane, nr - 1);
    const int a = A.idx[0][r0 + l], e = A.idx[0][r0 + l + 1];
    const uint32_t n = lane < nr ? (uint32_t)(e - a) : 0u;
    const uint32_t xs = (uint32_t)(bs + a), xq = (uint32_t)(bq + a);
    v4u rec;
    if (UNAL) rec = v4u{xs, xq, n, 0u};
    else rec = v4u{xs & ~3u, xq & ~3u, n | ((xs & 3u) << 16) | ((xq & 3u) << 20), 0u};
    *reinterpret_cast<v4u *>(wtab + tb * 256 + 4 * lane) = rec;
    __builtin_amdgcn_wave_barrier();   // other lanes read it (LDS is in order per wave)
    return n;
  };
  // lane -> its segment's read (entry `src` of read table tb)
  auto gather = [&](int tb, int src, TriPending &pd) {
    const v4u rec = *reinterpret_cast<const v4u *>(wtab + tb * 256 + 4 * src);
    pd.n = rec.z;
    pd.s = __builtin_amdgcn_raw_buffer_load_b64(rs, rec.x + lane8, 0, 0);
    pd.q = __builtin_amdgcn_raw_buffer_load_b64(rq, rec.y + lane8, 0, 0);
  };

  TriPending grp[2][kTriU];
  // issue group g (kTriU triples); triples past the block end gather lane 63
  // (length 0), so they add nothing
  auto load_group = [&](int tb, int nt, int g, int slot) {
#pragma unroll
    for (int u = 0; u < kTriU; ++u) {
      const int t = g * kTriU + u;
      gather(tb, t < nt ? min(3 * t + seg, 63) : 63, grp[slot][u]);
    }
  };

  // one triple: per-lane partial (raw quality | G+C << 18); adds (SUB = false)
  // or removes (SUB = true) the lane's positions from the counters
  auto account = [&](const TriPending &pd, bool count, auto sub_tag) -> uint32_t {
    constexpr bool SUB = decltype(sub_tag)::value;
    uint32_t s0 = pd.s.x, s1 = pd.s.y, q0 = pd.q.x, q1 = pd.q.y;
    if (!UNAL) {
      const uint32_t als = (pd.n >> 16) & 3u, alq = (pd.n >> 20) & 3u;
      s0 = __builtin_amdgcn_alignbyte(pd.s.y, pd.s.x, als);
      s1 = __builtin_amdgcn_alignbyte(next_lane0(pd.s.x), pd.s.y, als);
      q0 = __builtin_amdgcn_alignbyte(pd.q.y, pd.q.x, alq);
      q1 = __builtin_amdgcn_alignbyte(next_lane0(pd.q.x), pd.q.y, alq);
    }
    uint32_t m0, m1;
    tri_masks((int)(pd.n & 0xFFFFu) - p0, m0, m1);
    const uint32_t qm0 = q0 & m0, qm1 = q1 & m1;
    uint32_t bad = 0;
    uint32_t c0 = tri_codes(s0, m0, bad);
    uint32_t c1 = tri_codes(s1, m1, bad);
    if (__builtin_expect(bad != 0, 0)) {
      const uint32_t sign = SUB ? 0xFFFFFFFFu : 1u;
      c0 = tri_fix(s0, m0, c0, other, count ? lmax : 0, p0, sign);
      c1 = tri_fix(s1, m1, c1, other, count ? lmax : 0, p0 + 4, sign);
    }
    const uint32_t cg0 = __builtin_amdgcn_perm(kCGHi, kCGLo, c0);
    const uint32_t cg1 = __builtin_amdgcn_perm(kCGHi, kCGLo, c1);
    if (count) {
      const uint32_t at0 = __builtin_amdgcn_perm(kATHi, kATLo, c0);
      const uint32_t at1 = __builtin_amdgcn_perm(kATHi, kATLo, c1);
      const uint32_t h0 = __builtin_amdgcn_perm(0u, qm0, 0x0C030C01u);   // bytes 1, 3
      const uint32_t h1 = __builtin_amdgcn_perm(0u, qm1, 0x0C030C01u);
      if (SUB) {
        acc.c8[0][1] -= cg0 & 0x0F0F0F0Fu;
        acc.c8[0][2] -= (cg0 >> 4) & 0x0F0F0F0Fu;
        acc.c8[0][0] -= at0 & 0x0F0F0F0Fu;
        acc.c8[0][3] -= (at0 >> 4) & 0x0F0F0F0Fu;
        acc.c8[1][1] -= cg1 & 0x0F0F0F0Fu;
        acc.c8[1][2] -= (cg1 >> 4) & 0x0F0F0F0Fu;
        acc.c8[1][0] -= at1 & 0x0F0F0F0Fu;
        acc.c8[1][3] -= (at1 >> 4) & 0x0F0F0F0Fu;
        acc.q02[0] -= qm0 & 0x00FF00FFu;
        acc.q13[0] -= h0;
        acc.q02[1] -= qm1 & 0x00FF00FFu;
        acc.q13[1] -= h1;
      } else {
        acc.n4[0][0] += cg0;
        acc.n4[0][1] += at0;
        acc.n4[1][0] += cg1;
        acc.n4[1][1] += at1;
        acc.q02[0] += qm0 & 0x00FF00FFu;
        acc.q13[0] += h0;
        acc.q02[1] += qm1 & 0x00FF00FFu;
        acc.q13[1] += h1;
      }
    }
    const uint32_t gc = (uint32_t)__builtin_popcount(cg1) + (uint32_t)__builtin_popcount(cg0);
    const uint32_t qs = __builtin_amdgcn_sad_u8(qm1, 0u, __builtin_amdgcn_sad_u8(qm0, 0u, 0u));
    return qs + (gc << 18);
  };

  uint32_t len = 0, lenn = 0;
  int tb = 0;   // read table of the current block
  int64_t blk = gw;
  if (blk < nblocks) {
    len = load_block(blk, tb);
    const int nr0 = (int)min((int64_t)kTriBlock, A.num_reads - blk * kTriBlock);
    load_group(tb, (nr0 + 2) / 3, 0, 0);
  }
  const uint64_t not_seg_first = 0x6DB6DB6DB6DB6DB6ull;   // lanes j with j % 3 != 0
  for (; blk < nblocks; blk += nw) {
    const int64_t r0 = blk * kTriBlock;
    const int nr = (int)min((int64_t)kTriBlock, A.num_reads - r0);
    const int nt = (nr + 2) / 3;
    const int64_t nblk = blk + nw < nblocks ? blk + nw : blk;   // next block (or self)
    const int nnt = ((int)min((int64_t)kTriBlock, A.num_reads - nblk * kTriBlock) + 2) / 3;
    lenn = load_block(nblk, tb ^ 1);
    if (stats && since_flush > kByteEvery - kTriBlock / 3) {   // keep every byte <= 255
      acc.flush(pos_acc, lmax, p0);
      since_flush = 0;
    }

    auto process_group = [&](int g, int slot) {
#pragma unroll
      for (int u = 0; u < kTriU; ++u) {
        const int t = g * kTriU + u;
        // every read is added; failed ones are taken out in the block epilogue
        const uint32_t x = account(grp[slot][u], stats, AddTag{});
        const uint32_t P = wave_scan(x);
        // segment ends (lanes 20, 41, 62) -> wends[3t + seg], no wait needed
        if (ls == 20 && seg < 3 && t < nt) wends[3 * t + seg] = P;
      }
    };

    const int ngroups = (nt + kTriU - 1) / kTriU;
    for (int g = 0; g < ngroups; g += 2) {
      if (g + 1 < ngroups) load_group(tb, nt, g + 1, 1);
      else load_group(tb ^ 1, nnt, 0, 1);
      process_group(g, 0);
      if (g + 1 < ngroups) {
        if (g + 2 < ngroups) load_group(tb, nt, g + 2, 0);
        else load_group(tb ^ 1, nnt, 0, 0);
        process_group(g + 1, 1);
      }
      // nibbles hold at most 15 triples: widen after groups 0-3 and at block end
      static_assert(4 * kTriU <= kNibbleEvery && kTriBlock / 3 - 4 * kTriU <= kNibbleEvery, "");
      if (stats && g == 2) acc.widen();
    }
    if (stats) acc.widen();
    since_flush += nt;

    // ---- block epilogue (lane j = read r0 + j) ----------------------------
    const bool valid = lane < nr;
    const int n = (int)len;
    // per-read sums: difference of consecutive segment ends within a triple
    // (wends[3t + k] = inclusive wave prefix at the end of segment k)
    __builtin_amdgcn_wave_barrier();
    const uint32_t ends = lane < nr ? wends[lane] : 0u;
    const uint32_t prev = __builtin_amdgcn_mov_dpp(ends, 0x138, 0xF, 0xF, true);   // lane j-1
    const uint32_t r1 = ends - (((not_seg_first >> lane) & 1u) ? prev : 0u);
    const int sraw = (int)(r1 & 0x3FFFFu);
    bool pass = valid;
    if (filter)
      pass = pass && n >= A.min_len && n <= A.max_len && lo_r * n <= sraw && sraw <= hi_r * n;
    const bool lg = valid && n > lmax;
    if (valid && A.mask) A.mask[r0 + lane] = (uint8_t)pass;
    const uint64_t failed = __ballot(valid && !pass);
    cnt[0] += (uint32_t)nr;
    cnt[1] += (uint32_t)__builtin_popcountll(__ballot(pass));
    cnt[2] += (uint32_t)__builtin_popcountll(failed);
    cnt[6] += (uint32_t)__builtin_popcountll(__ballot(lg));
    if (stats) {
      cnt[4] += (uint32_t)__builtin_popcountll(__ballot(pass));
      cnt[5] += (uint32_t)__builtin_popcountll(__ballot(pass && lg));
      if (pass && !lg) {
        const uint32_t gc = r1 >> 18, wn = (uint32_t)n, s = (uint32_t)sraw;
        atomicAdd(&hist[wn], 1u);
        if (wn > 0) {
          atomicAdd(&hist[lmax + 1 + (2 * s + wn) / (2 * wn)], 1u);
          atomicAdd(&hist[lmax + 1 + HPGQ_MEANQ_BINS + (100 * gc) / wn], 1u);
          const uint32_t q = s / wn, rem = s - q * wn;
          fx16 += ((uint64_t)q << 16) + (((uint32_t)rem << 16) / wn);
        }
      }
      // take the failed reads back out, a triple at a time (same lanes as the add)
      uint64_t fl = failed;
      while (fl) {
        const int j = (int)__builtin_ctzll(fl);
        const int t = j / 3;
        const uint32_t fbits = (uint32_t)(fl >> (3 * t)) & 7u;
        fl &= ~(7ull << (3 * t));
        TriPending pd;
        gather(tb, ((fbits >> (seg & 3)) & 1u) ? min(3 * t + seg, 63) : 63, pd);
        (void)account(pd, true, SubTag{});
      }
    }
    len = lenn;
    tb ^= 1;
  }

  // ---- workgroup epilogue ---------------------------------------------------
  acc.widen();
  acc.flush(pos_acc, lmax, p0);
  {
    const uint32_t lo = (uint32_t)fx16, hi = (uint32_t)(fx16 >> 32);
    const uint64_t tot = (uint64_t)wave_sum(lo & 0xFFFFu) + ((uint64_t)wave_sum(lo >> 16) << 16) +
                         ((uint64_t)wave_sum(hi) << 32);
    if (lane == 0) {
      if (cnt[0]) atomicAdd(&sc[HPGQ_S_NUM_INPUT], (unsigned long long)cnt[0]);
      if (cnt[1]) atomicAdd(&sc[HPGQ_S_NUM_PASSED], (unsigned long long)cnt[1]);
      if (cnt[2]) atomicAdd(&sc[HPGQ_S_NUM_FAILED], (unsigned long long)cnt[2]);
      if (cnt[4]) atomicAdd(&sc[HPGQ_S_NUM_STATS], (unsigned long long)cnt[4]);
      if (cnt[5]) atomicAdd(&sc[HPGQ_S_LONG_READS], (unsigned long long)cnt[5]);
      if (tot) atomicAdd(&sc[HPGQ_S_ACC_MEANQ_FX16], (unsigned long long)tot);
      if (cnt[6] && A.err) atomicOr(A.err, 1);
    }
  }
  __syncthreads();
  // N at position p = (stats reads longer than p) - A - C - G - T - other
  for (int p = tid; p < lmax; p += kWG) {
    uint32_t c = 0;
    for (int L = p + 1; L <= lmax; ++L) c += hist[L];
    other[p] = c - pos_acc[lmax + p] - pos_acc[2 * lmax + p] - pos_acc[3 * lmax + p] -
               pos_acc[4 * lmax + p] - other[p];
  }
  __syncthreads();
  uint64_t *row = A.slab + (size_t)blockIdx.x * A.clen;
  const int off_pos = HPGQ_NUM_SCALARS + hlen;
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += kWG) row[i] += sc[i];
  for (int i = tid; i < hlen; i += kWG) row[HPGQ_NUM_SCALARS + i] += hist[i];
  for (int i = tid; i < 6 * lmax; i += kWG) row[off_pos + i] += pos_acc[i];
}

}  // namespace hpgq
