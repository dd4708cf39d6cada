// hpgq_engine_tri.h — FAST single-end stats/filter kernel, three reads per wave.
//
// Same contract and outputs as engine_kernel<1, *, false> (hpgq_engine_kernel.h)
// for batches whose reads are at most 160 bases: the per-read fixed cost (the
// DPP reduction, the scalar pass/fail decision, bookkeeping) is shared by three
// reads and lane utilisation goes from 38/64 to 57/64 at 150 bp.
//
//   * the wave is cut into 3 segments of 21 lanes (lane 63 idle); segment k
//     works on read 3t + k of the block.  Lane ls < 20 of a segment owns
//     positions 8ls..8ls+7 (160 per read); lane 20 only donates its first dword
//     to lane 19.
//   * each lane fetches its segment's read offsets from the block prologue
//     registers with ds_bpermute, then ONE buffer_load_dwordx2 per buffer
//     (SRD bounds check), DPP wave_shl:1 for the neighbour's dword and two
//     v_alignbyte per buffer realign the 8 bytes.
//   * per-read sums (raw quality | G+C << 18) use ONE inclusive DPP prefix scan
//     for the three segments; segment totals are differences of the scan at
//     lanes 20, 41, 62 (SALU).
//   * per-position counters as in engine_kernel (6-bit base fields, 16-bit
//     quality pairs), 8 positions per lane, segment masks from the pass bits.
// The stats layout, histogram rules and workgroup epilogue are identical, so
// the two kernels are interchangeable (the tests run both against the oracle).
#pragma once
#include "hpgq_engine_kernel.h"

namespace hpgq {

constexpr int kTriW = 21;       // lanes per segment
constexpr int kTriPos = 160;    // positions per segment (20 owning lanes x 8)
constexpr int kTriBlock = 54;   // reads per block (18 triples)
constexpr int kTriU = 3;        // triples per pipeline group (6 groups per full block)

typedef unsigned v2u __attribute__((ext_vector_type(2)));

struct TriPending {
  v2u s, q;        // raw dword pairs
  uint32_t info;   // this lane's read: n | als << 16 | alq << 20
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

struct TriAcc {
  uint32_t pk[8];           // positions p0..p0+7, 6-bit base fields
  uint32_t q02[2], q13[2];  // quality 16-bit pairs per dword
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) pk[i] = 0;
    q02[0] = q02[1] = q13[0] = q13[1] = 0;
  }
  // SUB = true takes a read back out (it was added in the same flush window,
  // so no field underflows)
  template <bool SUB>
  __device__ __forceinline__ void add_word(int w, uint32_t sw, uint32_t qw, uint32_t m) {
    const uint32_t s = (sw & m) | (0x08080808u & ~m);   // pad -> garbage field
    const uint32_t q = qw & m;
    const uint32_t codes = s & 0x07070707u;
    uint32_t sh = __builtin_amdgcn_perm(kShHi, kShLo, codes);
    const uint32_t ex = __builtin_amdgcn_perm(kExpHi, kExpLo, codes);
    if (__builtin_expect(s != ex, 0)) {   // bytes that are not exactly A/C/G/T/N
      const uint32_t d = s ^ ex;
      const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
      const uint32_t ff = (nz >> 7) * 0xFFu;
      sh = (sh & ~ff) | (0x1E1E1E1Eu & ff);
    }
    if (SUB) {
      pk[4 * w + 0] -= 1u << (sh & 31u);
      pk[4 * w + 1] -= 1u << ((sh >> 8) & 31u);
      pk[4 * w + 2] -= 1u << ((sh >> 16) & 31u);
      pk[4 * w + 3] -= 1u << ((sh >> 24) & 31u);
      q02[w] -= q & 0x00FF00FFu;
      q13[w] -= (q >> 8) & 0x00FF00FFu;
    } else {
      pk[4 * w + 0] += 1u << (sh & 31u);
      pk[4 * w + 1] += 1u << ((sh >> 8) & 31u);
      pk[4 * w + 2] += 1u << ((sh >> 16) & 31u);
      pk[4 * w + 3] += 1u << ((sh >> 24) & 31u);
      q02[w] += q & 0x00FF00FFu;
      q13[w] += (q >> 8) & 0x00FF00FFu;
    }
  }
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
          for (int b = 0; b < 5; ++b)
            atomicAdd(&pos_acc[(1 + b) * lmax + pos], (pk[4 * w + i] >> (6 * b)) & 63u);
        }
        pk[4 * w + i] = 0;
      }
      q02[w] = q13[w] = 0;
    }
  }
};

// MINW: minimum waves per SIMD the register allocation must allow (occupancy)
template <int MINW>
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
  const int p0 = owner ? 8 * ls : 0x40000000;   // first position of this lane
  const uint32_t lane8 = 8u * (uint32_t)ls;
  const bool stats = A.flags & F_STATS, filter = A.flags & F_FILTER;
  // raw-sum bounds: pass iff min_len <= n <= max_len and lo_r*n <= S <= hi_r*n
  const int lo_r = A.min_q + A.phred, hi_r = A.max_q + A.phred;

  // LDS: pos_acc [6][lmax] u32 | hist [hlen] u32 | sc [8] u64 | per-wave tables
  uint32_t *pos_acc = reinterpret_cast<uint32_t *>(lds);
  uint32_t *hist = pos_acc + 6 * lmax;
  const int hist_words = (hlen + 1) & ~1;
  unsigned long long *sc = reinterpret_cast<unsigned long long *>(hist + hist_words);
  // per wave: two read tables [64][4] u32 (os, oq, info, -) and the segment
  // ends [64] u32; tables alternate between consecutive blocks
  const int tab_words = (6 * lmax + hist_words + 2 * HPGQ_NUM_SCALARS + 3) & ~3;   // 16 B aligned
  uint32_t *wtab = pos_acc + tab_words + wave * (2 * 256 + 64);
  uint32_t *wends = wtab + 2 * 256;
  for (int i = tid; i < 6 * lmax + hist_words; i += kWG) pos_acc[i] = 0;
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += kWG) sc[i] = 0;
  __syncthreads();

  const MateBuf mb = make_mate(A.seq[0], A.qual[0], uni(A.idx[0][A.num_reads]));
  TriAcc acc;
  acc.zero();
  int since_flush = 0;   // triples added since the last flush (a field grows <= 1 per triple)
  uint64_t fx16 = 0;
  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};   // input, passed, failed, edited, stats, long, any-long

  const int64_t nblocks = (A.num_reads + kTriBlock - 1) / kTriBlock;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kWaves;

  // block prologue: lane j describes read r0 + j in read table `tb`; lanes >=
  // nr get length 0, so whatever gathers them contributes nothing.  Returns
  // this lane's info word (the epilogue needs the lengths).
  auto load_block = [&](int64_t blk, int tb) -> uint32_t {
    const int64_t r0 = blk * kTriBlock;
    const int nr = (int)min((int64_t)kTriBlock, A.num_reads - r0);
    const int l = min(lane, nr - 1);
    const int a = A.idx[0][r0 + l], e = A.idx[0][r0 + l + 1];
    const uint32_t xs = (uint32_t)(mb.bs + a), xq = (uint32_t)(mb.bq + a);
    const uint32_t inf = (lane < nr ? (uint32_t)(e - a) : 0u) | ((xs & 3u) << 16) | ((xq & 3u) << 20);
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    v4u rec = {xs & ~3u, xq & ~3u, inf, 0u};
    *reinterpret_cast<v4u *>(wtab + tb * 256 + 4 * lane) = rec;
    __builtin_amdgcn_wave_barrier();   // other lanes read it (LDS is in order per wave)
    return inf;
  };
  // lane -> its segment's read (entry `src` of read table tb): one ds_read_b128
  auto gather = [&](int tb, int src, TriPending &pd) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u rec = *reinterpret_cast<const v4u *>(wtab + tb * 256 + 4 * src);
    pd.info = rec.z;
    pd.s = __builtin_amdgcn_raw_buffer_load_b64(mb.rs, rec.x + lane8, 0, 0);
    pd.q = __builtin_amdgcn_raw_buffer_load_b64(mb.rq, rec.y + lane8, 0, 0);
  };
  // window-aligned words of a gathered triple
  auto unpack = [&](const TriPending &pd, uint32_t &s0, uint32_t &s1, uint32_t &q0, uint32_t &q1,
                    uint32_t &m0, uint32_t &m1) {
    const int n = (int)(pd.info & 0xFFFFu);
    const uint32_t als = (pd.info >> 16) & 3u, alq = (pd.info >> 20) & 3u;
    s0 = __builtin_amdgcn_alignbyte(pd.s.y, pd.s.x, als);
    s1 = __builtin_amdgcn_alignbyte(next_lane0(pd.s.x), pd.s.y, als);
    q0 = __builtin_amdgcn_alignbyte(pd.q.y, pd.q.x, alq);
    q1 = __builtin_amdgcn_alignbyte(next_lane0(pd.q.x), pd.q.y, alq);
    const int nv = n - p0;
    m0 = byte_mask(nv);
    m1 = byte_mask(nv - 4);
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

  uint32_t inf = 0, infn = 0;
  int tb = 0;   // read table of the current block
  int64_t blk = gw;
  if (blk < nblocks) {
    inf = load_block(blk, tb);
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
    infn = load_block(nblk, tb ^ 1);
    if (stats && since_flush > kFlushEvery - kTriBlock / 3) {   // keep every field <= 63
      acc.flush(pos_acc, lmax, p0);
      since_flush = 0;
    }

    auto process_group = [&](int g, int slot) {
#pragma unroll
      for (int u = 0; u < kTriU; ++u) {
        const int t = g * kTriU + u;
        uint32_t s0, s1, q0, q1, m0, m1;
        unpack(grp[slot][u], s0, s1, q0, q1, m0, m1);
        // packed per-lane partial: raw quality | G+C << 18
        uint32_t x = __builtin_amdgcn_sad_u8(q1 & m1, 0u, __builtin_amdgcn_sad_u8(q0 & m0, 0u, 0u));
        const uint32_t g0 = zero_bytes((s0 | 0x04040404u) ^ 0x47474747u) & m0 & 0x80808080u;
        const uint32_t g1 = zero_bytes((s1 | 0x04040404u) ^ 0x47474747u) & m1 & 0x80808080u;
        x += (uint32_t)(__builtin_popcount(g0) + __builtin_popcount(g1)) << 18;
        const uint32_t P = wave_scan(x);
        // segment ends (lanes 20, 41, 62) -> wends[3t + seg], no wait needed
        if (ls == 20 && seg < 3 && t < nt) wends[3 * t + seg] = P;
        // every read is added; failed ones are subtracted in the block epilogue
        if (stats) {
          acc.add_word<false>(0, s0, q0, m0);
          acc.add_word<false>(1, s1, q1, m1);
        }
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
    }
    since_flush += nt;

    // ---- block epilogue (lane j = read r0 + j) ----------------------------
    const bool valid = lane < nr;
    const int n = (int)(inf & 0xFFFFu);
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
        uint32_t s0, s1, q0, q1, m0, m1;
        unpack(pd, s0, s1, q0, q1, m0, m1);
        acc.add_word<true>(0, s0, q0, m0);
        acc.add_word<true>(1, s1, q1, m1);
      }
    }
    inf = infn;
    tb ^= 1;
  }

  // ---- workgroup epilogue ---------------------------------------------------
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
  uint64_t *row = A.slab + (size_t)blockIdx.x * A.clen;
  const int off_pos = HPGQ_NUM_SCALARS + hlen;
  for (int i = tid; i < HPGQ_NUM_SCALARS; i += kWG) row[i] += sc[i];
  for (int i = tid; i < hlen; i += kWG) row[HPGQ_NUM_SCALARS + i] += hist[i];
  for (int i = tid; i < 6 * lmax; i += kWG) row[off_pos + i] += pos_acc[i];
}

}  // namespace hpgq
