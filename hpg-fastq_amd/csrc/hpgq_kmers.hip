// hpgq_kmers.hip — `stats --kmers`: 5-mer counts, global and per position.
//
// Replaces the per-read kmer fields of fastq_reads_stats (bioinfo-libs,
// absent) and their merge in the stats consumer, src/stats_fastq.c:384-410
// (kmer_out->counter += ..., counter_by_pos[k] += ...).  Semantics are
// build-defined: 5-mers of exact uppercase A/C/G/T, id =
// sum code_i * 4^(4-i) with A=0 C=1 G=2 T=3 (first base most significant),
// counted at every start position p <= len-5 of every merged read.  Output:
// by_pos[1024][lmax-4] u64; the global counter of a k-mer is its row sum.
//
// Kernels.  A 5-mer's counter lives at (start position, id): 1024 x lmax-4
// counters, too many for one workgroup's LDS, so a workgroup owns a TILE of
// kP = 32 start positions ([1024][kP] u32 = 128 KB) for the whole call and
// stores it to its slab at the end; kmer_reduce_kernel adds a tile's slabs
// into by_pos.  Every tile re-reads the reads' windows; the workgroups that
// hold the T tiles of one read group sit on one XCD and walk the same reads in
// the same order, so the re-reads hit that XCD's L2 (blockIdx -> XCD is round
// robin: b mod 8).  When lmax allows more than 8 tiles a prepass takes the
// longest counted read, so tiles past it (the CLI's lmax 1024 on 150 bp
// reads) exit at once instead of scanning every read.
//   kmer_maxlen_kernel  max length over the counted reads (atomicMax)
//   kmer_tile_kernel    two lanes per read and tile (20 bytes each: 16
//                       starts + 4, loaded dword-aligned as 24 and shifted
//                       into place by v_alignbyte: a misaligned 16-byte
//                       gather costs the texture addresser far more),
//                       software-pipelined two groups deep on two
//                       alternating register sets (the windows of the next
//                       two groups and the offsets of the one after are in
//                       flight while a group is counted).  Table id-major,
//                       cell (p, id) at id * 32 + p: a start position is an
//                       LDS bank.  The 32 lanes of a group visit their starts
//                       in rotated orders, so at every step they sit on 32
//                       distinct positions and their ds_add_u32 hit 32
//                       distinct banks (position-major with every lane at the
//                       same position made random ids collide: 71 % of the
//                       LDS cycles were bank conflicts).  Per byte: a v_perm
//                       LUT for the 2-bit code and one for the exactness test;
//                       per start: one v_alignbit (the lane's shift for that
//                       step), one v_bitop3 (its position's bank), one v_bfe
//                       (0 or 1) and the add.  Bound: VALU issue beside the
//                       window gathers (one lane per read made
//                       1024-read groups whose L2 re-reads doubled the HBM
//                       traffic).
#include "hpgq_common.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

namespace hpgq {
namespace kmers {

constexpr int kK = 5;
constexpr int kNum = 1 << (2 * kK);   // 1024
constexpr int kP = 32;                // start positions per tile (one LDS bank each)
constexpr int kWG = 1024;
constexpr int kReadsPerWave = 32;     // two lanes per read
constexpr int kGroup = kWG / 2;       // reads per workgroup step
constexpr int kSpill = 8;             // tiles above which the maxlen prepass runs
static_assert(kWG == kNum, "the flush gives each thread one id");

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// byte & 7 is one-to-one on A(1) C(3) T(4) G(7).  kEx*: the expected byte per
// code; the codes no base has get bytes whose low 3 bits are neither the code
// nor the code ^ 4, so that (byte ^ expected) is never 0 or 0x0C for them
// (see codes4).  kVal*: the 2-bit code per code.
constexpr uint32_t kExLo = 0x43014101u;   // codes 0..3: -, A, -, C
constexpr uint32_t kExHi = 0x47010454u;   // codes 4..7: T, -, -, G
constexpr uint32_t kValLo = 0x01000000u;  // C = 1 at code 3
constexpr uint32_t kValHi = 0x02000003u;  // T = 3 at code 4, G = 2 at code 7

// 4 bytes -> their 2-bit codes packed first byte highest (byte i of 4 at
// bits 2(3-i)) and a bit per byte that is NOT exactly A/C/G/T (bit i).
// d = byte ^ expected is 0 exactly for A/C/G/T; as a v_perm selector over
// {0xFFFFFFFF, 0xFFFFFF00} it gives 0x00 for 0 and 0xFF for any other value
// but 12 (selectors 1-11 pick 0xFF bytes or sign bits that are set, >= 13 is
// 0xFF), and 12 cannot occur: byte ^ 0x0C has low 3 bits code ^ 4, and no
// expected byte's low 3 bits are its code ^ 4.
__device__ __forceinline__ void codes4(uint32_t w, uint32_t &packed, uint32_t &bad) {
  const uint32_t code = w & 0x07070707u;
  const uint32_t d = w ^ __builtin_amdgcn_perm(kExHi, kExLo, code);
  const uint32_t bm = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xFFFFFF00u, d);
  bad = __builtin_amdgcn_udot4(bm & 0x01010101u, 0x08040201u, 0u, false);
  packed = __builtin_amdgcn_udot4(__builtin_amdgcn_perm(kValHi, kValLo, code), 0x01041040u, 0u, false);
}

__device__ __forceinline__ bool counted(const uint8_t *mask, int64_t r) { return !mask || mask[r] == 1; }

// eight workgroups per CU, grid-stride, four reads per thread (one 16-byte
// offset load); one atomic per workgroup (one per wave made 8 K atomics on
// one word: 112 us per 10 M reads)
__global__ void __launch_bounds__(1024) kmer_maxlen_kernel(const int32_t *idx, int64_t n, const uint8_t *mask,
                                                           int *maxlen) {
  __shared__ int wm[16];
  const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
      (void *)idx, (short)0, (uint32_t)((n + 1) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
      (void *)mask, (short)0, mask ? (uint32_t)n : 0u, 0x00020000);
  int m = 0;
  for (int64_t r = 4 * ((int64_t)blockIdx.x * 1024 + threadIdx.x); r < n; r += 4 * (int64_t)gridDim.x * 1024) {
    if (r + 4 > n) {   // the last reads: one by one (a dword past n would read 0)
      for (int64_t i = r; i < n; ++i)
        if (counted(mask, i)) m = max(m, idx[i + 1] - idx[i]);
      break;
    }
    const v4u a = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)r * 4u, 0, 0);
    const int32_t e = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ri, (uint32_t)r * 4u + 16u, 0, 0);
    const uint32_t mk = mask ? __builtin_amdgcn_raw_buffer_load_b32(rm, (uint32_t)r, 0, 0) : 0x01010101u;
    const int32_t b[5] = {(int32_t)a[0], (int32_t)a[1], (int32_t)a[2], (int32_t)a[3], e};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (((mk >> (8 * i)) & 0xFFu) == 1u) m = max(m, b[i + 1] - b[i]);
  }
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) m = max(m, wm[w]);
    if (m) atomicMax(maxlen, m);
  }
}

// the 16 starts of one half-tile of a lane's window: its code stream shifted
// for the alignbit cuts (t1:t0 = the 20 bytes' codes << 7, first byte
// highest: the 5-mer at half position h is bits [2(15 - h) + 7, + 10)) and
// its count mask rotated to the lane's visiting order (bit j = the start the
// lane visits at step j)
struct Half {
  uint32_t t1, t0, er;
};

__device__ __forceinline__ Half half_of(const uint32_t (&pk)[5], const uint32_t (&bd)[5], int last, int q) {
  const uint32_t s0 = (pk[1] << 24) | (pk[2] << 16) | (pk[3] << 8) | pk[4];
  const uint32_t b = bd[0] | (bd[1] << 4) | (bd[2] << 8) | (bd[3] << 12) | (bd[4] << 16);
  // the 5-mer at h counts iff bytes h..h+4 are A/C/G/T and h <= last
  uint32_t e = ~(b | (b >> 1) | (b >> 2) | (b >> 3) | (b >> 4));
  e &= last >= 15 ? 0xFFFFu : last >= 0 ? (2u << last) - 1u : 0u;
  Half H;
  H.t1 = __builtin_amdgcn_alignbit(pk[0], s0, 25);
  H.t0 = s0 << 7;
  H.er = (e | (e << 16)) >> q;
  return H;
}

// MASK: mask is not null (a compile-time choice: a runtime one put a branch
// around the mask load, whose merge made hipcc wait for every load in flight)
template <bool MASK>
__global__ void __launch_bounds__(kWG) kmer_tile_kernel(const char *seq, const int32_t *idx, int64_t n,
                                                        const uint8_t *mask, int npos, const int *maxlen,
                                                        uint32_t *slab) {
  __shared__ uint32_t t[kNum * kP];   // [id][position]
  // tiles with a start position some counted read reaches
  const int last_start = min(npos, (maxlen ? *maxlen : npos + kK - 1) - (kK - 1));   // starts 0 .. last_start-1
  const int T = last_start > 0 ? (last_start + kP - 1) / kP : 0;
  const int b = (int)blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int classes = T ? (int)(gridDim.x >> 3) / T : 0;   // read-group classes per XCD
  if (T == 0 || slot >= classes * T) return;
  const int tile = slot % T, cls = slot / T;
  const int p0 = tile * kP;
  for (int i = threadIdx.x; i < kP * kNum; i += kWG) t[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // lanes 2i, 2i + 1 take read i's half-tiles hl = 0, 1 (starts 16 hl + [0,
  // 16)); the lane visits start 16 hl + (q + j) mod 16 at step j, so the 32
  // lanes of a group (lanes 0-31, 32-63: one LDS cycle each) sit on 32
  // distinct positions at every step
  const int q = (lane >> 1) & 15, hl = lane & 1;
  const int32_t data_end = __builtin_amdgcn_readfirstlane(idx[n]);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)seq, (short)0, data_end + HPGQ_DEVICE_SLACK, 0x00020000);
  // read offsets and mask through descriptors too: the loads past the batch
  // (the pipeline's prefetch past the last group) read 0 and move nothing
  const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
      (void *)idx, (short)0, (uint32_t)((n + 1) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
      (void *)mask, (short)0, mask ? (uint32_t)n : 0u, 0x00020000);
  const int64_t ngroups = (n + kGroup - 1) / kGroup;
  const int64_t gstride = 8 * (int64_t)classes;
  const int64_t g0 = xcd + 8 * (int64_t)cls;
  // a read's offsets and mask byte.  The wave's 32 reads take ONE coalesced
  // load of their 33 offsets (lane l: idx[rb + l]) and one of their 32 mask
  // bytes (lane l: mask[rb + l]), handed to the read's lane pair by
  // ds_bpermute when the group is used (per-lane loads of idx[r], idx[r + 1]
  // and mask[r] were three addresser passes per wave and tile visit).
  // Unconditional loads: past the end they read 0, so the compiler counts the
  // loads in flight exactly.
  struct Meta {
    int32_t a, e;
    uint32_t m;
  };
  struct Raw {
    int32_t ix;
    uint32_t mk;
    int64_t rb;
  };
  auto meta_raw = [&](int64_t g) __attribute__((always_inline)) {
    Raw R;
    R.rb = g * kGroup + wave * kReadsPerWave;
    const int64_t r = R.rb + lane;
    const uint32_t ro = r <= n && lane <= kReadsPerWave ? (uint32_t)r : 0x3FFFFFF0u;
    R.ix = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ri, ro * 4u, 0, 0);
    const bool on = r < n && lane < kReadsPerWave;
    R.mk = MASK ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rm, on ? (uint32_t)r : 0x3FFFFFF0u, 0, 0)
                : (on ? 1u : 0u);
    return R;
  };
  auto resolve = [&](const Raw &R) __attribute__((always_inline)) {
    const int i = lane >> 1;
    Meta M;
    M.a = __builtin_amdgcn_ds_bpermute(4 * i, R.ix);
    M.e = __builtin_amdgcn_ds_bpermute(4 * (i + 1), R.ix);
    M.m = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * i, (int)R.mk);
    return M;
  };
  // the lane's 20 bytes (16 starts + 4): a read's two lanes read 36
  // contiguous bytes.  The loads are dword-aligned: 24 bytes from the dword
  // at or below the window (a b128 and a b64), shifted into place by
  // v_alignbyte when the group is counted.  Reads start at any byte (150-byte
  // reads back to back: every other one at 2 mod 4), and a 16-byte load that
  // is not dword-aligned costs the addresser far more than an aligned one
  // (tools/ubench/window_rates.hip: 405 vs 248 us for the same windows).
  struct Win {
    v4u a;
    v2u c;
  };
  // (the b64 tail only on the odd lane of a pair: the even lane's bytes 16..23
  // are its partner's first 8, handed over by DPP when the group is counted;
  // the even lanes' tail offset is out of range: zeros, no traffic)
  auto window = [&](const Meta &M) __attribute__((always_inline)) {
    const uint32_t o = (uint32_t)(M.a + p0 + 16 * hl) & ~3u;
    Win W;
    W.a = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
    W.c = __builtin_amdgcn_raw_buffer_load_b64(rs, hl ? o + 16u : 0x80000000u, 0, 0);
    return W;
  };
  // per step j: the alignbit shift of the visited start (30 - 2 (q + j mod
  // 16); alignbit reads 5 bits) and its cell's position bits
  uint32_t sh[16], row[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t h = (uint32_t)((q + j) & 15);
    sh[j] = 30u - 2u * h;
    row[j] = 4u * (h + 16u * (uint32_t)hl);
  }
  constexpr uint32_t kIdBits = (uint32_t)(kNum - 1) << 7;   // id * 128 = id * kP * 4
  // software pipeline: group g is counted while the windows of g + stride and
  // g + 2 stride and the offsets of g + 3 stride are in flight.  Two register
  // sets alternate (unrolled by two), so no loop-carried copy of a register
  // whose load is pending makes the wave wait for it; each group's offsets
  // are loaded before the window issued in the same step, so waiting for them
  // (vmcnt is in order) never waits for that younger window.  (Round 3/4's
  // one-group pipeline rotated its registers by copies, and the copies drained
  // every load at the loop latch.)
  // the starts of one group: c / wc (its offsets and window) are counted, then
  // refilled with group g + 2 stride (offsets from rin, loaded a step ago);
  // rout takes the offsets of g + 3 stride
  auto step = [&](int64_t g, Meta &c, Win &wc, Raw &rin, Raw &rout) __attribute__((always_inline)) {
    // the read's last start, relative to the tile's first (< 0: none here;
    // masked-out reads: none)
    const int last = c.m == 1u ? min(c.e - c.a - kK, npos - 1) - p0 : -1;
    uint32_t pk[5], bd[5];
    const uint32_t ab = (uint32_t)c.a & 3u;   // the window's byte offset in its first dword
                                              // (p0 and 16 hl are multiples of 4)
    {   // even lanes: the tail from the odd partner's first 8 bytes (quad_perm [1,1,3,3])
      const uint32_t n0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)wc.a[0], 0xF5, 0xF, 0xF, false);
      const uint32_t n1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)wc.a[1], 0xF5, 0xF, 0xF, false);
      if (!hl) {
        wc.c[0] = n0;
        wc.c[1] = n1;
      }
    }
    const uint32_t wd[5] = {__builtin_amdgcn_alignbyte(wc.a[1], wc.a[0], ab), __builtin_amdgcn_alignbyte(wc.a[2], wc.a[1], ab),
                            __builtin_amdgcn_alignbyte(wc.a[3], wc.a[2], ab), __builtin_amdgcn_alignbyte(wc.c[0], wc.a[3], ab),
                            __builtin_amdgcn_alignbyte(wc.c[1], wc.c[0], ab)};
#pragma unroll
    for (int i = 0; i < 5; ++i) codes4(wd[i], pk[i], bd[i]);
    // (the set's registers are dead here: keep the refill below this point, so
    // the loads reuse them instead of living beside them -- else the loop
    // latch copies a register whose load is pending, which waits for it)
    __builtin_amdgcn_sched_barrier(0);
    rout = meta_raw(g + 3 * gstride);
    c = resolve(rin);
    wc = window(c);
    // (no early exit for a wave whose reads all end before these starts: a
    // branch here lets hipcc sink the codes below the refill, and the set's
    // registers then live beside their own refill -- copies that wait; such a
    // wave adds zeros)
    const Half hf = half_of(pk, bd, last - 16 * hl, q);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // cell byte address id * 128 + position * 4: the id cut out at bits
      // 7..16 by one v_alignbit, the position's bits from row (v_bitop3);
      // a start that does not count adds 0
      const uint32_t win = __builtin_amdgcn_alignbit(hf.t1, hf.t0, sh[j]);
      const uint32_t addr = __builtin_amdgcn_bitop3_b32(win, kIdBits, row[j], 0xEA);   // (a & b) | c
      atomicAdd(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(t) + addr), __builtin_amdgcn_ubfe(hf.er, j, 1));
    }
  };
  Meta ca = resolve(meta_raw(g0));
  Win wa = window(ca);
  Raw ra = meta_raw(g0 + gstride), rb;
  Meta cb = resolve(ra);
  Win wb = window(cb);
  rb = meta_raw(g0 + 2 * gstride);
  // (no exit between the two steps: a group past the last has no counted
  // read -- its offsets and mask bytes load as 0 -- and adds nothing)
  for (int64_t g = g0; g < ngroups; g += 2 * gstride) {
    // every load drained once per iteration, on purpose: the drain keeps the T
    // tile workgroups of a class in step, so their re-reads of a read's window
    // hit the XCD's L2.  Exact waits (the windows of two groups in flight
    // throughout) let them drift apart: HBM traffic 1.06x -> 2.0x, 570 -> 633
    // us; lockstep by progress counters instead cost more than it saved
    // (profiles/r05_kmers_waits_ab.json)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    step(g, ca, wa, rb, ra);
    step(g + gstride, cb, wb, ra, rb);
  }
  __syncthreads();
  // the table goes to this workgroup's slab with plain coalesced stores;
  // kmer_reduce_kernel sums a tile's slabs into by_pos (u64 atomics straight
  // from here -- one cache line per lane, 48 workgroups per cell -- took 300
  // us of a 970 us launch)
  uint32_t *my = slab + (size_t)b * (kP * kNum);
  for (int i = threadIdx.x; i < kP * kNum; i += kWG) my[i] = t[i];
}

// The starts >= npos of the counted reads longer than lmax (the reference's
// counter_by_pos grows with the read, src/stats_fastq.c:394-407).  Shaped like
// the maxlen prepass: each thread checks four reads (one 16-byte offset load +
// one, the four mask bytes), so the batch's 5 B per read stream at full rate
// (round 6 first had each wave walk 64 reads per step, a dependent load chain:
// +38 us per 10 M reads); a wave holding such a read takes it with all its
// lanes over its starts [max(lo, npos), hi), one u64 atomic per 5-mer into the
// tail [cap][kNum] (start npos + i).  flags[0]: the longest such read
// (atomicMax), flags[1]: the longest whose starts reach past hi -- a device
// batch beyond the tail reserved so far; its call's flag is set and
// hpgq_kmers_sync adds the rest (tail_only: starts [lo, hi) only, no maxima).
// A maxlen prepass of the same call (lmax > 260) that found no counted read
// past npos + 4 ends it at once.
struct LongArgs {
  const char *seq;
  const int32_t *idx;
  int64_t n;
  const uint8_t *mask;
  const int *maxlen_pre;
  unsigned long long *tail;
  int lo, hi;
  uint32_t *flags, *ovf;
  int tail_only;
};

__device__ __forceinline__ void long_reads_block(const LongArgs &L, int npos, int64_t blk) {
  if (L.maxlen_pre && *L.maxlen_pre < npos + kK) return;
  const int lane = threadIdx.x & 63;
  const int64_t r0 = 4 * (blk * 256 + threadIdx.x);
  uint32_t lng = 0;   // bit i: read r0 + i counts and has starts >= npos
  int32_t a[5] = {0, 0, 0, 0, 0};
  if (r0 < L.n) {
    // (through descriptors, as kmer_maxlen_kernel: any dword alignment; past
    // the batch the offsets read 0 and the mask bytes 0)
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
        (void *)L.idx, (short)0, (uint32_t)((L.n + 1) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
        (void *)L.mask, (short)0, L.mask ? (uint32_t)L.n : 0u, 0x00020000);
    if (r0 + 4 <= L.n) {
      const v4u x = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)r0 * 4u, 0, 0);
      a[0] = (int32_t)x[0]; a[1] = (int32_t)x[1]; a[2] = (int32_t)x[2]; a[3] = (int32_t)x[3];
      a[4] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ri, (uint32_t)r0 * 4u + 16u, 0, 0);
    } else {   // the batch's last reads: one by one (a load reaching past the range reads 0)
      for (int i = 0; i < 5; ++i)
        a[i] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ri, (uint32_t)min(r0 + i, L.n) * 4u, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (r0 + i < L.n && a[i + 1] - a[i] >= npos + kK) lng |= 1u << i;
    // the mask only for the (rare) long ones: 4 B per read streamed, not 5
    if (lng && L.mask) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (((lng >> i) & 1u) && __builtin_amdgcn_raw_buffer_load_b8(rm, (uint32_t)(r0 + i), 0, 0) != 1u)
          lng &= ~(1u << i);
    }
  }
  uint64_t b = __ballot(lng != 0);
  while (b) {   // (rare) the wave's long reads, one at a time
    const int j = __builtin_ctzll(b);
    b &= b - 1;
    uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)lng, j);
    while (bits) {
      const int i = __builtin_ctz(bits);
      bits &= bits - 1;
      const int32_t aj = __builtin_amdgcn_readlane(i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3], j);
      const int32_t lj = __builtin_amdgcn_readlane(i == 0 ? a[1] : i == 1 ? a[2] : i == 2 ? a[3] : a[4], j) - aj;
      const int last = lj - kK;   // its last start
      if (!L.tail_only && lane == 0) atomicMax(&L.flags[0], (uint32_t)lj);
      const int end = min(last + 1, L.hi);
      const uint8_t *sq = reinterpret_cast<const uint8_t *>(L.seq) + aj;
      for (int p = max(L.lo, npos) + lane; p < end; p += 64) {
        int id = 0;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < kK; ++k) {
          const uint8_t c = sq[p + k];
          const int code = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
          ok = ok && code >= 0;
          id = id * 4 + (code & 3);
        }
        if (ok) atomicAdd(&L.tail[(size_t)(p - npos) * kNum + id], 1ull);
      }
      if (last + 1 > L.hi && lane == 0) {
        atomicMax(&L.flags[1], (uint32_t)lj);
        if (L.ovf) *L.ovf = 1u;
      }
    }
  }
}

// by_pos[id][p0 + row] += the sum of a tile's slabs (8 XCDs x classes); one
// thread per (tile, id, row), consecutive threads consecutive positions (the
// slab reads and the by_pos adds coalesce).  Blocks past the reduction's are
// the long-read pass (long_reads_block): one launch, the scan overlapping the
// reduction.
__global__ void __launch_bounds__(256) kmer_reduce_kernel(const uint32_t *slab, int npos, const int *maxlen, int grid,
                                                          unsigned long long *out, int reduce_blocks, LongArgs L) {
  if ((int)blockIdx.x >= reduce_blocks) {
    long_reads_block(L, npos, (int64_t)blockIdx.x - reduce_blocks);
    return;
  }
  const int last_start = min(npos, (maxlen ? *maxlen : npos + kK - 1) - (kK - 1));
  const int T = last_start > 0 ? (last_start + kP - 1) / kP : 0;
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;   // tile * kP * kNum + id * kP + row
  const int tile = (int)(f / (kP * kNum)), cell = (int)(f % (kP * kNum));
  const int classes = T ? (grid >> 3) / T : 0;
  if (tile >= T) return;
  const int p = tile * kP + cell % kP;
  if (p >= npos) return;
  uint32_t sum = 0;
  for (int cls = 0; cls < classes; ++cls)
#pragma unroll
    for (int x = 0; x < 8; ++x) sum += slab[((size_t)(8 * (cls * T + tile) + x)) * (kP * kNum) + cell];
  if (sum) out[(size_t)(cell / kP) * npos + p] += sum;
}

// the long-read pass alone (lmax < 5: no dense table; the second pass)
__global__ void __launch_bounds__(256) kmer_long_kernel(int npos, LongArgs L) {
  long_reads_block(L, npos, blockIdx.x);
}

}  // namespace kmers
}  // namespace hpgq

namespace {
// a call since the last sync, kept for the tail's second pass
struct KCall {
  const char *seq;
  const int32_t *idx;
  const uint8_t *mask;
  int64_t n;
  int hi;
};
constexpr size_t kKOvfChunk = 4096;
}  // namespace

struct hpgq_kmers {
  int device = 0;
  int lmax = 0, npos = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  unsigned long long *d_out = nullptr;
  int *d_maxlen = nullptr;   // per call: the longest counted read
  uint32_t *d_slab = nullptr;   // per tile workgroup: its table of the call
  int grid = 0;
  int cus = 0;
  // the tail: [tail_cap][kNum] u64, start npos + i; d_flags [longest long
  // read, longest one past the tail]; h_flags their pinned copy
  unsigned long long *d_tail = nullptr;
  int64_t tail_cap = 0;
  uint32_t *d_flags = nullptr, *h_flags = nullptr;
  std::vector<KCall> calls;
  std::vector<uint32_t *> ovf_chunks;
};

namespace {
int k_tail_hi(const hpgq_kmers *k) { return (int)std::min<int64_t>((int64_t)k->npos + k->tail_cap, INT32_MAX); }

// grow the tail to starts [npos, npos + cap) (waits for the stream; zero-extended)
int k_ensure_tail(hpgq_kmers *k, int64_t cap) {
  if (cap <= k->tail_cap) return HPGQ_OK;
  const int64_t limit = (int64_t)INT32_MAX - k->npos;
  if (cap > limit) return HPGQ_E_INVALID;
  int64_t nc = std::max<int64_t>(cap, k->tail_cap + k->tail_cap / 2);
  nc = std::min<int64_t>((nc + 63) & ~(int64_t)63, limit);
  const size_t row = (size_t)hpgq::kmers::kNum * 8;
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  unsigned long long *d = nullptr;
  if (hipMalloc(&d, (size_t)nc * row) != hipSuccess) return HPGQ_E_NOMEM;
  const size_t old = (size_t)k->tail_cap * row;
  if (old) HPGQ_HIP_TRY(hipMemcpyAsync(d, k->d_tail, old, hipMemcpyDeviceToDevice, k->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(reinterpret_cast<char *>(d) + old, 0, (size_t)nc * row - old, k->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  (void)hipFree(k->d_tail);
  k->d_tail = d;
  k->tail_cap = nc;
  return HPGQ_OK;
}

// blocks of the long-read pass: four reads per thread
int k_long_blocks(int64_t n) { return (int)std::max<int64_t>(1, (n + 1023) / 1024); }

// the tail's second pass (the stream idle, h_flags current): see hpgq.h / the engine's resolve
int k_resolve(hpgq_kmers *k) {
  const uint32_t need = k->h_flags[1];
  const size_t nc = k->calls.size();
  if (need == 0) {
    k->calls.clear();
    return HPGQ_OK;
  }
  int rc = k_ensure_tail(k, (int64_t)need - hpgq::kmers::kK + 1 - k->npos);
  if (rc) return rc;
  std::vector<uint32_t> fl(nc, 0);
  for (size_t k0 = 0; k0 < nc; k0 += kKOvfChunk)
    HPGQ_HIP_TRY(hipMemcpy(fl.data() + k0, k->ovf_chunks[k0 / kKOvfChunk], std::min(kKOvfChunk, nc - k0) * 4,
                           hipMemcpyDeviceToHost));
  for (size_t i = 0; i < nc; ++i) {
    if (!fl[i]) continue;
    const KCall &c = k->calls[i];
    const hpgq::kmers::LongArgs L{c.seq, c.idx, c.n, c.mask, nullptr, k->d_tail, c.hi, k_tail_hi(k), k->d_flags,
                                  nullptr, 1};
    hipLaunchKernelGGL(hpgq::kmers::kmer_long_kernel, dim3((unsigned)k_long_blocks(c.n)), dim3(256), 0, k->stream,
                       k->npos, L);
    HPGQ_HIP_TRY(hipGetLastError());
  }
  HPGQ_HIP_TRY(hipMemsetAsync(k->d_flags + 1, 0, 4, k->stream));
  for (size_t k0 = 0; k0 < nc; k0 += kKOvfChunk)
    HPGQ_HIP_TRY(hipMemsetAsync(k->ovf_chunks[k0 / kKOvfChunk], 0, std::min(kKOvfChunk, nc - k0) * 4, k->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  k->h_flags[1] = 0;
  k->calls.clear();
  return HPGQ_OK;
}

int k_sync_resolve(hpgq_kmers *k) {
  HPGQ_HIP_TRY(hipMemcpyAsync(k->h_flags, k->d_flags, 8, hipMemcpyDeviceToHost, k->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  return k_resolve(k);
}
}  // namespace

extern "C" {

int hpgq_kmers_open(hpgq_kmers_t **km, int device, int lmax, void *stream) {
  if (!km || lmax < 1 || lmax > HPGQ_LMAX_LIMIT) return HPGQ_E_INVALID;
  *km = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return HPGQ_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(device));
  hpgq_kmers *k = new hpgq_kmers;
  k->device = device;
  k->lmax = lmax;
  k->npos = lmax > hpgq::kmers::kK - 1 ? lmax - (hpgq::kmers::kK - 1) : 0;
  if (stream) {
    k->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking) != hipSuccess) {
      delete k;
      return HPGQ_E_HIP;
    }
    k->own_stream = true;
  }
  const size_t bytes = (size_t)hpgq::kmers::kNum * (size_t)(k->npos > 0 ? k->npos : 1) * 8;
  if (hipMalloc(&k->d_out, bytes) != hipSuccess || hipMalloc(&k->d_maxlen, sizeof(int)) != hipSuccess ||
      hipMalloc(&k->d_flags, 8) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void **>(&k->h_flags), 8, hipHostMallocDefault) != hipSuccess) {
    hpgq_kmers_close(k);
    return HPGQ_E_NOMEM;
  }
  k->h_flags[0] = k->h_flags[1] = 0;
  if (hipMemsetAsync(k->d_out, 0, bytes, k->stream) != hipSuccess ||
      hipMemsetAsync(k->d_flags, 0, 8, k->stream) != hipSuccess ||
      hipDeviceGetAttribute(&k->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    hpgq_kmers_close(k);
    return HPGQ_E_HIP;
  }
  {
    using namespace hpgq::kmers;
    // one resident workgroup per CU (128 KB of LDS); 8 x (tiles the lmax
    // allows) x read-group classes, so every tile of a class has its
    // workgroup on each XCD (the kernel takes the tiles the longest read
    // needs and idles the rest)
    const int tmax = std::max(1, (k->npos + kP - 1) / kP);
    k->grid = 8 * tmax * std::max(1, k->cus / (8 * tmax));
    if (k->npos > 0 && hipMalloc(&k->d_slab, (size_t)k->grid * kP * kNum * sizeof(uint32_t)) != hipSuccess) {
      hpgq_kmers_close(k);
      return HPGQ_E_NOMEM;
    }
  }
  *km = k;
  return HPGQ_OK;
}

void hpgq_kmers_close(hpgq_kmers_t *k) {
  if (!k) return;
  (void)hipSetDevice(k->device);
  if (k->stream) (void)hipStreamSynchronize(k->stream);
  (void)hipFree(k->d_out);
  (void)hipFree(k->d_maxlen);
  (void)hipFree(k->d_slab);
  (void)hipFree(k->d_tail);
  (void)hipFree(k->d_flags);
  if (k->h_flags) (void)hipHostFree(k->h_flags);
  for (uint32_t *q : k->ovf_chunks) (void)hipFree(q);
  if (k->own_stream) (void)hipStreamDestroy(k->stream);
  delete k;
}

int hpgq_kmers_count_device(hpgq_kmers_t *k, const hpgq_batch_t *b, const uint8_t *mask) {
  if (!k || !b || b->num_reads < 0) return HPGQ_E_INVALID;
  if (b->num_reads == 0) return HPGQ_OK;
  if (!b->seq || !b->data_indices) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  using namespace hpgq::kmers;
  const int tmax = (k->npos + kP - 1) / kP;
  constexpr int64_t kPart = (int64_t)1 << 28;   // reads per launch (32-bit offsets into idx)
  for (int64_t lo = 0; lo < b->num_reads; lo += kPart) {
    const int64_t n = std::min(kPart, b->num_reads - lo);
    const int32_t *ix = b->data_indices + lo;
    const uint8_t *mk = mask ? mask + lo : nullptr;
    // few tiles (lmax <= 260): every tile is work for reads near lmax, and
    // the prepass (~30 us per 10 M reads) would cost more than it saves
    const int *ml = nullptr;
    if (tmax > kSpill) {   // (also lets the long-read pass below end at once)
      HPGQ_HIP_TRY(hipMemsetAsync(k->d_maxlen, 0, sizeof(int), k->stream));
      hipLaunchKernelGGL(kmer_maxlen_kernel, dim3((unsigned)std::min<int64_t>((n + 4095) / 4096, 8 * k->cus)),
                         dim3(1024), 0, k->stream, ix, n, mk, k->d_maxlen);
      HPGQ_HIP_TRY(hipGetLastError());
      ml = k->d_maxlen;
    }
    // starts >= npos of longer reads (the call is kept for the tail's second pass)
    const size_t ci = k->calls.size();
    if (ci / kKOvfChunk >= k->ovf_chunks.size()) {
      uint32_t *q = nullptr;
      if (hipMalloc(&q, kKOvfChunk * 4) != hipSuccess) return HPGQ_E_NOMEM;
      k->ovf_chunks.push_back(q);
      HPGQ_HIP_TRY(hipMemsetAsync(q, 0, kKOvfChunk * 4, k->stream));
    }
    k->calls.push_back(KCall{b->seq, ix, mk, n, k_tail_hi(k)});
    const LongArgs L{b->seq, ix, n, mk, ml, k->d_tail, k->npos, k_tail_hi(k), k->d_flags,
                     k->ovf_chunks[ci / kKOvfChunk] + ci % kKOvfChunk, 0};
    if (k->npos > 0) {   // (lmax < 5: every start is in the tail)
      if (mk)
        hipLaunchKernelGGL(kmer_tile_kernel<true>, dim3((unsigned)k->grid), dim3(kWG), 0, k->stream, b->seq, ix, n, mk,
                           k->npos, ml, k->d_slab);
      else
        hipLaunchKernelGGL(kmer_tile_kernel<false>, dim3((unsigned)k->grid), dim3(kWG), 0, k->stream, b->seq, ix, n, mk,
                           k->npos, ml, k->d_slab);
      HPGQ_HIP_TRY(hipGetLastError());
      // the reduction and, in the same launch, the long-read pass
      const int rb = (int)(((int64_t)tmax * kP * kNum + 255) / 256);
      hipLaunchKernelGGL(kmer_reduce_kernel, dim3((unsigned)(rb + k_long_blocks(n))), dim3(256), 0, k->stream,
                         (const uint32_t *)k->d_slab, k->npos, ml, k->grid, k->d_out, rb, L);
    } else {
      hipLaunchKernelGGL(kmer_long_kernel, dim3((unsigned)k_long_blocks(n)), dim3(256), 0, k->stream, k->npos, L);
    }
    HPGQ_HIP_TRY(hipGetLastError());
  }
  return HPGQ_OK;
}

int hpgq_kmers_sync(hpgq_kmers_t *k) {
  if (!k) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  return k_sync_resolve(k);
}

int hpgq_kmers_reset(hpgq_kmers_t *k) {
  if (!k) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  if (hpgq_kmers_size(k)) HPGQ_HIP_TRY(hipMemsetAsync(k->d_out, 0, hpgq_kmers_size(k) * 8, k->stream));
  if (k->tail_cap)
    HPGQ_HIP_TRY(hipMemsetAsync(k->d_tail, 0, (size_t)k->tail_cap * hpgq::kmers::kNum * 8, k->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(k->d_flags, 0, 8, k->stream));
  const size_t nc = k->calls.size();
  for (size_t k0 = 0; k0 < nc; k0 += kKOvfChunk)
    HPGQ_HIP_TRY(hipMemsetAsync(k->ovf_chunks[k0 / kKOvfChunk], 0, std::min(kKOvfChunk, nc - k0) * 4, k->stream));
  k->calls.clear();
  return HPGQ_OK;
}

int hpgq_kmers_reserve_length(hpgq_kmers_t *k, int64_t max_len) {
  if (!k || max_len < 0 || max_len > INT32_MAX) return HPGQ_E_INVALID;
  const int64_t cap = max_len - (hpgq::kmers::kK - 1) - k->npos;   // starts npos .. max_len - 5
  if (cap <= k->tail_cap) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  return k_ensure_tail(k, cap);
}

int hpgq_kmers_read_ext(hpgq_kmers_t *k, uint64_t *by_pos, size_t n, int32_t *npos_ext) {
  if (!k || !npos_ext) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  const int rc = k_sync_resolve(k);
  if (rc) return rc;
  using hpgq::kmers::kNum;
  const uint32_t ml = k->h_flags[0];   // the longest counted read with starts >= npos
  const int64_t T = ml ? (int64_t)ml - (hpgq::kmers::kK - 1) - k->npos : 0;
  const int64_t P = k->npos + T;
  *npos_ext = (int32_t)P;
  if (!by_pos) return HPGQ_OK;
  if (n < (size_t)kNum * (size_t)P) return HPGQ_E_INVALID;
  std::vector<uint64_t> dense((size_t)kNum * k->npos), tail((size_t)T * kNum);
  if (!dense.empty())
    HPGQ_HIP_TRY(hipMemcpyAsync(dense.data(), k->d_out, dense.size() * 8, hipMemcpyDeviceToHost, k->stream));
  if (T) HPGQ_HIP_TRY(hipMemcpyAsync(tail.data(), k->d_tail, tail.size() * 8, hipMemcpyDeviceToHost, k->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(k->stream));
  for (int id = 0; id < kNum; ++id) {
    uint64_t *o = by_pos + (size_t)id * P;
    if (k->npos) std::memcpy(o, dense.data() + (size_t)id * k->npos, (size_t)k->npos * 8);
    for (int64_t i = 0; i < T; ++i) o[k->npos + i] = tail[(size_t)i * kNum + id];
  }
  return HPGQ_OK;
}

size_t hpgq_kmers_size(const hpgq_kmers_t *k) {
  return k ? (size_t)hpgq::kmers::kNum * (size_t)k->npos : 0;
}

int hpgq_kmers_read(hpgq_kmers_t *k, uint64_t *by_pos, size_t n) {
  if (!k || (!by_pos && n) || n < hpgq_kmers_size(k)) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(k->device));
  const int rc = k_sync_resolve(k);
  if (rc) return rc;
  if (hpgq_kmers_size(k))
    HPGQ_HIP_TRY(hipMemcpy(by_pos, k->d_out, hpgq_kmers_size(k) * 8, hipMemcpyDeviceToHost));
  return HPGQ_OK;
}

uint64_t *hpgq_kmers_device(hpgq_kmers_t *k) { return k ? (uint64_t *)k->d_out : nullptr; }

}  // extern "C"
