// hpgq_engine.hip — libhpgq: engine context, the kernel chain and the C-ABI.
// The kernels live in hpgq_engine_kernel.h (catch-all, routing) and
// hpgq_engine_tri.h (segmented), instantiated per geometry in
// hpgq_engine_geo.hip.

#include "hpgq_engine_kernel.h"
#include "hpgq_engine_tri.h"

// ===========================================================================
// C-ABI
// ===========================================================================

#include <cctype>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rccl/rccl.h>
#include <vector>

namespace {

// one kernel of the chain
struct Stage {
  const void *fn = nullptr;
  size_t lds = 0;
  int grid = 0;
  int block = 0;           // reads per unit (direct stages)
  int defer_len = INT_MAX;
  bool follow = false;
  char name[80] = {0};
};

// the kernels of one call: s1 takes the batch; s2 (wide segmented) and s3
// (catch-all) take what the stage before deferred
struct Chain {
  Stage s1, s2, s3;
  bool has2 = false, has3 = false;
};

// flags words behind the counters (one memset clears both): deferred-read
// counts by call parity, the longest merged window longer than lmax, the
// longest one the tail could not hold (hpgq_sync's second pass), and that
// pass's read count
enum { FL_PEND1 = 0, FL_PEND2 = 2, FL_MAXLEN = 5, FL_NEED = 6, FL_REDO = 7, FL_WORDS = 8 };

// a device-path call since the last sync, kept for the long-read tail's second
// pass (hpgq_sync): its batch and the tail's end when it ran
struct CallRec {
  const char *seq[2], *qual[2];
  const int32_t *idx[2];
  int64_t n;
  int tail_hi;
};
constexpr size_t kOvfChunk = 4096;   // per-call overflow flags per device chunk

// adaptive first stage: a ctx whose reads may be long keeps two chains, hex
// first (short reads; long ones deferred to wide) and wide first (long reads),
// and picks per call from the previous calls' deferral reports
constexpr int kProbeEvery = 16;   // wide-first calls between two hex-first probes

}  // namespace

struct hpgq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hpgq_params_t p{};
  int nm = 1;
  size_t clen = 0;
  // d_state: [nm * clen] u64 counters | FL_WORDS u32 (deferred-read counts by
  // call parity, error flag)
  uint64_t *d_state = nullptr;
  uint32_t *d_flags = nullptr;
  uint64_t *d_global = nullptr;   // hpgq_allreduce output
  bool reduced = false;           // d_global is current (no run / reset since)
  hpgq::ColdParams *d_cold = nullptr;
  Chain ch[2];              // [0]: the ctx's chain; [1]: wide first (adaptive only)
  bool adaptive = false;
  int mode = 0;              // chain of the next call
  int wide_calls = 0;        // calls since the last probe in wide-first mode
  // mapped host word: deferred count | call sequence number << 32 (one 8-byte
  // store by the follow-up stage); the call's read count stays on the host
  uint32_t *h_report = nullptr, *d_report = nullptr;
  uint32_t seq = 0;          // sequence number of the last call's report
  int64_t rep_reads[16] = {0};   // reads of call `seq`, by seq & 15
  uint32_t min_seq = 0;      // reports older than this (before a probe) are ignored
  int parity = 0;
  int route = HPGQ_ROUTE_AUTO;   // hpgq_debug_set_route (tests, A/B); never from the environment
  int cus = 0;
  uint64_t *d_bits1 = nullptr, *d_bits2 = nullptr;   // deferred reads per s1 unit
  size_t bits_cap = 0;
  // host path (hpgq_run_host): two staging slots, each a pinned host buffer
  // and a device buffer for one batch and its outputs.  The caller's batch is
  // copied into the slot's pinned buffer in chunks, each chunk's H2D queued on
  // the copy stream as soon as it is filled; the engine stream waits for the
  // slot's copies only, so one batch's H2D overlaps the previous batch's
  // kernels.  Outputs come back into the slot's pinned buffer and reach the
  // caller's arrays in hpgq_sync (or when the slot is reused).
  hipStream_t cstream = nullptr;
  struct Slot {
    char *h = nullptr, *d = nullptr;   // [seq | qual | idx] per mate, then mask | trim
    size_t cap = 0;
    hipEvent_t copied = nullptr, used = nullptr;   // H2D done / the slot's kernels + D2H done
    bool busy = false;
    uint8_t *mask_dst = nullptr;   // caller outputs waiting for this slot's D2H
    uint32_t *trim_dst = nullptr;
    size_t mask_off = 0, trim_off = 0, nreads = 0, ntrim = 0;   // ntrim: reads x mates
  } slot[2];
  int cur_slot = 0;
  // hpgq_host_batch: the slot reserved for a batch the caller writes in place
  // (-1: none), and its size; hpgq_run_host on exactly that batch DMAs it
  int staged = -1;
  int64_t staged_n = 0;
  size_t staged_bytes[2] = {0, 0};
  uint32_t *h_flags = nullptr;   // pinned: the FL_WORDS flags, copied back by hpgq_sync
  ncclComm_t comm = nullptr;
  // the long-read tail: [tail_cap][nm][8] u64 from position
  // lmax on (EngineArgs::tail); grown by the host, never by a kernel
  uint64_t *d_tail = nullptr;
  int64_t tail_cap = 0;
  uint64_t *d_gtail = nullptr;   // its sum over the ranks (hpgq_read_counters_ext)
  size_t gtail_cap = 0;
  uint32_t *d_scratch = nullptr;   // 16 u32 for small RCCL exchanges
  std::vector<CallRec> calls;           // device-path calls since the last sync
  std::vector<uint32_t *> ovf_chunks;   // their overflow flags, kOvfChunk per chunk
  Stage redo;                           // the catch-all's follow-up instance (TAIL_ONLY pass)
};

// biased thresholds for "signed byte in [phred+lo, phred+hi]" (the kernels
// compare b ^ 0x80 = (signed char)b + 128, hpgq_engine_kernel.h kQFlip) with
// the clamps folded into flags
static void raw_range(int phred, int lo_q, int hi_q, uint32_t &lo4, uint32_t &hi4, int &lo_none,
                      int &hi_none, int &none_in) {
  const int64_t lo = (int64_t)phred + hpgq::kQBias + lo_q;
  const int64_t hi1 = (int64_t)phred + hpgq::kQBias + hi_q + 1;
  lo_none = lo <= 0;
  hi_none = hi1 > 255;
  none_in = lo > 255 || hi1 <= 0 || lo >= hi1;
  const uint32_t lob = (uint32_t)(lo < 0 ? 0 : lo > 255 ? 255 : lo);
  const uint32_t hib = (uint32_t)(hi1 < 0 ? 0 : hi1 > 255 ? 255 : hi1);
  lo4 = lob * 0x01010101u;
  hi4 = hib * 0x01010101u;
}

// the segmented kernels' branch-free form of one edit side's range (TrimSide)
static void trim_side(uint32_t lo4, uint32_t hi4, int hi_none, int none_in, hpgq::TrimSide &S) {
  if (none_in) lo4 = hi4 = 0;   // every byte >= both bounds: none in range
  S.lq = lo4 ^ hpgq::kQFlip;
  S.l7 = lo4 & 0x7F7F7F7Fu;
  S.hq = hi_none && !none_in ? 0u : hi4 ^ hpgq::kQFlip;   // (no upper bound: ">= hi" never holds)
  S.h7 = hi_none && !none_in ? hpgq::kQFlip : hi4 & 0x7F7F7F7Fu;
}

static int clamp_q(int q) { return q < -512 ? -512 : (q > 512 ? 512 : q); }

// engine flags from the parameters
static int engine_flags(const hpgq_params_t &p) {
  int f = 0;
  if (p.filter_on) f |= hpgq::F_FILTER;
  if (p.edit_on) f |= hpgq::F_EDIT;
  if (p.stats_on) f |= hpgq::F_STATS;
  // reads of any length are filtered, so any bound can bite (the segmented
  // kernels only count N / out-of-range when it can bite on their reads: nx_bites)
  if (p.filter_on && p.max_N < INT_MAX) f |= hpgq::F_NEED_N;
  if (p.filter_on && p.max_out_of_quality < INT_MAX) f |= hpgq::F_NEED_OOR;
  if (p.filter_on && (p.left_length > 0 || p.right_length > 0)) f |= hpgq::F_NEED_LR;
  // out of range  <=>  raw < phred + min_q  or  raw > phred + max_q
  uint32_t lo4, hi4;
  int lo_none = 0, hi_none = 0, none_in = 0;
  raw_range(p.phred, p.min_read_quality, p.max_read_quality, lo4, hi4, lo_none, hi_none, none_in);
  if (lo_none) f |= hpgq::F_OOR_LO_NONE;
  if (hi_none) f |= hpgq::F_OOR_HI_NONE;
  if (none_in) f |= hpgq::F_OOR_ALL;
  return f;
}

static bool needs_generic(int flags) {
  return flags & (hpgq::F_EDIT | hpgq::F_NEED_N | hpgq::F_NEED_OOR | hpgq::F_NEED_LR);
}

static void fill_args(const hpgq_ctx *c, hpgq::EngineArgs &A) {
  const hpgq_params_t &p = c->p;
  A.lmax = p.lmax;
  A.clen = (int)c->clen;
  A.phred = p.phred + hpgq::kQBias;   // the kernels sum biased bytes (signed char + 128)
  A.cold = c->d_cold;
  A.flags = engine_flags(p);
  A.min_len = p.min_read_length;
  A.max_len = p.max_read_length;
  // mean Q = (signed) raw - phred lies in [-383, 127]: clamping keeps every product in int32
  A.min_q = clamp_q(p.min_read_quality);
  A.max_q = clamp_q(p.max_read_quality);
}

static void cold_params(const hpgq_params_t &p, hpgq::ColdParams &C) {
  C.left_len = p.left_length;
  C.min_left = p.min_left_quality;
  C.max_left = p.max_left_quality;
  C.right_len = p.right_length;
  C.min_right = p.min_right_quality;
  C.max_right = p.max_right_quality;
  C.e_left_len = p.edit_on ? p.edit_left_length : 0;
  C.e_right_len = p.edit_on ? p.edit_right_length : 0;
  raw_range(p.phred, p.edit_min_left_quality, p.edit_max_left_quality, C.el_lo4, C.el_hi4,
            C.el_lo_none, C.el_hi_none, C.el_none_in);
  raw_range(p.phred, p.edit_min_right_quality, p.edit_max_right_quality, C.er_lo4, C.er_hi4,
            C.er_lo_none, C.er_hi_none, C.er_none_in);
  trim_side(C.el_lo4, C.el_hi4, C.el_hi_none, C.el_none_in, C.tl);
  trim_side(C.er_lo4, C.er_hi4, C.er_hi_none, C.er_none_in, C.tr);
  int lo_none, hi_none, none_in;
  raw_range(p.phred, p.min_read_quality, p.max_read_quality, C.oor_lo4, C.oor_hi4, lo_none,
            hi_none, none_in);
  trim_side(C.oor_lo4, C.oor_hi4, hi_none, none_in, C.to);   // (no lower bound: lo4 = 0, ">= lo" always holds)
  C.max_n = p.max_N;
  C.max_oor = p.max_out_of_quality;
}

template <int NM, bool GEN>
static const void *kernel_nch(int nch) {
  switch (nch) {
    case 1: return (const void *)hpgq::engine_kernel<NM, 1, GEN, false>;
    case 2: return (const void *)hpgq::engine_kernel<NM, 2, GEN, false>;
    default: return (const void *)hpgq::engine_kernel<NM, 5, GEN, false>;
  }
}

// the catch-all kernel: chunk count from lmax (the pipelined loads must hold
// every read the counters can hold; longer reads take its chunk loop)
static void catch_all(Stage &s, int nm, int lmax, bool gen, bool follow) {
  int nch = (lmax + hpgq::kChunk - 1) / hpgq::kChunk;
  if (nch > 2 || follow) nch = 5;   // instantiated chunk counts: 1, 2, 5
  if (follow)   // the follow-up instance: every option, five chunks (reads <= 1260 pipelined)
    s.fn = nm == 2 ? (const void *)hpgq::engine_kernel<2, 5, true, true>
                   : (const void *)hpgq::engine_kernel<1, 5, true, true>;
  else
    s.fn = nm == 2 ? (gen ? kernel_nch<2, true>(nch) : kernel_nch<2, false>(nch))
                   : (gen ? kernel_nch<1, true>(nch) : kernel_nch<1, false>(nch));
  s.follow = follow;
  s.block = 64;
  std::snprintf(s.name, sizeof(s.name), "hpgq::engine_kernel<%d, %d, %s>%s", nm, nch, gen ? "true" : "false",
                follow ? " (follow-up)" : "");
}

static size_t seg_lds(const hpgq_params_t &p, int nm, int xm, int pos, bool follow = false, int block = 0) {
  const size_t lp = (size_t)std::min(p.lmax, pos);   // the kernel's on-chip positions (tri_body: lp)
  const size_t hlen = lp + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  const size_t mate_words = (size_t)6 * lp + ((hlen + 1) & ~(size_t)1) + 2 * HPGQ_NUM_SCALARS;
  // per mate [6][lmax] + hist + scalars, 16 B alignment, the byte-mask table,
  // per wave and mate two read tables (2 x 1 KB) + segment ends (+ one list per
  // extra scan) + the per-lane mean-quality sums, per wave a compaction scratch
  // and a deferral word
  const size_t lists = 1 + ((xm & hpgq::X_NOOR) ? 1 : 0) + ((xm & hpgq::X_LR) ? 1 : 0);
  // (+ paired-end edit, first stage, no extra scans: the DMA rows of the next
  // unit's trim windows, 3 x block x 16 B per mate, tri_body TDMA)
  const bool tdma = p.edit_on && !follow && nm == 2 && xm == 0;
  const size_t dma_words = tdma ? (size_t)nm * 3 * (size_t)block * 4 : 0;
  const size_t st_words = (xm & hpgq::X_ST) ? (size_t)hpgq::kStWords : 0;   // (tri_body ST's shift buffers)
  // (after the byte-mask table: the reciprocal table [pos + 1] of the epilogue's divisions)
  return (size_t)nm * mate_words * 4 + 16 + 17 * 16 + ((size_t)pos + 1) * 4 +
         (size_t)hpgq::kWaves * ((size_t)nm * (2 * 256 + 64 * lists + hpgq::kFxWords) + 64 + 4 + dma_words + st_words) * 4;
}

static size_t catch_all_lds(const hpgq_params_t &p, int nm) {
  const size_t hlen = (size_t)p.lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
  const size_t hist_words = ((size_t)nm * hlen + 1) & ~(size_t)1;
  return ((size_t)nm * 6 * p.lmax + hist_words) * 4 + (size_t)nm * HPGQ_NUM_SCALARS * 8 +
         sizeof(hpgq::ColdParams) + (size_t)hpgq::kWaves * 64 * 4;
}

static int seg_block(int geo) {
  return geo == hpgq::GEO_TRI ? hpgq::Geo<hpgq::GEO_TRI>::kBlock
                              : (geo == hpgq::GEO_HEX ? hpgq::Geo<hpgq::GEO_HEX>::kBlock
                                                      : hpgq::Geo<hpgq::GEO_WIDE>::kBlock);
}

static int seg_pos(int geo) {
  return geo == hpgq::GEO_TRI ? hpgq::Geo<hpgq::GEO_TRI>::kPos
                              : (geo == hpgq::GEO_HEX ? hpgq::Geo<hpgq::GEO_HEX>::kPos
                                                      : hpgq::Geo<hpgq::GEO_WIDE>::kPos);
}

static bool seg_stage(Stage &s, int geo, int nm, bool edit, int xm, bool follow) {
  hpgq::SegChoice ch{};
  if (geo == hpgq::GEO_TRI) ch = hpgq::seg_kernel_tri(nm, edit, xm, follow, s.name, sizeof(s.name));
  else if (geo == hpgq::GEO_HEX) ch = hpgq::seg_kernel_hex(nm, edit, xm, follow, s.name, sizeof(s.name));
  else ch = hpgq::seg_kernel_wide(nm, edit, xm, follow, s.name, sizeof(s.name));
  s.fn = ch.fn;
  s.follow = follow;
  s.block = seg_block(geo);
  return ch.fn != nullptr;
}

static int finish_stage(hpgq_ctx *c, Stage &s, size_t lds, int cus) {
  s.lds = lds;
  if (s.lds > 64 * 1024)
    HPGQ_HIP_TRY(hipFuncSetAttribute(s.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s.lds));
  int per_cu = 0;
  HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, s.fn, hpgq::kWG, s.lds));
  if (per_cu < 1) per_cu = 1;
  s.grid = cus * per_cu;   // persistent: every workgroup resident, grid-stride over units
  return HPGQ_OK;
}

// Route by the reads' ACTUAL lengths: the first stage is the
// segmented kernel whenever the options allow one; it defers the reads it
// cannot hold, the wide geometry takes those up to 252 bases and the
// catch-all takes the rest.  lmax only sizes the counters, so a ctx opened
// with the CLI's lmax 1024 runs 150 bp reads on the hex geometry.
static int plan_chain(hpgq_ctx *c, Chain &ch, int cus, int geo_force) {
  const hpgq_params_t &p = c->p;
  const int fl = engine_flags(p);
  const bool stats = fl & hpgq::F_STATS;
  const bool lr = fl & hpgq::F_NEED_LR;
  // N / out-of-range limits can only bite on a segmented kernel's reads (<= 252
  // bases) when they are below 252; else the plain variant runs
  const int posw = hpgq::Geo<hpgq::GEO_WIDE>::kPos;
  const bool nx = p.filter_on && (p.max_N < posw || p.max_out_of_quality < posw);
  // extra per-step scans: N / out-of-range counts, window sums
  const int xm = (nx ? hpgq::X_NOOR : 0) | (lr ? hpgq::X_LR : 0);
  const bool edit = fl & hpgq::F_EDIT;
  if ((c->route & 0xF) == HPGQ_ROUTE_CATCH_ALL) {   // the catch-all alone (tests)
    catch_all(ch.s1, c->nm, p.lmax, needs_generic(fl), false);
    return finish_stage(c, ch.s1, catch_all_lds(p, c->nm), cus);
  }
  // first geometry: hex for short reads; wide when the counters say reads are
  // 157..252 long (or when forced: adaptive wide-first chain, hpgq_debug_set_route)
  int geo = (stats && p.lmax > hpgq::Geo<hpgq::GEO_HEX>::kPos && p.lmax <= posw) ? hpgq::GEO_WIDE
                                                                                 : hpgq::GEO_HEX;
  if (geo_force >= 0) geo = geo_force;
  // single-end edit on hex with the usual trim windows and a left length <= 12
  // (every shift fits one lane's bytes and its neighbour's): the trims are
  // applied at the step (tri_body ST), so no load waits for them
#ifndef HPGQ_NO_ST
  const bool st = edit && c->nm == 1 && xm == 0 && geo == hpgq::GEO_HEX && p.edit_left_length <= 12 &&
                  p.edit_right_length <= 32;
#else
  const bool st = false;   // (A/B builds: the unit-prologue trims)
#endif
  const int xm1 = st ? hpgq::X_ST : xm;
  if (!seg_stage(ch.s1, geo, c->nm, edit, xm1, false)) return HPGQ_E_INVALID;
  const int pos1 = seg_pos(geo);
  // a merged read longer than lmax leaves the segmented kernels (the
  // catch-all counts it as a long read)
  ch.s1.defer_len = stats ? std::min(pos1, p.lmax) : pos1;
  int rc = finish_stage(c, ch.s1, seg_lds(p, c->nm, xm1, pos1, false, seg_block(geo)), cus);
  if (rc) return rc;
  ch.has2 = geo != hpgq::GEO_WIDE && ch.s1.defer_len < posw && !(stats && p.lmax <= pos1);
  if (ch.has2) {
    if (!seg_stage(ch.s2, hpgq::GEO_WIDE, c->nm, edit, xm, true)) return HPGQ_E_INVALID;
    ch.s2.defer_len = stats ? std::min(posw, p.lmax) : posw;
    rc = finish_stage(c, ch.s2, seg_lds(p, c->nm, xm, posw, true), cus);
    if (rc) return rc;
  }
  ch.has3 = true;
  catch_all(ch.s3, c->nm, p.lmax, true, true);
  return finish_stage(c, ch.s3, catch_all_lds(p, c->nm), cus);
}

static int plan(hpgq_ctx *c, int cus) {
  // a fixed first geometry only when hpgq_debug_set_route asks for one (tests, A/B)
  const int r = c->route & 0xF;
  const int geo_force = r == HPGQ_ROUTE_FIRST_TRI ? hpgq::GEO_TRI
                        : r == HPGQ_ROUTE_FIRST_HEX ? hpgq::GEO_HEX
                        : r == HPGQ_ROUTE_FIRST_WIDE ? hpgq::GEO_WIDE : -1;
  int rc = plan_chain(c, c->ch[0], cus, geo_force);
  if (rc) return rc;
  // hex first with a wide follow-up: batches of mostly long reads run better
  // wide first, so keep that chain too and choose per call
  c->adaptive = c->ch[0].has2 && geo_force < 0 && !(c->route & HPGQ_ROUTE_NO_ADAPTIVE);
  if (!c->adaptive) return HPGQ_OK;
  rc = plan_chain(c, c->ch[1], cus, hpgq::GEO_WIDE);
  if (rc) return rc;
  void *h = nullptr;
  HPGQ_HIP_TRY(hipHostMalloc(&h, 64, hipHostMallocMapped));
  c->h_report = static_cast<uint32_t *>(h);
  *reinterpret_cast<volatile uint64_t *>(c->h_report) = 0;
  void *d = nullptr;
  HPGQ_HIP_TRY(hipHostGetDevicePointer(&d, h, 0));
  c->d_report = static_cast<uint32_t *>(d);
  return HPGQ_OK;
}

// the chain for the next call: wide first when the last report says at least
// half of a batch's reads were deferred past hex; a hex-first probe every
// kProbeEvery wide-first calls (its report clears the way back)
static int pick_chain(hpgq_ctx *c) {
  if (!c->adaptive) return 0;
  const uint64_t r = *reinterpret_cast<volatile uint64_t *>(c->h_report);
  const uint32_t deferred = (uint32_t)r, rseq = (uint32_t)(r >> 32);
  const int64_t reads = c->rep_reads[rseq & 15];
  // (a report from before the last probe may still land after it: ignored;
  // so is one too old for the read-count ring, which cannot happen in practice)
  const bool known = rseq != 0 && reads > 0 && (int32_t)(rseq - c->min_seq) >= 0 && c->seq - rseq < 16;
  const bool mostly_long = known && (uint64_t)deferred * 2 >= reads;
  if (c->mode == 0) {
    if (mostly_long) {
      c->mode = 1;
      c->wide_calls = 0;
    }
  } else if (known && !mostly_long) {
    c->mode = 0;
  } else if (++c->wide_calls >= kProbeEvery) {
    c->wide_calls = 0;
    c->min_seq = c->seq + 1;   // the probe's own report decides
    return 0;
  }
  return c->mode;
}

// The long-read tail's second pass (hpgq_sync): per 64-read unit, the reads
// (pairs) with a mate longer than p0 -- the only ones whose windows can reach
// past the tail a call had -- as bits + a count for the catch-all's follow-up
// instance (F_TAIL_ONLY).  Every unit's word is written.
__global__ void __launch_bounds__(256) tail_bits_kernel(const int32_t *idx0, const int32_t *idx1, int64_t n,
                                                        int p0, uint64_t *bits, uint32_t *count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool on = false;
  if (r < n) {
    on = idx0[r + 1] - idx0[r] > p0;
    if (idx1) on = on || idx1[r + 1] - idx1[r] > p0;
  }
  const uint64_t b = __ballot(on);
  if ((threadIdx.x & 63) == 0 && r < n) {
    bits[r >> 6] = b;
    if (b) atomicAdd(count, (uint32_t)__builtin_popcountll(b));
  }
}

extern "C" {

const char *hpgq_kernel_name(const hpgq_ctx_t *ctx) { return ctx ? ctx->ch[0].s1.name : ""; }

const char *hpgq_kernel_chain(const hpgq_ctx_t *ctx) {
  static thread_local char buf[700];
  if (!ctx) return "";
  int o = 0;
  for (int k = 0; k < (ctx->adaptive ? 2 : 1); ++k) {
    const Chain &ch = ctx->ch[k];
    o += std::snprintf(buf + o, sizeof(buf) - o, "%s%s%s%s%s%s", k ? " | adaptive: " : "", ch.s1.name,
                       ch.has2 ? " -> " : "", ch.has2 ? ch.s2.name : "", ch.has3 ? " -> " : "",
                       ch.has3 ? ch.s3.name : "");
  }
  return buf;
}

int hpgq_host_alloc(void **ptr, size_t bytes) {
  if (!ptr) return HPGQ_E_INVALID;
  *ptr = nullptr;
  if (hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return HPGQ_E_NOMEM;
  return HPGQ_OK;
}

void hpgq_host_free(void *ptr) {
  if (ptr) (void)hipHostFree(ptr);
}

int hpgq_device_alloc(int device, void **ptr, size_t bytes) {
  if (!ptr) return HPGQ_E_INVALID;
  *ptr = nullptr;
  HPGQ_HIP_TRY(hipSetDevice(device));
  if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess) return HPGQ_E_NOMEM;
  return HPGQ_OK;
}

void hpgq_device_free(void *ptr) {
  if (ptr) (void)hipFree(ptr);
}

int hpgq_copy_to_host(hpgq_ctx_t *c, void *dst, const void *src_dev, size_t bytes) {
  if (!c || (!dst && bytes) || (!src_dev && bytes)) return HPGQ_E_INVALID;
  if (!bytes) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemcpyAsync(dst, src_dev, bytes, hipMemcpyDeviceToHost, c->stream));
  return HPGQ_OK;
}

int hpgq_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hpgq_device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device) != hipSuccess) return -1;
  for (char *q = bus; *q; ++q) *q = (char)std::tolower((unsigned char)*q);   // sysfs names are lower case
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

static int validate_params(const hpgq_params_t *p) {
  if (!p) return HPGQ_E_INVALID;
  if (p->lmax < 1 || p->lmax > HPGQ_LMAX_LIMIT) return HPGQ_E_INVALID;
  if (p->phred < 0 || p->phred > 255) return HPGQ_E_INVALID;
  // trims come back as two 16-bit fields (trim_out): a window is at most 65535
  if (p->edit_on && (p->edit_left_length > HPGQ_MAX_EDIT_LENGTH || p->edit_right_length > HPGQ_MAX_EDIT_LENGTH))
    return HPGQ_E_INVALID;
  return HPGQ_OK;
}

static size_t state_bytes(const hpgq_ctx *c) { return c->clen * c->nm * sizeof(uint64_t) + FL_WORDS * 4; }

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
  HPGQ_HIP_TRY(hipSetDevice(device));
  HPGQ_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HPGQ_HIP_TRY(hipMalloc(&c->d_state, state_bytes(c)));
  c->d_flags = reinterpret_cast<uint32_t *>(c->d_state + c->clen * c->nm);
  HPGQ_HIP_TRY(hipMalloc(&c->d_global, c->clen * c->nm * sizeof(uint64_t)));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_state, 0, state_bytes(c), c->stream));
  HPGQ_HIP_TRY(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  HPGQ_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->h_flags), FL_WORDS * 4, hipHostMallocDefault));
  std::memset(c->h_flags, 0, FL_WORDS * 4);
  HPGQ_HIP_TRY(hipMalloc(&c->d_scratch, 64));
  for (auto &sl : c->slot) {
    HPGQ_HIP_TRY(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
    HPGQ_HIP_TRY(hipEventCreateWithFlags(&sl.used, hipEventDisableTiming));
  }
  HPGQ_HIP_TRY(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device));
  rc = plan(c, c->cus);
  if (rc == HPGQ_OK) {   // the long-read tail's second pass: the catch-all's follow-up instance
    catch_all(c->redo, c->nm, p->lmax, true, true);
    rc = finish_stage(c, c->redo, catch_all_lds(c->p, c->nm), c->cus);
  }
  if (rc) {
    hpgq_close(c);
    return rc;
  }
  {
    hpgq::ColdParams cp{};
    cold_params(c->p, cp);
    HPGQ_HIP_TRY(hipMalloc(&c->d_cold, sizeof(cp)));
    HPGQ_HIP_TRY(hipMemcpy(c->d_cold, &cp, sizeof(cp), hipMemcpyHostToDevice));
  }
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  *out = c;
  return HPGQ_OK;
}

void hpgq_close(hpgq_ctx_t *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  // outputs of host-path calls not yet delivered (no hpgq_sync since) are
  // dropped, never written: the caller may already have freed those arrays
  for (auto &sl : c->slot) {
    sl.mask_dst = nullptr;
    sl.trim_dst = nullptr;
    sl.busy = false;
  }
  if (c->comm) ncclCommDestroy(c->comm);
  (void)hipFree(c->d_state);
  (void)hipFree(c->d_global);
  (void)hipFree(c->d_cold);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  (void)hipFree(c->d_bits1);
  (void)hipFree(c->d_bits2);
  for (auto &sl : c->slot) {
    (void)hipFree(sl.d);
    if (sl.h) (void)hipHostFree(sl.h);
    if (sl.copied) (void)hipEventDestroy(sl.copied);
    if (sl.used) (void)hipEventDestroy(sl.used);
  }
  if (c->h_flags) (void)hipHostFree(c->h_flags);
  (void)hipFree(c->d_tail);
  (void)hipFree(c->d_gtail);
  (void)hipFree(c->d_scratch);
  for (uint32_t *q : c->ovf_chunks) (void)hipFree(q);
  if (c->h_report) (void)hipHostFree(c->h_report);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// per-unit deferral masks for a batch of n reads
static int ensure_bits(hpgq_ctx *c, int64_t n) {
  const int block = std::min(c->ch[0].s1.block, c->adaptive ? c->ch[1].s1.block : INT_MAX);
  const size_t units = (size_t)((n + block - 1) / block) + 1;
  if (units <= c->bits_cap) return HPGQ_OK;
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  (void)hipFree(c->d_bits1);
  (void)hipFree(c->d_bits2);
  c->d_bits1 = c->d_bits2 = nullptr;
  c->bits_cap = 0;
  const size_t cap = units + units / 4 + 64;
  if (hipMalloc(&c->d_bits1, cap * 8) != hipSuccess) return HPGQ_E_NOMEM;
  if (hipMalloc(&c->d_bits2, cap * 8) != hipSuccess) return HPGQ_E_NOMEM;
  c->bits_cap = cap;
  return HPGQ_OK;
}

static int launch_stage(hpgq_ctx *c, const Stage &s, hpgq::EngineArgs &A) {
  const int64_t units = s.follow ? A.nunits : (A.num_reads + s.block - 1) / s.block;
  const int64_t need = (units + hpgq::kWaves - 1) / hpgq::kWaves;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(need, s.grid));
  void *args[] = {&A};
  HPGQ_HIP_TRY(hipLaunchKernel(s.fn, dim3(grid), dim3(hpgq::kWG), args, s.lds, c->stream));
  return HPGQ_OK;
}

// Grow the long-read tail to hold positions [lmax, lmax + cap).  Waits for
// the ctx stream first (kernels in flight add into the old tail); the new
// entries are zero.  Host decisions only: a kernel never needs more than the
// tail it was launched with (a longer window flags its call, see resolve).
static int ensure_tail(hpgq_ctx *c, int64_t cap) {
  if (cap <= c->tail_cap) return HPGQ_OK;
  const int64_t limit = (int64_t)INT32_MAX - c->p.lmax;   // tail_hi is an int
  if (cap > limit) return HPGQ_E_INVALID;
  int64_t nc = std::max<int64_t>(cap, c->tail_cap + c->tail_cap / 2);
  nc = std::min<int64_t>((nc + 255) & ~(int64_t)255, limit);
  const size_t row = (size_t)c->nm * 8 * sizeof(uint64_t);
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  uint64_t *d = nullptr;
  if (hipMalloc(&d, (size_t)nc * row) != hipSuccess) return HPGQ_E_NOMEM;
  const size_t old = (size_t)c->tail_cap * row;
  if (old) HPGQ_HIP_TRY(hipMemcpyAsync(d, c->d_tail, old, hipMemcpyDeviceToDevice, c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(reinterpret_cast<char *>(d) + old, 0, (size_t)nc * row - old, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  (void)hipFree(c->d_tail);
  c->d_tail = d;
  c->tail_cap = nc;
  return HPGQ_OK;
}

static int tail_hi(const hpgq_ctx *c) {
  return (int)std::min<int64_t>((int64_t)c->p.lmax + c->tail_cap, INT32_MAX);
}

// the chain over one batch (A: batch, outputs and options filled in).
// record: a device-path call, kept (batch pointers + the tail's end) for the
// tail's second pass in case one of its windows is longer than the tail
static int launch(hpgq_ctx *c, hpgq::EngineArgs &A, bool record) {
  if (A.num_reads <= 0) return HPGQ_OK;
  if (A.num_reads > INT32_MAX) return HPGQ_E_INVALID;   // read ids are 32-bit in the follow-up stages
  A.counters = c->d_state;
  A.err = nullptr;
  A.report = nullptr;
  A.tail = c->d_tail;
  A.tail_lo = c->p.lmax;
  A.tail_hi = tail_hi(c);
  A.maxlen = c->d_flags + FL_MAXLEN;
  A.need = c->d_flags + FL_NEED;
  A.ovf = nullptr;
  if (record && c->p.stats_on) {
    const size_t k = c->calls.size();
    if (k / kOvfChunk >= c->ovf_chunks.size()) {
      uint32_t *q = nullptr;
      if (hipMalloc(&q, kOvfChunk * 4) != hipSuccess) return HPGQ_E_NOMEM;
      c->ovf_chunks.push_back(q);
      HPGQ_HIP_TRY(hipMemsetAsync(q, 0, kOvfChunk * 4, c->stream));
    }
    A.ovf = c->ovf_chunks[k / kOvfChunk] + k % kOvfChunk;
    CallRec r{};
    for (int m = 0; m < c->nm; ++m) {
      r.seq[m] = A.seq[m];
      r.qual[m] = A.qual[m];
      r.idx[m] = A.idx[m];
    }
    r.n = A.num_reads;
    r.tail_hi = A.tail_hi;
    c->calls.push_back(r);
  }
  c->reduced = false;
  const int k = pick_chain(c);
  const Chain &ch = c->ch[k];
  if (!ch.has3) {   // the catch-all alone
    A.unit_bits = A.unit_and = nullptr;
    A.pending = A.pending_clear = A.pending_clear2 = nullptr;
    A.defer_bits = nullptr;
    A.defer_count = nullptr;
    A.defer_len = INT_MAX;
    return launch_stage(c, ch.s1, A);
  }
  int rc = ensure_bits(c, A.num_reads);
  if (rc) return rc;
  const int s = c->parity, o = s ^ 1;
  c->parity = o;
  uint32_t *f = c->d_flags;
  // stage 1: every read; deferrals -> bits1, count -> PEND1[s]
  hpgq::EngineArgs A1 = A;
  A1.unit_bits = A1.unit_and = nullptr;
  A1.pending = A1.pending_clear = A1.pending_clear2 = nullptr;
  A1.defer_bits = c->d_bits1;
  A1.defer_count = f + FL_PEND1 + s;
  A1.defer_len = ch.s1.defer_len;
  rc = launch_stage(c, ch.s1, A1);
  if (rc) return rc;
  const int64_t nunits = (A.num_reads + ch.s1.block - 1) / ch.s1.block;
  const uint64_t *last_bits = c->d_bits1;
  const uint32_t *last_count = f + FL_PEND1 + s;
  uint32_t *last_clear = f + FL_PEND1 + o;
  const uint64_t *and_bits = nullptr;
  if (ch.has2) {   // stage 2: the deferred reads up to 252 bases; longer -> bits2, PEND2[s]
    hpgq::EngineArgs A2 = A;
    A2.unit_bits = c->d_bits1;
    A2.unit_and = nullptr;
    A2.nunits = nunits;
    A2.unit_reads = ch.s1.block;
    A2.pending = last_count;
    A2.pending_clear = last_clear;
    A2.pending_clear2 = nullptr;
    A2.defer_bits = c->d_bits2;
    A2.defer_count = f + FL_PEND2 + s;
    A2.defer_len = ch.s2.defer_len;
    A2.report = c->d_report;   // how many reads hex deferred: the next call's choice
    A2.report_seq = ++c->seq;
    if (!c->seq) A2.report_seq = ++c->seq;   // 0 means "no report yet"
    c->rep_reads[c->seq & 15] = A.num_reads;
    rc = launch_stage(c, ch.s2, A2);
    if (rc) return rc;
    and_bits = c->d_bits1;   // bits2 words are only written for units with bits1 set
    last_bits = c->d_bits2;
    last_count = f + FL_PEND2 + s;
    last_clear = f + FL_PEND2 + o;
  }
  hpgq::EngineArgs A3 = A;   // stage 3: the catch-all, whatever is left
  A3.unit_bits = last_bits;
  A3.unit_and = and_bits;
  A3.nunits = nunits;
  A3.unit_reads = ch.s1.block;
  A3.pending = last_count;
  A3.pending_clear = last_clear;
  // a chain without stage 2 (wide first) leaves PEND2 alone: clear the next
  // call's, or a stale count from an earlier hex-first call of that parity
  // makes its catch-all walk every unit
  A3.pending_clear2 = ch.has2 ? nullptr : f + FL_PEND2 + o;
  A3.defer_bits = nullptr;
  A3.defer_count = nullptr;
  A3.defer_len = INT_MAX;
  return launch_stage(c, ch.s3, A3);
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
  return launch(c, A, true);
}

// hand a slot's finished outputs to the caller's arrays (its D2H is done)
static void slot_deliver(hpgq_ctx::Slot &sl) {
  if (sl.mask_dst) std::memcpy(sl.mask_dst, sl.h + sl.mask_off, sl.nreads);
  if (sl.trim_dst) std::memcpy(sl.trim_dst, sl.h + sl.trim_off, sl.ntrim * sizeof(uint32_t));
  sl.mask_dst = nullptr;
  sl.trim_dst = nullptr;
  sl.busy = false;
}

// a slot for the next batch: its previous batch finished (outputs delivered)
// and room for `bytes` in both of its buffers
static int slot_acquire(hpgq_ctx *c, size_t bytes, hpgq_ctx::Slot *&out) {
  c->cur_slot ^= 1;
  hpgq_ctx::Slot &sl = c->slot[c->cur_slot];
  if (sl.busy) {
    HPGQ_HIP_TRY(hipEventSynchronize(sl.used));
    slot_deliver(sl);
  }
  if (bytes > sl.cap) {
    (void)hipFree(sl.d);
    if (sl.h) (void)hipHostFree(sl.h);
    sl.d = nullptr;
    sl.h = nullptr;
    sl.cap = 0;
    const size_t cap = bytes + bytes / 4 + 4096;
    if (hipMalloc(&sl.d, cap) != hipSuccess) return HPGQ_E_NOMEM;
    if (hipHostMalloc(reinterpret_cast<void **>(&sl.h), cap, hipHostMallocDefault) != hipSuccess) {
      sl.h = nullptr;
      return HPGQ_E_NOMEM;
    }
    sl.cap = cap;
  }
  out = &sl;
  return HPGQ_OK;
}

// the caller's bytes into the slot's pinned buffer, each kChunk piece's H2D
// queued on the copy stream as soon as it is filled (the DMA of one piece
// overlaps the memcpy of the next)
static int stage_copy(hpgq_ctx *c, hpgq_ctx::Slot &sl, size_t off, const void *src, size_t bytes) {
  constexpr size_t kChunk = (size_t)1 << 20;
  for (size_t o = 0; o < bytes; o += kChunk) {
    const size_t n = std::min(kChunk, bytes - o);
    std::memcpy(sl.h + off + o, static_cast<const char *>(src) + o, n);
    HPGQ_HIP_TRY(hipMemcpyAsync(sl.d + off + o, sl.h + off + o, n, hipMemcpyHostToDevice, c->cstream));
  }
  return HPGQ_OK;
}

// a host batch's layout in a staging slot: per mate [seq | quality |
// data_indices] (seq and quality padded by HPGQ_DEVICE_SLACK), then the mask and
// the trims; returns the slot bytes
static size_t host_layout(int nm, int64_t n, const size_t (&bytes)[2], size_t (&off)[2][3], size_t &mask_off,
                          size_t &trim_off) {
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t total = 0;
  for (int m = 0; m < nm; ++m) {
    off[m][0] = total; total += al(bytes[m] + HPGQ_DEVICE_SLACK);   // seq
    off[m][1] = total; total += al(bytes[m] + HPGQ_DEVICE_SLACK);   // quality
    off[m][2] = total; total += al((size_t)(n + 1) * 4);            // data_indices
  }
  mask_off = total;
  total += al((size_t)n);
  trim_off = total;
  total += al((size_t)n * nm * 4);
  return total;
}

int hpgq_host_batch(hpgq_ctx_t *c, int64_t num_reads, size_t nbytes, size_t nbytes2, hpgq_batch_t *b,
                    hpgq_batch_t *b2) {
  if (!c || !b || num_reads < 0 || nbytes > (size_t)INT32_MAX || nbytes2 > (size_t)INT32_MAX) return HPGQ_E_INVALID;
  if ((c->nm == 2) != (b2 != nullptr)) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  const size_t bytes[2] = {nbytes, c->nm == 2 ? nbytes2 : 0};
  size_t off[2][3], mask_off, trim_off;
  const size_t total = host_layout(c->nm, num_reads, bytes, off, mask_off, trim_off);
  c->staged = -1;
  hpgq_ctx::Slot *sp = nullptr;
  const int rc = slot_acquire(c, total, sp);
  if (rc) return rc;
  hpgq_batch_t *bs[2] = {b, b2};
  for (int m = 0; m < c->nm; ++m) {
    bs[m]->num_reads = num_reads;
    bs[m]->seq = sp->h + off[m][0];
    bs[m]->quality = sp->h + off[m][1];
    bs[m]->data_indices = reinterpret_cast<int32_t *>(sp->h + off[m][2]);
  }
  c->staged = c->cur_slot;
  c->staged_n = num_reads;
  c->staged_bytes[0] = bytes[0];
  c->staged_bytes[1] = bytes[1];
  return HPGQ_OK;
}

static int run_host_slot(hpgq_ctx *c, hpgq_ctx::Slot &sl, const hpgq_batch_t *const (&bs)[2], int64_t n,
                         const size_t (&bytes)[2], const size_t (&off)[2][3], size_t mask_off, size_t trim_off,
                         bool in_place, uint8_t *mask_out, uint32_t *trim_out);

int hpgq_run_host(hpgq_ctx_t *c, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                  uint8_t *mask_out, uint32_t *trim_out) {
  if (!c || !b) return HPGQ_E_INVALID;
  if (c->nm == 2 && (!b2 || b2->num_reads != b->num_reads)) return HPGQ_E_INVALID;
  if (c->nm == 1 && b2) return HPGQ_E_INVALID;
  const int64_t n = b->num_reads;
  if (n < 0) return HPGQ_E_INVALID;
  if (n == 0) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  const hpgq_batch_t *const bs[2] = {b, b2};
  size_t bytes[2] = {0, 0}, off[2][3], mask_off, trim_off;
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    bytes[m] = (size_t)(ix[n] - ix[0]);
  }
  const size_t total = host_layout(c->nm, n, bytes, off, mask_off, trim_off);
  if (c->p.stats_on) {   // the long-read tail from the batch's own offsets: this path never needs a second pass
    int64_t ml = 0;
    for (int m = 0; m < c->nm; ++m) {
      const int32_t *ix = bs[m]->data_indices;
      if ((int64_t)bytes[m] <= (int64_t)c->p.lmax + c->tail_cap) continue;   // no read can be longer
      for (int64_t i = 0; i < n; ++i) ml = std::max<int64_t>(ml, (int64_t)ix[i + 1] - ix[i]);
    }
    if (ml > (int64_t)c->p.lmax + c->tail_cap) {
      const int rc = ensure_tail(c, ml - c->p.lmax);
      if (rc) return rc;
    }
  }
  // a batch written in place by hpgq_host_batch: the same slot and layout
  // (sized by the staged byte counts), no host copy
  bool in_place = false;
  if (c->staged >= 0) {
    const hpgq_ctx::Slot &st = c->slot[c->staged];
    size_t so[2][3], smask, strim;
    (void)host_layout(c->nm, c->staged_n, c->staged_bytes, so, smask, strim);
    in_place = c->staged == c->cur_slot && n == c->staged_n;
    for (int m = 0; m < c->nm && in_place; ++m) {
      const int32_t *ix = bs[m]->data_indices;
      in_place = bs[m]->seq == st.h + so[m][0] && bs[m]->quality == st.h + so[m][1] &&
                 ix == reinterpret_cast<const int32_t *>(st.h + so[m][2]) && ix[0] == 0 &&
                 bytes[m] <= c->staged_bytes[m];
    }
    if (in_place) {
      std::memcpy(off, so, sizeof(off));
      mask_off = smask;
      trim_off = strim;
    }
    c->staged = -1;
  }
  hpgq_ctx::Slot *sp = nullptr;
  int rc = HPGQ_OK;
  if (in_place) sp = &c->slot[c->cur_slot];
  else if ((rc = slot_acquire(c, total, sp))) return rc;
  rc = run_host_slot(c, *sp, bs, n, bytes, off, mask_off, trim_off, in_place, mask_out, trim_out);
  if (rc) {
    // uploads may already be queued into this slot, which is not marked busy:
    // let them finish before a later call may refill or reallocate the slot
    // 
    (void)hipStreamSynchronize(c->cstream);
    (void)hipStreamSynchronize(c->stream);
  }
  return rc;
}

static int run_host_slot(hpgq_ctx *c, hpgq_ctx::Slot &sl, const hpgq_batch_t *const (&bs)[2], int64_t n,
                         const size_t (&bytes)[2], const size_t (&off)[2][3], size_t mask_off, size_t trim_off,
                         bool in_place, uint8_t *mask_out, uint32_t *trim_out) {
  int rc = HPGQ_OK;
  hpgq::EngineArgs A{};
  fill_args(c, A);
  A.num_reads = n;
  if (in_place)   // the caller wrote the slot: ONE DMA of its inputs (each HIP call costs host time)
    HPGQ_HIP_TRY(hipMemcpyAsync(sl.d, sl.h, off[c->nm - 1][2] + (size_t)(n + 1) * 4, hipMemcpyHostToDevice,
                                c->cstream));
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    if (!in_place) {
      if ((rc = stage_copy(c, sl, off[m][2], ix, (size_t)(n + 1) * 4))) return rc;
      if ((rc = stage_copy(c, sl, off[m][0], bs[m]->seq + ix[0], bytes[m]))) return rc;
      if ((rc = stage_copy(c, sl, off[m][1], bs[m]->quality + ix[0], bytes[m]))) return rc;
    }
    // absolute indices: shift the base pointers so data_indices need no rewrite
    A.seq[m] = sl.d + off[m][0] - ix[0];
    A.qual[m] = sl.d + off[m][1] - ix[0];
    A.idx[m] = reinterpret_cast<int32_t *>(sl.d + off[m][2]);
  }
  HPGQ_HIP_TRY(hipEventRecord(sl.copied, c->cstream));
  HPGQ_HIP_TRY(hipStreamWaitEvent(c->stream, sl.copied, 0));
  A.mask = mask_out ? reinterpret_cast<uint8_t *>(sl.d + mask_off) : nullptr;
  A.trim = trim_out ? reinterpret_cast<uint32_t *>(sl.d + trim_off) : nullptr;
  rc = launch(c, A, false);
  if (rc) return rc;
  if (mask_out)
    HPGQ_HIP_TRY(hipMemcpyAsync(sl.h + mask_off, sl.d + mask_off, (size_t)n, hipMemcpyDeviceToHost, c->stream));
  if (trim_out)
    HPGQ_HIP_TRY(hipMemcpyAsync(sl.h + trim_off, sl.d + trim_off, (size_t)n * c->nm * 4, hipMemcpyDeviceToHost,
                                c->stream));
  HPGQ_HIP_TRY(hipEventRecord(sl.used, c->stream));
  sl.busy = true;
  sl.mask_dst = mask_out;
  sl.trim_dst = trim_out;
  sl.mask_off = mask_off;
  sl.trim_off = trim_off;
  sl.nreads = (size_t)n;
  sl.ntrim = (size_t)n * c->nm;
  return HPGQ_OK;
}

// The long-read tail's second pass (the stream is idle, h_flags current): a
// device-path window longer than the tail its call had (FL_NEED: the longest)
// flagged its call; grow the tail and run each flagged call's batch again
// through the catch-all's follow-up instance in TAIL_ONLY mode over the reads
// with a mate longer than that call's tail end, adding the positions from
// there on and the lengths above it -- exactly what the first pass left out
// (long_merge).  Forgets the recorded calls either way.
static int resolve(hpgq_ctx *c) {
  const uint32_t need = c->h_flags[FL_NEED];
  const size_t nc = c->calls.size();
  if (need == 0) {
    c->calls.clear();
    return HPGQ_OK;
  }
  int rc = ensure_tail(c, (int64_t)need - c->p.lmax);
  if (rc) return rc;
  std::vector<uint32_t> fl(nc, 0);
  for (size_t k0 = 0; k0 < nc; k0 += kOvfChunk)
    HPGQ_HIP_TRY(hipMemcpy(fl.data() + k0, c->ovf_chunks[k0 / kOvfChunk], std::min(kOvfChunk, nc - k0) * 4,
                           hipMemcpyDeviceToHost));
  uint32_t *f = c->d_flags;
  for (size_t k = 0; k < nc; ++k) {
    if (!fl[k]) continue;
    const CallRec &r = c->calls[k];
    if ((rc = ensure_bits(c, r.n))) return rc;
    HPGQ_HIP_TRY(hipMemsetAsync(f + FL_REDO, 0, 4, c->stream));
    hipLaunchKernelGGL(tail_bits_kernel, dim3((unsigned)((r.n + 255) / 256)), dim3(256), 0, c->stream, r.idx[0],
                       c->nm == 2 ? r.idx[1] : nullptr, r.n, r.tail_hi, c->d_bits1, f + FL_REDO);
    HPGQ_HIP_TRY(hipGetLastError());
    hpgq::EngineArgs A{};
    fill_args(c, A);
    A.flags |= hpgq::F_TAIL_ONLY;
    A.num_reads = r.n;
    for (int m = 0; m < c->nm; ++m) {
      A.seq[m] = r.seq[m];
      A.qual[m] = r.qual[m];
      A.idx[m] = r.idx[m];
    }
    A.counters = c->d_state;
    A.tail = c->d_tail;
    A.tail_lo = r.tail_hi;
    A.tail_hi = tail_hi(c);
    A.maxlen = f + FL_MAXLEN;
    A.need = f + FL_NEED;
    A.unit_bits = c->d_bits1;
    A.nunits = (r.n + 63) / 64;
    A.unit_reads = 64;
    A.pending = f + FL_REDO;
    A.defer_len = INT_MAX;
    if ((rc = launch_stage(c, c->redo, A))) return rc;
  }
  HPGQ_HIP_TRY(hipMemsetAsync(f + FL_NEED, 0, 4, c->stream));
  for (size_t k0 = 0; k0 < nc; k0 += kOvfChunk)
    HPGQ_HIP_TRY(hipMemsetAsync(c->ovf_chunks[k0 / kOvfChunk], 0, std::min(kOvfChunk, nc - k0) * 4, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  c->h_flags[FL_NEED] = 0;
  c->calls.clear();
  return HPGQ_OK;
}

// wait for the stream with the flags riding back on it (no blocking copy
// after the sync), deliver the host-path outputs, then the tail's second pass
static int sync_resolve(hpgq_ctx *c) {
  HPGQ_HIP_TRY(hipMemcpyAsync(c->h_flags, c->d_flags, FL_WORDS * 4, hipMemcpyDeviceToHost, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  for (int k = 0; k < 2; ++k) {   // the older slot first (input order of the outputs is per slot anyway)
    hpgq_ctx::Slot &sl = c->slot[c->cur_slot ^ 1 ^ k];
    if (sl.busy) slot_deliver(sl);
  }
  return resolve(c);
}

int hpgq_sync(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  return sync_resolve(c);
}

int hpgq_reserve_length(hpgq_ctx_t *c, int64_t max_len) {
  if (!c || max_len < 0 || max_len > INT32_MAX) return HPGQ_E_INVALID;
  if (!c->p.stats_on || max_len <= (int64_t)c->p.lmax + c->tail_cap) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  return ensure_tail(c, max_len - c->p.lmax);
}

int hpgq_reset(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_state, 0, state_bytes(c), c->stream));
  if (c->tail_cap)
    HPGQ_HIP_TRY(hipMemsetAsync(c->d_tail, 0, (size_t)c->tail_cap * c->nm * 8 * sizeof(uint64_t), c->stream));
  // calls before the reset need no second pass any more (their flags are
  // cleared behind them on the stream)
  const size_t nc = c->calls.size();
  for (size_t k0 = 0; k0 < nc; k0 += kOvfChunk)
    HPGQ_HIP_TRY(hipMemsetAsync(c->ovf_chunks[k0 / kOvfChunk], 0, std::min(kOvfChunk, nc - k0) * 4, c->stream));
  c->calls.clear();
  c->reduced = false;
  return HPGQ_OK;
}

// the kernels add into the counters themselves: nothing to fold (kept for the ABI)
int hpgq_fold(hpgq_ctx_t *c) { return c ? HPGQ_OK : HPGQ_E_INVALID; }

size_t hpgq_counters_size(const hpgq_ctx_t *c) { return c ? c->clen * c->nm : 0; }

int hpgq_read_counters(hpgq_ctx_t *c, uint64_t *out, size_t n) {
  if (!c || !out || n < c->clen * c->nm) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemcpyAsync(out, c->reduced ? c->d_global : c->d_state, c->clen * c->nm * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, c->stream));
  // the stream has run every queued batch: their masks / trims reach the
  // caller's arrays here too, as in hpgq_sync; the dense set does
  // not depend on the tail's second pass, which runs here too
  return sync_resolve(c);
}

int hpgq_read_counters_ext(hpgq_ctx_t *c, uint64_t *out, size_t n, int32_t *lmax_ext) {
  if (!c || !lmax_ext) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  int rc = sync_resolve(c);
  if (rc) return rc;
  const int lmax = c->p.lmax, nm = c->nm;
  const uint32_t ml = c->h_flags[FL_MAXLEN];
  int64_t T = ml > (uint32_t)lmax ? (int64_t)ml - lmax : 0;
  const uint64_t *src_tail = c->d_tail;
  const bool global = c->reduced && c->comm;
  if (global) {   // the ranks agree on the tail length, then sum their tails (out of place)
    uint32_t t32 = (uint32_t)T;
    HPGQ_HIP_TRY(hipMemcpyAsync(c->d_scratch, &t32, 4, hipMemcpyHostToDevice, c->stream));
    if (ncclAllReduce(c->d_scratch, c->d_scratch + 1, 1, ncclUint32, ncclMax, c->comm, c->stream) != ncclSuccess)
      return HPGQ_E_RCCL;
    HPGQ_HIP_TRY(hipMemcpyAsync(&t32, c->d_scratch + 1, 4, hipMemcpyDeviceToHost, c->stream));
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    T = t32;
    if ((rc = ensure_tail(c, T))) return rc;
    const size_t words = (size_t)T * nm * 8;
    if (words > c->gtail_cap) {
      (void)hipFree(c->d_gtail);
      c->d_gtail = nullptr;
      c->gtail_cap = 0;
      if (hipMalloc(&c->d_gtail, words * 8) != hipSuccess) return HPGQ_E_NOMEM;
      c->gtail_cap = words;
    }
    if (words && ncclAllReduce(c->d_tail, c->d_gtail, words, ncclUint64, ncclSum, c->comm, c->stream) != ncclSuccess)
      return HPGQ_E_RCCL;
    src_tail = c->d_gtail;
  }
  const int64_t L = lmax + T;
  *lmax_ext = (int32_t)L;
  if (!out) {
    if (global) HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    return HPGQ_OK;
  }
  const size_t clen_x = hpgq_counters_len((int)L);
  if (n < clen_x * nm) return HPGQ_E_INVALID;
  std::vector<uint64_t> dense(c->clen * nm), tail((size_t)T * nm * 8);
  HPGQ_HIP_TRY(hipMemcpyAsync(dense.data(), c->reduced ? c->d_global : c->d_state, dense.size() * 8,
                              hipMemcpyDeviceToHost, c->stream));
  if (T) HPGQ_HIP_TRY(hipMemcpyAsync(tail.data(), src_tail, tail.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  // one set per mate in the layout of lmax_ext: the dense entries, then the
  // tail's lengths lmax + 1 .. L and positions lmax .. L - 1
  for (int m = 0; m < nm; ++m) {
    const uint64_t *d = dense.data() + (size_t)m * c->clen;
    uint64_t *o = out + (size_t)m * clen_x;
    std::memset(o, 0, clen_x * 8);
    std::memcpy(o, d, HPGQ_NUM_SCALARS * 8);
    o[HPGQ_S_LONG_READS] = 0;   // no merged read is longer than lmax_ext
    std::memcpy(o + hpgq_off_hist_len((int)L), d + hpgq_off_hist_len(lmax), (size_t)(lmax + 1) * 8);
    std::memcpy(o + hpgq_off_hist_meanq((int)L), d + hpgq_off_hist_meanq(lmax), HPGQ_MEANQ_BINS * 8);
    std::memcpy(o + hpgq_off_hist_gc((int)L), d + hpgq_off_hist_gc(lmax), HPGQ_GC_BINS * 8);
    std::memcpy(o + hpgq_off_pos_qsum((int)L), d + hpgq_off_pos_qsum(lmax), (size_t)lmax * 8);
    for (int b = 0; b < 5; ++b)
      std::memcpy(o + hpgq_off_pos_base((int)L, b), d + hpgq_off_pos_base(lmax, b), (size_t)lmax * 8);
    for (int64_t i = 0; i < T; ++i) {
      const uint64_t *t = tail.data() + ((size_t)i * nm + m) * 8;
      o[hpgq_off_hist_len((int)L) + lmax + 1 + i] = t[0];
      o[hpgq_off_pos_qsum((int)L) + lmax + i] = t[1];
      for (int b = 0; b < 5; ++b) o[hpgq_off_pos_base((int)L, b) + lmax + i] = t[2 + b];
    }
  }
  return HPGQ_OK;
}

uint64_t *hpgq_counters_device(hpgq_ctx_t *c) { return c ? c->d_state : nullptr; }
void *hpgq_stream(hpgq_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

// ---------------------------------------------------------------------------
// RCCL (one process per GPU): one sum of the packed counters
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

// out of place: the ctx's own counters keep accumulating, so repeated calls
// (or batches after one) never count another rank's reads twice
int hpgq_allreduce(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  if (!c->comm) return HPGQ_E_STATE;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  if (ncclAllReduce(c->d_state, c->d_global, c->clen * c->nm, ncclUint64, ncclSum, c->comm, c->stream) !=
      ncclSuccess)
    return HPGQ_E_RCCL;
  c->reduced = true;
  return HPGQ_OK;
}

uint64_t *hpgq_global_counters_device(hpgq_ctx_t *c) { return c ? c->d_global : nullptr; }

int hpgq_comm_count(hpgq_ctx_t *c, int *count) {
  if (!c || !count) return HPGQ_E_INVALID;
  *count = 0;
  if (!c->comm) return HPGQ_E_STATE;
  return ncclCommCount(c->comm, count) == ncclSuccess ? HPGQ_OK : HPGQ_E_RCCL;
}

// ---------------------------------------------------------------------------
// routing for tests and A/B runs (never read from the environment)
// ---------------------------------------------------------------------------

int hpgq_debug_set_route(hpgq_ctx_t *c, int route) {
  if (!c) return HPGQ_E_INVALID;
  const int r = route & 0xF;
  if (r > HPGQ_ROUTE_FIRST_WIDE || (route & ~(0xF | HPGQ_ROUTE_NO_ADAPTIVE))) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));   // no call of the old chain in flight
  // plan the new route beside the old state (chains are plain values; the
  // report word is the one resource) and swap it in only on success: a failed
  // plan leaves the ctx exactly as it was
  const Chain old0 = c->ch[0], old1 = c->ch[1];
  const bool old_adaptive = c->adaptive;
  uint32_t *const old_h = c->h_report, *const old_d = c->d_report;
  const int old_route = c->route;
  c->ch[0] = Chain{};
  c->ch[1] = Chain{};
  c->adaptive = false;
  c->h_report = c->d_report = nullptr;
  c->route = route;
  const int rc = plan(c, c->cus);
  if (rc) {
    if (c->h_report) (void)hipHostFree(c->h_report);   // (a plan that failed after its allocation)
    c->ch[0] = old0;
    c->ch[1] = old1;
    c->adaptive = old_adaptive;
    c->h_report = old_h;
    c->d_report = old_d;
    c->route = old_route;
    return rc;
  }
  if (old_h) (void)hipHostFree(old_h);
  c->mode = 0;
  c->wide_calls = 0;
  c->min_seq = c->seq + 1;
  return HPGQ_OK;
}

}  // extern "C"
