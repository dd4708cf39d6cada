// hpgq_engine.hip — libhpgq: engine context, launches and the C-ABI.
// The kernel itself lives in hpgq_engine_kernel.h (design notes there).

#include "hpgq_engine_kernel.h"
#include "hpgq_engine_tri.h"

// ===========================================================================
// C-ABI
// ===========================================================================

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rccl/rccl.h>

struct hpgq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hpgq_params_t p{};
  int nm = 1;
  size_t clen = 0;
  uint64_t *d_counters = nullptr;
  int32_t *d_err = nullptr;
  size_t lds_bytes = 0;
  char kname[64] = {0};   // the engine kernel instance hpgq_open chose
  const void *kfn = nullptr;
  int nch = 1;
  bool gen = false;               // generic (edit / N / OOR / left-right) kernel variant
  bool tri = false;               // segmented FAST kernel (lmax <= 160)
  bool hex = false;               // ... in its 16-byte-lane geometry (lmax <= 156)
  bool tri_edit = false;          // ... trimming in its block prologue (single-end edit)
  bool tri_x = false;             // ... with the N / out-of-range read filters
  int grid = 0;
  uint64_t *d_slab = nullptr;     // [grid][nm * clen] per-workgroup partials
  hpgq::ColdParams *d_cold = nullptr;
  bool dirty = false;             // slab holds partials not yet folded into d_counters
  // host-path device staging
  char *d_buf = nullptr;
  size_t d_buf_cap = 0;
  uint8_t *d_mask = nullptr;
  uint32_t *d_trim = nullptr;
  size_t d_out_cap = 0;
  ncclComm_t comm = nullptr;
};

// raw thresholds for "raw byte in [phred+lo, phred+hi]" with the clamps folded into flags
static void raw_range(int phred, int lo_q, int hi_q, uint32_t &lo4, uint32_t &hi4, int &lo_none,
                      int &hi_none, int &none_in) {
  const int64_t lo = (int64_t)phred + lo_q;
  const int64_t hi1 = (int64_t)phred + hi_q + 1;
  lo_none = lo <= 0;
  hi_none = hi1 > 255;
  none_in = lo > 255 || hi1 <= 0 || lo >= hi1;
  const uint32_t lob = (uint32_t)(lo < 0 ? 0 : lo > 255 ? 255 : lo);
  const uint32_t hib = (uint32_t)(hi1 < 0 ? 0 : hi1 > 255 ? 255 : hi1);
  lo4 = lob * 0x01010101u;
  hi4 = hib * 0x01010101u;
}

static int clamp_q(int q) { return q < -256 ? -256 : (q > 256 ? 256 : q); }

// engine flags from the parameters
static int engine_flags(const hpgq_params_t &p) {
  int f = 0;
  if (p.filter_on) f |= hpgq::F_FILTER;
  if (p.edit_on) f |= hpgq::F_EDIT;
  if (p.stats_on) f |= hpgq::F_STATS;
  // reads never exceed lmax (else the call fails), so a bound >= lmax cannot bite
  if (p.filter_on && p.max_N < p.lmax) f |= hpgq::F_NEED_N;
  if (p.filter_on && p.max_out_of_quality < p.lmax) f |= hpgq::F_NEED_OOR;
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
  A.phred = p.phred;
  A.cold = c->d_cold;
  A.flags = engine_flags(p);
  A.min_len = p.min_read_length;
  A.max_len = p.max_read_length;
  // mean Q = raw - phred lies in [-255, 255]: clamping keeps every product in int32
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
  int lo_none, hi_none, none_in;
  raw_range(p.phred, p.min_read_quality, p.max_read_quality, C.oor_lo4, C.oor_hi4, lo_none,
            hi_none, none_in);
  C.max_n = p.max_N;
  C.max_oor = p.max_out_of_quality;
}

template <int NM, bool GEN>
static const void *kernel_nch(int nch) {
  switch (nch) {
    case 1: return (const void *)hpgq::engine_kernel<NM, 1, GEN>;
    case 2: return (const void *)hpgq::engine_kernel<NM, 2, GEN>;
    default: return (const void *)hpgq::engine_kernel<NM, 5, GEN>;
  }
}

template <int NW>
static const void *tri_for(int mw, bool un, int nm, bool edit) {
  using hpgq::engine_tri_kernel;
  if (edit) return mw <= 4 ? (const void *)engine_tri_kernel<4, false, 1, true, NW>
                           : (const void *)engine_tri_kernel<5, false, 1, true, NW>;
  if constexpr (NW == 4) {
    if (un && !edit) return (const void *)engine_tri_kernel<4, true, 1, false, 4>;
    if (nm == 2) return (const void *)engine_tri_kernel<3, false, 2, false, 4>;   // 3 waves/SIMD: two mates' accumulators
  }
  if constexpr (NW == 2) {
    if (nm == 2) {   // paired-end (tri geometry: two mates' accumulators do not fit hex's registers)
      if (mw <= 4) return (const void *)engine_tri_kernel<4, false, 2, false, 2>;
      if (mw == 5) return (const void *)engine_tri_kernel<5, false, 2, false, 2>;
      return (const void *)engine_tri_kernel<6, false, 2, false, 2>;
    }
    if (un) {
      if (mw <= 4) return (const void *)engine_tri_kernel<4, true, 1, false, 2>;
      if (mw == 5) return (const void *)engine_tri_kernel<5, true, 1, false, 2>;
      return (const void *)engine_tri_kernel<6, true, 1, false, 2>;
    }
  }
  if (mw <= 4) return (const void *)engine_tri_kernel<4, false, 1, false, NW>;
  if (mw == 5) return (const void *)engine_tri_kernel<5, false, 1, false, NW>;
  return (const void *)engine_tri_kernel<6, false, 1, false, NW>;
}

// tri: the segmented kernel (hpgq_engine_tri.h), hex selects its 16-byte-lane geometry
static const void *kernel_for(int nm, int nch, bool gen, bool tri, bool hex, bool edit, bool tx, char *name,
                              size_t cap) {
  if (tri && tx) {   // spill-free occupancy per variant, as below
    using hpgq::engine_tri_x_kernel;
    const int mw = hex ? (nm == 2 ? 3 : 4) : (nm == 2 ? 3 : 5);
    std::snprintf(name, cap, "hpgq::engine_tri_x_kernel<%d, %d, %d>", mw, nm, hex ? 4 : 2);
    if (hex) return nm == 2 ? (const void *)engine_tri_x_kernel<3, 2, 4> : (const void *)engine_tri_x_kernel<4, 1, 4>;
    return nm == 2 ? (const void *)engine_tri_x_kernel<3, 2, 2> : (const void *)engine_tri_x_kernel<5, 1, 2>;
  }
  if (tri) {
    const char *w = std::getenv("HPGQ_TRI_WAVES");      // occupancy experiment knob
    const char *u = std::getenv("HPGQ_TRI_UNALIGNED");  // load-scheme experiment knob (tri only)
    const int nw = hex ? 4 : 2;
    int mw = w ? std::atoi(w) : (hex ? 4 : (nm == 2 ? 4 : 5));   // spill-free occupancy per variant
    mw = mw <= 4 ? 4 : (mw == 5 ? 5 : 6);
    if (hex) mw = nm == 2 ? 3 : 4;   // 116-123 VGPRs (SE)
    if (edit && mw > 5) mw = 5;
    const bool un = !edit && nm == 1 && u && std::atoi(u) != 0;
    std::snprintf(name, cap, "hpgq::engine_tri_kernel<%d, %s, %d, %s, %d>", mw, un ? "true" : "false", edit ? 1 : nm,
                  edit ? "true" : "false", nw);
    return hex ? tri_for<4>(mw, un, nm, edit) : tri_for<2>(mw, un, nm, edit);
  }
  std::snprintf(name, cap, "hpgq::engine_kernel<%d, %d, %s>", nm, nch == 1 ? 1 : (nch == 2 ? 2 : 5),
                gen ? "true" : "false");
  if (nm == 2) return gen ? kernel_nch<2, true>(nch) : kernel_nch<2, false>(nch);
  return gen ? kernel_nch<1, true>(nch) : kernel_nch<1, false>(nch);
}

extern "C" {

void hpgq_params_init(hpgq_params_t *p) {
  std::memset(p, 0, sizeof(*p));
  p->phred = HPGQ_PHRED33;
  p->lmax = 256;
  p->stats_on = 1;
  p->min_read_length = HPGQ_MIN_VALUE;
  p->max_read_length = HPGQ_MAX_VALUE;
  p->min_read_quality = HPGQ_MIN_VALUE;
  p->max_read_quality = HPGQ_MAX_VALUE;
  p->max_out_of_quality = HPGQ_MAX_VALUE;
  p->left_length = HPGQ_MIN_VALUE;
  p->min_left_quality = HPGQ_MIN_VALUE;
  p->max_left_quality = HPGQ_MAX_VALUE;
  p->right_length = HPGQ_MIN_VALUE;
  p->min_right_quality = HPGQ_MIN_VALUE;
  p->max_right_quality = HPGQ_MAX_VALUE;
  p->max_N = HPGQ_MAX_VALUE;
  p->edit_left_length = HPGQ_MIN_VALUE;
  p->edit_min_left_quality = HPGQ_MIN_VALUE;
  p->edit_max_left_quality = HPGQ_MAX_VALUE;
  p->edit_right_length = HPGQ_MIN_VALUE;
  p->edit_min_right_quality = HPGQ_MIN_VALUE;
  p->edit_max_right_quality = HPGQ_MAX_VALUE;
}

const char *hpgq_strerror(int code) {
  switch (code) {
    case HPGQ_OK: return "ok";
    case HPGQ_E_INVALID: return "invalid argument";
    case HPGQ_E_HIP: return "HIP runtime error";
    case HPGQ_E_NOMEM: return "out of memory";
    case HPGQ_E_READ_TOO_LONG: return "read longer than lmax";
    case HPGQ_E_NO_DEVICE: return "no HIP device";
    case HPGQ_E_RCCL: return "RCCL error";
    case HPGQ_E_STATE: return "invalid ctx state";
    case HPGQ_E_FORMAT: return "malformed FASTQ text";
    case HPGQ_E_IO: return "file i/o error";
    default: return "unknown error";
  }
}

const char *hpgq_version(void) { return "hpgq 0.1 (gfx950)"; }

const char *hpgq_kernel_name(const hpgq_ctx_t *ctx) { return ctx ? ctx->kname : ""; }

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

static int validate_params(const hpgq_params_t *p) {
  if (!p) return HPGQ_E_INVALID;
  if (p->lmax < 1 || p->lmax > HPGQ_LMAX_LIMIT) return HPGQ_E_INVALID;
  if (p->phred < 0 || p->phred > 255) return HPGQ_E_INVALID;
  return HPGQ_OK;
}

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
  c->nch = (p->lmax + hpgq::kChunk - 1) / hpgq::kChunk;
  if (c->nch > 2) c->nch = 5;   // instantiated chunk counts: 1, 2, 5
  c->gen = needs_generic(engine_flags(*p));
  {
    const char *force = std::getenv("HPGQ_KERNEL");   // "single" forces the one-read kernel
    const int fl = engine_flags(*p);
    const bool lr = fl & hpgq::F_NEED_LR;                          // window filters: engine_kernel
    const bool nx = fl & (hpgq::F_NEED_N | hpgq::F_NEED_OOR);     // N / out-of-range: engine_tri_x_kernel
    const bool edit = fl & hpgq::F_EDIT;
    c->tri = !lr && !(nx && edit) && (!edit || c->nm == 1) && p->lmax <= hpgq::kTriPos &&
             !(force && std::strcmp(force, "single") == 0);
    c->tri_edit = c->tri && edit;
    c->tri_x = c->tri && nx;
    const char *geo = std::getenv("HPGQ_TRI_GEO");   // "tri" forces the 8-byte-lane geometry
    c->hex = c->tri && p->lmax <= hpgq::kHexPos &&
             !(geo && std::strcmp(geo, "tri") == 0);
  }
  {
    const int hlen = p->lmax + 1 + HPGQ_MEANQ_BINS + HPGQ_GC_BINS;
    const size_t hist_words = ((size_t)c->nm * hlen + 1) & ~(size_t)1;
    c->lds_bytes = ((size_t)c->nm * 6 * p->lmax + hist_words) * 4 +
                   (size_t)c->nm * HPGQ_NUM_SCALARS * 8 + sizeof(hpgq::ColdParams);
    // the three-read kernel: per mate [6][lmax] + hist + scalars, and per wave
    // and mate two read tables (2 x 1 KB) + segment ends (256 B)
    const size_t mate_words = (size_t)6 * p->lmax + (((size_t)hlen + 1) & ~(size_t)1) + 2 * HPGQ_NUM_SCALARS;
    const size_t tri_lds = (size_t)c->nm * mate_words * 4 + 16 + 17 * 16 +   // + the byte-mask table
                           (size_t)hpgq::kWaves * c->nm * (2 * 256 + (c->tri_x ? 128 : 64)) * 4;
    if (tri_lds > c->lds_bytes) c->lds_bytes = tri_lds;
  }
  HPGQ_HIP_TRY(hipSetDevice(device));
  HPGQ_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HPGQ_HIP_TRY(hipMalloc(&c->d_counters, c->clen * c->nm * sizeof(uint64_t)));
  HPGQ_HIP_TRY(hipMalloc(&c->d_err, sizeof(int32_t)));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_counters, 0, c->clen * c->nm * sizeof(uint64_t), c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
  int cus = 0;
  HPGQ_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const void *kfn = kernel_for(c->nm, c->nch, c->gen, c->tri, c->hex, c->tri_edit, c->tri_x, c->kname,
                               sizeof(c->kname));
  c->kfn = kfn;
  if (c->lds_bytes > 64 * 1024)
    HPGQ_HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)c->lds_bytes));
  int per_cu = 0;
  HPGQ_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, hpgq::kWG, c->lds_bytes));
  if (per_cu < 1) per_cu = 1;
  c->grid = cus * per_cu;   // persistent: every workgroup resident, grid-stride over reads
  HPGQ_HIP_TRY(hipMalloc(&c->d_slab, (size_t)c->grid * c->nm * c->clen * sizeof(uint64_t)));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_slab, 0, (size_t)c->grid * c->nm * c->clen * sizeof(uint64_t),
                              c->stream));
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
  if (c->comm) ncclCommDestroy(c->comm);
  (void)hipFree(c->d_counters);
  (void)hipFree(c->d_err);
  (void)hipFree(c->d_slab);
  (void)hipFree(c->d_cold);
  (void)hipFree(c->d_buf);
  (void)hipFree(c->d_mask);
  (void)hipFree(c->d_trim);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int launch(hpgq_ctx *c, hpgq::EngineArgs &A) {
  if (A.num_reads <= 0) return HPGQ_OK;
  A.slab = c->d_slab;
  A.err = c->d_err;
  const int64_t per_block = c->tri ? (c->hex ? hpgq::kHexBlock : hpgq::kTriBlock) : 64;
  const int64_t nblocks = (A.num_reads + per_block - 1) / per_block;
  const int64_t need = (nblocks + hpgq::kWaves - 1) / hpgq::kWaves;
  const int grid = (int)std::min<int64_t>(need, c->grid);
  void *args[] = {&A};
  HPGQ_HIP_TRY(hipLaunchKernel(c->kfn, dim3(grid), dim3(hpgq::kWG), args,
                               c->lds_bytes, c->stream));
  c->dirty = true;
  return HPGQ_OK;
}

// fold the per-workgroup slab rows into d_counters (async on the ctx stream)
static int fold(hpgq_ctx *c) {
  if (!c->dirty) return HPGQ_OK;
  const int len = (int)(c->clen * c->nm);
  hipLaunchKernelGGL(hpgq::slab_reduce_kernel, dim3((len + 255) / 256), dim3(256), 0, c->stream,
                     c->d_slab, c->grid, len, c->d_counters);
  HPGQ_HIP_TRY(hipGetLastError());
  c->dirty = false;
  return HPGQ_OK;
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
  return launch(c, A);
}

static int ensure_dev(hpgq_ctx *c, size_t bytes, size_t nreads) {
  if (bytes > c->d_buf_cap) {
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_buf);
    c->d_buf = nullptr;
    size_t cap = bytes + bytes / 4 + 4096;
    if (hipMalloc(&c->d_buf, cap) != hipSuccess) { c->d_buf_cap = 0; return HPGQ_E_NOMEM; }
    c->d_buf_cap = cap;
  }
  if (nreads > c->d_out_cap) {
    HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_mask);
    (void)hipFree(c->d_trim);
    size_t cap = nreads + nreads / 4 + 64;
    if (hipMalloc(&c->d_mask, cap) != hipSuccess) return HPGQ_E_NOMEM;
    if (hipMalloc(&c->d_trim, cap * 2 * sizeof(uint32_t)) != hipSuccess) return HPGQ_E_NOMEM;
    c->d_out_cap = cap;
  }
  return HPGQ_OK;
}

int hpgq_run_host(hpgq_ctx_t *c, const hpgq_batch_t *b, const hpgq_batch_t *b2,
                  uint8_t *mask_out, uint32_t *trim_out) {
  if (!c || !b) return HPGQ_E_INVALID;
  if (c->nm == 2 && (!b2 || b2->num_reads != b->num_reads)) return HPGQ_E_INVALID;
  if (c->nm == 1 && b2) return HPGQ_E_INVALID;
  const int64_t n = b->num_reads;
  if (n < 0) return HPGQ_E_INVALID;
  if (n == 0) return HPGQ_OK;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  const hpgq_batch_t *bs[2] = {b, b2};
  size_t bytes[2] = {0, 0}, off[2][4];
  size_t total = 0;
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    bytes[m] = (size_t)(ix[n] - ix[0]);
    off[m][0] = total; total += (bytes[m] + 255) & ~(size_t)255;   // seq
    off[m][1] = total; total += (bytes[m] + 255) & ~(size_t)255;   // quality
    off[m][2] = total; total += ((size_t)(n + 1) * 4 + 255) & ~(size_t)255;
  }
  int rc = ensure_dev(c, total, (size_t)n);
  if (rc) return rc;
  hpgq::EngineArgs A{};
  fill_args(c, A);
  A.num_reads = n;
  for (int m = 0; m < c->nm; ++m) {
    const int32_t *ix = bs[m]->data_indices;
    char *ds = c->d_buf + off[m][0], *dq = c->d_buf + off[m][1];
    int32_t *di = reinterpret_cast<int32_t *>(c->d_buf + off[m][2]);
    HPGQ_HIP_TRY(hipMemcpyAsync(ds, bs[m]->seq + ix[0], bytes[m], hipMemcpyHostToDevice, c->stream));
    HPGQ_HIP_TRY(hipMemcpyAsync(dq, bs[m]->quality + ix[0], bytes[m], hipMemcpyHostToDevice, c->stream));
    HPGQ_HIP_TRY(hipMemcpyAsync(di, ix, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    // absolute indices: shift the base pointers so data_indices need no rewrite
    A.seq[m] = ds - ix[0];
    A.qual[m] = dq - ix[0];
    A.idx[m] = di;
  }
  A.mask = mask_out ? c->d_mask : nullptr;
  A.trim = trim_out ? c->d_trim : nullptr;
  rc = launch(c, A);
  if (rc) return rc;
  if (mask_out) HPGQ_HIP_TRY(hipMemcpyAsync(mask_out, c->d_mask, (size_t)n, hipMemcpyDeviceToHost, c->stream));
  if (trim_out)
    HPGQ_HIP_TRY(hipMemcpyAsync(trim_out, c->d_trim, (size_t)n * c->nm * 4, hipMemcpyDeviceToHost,
                                c->stream));
  return HPGQ_OK;
}

int hpgq_sync(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  int32_t err = 0;
  HPGQ_HIP_TRY(hipMemcpy(&err, c->d_err, sizeof(err), hipMemcpyDeviceToHost));
  return err ? HPGQ_E_READ_TOO_LONG : HPGQ_OK;
}

int hpgq_reset(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_counters, 0, c->clen * c->nm * sizeof(uint64_t), c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_slab, 0, (size_t)c->grid * c->nm * c->clen * sizeof(uint64_t),
                              c->stream));
  HPGQ_HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));
  c->dirty = false;
  return HPGQ_OK;
}

int hpgq_fold(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  return fold(c);
}

size_t hpgq_counters_size(const hpgq_ctx_t *c) { return c ? c->clen * c->nm : 0; }

int hpgq_read_counters(hpgq_ctx_t *c, uint64_t *out, size_t n) {
  if (!c || !out || n < c->clen * c->nm) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  int rc = fold(c);
  if (rc) return rc;
  HPGQ_HIP_TRY(hipMemcpyAsync(out, c->d_counters, c->clen * c->nm * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, c->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(c->stream));
  return HPGQ_OK;
}

uint64_t *hpgq_counters_device(hpgq_ctx_t *c) { return c ? c->d_counters : nullptr; }
void *hpgq_stream(hpgq_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

// ---------------------------------------------------------------------------
// RCCL (one process per GPU): one in-place sum of the packed counters
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

int hpgq_allreduce(hpgq_ctx_t *c) {
  if (!c) return HPGQ_E_INVALID;
  if (!c->comm) return HPGQ_E_STATE;
  HPGQ_HIP_TRY(hipSetDevice(c->device));
  int rc = fold(c);
  if (rc) return rc;
  if (ncclAllReduce(c->d_counters, c->d_counters, c->clen * c->nm, ncclUint64, ncclSum, c->comm,
                    c->stream) != ncclSuccess)
    return HPGQ_E_RCCL;
  return HPGQ_OK;
}

// ---------------------------------------------------------------------------
// derived summary (stats_counters_t view)
// ---------------------------------------------------------------------------

int hpgq_counters_summary(const uint64_t *set, int lmax, hpgq_summary_t *o) {
  if (!set || !o || lmax < 1) return HPGQ_E_INVALID;
  std::memset(o, 0, sizeof(*o));
  o->num_input = set[HPGQ_S_NUM_INPUT];
  o->num_passed = set[HPGQ_S_NUM_PASSED];
  o->num_failed = set[HPGQ_S_NUM_FAILED];
  o->num_edited = set[HPGQ_S_NUM_EDITED];
  o->num_reads = set[HPGQ_S_NUM_STATS];
  o->min_length = 100000;   // stats_counters_new, src/stats_fastq.c:108-109
  o->max_length = 0;
  const uint64_t *hl = set + hpgq_off_hist_len(lmax);
  for (int L = 0; L <= lmax; ++L) {
    if (!hl[L]) continue;
    if (L < o->min_length) o->min_length = L;
    if (L > o->max_length) o->max_length = L;
    o->acc_length += (uint64_t)L * hl[L];
  }
  uint64_t *tot[5] = {&o->num_A, &o->num_C, &o->num_G, &o->num_T, &o->num_N};
  for (int b = 0; b < 5; ++b) {
    const uint64_t *pb = set + hpgq_off_pos_base(lmax, b);
    for (int j = 0; j < lmax; ++j) *tot[b] += pb[j];
  }
  if (o->num_reads) {
    o->mean_length = (double)o->acc_length / (double)o->num_reads;
    o->mean_quality_raw = (double)set[HPGQ_S_ACC_MEANQ_FX16] / 65536.0 / (double)o->num_reads;
  }
  return HPGQ_OK;
}

}  // extern "C"
