// hpgq_parse.hip — FASTQ text -> SoA batch on the device.
//
// Replaces the parsing half of the reference's producer (fastq_fread_se,
// src/stats_fastq.c:183; the reader lives in the absent bioinfo-libs) for the
// GPU path: the host streams raw file bytes to HBM and the batch the engine
// reads (hpgq_batch_t: concatenated seq / quality + data_indices) is built on
// the device.  Records are 4 lines — "@header", sequence, "+[header]",
// quality of the sequence's length — with "\n" or "\r\n" line ends.
//
//   nl_count_kernel    newlines per 16 KB tile (SWAR byte compare)
//   (hipCUB scan)      tile offsets
//   nl_write_kernel    newline positions, in order (block scan per tile)
//   record_kernel      one thread per record: line bounds, validation, length
//   (hipCUB scan)      lengths -> data_indices
//   copy_kernel        one wave per record: seq / quality bytes into the batch
// Per-record offsets (record start, sequence, '+' line, quality) stay on the
// device for writers (hpgq_parse_records).
#include "hpgq_common.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

namespace hpgq {
namespace parse {

constexpr int kTB = 256;               // threads per tile block
constexpr int kPerThread = 64;         // bytes per thread
constexpr int kTile = kTB * kPerThread;

__device__ __forceinline__ uint32_t nl_bytes(uint32_t w) {   // 0x80 per '\n' byte
  const uint32_t v = w ^ 0x0A0A0A0Au;
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

// newlines in this thread's 64 bytes; optionally their positions
__device__ __forceinline__ uint32_t thread_count(const uint8_t *t, int64_t n, int64_t base) {
  if (base + kPerThread <= n) {
    const uint4 *p = reinterpret_cast<const uint4 *>(t + base);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < kPerThread / 16; ++i) {
      const uint4 v = p[i];
      c += __builtin_popcount(nl_bytes(v.x)) + __builtin_popcount(nl_bytes(v.y)) +
           __builtin_popcount(nl_bytes(v.z)) + __builtin_popcount(nl_bytes(v.w));
    }
    return c;
  }
  uint32_t c = 0;
  for (int64_t i = base; i < n && i < base + kPerThread; ++i) c += t[i] == '\n';
  return c;
}

__global__ void __launch_bounds__(kTB) nl_count_kernel(const uint8_t *t, int64_t n, uint32_t *tiles) {
  typedef hipcub::BlockReduce<uint32_t, kTB> R;
  __shared__ typename R::TempStorage tmp;
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kPerThread;
  const uint32_t c = base < n ? thread_count(t, n, base) : 0u;
  const uint32_t s = R(tmp).Sum(c);
  if (threadIdx.x == 0) tiles[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kTB) nl_write_kernel(const uint8_t *t, int64_t n,
                                                       const uint32_t *tile_off, uint32_t *nl) {
  typedef hipcub::BlockScan<uint32_t, kTB> S;
  __shared__ typename S::TempStorage tmp;
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kPerThread;
  const uint32_t c = base < n ? thread_count(t, n, base) : 0u;
  uint32_t off;
  S(tmp).ExclusiveSum(c, off);
  off += tile_off[blockIdx.x];
  if (!c) return;
  const int64_t end = std::min<int64_t>(base + kPerThread, n);
  for (int64_t i = base; i < end; ++i)
    if (t[i] == '\n') nl[off++] = (uint32_t)i;
}

struct Rec {
  uint32_t *start, *seq, *plus, *qual;   // per-record offsets into the text
  int32_t *len;
};

// line [b, e) without a trailing '\r'
__device__ __forceinline__ uint32_t line_end(const uint8_t *t, uint32_t b, uint32_t e) {
  return (e > b && t[e - 1] == '\r') ? e - 1 : e;
}

// record i: its line bounds, the checks, its length (0 when malformed)
__device__ __forceinline__ int32_t record_one(const uint8_t *t, const uint32_t *nl, int64_t i, Rec R, int32_t *bad) {
  const uint32_t start = i ? nl[4 * i - 1] + 1 : 0u;
  const uint32_t n0 = nl[4 * i], n1 = nl[4 * i + 1], n2 = nl[4 * i + 2], n3 = nl[4 * i + 3];
  const uint32_t sb = n0 + 1, se = line_end(t, sb, n1);
  const uint32_t pb = n1 + 1, qb = n2 + 1, qe = line_end(t, qb, n3);
  const bool ok = n0 > start && t[start] == '@' && pb < n2 && t[pb] == '+' && (se - sb) == (qe - qb);
  R.start[i] = start;
  R.seq[i] = sb;
  R.plus[i] = pb;
  R.qual[i] = qb;
  R.len[i] = ok ? (int32_t)(se - sb) : 0;
  if (!ok) atomicMin(bad, (int32_t)min<int64_t>(i, 0x7FFFFFFF));
  return ok ? (int32_t)(se - sb) : 0;
}

// bad[0]: the first malformed record (atomicMin); bad[1]: the longest record
// (the long-read tail's reservation, hpgq_parser_max_length)
__global__ void __launch_bounds__(256) record_kernel(const uint8_t *t, const uint32_t *nl, int64_t nrec,
                                                     Rec R, int32_t *bad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int32_t len = 0;
  if (i < nrec) len = record_one(t, nl, i, R, bad);
  for (int o = 32; o > 0; o >>= 1) len = max(len, __shfl_xor(len, o));
  if ((threadIdx.x & 63) == 0 && len > 0) atomicMax(bad + 1, len);
}

// one wave per record
__global__ void __launch_bounds__(256) copy_kernel(const uint8_t *t, Rec R, const int32_t *idx,
                                                   int64_t nrec, uint8_t *seq, uint8_t *qual) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nrec) return;
  const int lane = threadIdx.x & 63;
  const int32_t o = idx[i], L = idx[i + 1] - o;
  const uint8_t *s = t + R.seq[i], *q = t + R.qual[i];
  for (int j = lane; j < L; j += 64) {
    seq[o + j] = s[j];
    qual[o + j] = q[j];
  }
}

}  // namespace parse
}  // namespace hpgq

struct hpgq_parser {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint8_t *d_text = nullptr;
  size_t text_cap = 0;
  uint32_t *d_tiles = nullptr;   // counts, then offsets (+ total)
  size_t tiles_cap = 0;
  uint32_t *d_nl = nullptr;
  size_t nl_cap = 0;
  uint32_t *d_rec = nullptr;     // 4 arrays of rec_cap
  int32_t *d_len = nullptr;      // rec_cap + 1 (data_indices)
  int32_t *d_idx = nullptr;
  size_t rec_cap = 0;
  uint8_t *d_seq = nullptr, *d_qual = nullptr;
  size_t data_cap = 0;
  int32_t *d_bad = nullptr;
  void *d_tmp = nullptr;
  size_t tmp_cap = 0;
  int64_t last_n = 0;            // records of the last parse
  int64_t max_len = 0;           // its longest record
};

static int grow(void **p, size_t *cap, size_t need) {
  if (need <= *cap) return HPGQ_OK;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t c = need + need / 4 + 4096;
  if (hipMalloc(p, c) != hipSuccess) return HPGQ_E_NOMEM;
  *cap = c;
  return HPGQ_OK;
}

static int scan_tmp(hpgq_parser *p, size_t need) {
  return grow(&p->d_tmp, &p->tmp_cap, need);
}

extern "C" {

int64_t hpgq_fastq_complete_prefix(const char *buf, int64_t n, int at_eof) {
  if (!buf || n <= 0) return 0;
  if (at_eof) return n;
  // from the end: the last line start '@' whose 4 lines are complete and
  // well formed ('+' third line, quality as long as the sequence)
  for (int64_t p = n - 1; p >= 0; --p) {
    if (buf[p] != '@' || (p > 0 && buf[p - 1] != '\n')) continue;
    int64_t b[4], e[4], q = p;
    int k = 0;
    for (; k < 4; ++k) {
      const void *nl = std::memchr(buf + q, '\n', (size_t)(n - q));
      if (!nl) break;
      b[k] = q;
      e[k] = (const char *)nl - buf;
      q = e[k] + 1;
    }
    if (k < 4) continue;   // a partial record: look further back
    auto len = [&](int j) { return (e[j] > b[j] && buf[e[j] - 1] == '\r') ? e[j] - 1 - b[j] : e[j] - b[j]; };
    if (buf[b[2]] == '+' && len(1) == len(3)) return e[3] + 1;
  }
  return 0;
}

int hpgq_parser_open(hpgq_parser_t **ps, int device, void *stream) {
  if (!ps) return HPGQ_E_INVALID;
  *ps = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return HPGQ_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return HPGQ_E_INVALID;
  hpgq_parser *p = new hpgq_parser();
  p->device = device;
  HPGQ_HIP_TRY(hipSetDevice(device));
  if (stream) {
    p->stream = (hipStream_t)stream;
  } else {
    HPGQ_HIP_TRY(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    p->own_stream = true;
  }
  HPGQ_HIP_TRY(hipMalloc(&p->d_bad, 8));
  *ps = p;
  return HPGQ_OK;
}

void hpgq_parser_close(hpgq_parser_t *p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  (void)hipStreamSynchronize(p->stream);
  (void)hipFree(p->d_text);
  (void)hipFree(p->d_tiles);
  (void)hipFree(p->d_nl);
  (void)hipFree(p->d_rec);
  (void)hipFree(p->d_len);
  (void)hipFree(p->d_idx);
  (void)hipFree(p->d_seq);
  (void)hipFree(p->d_qual);
  (void)hipFree(p->d_bad);
  (void)hipFree(p->d_tmp);
  if (p->own_stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

// length of the text without trailing blank lines ("...\n\n", "\r\n\r\n" at the
// end of a file hold no record); tail: its last `nt` bytes
static int64_t trim_blank_tail(const char *tail, int64_t nt, int64_t n, bool &more) {
  more = false;
  const int64_t base = n - nt;   // text offset of tail[0]
  for (;;) {
    if (n < 1 || tail[n - 1 - base] != '\n') break;
    int64_t b = n - 1;   // content end of the last line
    if (b > base && tail[b - 1 - base] == '\r') --b;
    if (b == 0) {   // the text is blank lines only
      n = 0;
      break;
    }
    if (b - 1 < base) {   // the byte before lies past the fetched tail: fetch again, ending at n
      more = true;
      break;
    }
    if (tail[b - 1 - base] != '\n') break;   // the last line is not blank
    n = b;
  }
  return n;
}

int hpgq_parse_device(hpgq_parser_t *p, const char *text, int64_t n, hpgq_batch_t *out) {
  using namespace hpgq::parse;
  if (!p || !out || n < 0 || n >= ((int64_t)1 << 31)) return HPGQ_E_INVALID;
  *out = hpgq_batch_t{0, nullptr, nullptr, nullptr};
  p->last_n = 0;
  p->max_len = 0;
  HPGQ_HIP_TRY(hipSetDevice(p->device));
  for (bool more = n > 0; more;) {   // drop trailing blank lines
    char tail[64];
    const int64_t nt = n < 64 ? n : 64;
    HPGQ_HIP_TRY(hipMemcpyAsync(tail, text + n - nt, (size_t)nt, hipMemcpyDeviceToHost, p->stream));
    HPGQ_HIP_TRY(hipStreamSynchronize(p->stream));
    n = trim_blank_tail(tail, nt, n, more);
  }
  const uint8_t *t = reinterpret_cast<const uint8_t *>(text);
  // 1. newline count per tile, tile offsets, total
  const int64_t ntiles = (n + kTile - 1) / kTile;
  // counts [0, ntiles + 1) then offsets [ntiles + 1, 2 (ntiles + 1))
  if (grow((void **)&p->d_tiles, &p->tiles_cap, (size_t)(ntiles + 1) * 8)) return HPGQ_E_NOMEM;
  uint32_t *d_off = p->d_tiles + ntiles + 1;
  HPGQ_HIP_TRY(hipMemsetAsync(p->d_tiles, 0, (size_t)(ntiles + 1) * 4, p->stream));
  if (ntiles) {
    nl_count_kernel<<<(unsigned)ntiles, kTB, 0, p->stream>>>(t, n, p->d_tiles);
    HPGQ_HIP_TRY(hipGetLastError());
  }
  size_t tb = 0;
  HPGQ_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, p->d_tiles, d_off, (int)ntiles + 1, p->stream));
  if (scan_tmp(p, tb)) return HPGQ_E_NOMEM;
  HPGQ_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(p->d_tmp, tb, p->d_tiles, d_off, (int)ntiles + 1, p->stream));
  uint32_t total = 0;
  HPGQ_HIP_TRY(hipMemcpyAsync(&total, d_off + ntiles, 4, hipMemcpyDeviceToHost, p->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(p->stream));
  if (total % 4 != 0) return HPGQ_E_FORMAT;   // not whole 4-line records
  const int64_t nrec = total / 4;
  if (nrec == 0) return HPGQ_OK;
  // 2. newline positions
  if (grow((void **)&p->d_nl, &p->nl_cap, (size_t)total * 4)) return HPGQ_E_NOMEM;
  nl_write_kernel<<<(unsigned)ntiles, kTB, 0, p->stream>>>(t, n, d_off, p->d_nl);
  HPGQ_HIP_TRY(hipGetLastError());
  // 3. records
  if ((size_t)nrec + 1 > p->rec_cap) {
    (void)hipFree(p->d_rec);
    (void)hipFree(p->d_len);
    (void)hipFree(p->d_idx);
    p->d_rec = nullptr;
    p->d_len = p->d_idx = nullptr;
    p->rec_cap = 0;
    const size_t c = (size_t)nrec + nrec / 4 + 1024;
    if (hipMalloc(&p->d_rec, c * 16) != hipSuccess || hipMalloc(&p->d_len, c * 4) != hipSuccess ||
        hipMalloc(&p->d_idx, (c + 1) * 4) != hipSuccess)
      return HPGQ_E_NOMEM;
    p->rec_cap = c;
  }
  Rec R{p->d_rec, p->d_rec + p->rec_cap, p->d_rec + 2 * p->rec_cap, p->d_rec + 3 * p->rec_cap, p->d_len};
  const int32_t init[2] = {0x7FFFFFFF, 0};   // first malformed record, longest record
  const int32_t big = init[0];
  HPGQ_HIP_TRY(hipMemcpyAsync(p->d_bad, init, 8, hipMemcpyHostToDevice, p->stream));
  record_kernel<<<(unsigned)((nrec + 255) / 256), 256, 0, p->stream>>>(t, p->d_nl, nrec, R, p->d_bad);
  HPGQ_HIP_TRY(hipGetLastError());
  // 4. data_indices = [0, inclusive scan of the lengths]
  HPGQ_HIP_TRY(hipMemsetAsync(p->d_idx, 0, 4, p->stream));
  tb = 0;
  HPGQ_HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, p->d_len, p->d_idx + 1, (int)nrec, p->stream));
  if (scan_tmp(p, tb)) return HPGQ_E_NOMEM;
  HPGQ_HIP_TRY(hipcub::DeviceScan::InclusiveSum(p->d_tmp, tb, p->d_len, p->d_idx + 1, (int)nrec, p->stream));
  int32_t bad[2] = {0, 0}, data_end = 0;
  HPGQ_HIP_TRY(hipMemcpyAsync(bad, p->d_bad, 8, hipMemcpyDeviceToHost, p->stream));
  HPGQ_HIP_TRY(hipMemcpyAsync(&data_end, p->d_idx + nrec, 4, hipMemcpyDeviceToHost, p->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(p->stream));
  if (bad[0] != big) return HPGQ_E_FORMAT;
  // 5. the batch bytes (+ the engine's readable slack)
  const size_t need = (size_t)data_end + HPGQ_DEVICE_SLACK + 64;
  if (need > p->data_cap) {
    (void)hipFree(p->d_seq);
    (void)hipFree(p->d_qual);
    p->d_seq = p->d_qual = nullptr;
    p->data_cap = 0;
    const size_t c = need + need / 4 + 4096;
    if (hipMalloc(&p->d_seq, c) != hipSuccess || hipMalloc(&p->d_qual, c) != hipSuccess)
      return HPGQ_E_NOMEM;
    p->data_cap = c;
  }
  copy_kernel<<<(unsigned)((nrec + 3) / 4), 256, 0, p->stream>>>(t, R, p->d_idx, nrec, p->d_seq, p->d_qual);
  HPGQ_HIP_TRY(hipGetLastError());
  out->num_reads = nrec;
  out->seq = reinterpret_cast<const char *>(p->d_seq);
  out->quality = reinterpret_cast<const char *>(p->d_qual);
  out->data_indices = p->d_idx;
  p->last_n = nrec;
  p->max_len = bad[1];
  return HPGQ_OK;
}

int hpgq_parse_host(hpgq_parser_t *p, const char *text, int64_t n, hpgq_batch_t *out) {
  if (!p || (!text && n > 0) || n < 0 || n >= ((int64_t)1 << 31)) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(p->device));
  if (grow((void **)&p->d_text, &p->text_cap, (size_t)n + 16)) return HPGQ_E_NOMEM;
  if (n) HPGQ_HIP_TRY(hipMemcpyAsync(p->d_text, text, (size_t)n, hipMemcpyHostToDevice, p->stream));
  return hpgq_parse_device(p, reinterpret_cast<const char *>(p->d_text), n, out);
}

int hpgq_parse_records(hpgq_parser_t *p, uint32_t *rec_start, uint32_t *seq_start,
                       uint32_t *plus_start, uint32_t *qual_start) {
  if (!p) return HPGQ_E_INVALID;
  HPGQ_HIP_TRY(hipSetDevice(p->device));
  const size_t b = (size_t)p->last_n * 4;
  uint32_t *dst[4] = {rec_start, seq_start, plus_start, qual_start};
  for (int k = 0; k < 4; ++k)
    if (dst[k] && b)
      HPGQ_HIP_TRY(hipMemcpyAsync(dst[k], p->d_rec + (size_t)k * p->rec_cap, b, hipMemcpyDeviceToHost,
                                  p->stream));
  HPGQ_HIP_TRY(hipStreamSynchronize(p->stream));
  return HPGQ_OK;
}

void *hpgq_parser_stream(hpgq_parser_t *p) { return p ? (void *)p->stream : nullptr; }

int64_t hpgq_parser_max_length(hpgq_parser_t *p) { return p ? p->max_len : 0; }

}  // extern "C"
