// hpgq_cgr_post.cpp — chaos-game post-processing on the host (O(4^k) per run):
// genomic-signature files, the difference table against a reference, its
// mean / standard deviation, quality normalisation and the PGM images.
// Restates old/chaos_game.c:43-50 (header_gs_init), :269-318 (GS loaders),
// :320-373 (chaos_game_calculate_table_dif), :375-408 (validate),
// :410-472 (write_table_images), :484-593 (private helpers); constants
// old/chaos_game.h:33-49, header_gs_t :65-70.  Tables are row-major
// [co_x][co_y] u32, as hpgq_cgr_read returns them.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hpgq.h"

namespace {

constexpr int kMinKImage = 7;        // MIN_K_IMAGE_VALUE
constexpr int kMinImagePixels = 128; // MIN_IMAGE_PIXEL_SIZE
constexpr int kMaxQualityInTable = 62;   // MAX_QUALITY_IN_TABLE

// header_gs_t (old/chaos_game.h:65-70): char[180] + 4 x unsigned int, no padding
struct GsHeader {
  char gs_filename[180];
  uint32_t word_size_k, dim_x, dim_y, ref_word_count;
};
static_assert(sizeof(GsHeader) == HPGQ_GS_HEADER_BYTES, "header_gs_t layout");

bool valid_k(int k) { return k >= 1 && k <= 12; }

}  // namespace

extern "C" {

int hpgq_cgr_write_gs(const char *path, int k, const uint32_t *table, uint32_t word_count) {
  if (!path || !table || !valid_k(k)) return HPGQ_E_INVALID;
  const int dim = 1 << k;
  GsHeader h;
  std::memset(&h, 0, sizeof(h));
  std::strncpy(h.gs_filename, path, sizeof(h.gs_filename) - 1);   // header_gs_init (:43-50)
  h.word_size_k = (uint32_t)k;
  h.dim_x = (uint32_t)dim;
  h.dim_y = (uint32_t)dim;   // (:47 sets dim_x twice; dim_y is written here)
  h.ref_word_count = word_count;
  FILE *f = std::fopen(path, "wb");
  if (!f) return HPGQ_E_IO;
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1 &&
            std::fwrite(table, sizeof(uint32_t), (size_t)dim * dim, f) == (size_t)dim * dim;
  ok = std::fclose(f) == 0 && ok;
  return ok ? HPGQ_OK : HPGQ_E_IO;
}

int hpgq_cgr_load_gs(const char *path, int k, uint32_t *table_gs, uint32_t *ref_word_count) {
  if (!path || !table_gs || !valid_k(k)) return HPGQ_E_INVALID;
  const int dim = 1 << k;
  FILE *f = std::fopen(path, "rb");   // chaos_game_load_table_gs_direct (:297-318)
  if (!f) return HPGQ_E_IO;
  GsHeader h;
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 &&
            std::fread(table_gs, sizeof(uint32_t), (size_t)dim * dim, f) == (size_t)dim * dim;
  std::fclose(f);
  if (!ok) return HPGQ_E_IO;
  if (ref_word_count) *ref_word_count = h.ref_word_count;
  return HPGQ_OK;
}

// chaos_game_calculate_table_dif (:320-373): the tables scaled to 128 per cell
// on average (norm = 128 / (words / 4^k)), subtracted in double, stored as int
int hpgq_cgr_table_dif(int k, const uint32_t *table_seq, uint32_t fq_word_count, const uint32_t *table_gs,
                       uint32_t ref_word_count, int32_t *table_dif, int32_t *highest, int32_t *lowest) {
  if (!table_seq || !table_gs || !table_dif || !valid_k(k)) return HPGQ_E_INVALID;
  const int dim = 1 << k;
  const int memory_size = 1 << (2 * k);
  double fq_norm = (double)(1.0 * fq_word_count / memory_size);
  if (!(fq_norm > 0.0)) return HPGQ_E_INVALID;   // LOG_FATAL in the reference
  fq_norm = 128.0 / fq_norm;
  double gs_norm = (double)(1.0 * ref_word_count / memory_size);
  if (!(gs_norm > 0.0)) return HPGQ_E_INVALID;
  gs_norm = 128.0 / gs_norm;
  int hi = -32768, lo = 32768;
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) {
      const size_t c = (size_t)i * dim + j;
      const double d = (table_seq[c] * fq_norm) - (table_gs[c] * gs_norm);
      const int v = (int)d;   // truncation toward zero, as the int table stores it
      table_dif[c] = v;
      if (hi < v) hi = v;
      if (lo > v) lo = v;
    }
  if (highest) *highest = hi;
  if (lowest) *lowest = lo;
  return HPGQ_OK;
}

// chaos_game_validate_table_dif (:375-408); the accumulators start at 0 (quirk
// Q12: uninitialised locals in the reference)
int hpgq_cgr_dif_stats(int k, const int32_t *table_dif, double *mean, double *std_dev) {
  if (!table_dif || !valid_k(k)) return HPGQ_E_INVALID;
  const int dim = 1 << k;
  double m = 0.0, s = 0.0;
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) m += table_dif[(size_t)i * dim + j];
  m /= (double)(1.0 * dim * dim);
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) s += std::pow((table_dif[(size_t)i * dim + j] - m), 2);
  s /= (double)(1.0 * dim * dim);
  s = std::sqrt(s);
  if (mean) *mean = m;
  if (std_dev) *std_dev = s;
  return HPGQ_OK;
}

// chaos_game_normalize_quality_table_ (:487-502), in place: per-word mean quality
int hpgq_cgr_normalize_quality(int k, const uint32_t *table_seq, uint32_t *table_q) {
  if (!table_seq || !table_q || !valid_k(k)) return HPGQ_E_INVALID;
  const size_t cells = (size_t)1 << (2 * k);
  for (size_t c = 0; c < cells; ++c) {
    if (table_seq[c] > 0) {
      table_q[c] /= (uint32_t)k;
      table_q[c] /= table_seq[c];
    } else {
      table_q[c] = 0;
    }
  }
  return HPGQ_OK;
}

// chaos_game_generate_pgm_file_ (:521-593): binary PGM, pixel = (uchar)(int)
// (float)(table * norm); k < 7 is zoomed to 128 x 128
int hpgq_cgr_write_pgm(const char *path, int k, const uint32_t *table, double norm) {
  if (!path || !table || !valid_k(k)) return HPGQ_E_INVALID;
  const int dim = 1 << k;
  const int redim = k < kMinKImage ? kMinImagePixels : dim;
  const int zoom = k < kMinKImage ? 1 << (kMinKImage - k) : 1;
  std::vector<unsigned char> img((size_t)redim * redim, 0);
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) {
      float v = (float)table[(size_t)i * dim + j];
      v = v * norm;   // float * double, rounded back to float
      const unsigned char px = (unsigned char)(int)v;
      for (int ii = 0; ii < zoom; ++ii)
        for (int jj = 0; jj < zoom; ++jj) img[(size_t)(i * zoom + ii) * redim + (j * zoom + jj)] = px;
    }
  FILE *f = std::fopen(path, "wb");
  if (!f) return HPGQ_E_IO;
  std::fprintf(f, "P5\n%d %d\n%d\n", redim, redim, 255);
  bool ok = std::fwrite(img.data(), 1, img.size(), f) == img.size();
  ok = std::fclose(f) == 0 && ok;
  return ok ? HPGQ_OK : HPGQ_E_IO;
}

// chaos_game_write_table_images (:410-472): <dir>/<fq name>_k=<k>_FG.pgm (the
// sequence table, norm 128 / (words / 4^k)), _QQ.pgm (the quality table
// normalised in place, norm 256 / 62) and, with a difference table,
// _FG_dif.pgm (|dif| clamped to 255, norm 1)
int hpgq_cgr_write_images(const char *report_dir, const char *fq_path, int k, const uint32_t *table_seq,
                          uint32_t *table_q, uint32_t fq_word_count, const int32_t *table_dif) {
  if (!report_dir || !fq_path || !table_seq || !table_q || !valid_k(k)) return HPGQ_E_INVALID;
  const char *slash = std::strrchr(fq_path, '/');
  const char *name = slash ? slash + 1 : fq_path;   // get_filename_from_path
  const std::string base = std::string(report_dir) + "/" + name + "_k=" + std::to_string(k);
  const int memory_size = 1 << (2 * k);
  double fq_norm = (double)fq_word_count;
  fq_norm = fq_norm / memory_size;
  if (!(fq_norm > 0.0)) return HPGQ_E_INVALID;
  fq_norm = 128.0 / fq_norm;
  int rc = hpgq_cgr_write_pgm((base + "_FG.pgm").c_str(), k, table_seq, fq_norm);
  if (rc) return rc;
  rc = hpgq_cgr_normalize_quality(k, table_seq, table_q);
  if (rc) return rc;
  rc = hpgq_cgr_write_pgm((base + "_QQ.pgm").c_str(), k, table_q, 256.0 / kMaxQualityInTable);
  if (rc || !table_dif) return rc;
  std::vector<uint32_t> absd((size_t)memory_size);   // chaos_game_absolute_diff_table_ (:504-519)
  for (int c = 0; c < memory_size; ++c) {
    int v = std::abs(table_dif[c]);
    if (v > 255) v = 255;
    absd[c] = (unsigned char)v;
  }
  return hpgq_cgr_write_pgm((base + "_FG_dif.pgm").c_str(), k, absd.data(), 1);
}

}  // extern "C"
