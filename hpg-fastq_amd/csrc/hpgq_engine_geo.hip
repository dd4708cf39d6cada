// hpgq_engine_geo.hip — instances of the segmented kernel for ONE geometry
// (built once per geometry with -DHPGQ_GEO=0|1|2, so the three compile in
// parallel).  Occupancy per variant (MINW, waves per SIMD) is the highest at
// which the variant's registers fit without spills: single-end 4 (tri 5),
// paired-end 3 (two mates' accumulators), single-end edit 3 (its next trim
// windows held in VGPRs, tri_body EG; 4 with the extra scans or as a
// follow-up; 4 with the trims at the step, tri_body ST), see DESIGN.md §4.1.  Every
// combination of paired-end, edit and the extra filter scans has an instance.
#include <cstdio>

#include "hpgq_engine_tri.h"

#ifndef HPGQ_GEO
#error "build with -DHPGQ_GEO=0 (tri), 1 (hex) or 2 (wide)"
#endif

namespace hpgq {

namespace {

constexpr int G = HPGQ_GEO;
#ifndef HPGQ_SE_WAVES
#define HPGQ_SE_WAVES (G == GEO_TRI ? 5 : 4)
#endif
constexpr int kSeW = HPGQ_SE_WAVES;          // single-end
#ifndef HPGQ_PE_WAVES
#define HPGQ_PE_WAVES 3
#endif
constexpr int kPeW = HPGQ_PE_WAVES;          // paired-end
#ifndef HPGQ_EDIT_WAVES
#define HPGQ_EDIT_WAVES 3
#endif
constexpr int kEdW = HPGQ_EDIT_WAVES;        // single-end edit (its trim windows in VGPRs a group early: tri_body EG)
constexpr int kEdXW = kSeW;                  // single-end edit with extra filter scans
#ifndef HPGQ_ST_WAVES
#define HPGQ_ST_WAVES 4
#endif
constexpr int kStW = HPGQ_ST_WAVES;          // single-end edit, trims at the step (tri_body ST; its 7
                                             // spilled VGPRs sit outside the group loop)
constexpr const char *kGeoName = G == GEO_TRI ? "tri" : (G == GEO_HEX ? "hex" : "wide");

template <bool F, int XM, bool EDIT>
const void *x_kernel(int nm) {
  return nm == 2 ? (const void *)engine_tri_x_kernel<kPeW, 2, G, F, XM, EDIT>
                 : (const void *)engine_tri_x_kernel<EDIT ? kEdXW : kSeW, 1, G, F, XM, EDIT>;
}

template <bool F, bool EDIT>
const void *x_kernel_for(int nm, int xm) {
  return xm == X_NOOR ? x_kernel<F, X_NOOR, EDIT>(nm) : xm == X_LR ? x_kernel<F, X_LR, EDIT>(nm)
                                                            : x_kernel<F, X_NOOR | X_LR, EDIT>(nm);
}

template <bool F>
SegChoice pick(int nm, bool edit, int xm, char *name, size_t cap) {
  const void *fn = nullptr;
  if (xm == X_ST) {   // single-end edit with the trims applied at the step (hex, first stage: tri_body ST)
    if constexpr (G == GEO_HEX && !F) {
      if (nm == 1 && edit) fn = (const void *)engine_tri_x_kernel<kStW, 1, G, false, X_ST, true>;
    }
    std::snprintf(name, cap, "hpgq::engine_tri_kernel<%d, 1, edit, %s, st>", kStW, kGeoName);
    return SegChoice{fn, kStW};
  }
  const int w = nm == 2 ? kPeW : (edit ? (xm || F ? kEdXW : kEdW) : kSeW);
  if (xm) {
    fn = edit ? x_kernel_for<F, true>(nm, xm) : x_kernel_for<F, false>(nm, xm);
    std::snprintf(name, cap, "hpgq::engine_tri_x_kernel<%d, %d, %s%s%s%s%s>", w, nm, kGeoName,
                  edit ? ", edit" : "", F ? ", follow" : "", (xm & X_NOOR) ? ", noor" : "",
                  (xm & X_LR) ? ", window" : "");
  } else {
    if (nm == 2) fn = edit ? (const void *)engine_tri_kernel<kPeW, 2, true, G, F>
                           : (const void *)engine_tri_kernel<kPeW, 2, false, G, F>;
    else if (edit) fn = (const void *)engine_tri_kernel<F ? kSeW : kEdW, 1, true, G, F>;
    else fn = (const void *)engine_tri_kernel<kSeW, 1, false, G, F>;
    std::snprintf(name, cap, "hpgq::engine_tri_kernel<%d, %d, %s, %s%s>", w, nm, edit ? "edit" : "filter", kGeoName,
                  F ? ", follow" : "");
  }
  return SegChoice{fn, w};
}

}  // namespace

#if HPGQ_GEO == 0
SegChoice seg_kernel_tri(int nm, bool edit, int xm, bool follow, char *name, size_t cap) {
  return follow ? SegChoice{nullptr, 0} : pick<false>(nm, edit, xm, name, cap);
}
#elif HPGQ_GEO == 1
SegChoice seg_kernel_hex(int nm, bool edit, int xm, bool follow, char *name, size_t cap) {
  return follow ? SegChoice{nullptr, 0} : pick<false>(nm, edit, xm, name, cap);
}
#else
SegChoice seg_kernel_wide(int nm, bool edit, int xm, bool follow, char *name, size_t cap) {
  return follow ? pick<true>(nm, edit, xm, name, cap) : pick<false>(nm, edit, xm, name, cap);
}
#endif

}  // namespace hpgq
