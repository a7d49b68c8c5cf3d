// ik_vp8.h -- VP8 basics shared by the exact WebP coder (ik_vp8x.h / ik_vp8x.hip /
// ik_vp8x_host.cpp) and the segment analysis (ik_vp8_analysis.hip): the reference's
// WebP branch (src/transform.rs:129-137 -> webp 0.3.1 -> libwebp), restated for
// gfx950.  Mode numbering and scan orders are RFC 6386's / libwebp's; the tables
// are libwebp's read-only data (ik_vp8_tables.h).
#pragma once
#include <cstdint>

#include "ik_vp8_tables.h"

#if defined(__HIPCC__)
#define IK_HD __host__ __device__ inline
#define IK_UNROLL _Pragma("unroll")
#else
#define IK_HD inline
#define IK_UNROLL _Pragma("GCC unroll 16")
#endif

namespace ik {
namespace vp8 {

// libwebp's mode numbering: 4x4 modes, and the 16x16 / chroma modes that share
// the values of their 4x4 counterparts (used as contexts by neighbouring B_PRED MBs)
enum { B_DC = 0, B_TM, B_VE, B_HE, B_RD, B_VR, B_LD, B_VL, B_HD, B_HU, NUM_BMODES };
enum { DC_PRED = B_DC, TM_PRED = B_TM, V_PRED = B_VE, H_PRED = B_HE, B_PRED = 10 };

constexpr int kBps = 32;  // stride of the per-MB work buffers

IK_HD int zigzag(int n) {
    constexpr uint8_t z[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
    return z[n];
}
IK_HD int izigzag(int j) {  // raster position -> zigzag index
    constexpr uint8_t iz[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
    return iz[j];
}
IK_HD int band(int n) {
    constexpr uint8_t b[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
    return b[n];
}
IK_HD int clipi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace vp8
}  // namespace ik
