// ik_vp8x_gpu.h -- launchers of the exact WebP coder's device half (ik_vp8x.hip); the
// host driver and bitstream writer are ik_vp8x.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "ik_vp8x.h"

namespace ik {
namespace vp8x {

struct XArgs {
    const uint8_t* yuv;  // per image: Y (w*h), U, V ((w+1)/2 * (h+1)/2)
    size_t yuv_stride;
    int w, h, mb_w, mb_h;
    uint8_t* rec;        // per image: reconstruction Y (mb_w*16 x mb_h*16), U, V (mb_w*8 x mb_h*8)
    size_t rec_stride;
    XMB* mbs;            // per image mb_w*mb_h records
    uint32_t* nz;        // per image per MB: the packed non-zero contexts after it
    int8_t* derr;        // per image per MB: chroma DC errors handed down [0..3] and right [4..7]
    const uint8_t* seg;  // per image per MB: segment
    const XSeg* segs;    // per image 4
    uint16_t* lc;        // per image: level costs [96][68]
    uint8_t* pr;         // per image: coefficient probabilities [1056]
    uint32_t* stats;     // per image: token statistics [1056]
    int* max_edge;       // per image 4
    int use_derr;
};

hipError_t launch_vp8x_mb(const XArgs& a, const int* list, int count, int n, hipStream_t s);
hipError_t launch_vp8x_stats(const XArgs& a, int k0, int k1, int n, hipStream_t s);

}  // namespace vp8x
}  // namespace ik
