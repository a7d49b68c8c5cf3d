// ik_vp8_gpu.h -- launcher of the GPU VP8 macroblock encoder (ik_vp8.hip).
// Host code (ik_pipeline.cpp, ik_host.cpp) drives it; the bitstream is written on
// the host from the MBOut records (ik_vp8_enc.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "ik_vp8.h"

namespace ik {
namespace vp8 {

struct Vp8Args {
    const uint8_t* yuv;  // per image: Y (w*h), U, V ((w+1)/2 * (h+1)/2), back to back
    size_t yuv_stride;   // bytes between images
    int w, h, mb_w, mb_h;
    uint8_t* rec;        // per image: reconstruction Y (mb_w*16 x mb_h*16), U, V (mb_w*8 x mb_h*8)
    size_t rec_stride;
    MBOut* mbs;          // per image: mb_w*mb_h records, raster order
    uint8_t* nz;         // per image: mb_w*mb_h x 18 outgoing non-zero contexts (top[9], left[9])
    QParams q;
    unsigned long long* stamps;  // dev tool (IK_VP8_STAMPS): per diagonal, 8 phase clocks of image 0's first MB
};

inline size_t vp8_rec_bytes(int w, int h) {
    const size_t mw = (size_t)((w + 15) >> 4), mh = (size_t)((h + 15) >> 4);
    return mw * 16 * mh * 16 + 2 * mw * 8 * mh * 8;
}

// Compact MB stream of one image (k_vp8_pack -> host), cap bytes per image:
//   PackHeader {u32 bytes (header included), u32 mb count, u32 kPackMagic, u32 0}
//   per MB, raster order: u8 ymode, u8 uvmode, u8 skip, u8 0, u32 nzmask (bit b:
//   block b of MBOut.lv has a nonzero level); if ymode == B_PRED u8 bmodes[16];
//   then per set bit of nzmask, in block order: u16 coefficient mask (bit n:
//   lv[b][n] != 0), then the nonzero levels as int16, in coefficient order.
constexpr int kPackHeaderBytes = 16;
constexpr uint32_t kPackMagic = 0x4b503856u;  // "V8PK"
constexpr int kMaxPackMBs = 4096;             // one image's MBs (scan in LDS): 1024x1024
constexpr size_t kPackMaxMBBytes = 8 + 16 + 25 * (2 + 32);
inline size_t vp8_pack_cap(size_t nmb) { return (kPackHeaderBytes + nmb * kPackMaxMBBytes + 15) & ~(size_t)15; }
// libwebp's segment analysis (ik_vp8_analysis.hip): per image the k-means result
struct SegRecord {
    int32_t centers[4];
    int32_t mid;  // AssignSegments' weighted_average
    int32_t nmb;
    unsigned long long alpha_sum, uv_alpha_sum;  // MBAnalyze's accumulators
};
// n images of w x h YUV420 planes (Vp8Args layout) -> alpha/uva per MB, seg per MB
// (the k-means cluster, before SimplifySegments), rec per image
hipError_t launch_vp8_analysis(const uint8_t* yuv, size_t yuv_stride, int n, int w, int h, uint8_t* alpha,
                               uint16_t* uva, uint8_t* seg, SegRecord* rec, hipStream_t s);

hipError_t launch_vp8_pack(const MBOut* mbs, int nmb, int n, uint8_t* scratch, uint8_t* host_dst, size_t cap_img,
                           hipStream_t s);

// the whole wavefront for n images: (mb_w-1) + 2*(mb_h-1) + 1 launches on stream s
hipError_t launch_vp8_encode(const Vp8Args& a, int n, hipStream_t s);

}  // namespace vp8
}  // namespace ik
