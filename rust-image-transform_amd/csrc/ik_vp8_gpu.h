// ik_vp8_gpu.h -- launcher of libwebp's segment analysis on the GPU
// (ik_vp8_analysis.hip), the first stage of the exact WebP coder (ik_vp8x.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "ik_vp8.h"

namespace ik {
namespace vp8 {

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

}  // namespace vp8
}  // namespace ik
