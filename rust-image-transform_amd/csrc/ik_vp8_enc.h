// ik_vp8_enc.h -- host half of the GPU WebP (VP8 key frame) encoder: everything
// after the macroblock decisions -- coefficient-probability adaptation, the
// boolean entropy coder, the frame header and the RIFF/WEBP container.
#pragma once
#include <cstdint>
#include <vector>

#include "ik_vp8.h"

namespace ik {
namespace vp8 {

// libwebp's quality -> quantiser index (VP8SetSegmentParams, one segment at the
// mid susceptibility): c = QualityToCompression(q/100), qindex = 127 * (1 - c)
int quality_to_qindex(float quality);

// the quantiser / lambda / filter parameters the encoder uses for `quality`
// (chroma DC delta -4 * sns_strength / 100 = -2 at libwebp's default sns 50)
QParams qparams_for_quality(float quality);

// Bitstream for one frame of mb_w x mb_h macroblocks (raster order) with the
// decisions in `mbs`.  `filter_level` < 0 uses q.filter_level.
void write_webp(int width, int height, const QParams& q, const MBOut* mbs, int filter_level,
                std::vector<uint8_t>& out);

// zigzag index after the last nonzero level of a block (== first when none)
int last_nz(const int16_t* lv, int first);

}  // namespace vp8
}  // namespace ik
