// ik_vp8_enc.h -- host half of the GPU WebP (VP8 key frame) encoder: everything
// after the macroblock decisions -- coefficient-probability adaptation, the
// boolean entropy coder, the frame header and the RIFF/WEBP container.
#pragma once
#include <cstddef>
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

// The same bitstream from the compact MB stream k_vp8_pack writes (layout in
// ik_vp8_gpu.h; at most cap bytes): false, and no output, when it is malformed.
bool write_webp_packed(int width, int height, const QParams& q, const uint8_t* pack, size_t cap, int filter_level,
                       std::vector<uint8_t>& out);

// the host form of k_vp8_pack (same bytes) for records already on the host
void pack_mbs(const MBOut* mbs, size_t nmb, std::vector<uint8_t>& out);

// zigzag index after the last nonzero level of a block (== first when none)
int last_nz(const int16_t* lv, int first);

}  // namespace vp8
}  // namespace ik
