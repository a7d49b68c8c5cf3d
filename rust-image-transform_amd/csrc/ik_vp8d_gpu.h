// ik_vp8d_gpu.h -- launchers of the WebP (VP8) decoder's device half (ik_vp8d.hip); the
// host half (container, frame header, partition 0, the token partitions, driver) is
// ik_vp8d_host.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "ik_vp8d.h"

namespace ik {
namespace vp8d {

// One image of a decode launch (device addresses).  The planes are macroblock-aligned
// (mb_w * 16 by mb_h * 16 luma, half that chroma); top holds the unfiltered bottom rows
// the next MB row predicts from, two MB rows of them (32 bytes per MB: Y 16, U 8, V 8).
struct alignas(16) DImg {
    const DFrame* fr;
    const DMB* mbs;
    const uint32_t* coef;    // the frame's non-zero coefficients: (value << 16) | position in
                             // the MB's 384 (Y 16x16, U 4x16, V 4x16; dequantised, Y2 applied)
    const uint32_t* coef_at; // per MB its first entry; [mb_w * mb_h] = the total
    const uint8_t* flags;    // per MB: 1 = some coefficient is non-zero (libwebp !skip)
    uint8_t *y, *u, *v;
    uint8_t* top;
    uint8_t* out;            // the ik_image's pixels (RGB)
    uint32_t ys, uvs;        // plane pitches
    uint32_t out_pitch;
    uint32_t row0, rows;     // the launch's tickets of this image's MB rows: [row0, row0 + rows)
    uint32_t* prog;          // per MB row: MBs done (zeroed per launch)
    uint32_t* err;           // set when a row's wait times out (zeroed per launch)
};

// ticket: zeroed per launch; total_rows: the images' MB rows together
hipError_t launch_vp8d_recon(const DImg* imgs, int n, uint32_t total_rows, uint32_t* ticket, hipStream_t s);
hipError_t launch_vp8d_rgb(const DImg* imgs, int n, int max_h, hipStream_t s);

}  // namespace vp8d
}  // namespace ik
