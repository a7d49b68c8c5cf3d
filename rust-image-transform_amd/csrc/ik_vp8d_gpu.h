// ik_vp8d_gpu.h -- launchers of the WebP (VP8) decoder's device half (ik_vp8d.hip); the
// host half (container, frame header, partition 0, driver) is ik_vp8d_host.cpp.
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
    const uint8_t* file;  // the file bytes (16-byte aligned, 16 bytes of slack after)
    int16_t* coef;        // per MB 384 dequantised coefficients (Y 16x16, U 4x16, V 4x16)
    uint8_t* flags;       // per MB: 1 = some coefficient is non-zero (libwebp !skip)
    uint8_t *y, *u, *v;
    uint8_t* top;
    uint8_t* out;         // the ik_image's pixels (RGB)
    uint32_t ys, uvs;     // plane pitches
    uint32_t out_pitch;
    uint32_t* err;        // set to 1 when a token partition runs out of data
};

constexpr int kReconWaves = 8;  // MB rows in flight per image

hipError_t launch_vp8d_tokens(const DImg* imgs, int n, hipStream_t s);
hipError_t launch_vp8d_recon(const DImg* imgs, int n, hipStream_t s);
hipError_t launch_vp8d_rgb(const DImg* imgs, int n, int max_h, hipStream_t s);

}  // namespace vp8d
}  // namespace ik
