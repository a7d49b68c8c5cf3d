// ik_png.h -- device-side descriptors and launchers of the GPU PNG decoder
// (kernels: ik_png.hip; host orchestration: ik_png_decode.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ik_inflate.h"

namespace ik {

constexpr int kPngInflateThreads = 64;     // decoder lanes per workgroup (one wave: LDS 320 B per lane)
constexpr int kPngExpandThreads = 64;      // expand lanes per workgroup (LDS: 256 B literal table each)
constexpr int kPngUnfilterThreads = 1024;  // 16 waves, one 64-row band each
constexpr int kPngUnfilterWaves = kPngUnfilterThreads / 64;
// workgroups per image for the unfilter pass: one per 16 bands of 64 rows, at
// most 32 (all of an image's workgroups must be resident together)
IK_HD int png_unfilter_groups(int h) {
    const int g = ((h + 63) / 64 + kPngUnfilterWaves - 1) / kPngUnfilterWaves;
    return g < 32 ? g : 32;
}
constexpr uint64_t kPngChunkBytes = 16384; // candidate-search chunk of the compressed stream
constexpr int kPngPageShift = 12;          // resolve: output page -> decoder table

// one image of a batch, as the kernels see it
struct PngImgDev {
    const uint32_t* words;   // zlib stream (little-endian words, zero padded)
    uint64_t bit0;           // first DEFLATE bit (after the 2-byte zlib header)
    uint64_t nbits;          // stream length in bits
    uint16_t* u16;           // expand pass output: raw_total symbols (+ padding)
    uint64_t raw_total;      // bytes of the filtered image (H rows of 1 + rowbytes)
    const int64_t* obase;    // output offset of each decoder lane (ascending)
    const int* page_lane;    // decoder holding the first byte of each output page
    int nlanes;
    int rowbytes, H, bpp;
    uint8_t* ft;             // filter type of every row
    uint8_t* dst;            // the image (pitched); filtered rows, then pixels in place
    size_t pitch;
};

struct PngLaneDev {
    uint64_t start, stop;    // decode: block boundary to start at; next lane's start (~0 = last)
    uint64_t tbase;          // token region: index into the batch's token area (a multiple of 8)
    int64_t obase;           // expand: output offset
    uint64_t out_len;        // expand: output bytes
    uint32_t ntok;           // decode: region capacity (tokens); expand: tokens to read
    uint32_t img;            // image of the batch
    uint32_t first;          // lane 0 of its image (no distance reaches before its output)
    uint32_t pad;
};

// dst[i] = src[i] for n words, on the compute stream; one side may be pinned host
// memory (the small transfers of the PNG kernel phase: ik_png_decode.cpp Xfer)
hipError_t launch_copy_words(const uint32_t* src, uint32_t* dst, size_t n, hipStream_t s);
hipError_t launch_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx, int n,
                           uint64_t chunk_bits, int64_t* cand, hipStream_t s);
hipError_t launch_png_decode(const PngImgDev* imgs, const PngLaneDev* lanes, int n, uint16_t* tok,
                             infl::LaneResult* res, hipStream_t s);
hipError_t launch_png_expand(const PngImgDev* imgs, const PngLaneDev* lanes, int n, const uint16_t* tok, int* status,
                             hipStream_t s);
hipError_t launch_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows, int* err, hipStream_t s);
// groups[t] = (image, band group) of the workgroup holding ticket t; prog: one
// zeroed counter per band (the image's at prog_base[image]); ticket: zeroed
hipError_t launch_png_unfilter(const PngImgDev* imgs, const int2* groups, int ngroups, const int* prog_base,
                               unsigned* prog, unsigned* ticket, int bpp, hipStream_t s);

}  // namespace ik
