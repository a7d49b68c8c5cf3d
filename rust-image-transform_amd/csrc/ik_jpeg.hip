// ik_jpeg.hip -- gfx950 kernels of decode_image's JPEG reconstruction (reference
// src/transform.rs:31 -> image 0.25.8 -> zune-jpeg 0.4.21), fed by the host
// entropy decoder in ik_jpeg_decode.cpp:
//
//   k_jpeg_idct   one lane per 8x8 block: dequantise (coef * qt) and a 2-D
//                 integer IDCT into the component's u8 sample plane (MCU-padded).
//   k_jpeg_color  one lane per four output pixels: chroma upsampling and colour
//                 conversion, written into the device image as whole dwords.
//
// Two reconstructions over the same coefficients (JpegGeom::recon):
//   IK_JPEG_RECON_ZUNE (default; the reference's decoder) -- zune-jpeg 0.4.21
//     restated: idct/scalar.rs (stb_image-derived fixed point; a block with 63
//     zero AC coefficients takes clamp((dc >> 3) + 128)), upsampler/scalar.rs
//     (separable (3 near + far + 2) >> 2, vertical first, over the MCU-padded
//     rows), color_convert/scalar.rs (i16: 45/32, 11/32 + 23/32, 113/64).  Parity
//     unpinned (no zune-jpeg here); equal to the oracle's restatement
//     (oracle/jpeg_dec.c) bit for bit.
//   IK_JPEG_RECON_LIBJPEG -- libjpeg-turbo: jidctint.c islow, jdsample.c fancy
//     upsampling over the real component size, jdcolor.c (SCALEBITS 16); equal to
//     Pillow's decoder bit for bit (tests/test_gpu_decode.py).
// CMYK / YCCK (Adobe APP14 transform 0 / 2) convert to RGB8 as Pillow does
// (inverted Adobe samples, Convert.c cmyk2rgb), in both modes.
#include "../../include/imagekit_hip.h"
#include "ik_internal.h"
#include "ik_jpeg_idct.h"

namespace ik {

namespace {

using namespace jidct;

__device__ __forceinline__ void idct_block(const JpegGeom& g, long long blk) {
    if (blk >= g.nblocks) return;
    int ci = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (i < g.ncomp && blk >= g.blk0[i]) ci = i;
    const long long l = blk - g.blk0[ci];
    const int bw = g.bw[ci];
    const int by = (int)(l / bw), bx = (int)(l - (long long)by * bw);
    const int pw = bw * 8;
    uint8_t* out = g.planes + g.plane0[ci] + (size_t)by * 8 * pw + (size_t)bx * 8;

    // dequantised coefficients (JCOEF * ISLOW_MULT_TYPE), natural order
    int in[64];
    const int4* cp = reinterpret_cast<const int4*>(g.coef + blk * 64);
    const uint16_t* q = g.qt + ci * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int4 v = cp[i];
        const int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = i * 8 + 2 * j;
            in[k] = (int)(int16_t)(w[j] & 0xffff) * (int)q[k];
            in[k + 1] = (int)(int16_t)((unsigned)w[j] >> 16) * (int)q[k + 1];
        }
    }
    if (g.recon == IK_JPEG_RECON_ZUNE) {
        idct_zune(in, out, pw);
        return;
    }
    idct_islow(in, out, pw);
}

// the first pixel column past a zune_fast image's interior groups of eight
// (k_jpeg_color_fast_b takes x0 in [8, xc), k_jpeg_color_ends_b the rest)
__device__ __forceinline__ int fast_xc(const JpegGeom& g) {
    const int lim = 2 * g.bw[1] * 8 - 2;
    const int xm = (g.W - 8 < lim - 8 ? g.W - 8 : lim - 8);
    return xm < 8 ? 8 : (xm & ~7) + 8;
}

__global__ __launch_bounds__(256) void k_jpeg_idct(JpegGeom g) { idct_block(g, (long long)blockIdx.x * 256 + threadIdx.x); }
// the batch's images in one launch: blockIdx.y = image
__global__ __launch_bounds__(256) void k_jpeg_idct_b(const JpegReconItem* __restrict__ items) {
    const JpegReconItem& it = items[blockIdx.y];
    const long long blk = (long long)blockIdx.x * 256 + threadIdx.x;
    if (it.fast && blk < it.g.blk0[1]) {
        // a zune_fast image's luma blocks in the interior columns are k_jpeg_color_fast_b's own
        // (its groups x0 in [8, xc) step 8 are block columns 1 .. xc/8 - 1; the row ends'
        // columns stay here, for k_jpeg_color_ends_b)
        const JpegGeom& g = it.g;
        const int bx = (int)(blk % g.bw[0]);
        if (bx >= 1 && bx < fast_xc(g) / 8) return;
    }
    idct_block(it.g, blk);
}

// upsampled sample of component ci at output pixel (x, y)
__device__ __forceinline__ int upsampled(const JpegGeom& g, int ci, int x, int y) {
    const int fh = g.hmax / g.h[ci], fv = g.vmax / g.v[ci];
    const int dw = g.dw[ci], dh = g.dh[ci], pw = g.bw[ci] * 8;
    const uint8_t* p = g.planes + g.plane0[ci];
    const int ow = dw * fh, oh = dh * fv;
    const int xs = x < ow ? x : ow - 1, ys = y < oh ? y : oh - 1;
    auto row = [&](int r) { return p + (size_t)(r < 0 ? 0 : (r >= dh ? dh - 1 : r)) * pw; };
    if (fh == 1 && fv == 1) return row(ys)[xs];
    if (fh == 2 && fv == 1) {  // h2v1_fancy_upsample
        const uint8_t* ip = row(ys);
        const int X = xs >> 1;
        if (dw == 1) return ip[0];
        if (!(xs & 1)) return X == 0 ? ip[0] : (ip[X] * 3 + ip[X - 1] + 1) >> 2;
        return X == dw - 1 ? ip[X] : (ip[X] * 3 + ip[X + 1] + 2) >> 2;
    }
    if (fh == 2 && fv == 2) {  // h2v2_fancy_upsample
        const int Y = ys >> 1, X = xs >> 1;
        const uint8_t* i0 = row(Y);
        const uint8_t* i1 = row((ys & 1) ? Y + 1 : Y - 1);
        const int thiss = i0[X] * 3 + i1[X];
        if (dw == 1) return (xs & 1) ? (thiss * 4 + 7) >> 4 : (thiss * 4 + 8) >> 4;
        if (!(xs & 1)) {
            if (X == 0) return (thiss * 4 + 8) >> 4;
            const int lasts = i0[X - 1] * 3 + i1[X - 1];
            return (thiss * 3 + lasts + 8) >> 4;
        }
        if (X == dw - 1) return (thiss * 4 + 7) >> 4;
        const int nexts = i0[X + 1] * 3 + i1[X + 1];
        return (thiss * 3 + nexts + 7) >> 4;
    }
    if (fh == 1 && fv == 2) {  // h1v2_fancy_upsample (libjpeg-turbo)
        const int Y = ys >> 1;
        const bool lower = ys & 1;
        const uint8_t* i0 = row(Y);
        const uint8_t* i1 = row(lower ? Y + 1 : Y - 1);
        return (i0[xs] * 3 + i1[xs] + (lower ? 2 : 1)) >> 2;
    }
    return row(ys / fv)[xs / fh];  // int_upsample: replication
}

// zune-jpeg 0.4.21 upsampler/scalar.rs at output pixel (x, y): over the whole
// MCU-padded plane (n = bw * 8 samples per row, bh * 8 rows), rows above / below
// replicated at the padded edges; h2v2 = upsample_vertical into i16, then
// upsample_horizontal on that row
__device__ __forceinline__ int upsampled_zune(const JpegGeom& g, int ci, int x, int y) {
    const int fh = g.hmax / g.h[ci], fv = g.vmax / g.v[ci];
    const int n = g.bw[ci] * 8, ph = g.bh[ci] * 8;
    const uint8_t* p = g.planes + g.plane0[ci];
    auto row = [&](int r) { return p + (size_t)(r < 0 ? 0 : (r >= ph ? ph - 1 : r)) * n; };
    if (fh == 1 && fv == 1) return row(y)[x];
    if (fh == 1 && fv == 2) {
        const int Y = y >> 1;
        return (row(Y)[x] * 3 + row((y & 1) ? Y + 1 : Y - 1)[x] + 2) >> 2;
    }
    if (fh == 2 && (fv == 1 || fv == 2)) {
        const uint8_t* i0 = row(fv == 2 ? y >> 1 : y);
        const uint8_t* i1 = fv == 2 ? row((y & 1) ? (y >> 1) + 1 : (y >> 1) - 1) : i0;
        // the (vertically upsampled) sample k of the row
        auto at = [&](int k) { return fv == 2 ? (i0[k] * 3 + i1[k] + 2) >> 2 : (int)i0[k]; };
        const int i = x >> 1;
        if (x == 0) return at(0);
        if (x == 1) return (at(0) * 3 + at(1) + 2) >> 2;
        if (x == 2 * n - 2) return (at(n - 2) * 3 + at(n - 1) + 2) >> 2;
        if (x == 2 * n - 1) return at(n - 1);
        return (x & 1) ? (at(i) * 3 + at(i + 1) + 2) >> 2 : (at(i) * 3 + at(i - 1) + 2) >> 2;
    }
    return row(y / fv)[x / fh];  // upsample_generic: replication
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Pillow Convert.c MULDIV255
__device__ __forceinline__ int muldiv255(int a, int b) {
    const int t = a * b + 128;
    return ((t >> 8) + t) >> 8;
}

// one output pixel (x, y): gray -> o[0]; otherwise RGB -> o[0..2]
__device__ __forceinline__ void color_pixel(const JpegGeom& g, int x, int y, uint8_t* o) {
    const bool zune = g.recon == IK_JPEG_RECON_ZUNE;
    auto sample = [&](int ci) { return zune ? upsampled_zune(g, ci, x, y) : upsampled(g, ci, x, y); };
    if (g.colorspace == 0) {
        o[0] = (uint8_t)sample(0);
        return;
    }
    const int c0 = sample(0), c1 = sample(1), c2 = sample(2);
    int r, gg, b;
    if (g.colorspace == 2 || g.colorspace == 3) {
        r = c0; gg = c1; b = c2;
    } else if (zune) {
        // color_convert/scalar.rs ycbcr_to_rgb_inner_16_scalar, i16 arithmetic
        const int16_t cb = (int16_t)(c1 - 128), cr = (int16_t)(c2 - 128);
        r = c0 + ((int16_t)(45 * cr) >> 5);
        gg = c0 - ((int16_t)(11 * cb + 23 * cr) >> 5);
        b = c0 + ((int16_t)(113 * cb) >> 6);
    } else {
        // jdcolor.c ycc_rgb_convert, SCALEBITS 16: FIX(1.402) 91881, FIX(1.772) 116130,
        // FIX(0.71414) 46802, FIX(0.34414) 22554
        const int cb = c1 - 128, cr = c2 - 128;
        r = c0 + ((91881 * cr + 32768) >> 16);
        gg = c0 + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
        b = c0 + ((116130 * cb + 32768) >> 16);
    }
    if (g.colorspace < 3) {
        o[0] = clamp255(r);
        o[1] = clamp255(gg);
        o[2] = clamp255(b);
        return;
    }
    // CMYK / YCCK -> RGB8: YCCK's YCbCr part gives inverted C, M, Y (jdcolor.c
    // ycck_cmyk_convert); Adobe samples are inverted (Pillow rawmode "CMYK;I");
    // then Pillow Convert.c cmyk2rgb
    int cc = r, mm = gg, yy = b;
    if (g.colorspace == 4) { cc = 255 - clamp255(r); mm = 255 - clamp255(gg); yy = 255 - clamp255(b); }
    int k = sample(3);
    if (g.adobe) { cc = 255 - cc; mm = 255 - mm; yy = 255 - yy; k = 255 - k; }
    const int nk = 255 - k;
    o[0] = clamp255(nk - muldiv255(cc, nk));
    o[1] = clamp255(nk - muldiv255(mm, nk));
    o[2] = clamp255(nk - muldiv255(yy, nk));
}

// Four consecutive pixels per thread: the row's output goes out as whole dwords (3
// per thread for RGB, 1 for gray; rows are 256-B pitched, so 4 pixels start on a
// 4-byte boundary) instead of three byte stores per pixel; a partial group at the
// row's end is stored byte by byte.
// zune YCbCr with chroma at half width (4:2:0 / 4:2:2) and full-resolution luma,
// four pixels x0 .. x0+3 away from the row's ends (x0 >= 4, x0 + 3 < 2n - 2; n =
// the chroma plane's padded width): upsampled_zune's interior formulas and
// color_pixel's arithmetic on whole dwords -- one luma dword, four chroma bytes
// per row and plane -- instead of per-sample byte loads and the generic branches.
__host__ __device__ __forceinline__ bool zune_fast(const JpegGeom& g) {
    return g.recon == IK_JPEG_RECON_ZUNE && g.colorspace == 1 && g.ncomp == 3 && g.h[0] == g.hmax &&
           g.v[0] == g.vmax && g.hmax == 2 * g.h[1] && g.hmax == 2 * g.h[2] && g.v[1] == g.v[2] &&
           (g.vmax == g.v[1] || g.vmax == 2 * g.v[1]) && g.bw[1] == g.bw[2] && g.bh[1] == g.bh[2];
}

// bytes i .. i+3 of a 4-B-aligned row (i odd here, so both dwords hold bytes used:
// no read past the row)
__device__ __forceinline__ uint32_t bytes4(const uint8_t* p, uint32_t i) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p) + (i >> 2);
    return __builtin_amdgcn_alignbyte(w[1], w[0], i & 3u);
}

__device__ __forceinline__ void color4_zune(const JpegGeom& g, int x0, int y, uint8_t* px) {
    const int fv = g.vmax / g.v[1];
    const int nY = g.bw[0] * 8, n = g.bw[1] * 8, ph = g.bh[1] * 8;
    const uint32_t yv = *reinterpret_cast<const uint32_t*>(g.planes + g.plane0[0] + (size_t)y * nY + x0);
    const int Y = fv == 2 ? y >> 1 : y;
    int r1 = fv == 2 ? ((y & 1) ? Y + 1 : Y - 1) : Y;
    r1 = r1 < 0 ? 0 : (r1 >= ph ? ph - 1 : r1);
    const uint32_t i = (uint32_t)x0 >> 1;  // samples i-1 .. i+2 of the chroma row
    int at[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const uint8_t* p = g.planes + g.plane0[1 + c];
        const uint32_t a = bytes4(p + (size_t)Y * n, i - 1), b = bytes4(p + (size_t)r1 * n, i - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int s0 = (int)((a >> (8 * k)) & 255u), s1 = (int)((b >> (8 * k)) & 255u);
            at[c][k] = fv == 2 ? (s0 * 3 + s1 + 2) >> 2 : s0;
        }
    }
    // pixel x0 + j: even -> (at(i') * 3 + at(i' - 1) + 2) >> 2, odd -> (at(i') * 3 + at(i' + 1) + 2) >> 2,
    // i' = (x0 + j) >> 1; at index k <-> sample i - 1 + k
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ip = 1 + (j >> 1), nb = (j & 1) ? ip + 1 : ip - 1;
        const int c0 = (int)((yv >> (8 * j)) & 255u);
        const int c1 = (at[0][ip] * 3 + at[0][nb] + 2) >> 2, c2 = (at[1][ip] * 3 + at[1][nb] + 2) >> 2;
        const int16_t cb = (int16_t)(c1 - 128), cr = (int16_t)(c2 - 128);
        const int r = c0 + ((int16_t)(45 * cr) >> 5);
        const int gg = c0 - ((int16_t)(11 * cb + 23 * cr) >> 5);
        const int b = c0 + ((int16_t)(113 * cb) >> 6);
        px[3 * j] = clamp255(r);
        px[3 * j + 1] = clamp255(gg);
        px[3 * j + 2] = clamp255(b);
    }
}

// one pixel of a zune_fast image anywhere in the row (color_pixel's zune YCbCr path
// without its other modes): the row ends, where color4_zune does not apply.  A
// wave holding a row-end thread otherwise ran all of color_pixel's branches.
__device__ __forceinline__ void color1_zune(const JpegGeom& g, int x, int y, uint8_t* o) {
    const int c0 = upsampled_zune(g, 0, x, y), c1 = upsampled_zune(g, 1, x, y), c2 = upsampled_zune(g, 2, x, y);
    const int16_t cb = (int16_t)(c1 - 128), cr = (int16_t)(c2 - 128);
    const int r = c0 + ((int16_t)(45 * cr) >> 5);
    const int gg = c0 - ((int16_t)(11 * cb + 23 * cr) >> 5);
    const int b = c0 + ((int16_t)(113 * cb) >> 6);
    o[0] = clamp255(r);
    o[1] = clamp255(gg);
    o[2] = clamp255(b);
}

__device__ __forceinline__ void color_group(const JpegGeom& g, uint8_t* __restrict__ dst, size_t pitch, int x0, int y,
                                            bool fast) {
    if (x0 >= g.W || y >= g.H) return;
    const int C = g.colorspace == 0 ? 1 : 3;
    uint8_t px[12];
    if (fast && x0 >= 4 && x0 + 4 <= g.W && x0 + 3 < 2 * g.bw[1] * 8 - 2) {
        color4_zune(g, x0, y, px);
        uint32_t w[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            w[i] = (uint32_t)px[4 * i] | (uint32_t)px[4 * i + 1] << 8 | (uint32_t)px[4 * i + 2] << 16 |
                   (uint32_t)px[4 * i + 3] << 24;
        uint32_t* o32 = reinterpret_cast<uint32_t*>(dst + (size_t)y * pitch + (size_t)3 * x0);
        o32[0] = w[0];
        o32[1] = w[1];
        o32[2] = w[2];
        return;
    }
    if (fast) return;  // a row end: k_jpeg_color_ends
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (x0 + k < g.W) color_pixel(g, x0 + k, y, px + C * k);
    uint8_t* o = dst + (size_t)y * pitch + (size_t)C * x0;
    if (x0 + 4 <= g.W) {
        uint32_t w[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            w[i] = (uint32_t)px[4 * i] | (uint32_t)px[4 * i + 1] << 8 | (uint32_t)px[4 * i + 2] << 16 |
                   (uint32_t)px[4 * i + 3] << 24;
        uint32_t* o32 = reinterpret_cast<uint32_t*>(o);
        o32[0] = w[0];
        if (C == 3) { o32[1] = w[1]; o32[2] = w[2]; }
        return;
    }
    for (int i = 0; i < C * (g.W - x0); ++i) o[i] = px[i];
}

__global__ __launch_bounds__(256) void k_jpeg_color(JpegGeom g, uint8_t* __restrict__ dst, size_t pitch) {
    color_group(g, dst, pitch, 4 * (blockIdx.x * 256 + threadIdx.x), blockIdx.y, zune_fast(g));
}
// the batch's images that are not zune_fast in one launch: blockIdx.z = image.
// (zune_fast comes from the host with the entry: tested here field by field it is a chain of dependent
// scalar loads per workgroup; the whole entry copied to registers instead costs
// ~100 SGPRs and half the waves)
// A workgroup takes kColorRows rows, so that each entry's fields are loaded once per
// eight rows of work, not once per row.
constexpr int kColorRows = 8;
__global__ __launch_bounds__(256) void k_jpeg_color_b(const JpegReconItem* __restrict__ items) {
    const JpegReconItem& it = items[blockIdx.z];  // (restrict: its loads hoist past the row stores)
    if (it.fast) return;  // k_jpeg_color_fast_b + k_jpeg_color_ends_b
    const int x0 = 4 * (blockIdx.x * 256 + threadIdx.x);
    for (int r = 0; r < kColorRows; ++r) color_group(it.g, it.dst, it.pitch, x0, blockIdx.y * kColorRows + r, false);
}

// The row ends of a zune_fast image (the groups of four k_jpeg_color leaves:
// x0 = 0, and from the first group that reaches the plane's last two chroma
// samples or the image's right edge), one thread per (row, end): kept out of
// k_jpeg_color, where a wave holding a row-end thread ran these branches for all
// of its lanes (50 vs 27 us per 4096^2 frame with them outside).
// G: the interior kernel's group width (4: k_jpeg_color, 8: k_jpeg_color_fast_b)
template <int G>
__device__ __forceinline__ void color_ends(const JpegGeom& g, uint8_t* __restrict__ dst, size_t pitch, int t) {
    if (t >= 2 * g.H) return;
    const int y = t >> 1;
    const int lim = 2 * g.bw[1] * 8 - 2;  // a group is interior iff x0 >= G, x0 + G <= W and x0 + G - 1 < lim
    // the first group past the interior ones: the last interior x0 is the largest
    // multiple of G <= min(W - G, lim - G)
    const int xm = (g.W - G < lim - G ? g.W - G : lim - G);
    const int xc = xm < G ? G : (xm & ~(G - 1)) + G;
    int xa, xb;
    if (t & 1) { xa = xc; xb = g.W; }
    else { xa = 0; xb = g.W < G ? g.W : G; }
    uint8_t* o = dst + (size_t)y * pitch;
    for (int x = xa; x < xb; ++x) color1_zune(g, x, y, o + 3 * x);
}

__global__ __launch_bounds__(256) void k_jpeg_color_ends(JpegGeom g, uint8_t* __restrict__ dst, size_t pitch) {
    color_ends<4>(g, dst, pitch, blockIdx.x * 256 + threadIdx.x);
}
constexpr int kFastPx = 8;  // k_jpeg_color_fast_b's pixels per thread
// one pixel of a zune_fast image with its vertical factor fv known: color1_zune
// (upsampled_zune's horizontal cases x = 0, 1, 2n-2, 2n-1 and the interior one)
// without the per-component factor divisions and the other modes' branches
__device__ __forceinline__ void color1_fast(const JpegGeom& g, int fv, int x, int y, uint8_t* o) {
    const int n = g.bw[1] * 8, ph = g.bh[1] * 8;
    const int c0 = g.planes[g.plane0[0] + (size_t)y * (g.bw[0] * 8) + x];
    const int Y = fv == 2 ? y >> 1 : y;
    int r1 = fv == 2 ? ((y & 1) ? Y + 1 : Y - 1) : Y;
    r1 = r1 < 0 ? 0 : (r1 >= ph ? ph - 1 : r1);
    int cc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const uint8_t* p0 = g.planes + g.plane0[1 + c] + (size_t)Y * n;
        const uint8_t* p1 = g.planes + g.plane0[1 + c] + (size_t)r1 * n;
        auto at = [&](int k) { return fv == 2 ? (p0[k] * 3 + p1[k] + 2) >> 2 : (int)p0[k]; };
        const int i = x >> 1;
        int v;
        if (x == 0) v = at(0);
        else if (x == 1) v = (at(0) * 3 + at(1) + 2) >> 2;
        else if (x == 2 * n - 2) v = (at(n - 2) * 3 + at(n - 1) + 2) >> 2;
        else if (x == 2 * n - 1) v = at(n - 1);
        else v = (x & 1) ? (at(i) * 3 + at(i + 1) + 2) >> 2 : (at(i) * 3 + at(i - 1) + 2) >> 2;
        cc[c] = v;
    }
    const int16_t cb = (int16_t)(cc[0] - 128), cr = (int16_t)(cc[1] - 128);
    o[0] = clamp255(c0 + ((int16_t)(45 * cr) >> 5));
    o[1] = clamp255(c0 - ((int16_t)(11 * cb + 23 * cr) >> 5));
    o[2] = clamp255(c0 + ((int16_t)(113 * cb) >> 6));
}

// the batch's zune_fast images in one launch: blockIdx.y = image (the others
// return).  One thread per end pixel: slots 0 .. 15 of a row are its left end
// [0, min(W, 8)), slots 16 .. 31 its right end [xc, W) (at most 9 pixels unless
// W < 16; slot 31 takes any past xc + 16)
__global__ __launch_bounds__(256) void k_jpeg_color_ends_b(const JpegReconItem* __restrict__ items) {
    const JpegReconItem& it = items[blockIdx.y];
    if (!it.fast) return;
    const JpegGeom& g = it.g;
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int y = t >> 5, k = t & 31;
    if (y >= g.H) return;
    uint8_t* o = it.dst + (size_t)y * it.pitch;
    const int fv = g.vmax == 2 * g.v[1] ? 2 : 1;
    if (k < 16) {
        if (k < kFastPx && k < g.W) color1_fast(g, fv, k, y, o + 3 * k);
        return;
    }
    const int xc = fast_xc(g);
    const int x = xc + (k - 16);
    if (k < 31) {
        if (x < g.W) color1_fast(g, fv, x, y, o + 3 * x);
        return;
    }
    for (int xx = x; xx < g.W; ++xx) color1_fast(g, fv, xx, y, o + 3 * xx);
}

// ---- the batch's zune_fast images: eight pixels by kFastRows rows per thread ----
// k_jpeg_color_b's per-pixel path re-derived the geometry per row (a scalar
// division for the vertical factor), loaded through generic pointers and waited
// on every load in turn: 7.9 ms per 256 4096^2 frames, about a third of HBM
// speed.  Here a thread keeps its column's three chroma rows (above, this,
// below) of both planes in registers and walks down its rows: per output row one
// 8-byte luma load, per chroma row one 12-byte load per plane (bytes i-4 .. i+7,
// i = x0 / 2: the samples i-1 .. i+4 the eight pixels use), and two 12-byte
// stores.  The arithmetic is color4_zune's (upsampler/scalar.rs vertical then
// horizontal (3 near + far + 2) >> 2, color_convert/scalar.rs i16 YCbCr).
constexpr int kFastRowsT = 16;  // rows per thread (two luma blocks)
typedef __attribute__((address_space(1))) uint8_t g8;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ uint32_t pack_px(int v) { return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// one output row's eight pixels: yv = luma bytes x0 .. x0+7; s[c] / t[c]: plane
// c's chroma row (near) and its vertical neighbour (far), bytes i-4 .. i+7
template <int FV>
__device__ __forceinline__ void color8_row(u32x2 yv, const u32x3 (&s)[2], const u32x3 (&t)[2], g8* __restrict__ o) {
    int at[2][6];  // the vertically upsampled samples i-1 .. i+4
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int b = 3 + k;  // byte of the 12 (i-4 .. i+7)
            const uint32_t ws = b < 4 ? s[c].x : b < 8 ? s[c].y : s[c].z;
            const int s0 = (int)((ws >> (8 * (b & 3))) & 255u);
            if (FV == 2) {
                const uint32_t wt = b < 4 ? t[c].x : b < 8 ? t[c].y : t[c].z;
                const int s1 = (int)((wt >> (8 * (b & 3))) & 255u);
                at[c][k] = (s0 * 3 + s1 + 2) >> 2;
            } else {
                at[c][k] = s0;
            }
        }
    }
    uint32_t px[8];  // 0x00BBGGRR per pixel
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int ip = 1 + (j >> 1), nb = (j & 1) ? ip + 1 : ip - 1;
        const int c0 = (int)(((j < 4 ? yv.x : yv.y) >> (8 * (j & 3))) & 255u);
        const int c1 = (at[0][ip] * 3 + at[0][nb] + 2) >> 2, c2 = (at[1][ip] * 3 + at[1][nb] + 2) >> 2;
        const int16_t cb = (int16_t)(c1 - 128), cr = (int16_t)(c2 - 128);
        const int r = c0 + ((int16_t)(45 * cr) >> 5);
        const int gg = c0 - ((int16_t)(11 * cb + 23 * cr) >> 5);
        const int b = c0 + ((int16_t)(113 * cb) >> 6);
        px[j] = pack_px(r) | pack_px(gg) << 8 | pack_px(b) << 16;
    }
    // 24 bytes R0 G0 B0 R1 G1 B1 ... as six dwords
    u32x3 lo, hi;
    lo.x = px[0] | px[1] << 24;
    lo.y = px[1] >> 8 | px[2] << 16;
    lo.z = px[2] >> 16 | px[3] << 8;
    hi.x = px[4] | px[5] << 24;
    hi.y = px[5] >> 8 | px[6] << 16;
    hi.z = px[6] >> 16 | px[7] << 8;
    *reinterpret_cast<u32x3 __attribute__((address_space(1)))*>(o) = lo;
    *reinterpret_cast<u32x3 __attribute__((address_space(1)))*>(o + 12) = hi;
}

// the luma IDCT's rows into registers (k_jpeg_color_fast_b with LI): idct_zune's
// row stores through this sink land in v[2 r], v[2 r + 1] (constant indices once
// unrolled, so the block stays in VGPRs)
struct RegRow {
    uint32_t* v;
};
struct RegSink {
    uint32_t* v;
    __device__ RegRow operator+(size_t off) const { return RegRow{v + 2 * (off >> 3)}; }
};
__device__ __forceinline__ void store8(RegRow p, uint32_t lo, uint32_t hi) {
    p.v[0] = lo;
    p.v[1] = hi;
}

// luma block (bx, by) of g: dequantised and through zune's IDCT into yr[0..15]
__device__ __forceinline__ void luma_idct(const JpegGeom& g, int bx, int by, uint32_t (&yr)[16]) {
    const long long blk = g.blk0[0] + (long long)by * g.bw[0] + bx;
    const int4* cp = reinterpret_cast<const int4*>(g.coef + blk * 64);
    const __attribute__((address_space(4))) uint16_t* q = (const __attribute__((address_space(4))) uint16_t*)g.qt;
    int in[64];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int4 v = cp[i];
        const int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = i * 8 + 2 * j;
            in[k] = (int)(int16_t)(w[j] & 0xffff) * (int)q[k];
            in[k + 1] = (int)(int16_t)((unsigned)w[j] >> 16) * (int)q[k + 1];
        }
    }
    idct_zune(in, RegSink{yr}, 8);
}

// LI: the luma rows come from the thread's own IDCT of its two luma blocks (8 x 16
// pixels = blocks (x0/8, y0/8) and (x0/8, y0/8 + 1)) instead of the luma plane:
// k_jpeg_idct_b leaves those blocks to this kernel, and the plane's write and read
// (a third of the reconstruction's bytes) are not made
template <int FV, bool LI>
__device__ __forceinline__ void color_fast_rows(const JpegGeom& g, g8* __restrict__ dst, size_t pitch, int x0, int y0,
                                                int y1) {
    const int nY = g.bw[0] * 8, n = g.bw[1] * 8, ph = g.bh[1] * 8;
    const g8* yp = (const g8*)g.planes + g.plane0[0] + x0;
    const g8* cp[2] = {(const g8*)g.planes + g.plane0[1] + (x0 >> 1) - 4,
                       (const g8*)g.planes + g.plane0[2] + (x0 >> 1) - 4};
    auto ldc = [&](int c, int r) -> u32x3 {
        r = r < 0 ? 0 : (r >= ph ? ph - 1 : r);
        return *reinterpret_cast<const u32x3 __attribute__((address_space(1)))*>(cp[c] + (size_t)r * n);
    };
    uint32_t yr[2][16];
    if (LI) {
        luma_idct(g, x0 >> 3, y0 >> 3, yr[0]);
        if (y0 + 8 < y1) luma_idct(g, x0 >> 3, (y0 >> 3) + 1, yr[1]);
    }
    // row rr (0 .. 15) of the thread's band: registers (LI, rr constant once unrolled) or the plane
    auto ldy = [&](int rr) -> u32x2 {
        if (LI) return u32x2{yr[rr >> 3][2 * (rr & 7)], yr[rr >> 3][2 * (rr & 7) + 1]};
        return *reinterpret_cast<const u32x2 __attribute__((address_space(1)))*>(yp + (size_t)(y0 + rr) * nY);
    };
    g8* o = dst + (size_t)y0 * pitch + (size_t)3 * x0;
    if (FV == 2) {
        // y0 even: rows 2Y and 2Y+1 share chroma row Y (far rows Y-1 and Y+1)
        int Y = y0 >> 1;
        u32x3 up[2] = {ldc(0, Y - 1), ldc(1, Y - 1)}, mid[2] = {ldc(0, Y), ldc(1, Y)};
#pragma unroll
        for (int rr = 0; rr < kFastRowsT; rr += 2, ++Y) {
            if (y0 + rr >= y1) break;
            const u32x3 dn[2] = {ldc(0, Y + 1), ldc(1, Y + 1)};
            color8_row<2>(ldy(rr), mid, up, o);
            o += pitch;
            if (y0 + rr + 1 < y1) color8_row<2>(ldy(rr + 1), mid, dn, o);
            o += pitch;
            up[0] = mid[0]; up[1] = mid[1];
            mid[0] = dn[0]; mid[1] = dn[1];
        }
    } else {
#pragma unroll
        for (int rr = 0; rr < kFastRowsT; ++rr) {
            if (y0 + rr >= y1) break;
            const u32x3 c[2] = {ldc(0, y0 + rr), ldc(1, y0 + rr)};
            color8_row<1>(ldy(rr), c, c, o);
            o += pitch;
        }
    }
}

// grid: (column groups of 8 x 256, row bands of kFastRows, image); the interior
// groups only (x0 >= 8, x0 + 8 <= W, x0 + 7 < 2n - 2), k_jpeg_color_ends_b the rest
constexpr int kFastRows = kFastRowsT;
template <bool LI>
__global__ __launch_bounds__(256) void k_jpeg_color_fast_b(const JpegReconItem* __restrict__ items) {
    const JpegReconItem& it = items[blockIdx.z];
    if (!it.fast) return;
    const JpegGeom& g = it.g;
    const int x0 = kFastPx * (blockIdx.x * 256 + threadIdx.x);
    const int y0 = blockIdx.y * kFastRows;
    if (y0 >= g.H || x0 < kFastPx || x0 + kFastPx > g.W || x0 + kFastPx - 1 >= 2 * g.bw[1] * 8 - 2) return;
    const int y1 = y0 + kFastRows < g.H ? y0 + kFastRows : g.H;
    g8* dst = (g8*)it.dst;
    if (g.vmax == 2 * g.v[1]) color_fast_rows<2, LI>(g, dst, it.pitch, x0, y0, y1);
    else color_fast_rows<1, LI>(g, dst, it.pitch, x0, y0, y1);
}

}  // namespace

// ---- baseline Huffman decoding, one thread per restart interval ---------------
// A restart interval is self-contained: the DC predictors reset and the bit
// stream realigns at its RSTn marker, so the host only has to find the markers
// (a byte scan) and each lane decodes its interval's MCUs into the dense
// coefficient image with the same rules as the host decoder (ITU T.81 F.2.2,
// libjpeg jdhuff.c): byte-stuffed 0xFF 0x00, zeros fed past a marker, 9-bit
// lookahead then the canonical maxcode walk.  Tables live in LDS.
namespace {

constexpr int kHuffThreads = 64;

__device__ const uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Bit reader over a per-lane LDS ring of the scan bytes.  Global memory is only
// touched in 64-byte chunks (16 independent dword loads); at every block start
// all lanes of the wave top their rings up together (a wave vote), so the wave
// waits for memory once per many blocks instead of once per symbol.
constexpr int kRingDw = 64;  // 256 bytes per lane

struct GpuBits {
    const __attribute__((address_space(1))) uint32_t* g;  // the scan bytes as dwords (256-B aligned base, padded past the end)
    uint32_t* ring;     // this lane's ring
    uint32_t pos, fetched, size;  // next byte, ring filled up to (multiple of 4), scan end
    unsigned long long acc;
    int n;
    bool marker;
    __device__ void chunk() {
        uint32_t v[16];
        const uint32_t d0 = fetched >> 2;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = g[d0 + i];
#pragma unroll
        for (int i = 0; i < 16; ++i) ring[(d0 + i) & (kRingDw - 1)] = v[i];
        fetched += 64;
    }
    __device__ void top_up() {  // uniform point: every lane ends with >= 128 bytes ahead
        while (__any((int)(fetched - pos) < 128))  // signed: the ring starts at pos rounded down
            if ((int)(fetched - pos) < 128) chunk();
    }
    __device__ uint32_t byte_at(uint32_t o) const { return (ring[(o >> 2) & (kRingDw - 1)] >> ((o & 3) * 8)) & 0xffu; }
    __device__ void fill() {  // called with n < 16
        // four bytes at once when none of them is 0xFF (no stuffing, no marker):
        // entropy-coded data holds an 0xFF in about 1 of 256 bytes
        if (!marker && pos + 4 <= size && (int)(fetched - pos) >= 4) {
            const uint32_t w0 = ring[(pos >> 2) & (kRingDw - 1)], w1 = ring[((pos >> 2) + 1) & (kRingDw - 1)];
            const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, pos & 3u);  // bytes pos .. pos+3, little-endian
            const uint32_t nx = ~x;
            if (!((nx - 0x01010101u) & ~nx & 0x80808080u)) {
                acc |= (unsigned long long)__builtin_bswap32(x) << (32 - n);
                n += 32;
                pos += 4;
                return;
            }
        }
        while (n <= 56) {
            uint32_t v = 0;
            if (!marker && pos < size) {
                if ((int)(fetched - pos) < 2) chunk();  // a block longer than the lookahead (rare)
                v = byte_at(pos);
                if (v == 0xFF) {
                    const uint32_t nx = pos + 1 < size ? byte_at(pos + 1) : 0;  // 0 past the end, as on the host
                    if (nx == 0) pos += 2;
                    else { marker = true; v = 0; }
                } else {
                    ++pos;
                }
            }
            acc |= (unsigned long long)v << (56 - n);
            n += 8;
        }
    }
    __device__ int peek(int k) {
        if (n < k) fill();
        return (int)(acc >> (64 - k));
    }
    __device__ void skip(int k) { acc <<= k; n -= k; }
    __device__ int get(int k) {
        if (!k) return 0;
        const int v = peek(k);
        skip(k);
        return v;
    }
};

__device__ __forceinline__ int extend_dev(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

__device__ int decode_sym(GpuBits& br, const JpegHuffTables& T, int t) {
    const int look = br.peek(9);
    const int lv = T.look[t][look];
    if (lv >> 8) {
        br.skip(lv >> 8);
        return lv & 0xff;
    }
    // longer codes: the length is 10 + the number of left-justified bounds the
    // 16-bit window reaches (canonical codes; one round of LDS reads, no loop)
    const int code = br.peek(16);
    int len = 10;
#pragma unroll
    for (int l = 10; l <= 16; ++l) len += code >= T.lj[t][l];
    if (len > 16) return -1;
    br.skip(len);
    const int c = code >> (16 - len);
    return T.vals[t][T.valptr[t][len] + c - T.mincode[t][len]];
}

}  // namespace

__device__ __forceinline__ void load_tables(const JpegHuffTables* g, JpegHuffTables& T, uint8_t* s_zz) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&T);
    for (int i = threadIdx.x; i < (int)(sizeof(JpegHuffTables) / 4); i += kHuffThreads) dst[i] = src[i];
    if (threadIdx.x < 64) s_zz[threadIdx.x] = kZz[threadIdx.x];
}

// ---- progressive scans with restart intervals ----------------------------------
// One lane per restart interval of one scan (ITU T.81 G.1.2; the host decoder's
// block_dc_first / block_dc_refine / block_ac_first / block_ac_refine, libjpeg
// jdphuff.c): the interval's DC predictions and EOB run start at zero, so the
// intervals are independent; a refinement scan reads the coefficients the scans
// before it wrote, which the stream order of the launches guarantees.
__device__ void prog_interval(const JpegScanArgs& a, const JpegHuffTables& T, const uint8_t* s_zz, uint32_t* ring,
                              int seg) {
    GpuBits br;
    br.g = (const __attribute__((address_space(1))) uint32_t*)a.data;
    br.ring = ring;
    br.pos = a.seg[seg];
    br.fetched = br.pos & ~3u;
    br.size = (uint32_t)a.size;
    br.acc = 0;
    br.n = 0;
    br.marker = false;
    int pred[4] = {0, 0, 0, 0};
    int eobrun = 0;
    const int kind = a.kind, Ss = a.Ss, Se = a.Se, Al = a.Al;
    const int p1 = 1 << Al, m1 = -p1;
    const long long m0 = (long long)seg * a.restart;
    const int nm = (int)min((long long)a.restart, a.total_mcu - m0);
    const int row_len = a.single ? a.single_bw : a.mcux;
    int mx = (int)(m0 % row_len), my = (int)(m0 / row_len);
    for (int i = 0; i < nm; ++i) {
        for (int ci = 0; ci < a.ns; ++ci) {
            const int nby = a.single ? 1 : a.v[ci], nbx = a.single ? 1 : a.h[ci];
            for (int by = 0; by < nby; ++by)
                for (int bx = 0; bx < nbx; ++bx) {
                    const long long bi = a.single ? a.blk0[ci] + (long long)my * a.bw[ci] + mx
                                                  : a.blk0[ci] + (long long)(my * a.v[ci] + by) * a.bw[ci] + mx * a.h[ci] + bx;
                    int16_t* blk = a.coef + bi * 64;
                    br.top_up();
                    if (kind == 1) {  // DC first
                        const int t = decode_sym(br, T, a.td[ci]);
                        if (t < 0 || t > 11) { atomicOr(a.err, 1); return; }
                        pred[ci] += t ? extend_dev(br.get(t), t) : 0;
                        blk[0] = (int16_t)(pred[ci] * p1);
                    } else if (kind == 2) {  // DC refine
                        if (br.get(1)) blk[0] = (int16_t)(blk[0] | p1);
                    } else if (kind == 3) {  // AC first
                        if (eobrun > 0) { --eobrun; continue; }
                        for (int k = Ss; k <= Se; ++k) {
                            const int rs = decode_sym(br, T, 4 + a.ta[ci]);
                            if (rs < 0) { atomicOr(a.err, 2); return; }
                            const int r = rs >> 4, sz = rs & 15;
                            if (sz) {
                                k += r;
                                if (k > Se) { atomicOr(a.err, 4); return; }
                                blk[s_zz[k]] = (int16_t)(extend_dev(br.get(sz), sz) * p1);
                            } else if (r == 15) {
                                k += 15;
                            } else {
                                eobrun = (1 << r) + (r ? br.get(r) : 0) - 1;
                                break;
                            }
                        }
                    } else {  // AC refine
                        int k = Ss;
                        if (eobrun == 0) {
                            for (; k <= Se; ++k) {
                                const int rs = decode_sym(br, T, 4 + a.ta[ci]);
                                if (rs < 0) { atomicOr(a.err, 2); return; }
                                int r = rs >> 4, val = 0;
                                const int sz = rs & 15;
                                if (sz) {
                                    if (sz != 1) { atomicOr(a.err, 8); return; }
                                    val = br.get(1) ? p1 : m1;
                                } else if (r != 15) {
                                    eobrun = (1 << r) + (r ? br.get(r) : 0);
                                    break;  // the rest of the band: the EOB-run pass below
                                }
                                // skip r zero-history coefficients, refining the nonzero ones passed
                                do {
                                    int16_t* co = blk + s_zz[k];
                                    if (*co != 0) {
                                        if (br.get(1) && (*co & p1) == 0) *co = (int16_t)(*co >= 0 ? *co + p1 : *co + m1);
                                    } else if (--r < 0) {
                                        break;
                                    }
                                    ++k;
                                } while (k <= Se);
                                if (val) {
                                    if (k > Se) { atomicOr(a.err, 4); return; }
                                    blk[s_zz[k]] = (int16_t)val;
                                }
                            }
                        }
                        if (eobrun > 0) {
                            for (; k <= Se; ++k) {
                                int16_t* co = blk + s_zz[k];
                                if (*co != 0 && br.get(1) && (*co & p1) == 0) *co = (int16_t)(*co >= 0 ? *co + p1 : *co + m1);
                            }
                            --eobrun;
                        }
                    }
                }
        }
        if (++mx == row_len) { mx = 0; ++my; }
    }
}

__global__ __launch_bounds__(kHuffThreads) void k_jpeg_prog(JpegScanArgs a) {
    __shared__ JpegHuffTables T;
    __shared__ uint8_t s_zz[64];
    extern __shared__ uint32_t s_rings[];  // a.lanes rings of kRingDw + 1 dwords
    load_tables(a.tabs, T, s_zz);
    __syncthreads();
    const int seg = blockIdx.x * a.lanes + threadIdx.x;
    if ((int)threadIdx.x < a.lanes && seg < a.n_seg) prog_interval(a, T, s_zz, s_rings + threadIdx.x * (kRingDw + 1), seg);
}

namespace {
int huff_lanes(int v) { return v < 1 ? 1 : (v > kHuffThreads ? kHuffThreads : v); }
}  // namespace

int jpeg_lanes_for(long long total) {
    int want = 1;
    while (want < 32 && (long long)want * 2 * 1024 <= total) want *= 2;
    return huff_lanes(want);
}

hipError_t launch_jpeg_prog(const JpegScanArgs& a, hipStream_t s) {
    if (a.n_seg <= 0 || a.restart <= 0 || a.ns < 1 || a.ns > 4 || a.kind < 1 || a.kind > 4 || a.Ss < 0 || a.Se > 63 ||
        a.Al > 13)
        return hipErrorInvalidValue;
    JpegScanArgs b = a;
    b.lanes = jpeg_lanes_for(a.n_seg);
    hipLaunchKernelGGL(k_jpeg_prog, dim3((a.n_seg + b.lanes - 1) / b.lanes), dim3(kHuffThreads),
                       sizeof(uint32_t) * (kRingDw + 1) * b.lanes, s, b);
    return hipGetLastError();
}

// the reconstruction of a batch's images, three launches for all of them (items:
// device array of m; maxima over the images: blocks, width, height; idct: false
// when the sample planes are already there)
hipError_t launch_jpeg_reconstruct_batch(const JpegReconItem* items, int m, long long max_blocks, int max_w, int max_h,
                                         bool any_fast, bool any_slow, bool idct, hipStream_t s) {
    if (m <= 0) return hipSuccess;
    if (max_blocks <= 0 || max_w <= 0 || max_h <= 0 || m > 65535 || max_h > 65535) return hipErrorInvalidValue;
    if (idct) hipLaunchKernelGGL(k_jpeg_idct_b, dim3((unsigned)((max_blocks + 255) / 256), m), dim3(256), 0, s, items);
    if (any_slow)
        hipLaunchKernelGGL(k_jpeg_color_b, dim3((max_w + 1023) / 1024, (max_h + kColorRows - 1) / kColorRows, m),
                           dim3(256), 0, s, items);
    if (any_fast) {
        const dim3 gf((max_w + 256 * kFastPx - 1) / (256 * kFastPx), (max_h + kFastRows - 1) / kFastRows, m);
        if (idct) hipLaunchKernelGGL(k_jpeg_color_fast_b<true>, gf, dim3(256), 0, s, items);
        else hipLaunchKernelGGL(k_jpeg_color_fast_b<false>, gf, dim3(256), 0, s, items);
        hipLaunchKernelGGL(k_jpeg_color_ends_b, dim3((32 * max_h + 255) / 256, m), dim3(256), 0, s, items);
    }
    return hipGetLastError();
}
bool jpeg_zune_fast(const JpegGeom& g) { return zune_fast(g); }

hipError_t launch_jpeg_reconstruct(const JpegGeom& g, uint8_t* dst, size_t dst_pitch, hipStream_t s) {
    if (g.nblocks <= 0 || g.W <= 0 || g.H <= 0) return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((g.nblocks + 255) / 256);
    hipLaunchKernelGGL(k_jpeg_idct, dim3(nb), dim3(256), 0, s, g);
    hipLaunchKernelGGL(k_jpeg_color, dim3((g.W + 1023) / 1024, g.H), dim3(256), 0, s, g, dst, dst_pitch);
    if (zune_fast(g))
        hipLaunchKernelGGL(k_jpeg_color_ends, dim3((2 * g.H + 255) / 256), dim3(256), 0, s, g, dst, dst_pitch);
    return hipGetLastError();
}

}  // namespace ik
