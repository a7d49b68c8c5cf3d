// ik_jpeg.hip -- gfx950 kernels of decode_image's JPEG reconstruction (reference
// src/transform.rs:31 -> image 0.25.8 -> zune-jpeg 0.4.21), fed by the host
// entropy decoder in ik_jpeg_decode.cpp:
//
//   k_jpeg_idct   one lane per 8x8 block: dequantise (coef * qt) and the libjpeg
//                 jidctint.c "islow" 2-D IDCT with its descale/range-limit, into the
//                 component's u8 sample plane.
//   k_jpeg_color  one lane per output pixel: libjpeg(-turbo) "fancy" chroma
//                 upsampling (h2v1 / h2v2 / h1v2 triangle filters with replicated
//                 edge context, integer replication otherwise) and jdcolor.c's
//                 fixed-point YCbCr->RGB, written into the device image.
//
// All integer arithmetic; results equal libjpeg-turbo's decoder (Pillow) bit for
// bit on the tests' streams (tests/test_gpu_decode.py).
#include "ik_internal.h"

namespace ik {

namespace {

constexpr int kCB = 13;  // CONST_BITS
constexpr int kP1 = 2;   // PASS1_BITS

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
__device__ __forceinline__ uint8_t range_limit(int x) {
    x += 128;
    return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x));
}

// jpeg_idct_islow's odd/even butterfly on eight inputs (a column or a row)
struct Idct8 {
    int o0, o1, o2, o3, o4, o5, o6, o7;  // pre-descale outputs
};
__device__ __forceinline__ Idct8 idct8(int i0, int i1, int i2, int i3, int i4, int i5, int i6, int i7) {
    int z2 = i2, z3 = i6;
    int z1 = (z2 + z3) * 4433;
    int tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
    int tmp0 = (i0 + i4) * (1 << kCB), tmp1 = (i0 - i4) * (1 << kCB);
    const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = i7; tmp1 = i5; tmp2 = i3; tmp3 = i1;
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * 9633;
    tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    return {t10 + tmp3, t11 + tmp2, t12 + tmp1, t13 + tmp0, t13 - tmp0, t12 - tmp1, t11 - tmp2, t10 - tmp3};
}

__global__ __launch_bounds__(256) void k_jpeg_idct(JpegGeom g) {
    const long long blk = (long long)blockIdx.x * 256 + threadIdx.x;
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
    // pass 1: columns -> ws (scaled by 2^PASS1_BITS)
    int ws[64];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (!in[8 + c] && !in[16 + c] && !in[24 + c] && !in[32 + c] && !in[40 + c] && !in[48 + c] &&
            !in[56 + c]) {
            const int dc = in[c] * (1 << kP1);
#pragma unroll
            for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
            continue;
        }
        const Idct8 o = idct8(in[c], in[8 + c], in[16 + c], in[24 + c], in[32 + c], in[40 + c], in[48 + c],
                              in[56 + c]);
        ws[0 * 8 + c] = descale(o.o0, kCB - kP1); ws[1 * 8 + c] = descale(o.o1, kCB - kP1);
        ws[2 * 8 + c] = descale(o.o2, kCB - kP1); ws[3 * 8 + c] = descale(o.o3, kCB - kP1);
        ws[4 * 8 + c] = descale(o.o4, kCB - kP1); ws[5 * 8 + c] = descale(o.o5, kCB - kP1);
        ws[6 * 8 + c] = descale(o.o6, kCB - kP1); ws[7 * 8 + c] = descale(o.o7, kCB - kP1);
    }
    // pass 2: rows -> samples
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int* w = ws + r * 8;
        uint8_t o[8];
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t dc = range_limit(descale(w[0], kP1 + 3));
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = dc;
        } else {
            // the even part's (w0 +- w4) << CONST_BITS is taken before the descale
            const Idct8 t = idct8(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
            constexpr int sh = kCB + kP1 + 3;
            o[0] = range_limit(descale(t.o0, sh)); o[1] = range_limit(descale(t.o1, sh));
            o[2] = range_limit(descale(t.o2, sh)); o[3] = range_limit(descale(t.o3, sh));
            o[4] = range_limit(descale(t.o4, sh)); o[5] = range_limit(descale(t.o5, sh));
            o[6] = range_limit(descale(t.o6, sh)); o[7] = range_limit(descale(t.o7, sh));
        }
        const unsigned lo = o[0] | (o[1] << 8) | (o[2] << 16) | ((unsigned)o[3] << 24);
        const unsigned hi = o[4] | (o[5] << 8) | (o[6] << 16) | ((unsigned)o[7] << 24);
        *reinterpret_cast<uint2*>(out + (size_t)r * pw) = make_uint2(lo, hi);  // 8-B aligned
    }
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

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

__global__ __launch_bounds__(256) void k_jpeg_color(JpegGeom g, uint8_t* __restrict__ dst, size_t pitch) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= g.W) return;
    uint8_t* o = dst + (size_t)y * pitch;
    if (g.colorspace == 0) {
        o[x] = (uint8_t)upsampled(g, 0, x, y);
        return;
    }
    const int c0 = upsampled(g, 0, x, y), c1 = upsampled(g, 1, x, y), c2 = upsampled(g, 2, x, y);
    uint8_t r, gg, b;
    if (g.colorspace == 2) {
        r = (uint8_t)c0; gg = (uint8_t)c1; b = (uint8_t)c2;
    } else {
        // jdcolor.c ycc_rgb_convert, SCALEBITS 16: FIX(1.402) 91881, FIX(1.772) 116130,
        // FIX(0.71414) 46802, FIX(0.34414) 22554
        const int cb = c1 - 128, cr = c2 - 128;
        r = clamp255(c0 + ((91881 * cr + 32768) >> 16));
        gg = clamp255(c0 + ((-22554 * cb + 32768 - 46802 * cr) >> 16));
        b = clamp255(c0 + ((116130 * cb + 32768) >> 16));
    }
    o[3 * x] = r;
    o[3 * x + 1] = gg;
    o[3 * x + 2] = b;
}

}  // namespace

hipError_t launch_jpeg_reconstruct(const JpegGeom& g, uint8_t* dst, size_t dst_pitch, hipStream_t s) {
    if (g.nblocks <= 0 || g.W <= 0 || g.H <= 0) return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((g.nblocks + 255) / 256);
    hipLaunchKernelGGL(k_jpeg_idct, dim3(nb), dim3(256), 0, s, g);
    hipLaunchKernelGGL(k_jpeg_color, dim3((g.W + 255) / 256, g.H), dim3(256), 0, s, g, dst, dst_pitch);
    return hipGetLastError();
}

}  // namespace ik
