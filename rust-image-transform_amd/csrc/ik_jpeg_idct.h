// ik_jpeg_idct.h -- the two reconstructions' 8x8 inverse DCTs on dequantised
// coefficients, shared by the reconstruction kernels (ik_jpeg.hip k_jpeg_idct*)
// and the self-synchronising decoder's decode pass (ik_jsync.hip), which runs
// them as it decodes each block.
//   zune-jpeg 0.4.21 idct/scalar.rs idct_int (stb_image-derived fixed point; a
//   block with 63 zero AC coefficients takes clamp((dc >> 3) + 128));
//   libjpeg-turbo jidctint.c jpeg_idct_islow.
// Out: a generic or a global-address-space byte pointer (the latter keeps the
// row stores out of the LDS counter in kernels that also read LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ik {
namespace jidct {

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

// zune-jpeg idct_int's butterfly (stb_image stbi__idct_block constants, f2f =
// (int)(x * 4096 + 0.5)): even part x[0..3] (+ bias), odd part t[0..3]
__device__ __forceinline__ void zune8(int i0, int i1, int i2, int i3, int i4, int i5, int i6, int i7, int bias,
                                      int (&x)[4], int (&t)[4]) {
    int p2 = i2, p3 = i6;
    int p1 = (p2 + p3) * 2217;
    int t2 = p1 + p3 * -7567, t3 = p1 + p2 * 3135;
    int t0 = (i0 + i4) * 4096, t1 = (i0 - i4) * 4096;
    x[0] = t0 + t3 + bias; x[3] = t0 - t3 + bias; x[1] = t1 + t2 + bias; x[2] = t1 - t2 + bias;
    t0 = i7; t1 = i5; t2 = i3; t3 = i1;
    p3 = t0 + t2;
    int p4 = t1 + t3;
    p1 = t0 + t3;
    p2 = t1 + t2;
    const int p5 = (p3 + p4) * 4816;
    t0 *= 1223; t1 *= 8410; t2 *= 12586; t3 *= 6149;
    p1 = p5 + p1 * -3685; p2 = p5 + p2 * -10497; p3 *= -8034; p4 *= -1597;
    t3 += p1 + p4; t2 += p2 + p3; t1 += p2 + p4; t0 += p1 + p3;
    t[0] = t0; t[1] = t1; t[2] = t2; t[3] = t3;
}

__device__ __forceinline__ uint8_t clamp_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// (x >> 17) clamped to 0..255, as a u32.  The empty asm keeps the shift and the
// clamp apart: otherwise the compiler fuses pairs of them into gfx950's
// v_ashr_pk_u8_i32 (16-bit result) and ORs the next two bytes into the same
// register as if its upper half were zero -- measured on MI355X: bytes 2 and 3 of
// every packed word came out corrupted.
__device__ __forceinline__ uint32_t sat17(int x) {
    int v = x >> 17;
    asm volatile("" : "+v"(v));
    return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// zune-jpeg 0.4.21 idct/scalar.rs idct_int on dequantised coefficients
__device__ __forceinline__ void store8(uint8_t* p, uint32_t lo, uint32_t hi) {
    *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}
__device__ __forceinline__ void store8(__attribute__((address_space(1))) uint8_t* p, uint32_t lo, uint32_t hi) {
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    *(__attribute__((address_space(1))) u2v*)p = u2v{lo, hi};
}

template <typename Out>
__device__ __forceinline__ void idct_zune(const int (&in)[64], Out out, int pw) {
    int ac = 0;
#pragma unroll
    for (int k = 1; k < 64; ++k) ac |= in[k];
    if (!ac) {  // "the array has 63 zeroes": (dc >> 3) + 128 everywhere
        const uint32_t v = clamp_u8((in[0] >> 3) + 128) * 0x01010101u;
#pragma unroll
        for (int r = 0; r < 8; ++r) store8(out + (size_t)r * pw, v, v);
        return;
    }
    int ws[64];
    int x[4], t[4];
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // vertical pass, 2 extra bits kept
        zune8(in[c], in[8 + c], in[16 + c], in[24 + c], in[32 + c], in[40 + c], in[48 + c], in[56 + c], 512, x, t);
        ws[c] = (x[0] + t[3]) >> 10; ws[8 + c] = (x[1] + t[2]) >> 10;
        ws[16 + c] = (x[2] + t[1]) >> 10; ws[24 + c] = (x[3] + t[0]) >> 10;
        ws[32 + c] = (x[3] - t[0]) >> 10; ws[40 + c] = (x[2] - t[1]) >> 10;
        ws[48 + c] = (x[1] - t[2]) >> 10; ws[56 + c] = (x[0] - t[3]) >> 10;
    }
    constexpr int kScale = 512 + 65536 + (128 << 17);  // SCALE_BITS: rounding + the +128 level shift
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int* w = ws + r * 8;
        zune8(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], kScale, x, t);
        const unsigned lo = sat17(x[0] + t[3]) | (sat17(x[1] + t[2]) << 8) | (sat17(x[2] + t[1]) << 16) |
                            (sat17(x[3] + t[0]) << 24);
        const unsigned hi = sat17(x[3] - t[0]) | (sat17(x[2] - t[1]) << 8) | (sat17(x[1] - t[2]) << 16) |
                            (sat17(x[0] - t[3]) << 24);
        store8(out + (size_t)r * pw, lo, hi);
    }
}

// libjpeg-turbo jidctint.c jpeg_idct_islow on dequantised coefficients
template <typename Out>
__device__ __forceinline__ void idct_islow(const int (&in)[64], Out out, int pw) {
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
        store8(out + (size_t)r * pw, lo, hi);  // 8-B aligned
    }
}


}  // namespace jidct
}  // namespace ik
