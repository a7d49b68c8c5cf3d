// ik_unfilter.h -- PNG row filters (png 0.18 unfilter: Sub / Up / Average / Paeth,
// reference src/transform.rs:31 -> image 0.25.8 -> png) on a 32-bit word of four
// bytes at once, for pixels of 4 or 8 bytes (RGBA8, RGBA16 / Rgb16-free layouts):
// there the byte `bpp` back of every byte of a word lies in one earlier word, so
// the word is one step of the left-to-right chain instead of four.  The bytes
// are split into two words of 16-bit lanes (bytes 0, 2 and bytes 1, 3), where the
// Paeth arithmetic (differences up to +-510) fits; on the GPU each half is a few
// packed 16-bit instructions (v_pk_sub_i16, v_pk_max_i16, v_pk_ashrrev_i16) and
// selects (v_bfi_b32).  Shared by ik_png.hip (k_png_unfilter) and the CPU model
// (ik_png_model.cpp), whose exhaustive test holds it to the byte-wise definition.
#pragma once
#include <cstdint>

#include "ik_inflate.h"

namespace ik {

// one half: r, a, b, c hold two bytes each in 16-bit lanes (0..255); the masks are
// 0 or ~0 (the row's filter type); returns the two unfiltered bytes in the same lanes
IK_HD uint32_t unfilter_half(uint32_t r, uint32_t a, uint32_t b, uint32_t c, uint32_t msub, uint32_t mup,
                             uint32_t mavg, uint32_t mpaeth) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef short s2 __attribute__((ext_vector_type(2)));
    const s2 A = __builtin_bit_cast(s2, a), B = __builtin_bit_cast(s2, b), C = __builtin_bit_cast(s2, c);
    const s2 z = {0, 0};
    const s2 d1 = B - C, d2 = A - C, s = d1 + d2;  // p - a, p - b, p - c  (p = a + b - c)
    const s2 pa = __builtin_elementwise_max(d1, z - d1);
    const s2 pb = __builtin_elementwise_max(d2, z - d2);
    const s2 pc = __builtin_elementwise_max(s, z - s);
    const s2 t = __builtin_elementwise_min(pb, pc);
    // ~0 in a lane where pa > min(pb, pc) / where pb > pc: the sign of a packed
    // difference spread over its lane (one v_pk_ashrrev_i16; written out, as the
    // compiler otherwise turns the shift into per-lane compares and selects).  The
    // shift count comes from a register holding 15 in both halves: an inline
    // constant would give the high half a count of 0 (it reads the constant's high bits).
    uint32_t m1, m2;
    const uint32_t e1 = __builtin_bit_cast(uint32_t, (s2)(t - pa)), e2 = __builtin_bit_cast(uint32_t, (s2)(pc - pb));
    const uint32_t k15 = 0x000F000Fu;
    asm("v_pk_ashrrev_i16 %0, %2, %1" : "=v"(m1) : "v"(e1), "v"(k15));
    asm("v_pk_ashrrev_i16 %0, %2, %1" : "=v"(m2) : "v"(e2), "v"(k15));
    const uint32_t avg = __builtin_bit_cast(uint32_t, (s2)((A + B) >> 1));
#else
    typedef short s2 __attribute__((vector_size(4)));
    s2 A, B, C;
    __builtin_memcpy(&A, &a, 4);
    __builtin_memcpy(&B, &b, 4);
    __builtin_memcpy(&C, &c, 4);
    const s2 z = {0, 0};
    const s2 d1 = B - C, d2 = A - C, s = d1 + d2;
    auto vmax = [](s2 x, s2 y) { const s2 m = x > y; return (x & m) | (y & ~m); };
    auto vmin = [](s2 x, s2 y) { const s2 m = x < y; return (x & m) | (y & ~m); };
    const s2 pa = vmax(d1, z - d1), pb = vmax(d2, z - d2), pc = vmax(s, z - s);
    const s2 t = vmin(pb, pc);
    const s2 v1 = (t - pa) >> 15, v2 = (pc - pb) >> 15, va = (A + B) >> 1;
    uint32_t m1, m2, avg;
    __builtin_memcpy(&m1, &v1, 4);
    __builtin_memcpy(&m2, &v2, 4);
    __builtin_memcpy(&avg, &va, 4);
#endif
    const uint32_t x = (m2 & c) | (~m2 & b);           // pb <= pc ? b : c
    const uint32_t paeth = (m1 & x) | (~m1 & a);      // pa <= pb && pa <= pc ? a : ...
    const uint32_t pred = (a & msub) | (b & mup) | (avg & mavg) | (paeth & mpaeth);
    return (r + pred) & 0x00FF00FFu;                  // (each lane <= 510: no carry across lanes)
}

// four bytes: raw (filtered), a (the unfiltered word bpp bytes back), b (the word
// above), c (the word above a); masks as unfilter_half
IK_HD uint32_t unfilter_word(uint32_t raw, uint32_t a, uint32_t b, uint32_t c, uint32_t msub, uint32_t mup,
                             uint32_t mavg, uint32_t mpaeth) {
    constexpr uint32_t M = 0x00FF00FFu;
    const uint32_t lo = unfilter_half(raw & M, a & M, b & M, c & M, msub, mup, mavg, mpaeth);
    const uint32_t hi = unfilter_half((raw >> 8) & M, (a >> 8) & M, (b >> 8) & M, (c >> 8) & M, msub, mup, mavg, mpaeth);
    return lo | (hi << 8);
}

}  // namespace ik
