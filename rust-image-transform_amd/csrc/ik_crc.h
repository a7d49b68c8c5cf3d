// ik_crc.h -- CRC-32 of PNG chunks (ISO 3309 / zlib crc32: reflected polynomial
// 0xEDB88320, register preset to all ones, final complement) in independent
// pieces, and the algebra that joins them (zlib's crc32_combine: appending n
// bytes to a message multiplies its CRC register by x^(8n) modulo P, so
// crc(A || B) = crc(A) * x^(8 |B|) + crc(B) in GF(2)[x] / P).  png 0.18 verifies
// every chunk's CRC (reference decode path src/transform.rs:31); the GPU gather
// kernel (ik_png.hip k_png_gather) checks the IDAT chunks with these functions and
// the CPU model (ik_png_model.cpp) runs the same functions against zlib.
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define IK_CRC_HD __host__ __device__
#else
#define IK_CRC_HD
#endif

namespace ik {
namespace crc {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected
constexpr uint32_t kOne = 0x80000000u;   // the polynomial 1 in the reflected representation

// a * b modulo P (reflected representation; zlib crc32.c multmodp)
IK_CRC_HD inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = kOne, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1u)) == 0) break;
        }
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

// x2n[k] = x^(2^k) modulo P, k = 0..31
IK_CRC_HD inline void x2n_table(uint32_t* x2n) {
    uint32_t p = kOne >> 1;  // x^1
    for (int k = 0; k < 32; ++k) {
        x2n[k] = p;
        p = multmodp(p, p);
    }
}

// x^(8 n) modulo P: the operator that appends n zero bytes
IK_CRC_HD inline uint32_t x8n(uint64_t n, const uint32_t* x2n) {
    uint32_t p = kOne;
    int k = 3;
    while (n) {
        if (n & 1u) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

// crc(A || B) from crc(A), crc(B) and |B| (finished CRC values, as zlib's)
IK_CRC_HD inline uint32_t combine_op(uint32_t crc_a, uint32_t crc_b, uint32_t op_b) {
    return multmodp(op_b, crc_a) ^ crc_b;
}

// the byte table (slice 0) and slices 1..3 for slicing-by-4: t[256 * s + i]
IK_CRC_HD inline uint32_t table_entry(uint32_t i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    return c;
}

// CRC register update over one little-endian word (4 message bytes in address
// order) and over one byte; the register is kept un-complemented here
IK_CRC_HD inline uint32_t step_word(uint32_t c, uint32_t v, const uint32_t* t) {
    c ^= v;
    return t[768 + (c & 255u)] ^ t[512 + ((c >> 8) & 255u)] ^ t[256 + ((c >> 16) & 255u)] ^ t[c >> 24];
}
IK_CRC_HD inline uint32_t step_byte(uint32_t c, uint32_t b, const uint32_t* t) {
    return t[(c ^ b) & 255u] ^ (c >> 8);
}

}  // namespace crc
}  // namespace ik
