/*
 * jpeg_enc.c -- ORACLE (test infrastructure only, see ik_oracle.h).
 *
 * Restates the JPEG branch of reference src/transform.rs:121-128:
 *   img.to_rgb8(); JpegEncoder::new_with_quality(&mut out, q).write_image(rgb, w, h, Rgb8)
 * i.e. image 0.25.8 src/codecs/jpeg/encoder.rs + src/codecs/jpeg/transform.rs:
 *   - quality scale: s = q<50 ? 5000/q : 200-2q; t = clamp((t*s+50)/100, 1, 255)
 *   - baseline, 3 components all h=v=1 (4:4:4), std Annex-K Huffman tables
 *   - per pixel rgb_to_ycbcr in f32 (JFIF coefficients x 255/max) + `as u8`
 *   - edge blocks replicate the last row/column (pixel_at_or_near)
 *   - fdct = libjpeg 9a jfdctint islow port (output scaled by 8)
 *   - quantise: ((coef / 8) as f32 / q as f32).round() as i32
 *   - BitWriter with 0xFF byte stuffing, pad_byte = write_bits(0x7F, 7)
 * The crate source is not vendored in the reference tree: "parity unpinned"
 * against the real crate; the GPU path is checked byte-for-byte against this.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ik_oracle.h"

static const uint8_t STD_LUMA_Q[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const uint8_t STD_CHROMA_Q[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

static const uint8_t LUMA_DC_LEN[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t CHROMA_DC_LEN[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t DC_VALS[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t LUMA_AC_LEN[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t LUMA_AC_VALS[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
static const uint8_t CHROMA_AC_LEN[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t CHROMA_AC_VALS[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

static const uint8_t UNZIGZAG[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* ---- growable byte buffer + BitWriter (encoder.rs BitWriter) ---- */
typedef struct { uint8_t *p; size_t n, cap; uint32_t acc; uint8_t nbits; } bw_t;

static void put(bw_t *b, uint8_t v) {
    if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 4096; b->p = realloc(b->p, b->cap); }
    b->p[b->n++] = v;
}
static void write_bits(bw_t *b, uint16_t bits, uint8_t size) {
    if (size == 0) return;
    b->nbits += size;
    b->acc |= (uint32_t)bits << (32 - b->nbits);
    while (b->nbits >= 8) {
        uint8_t byte = (uint8_t)(b->acc >> 24);
        put(b, byte);
        if (byte == 0xFF) put(b, 0x00);
        b->nbits -= 8;
        b->acc <<= 8;
    }
}
static void write_segment(bw_t *b, uint8_t marker, const uint8_t *d, size_t n) {
    put(b, 0xFF); put(b, marker);
    put(b, (uint8_t)((n + 2) >> 8)); put(b, (uint8_t)((n + 2) & 0xFF));
    for (size_t i = 0; i < n; ++i) put(b, d[i]);
}

/* Huffman LUT (size, code) from the Annex-C canonical code construction */
typedef struct { uint8_t size; uint16_t code; } huff_t;
static void build_lut(const uint8_t len[16], const uint8_t *vals, huff_t lut[256]) {
    memset(lut, 0, sizeof(huff_t) * 256);
    int k = 0; uint16_t code = 0;
    for (int i = 0; i < 16; ++i) {
        for (int j = 0; j < len[i]; ++j) { lut[vals[k]].size = (uint8_t)(i + 1); lut[vals[k]].code = code; ++k; ++code; }
        code <<= 1;
    }
}

static void encode_coefficient(int c, uint8_t *nb, uint16_t *val) {
    uint32_t mag = c < 0 ? (uint32_t)(-(int64_t)c) : (uint32_t)c;
    uint16_t m = (uint16_t)mag;
    uint8_t n = 0;
    while (m > 0) { m >>= 1; ++n; }
    uint16_t mask = (uint16_t)((1u << n) - 1);
    *val = c < 0 ? (uint16_t)((uint16_t)(c - 1) & mask) : (uint16_t)((uint16_t)c & mask);
    *nb = n;
}

static int write_block(bw_t *b, const int32_t blk[64], int prevdc, const huff_t *dc,
                       const huff_t *ac) {
    int dcval = blk[0];
    uint8_t sz; uint16_t v;
    encode_coefficient(dcval - prevdc, &sz, &v);
    write_bits(b, dc[sz].code, dc[sz].size);
    write_bits(b, v, sz);
    int zr = 0;
    for (int i = 1; i < 64; ++i) {
        int k = UNZIGZAG[i];
        if (blk[k] == 0) { ++zr; continue; }
        while (zr > 15) { write_bits(b, ac[0xF0].code, ac[0xF0].size); zr -= 16; }
        encode_coefficient(blk[k], &sz, &v);
        uint8_t sym = (uint8_t)((zr << 4) | sz);
        write_bits(b, ac[sym].code, ac[sym].size);
        write_bits(b, v, sz);
        zr = 0;
    }
    if (blk[UNZIGZAG[63]] == 0) write_bits(b, ac[0x00].code, ac[0x00].size);
    return dcval;
}

/* ---- transform.rs fdct (libjpeg 9a jfdctint islow) ---- */
#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172

static void fdct(const uint8_t s[64], int32_t c[64]) {
    for (int y = 0; y < 8; ++y) {
        const int y0 = y * 8;
        int t0 = s[y0] + s[y0 + 7], t1 = s[y0 + 1] + s[y0 + 6];
        int t2 = s[y0 + 2] + s[y0 + 5], t3 = s[y0 + 3] + s[y0 + 4];
        int t10 = t0 + t3, t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
        t0 = s[y0] - s[y0 + 7]; t1 = s[y0 + 1] - s[y0 + 6];
        t2 = s[y0 + 2] - s[y0 + 5]; t3 = s[y0 + 3] - s[y0 + 4];
        c[y0] = (t10 + t11 - 8 * 128) << PASS1_BITS;
        c[y0 + 4] = (t10 - t11) << PASS1_BITS;
        int z1 = (t12 + t13) * FIX_0_541196100;
        z1 += 1 << (CONST_BITS - PASS1_BITS - 1);
        c[y0 + 2] = (z1 + t12 * FIX_0_765366865) >> (CONST_BITS - PASS1_BITS);
        c[y0 + 6] = (z1 - t13 * FIX_1_847759065) >> (CONST_BITS - PASS1_BITS);
        t12 = t0 + t2; t13 = t1 + t3;
        z1 = (t12 + t13) * FIX_1_175875602;
        z1 += 1 << (CONST_BITS - PASS1_BITS - 1);
        t12 = t12 * (-FIX_0_390180644); t13 = t13 * (-FIX_1_961570560);
        t12 += z1; t13 += z1;
        z1 = (t0 + t3) * (-FIX_0_899976223);
        t0 = t0 * FIX_1_501321110; t3 = t3 * FIX_0_298631336;
        t0 += z1 + t12; t3 += z1 + t13;
        z1 = (t1 + t2) * (-FIX_2_562915447);
        t1 = t1 * FIX_3_072711026; t2 = t2 * FIX_2_053119869;
        t1 += z1 + t13; t2 += z1 + t12;
        c[y0 + 1] = t0 >> (CONST_BITS - PASS1_BITS);
        c[y0 + 3] = t1 >> (CONST_BITS - PASS1_BITS);
        c[y0 + 5] = t2 >> (CONST_BITS - PASS1_BITS);
        c[y0 + 7] = t3 >> (CONST_BITS - PASS1_BITS);
    }
    for (int x = 7; x >= 0; --x) {
        int t0 = c[x] + c[x + 56], t1 = c[x + 8] + c[x + 48];
        int t2 = c[x + 16] + c[x + 40], t3 = c[x + 24] + c[x + 32];
        int t10 = t0 + t3 + (1 << (PASS1_BITS - 1)), t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
        t0 = c[x] - c[x + 56]; t1 = c[x + 8] - c[x + 48];
        t2 = c[x + 16] - c[x + 40]; t3 = c[x + 24] - c[x + 32];
        c[x] = (t10 + t11) >> PASS1_BITS;
        c[x + 32] = (t10 - t11) >> PASS1_BITS;
        int z1 = (t12 + t13) * FIX_0_541196100;
        z1 += 1 << (CONST_BITS + PASS1_BITS - 1);
        c[x + 16] = (z1 + t12 * FIX_0_765366865) >> (CONST_BITS + PASS1_BITS);
        c[x + 48] = (z1 - t13 * FIX_1_847759065) >> (CONST_BITS + PASS1_BITS);
        t12 = t0 + t2; t13 = t1 + t3;
        z1 = (t12 + t13) * FIX_1_175875602;
        z1 += 1 << (CONST_BITS + PASS1_BITS - 1);
        t12 = t12 * (-FIX_0_390180644); t13 = t13 * (-FIX_1_961570560);
        t12 += z1; t13 += z1;
        z1 = (t0 + t3) * (-FIX_0_899976223);
        t0 = t0 * FIX_1_501321110; t3 = t3 * FIX_0_298631336;
        t0 += z1 + t12; t3 += z1 + t13;
        z1 = (t1 + t2) * (-FIX_2_562915447);
        t1 = t1 * FIX_3_072711026; t2 = t2 * FIX_2_053119869;
        t1 += z1 + t13; t2 += z1 + t12;
        c[x + 8] = t0 >> (CONST_BITS + PASS1_BITS);
        c[x + 24] = t1 >> (CONST_BITS + PASS1_BITS);
        c[x + 40] = t2 >> (CONST_BITS + PASS1_BITS);
        c[x + 56] = t3 >> (CONST_BITS + PASS1_BITS);
    }
}

/* Rust `f32 as u8`: saturating, truncating, NaN -> 0 */
static uint8_t f32_as_u8(float v) {
    if (!(v > 0.0f)) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}

/* encoder.rs rgb_to_ycbcr (max = 255) */
static void rgb_to_ycbcr(uint8_t R, uint8_t G, uint8_t B, uint8_t *y, uint8_t *cb, uint8_t *cr) {
    const float max = 255.0f;
    float r = R, g = G, b = B;
    float yy = 76.245f / max * r + 149.685f / max * g + 29.07f / max * b;
    float cbb = -43.0185f / max * r - 84.4815f / max * g + 127.5f / max * b + 128.0f;
    float crr = 127.5f / max * r - 106.7685f / max * g - 20.7315f / max * b + 128.0f;
    *y = f32_as_u8(yy); *cb = f32_as_u8(cbb); *cr = f32_as_u8(crr);
}

static void quant_tables(int quality, uint8_t t[2][64]) {
    uint32_t s = (uint32_t)(quality < 1 ? 1 : quality > 100 ? 100 : quality);
    s = s < 50 ? 5000 / s : 200 - s * 2;
    for (int i = 0; i < 64; ++i) {
        uint32_t a = (STD_LUMA_Q[i] * s + 50) / 100, b = (STD_CHROMA_Q[i] * s + 50) / 100;
        t[0][i] = (uint8_t)(a < 1 ? 1 : a > 255 ? 255 : a);
        t[1][i] = (uint8_t)(b < 1 ? 1 : b > 255 ? 255 : b);
    }
}

/* one MCU (8x8, 4:4:4): colour convert + fdct + quantise, natural order */
static void mcu_coeffs(const uint8_t *rgb, uint32_t w, uint32_t h, uint32_t x0, uint32_t y0,
                       const uint8_t qt[2][64], int32_t out[3][64]) {
    uint8_t blk[3][64];
    for (uint32_t y = 0; y < 8; ++y)
        for (uint32_t x = 0; x < 8; ++x) {
            uint32_t px = x0 + x, py = y0 + y;
            if (px >= w) px = w - 1; /* pixel_at_or_near */
            if (py >= h) py = h - 1;
            const uint8_t *p = rgb + ((size_t)py * w + px) * 3;
            rgb_to_ycbcr(p[0], p[1], p[2], &blk[0][y * 8 + x], &blk[1][y * 8 + x], &blk[2][y * 8 + x]);
        }
    for (int c = 0; c < 3; ++c) {
        int32_t d[64];
        fdct(blk[c], d);
        const uint8_t *q = qt[c ? 1 : 0];
        for (int i = 0; i < 64; ++i) out[c][i] = (int32_t)roundf((float)(d[i] / 8) / (float)q[i]);
    }
}

int iko_jpeg_coeffs_rgb(const uint8_t *rgb, uint32_t w, uint32_t h, int quality, int16_t *coef) {
    uint8_t qt[2][64];
    quant_tables(quality, qt);
    size_t m = 0;
    for (uint32_t y = 0; y < h; y += 8)
        for (uint32_t x = 0; x < w; x += 8, ++m) {
            int32_t o[3][64];
            mcu_coeffs(rgb, w, h, x, y, qt, o);
            for (int c = 0; c < 3; ++c)
                for (int i = 0; i < 64; ++i) coef[(m * 3 + c) * 64 + i] = (int16_t)o[c][i];
        }
    return 0;
}

long iko_jpeg_encode_rgb(const uint8_t *rgb, uint32_t w, uint32_t h, int quality, uint8_t **out) {
    if (w > 65535 || h > 65535) return -1; /* u16::try_from(width) */
    uint8_t qt[2][64];
    quant_tables(quality, qt);
    huff_t ldc[256], lac[256], cdc[256], cac[256];
    build_lut(LUMA_DC_LEN, DC_VALS, ldc);
    build_lut(LUMA_AC_LEN, LUMA_AC_VALS, lac);
    build_lut(CHROMA_DC_LEN, DC_VALS, cdc);
    build_lut(CHROMA_AC_LEN, CHROMA_AC_VALS, cac);
    bw_t b = {0};
    put(&b, 0xFF); put(&b, 0xD8); /* SOI */
    const uint8_t jfif[14] = {'J', 'F', 'I', 'F', 0, 1, 2, 0, 0, 1, 0, 1, 0, 0};
    write_segment(&b, 0xE0, jfif, 14);
    uint8_t sof[15] = {8, (uint8_t)(h >> 8), (uint8_t)h, (uint8_t)(w >> 8), (uint8_t)w, 3,
                       1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1};
    write_segment(&b, 0xC0, sof, 15);
    for (int t = 0; t < 2; ++t) {
        uint8_t dqt[65];
        dqt[0] = (uint8_t)t;
        for (int i = 0; i < 64; ++i) dqt[1 + i] = qt[t][UNZIGZAG[i]];
        write_segment(&b, 0xDB, dqt, 65);
    }
    struct { uint8_t tc; const uint8_t *len; const uint8_t *vals; int nv; } dht[4] = {
        {0x00, LUMA_DC_LEN, DC_VALS, 12}, {0x10, LUMA_AC_LEN, LUMA_AC_VALS, 162},
        {0x01, CHROMA_DC_LEN, DC_VALS, 12}, {0x11, CHROMA_AC_LEN, CHROMA_AC_VALS, 162}};
    for (int t = 0; t < 4; ++t) {
        uint8_t seg[1 + 16 + 162];
        seg[0] = dht[t].tc;
        memcpy(seg + 1, dht[t].len, 16);
        memcpy(seg + 17, dht[t].vals, (size_t)dht[t].nv);
        write_segment(&b, 0xC4, seg, (size_t)(17 + dht[t].nv));
    }
    const uint8_t sos[10] = {3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    write_segment(&b, 0xDA, sos, 10);
    int pdc[3] = {0, 0, 0};
    for (uint32_t y = 0; y < h; y += 8)
        for (uint32_t x = 0; x < w; x += 8) {
            int32_t o[3][64];
            mcu_coeffs(rgb, w, h, x, y, qt, o);
            pdc[0] = write_block(&b, o[0], pdc[0], ldc, lac);
            pdc[1] = write_block(&b, o[1], pdc[1], cdc, cac);
            pdc[2] = write_block(&b, o[2], pdc[2], cdc, cac);
        }
    write_bits(&b, 0x7F, 7); /* pad_byte */
    put(&b, 0xFF); put(&b, 0xD9); /* EOI */
    *out = b.p;
    return (long)b.n;
}

/* the reference transform on a decoded 8-bit image (cpu_baseline "port") */
long iko_transform_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, int64_t w_opt,
                      int64_t h_opt, int filter, int fmt, int quality, uint8_t **out,
                      uint32_t *ow, uint32_t *oh) {
    uint32_t nw, nh;
    int resample = iko_resize_image_dims(W, H, w_opt, h_opt, &nw, &nh);
    const uint8_t *img = src;
    uint8_t *rs = NULL;
    if (resample) {
        rs = malloc((size_t)nw * nh * C);
        if (!rs || iko_resize_u8(src, W, H, C, nw, nh, filter, rs)) { free(rs); return -1; }
        img = rs;
    }
    uint8_t *rgb = malloc((size_t)nw * nh * 3);
    iko_to_rgb8(img, nw * nh, C, rgb);
    free(rs);
    int q = quality < 1 ? 1 : quality > 100 ? 100 : quality;
    long n = fmt == 0 ? iko_jpeg_encode_rgb(rgb, nw, nh, q, out)
                      : iko_webp_encode_rgb(rgb, (int)nw, (int)nh, (int)nw * 3, (float)q, out);
    free(rgb);
    *ow = nw; *oh = nh;
    return n;
}
