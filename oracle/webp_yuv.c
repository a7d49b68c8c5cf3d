/*
 * webp_yuv.c -- ORACLE (test infrastructure only, see ik_oracle.h).
 *
 * Restates libwebp's RGB -> YUV420 import, the colour conversion inside
 * webp 0.3.1 Encoder::encode (reference src/transform.rs:131-136 ->
 * WebPPictureImport* -> ImportYUVAFromRGBA in src/enc/picture_csp_enc.c,
 * non-iterative, dithering 0, opaque):
 *   Y  = VP8RGBToY(r,g,b, YUV_HALF)              (src/dsp/yuv.h)
 *   UV = VP8RGBToU/V over gamma-corrected 2x2 sums (AccumulateRGB, SUM4/SUM2,
 *        kGamma 0.80, kGammaFix 12, kGammaTabFix 7), rounding YUV_HALF << 2.
 * Pinned against the system libwebp 1.2.2 (tests/test_oracle_webp.py).
 */
#include <math.h>
#include <stdint.h>

#include "ik_oracle.h"

#define YUV_FIX 16
#define YUV_HALF (1 << (YUV_FIX - 1))
#define GAMMA_FIX 12
#define GAMMA_SCALE ((1 << GAMMA_FIX) - 1)
#define GAMMA_TAB_FIX 7
#define GAMMA_TAB_SCALE (1 << GAMMA_TAB_FIX)
#define GAMMA_TAB_ROUNDER (GAMMA_TAB_SCALE >> 1)
#define GAMMA_TAB_SIZE (1 << (GAMMA_FIX - GAMMA_TAB_FIX))

static uint16_t g_to_lin[256];
static int lin_to_g[GAMMA_TAB_SIZE + 1];
static int g_tables_ok = 0;

static void init_gamma(void) {
    if (g_tables_ok) return;
    const double scale = (double)(1 << GAMMA_TAB_FIX) / GAMMA_SCALE;
    const double norm = 1. / 255.;
    for (int v = 0; v <= 255; ++v) g_to_lin[v] = (uint16_t)(pow(norm * v, 0.80) * GAMMA_SCALE + .5);
    for (int v = 0; v <= GAMMA_TAB_SIZE; ++v) lin_to_g[v] = (int)(255. * pow(scale * v, 1. / 0.80) + .5);
    g_tables_ok = 1;
}

static int interpolate(int v) {
    const int tab_pos = v >> (GAMMA_TAB_FIX + 2);
    const int x = v & ((GAMMA_TAB_SCALE << 2) - 1);
    const int v0 = lin_to_g[tab_pos];
    const int v1 = lin_to_g[tab_pos + 1];
    return v1 * x + v0 * ((GAMMA_TAB_SCALE << 2) - x);
}

static int linear_to_gamma(uint32_t base, int shift) {
    const int y = interpolate((int)(base << shift));
    return (y + GAMMA_TAB_ROUNDER) >> GAMMA_TAB_FIX;
}

static int rgb_to_y(int r, int g, int b) {
    const int luma = 16839 * r + 33059 * g + 6420 * b;
    return (luma + YUV_HALF + (16 << YUV_FIX)) >> YUV_FIX;
}

static int clip_uv(int uv, int rounding) {
    uv = (uv + rounding + (128 << (YUV_FIX + 2))) >> (YUV_FIX + 2);
    return ((uv & ~0xff) == 0) ? uv : (uv < 0) ? 0 : 255;
}

void iko_webp_rgb_to_yuv420(const uint8_t *rgb, int width, int height, int stride, uint8_t *y,
                            int y_stride, uint8_t *u, uint8_t *v, int uv_stride) {
    init_gamma();
    const int uvw = (width + 1) >> 1;
    for (int row = 0; row < height; ++row) {
        const uint8_t *p = rgb + (size_t)row * stride;
        for (int x = 0; x < width; ++x)
            y[(size_t)row * y_stride + x] = (uint8_t)rgb_to_y(p[3 * x], p[3 * x + 1], p[3 * x + 2]);
    }
    for (int cy = 0; cy < (height + 1) / 2; ++cy) {
        const uint8_t *r0 = rgb + (size_t)(2 * cy) * stride;
        /* last odd row: rgb_stride = 0 (the row is summed with itself) */
        const int rs = (2 * cy + 1 < height) ? stride : 0;
        for (int cx = 0; cx < uvw; ++cx) {
            int sum[3];
            const int j = 2 * cx * 3;
            for (int c = 0; c < 3; ++c) {
                const uint8_t *q = r0 + j + c;
                if (2 * cx + 1 < width) {
                    uint32_t s = g_to_lin[q[0]] + g_to_lin[q[3]] + g_to_lin[q[rs]] + g_to_lin[q[rs + 3]];
                    sum[c] = linear_to_gamma(s, 0);
                } else {
                    uint32_t s = g_to_lin[q[0]] + g_to_lin[q[rs]];
                    sum[c] = linear_to_gamma(s, 1);
                }
            }
            const int r = sum[0], g = sum[1], b = sum[2];
            u[(size_t)cy * uv_stride + cx] =
                (uint8_t)clip_uv(-9719 * r - 19081 * g + 28800 * b, YUV_HALF << 2);
            v[(size_t)cy * uv_stride + cx] =
                (uint8_t)clip_uv(+28800 * r - 24116 * g - 4684 * b, YUV_HALF << 2);
        }
    }
}
