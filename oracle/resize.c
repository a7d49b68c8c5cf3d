/*
 * resize.c -- ORACLE (test infrastructure only, see ik_oracle.h).
 *
 * Restates, operation for operation in f32 (built with -ffp-contract=off so no
 * multiply-add is fused, as rustc never contracts):
 *   reference src/transform.rs:62-90  resize_image
 *   image 0.25.8 src/dynimage.rs       DynamicImage::resize / resize_dimensions
 *   image 0.25.8 src/imageops/sample.rs resize, vertical_sample, horizontal_sample,
 *                                       sinc, lanczos, triangle, bc_cubic_spline,
 *                                       gaussian, box kernel, FloatNearest rounding
 * Rust's f32::sin/exp lower to glibc sinf/expf on x86_64-linux-gnu, so the same
 * libm calls are used here.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ik_oracle.h"

#define PI_F 3.14159265358979323846264338327950288f

/* sample.rs: fn sinc(t: f32) -> f32 */
static float sinc_f(float t) {
    float a = t * PI_F;
    if (t == 0.0f) return 1.0f;
    return sinf(a) / a;
}

/* sample.rs: fn lanczos(x: f32, t: f32) -> f32 */
static float lanczos_f(float x, float t) {
    if (fabsf(x) < t) return sinc_f(x) * sinc_f(x / t);
    return 0.0f;
}

/* sample.rs: fn bc_cubic_spline(x, b, c); catmullrom_kernel = (b=0, c=0.5).
 * Coefficient expressions are constant-folded by rustc; evaluated here with
 * the same IEEE results. powi(3) == (a*a)*a, powi(2) == a*a. */
static float bc_cubic_spline_f(float x, float b, float c) {
    float a = fabsf(x);
    float k;
    if (a < 1.0f) {
        float a2 = a * a, a3 = a2 * a;
        k = (12.0f - 9.0f * b - 6.0f * c) * a3 + (-18.0f + 12.0f * b + 6.0f * c) * a2 +
            (6.0f - 2.0f * b);
    } else if (a < 2.0f) {
        float a2 = a * a, a3 = a2 * a;
        k = (-b - 6.0f * c) * a3 + (6.0f * b + 30.0f * c) * a2 + (-12.0f * b - 48.0f * c) * a +
            (8.0f * b + 24.0f * c);
    } else {
        k = 0.0f;
    }
    return k / 6.0f;
}

/* sample.rs: fn gaussian(x, r) = ((2π).sqrt() * r).recip() * (-x.powi(2) / (2 * r.powi(2))).exp();
 * gaussian_kernel(x) = gaussian(x, 0.5) */
static float gaussian_f(float x, float r) {
    float c = 1.0f / (sqrtf(2.0f * PI_F) * r);
    return c * expf(-(x * x) / (2.0f * (r * r)));
}

static float kernel_eval(int filter, float x) {
    switch (filter) {
    case IKO_NEAREST: return 1.0f; /* box_kernel: always 1 */
    case IKO_TRIANGLE: return fabsf(x) < 1.0f ? 1.0f - fabsf(x) : 0.0f;
    case IKO_CATMULLROM: return bc_cubic_spline_f(x, 0.0f, 0.5f);
    case IKO_GAUSSIAN: return gaussian_f(x, 0.5f);
    default: return lanczos_f(x, 3.0f); /* lanczos3_kernel */
    }
}

/* sample.rs resize(): Filter { support } per FilterType */
static float filter_support(int filter) {
    switch (filter) {
    case IKO_NEAREST: return 0.0f;
    case IKO_TRIANGLE: return 1.0f;
    case IKO_CATMULLROM: return 2.0f;
    default: return 3.0f; /* Gaussian, Lanczos3 */
    }
}

/* The weight computation shared by vertical_sample and horizontal_sample. */
int iko_axis_weights(uint32_t in, uint32_t out, int filter, int32_t *left_o, int32_t *count_o,
                     float *w_o, int maxtaps) {
    float ratio = (float)in / (float)out;
    float sratio = ratio < 1.0f ? 1.0f : ratio;
    float src_support = filter_support(filter) * sratio;
    int maxc = 0;
    for (uint32_t o = 0; o < out; ++o) {
        float inputx = ((float)o + 0.5f) * ratio;
        long long left = (long long)floorf(inputx - src_support);
        if (left < 0) left = 0;
        if (left > (long long)in - 1) left = (long long)in - 1;
        long long right = (long long)ceilf(inputx + src_support);
        if (right < left + 1) right = left + 1;
        if (right > (long long)in) right = (long long)in;
        inputx = inputx - 0.5f;
        int n = (int)(right - left);
        if (n > maxc) maxc = n;
        if (n > maxtaps) return -1;
        float sum = 0.0f;
        float *ws = w_o + (size_t)o * (size_t)maxtaps;
        for (int k = 0; k < n; ++k) {
            float wv = kernel_eval(filter, ((float)(left + k) - inputx) / sratio);
            ws[k] = wv;
            sum = sum + wv;
        }
        for (int k = 0; k < n; ++k) ws[k] = ws[k] / sum;
        for (int k = n; k < maxtaps; ++k) ws[k] = 0.0f;
        left_o[o] = (int32_t)left;
        count_o[o] = n;
    }
    return maxc;
}

static int max_taps_bound(uint32_t in, uint32_t out, int filter) {
    float ratio = (float)in / (float)out;
    float sratio = ratio < 1.0f ? 1.0f : ratio;
    return (int)ceilf(2.0f * filter_support(filter) * sratio) + 3;
}

/* vertical_sample: out is Rgba32F(W x nh); channels filtered independently,
 * so only the image's own C channels are kept. */
int iko_vertical_sample_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, uint32_t nh,
                           int filter, float *tmp) {
    int T = max_taps_bound(H, nh, filter);
    int32_t *left = malloc(sizeof(int32_t) * nh), *cnt = malloc(sizeof(int32_t) * nh);
    float *ws = malloc(sizeof(float) * (size_t)nh * (size_t)T);
    if (!left || !cnt || !ws) { free(left); free(cnt); free(ws); return -1; }
    iko_axis_weights(H, nh, filter, left, cnt, ws, T);
    size_t rowb = (size_t)W * C;
    for (uint32_t oy = 0; oy < nh; ++oy) {
        const float *w = ws + (size_t)oy * T;
        float *o = tmp + (size_t)oy * rowb;
        for (size_t b = 0; b < rowb; ++b) {
            float t = 0.0f;
            for (int k = 0; k < cnt[oy]; ++k) {
                float p = (float)src[(size_t)(left[oy] + k) * rowb + b];
                float prod = p * w[k];
                t = t + prod;
            }
            o[b] = t;
        }
    }
    free(left); free(cnt); free(ws);
    return 0;
}

/* Rust f32::round (half away from zero) of clamp(t, 0, 255) -> u8 */
static uint8_t float_nearest_u8(float t) {
    if (t < 0.0f) t = 0.0f;
    else if (t > 255.0f) t = 255.0f;
    return (uint8_t)roundf(t);
}

int iko_resize_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, uint32_t nw,
                  uint32_t nh, int filter, uint8_t *dst) {
    if (C < 1 || C > 4) return -1;
    if (W == 0 || H == 0) { /* "nothing to sample from": blank image */
        memset(dst, 0, (size_t)nw * nh * C);
        return 0;
    }
    if (nw == W && nh == H) { /* copy instead of resampling */
        memcpy(dst, src, (size_t)W * H * C);
        return 0;
    }
    float *tmp = malloc(sizeof(float) * (size_t)W * nh * C);
    if (!tmp) return -1;
    if (iko_vertical_sample_u8(src, W, H, C, nh, filter, tmp)) { free(tmp); return -1; }
    int T = max_taps_bound(W, nw, filter);
    int32_t *left = malloc(sizeof(int32_t) * nw), *cnt = malloc(sizeof(int32_t) * nw);
    float *ws = malloc(sizeof(float) * (size_t)nw * (size_t)T);
    if (!left || !cnt || !ws) { free(tmp); free(left); free(cnt); free(ws); return -1; }
    iko_axis_weights(W, nw, filter, left, cnt, ws, T);
    for (uint32_t ox = 0; ox < nw; ++ox) {
        const float *w = ws + (size_t)ox * T;
        for (uint32_t y = 0; y < nh; ++y) {
            const float *row = tmp + (size_t)y * W * C;
            for (uint32_t c = 0; c < C; ++c) {
                float t = 0.0f;
                for (int k = 0; k < cnt[ox]; ++k) {
                    float prod = row[(size_t)(left[ox] + k) * C + c] * w[k];
                    t = t + prod;
                }
                dst[((size_t)y * nw + ox) * C + c] = float_nearest_u8(t);
            }
        }
    }
    free(tmp); free(left); free(cnt); free(ws);
    return 0;
}

/* image 0.25.8 resize_dimensions (f64 ratio, aspect fit when fill == 0) */
void iko_resize_dimensions(uint32_t w, uint32_t h, uint32_t nw, uint32_t nh, int fill,
                           uint32_t *ow, uint32_t *oh) {
    double wratio = (double)nw / (double)w;
    double hratio = (double)nh / (double)h;
    double ratio = fill ? (wratio > hratio ? wratio : hratio) : (wratio < hratio ? wratio : hratio);
    double fw = round((double)w * ratio), fh = round((double)h * ratio);
    unsigned long long rw = fw < 0 ? 0 : (unsigned long long)fw;
    unsigned long long rh = fh < 0 ? 0 : (unsigned long long)fh;
    if (rw < 1) rw = 1;
    if (rh < 1) rh = 1;
    if (rw > 0xFFFFFFFFull) {
        double r2 = (double)0xFFFFFFFFu / (double)w;
        unsigned long long t = (unsigned long long)round((double)h * r2);
        *ow = 0xFFFFFFFFu; *oh = t < 1 ? 1 : (uint32_t)t;
    } else if (rh > 0xFFFFFFFFull) {
        double r2 = (double)0xFFFFFFFFu / (double)h;
        unsigned long long t = (unsigned long long)round((double)w * r2);
        *ow = t < 1 ? 1 : (uint32_t)t; *oh = 0xFFFFFFFFu;
    } else {
        *ow = (uint32_t)rw; *oh = (uint32_t)rh;
    }
}

/* Rust `f32 as u32`: saturating, NaN -> 0 */
static uint32_t f32_as_u32(float v) {
    if (!(v > 0.0f)) return 0;
    if (v >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

int iko_resize_image_dims(uint32_t W, uint32_t H, int64_t w_opt, int64_t h_opt, uint32_t *ow,
                          uint32_t *oh) {
    if (w_opt < 0 && h_opt < 0) { *ow = W; *oh = H; return 0; }
    uint32_t tw, th;
    if (w_opt >= 0) tw = (uint32_t)w_opt;
    else {
        float ratio = (float)(uint32_t)h_opt / (float)H;
        tw = f32_as_u32(roundf((float)W * ratio));
    }
    if (h_opt >= 0) th = (uint32_t)h_opt;
    else {
        float ratio = (float)(uint32_t)w_opt / (float)W;
        th = f32_as_u32(roundf((float)H * ratio));
    }
    if (tw < 1) tw = 1;
    if (th < 1) th = 1;
    /* DynamicImage::resize */
    if (tw == W && th == H) { *ow = W; *oh = H; return 0; }
    iko_resize_dimensions(W, H, tw, th, 0, ow, oh);
    if (*ow == W && *oh == H) return 0; /* imageops::resize copies */
    return 1;
}

void iko_to_rgb8(const uint8_t *src, uint32_t npix, uint32_t C, uint8_t *dst) {
    for (uint32_t i = 0; i < npix; ++i) {
        const uint8_t *p = src + (size_t)i * C;
        uint8_t *o = dst + (size_t)i * 3;
        if (C >= 3) { o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; }
        else { o[0] = o[1] = o[2] = p[0]; } /* Luma / LumaA: replicate, drop alpha */
    }
}

void iko_to_rgba8(const uint8_t *src, uint32_t npix, uint32_t C, uint8_t *dst) {
    for (uint32_t i = 0; i < npix; ++i) {
        const uint8_t *p = src + (size_t)i * C;
        uint8_t *o = dst + (size_t)i * 4;
        if (C >= 3) { o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = C == 4 ? p[3] : 255; }
        else { o[0] = o[1] = o[2] = p[0]; o[3] = C == 2 ? p[1] : 255; }
    }
}

void iko_free(void *p) { free(p); }
