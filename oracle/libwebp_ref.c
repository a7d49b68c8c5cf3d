/*
 * libwebp_ref.c -- ORACLE (test infrastructure only, see ik_oracle.h).
 *
 * The reference's WebP encoder is webp 0.3.1 (Cargo.lock:2811) over
 * libwebp-sys 0.9.6's vendored libwebp (Cargo.lock:1168); neither is present
 * here.  The same libwebp C API is reached through the system libwebp.so.7
 * (libwebp 1.2.2) with dlopen, so no webp headers are needed:
 *   webp::Encoder::from_rgb(rgb,w,h).encode(q)
 *     == WebPConfigInit + quality=q + lossless=0 + WebPPictureImportRGB + WebPEncode
 *     == WebPEncodeRGB(rgb, w, h, 3*w, q, &out)          (libwebp simple API)
 * Both take the same ImportYUVAFromRGBA path for opaque input (see webp_yuv.c).
 *
 * iko_libwebp_import_yuv() runs libwebp's own WebPPictureImportRGB and copies
 * the Y/U/V planes out; it pins webp_yuv.c (and through it the GPU kernel)
 * against the real library.  WebPPicture offsets are those of
 * WEBP_ENCODER_ABI_VERSION 0x020f (libwebp 1.2.x encode.h); the function
 * checks them against what WebPPictureAlloc writes before trusting them.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ik_oracle.h"

typedef size_t (*enc_rgb_fn)(const uint8_t *, int, int, int, float, uint8_t **);
typedef void (*free_fn)(void *);
typedef int (*pic_init_fn)(void *, int);
typedef int (*pic_import_fn)(void *, const uint8_t *, int);
typedef void (*pic_free_fn)(void *);

static void *g_webp = NULL;

static void *webp_lib(void) {
    if (!g_webp) g_webp = dlopen("libwebp.so.7", RTLD_NOW | RTLD_LOCAL);
    return g_webp;
}

long iko_webp_encode_rgb(const uint8_t *rgb, int w, int h, int stride, float q, uint8_t **out) {
    void *lib = webp_lib();
    if (!lib) return -1;
    enc_rgb_fn enc = (enc_rgb_fn)dlsym(lib, "WebPEncodeRGB");
    free_fn wfree = (free_fn)dlsym(lib, "WebPFree");
    if (!enc || !wfree) return -1;
    uint8_t *tmp = NULL;
    size_t n = enc(rgb, w, h, stride, q, &tmp);
    if (n == 0 || !tmp) return -1;
    *out = malloc(n);
    memcpy(*out, tmp, n);
    wfree(tmp);
    return (long)n;
}

#define PIC_WIDTH 8
#define PIC_HEIGHT 12
#define PIC_Y 16
#define PIC_U 24
#define PIC_V 32
#define PIC_Y_STRIDE 40
#define PIC_UV_STRIDE 44
#define PIC_MEMORY 224

int iko_libwebp_import_yuv(const uint8_t *rgb, int width, int height, int stride, uint8_t *y,
                           uint8_t *u, uint8_t *v) {
    void *lib = webp_lib();
    if (!lib) return -1;
    pic_init_fn init = (pic_init_fn)dlsym(lib, "WebPPictureInitInternal");
    pic_import_fn imp = (pic_import_fn)dlsym(lib, "WebPPictureImportRGB");
    pic_free_fn pfree = (pic_free_fn)dlsym(lib, "WebPPictureFree");
    if (!init || !imp || !pfree) return -1;
    _Alignas(16) unsigned char pic[1024];
    memset(pic, 0, sizeof(pic));
    if (!init(pic, 0x020f)) return -2;
    memcpy(pic + PIC_WIDTH, &width, 4);
    memcpy(pic + PIC_HEIGHT, &height, 4);
    if (!imp(pic, rgb, stride)) return -3;
    uint8_t *py, *pu, *pv;
    int ys, uvs;
    void *mem;
    memcpy(&py, pic + PIC_Y, 8); memcpy(&pu, pic + PIC_U, 8); memcpy(&pv, pic + PIC_V, 8);
    memcpy(&ys, pic + PIC_Y_STRIDE, 4); memcpy(&uvs, pic + PIC_UV_STRIDE, 4);
    memcpy(&mem, pic + PIC_MEMORY, 8);
    const int uvw = (width + 1) / 2, uvh = (height + 1) / 2;
    if (!py || !pu || !pv || !mem || ys != width || uvs != uvw) { pfree(pic); return -4; }
    for (int r = 0; r < height; ++r) memcpy(y + (size_t)r * width, py + (size_t)r * ys, width);
    for (int r = 0; r < uvh; ++r) {
        memcpy(u + (size_t)r * uvw, pu + (size_t)r * uvs, uvw);
        memcpy(v + (size_t)r * uvw, pv + (size_t)r * uvs, uvw);
    }
    pfree(pic);
    return 0;
}
