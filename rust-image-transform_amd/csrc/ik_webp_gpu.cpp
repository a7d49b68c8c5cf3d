// ik_webp_gpu.cpp -- the WebP coder selection (encode_image's WebP branch, reference
// src/transform.rs:129-137): libwebp on the host (IK_WEBP_LIBWEBP) or libwebp's own
// method-4 decisions on the GPU (IK_WEBP_EXACT, ik_vp8x.hip / ik_vp8x_host.cpp), both
// byte-identical to WebPEncodeRGB; and the segment-analysis entry point the exact
// coder starts with (ik_vp8_analyze_device).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {

namespace {

std::atomic<int> g_webp_encoder{-1};  // -1 = not yet read from IK_WEBP_ENCODER

}  // namespace

int default_webp_encoder() {
    int e = g_webp_encoder.load();
    if (e < 0) {
        const char* s = getenv("IK_WEBP_ENCODER");
        e = (s && (!strcmp(s, "libwebp") || !strcmp(s, "0"))) ? IK_WEBP_LIBWEBP
            : (s && (!strcmp(s, "exact") || !strcmp(s, "2"))) ? IK_WEBP_EXACT
            : (s && (!strcmp(s, "auto") || !strcmp(s, "3"))) ? IK_WEBP_AUTO : kDefaultWebpEncoder;
        int expected = -1;
        g_webp_encoder.compare_exchange_strong(expected, e);
        e = g_webp_encoder.load();
    }
    return e;
}

}  // namespace ik

using namespace ik;

extern "C" {

int ik_set_webp_encoder(int encoder) {
    if (encoder != IK_WEBP_LIBWEBP && encoder != IK_WEBP_EXACT && encoder != IK_WEBP_AUTO)
        return fail(IK_ERR_INVALID, "bad WebP encoder %d", encoder);
    (void)default_webp_encoder();
    g_webp_encoder.store(encoder);
    return IK_OK;
}

int ik_get_webp_encoder(void) { return default_webp_encoder(); }

int ik_vp8_analyze_device(const uint8_t* dev_yuv, size_t yuv_stride, uint32_t n, uint32_t w, uint32_t h,
                          float quality, uint8_t* seg, ik_vp8_segment_header* hdr) {
    IK_API_ENTER();
    if (!dev_yuv || !seg || !hdr) return fail(IK_ERR_INVALID, "null pointer");
    if (n < 1 || n > 65535 || w < 1 || h < 1 || w > 16383 || h > 16383)
        return fail(IK_ERR_INVALID, "bad VP8 analysis shape %ux%u x %u", w, h, n);
    if (!(quality >= 0.f)) quality = 0.f;
    if (quality > 100.f) quality = 100.f;
    const size_t ysz = (size_t)w * h + 2 * (size_t)((w + 1) / 2) * ((h + 1) / 2);
    if (n > 1 && yuv_stride < ysz) return fail(IK_ERR_INVALID, "image stride %zu under the planes' %zu bytes", yuv_stride, ysz);
    return vp8_analyze_setup(dev_yuv, yuv_stride, (int)n, (int)w, (int)h, quality, seg, hdr);
}

}  // extern "C"
