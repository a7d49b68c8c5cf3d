// ik_webp_gpu.cpp -- driver of the GPU WebP encoder (encode_image's WebP branch,
// reference src/transform.rs:129-137, as an alternative to libwebp on the host):
// device YUV420 planes -> k_vp8_diag wavefront (ik_vp8.hip) -> k_vp8_pack (compact
// MB records written into pinned host memory; a plain D2H of the records for
// frames over 4096 MBs) -> bitstream + RIFF on the host (ik_vp8_enc.cpp).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"
#include "ik_vp8_enc.h"
#include "ik_vp8_gpu.h"

namespace ik {

namespace {

std::atomic<int> g_webp_encoder{-1};  // -1 = not yet read from IK_WEBP_ENCODER

}  // namespace

int default_webp_encoder() {
    int e = g_webp_encoder.load();
    if (e < 0) {
        const char* s = getenv("IK_WEBP_ENCODER");
        e = (s && (!strcmp(s, "gpu") || !strcmp(s, "1"))) ? IK_WEBP_GPU : IK_WEBP_LIBWEBP;
        int expected = -1;
        g_webp_encoder.compare_exchange_strong(expected, e);
        e = g_webp_encoder.load();
    }
    return e;
}

int Vp8Work::reserve(int w_, int h_, int n_, bool host_buffers) {
    const int mbw = (w_ + 15) >> 4, mbh = (h_ + 15) >> 4;
    const size_t nmb = (size_t)mbw * mbh;
    const size_t rec = vp8::vp8_rec_bytes(w_, h_);
    if (d_rec && w_ == w && h_ == h && n_ <= cap_n) return IK_OK;
    release();
    IK_HIP(hipMalloc(&d_rec, rec * n_ + 256));
    IK_HIP(hipMalloc(&d_mbs, sizeof(vp8::MBOut) * nmb * n_ + 256));
    IK_HIP(hipMalloc(&d_nz, 18 * nmb * n_ + 256));
    const bool pack = nmb <= (size_t)vp8::kMaxPackMBs;
    if (pack) IK_HIP(hipMalloc(&d_pack, vp8::vp8_pack_cap(nmb) * n_));
    // pinned mirrors only for callers that copy through this object (the
    // pipeline keeps its own per-slot buffers): compact streams, or full
    // records for frames too big to pack
    if (host_buffers && pack) IK_HIP(hipHostMalloc(&h_pack, vp8::vp8_pack_cap(nmb) * n_, hipHostMallocDefault));
    if (host_buffers && !pack) IK_HIP(hipHostMalloc(&h_mbs, sizeof(vp8::MBOut) * nmb * n_, hipHostMallocDefault));
    w = w_; h = h_; cap_n = n_;
    return IK_OK;
}

void Vp8Work::release() {
    if (d_rec) (void)hipFree(d_rec);
    if (d_mbs) (void)hipFree(d_mbs);
    if (d_nz) (void)hipFree(d_nz);
    if (h_mbs) (void)hipHostFree(h_mbs);
    if (d_pack) (void)hipFree(d_pack);
    if (h_pack) (void)hipHostFree(h_pack);
    d_rec = nullptr; d_mbs = nullptr; d_nz = nullptr; h_mbs = nullptr; d_pack = nullptr; h_pack = nullptr;
    w = h = cap_n = 0;
}

size_t Vp8Work::mb_count() const { return (size_t)((w + 15) >> 4) * ((h + 15) >> 4); }

int Vp8Work::launch(const uint8_t* d_yuv, size_t yuv_stride, int n, int quality, hipStream_t s) {
    if (!d_rec || n > cap_n) return fail(IK_ERR_INVALID, "VP8 work buffers not reserved");
    vp8::Vp8Args a{};
    a.yuv = d_yuv;
    a.yuv_stride = yuv_stride;
    a.w = w; a.h = h;
    a.mb_w = (w + 15) >> 4; a.mb_h = (h + 15) >> 4;
    a.rec = d_rec;
    a.rec_stride = vp8::vp8_rec_bytes(w, h);
    a.mbs = d_mbs;
    a.nz = d_nz;
    a.q = vp8::qparams_for_quality((float)quality);
    a.stamps = nullptr;
    IK_HIP(vp8::launch_vp8_encode(a, n, s));
    return IK_OK;
}

size_t Vp8Work::record_bytes(int n) const { return sizeof(vp8::MBOut) * mb_count() * (size_t)n; }

int Vp8Work::fetch_to(vp8::MBOut* dst, int n, hipStream_t s) {
    IK_HIP(hipMemcpyAsync(dst, d_mbs, sizeof(vp8::MBOut) * mb_count() * n, hipMemcpyDeviceToHost, s));
    return IK_OK;
}

void Vp8Work::write_from(const vp8::MBOut* recs, int i, int quality, std::vector<uint8_t>& out) const {
    const vp8::QParams q = vp8::qparams_for_quality((float)quality);
    vp8::write_webp(w, h, q, recs + mb_count() * (size_t)i, -1, out);
}

bool Vp8Work::packable() const { return d_pack != nullptr; }

size_t Vp8Work::pack_cap() const { return vp8::vp8_pack_cap(mb_count()); }

int Vp8Work::pack_to(uint8_t* host_dst, int n, hipStream_t s) {
    if (!d_pack || n > cap_n) return fail(IK_ERR_INVALID, "VP8 pack buffers not reserved");
    IK_HIP(vp8::launch_vp8_pack(d_mbs, (int)mb_count(), n, d_pack, host_dst, pack_cap(), s));
    return IK_OK;
}

int Vp8Work::write_packed(const uint8_t* pack_img, int quality, std::vector<uint8_t>& out) const {
    const vp8::QParams q = vp8::qparams_for_quality((float)quality);
    if (!vp8::write_webp_packed(w, h, q, pack_img, pack_cap(), -1, out))
        return fail(IK_ERR_DEVICE, "malformed VP8 macroblock stream from the device");
    return IK_OK;
}

// one image from device YUV420 planes, on the calling thread's stream
int webp_encode_gpu(const uint8_t* d_yuv, int w, int h, int quality, std::vector<uint8_t>& out) {
    if (w < 1 || h < 1 || w > 16383 || h > 16383) return fail(IK_ERR_TRANSFORM, "WebP dimensions %dx%d out of range", w, h);
    static thread_local std::map<int, Vp8Work> works;
    Vp8Work& wk = works[current_device()];
    hipStream_t s = thread_stream();
    if (!s) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    if (int rc = wk.reserve(w, h, 1, true)) return rc;
    if (int rc = wk.launch(d_yuv, 0, 1, quality, s)) return rc;
    if (wk.packable()) {
        if (int rc = wk.pack_to(wk.h_pack, 1, s)) return rc;
        IK_HIP(hipStreamSynchronize(s));
        return wk.write_packed(wk.h_pack, quality, out);
    }
    if (int rc = wk.fetch(1, s)) return rc;
    IK_HIP(hipStreamSynchronize(s));
    wk.write(0, quality, out);
    return IK_OK;
}

}  // namespace ik

using namespace ik;

extern "C" {

int ik_set_webp_encoder(int encoder) {
    if (encoder != IK_WEBP_LIBWEBP && encoder != IK_WEBP_GPU) return fail(IK_ERR_INVALID, "bad WebP encoder %d", encoder);
    (void)default_webp_encoder();
    g_webp_encoder.store(encoder);
    return IK_OK;
}

int ik_get_webp_encoder(void) { return default_webp_encoder(); }

int ik_webp_encode_gpu_device(const uint8_t* dev_yuv, uint32_t w, uint32_t h, int quality, uint8_t** out,
                              size_t* out_len) {
    IK_API_ENTER();
    if (!dev_yuv || !out || !out_len) return fail(IK_ERR_INVALID, "null pointer");
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    std::vector<uint8_t> bytes;
    if (int rc = webp_encode_gpu(dev_yuv, (int)w, (int)h, q, bytes)) return rc;
    *out = (uint8_t*)malloc(bytes.size() ? bytes.size() : 1);
    if (!*out) return fail(IK_ERR_NOMEM, "out of host memory");
    std::memcpy(*out, bytes.data(), bytes.size());
    *out_len = bytes.size();
    return IK_OK;
}

}  // extern "C"
