// ik_webp_gpu.cpp -- driver of the GPU WebP encoder (encode_image's WebP branch,
// reference src/transform.rs:129-137, as an alternative to libwebp on the host):
// device YUV420 planes -> k_vp8_diag wavefront (ik_vp8.hip) -> k_vp8_pack (compact
// MB records written into pinned host memory; a plain D2H of the records for
// frames over 4096 MBs) -> bitstream + RIFF on the host (ik_vp8_enc.cpp).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
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
        e = (s && (!strcmp(s, "gpu") || !strcmp(s, "1"))) ? IK_WEBP_GPU
            : (s && (!strcmp(s, "exact") || !strcmp(s, "2"))) ? IK_WEBP_EXACT : IK_WEBP_LIBWEBP;
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

// The host half of libwebp's segment set-up, from k_vp8_kmeans' record and
// cluster map (ik_vp8_analysis.hip): SetSegmentAlphas (analysis_enc.c),
// VP8SetSegmentParams with its pow() quality curve, SetupFilterStrength
// (filter_enc.c, sharpness 0: kLevelsFromDelta[0] is the identity on 0..63),
// SimplifySegments (quant_enc.c) and SetSegmentProbas (frame_enc.c).  libwebp's
// WebPConfigInit defaults: segments 4, sns_strength 50, filter_strength 60.
// seg: the image's k-means clusters in, final segment ids out.
void vp8_segment_setup(const vp8::SegRecord& r, float quality, uint8_t* seg, ik_vp8_segment_header* hd) {
    constexpr int nb = 4, sns = 50, filter_strength = 60;
    auto clip = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
    int mn = r.centers[0], mx = r.centers[0];
    for (int k = 0; k < nb; ++k) {
        mn = r.centers[k] < mn ? r.centers[k] : mn;
        mx = r.centers[k] > mx ? r.centers[k] : mx;
    }
    if (mx == mn) mx = mn + 1;
    int s_alpha[nb], s_beta[nb], quant[nb], fstr[nb];
    for (int k = 0; k < nb; ++k) {
        s_alpha[k] = clip(255 * (r.centers[k] - r.mid) / (mx - mn), -127, 127);
        s_beta[k] = clip(255 * (r.centers[k] - mn) / (mx - mn), 0, 255);
    }
    const double amp = 0.9 * sns / 100. / 128.;  // SNS_TO_DQ
    const double Q = quality / 100.;
    const double linear_c = (Q < 0.75) ? Q * (2. / 3.) : 2. * Q - 1.;
    const double c_base = pow(linear_c, 1 / 3.);
    for (int k = 0; k < nb; ++k) {
        const double expn = 1. - amp * s_alpha[k];
        const double c = pow(c_base, expn);
        quant[k] = clip((int)(127. * (1. - c)), 0, 127);
    }
    const int total = r.nmb > 0 ? r.nmb : 1;
    const int uv_alpha = (int)(r.uv_alpha_sum / (unsigned long long)total);
    // MID_ALPHA 64, MIN_ALPHA 30, MAX_ALPHA 100; MIN/MAX_DQ_UV -4 / 6
    int dq_uv_ac = (uv_alpha - 64) * (6 - (-4)) / (100 - 30);
    dq_uv_ac = clip(dq_uv_ac * sns / 100, -4, 6);
    const int dq_uv_dc = clip(-4 * sns / 100, -15, 15);
    const int level0 = 5 * filter_strength;
    for (int k = 0; k < nb; ++k) {
        const int qstep = vp8::kAcTable[clip(quant[k], 0, 127)] >> 2;
        const int base = qstep < 63 ? qstep : 63;
        const int f = base * level0 / (256 + s_beta[k]);
        fstr[k] = f < 2 ? 0 : (f > 63 ? 63 : f);  // FSTRENGTH_CUTOFF 2
    }
    hd->base_quant = quant[0];
    int map[nb] = {0, 1, 2, 3}, nfinal = 1;
    for (int s1 = 1; s1 < nb; ++s1) {
        int s2 = 0;
        bool found = false;
        for (; s2 < nfinal; ++s2)
            if (quant[s1] == quant[s2] && fstr[s1] == fstr[s2]) { found = true; break; }
        map[s1] = s2;
        if (!found) {
            if (nfinal != s1) { quant[nfinal] = quant[s1]; fstr[nfinal] = fstr[s1]; }
            ++nfinal;
        }
    }
    int cnt[nb] = {0, 0, 0, 0};
    for (int i = 0; i < r.nmb; ++i) {
        seg[i] = (uint8_t)(nfinal < nb ? map[seg[i]] : seg[i]);
        ++cnt[seg[i]];
    }
    for (int k = nfinal; k < nb; ++k) { quant[k] = quant[nfinal - 1]; fstr[k] = fstr[nfinal - 1]; }
    auto proba = [](int a, int b) { const int t = a + b; return t == 0 ? 255 : (255 * a + t / 2) / t; };
    hd->probs[0] = proba(cnt[0] + cnt[1], cnt[2] + cnt[3]);
    hd->probs[1] = proba(cnt[0], cnt[1]);
    hd->probs[2] = proba(cnt[2], cnt[3]);
    hd->num_segments = nfinal;
    hd->update_map = nfinal > 1 && (hd->probs[0] != 255 || hd->probs[1] != 255 || hd->probs[2] != 255);
    if (nfinal > 1 && !hd->update_map) std::memset(seg, 0, (size_t)r.nmb);  // ResetSegments
    for (int k = 0; k < nb; ++k) { hd->quant[k] = quant[k]; hd->fstrength[k] = fstr[k]; }
    hd->dq_uv_dc = dq_uv_dc;
    hd->dq_uv_ac = dq_uv_ac;
    hd->alpha = (int)(r.alpha_sum / (unsigned long long)total);
    hd->uv_alpha = uv_alpha;
}

}  // namespace ik

using namespace ik;

extern "C" {

int ik_set_webp_encoder(int encoder) {
    if (encoder != IK_WEBP_LIBWEBP && encoder != IK_WEBP_GPU && encoder != IK_WEBP_EXACT)
        return fail(IK_ERR_INVALID, "bad WebP encoder %d", encoder);
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
    const int nmb = (int)(((w + 15) >> 4) * ((h + 15) >> 4));
    hipStream_t s = thread_stream();
    if (!s) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    const size_t per = (size_t)nmb * n;
    uint8_t* d = nullptr;
    const size_t o_uva = (per + 255) & ~(size_t)255, o_seg = o_uva + ((2 * per + 255) & ~(size_t)255);
    const size_t o_rec = o_seg + ((per + 255) & ~(size_t)255), bytes = o_rec + sizeof(vp8::SegRecord) * n;
    IK_HIP(hipMalloc((void**)&d, bytes));
    std::vector<vp8::SegRecord> recs(n);
    hipError_t e = vp8::launch_vp8_analysis(dev_yuv, yuv_stride, (int)n, (int)w, (int)h, d, (uint16_t*)(d + o_uva),
                                            d + o_seg, (vp8::SegRecord*)(d + o_rec), s);
    if (e == hipSuccess) e = hipMemcpyAsync(seg, d + o_seg, per, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(recs.data(), d + o_rec, sizeof(vp8::SegRecord) * n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(IK_ERR_DEVICE, "VP8 analysis: %s", hipGetErrorString(e));
    for (uint32_t i = 0; i < n; ++i) vp8_segment_setup(recs[i], quality, seg + (size_t)nmb * i, hdr + i);
    return IK_OK;
}

}  // extern "C"
