// Dev tool (not shipped): the scalar VP8 reference encoder + host bitstream writer
// as a plain shared library, so the bitstream can be checked against libwebp's
// decoder on a machine without a GPU (tools/vp8_cpu_check.py).
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <chrono>

#include "../rust-image-transform_amd/csrc/ik_vp8_enc.h"

namespace ik {
namespace vp8 {

// ---- scalar reference encoder --------------------------------------------------
// Scalar reference encoder over YUV420 planes (raster MB order, one MB at a time),
// returning the unfiltered reconstruction too.
void encode_frame_scalar(const uint8_t* Y, const uint8_t* U, const uint8_t* V, int width, int height,
                         const QParams& q, std::vector<MBOut>& mbs, std::vector<uint8_t>* recon_yuv) {
    const int mb_w = (width + 15) >> 4, mb_h = (height + 15) >> 4;
    const int yw = mb_w * 16, yh = mb_h * 16, cw = mb_w * 8, ch = mb_h * 8;
    const int uvw = (width + 1) >> 1, uvh = (height + 1) >> 1;
    std::vector<uint8_t> ry((size_t)yw * yh), ru((size_t)cw * ch), rv((size_t)cw * ch);
    mbs.assign((size_t)mb_w * mb_h, MBOut{});
    std::vector<uint8_t> top_nz((size_t)mb_w * 9, 0);
    for (int my = 0; my < mb_h; ++my) {
        uint8_t left_nz[9] = {0};
        for (int mx = 0; mx < mb_w; ++mx) {
            MBCtx c{};
            c.mb_x = mx; c.mb_y = my; c.mb_w = mb_w;
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) {
                    const int sx = std::min(mx * 16 + x, width - 1), sy = std::min(my * 16 + y, height - 1);
                    c.src_y[y * 16 + x] = Y[(size_t)sy * width + sx];
                }
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) {
                    const int sx = std::min(mx * 8 + x, uvw - 1), sy = std::min(my * 8 + y, uvh - 1);
                    c.src_u[y * 8 + x] = U[(size_t)sy * uvw + sx];
                    c.src_v[y * 8 + x] = V[(size_t)sy * uvw + sx];
                }
            // context rows / columns (libwebp ReconstructRow's fills)
            auto fill = [&](uint8_t* buf, const std::vector<uint8_t>& rec, int stride, int n, int extra) {
                const int x0 = mx * n, y0 = my * n;
                for (int x = -1; x < n + extra; ++x) {
                    int v;
                    if (my == 0) v = 127;
                    else if (x < 0) v = mx == 0 ? 129 : rec[(size_t)(y0 - 1) * stride + x0 - 1];
                    else if (x < n) v = rec[(size_t)(y0 - 1) * stride + x0 + x];
                    else v = mx == mb_w - 1 ? rec[(size_t)(y0 - 1) * stride + x0 + n - 1]
                                            : rec[(size_t)(y0 - 1) * stride + x0 + x];
                    buf[x + 1] = (uint8_t)v;
                }
                for (int y = 0; y < n; ++y)
                    buf[(y + 1) * kBps] = mx == 0 ? 129 : rec[(size_t)(y0 + y) * stride + x0 - 1];
            };
            fill(c.y, ry, yw, 16, 4);
            for (int r = 1; r < 4; ++r)
                for (int i = 0; i < 4; ++i) c.y[(4 * r) * kBps + 17 + i] = c.y[17 + i];
            fill(c.u, ru, cw, 8, 0);
            fill(c.v, rv, cw, 8, 0);
            for (int i = 0; i < 4; ++i) {
                c.top_bmodes[i] = my ? mbs[(size_t)(my - 1) * mb_w + mx].bmodes[12 + i] : B_DC;
                c.left_bmodes[i] = mx ? mbs[(size_t)my * mb_w + mx - 1].bmodes[i * 4 + 3] : B_DC;
            }
            std::memcpy(c.top_nz, &top_nz[(size_t)mx * 9], 9);
            std::memcpy(c.left_nz, left_nz, 9);
            MBOut& o = mbs[(size_t)my * mb_w + mx];
            encode_mb(c, q, kCoeffProbs0, o);
            // write the reconstruction back; carry non-zero contexts forward
            for (int y = 0; y < 16; ++y)
                std::memcpy(&ry[(size_t)(my * 16 + y) * yw + mx * 16], &c.y[(y + 1) * kBps + 1], 16);
            for (int y = 0; y < 8; ++y) {
                std::memcpy(&ru[(size_t)(my * 8 + y) * cw + mx * 8], &c.u[(y + 1) * kBps + 1], 8);
                std::memcpy(&rv[(size_t)(my * 8 + y) * cw + mx * 8], &c.v[(y + 1) * kBps + 1], 8);
            }
            const int first = o.ymode == B_PRED ? 0 : 1;
            uint8_t* t = &top_nz[(size_t)mx * 9];
            for (int i = 0; i < 4; ++i) {
                t[i] = last_nz(o.lv[12 + i], first) > first;
                left_nz[i] = last_nz(o.lv[i * 4 + 3], first) > first;
            }
            for (int chn = 0; chn < 2; ++chn)
                for (int i = 0; i < 2; ++i) {
                    t[4 + 2 * chn + i] = last_nz(o.lv[16 + 4 * chn + 2 + i], 0) > 0;
                    left_nz[4 + 2 * chn + i] = last_nz(o.lv[16 + 4 * chn + i * 2 + 1], 0) > 0;
                }
            if (o.ymode != B_PRED) t[8] = left_nz[8] = last_nz(o.lv[24], 0) > 0;
        }
    }
    if (recon_yuv) {
        recon_yuv->clear();
        for (int y = 0; y < height; ++y) recon_yuv->insert(recon_yuv->end(), &ry[(size_t)y * yw], &ry[(size_t)y * yw] + width);
        for (int y = 0; y < uvh; ++y) recon_yuv->insert(recon_yuv->end(), &ru[(size_t)y * cw], &ru[(size_t)y * cw] + uvw);
        for (int y = 0; y < uvh; ++y) recon_yuv->insert(recon_yuv->end(), &rv[(size_t)y * cw], &rv[(size_t)y * cw] + uvw);
    }
}

}  // namespace vp8
}  // namespace ik

extern "C" int vp8_dev_encode(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, float quality,
                              int filter_level, uint8_t* out, size_t cap, size_t* n, uint8_t* recon) {
    using namespace ik::vp8;
    const QParams q = qparams_for_quality(quality);
    std::vector<MBOut> mbs;
    std::vector<uint8_t> rec;
    encode_frame_scalar(y, u, v, w, h, q, mbs, &rec);
    std::vector<uint8_t> bytes;
    write_webp(w, h, q, mbs.data(), filter_level, bytes);
    *n = bytes.size();
    if (bytes.size() > cap) return 1;
    std::memcpy(out, bytes.data(), bytes.size());
    if (recon) std::memcpy(recon, rec.data(), rec.size());
    return 0;
}

// block_cost_fixed (the GPU kernel's register form) against the generic scan
extern "C" int vp8_dev_cost_pair(const int16_t* lv, int type, int first, int ctx, int* generic, int* fixed) {
    using namespace ik::vp8;
    const int last = last_nz(lv, first);
    *generic = block_cost(lv, first, last, ctx, type, kCoeffProbs0);
    switch (type * 2 + first) {
    case 0: *fixed = block_cost_fixed<0, 0>(lv, last, ctx); break;
    case 1: *fixed = block_cost_fixed<0, 1>(lv, last, ctx); break;
    case 2: *fixed = block_cost_fixed<1, 0>(lv, last, ctx); break;
    case 4: *fixed = block_cost_fixed<2, 0>(lv, last, ctx); break;
    case 6: *fixed = block_cost_fixed<3, 0>(lv, last, ctx); break;
    default: return 1;
    }
    return 0;
}

// pred4_px (the GPU kernel's per-pixel tap table) against pred4, on random contexts
extern "C" int vp8_dev_pred4_mismatches(unsigned seed, int trials) {
    using namespace ik::vp8;
    unsigned s = seed * 2654435761u + 1;
    int bad = 0;
    for (int t = 0; t < trials; ++t) {
        uint8_t buf[6 * kBps];
        for (auto& v : buf) { s = s * 1664525u + 1013904223u; v = (uint8_t)(s >> 24); }
        const uint8_t* d = buf + kBps + 1;
        for (int m = 0; m < NUM_BMODES; ++m) {
            uint8_t pr[16];
            pred4(m, d, pr);
            const int dcv = pred4_dc(d);
            for (int p = 0; p < 16; ++p) bad += pred4_px(m, p, d, dcv) != pr[p];
        }
    }
    return bad;
}

// host bitstream cost: mean seconds of write_webp_packed over `reps` runs on the
// scalar encoder's MB records (the host stage of the GPU WebP encoder)
extern "C" double vp8_dev_write_seconds(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h,
                                        float quality, int reps) {
    using namespace ik::vp8;
    const QParams q = qparams_for_quality(quality);
    std::vector<MBOut> mbs;
    encode_frame_scalar(y, u, v, w, h, q, mbs, nullptr);
    std::vector<uint8_t> bytes, pack;
    pack_mbs(mbs.data(), mbs.size(), pack);
    write_webp_packed(w, h, q, pack.data(), pack.size(), -1, bytes);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) write_webp_packed(w, h, q, pack.data(), pack.size(), -1, bytes);
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
}
