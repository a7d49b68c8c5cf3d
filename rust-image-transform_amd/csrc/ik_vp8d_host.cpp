// ik_vp8d_host.cpp -- host half of the GPU WebP (VP8 lossy) decoder: decode_image's WebP
// branch (reference src/transform.rs:31 load_from_memory_with_format -> image 0.25.8 ->
// WebP), with the pixels of libwebp's WebPDecodeRGB (tests/test_gpu_webp_decode.py).
//
// The host reads what is inherently serial and small: the RIFF container, the frame
// header and partition 0 (segment / filter / quantiser headers, the coefficient
// probabilities, every macroblock's modes; libwebp vp8_dec.c VP8GetHeaders,
// ParseIntraMode, quant_dec.c VP8ParseQuant, tree_dec.c VP8ParseProba, frame_dec.c
// PrecomputeFilterStrengths).  The device decodes the token partitions,
// reconstructs and loop-filters the frame and converts it to RGB (ik_vp8d.hip).
// Files it does not cover -- lossless (VP8L), alpha, animation, anything its parser
// finds unusual, data that runs out -- go to the host decoder (decode_webp), which
// then gives libwebp's answer, error message included.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ik_runtime.h"
#include "ik_vp8d_gpu.h"

namespace ik {

namespace {

using namespace vp8d;

uint32_t le16(const uint8_t* p) { return p[0] | (uint32_t)p[1] << 8; }
uint32_t le24(const uint8_t* p) { return le16(p) | (uint32_t)p[2] << 16; }
uint32_t le32(const uint8_t* p) { return le24(p) | (uint32_t)p[3] << 24; }

// the "VP8 " payload of a simple file, or of an extended one without alpha or
// animation (libwebp webp_dec.c ParseRIFF / ParseVP8X / ParseOptionalChunks /
// ParseVP8Header); false: leave the file to the host decoder
bool find_vp8(const uint8_t* b, size_t n, size_t& off, size_t& len, uint32_t& cw, uint32_t& ch) {
    cw = ch = 0;
    if (n < 20 || std::memcmp(b, "RIFF", 4) || std::memcmp(b + 8, "WEBP", 4)) return false;
    const size_t riff = le32(b + 4);
    if (riff < 12 || riff + 8 > n) return false;
    const size_t end = riff + 8;  // (libwebp reads no further than the RIFF size)
    size_t p = 12;
    if (p + 8 > end) return false;
    if (!std::memcmp(b + p, "VP8X", 4)) {
        const size_t sz = le32(b + p + 4);
        if (sz < 10 || p + 8 + sz > end) return false;
        const uint8_t flags = b[p + 8];
        if (flags & (0x10 | 0x02)) return false;  // alpha, animation
        cw = 1 + le24(b + p + 12);
        ch = 1 + le24(b + p + 15);
        p += 8 + sz + (sz & 1);
        for (;;) {
            if (p + 8 > end) return false;
            if (!std::memcmp(b + p, "VP8 ", 4)) break;
            if (!std::memcmp(b + p, "VP8L", 4) || !std::memcmp(b + p, "ALPH", 4) || !std::memcmp(b + p, "ANIM", 4) ||
                !std::memcmp(b + p, "ANMF", 4))
                return false;
            const size_t csz = le32(b + p + 4);
            p += 8 + csz + (csz & 1);
        }
    } else if (std::memcmp(b + p, "VP8 ", 4)) {
        return false;
    }
    len = le32(b + p + 4);
    off = p + 8;
    return len >= 10 && off + len <= end;
}

struct Parsed {
    DFrame fr;
    std::vector<DMB> mbs;
};

// frame header + partition 0; false: leave the file to the host decoder
bool parse_vp8(const uint8_t* b, size_t off, size_t len, uint32_t cw, uint32_t ch, Parsed& P) {
    const uint8_t* f = b + off;
    const uint32_t bits = le24(f);
    const int key = !(bits & 1), profile = (bits >> 1) & 7, show = (bits >> 4) & 1;
    const uint32_t part0 = bits >> 5;
    if (!key || profile > 3 || !show) return false;
    if (f[3] != 0x9d || f[4] != 0x01 || f[5] != 0x2a) return false;
    const int w = (int)(le16(f + 6) & 0x3fff), h = (int)(le16(f + 8) & 0x3fff);
    if (!w || !h) return false;
    if (cw && (cw != (uint32_t)w || ch != (uint32_t)h)) return false;
    if (part0 >= len || 10 + (size_t)part0 > len) return false;
    DFrame& fr = P.fr;
    std::memset(&fr, 0, sizeof(fr));
    fr.w = w;
    fr.h = h;
    fr.mb_w = (w + 15) >> 4;
    fr.mb_h = (h + 15) >> 4;
    const HostSrc src{b};
    BitReader br;
    const uint32_t p0 = (uint32_t)(off + 10), p0_end = p0 + part0;
    br_init(br, src, p0, p0_end);
    auto get = [&] { return br_bit(br, src, 0x80); };
    br_value(br, src, 1);  // colour space
    br_value(br, src, 1);  // clamping type

    // segment header (ParseSegmentHeader; the defaults of ResetSegmentHeader)
    int use_segment = get(), update_map = 0, absolute = 1;
    int quantizer[4] = {0, 0, 0, 0}, filter_strength[4] = {0, 0, 0, 0};
    int seg_p[3] = {255, 255, 255};
    if (use_segment) {
        update_map = get();
        if (get()) {
            absolute = get();
            for (int s = 0; s < 4; ++s) quantizer[s] = get() ? br_signed_value(br, src, 7) : 0;
            for (int s = 0; s < 4; ++s) filter_strength[s] = get() ? br_signed_value(br, src, 6) : 0;
        }
        if (update_map)
            for (int s = 0; s < 3; ++s) seg_p[s] = get() ? br_value(br, src, 8) : 255;
    }
    // filter header (ParseFilterHeader)
    const int simple = get(), level = br_value(br, src, 6), sharpness = br_value(br, src, 3);
    const int use_lf_delta = get();
    int ref_lf_delta0 = 0, mode_lf_delta0 = 0;
    if (use_lf_delta && get()) {
        for (int i = 0; i < 4; ++i)
            if (get()) {
                const int v = br_signed_value(br, src, 6);
                if (i == 0) ref_lf_delta0 = v;
            }
        for (int i = 0; i < 4; ++i)
            if (get()) {
                const int v = br_signed_value(br, src, 6);
                if (i == 0) mode_lf_delta0 = v;
            }
    }
    fr.filter_type = level == 0 ? 0 : simple ? 1 : 2;
    if (br.eof) return false;

    // token partitions (ParsePartitions): any clipped or empty one is left to libwebp
    const int last = (1 << br_value(br, src, 2)) - 1;
    fr.num_parts = last + 1;
    {
        const size_t start = off + 10 + part0, pend = off + len;
        if (pend - start < 3 * (size_t)last) return false;
        size_t ps = start + 3 * (size_t)last;
        for (int p = 0; p < last; ++p) {
            const size_t psize = le24(b + start + 3 * p);
            if (psize > pend - ps) return false;
            fr.part_off[p] = (uint32_t)ps;
            fr.part_end[p] = (uint32_t)(ps + psize);
            ps += psize;
        }
        if (ps >= pend) return false;
        fr.part_off[last] = (uint32_t)ps;
        fr.part_end[last] = (uint32_t)pend;
    }

    // quantisers (VP8ParseQuant)
    const int base_q0 = br_value(br, src, 7);
    const int dqy1_dc = get() ? br_signed_value(br, src, 4) : 0;
    const int dqy2_dc = get() ? br_signed_value(br, src, 4) : 0;
    const int dqy2_ac = get() ? br_signed_value(br, src, 4) : 0;
    const int dquv_dc = get() ? br_signed_value(br, src, 4) : 0;
    const int dquv_ac = get() ? br_signed_value(br, src, 4) : 0;
    auto clip = [](int v, int m) { return v < 0 ? 0 : v > m ? m : v; };
    for (int s = 0; s < 4; ++s) {
        int q;
        if (use_segment) {
            q = quantizer[s];
            if (!absolute) q += base_q0;
        } else {
            q = base_q0;  // (every segment: libwebp copies segment 0's matrices)
        }
        DSeg& g = fr.seg[s];
        g.y1[0] = (int16_t)kDcTable[clip(q + dqy1_dc, 127)];
        g.y1[1] = (int16_t)kAcTable[clip(q, 127)];
        g.y2[0] = (int16_t)(kDcTable[clip(q + dqy2_dc, 127)] * 2);
        int y2ac = (kAcTable[clip(q + dqy2_ac, 127)] * 101581) >> 16;
        g.y2[1] = (int16_t)(y2ac < 8 ? 8 : y2ac);
        g.uv[0] = (int16_t)kDcTable[clip(q + dquv_dc, 117)];
        g.uv[1] = (int16_t)kAcTable[clip(q + dquv_ac, 127)];
        // loop-filter strengths (PrecomputeFilterStrengths)
        int base_level = level;
        if (use_segment) {
            base_level = filter_strength[s];
            if (!absolute) base_level += level;
        }
        for (int i4 = 0; i4 <= 1; ++i4) {
            int lv = base_level;
            if (use_lf_delta) {
                lv += ref_lf_delta0;
                if (i4) lv += mode_lf_delta0;
            }
            lv = lv < 0 ? 0 : lv > 63 ? 63 : lv;
            if (lv > 0) {
                int il = lv;
                if (sharpness > 0) {
                    il >>= sharpness > 4 ? 2 : 1;
                    if (il > 9 - sharpness) il = 9 - sharpness;
                }
                if (il < 1) il = 1;
                g.ilevel[i4] = (uint8_t)il;
                g.limit[i4] = (uint8_t)(2 * lv + il);
                g.hev[i4] = (uint8_t)(lv >= 40 ? 2 : lv >= 15 ? 1 : 0);
            } else {
                g.limit[i4] = 0;
            }
        }
    }
    get();  // update_proba (ignored on key frames)
    // coefficient probabilities (VP8ParseProba), rows padded to 16
    for (int i = 0; i < 1056; ++i) {
        const int v = br_bit(br, src, kCoeffUpdateProbs[i]) ? br_value(br, src, 8) : kCoeffProbs0[i];
        fr.proba[(i / 11) * 16 + i % 11] = (uint8_t)v;
    }
    fr.use_skip = get();
    const int skip_p = fr.use_skip ? br_value(br, src, 8) : 0;
    if (br.eof) return false;

    // every MB's modes (ParseIntraMode; left contexts reset per row, top per frame)
    const int nmb = fr.mb_w * fr.mb_h;
    P.mbs.assign(nmb, DMB{});
    std::vector<uint8_t> intra_t(4 * fr.mb_w, B_DC);
    for (int mb_y = 0; mb_y < fr.mb_h; ++mb_y) {
        uint8_t intra_l[4] = {B_DC, B_DC, B_DC, B_DC};
        for (int mb_x = 0; mb_x < fr.mb_w; ++mb_x) {
            DMB& m = P.mbs[(size_t)mb_y * fr.mb_w + mb_x];
            uint8_t* top = intra_t.data() + 4 * mb_x;
            if (update_map)
                m.seg = (uint8_t)(!br_bit(br, src, seg_p[0]) ? br_bit(br, src, seg_p[1])
                                                             : br_bit(br, src, seg_p[2]) + 2);
            if (fr.use_skip) m.skip = (uint8_t)br_bit(br, src, skip_p);
            m.is_i4 = (uint8_t)!br_bit(br, src, 145);
            if (!m.is_i4) {
                const int ymode = br_bit(br, src, 156) ? (br_bit(br, src, 128) ? TM_PRED : H_PRED)
                                                       : (br_bit(br, src, 163) ? V_PRED : DC_PRED);
                m.ymode = (uint8_t)ymode;
                std::memset(top, ymode, 4);
                std::memset(intra_l, ymode, 4);
                std::memset(m.bmodes, ymode, 16);
            } else {
                for (int y = 0; y < 4; ++y) {
                    int ymode = intra_l[y];
                    for (int x = 0; x < 4; ++x) {
                        const uint8_t* pr = kBModeProbs + (top[x] * 10 + ymode) * 9;
                        ymode = !br_bit(br, src, pr[0])   ? B_DC
                              : !br_bit(br, src, pr[1])   ? B_TM
                              : !br_bit(br, src, pr[2])   ? B_VE
                              : !br_bit(br, src, pr[3])   ? (!br_bit(br, src, pr[4])   ? B_HE
                                                             : !br_bit(br, src, pr[5]) ? B_RD
                                                                                       : B_VR)
                              : !br_bit(br, src, pr[6])   ? B_LD
                              : !br_bit(br, src, pr[7])   ? B_VL
                              : !br_bit(br, src, pr[8])   ? B_HD
                                                          : B_HU;
                        top[x] = (uint8_t)ymode;
                        m.bmodes[4 * y + x] = (uint8_t)ymode;
                    }
                    intra_l[y] = (uint8_t)ymode;
                }
            }
            m.uvmode = (uint8_t)(!br_bit(br, src, 142)   ? DC_PRED
                                 : !br_bit(br, src, 114) ? V_PRED
                                 : br_bit(br, src, 183)  ? TM_PRED
                                                         : H_PRED);
        }
        if (br.eof) return false;  // (libwebp: "Premature end-of-partition0 encountered.")
    }
    return true;
}

size_t up16(size_t v) { return (v + 15) & ~size_t(15); }
size_t up256(size_t v) { return (v + 255) & ~size_t(255); }

}  // namespace

int webp_decode_mode() {  // IK_WEBP_DECODE: host / gpu (no host fallback: tests) / auto (default)
    const char* e = getenv("IK_WEBP_DECODE");
    if (e && !std::strcmp(e, "host")) return 0;
    if (e && !std::strcmp(e, "gpu")) return 2;
    return 1;
}

int decode_webp_device(const uint8_t* b, size_t n, ik_image** out) {
    if (!webp_decode_mode()) return kVp8dHost;
    size_t off = 0, len = 0;
    uint32_t cw, ch;
    if (!find_vp8(b, n, off, len, cw, ch)) return kVp8dHost;
    thread_local Parsed P;
    if (!parse_vp8(b, off, len, cw, ch, P)) return kVp8dHost;
    const DFrame& fr = P.fr;
    const size_t nmb = (size_t)fr.mb_w * fr.mb_h;

    // staged (one H2D): [DImg][DFrame][DMB x nmb][file]
    const size_t o_fr = up256(sizeof(DImg));
    const size_t o_mb = o_fr + up256(sizeof(DFrame));
    const size_t o_file = o_mb + up256(nmb * sizeof(DMB));
    const size_t stage = o_file + up16(off + len) + 16;
    // device work: [coefficients][flags][Y][U][V][top rows][error word]
    const uint32_t ys = (uint32_t)fr.mb_w * 16, uvs = (uint32_t)fr.mb_w * 8;
    const size_t o_coef = up256(stage);
    const size_t o_flags = o_coef + up256(nmb * 384 * sizeof(int16_t));
    const size_t o_y = o_flags + up256(nmb);
    const size_t o_u = o_y + up256((size_t)ys * fr.mb_h * 16);
    const size_t o_v = o_u + up256((size_t)uvs * fr.mb_h * 8);
    const size_t o_top = o_v + up256((size_t)uvs * fr.mb_h * 8);
    const size_t o_err = o_top + up256((size_t)2 * fr.mb_w * 32);
    const size_t total = o_err + 256;

    ik_image* img = nullptr;
    int st = alloc_image((uint32_t)fr.w, (uint32_t)fr.h, 3, &img);
    if (st) return st;
    uint8_t* d = scratch_slot(kScratchVp8d, total);
    uint8_t* h = d ? pinned_slot(kPinnedVp8d, stage + 16) : nullptr;
    if (!d || !h) {
        ik_image_free(img);
        return d ? IK_ERR_NOMEM : fail(IK_ERR_DEVICE, "cannot allocate the WebP decoder's device work area");
    }
    hipStream_t s = thread_stream();
    (void)hipStreamSynchronize(s);  // (the pinned area may still feed an earlier copy)
    DImg di{};
    di.fr = reinterpret_cast<const DFrame*>(d + o_fr);
    di.mbs = reinterpret_cast<const DMB*>(d + o_mb);
    di.file = d + o_file;
    di.coef = reinterpret_cast<int16_t*>(d + o_coef);
    di.flags = d + o_flags;
    di.y = d + o_y;
    di.u = d + o_u;
    di.v = d + o_v;
    di.top = d + o_top;
    di.out = img->d;
    di.ys = ys;
    di.uvs = uvs;
    di.out_pitch = (uint32_t)img->pitch;
    di.err = reinterpret_cast<uint32_t*>(d + o_err);
    std::memcpy(h, &di, sizeof(di));
    std::memcpy(h + o_fr, &fr, sizeof(DFrame));
    std::memcpy(h + o_mb, P.mbs.data(), nmb * sizeof(DMB));
    std::memcpy(h + o_file, b, off + len);
    std::memset(h + o_file + off + len, 0, stage - o_file - off - len);
    uint32_t* herr = reinterpret_cast<uint32_t*>(h + stage);
    const DImg* dimg = reinterpret_cast<const DImg*>(d);
    hipError_t e = hipMemcpyAsync(d, h, stage, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(d + o_err, 0, 4, s);
    if (e == hipSuccess) e = launch_vp8d_tokens(dimg, 1, s);
    if (e == hipSuccess) e = launch_vp8d_recon(dimg, 1, s);
    if (e == hipSuccess) e = launch_vp8d_rgb(dimg, 1, fr.h, s);
    if (e == hipSuccess) e = hipMemcpyAsync(herr, d + o_err, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        ik_image_free(img);
        return hip_fail(e, "WebP decode launches");
    }
    if (*herr) {  // a token partition ran out: libwebp's verdict (and message) decides
        ik_image_free(img);
        return kVp8dHost;
    }
    if (P.mbs.capacity() > (1u << 20)) std::vector<DMB>().swap(P.mbs);
    *out = img;
    return IK_OK;
}

}  // namespace ik
