// ik_vp8d_host.cpp -- host half of the GPU WebP (VP8 lossy) decoder: decode_image's WebP
// branch (reference src/transform.rs:31 load_from_memory_with_format -> image 0.25.8 ->
// WebP), with the pixels of libwebp's WebPDecodeRGB (tests/test_gpu_webp_decode.py).
//
// The host reads what is serial: the RIFF container, the frame header, partition 0
// (segment / filter / quantiser headers, the coefficient probabilities, every
// macroblock's modes; libwebp vp8_dec.c VP8GetHeaders, ParseIntraMode, quant_dec.c
// VP8ParseQuant, tree_dec.c VP8ParseProba, frame_dec.c PrecomputeFilterStrengths) and
// the token partitions (ParseResiduals), an arithmetic code that is one dependent
// chain per partition (libwebp writes one): a wave decoding it on the scalar unit
// took 776 ms for a 4096^2 frame that libwebp decodes whole in 72 ms on one core.  It
// hands the device each MB's non-zero dequantised coefficients; the device
// reconstructs and loop-filters the frame and converts it to RGB (ik_vp8d.hip).
// Files it does not cover -- lossless (VP8L), alpha, animation, anything its parser
// finds unusual, data that runs out -- go to the host decoder (decode_webp), which
// then gives libwebp's answer, error message included.
#include <chrono>
#include <cstdio>
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

// ---- the token partitions (vp8_dec.c VP8DecodeMB, ParseResiduals, GetCoeffs,
// GetLargeValue) into each MB's non-zero dequantised coefficients ----
struct Tokens {
    std::vector<uint32_t> coef;   // (value << 16) | position in the MB's 384
    std::vector<uint32_t> at;     // per MB its first entry, then the total
    std::vector<uint8_t> flags;   // per MB: some coefficient is non-zero
};

constexpr uint8_t kCat3[] = {173, 148, 140, 0}, kCat4[] = {176, 155, 140, 135, 0},
                  kCat5[] = {180, 157, 141, 134, 130, 0},
                  kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};
constexpr const uint8_t* kCat[4] = {kCat3, kCat4, kCat5, kCat6};

struct TokenReader {
    BitReader br;
    HostSrc src;
    const uint8_t* proba;  // DFrame::proba rows
    std::vector<uint32_t>* out;

    int bit(int p) { return br_bit(br, src, p); }
    const uint8_t* row(int type, int b, int ctx) const { return proba + ((type * 8 + b) * 3 + ctx) * 16; }
    int large_value(const uint8_t* p) {
        if (!bit(p[3])) return !bit(p[4]) ? 2 : 3 + bit(p[5]);
        if (!bit(p[6])) {
            if (!bit(p[7])) return 5 + bit(159);
            int v = 7 + 2 * bit(165);
            return v + bit(145);
        }
        const int b1 = bit(p[8]);
        const int b0 = bit(p[9 + b1]);
        const int cat = 2 * b1 + b0;
        int v = 0;
        for (const uint8_t* t = kCat[cat]; *t; ++t) v += v + bit(*t);
        return v + 3 + (8 << cat);
    }
    // one block from position n: its entries at base + zigzag(n); returns the position
    // after its last token, *dc the stored value of position 0
    int coeffs(int type, int ctx, int dq0, int dq1, int n, uint32_t base, int* dc) {
        const uint8_t* p = row(type, band(n), ctx);
        for (; n < 16; ++n) {
            if (!bit(p[0])) return n;
            while (!bit(p[1])) {
                if (++n == 16) return 16;
                p = row(type, band(n), 0);
            }
            int v;
            const uint8_t* next;
            if (!bit(p[2])) {
                v = 1;
                next = row(type, band(n + 1), 1);
            } else {
                v = large_value(p);
                next = row(type, band(n + 1), 2);
            }
            const int16_t q = (int16_t)((bit(0x80) ? -v : v) * (n > 0 ? dq1 : dq0));
            if (n == 0) *dc = q;
            out->push_back((uint32_t)(uint16_t)q << 16 | (base + (uint32_t)zigzag(n)));
            p = next;
        }
        return 16;
    }
};

// contexts packed as libwebp's: bits 0-3 luma columns / rows, 4-5 U, 6-7 V, 8 the Y2 block
bool decode_tokens(const uint8_t* b, const Parsed& P, Tokens& T) {
    const DFrame& fr = P.fr;
    const int mb_w = fr.mb_w, mb_h = fr.mb_h;
    const size_t nmb = (size_t)mb_w * mb_h;
    T.coef.clear();
    T.at.resize(nmb + 1);
    T.flags.resize(nmb);
    std::vector<uint32_t> tnz(mb_w, 0);
    TokenReader R[8];
    for (int p = 0; p < fr.num_parts; ++p) {
        R[p].src = HostSrc{b};
        R[p].proba = fr.proba;
        R[p].out = &T.coef;
        br_init(R[p].br, R[p].src, fr.part_off[p], fr.part_end[p]);
    }
    for (int mb_y = 0; mb_y < mb_h; ++mb_y) {
        TokenReader& t = R[mb_y & (fr.num_parts - 1)];
        uint32_t l = 0;
        for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
            const size_t mb = (size_t)mb_y * mb_w + mb_x;
            const DMB& m = P.mbs[mb];
            T.at[mb] = (uint32_t)T.coef.size();
            uint32_t tc = tnz[mb_x];
            int any = 0;
            if (!(fr.use_skip && m.skip)) {
                const DSeg& q = fr.seg[m.seg];
                int first = 0, ytype = 3;
                if (!m.is_i4) {  // the Y2 block, then its inverse WHT into the blocks' DCs
                    const size_t y2 = T.coef.size();
                    int dcv = 0;
                    const int nz = t.coeffs(1, (int)((tc >> 8) & 1) + (int)((l >> 8) & 1), q.y2[0], q.y2[1], 0, 0, &dcv);
                    const uint32_t bit = nz > 0;
                    tc = (tc & ~0x100u) | bit << 8;
                    l = (l & ~0x100u) | bit << 8;
                    int16_t dc[16] = {0}, out[256];
                    for (size_t k = y2; k < T.coef.size(); ++k) dc[T.coef[k] & 15] = (int16_t)(T.coef[k] >> 16);
                    T.coef.resize(y2);
                    vp8x::itransform_wht(dc, out);
                    for (int k = 0; k < 16; ++k)
                        if (out[16 * k]) {
                            T.coef.push_back((uint32_t)(uint16_t)out[16 * k] << 16 | (uint32_t)(16 * k));
                            any = 1;
                        }
                    first = 1;
                    ytype = 0;
                }
                for (int by = 0; by < 4; ++by) {
                    uint32_t lb = (l >> by) & 1;
                    for (int bx = 0; bx < 4; ++bx) {
                        int dcv = 0;
                        const int nz = t.coeffs(ytype, (int)lb + (int)((tc >> bx) & 1), q.y1[0], q.y1[1], first,
                                                (uint32_t)(4 * by + bx) * 16, &dcv);
                        lb = nz > first;
                        tc = (tc & ~(1u << bx)) | lb << bx;
                        any |= nz > 1 || (first == 0 && dcv != 0);
                    }
                    l = (l & ~(1u << by)) | lb << by;
                }
                for (int c = 0; c < 2; ++c) {
                    const int sh = 4 + 2 * c;
                    for (int by = 0; by < 2; ++by) {
                        uint32_t lb = (l >> (sh + by)) & 1;
                        for (int bx = 0; bx < 2; ++bx) {
                            int dcv = 0;
                            const int nz = t.coeffs(2, (int)lb + (int)((tc >> (sh + bx)) & 1), q.uv[0], q.uv[1], 0,
                                                    (uint32_t)(16 + 4 * c + 2 * by + bx) * 16, &dcv);
                            lb = nz > 0;
                            tc = (tc & ~(1u << (sh + bx))) | lb << (sh + bx);
                            any |= nz > 1 || dcv != 0;
                        }
                        l = (l & ~(1u << (sh + by))) | lb << (sh + by);
                    }
                }
            } else {  // a skipped MB clears the contexts; the Y2 one only for i16
                const uint32_t keep = m.is_i4 ? 0x100u : 0u;
                tc &= keep;
                l &= keep;
            }
            tnz[mb_x] = tc;
            T.flags[mb] = (uint8_t)any;
            if (t.br.eof) return false;  // (libwebp: "Premature end-of-file encountered.")
        }
    }
    T.at[nmb] = (uint32_t)T.coef.size();
    return true;
}

size_t up256(size_t v) { return (v + 255) & ~size_t(255); }

}  // namespace

int webp_decode_mode() {  // IK_WEBP_DECODE: host / gpu (no host fallback: tests) / auto (default)
    const char* e = getenv("IK_WEBP_DECODE");
    if (e && !std::strcmp(e, "host")) return 0;
    if (e && !std::strcmp(e, "gpu")) return 2;
    return 1;
}

// auto: the device path from this many pixels on.  Measured per frame (decode_image,
// one request; profiles/r06_webp_decode.log): 4096x4096 39.6 ms against libwebp's 62.2,
// 3000x2000 16.9 / 19.5, 2560x1440 11.4 / 12.0, 1920x1080 7.3 / 7.1, 512x512 1.65 / 0.93.
// The host's tokens cost ~1.6 ms per MPix and the reconstruction wavefront
// (mb_w + 2 mb_h) MB steps of ~12-25 us; libwebp ~4 ms per MPix.
constexpr uint64_t kWebpGpuMinPixels = 3000000;

int decode_webp_device(const uint8_t* b, size_t n, ik_image** out) {
    if (!webp_decode_mode()) return kVp8dHost;
    size_t off = 0, len = 0;
    uint32_t cw, ch;
    if (!find_vp8(b, n, off, len, cw, ch)) return kVp8dHost;
    const int mode = webp_decode_mode();
    if (mode == 1) {
        const uint32_t w = le16(b + off + 6) & 0x3fff, h = le16(b + off + 8) & 0x3fff;
        if ((uint64_t)w * h < kWebpGpuMinPixels) return kVp8dHost;
    }
    thread_local Parsed P;
    thread_local Tokens T;
    struct Trim {  // (per-thread buffers: released after frames over 16 MiB of them)
        ~Trim() {
            if (P.mbs.capacity() * sizeof(DMB) + T.coef.capacity() * 4 > (16u << 20)) {
                std::vector<DMB>().swap(P.mbs);
                std::vector<uint32_t>().swap(T.coef);
                std::vector<uint32_t>().swap(T.at);
                std::vector<uint8_t>().swap(T.flags);
            }
        }
    } trim;
    static const bool timing = getenv("IK_TIMING") != nullptr;  // dev: phase times to stderr
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = timing ? now() : 0;
    if (!parse_vp8(b, off, len, cw, ch, P)) return kVp8dHost;
    const double t1 = timing ? now() : 0;
    if (!decode_tokens(b, P, T)) return kVp8dHost;
    const double t2 = timing ? now() : 0;
    const DFrame& fr = P.fr;
    const size_t nmb = (size_t)fr.mb_w * fr.mb_h;

    // staged (one H2D): [DImg][DFrame][DMB x nmb][flags][entry starts][entries]
    const size_t o_fr = up256(sizeof(DImg));
    const size_t o_mb = o_fr + up256(sizeof(DFrame));
    const size_t o_flags = o_mb + up256(nmb * sizeof(DMB));
    const size_t o_at = o_flags + up256(nmb);
    const size_t o_coef = o_at + up256((nmb + 1) * 4);
    const size_t stage = o_coef + up256(T.coef.size() * 4 + 4);
    // device work: [ticket, error, progress per MB row][Y][U][V][top rows]
    const uint32_t ys = (uint32_t)fr.mb_w * 16, uvs = (uint32_t)fr.mb_w * 8;
    const size_t o_sync = stage;
    const size_t o_y = o_sync + up256(4 * (2 + (size_t)fr.mb_h));
    const size_t o_u = o_y + up256((size_t)ys * fr.mb_h * 16);
    const size_t o_v = o_u + up256((size_t)uvs * fr.mb_h * 8);
    const size_t o_top = o_v + up256((size_t)uvs * fr.mb_h * 8);
    const size_t total = o_top + up256((size_t)2 * fr.mb_w * 32);

    ik_image* img = nullptr;
    int st = alloc_image((uint32_t)fr.w, (uint32_t)fr.h, 3, &img);
    if (st) return st;
    uint8_t* d = scratch_slot(kScratchVp8d, total);
    uint8_t* h = d ? pinned_slot(kPinnedVp8d, stage) : nullptr;
    if (!d || !h) {
        ik_image_free(img);
        return d ? IK_ERR_NOMEM : fail(IK_ERR_DEVICE, "cannot allocate the WebP decoder's device work area");
    }
    hipStream_t s = thread_stream();
    (void)hipStreamSynchronize(s);  // (the pinned area may still feed an earlier copy)
    DImg di{};
    di.fr = reinterpret_cast<const DFrame*>(d + o_fr);
    di.mbs = reinterpret_cast<const DMB*>(d + o_mb);
    di.flags = d + o_flags;
    di.coef_at = reinterpret_cast<const uint32_t*>(d + o_at);
    di.coef = reinterpret_cast<const uint32_t*>(d + o_coef);
    di.y = d + o_y;
    di.u = d + o_u;
    di.v = d + o_v;
    di.top = d + o_top;
    di.out = img->d;
    di.ys = ys;
    di.uvs = uvs;
    di.out_pitch = (uint32_t)img->pitch;
    di.row0 = 0;
    di.rows = (uint32_t)fr.mb_h;
    uint32_t* const sync = reinterpret_cast<uint32_t*>(d + o_sync);
    di.err = sync + 1;
    di.prog = sync + 2;
    std::memcpy(h, &di, sizeof(di));
    std::memcpy(h + o_fr, &fr, sizeof(DFrame));
    std::memcpy(h + o_mb, P.mbs.data(), nmb * sizeof(DMB));
    std::memcpy(h + o_flags, T.flags.data(), nmb);
    std::memcpy(h + o_at, T.at.data(), (nmb + 1) * 4);
    if (!T.coef.empty()) std::memcpy(h + o_coef, T.coef.data(), T.coef.size() * 4);
    const DImg* dimg = reinterpret_cast<const DImg*>(d);
    const double t3 = timing ? now() : 0;
    hipError_t e = hipMemcpyAsync(d, h, o_coef + T.coef.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(sync, 0, 4 * (2 + (size_t)fr.mb_h), s);
    if (timing && e == hipSuccess) e = hipStreamSynchronize(s);
    const double t4 = timing ? now() : 0;
    if (e == hipSuccess) e = launch_vp8d_recon(dimg, 1, (uint32_t)fr.mb_h, sync, s);
    if (timing && e == hipSuccess) e = hipStreamSynchronize(s);
    const double t5 = timing ? now() : 0;
    if (e == hipSuccess) e = launch_vp8d_rgb(dimg, 1, fr.h, s);
    uint32_t* const herr = reinterpret_cast<uint32_t*>(h + stage - 4);  // (the staged area's last word: free)
    if (e == hipSuccess) e = hipMemcpyAsync(herr, sync + 1, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (timing)
        fprintf(stderr, "vp8d %dx%d: parse %.3f tokens %.3f (%zu coefs) stage %.3f h2d %.3f recon %.3f rgb %.3f ms\n", fr.w,
                fr.h, t1 - t0, t2 - t1, T.coef.size(), t3 - t2, t4 - t3, t5 - t4, now() - t5);
    if (e != hipSuccess) {
        ik_image_free(img);
        return hip_fail(e, "WebP decode launches");
    }
    if (*herr) {  // a row's wait timed out: the device is too busy or something is wrong; libwebp decides
        ik_image_free(img);
        return kVp8dHost;
    }
    *out = img;
    return IK_OK;
}

}  // namespace ik
