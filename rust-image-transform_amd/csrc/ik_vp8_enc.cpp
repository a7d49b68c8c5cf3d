// ik_vp8_enc.cpp -- host half of the GPU WebP encoder (see ik_vp8_enc.h): token
// statistics and coefficient-probability updates, the RFC 6386 boolean encoder,
// the key-frame header, per-MB mode coding, the token partition and the RIFF
// container.  Plain C++ (no HIP): tests/test_vp8_host.py builds it with the scalar
// macroblock reference (tools/vp8_cpu_check.cpp) to check the bitstream against
// libwebp's decoder without a GPU.
#include "ik_vp8_enc.h"

#include <cmath>
#include <cstring>

namespace ik {
namespace vp8 {
namespace {

// RFC 6386 section 7.3 boolean encoder
struct BoolEnc {
    std::vector<uint8_t> out;
    uint32_t range = 255, bottom = 0;
    int bit_count = 24;
    void carry() {
        size_t i = out.size();
        while (i > 0 && out[i - 1] == 255) out[--i] = 0;
        if (i > 0) ++out[i - 1];
    }
    void put(int bit, int prob) {
        const uint32_t split = 1 + (((range - 1) * (uint32_t)prob) >> 8);
        if (bit) { bottom += split; range -= split; }
        else range = split;
        while (range < 128) {
            range <<= 1;
            if (bottom & (1u << 31)) carry();
            bottom <<= 1;
            if (!--bit_count) {
                out.push_back((uint8_t)(bottom >> 24));
                bottom &= (1u << 24) - 1;
                bit_count = 8;
            }
        }
    }
    void literal(int v, int n) {
        for (int i = n - 1; i >= 0; --i) put((v >> i) & 1, 128);
    }
    void flush() {
        int c = bit_count;
        uint32_t v = bottom;
        if (v & (1u << (32 - c))) carry();
        v <<= c & 7;
        c >>= 3;
        while (--c >= 0) v <<= 8;
        c = 4;
        while (--c >= 0) {
            out.push_back((uint8_t)(v >> 24));
            v <<= 8;
        }
    }
};

// token sink: either counts node decisions (for probability adaptation) or codes them
struct TokenSink {
    BoolEnc* enc = nullptr;           // coding when non-null
    uint32_t (*counts)[2] = nullptr;  // [1056][2] when counting
    const uint8_t* probs = nullptr;
    void bit(int idx /* flat node index or -1 */, int prob, int b) {
        if (counts && idx >= 0) ++counts[idx][b];
        if (enc) enc->put(b, prob);
    }
};

}  // namespace

int last_nz(const int16_t* lv, int first) {
    for (int n = 15; n >= first; --n)
        if (lv[n]) return n + 1;
    return first;
}

namespace {

// one block's tokens (libwebp GetCoeffs in reverse); returns nz (any nonzero)
int write_block(TokenSink& s, const int16_t* lv, int first, int ctx, int type) {
    const int last = last_nz(lv, first);
    int n = first;
    auto base = [&](int nn, int c) { return ((type * 8 + band(nn)) * 3 + c) * 11; };
    int b = base(n, ctx);
    if (last <= first) {
        s.bit(b + 0, s.probs[b + 0], 0);
        return 0;
    }
    for (;;) {
        s.bit(b + 0, s.probs[b + 0], 1);
        while (lv[n] == 0) {
            s.bit(b + 1, s.probs[b + 1], 0);
            ++n;
            b = base(n, 0);
        }
        s.bit(b + 1, s.probs[b + 1], 1);
        const int v = lv[n] < 0 ? -lv[n] : lv[n];
        int nctx;
        if (v == 1) {
            s.bit(b + 2, s.probs[b + 2], 0);
            nctx = 1;
        } else {
            s.bit(b + 2, s.probs[b + 2], 1);
            if (v <= 4) {
                s.bit(b + 3, s.probs[b + 3], 0);
                if (v == 2) s.bit(b + 4, s.probs[b + 4], 0);
                else { s.bit(b + 4, s.probs[b + 4], 1); s.bit(b + 5, s.probs[b + 5], v == 4); }
            } else if (v <= 10) {
                s.bit(b + 3, s.probs[b + 3], 1);
                s.bit(b + 6, s.probs[b + 6], 0);
                if (v <= 6) {
                    s.bit(b + 7, s.probs[b + 7], 0);
                    s.bit(-1, 159, v - 5);
                } else {
                    s.bit(b + 7, s.probs[b + 7], 1);
                    s.bit(-1, 165, (v - 7) >> 1);
                    s.bit(-1, 145, (v - 7) & 1);
                }
            } else {
                s.bit(b + 3, s.probs[b + 3], 1);
                s.bit(b + 6, s.probs[b + 6], 1);
                static const uint8_t kCat3[] = {173, 148, 140, 0};
                static const uint8_t kCat4[] = {176, 155, 140, 135, 0};
                static const uint8_t kCat5[] = {180, 157, 141, 134, 130, 0};
                static const uint8_t kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};
                static const uint8_t* const kCat[4] = {kCat3, kCat4, kCat5, kCat6};
                const int cat = v <= 18 ? 0 : (v <= 34 ? 1 : (v <= 66 ? 2 : 3));
                s.bit(b + 8, s.probs[b + 8], cat >> 1);
                s.bit(b + 9 + (cat >> 1), s.probs[b + 9 + (cat >> 1)], cat & 1);
                const int extra = v - (3 + (8 << cat));
                const int nb = cat == 3 ? 11 : 3 + cat;
                for (int i = 0; i < nb; ++i) s.bit(-1, kCat[cat][i], (extra >> (nb - 1 - i)) & 1);
            }
            nctx = 2;
        }
        if (s.enc) s.enc->put(lv[n] < 0, 128);  // sign
        ++n;
        if (n == 16) return 1;
        b = base(n, nctx);
        if (n >= last) {
            s.bit(b + 0, s.probs[b + 0], 0);
            return 1;
        }
    }
}

// all residual tokens of the frame, with the decoder's non-zero contexts
void write_tokens(TokenSink& s, int mb_w, int mb_h, const MBOut* mbs, bool use_skip) {
    std::vector<uint8_t> top((size_t)mb_w * 9, 0);
    for (int my = 0; my < mb_h; ++my) {
        uint8_t left[9] = {0};
        for (int mx = 0; mx < mb_w; ++mx) {
            const MBOut& m = mbs[(size_t)my * mb_w + mx];
            uint8_t* t = &top[(size_t)mx * 9];
            const bool i4 = m.ymode == B_PRED;
            if (use_skip && m.skip) {
                for (int i = 0; i < 8; ++i) t[i] = left[i] = 0;
                if (!i4) t[8] = left[8] = 0;
                continue;
            }
            int first = 0, ytype = 3;
            if (!i4) {
                const int nz = write_block(s, m.lv[24], 0, t[8] + left[8], 1);
                t[8] = left[8] = (uint8_t)nz;
                first = 1;
                ytype = 0;
            }
            for (int y = 0; y < 4; ++y)
                for (int x = 0; x < 4; ++x) {
                    const int nz = write_block(s, m.lv[y * 4 + x], first, t[x] + left[y], ytype);
                    t[x] = left[y] = (uint8_t)nz;
                }
            for (int ch = 0; ch < 2; ++ch)
                for (int y = 0; y < 2; ++y)
                    for (int x = 0; x < 2; ++x) {
                        const int nz = write_block(s, m.lv[16 + 4 * ch + y * 2 + x], 0,
                                                   t[4 + 2 * ch + x] + left[4 + 2 * ch + y], 2);
                        t[4 + 2 * ch + x] = left[4 + 2 * ch + y] = (uint8_t)nz;
                    }
        }
    }
}

void put_bmode(BoolEnc& e, int mode, int top, int left) {
    const uint8_t* p = kBModeProbs + (top * 10 + left) * 9;
    switch (mode) {
    case B_DC: e.put(0, p[0]); return;
    case B_TM: e.put(1, p[0]); e.put(0, p[1]); return;
    case B_VE: e.put(1, p[0]); e.put(1, p[1]); e.put(0, p[2]); return;
    default: break;
    }
    e.put(1, p[0]); e.put(1, p[1]); e.put(1, p[2]);
    switch (mode) {
    case B_HE: e.put(0, p[3]); e.put(0, p[4]); return;
    case B_RD: e.put(0, p[3]); e.put(1, p[4]); e.put(0, p[5]); return;
    case B_VR: e.put(0, p[3]); e.put(1, p[4]); e.put(1, p[5]); return;
    case B_LD: e.put(1, p[3]); e.put(0, p[6]); return;
    case B_VL: e.put(1, p[3]); e.put(1, p[6]); e.put(0, p[7]); return;
    case B_HD: e.put(1, p[3]); e.put(1, p[6]); e.put(1, p[7]); e.put(0, p[8]); return;
    default: e.put(1, p[3]); e.put(1, p[6]); e.put(1, p[7]); e.put(1, p[8]); return;
    }
}

void le32(std::vector<uint8_t>& v, uint32_t x) {
    for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}

}  // namespace

int quality_to_qindex(float quality) {
    const double c = quality < 0 ? 0.0 : (quality > 100 ? 1.0 : quality / 100.0);
    const double linear = c < 0.75 ? c * (2.0 / 3.0) : 2.0 * c - 1.0;
    const double v = std::pow(linear, 1.0 / 3.0);
    const int q = (int)(127.0 * (1.0 - v));
    return q < 0 ? 0 : (q > 127 ? 127 : q);
}

QParams qparams_for_quality(float quality) { return make_qparams(quality_to_qindex(quality), -2); }

void write_webp(int width, int height, const QParams& q, const MBOut* mbs, int filter_level,
                std::vector<uint8_t>& out) {
    const int mb_w = (width + 15) >> 4, mb_h = (height + 15) >> 4;
    const size_t nmb = (size_t)mb_w * mb_h;
    // 1. token statistics under the frame's structure -> adapted probabilities
    std::vector<uint32_t> cnt(1056 * 2, 0);
    size_t nskip = 0;
    for (size_t i = 0; i < nmb; ++i) nskip += mbs[i].skip;
    const bool use_skip = nskip > 0;
    uint8_t probs[1056];
    std::memcpy(probs, kCoeffProbs0, sizeof(probs));
    {
        TokenSink s;
        s.counts = reinterpret_cast<uint32_t(*)[2]>(cnt.data());
        s.probs = probs;
        write_tokens(s, mb_w, mb_h, mbs, use_skip);
    }
    bool upd[1056];
    for (int i = 0; i < 1056; ++i) {
        upd[i] = false;
        const uint32_t c0 = cnt[2 * i], c1 = cnt[2 * i + 1], tot = c0 + c1;
        if (!tot) continue;
        int np = (int)((c0 * 256ull + tot / 2) / tot);
        np = np < 1 ? 1 : (np > 255 ? 255 : np);
        const long long old_cost = (long long)c0 * cost0(probs[i]) + (long long)c1 * cost1(probs[i]);
        const long long new_cost = (long long)c0 * cost0(np) + (long long)c1 * cost1(np);
        const long long upd_cost = cost1(kCoeffUpdateProbs[i]) - cost0(kCoeffUpdateProbs[i]) + 8 * 256;
        if (old_cost - new_cost > upd_cost) { upd[i] = true; probs[i] = (uint8_t)np; }
    }
    int skip_prob = 255;
    if (use_skip) {
        skip_prob = (int)((nmb - nskip) * 255 / nmb);
        skip_prob = skip_prob < 1 ? 1 : (skip_prob > 254 ? 254 : skip_prob);
    }
    // 2. first partition: header + per-MB modes
    BoolEnc h;
    h.literal(0, 1);  // color_space
    h.literal(0, 1);  // clamping_type
    h.literal(0, 1);  // segmentation_enabled
    h.literal(0, 1);  // filter_type: normal
    h.literal(filter_level < 0 ? q.filter_level : filter_level, 6);
    h.literal(0, 3);  // sharpness
    h.literal(0, 1);  // loop_filter_adj_enable
    h.literal(0, 2);  // one token partition
    h.literal(q.qindex, 7);
    const int deltas[5] = {0, 0, 0, q.dq_uv_dc, 0};  // y_dc, y2_dc, y2_ac, uv_dc, uv_ac
    for (int d : deltas) {
        if (!d) { h.literal(0, 1); continue; }
        h.literal(1, 1);
        h.literal(d < 0 ? -d : d, 4);
        h.literal(d < 0, 1);
    }
    h.literal(0, 1);  // refresh_entropy_probs
    for (int i = 0; i < 1056; ++i) {
        h.put(upd[i], kCoeffUpdateProbs[i]);
        if (upd[i]) h.literal(probs[i], 8);
    }
    h.literal(use_skip, 1);
    if (use_skip) h.literal(skip_prob, 8);
    std::vector<uint8_t> top_modes((size_t)mb_w * 4, B_DC);
    for (int my = 0; my < mb_h; ++my) {
        uint8_t left_modes[4] = {B_DC, B_DC, B_DC, B_DC};
        for (int mx = 0; mx < mb_w; ++mx) {
            const MBOut& m = mbs[(size_t)my * mb_w + mx];
            uint8_t* tm = &top_modes[(size_t)mx * 4];
            if (use_skip) h.put(m.skip, skip_prob);
            if (m.ymode == B_PRED) {
                h.put(0, 145);
                for (int b = 0; b < 16; ++b) {
                    const int bx = b & 3, by = b >> 2;
                    const int t = by ? m.bmodes[b - 4] : tm[bx];
                    const int l = bx ? m.bmodes[b - 1] : left_modes[by];
                    put_bmode(h, m.bmodes[b], t, l);
                }
                for (int i = 0; i < 4; ++i) { tm[i] = m.bmodes[12 + i]; left_modes[i] = m.bmodes[i * 4 + 3]; }
            } else {
                h.put(1, 145);
                switch (m.ymode) {
                case DC_PRED: h.put(0, 156); h.put(0, 163); break;
                case V_PRED: h.put(0, 156); h.put(1, 163); break;
                case H_PRED: h.put(1, 156); h.put(0, 128); break;
                default: h.put(1, 156); h.put(1, 128); break;
                }
                for (int i = 0; i < 4; ++i) { tm[i] = m.ymode; left_modes[i] = m.ymode; }
            }
            switch (m.uvmode) {
            case DC_PRED: h.put(0, 142); break;
            case V_PRED: h.put(1, 142); h.put(0, 114); break;
            case H_PRED: h.put(1, 142); h.put(1, 114); h.put(0, 183); break;
            default: h.put(1, 142); h.put(1, 114); h.put(1, 183); break;
            }
        }
    }
    h.flush();
    // 3. token partition
    BoolEnc t;
    {
        TokenSink s;
        s.enc = &t;
        s.probs = probs;
        write_tokens(s, mb_w, mb_h, mbs, use_skip);
    }
    t.flush();
    // 4. frame + container
    std::vector<uint8_t> vp8;
    const uint32_t first = (uint32_t)h.out.size();
    const uint32_t tag = 0u | (0u << 1) | (1u << 4) | (first << 5);  // key frame, v0, shown
    vp8.push_back((uint8_t)tag); vp8.push_back((uint8_t)(tag >> 8)); vp8.push_back((uint8_t)(tag >> 16));
    vp8.push_back(0x9d); vp8.push_back(0x01); vp8.push_back(0x2a);
    vp8.push_back((uint8_t)width); vp8.push_back((uint8_t)(width >> 8));
    vp8.push_back((uint8_t)height); vp8.push_back((uint8_t)(height >> 8));
    vp8.insert(vp8.end(), h.out.begin(), h.out.end());
    vp8.insert(vp8.end(), t.out.begin(), t.out.end());
    const uint32_t vsize = (uint32_t)vp8.size(), pad = vsize & 1;
    out.clear();
    out.reserve(20 + vsize + pad);
    out.insert(out.end(), {'R', 'I', 'F', 'F'});
    le32(out, 4 + 8 + vsize + pad);
    out.insert(out.end(), {'W', 'E', 'B', 'P', 'V', 'P', '8', ' '});
    le32(out, vsize);
    out.insert(out.end(), vp8.begin(), vp8.end());
    if (pad) out.push_back(0);
}

}  // namespace vp8
}  // namespace ik
