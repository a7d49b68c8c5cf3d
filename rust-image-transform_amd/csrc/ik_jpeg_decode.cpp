// ik_jpeg_decode.cpp -- JPEG branch of decode_image (reference src/transform.rs:31 ->
// image 0.25.8 -> zune-jpeg 0.4.21, Cargo.lock:3106).
//
// Baseline sequential Huffman JPEG (SOF0/SOF1, 8-bit), any sampling factors,
// restart intervals, 1 (gray -> L8) or 3 (YCbCr -> Rgb8) components.
// zune-jpeg's output cannot be checked offline (no crate sources), so the
// reconstruction follows the libjpeg decode pipeline that zune-jpeg aims to
// match: jidctint islow IDCT with the range-limit table, "fancy" h2v1 / h2v2 /
// h1v2 chroma upsampling with replicated edge context rows, and jdcolor's
// fixed-point YCbCr->RGB tables.  Parity is pinned against libjpeg-turbo
// (Pillow) in tests/test_gpu_decode.py.  Progressive, arithmetic-coded, 12-bit
// and CMYK JPEGs report IK_ERR_UNSUPPORTED.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {
namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct HuffTable {
    bool present = false;
    // canonical decode: maxcode[l], valptr[l], mincode[l]; plus a 9-bit lookahead
    int maxcode[18] = {}, valptr[17] = {}, mincode[17] = {};
    uint8_t vals[256] = {};
    uint8_t look_len[512] = {}, look_val[512] = {};
};

bool build_huff(const uint8_t* bits, const uint8_t* vals, int nvals, HuffTable& t) {
    t = HuffTable();
    std::memcpy(t.vals, vals, nvals);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        t.valptr[l] = k;
        t.mincode[l] = code;
        code += bits[l - 1];
        k += bits[l - 1];
        t.maxcode[l] = bits[l - 1] ? code - 1 : -1;
        if (code > (1 << l)) return false;
        code <<= 1;
    }
    t.maxcode[17] = 0x7fffffff;
    // lookahead for codes up to 9 bits
    code = 0;
    k = 0;
    for (int l = 1; l <= 9; ++l) {
        for (int i = 0; i < bits[l - 1]; ++i, ++k, ++code) {
            const int shift = 9 - l;
            for (int f = 0; f < (1 << shift); ++f) {
                t.look_len[(code << shift) | f] = (uint8_t)l;
                t.look_val[(code << shift) | f] = vals[k];
            }
        }
        code <<= 1;
    }
    t.present = true;
    return true;
}

struct Component {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0;          // blocks across/down (padded to MCUs)
    int dw = 0, dh = 0;          // downsampled width/height (libjpeg downsampled_width/height)
    std::vector<uint8_t> plane;  // bw*8 x bh*8 samples after IDCT
    int pred = 0;
};

struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc = 0;
    int n = 0;
    bool marker_hit = false;
    void fill() {
        while (n <= 56) {
            uint8_t b = 0;
            if (!marker_hit && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const uint8_t nx = p + 1 < end ? p[1] : 0;
                    if (nx == 0x00) { p += 2; }
                    else { marker_hit = true; b = 0; }  // feed zeros past a marker
                } else {
                    ++p;
                }
            }
            acc |= (uint64_t)b << (56 - n);
            n += 8;
        }
    }
    inline int peek(int k) { if (n < k) fill(); return (int)(acc >> (64 - k)); }
    inline void skip(int k) { acc <<= k; n -= k; }
    inline int get(int k) { if (!k) return 0; const int v = peek(k); skip(k); return v; }
    void reset_at_marker() { acc = 0; n = 0; marker_hit = false; }
};

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

int decode_symbol(BitReader& br, const HuffTable& t) {
    const int look = br.peek(9);
    const int l = t.look_len[look];
    if (l) { br.skip(l); return t.look_val[look]; }
    int code = br.peek(16);
    for (int len = 10; len <= 16; ++len) {
        const int c = code >> (16 - len);
        if (t.maxcode[len] >= 0 && c <= t.maxcode[len] && c >= t.mincode[len]) {
            br.skip(len);
            return t.vals[t.valptr[len] + c - t.mincode[len]];
        }
    }
    return -1;
}

// jidctint.c jpeg_idct_islow (libjpeg / libjpeg-turbo), dequantised input
#define CB 13
#define P1 2
void idct_islow(const int* in, uint8_t* out, int stride) {
    int ws[64];
    auto descale = [](long long x, int n) { return (int)((x + (1ll << (n - 1))) >> n); };
    auto clamp = [](int x) -> uint8_t { x += 128; return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); };
    for (int c = 0; c < 8; ++c) {
        const int* ip = in + c;
        if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
            const int dc = ip[0] * (1 << P1);
            for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
            continue;
        }
        long long z2 = ip[16], z3 = ip[48];
        long long z1 = (z2 + z3) * 4433;
        long long tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
        z2 = ip[0]; z3 = ip[32];
        long long tmp0 = (z2 + z3) * (1ll << CB), tmp1 = (z2 - z3) * (1ll << CB);
        long long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = ip[56]; tmp1 = ip[40]; tmp2 = ip[24]; tmp3 = ip[8];
        z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
        long long z4 = tmp1 + tmp3, z5 = (z3 + z4) * 9633;
        tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
        z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        ws[0 * 8 + c] = descale(t10 + tmp3, CB - P1);
        ws[7 * 8 + c] = descale(t10 - tmp3, CB - P1);
        ws[1 * 8 + c] = descale(t11 + tmp2, CB - P1);
        ws[6 * 8 + c] = descale(t11 - tmp2, CB - P1);
        ws[2 * 8 + c] = descale(t12 + tmp1, CB - P1);
        ws[5 * 8 + c] = descale(t12 - tmp1, CB - P1);
        ws[3 * 8 + c] = descale(t13 + tmp0, CB - P1);
        ws[4 * 8 + c] = descale(t13 - tmp0, CB - P1);
    }
    for (int r = 0; r < 8; ++r) {
        const int* w = ws + r * 8;
        uint8_t* o = out + (size_t)r * stride;
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t dc = clamp(descale(w[0], P1 + 3));
            for (int k = 0; k < 8; ++k) o[k] = dc;
            continue;
        }
        long long z2 = w[2], z3 = w[6];
        long long z1 = (z2 + z3) * 4433;
        long long tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
        long long tmp0 = ((long long)w[0] + w[4]) * (1ll << CB), tmp1 = ((long long)w[0] - w[4]) * (1ll << CB);
        long long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
        z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
        long long z4 = tmp1 + tmp3, z5 = (z3 + z4) * 9633;
        tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
        z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        const int sh = CB + P1 + 3;
        o[0] = clamp(descale(t10 + tmp3, sh)); o[7] = clamp(descale(t10 - tmp3, sh));
        o[1] = clamp(descale(t11 + tmp2, sh)); o[6] = clamp(descale(t11 - tmp2, sh));
        o[2] = clamp(descale(t12 + tmp1, sh)); o[5] = clamp(descale(t12 - tmp1, sh));
        o[3] = clamp(descale(t13 + tmp0, sh)); o[4] = clamp(descale(t13 - tmp0, sh));
    }
}
#undef CB
#undef P1

// jdcolor.c ycc_rgb_convert tables (SCALEBITS 16)
struct YccTables {
    int cr_r[256], cb_b[256];
    long long cr_g[256], cb_g[256];
    YccTables() {
        const long long half = 1ll << 15;
        auto fix = [](double x) { return (long long)(x * 65536.0 + 0.5); };
        for (int i = 0; i < 256; ++i) {
            const long long x = i - 128;
            cr_r[i] = (int)((fix(1.40200) * x + half) >> 16);
            cb_b[i] = (int)((fix(1.77200) * x + half) >> 16);
            cr_g[i] = -fix(0.71414) * x;
            cb_g[i] = -fix(0.34414) * x + half;
        }
    }
};

inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// upsample one component plane (dw x dh valid samples) to the full image size
void upsample(const Component& c, int hmax, int vmax, int W, int H, std::vector<uint8_t>& out) {
    const int pw = c.bw * 8;  // plane stride
    const int fh = hmax / c.h, fv = vmax / c.v;
    const int ow = c.dw * fh, oh = c.dh * fv;
    std::vector<uint8_t> full((size_t)ow * oh);
    auto in = [&](int y) { return c.plane.data() + (size_t)(y < 0 ? 0 : y >= c.dh ? c.dh - 1 : y) * pw; };
    if (fh == 1 && fv == 1) {
        for (int y = 0; y < oh; ++y) std::memcpy(&full[(size_t)y * ow], in(y), ow);
    } else if (fh == 2 && fv == 1) {  // h2v1_fancy_upsample
        for (int y = 0; y < c.dh; ++y) {
            const uint8_t* ip = in(y);
            uint8_t* op = &full[(size_t)y * ow];
            if (c.dw == 1) { op[0] = op[1] = ip[0]; continue; }
            op[0] = ip[0];
            op[1] = (uint8_t)((ip[0] * 3 + ip[1] + 2) >> 2);
            for (int x = 1; x < c.dw - 1; ++x) {
                const int v3 = ip[x] * 3;
                op[2 * x] = (uint8_t)((v3 + ip[x - 1] + 1) >> 2);
                op[2 * x + 1] = (uint8_t)((v3 + ip[x + 1] + 2) >> 2);
            }
            const int x = c.dw - 1;
            op[2 * x] = (uint8_t)((ip[x] * 3 + ip[x - 1] + 1) >> 2);
            op[2 * x + 1] = ip[x];
        }
    } else if (fh == 2 && fv == 2) {  // h2v2_fancy_upsample
        for (int y = 0; y < c.dh; ++y) {
            for (int v = 0; v < 2; ++v) {
                const uint8_t* i0 = in(y);
                const uint8_t* i1 = in(v == 0 ? y - 1 : y + 1);
                uint8_t* op = &full[(size_t)(2 * y + v) * ow];
                if (c.dw == 1) {
                    const int s = i0[0] * 3 + i1[0];
                    op[0] = (uint8_t)((s * 4 + 8) >> 4);
                    op[1] = (uint8_t)((s * 4 + 7) >> 4);
                    continue;
                }
                int thiss = i0[0] * 3 + i1[0];
                int nexts = i0[1] * 3 + i1[1];
                op[0] = (uint8_t)((thiss * 4 + 8) >> 4);
                op[1] = (uint8_t)((thiss * 3 + nexts + 7) >> 4);
                int lasts = thiss;
                thiss = nexts;
                for (int x = 1; x < c.dw - 1; ++x) {
                    nexts = i0[x + 1] * 3 + i1[x + 1];
                    op[2 * x] = (uint8_t)((thiss * 3 + lasts + 8) >> 4);
                    op[2 * x + 1] = (uint8_t)((thiss * 3 + nexts + 7) >> 4);
                    lasts = thiss;
                    thiss = nexts;
                }
                const int x = c.dw - 1;
                op[2 * x] = (uint8_t)((thiss * 3 + lasts + 8) >> 4);
                op[2 * x + 1] = (uint8_t)((thiss * 4 + 7) >> 4);
            }
        }
    } else if (fh == 1 && fv == 2) {  // h1v2_fancy_upsample (libjpeg-turbo)
        for (int y = 0; y < c.dh; ++y)
            for (int v = 0; v < 2; ++v) {
                const uint8_t* i0 = in(y);
                const uint8_t* i1 = in(v == 0 ? y - 1 : y + 1);
                const int bias = v == 0 ? 1 : 2;
                uint8_t* op = &full[(size_t)(2 * y + v) * ow];
                for (int x = 0; x < c.dw; ++x) op[x] = (uint8_t)((i0[x] * 3 + i1[x] + bias) >> 2);
            }
    } else {  // int_upsample: replication
        for (int y = 0; y < oh; ++y)
            for (int x = 0; x < ow; ++x) full[(size_t)y * ow + x] = in(y / fv)[x / fh];
    }
    out.assign((size_t)W * H, 0);
    for (int y = 0; y < H; ++y) {
        const int sy = y < oh ? y : oh - 1;
        for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = full[(size_t)sy * ow + (x < ow ? x : ow - 1)];
    }
}

}  // namespace

int decode_jpeg(const uint8_t* b, size_t n, uint32_t& W, uint32_t& H, uint32_t& C, std::vector<uint8_t>& px) {
    const uint8_t* p = b + 2;
    const uint8_t* end = b + n;
    uint16_t qt[4][64] = {};
    HuffTable dc[4], ac[4];
    std::vector<Component> comps;
    int width = 0, height = 0, restart = 0;
    bool have_frame = false, adobe = false;
    int adobe_transform = -1;
    auto be16 = [](const uint8_t* q) { return (int)q[0] << 8 | q[1]; };
    const char* fmt_err = "Format error decoding Jpeg";
    for (;;) {
        while (p < end && *p != 0xFF) ++p;  // tolerate garbage between segments
        while (p < end && *p == 0xFF) ++p;
        if (p >= end) return fail(IK_ERR_TRANSFORM, "%s: no SOS", fmt_err);
        const uint8_t m = *p++;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) return fail(IK_ERR_TRANSFORM, "%s: no SOS", fmt_err);
        if (p + 2 > end) return fail(IK_ERR_TRANSFORM, "%s: truncated", fmt_err);
        const int len = be16(p);
        if (len < 2 || p + len > end) return fail(IK_ERR_TRANSFORM, "%s: bad segment length", fmt_err);
        const uint8_t* s = p + 2;
        const uint8_t* se = p + len;
        if (m == 0xDB) {  // DQT
            while (s < se) {
                const int pq = s[0] >> 4, tq = s[0] & 15;
                if (tq > 3) return fail(IK_ERR_TRANSFORM, "%s: bad DQT", fmt_err);
                ++s;
                for (int i = 0; i < 64; ++i) {
                    qt[tq][kZigzag[i]] = pq ? (uint16_t)be16(s + 2 * i) : s[i];
                }
                s += pq ? 128 : 64;
            }
        } else if (m == 0xC4) {  // DHT
            while (s < se) {
                const int tc = s[0] >> 4, th = s[0] & 15;
                if (th > 3 || tc > 1 || s + 17 > se) return fail(IK_ERR_TRANSFORM, "%s: bad DHT", fmt_err);
                int total = 0;
                for (int i = 0; i < 16; ++i) total += s[1 + i];
                if (total > 256 || s + 17 + total > se) return fail(IK_ERR_TRANSFORM, "%s: bad DHT", fmt_err);
                if (!build_huff(s + 1, s + 17, total, tc ? ac[th] : dc[th]))
                    return fail(IK_ERR_TRANSFORM, "%s: bad Huffman table", fmt_err);
                s += 17 + total;
            }
        } else if (m == 0xDD) {  // DRI
            restart = be16(s);
        } else if (m == 0xEE) {  // APP14 Adobe
            if (len >= 14 && !std::memcmp(s, "Adobe", 5)) { adobe = true; adobe_transform = s[11]; }
        } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1 baseline
            if (s[0] != 8) return fail(IK_ERR_UNSUPPORTED, "12-bit JPEG is not supported");
            height = be16(s + 1);
            width = be16(s + 3);
            const int nc = s[5];
            if (!width || !height) return fail(IK_ERR_TRANSFORM, "%s: zero dimension", fmt_err);
            if (nc != 1 && nc != 3) return fail(IK_ERR_UNSUPPORTED, "JPEG with %d components is not supported", nc);
            comps.resize(nc);
            for (int i = 0; i < nc; ++i) {
                comps[i].id = s[6 + 3 * i];
                comps[i].h = s[7 + 3 * i] >> 4;
                comps[i].v = s[7 + 3 * i] & 15;
                comps[i].tq = s[8 + 3 * i] & 3;
                if (comps[i].h < 1 || comps[i].h > 4 || comps[i].v < 1 || comps[i].v > 4)
                    return fail(IK_ERR_TRANSFORM, "%s: bad sampling factors", fmt_err);
            }
            have_frame = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return fail(IK_ERR_UNSUPPORTED, "progressive / arithmetic / lossless JPEG (SOF%d) is not supported",
                        m - 0xC0);
        } else if (m == 0xDA) {  // SOS
            if (!have_frame) return fail(IK_ERR_TRANSFORM, "%s: SOS before SOF", fmt_err);
            const int ns = s[0];
            if (ns != (int)comps.size()) return fail(IK_ERR_UNSUPPORTED, "non-interleaved baseline scans are not supported");
            std::vector<int> order(ns);
            for (int i = 0; i < ns; ++i) {
                const int cid = s[1 + 2 * i];
                int k = -1;
                for (int j = 0; j < (int)comps.size(); ++j) if (comps[j].id == cid) k = j;
                if (k < 0) return fail(IK_ERR_TRANSFORM, "%s: bad scan component", fmt_err);
                comps[k].td = s[2 + 2 * i] >> 4;
                comps[k].ta = s[2 + 2 * i] & 15;
                if (comps[k].td > 3 || comps[k].ta > 3 || !dc[comps[k].td].present || !ac[comps[k].ta].present)
                    return fail(IK_ERR_TRANSFORM, "%s: missing Huffman table", fmt_err);
                order[i] = k;
            }
            // geometry
            int hmax = 1, vmax = 1;
            for (auto& c : comps) { hmax = std::max(hmax, c.h); vmax = std::max(vmax, c.v); }
            const int mcux = (width + 8 * hmax - 1) / (8 * hmax), mcuy = (height + 8 * vmax - 1) / (8 * vmax);
            if ((uint64_t)width * height > (512ull << 20) / 3) return fail(IK_ERR_TRANSFORM, "Limits are exceeded");
            for (auto& c : comps) {
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
                c.dw = (width * c.h + hmax - 1) / hmax;
                c.dh = (height * c.v + vmax - 1) / vmax;
                c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
                c.pred = 0;
            }
            BitReader br{se, end};
            int blk[64];
            const bool single = ns == 1;
            const int total_mcu = single ? ((comps[0].dw + 7) / 8) * ((comps[0].dh + 7) / 8) : mcux * mcuy;
            const int single_bw = single ? (comps[0].dw + 7) / 8 : 0;
            for (int mcu = 0; mcu < total_mcu; ++mcu) {
                if (restart && mcu > 0 && mcu % restart == 0) {
                    // expect RSTn: realign to the marker and reset predictors
                    const uint8_t* q = br.p;
                    while (q + 1 < end && !(q[0] == 0xFF && q[1] >= 0xD0 && q[1] <= 0xD7)) ++q;
                    if (q + 1 >= end) return fail(IK_ERR_TRANSFORM, "%s: missing restart marker", fmt_err);
                    br.p = q + 2;
                    br.reset_at_marker();
                    for (auto& c : comps) c.pred = 0;
                }
                for (int oi = 0; oi < ns; ++oi) {
                    Component& c = comps[order[oi]];
                    const int nby = single ? 1 : c.v, nbx = single ? 1 : c.h;
                    for (int by = 0; by < nby; ++by)
                        for (int bx = 0; bx < nbx; ++bx) {
                            std::memset(blk, 0, sizeof(blk));
                            const int t = decode_symbol(br, dc[c.td]);
                            if (t < 0 || t > 11) return fail(IK_ERR_TRANSFORM, "%s: bad DC code", fmt_err);
                            const int diff = t ? extend(br.get(t), t) : 0;
                            c.pred += diff;
                            blk[0] = c.pred * qt[c.tq][0];
                            for (int k = 1; k < 64;) {
                                const int rs = decode_symbol(br, ac[c.ta]);
                                if (rs < 0) return fail(IK_ERR_TRANSFORM, "%s: bad AC code", fmt_err);
                                const int r = rs >> 4, sz = rs & 15;
                                if (!sz) {
                                    if (r != 15) break;  // EOB
                                    k += 16;
                                    continue;
                                }
                                k += r;
                                if (k > 63) return fail(IK_ERR_TRANSFORM, "%s: AC overflow", fmt_err);
                                const int zz = kZigzag[k];
                                blk[zz] = extend(br.get(sz), sz) * qt[c.tq][zz];
                                ++k;
                            }
                            int bxx, byy;
                            if (single) { bxx = mcu % single_bw; byy = mcu / single_bw; }
                            else { bxx = (mcu % mcux) * c.h + bx; byy = (mcu / mcux) * c.v + by; }
                            idct_islow(blk, c.plane.data() + (size_t)byy * 8 * (c.bw * 8) + bxx * 8, c.bw * 8);
                        }
                }
            }
            // upsample + colour convert
            W = (uint32_t)width;
            H = (uint32_t)height;
            if (comps.size() == 1) {
                C = 1;
                px.resize((size_t)width * height);
                const Component& c = comps[0];
                for (int y = 0; y < height; ++y)
                    std::memcpy(&px[(size_t)y * width], c.plane.data() + (size_t)y * c.bw * 8, width);
                return IK_OK;
            }
            if (adobe && adobe_transform == 0)
                return fail(IK_ERR_UNSUPPORTED, "JPEG in RGB colour space (Adobe transform 0) is not supported");
            std::vector<uint8_t> Y, Cb, Cr;
            upsample(comps[0], hmax, vmax, width, height, Y);
            upsample(comps[1], hmax, vmax, width, height, Cb);
            upsample(comps[2], hmax, vmax, width, height, Cr);
            static const YccTables T;
            C = 3;
            px.resize((size_t)width * height * 3);
            for (size_t i = 0; i < (size_t)width * height; ++i) {
                const int y = Y[i], cb = Cb[i], cr = Cr[i];
                px[3 * i] = clamp255(y + T.cr_r[cr]);
                px[3 * i + 1] = clamp255(y + (int)((T.cb_g[cb] + T.cr_g[cr]) >> 16));
                px[3 * i + 2] = clamp255(y + T.cb_b[cb]);
            }
            return IK_OK;
        }
        p += len;
    }
}

}  // namespace ik
