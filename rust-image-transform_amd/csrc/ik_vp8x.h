// ik_vp8x.h -- the exact WebP (VP8) coder: libwebp method 4's macroblock decisions,
// shared by the GPU kernel (ik_vp8x.hip) and the host (ik_vp8x.cpp).  The reference's
// coder is libwebp (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp
// WebPEncode, config defaults): the same arithmetic as oracle/vp8_modes.c, whose output
// is byte-identical to WebPEncodeRGB (tests/test_vp8_modes.py).  BPS-pitched work
// buffers; the tables are libwebp's own read-only data (ik_vp8_tables.h).
#pragma once
#include <cstdint>

#include "ik_vp8.h"

namespace ik {
namespace vp8x {

using namespace ::ik::vp8;

constexpr int BPS = 32;
constexpr int QFIX = 17;
constexpr int kMaxVarLevel = 67;
constexpr int kLevelTab = (kMaxVarLevel + 1);  // u16 per level-cost row
constexpr int kCostRows = 4 * 8 * 3;           // [type][band][ctx]

struct XMatrix {
    uint16_t q[16], iq[16], sharpen[16];
    uint32_t bias[16], zthresh[16];
};

struct XSeg {
    XMatrix y1, y2, uv;
    int lambda_i4, lambda_i16, lambda_uv, lambda_mode, tlambda, min_disto;
};

IK_HD int xabs(int v) { return v < 0 ? -v : v; }
IK_HD uint8_t xclip8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
IK_HD int bit_cost(int bit, int p) { return !bit ? kEntropyCost[p] : kEntropyCost[255 - p]; }

// ---- set-up (quant_enc.c SetupMatrices) ----
IK_HD int expand_matrix(XMatrix& m, int type) {
    constexpr int kBias[3][2] = {{96, 110}, {96, 108}, {110, 115}};
    int sum = 0;
    for (int i = 0; i < 2; ++i) {
        m.iq[i] = (uint16_t)((1 << QFIX) / m.q[i]);
        m.bias[i] = (uint32_t)(kBias[type][i > 0] << (QFIX - 8));
        m.zthresh[i] = ((1u << QFIX) - 1 - m.bias[i]) / m.iq[i];
    }
    for (int i = 2; i < 16; ++i) {
        m.q[i] = m.q[1];
        m.iq[i] = m.iq[1];
        m.bias[i] = m.bias[1];
        m.zthresh[i] = m.zthresh[1];
    }
    for (int i = 0; i < 16; ++i) {
        m.sharpen[i] = type == 0 ? (uint16_t)((kFreqSharpening[i] * m.q[i]) >> 11) : 0;
        sum += m.q[i];
    }
    return (sum + 8) >> 4;
}

IK_HD XSeg setup_segment(int q, int dq_uv_dc, int dq_uv_ac, int sns) {
    auto clip = [](int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; };
    XSeg s{};
    s.y1.q[0] = kDcTable[clip(q, 0, 127)];
    s.y1.q[1] = kAcTable[clip(q, 0, 127)];
    s.y2.q[0] = (uint16_t)(kDcTable[clip(q, 0, 127)] * 2);
    s.y2.q[1] = (uint16_t)((kAcTable[clip(q, 0, 127)] * 101581) >> 16);
    if (s.y2.q[1] < 8) s.y2.q[1] = 8;
    s.uv.q[0] = kDcTable[clip(q + dq_uv_dc, 0, 117)];
    s.uv.q[1] = kAcTable[clip(q + dq_uv_ac, 0, 127)];
    const int q_i4 = expand_matrix(s.y1, 0), q_i16 = expand_matrix(s.y2, 1), q_uv = expand_matrix(s.uv, 2);
    s.lambda_i4 = (3 * q_i4 * q_i4) >> 7;
    s.lambda_i16 = 3 * q_i16 * q_i16;
    s.lambda_uv = (3 * q_uv * q_uv) >> 6;
    s.lambda_mode = (1 * q_i4 * q_i4) >> 7;
    s.tlambda = (sns * q_i4) >> 5;
    if (s.lambda_i4 < 1) s.lambda_i4 = 1;
    if (s.lambda_i16 < 1) s.lambda_i16 = 1;
    if (s.lambda_uv < 1) s.lambda_uv = 1;
    if (s.lambda_mode < 1) s.lambda_mode = 1;
    s.min_disto = 20 * s.y1.q[0];
    return s;
}

// VP8CalculateLevelCosts for one [type][band][ctx] row: table[0..67]
IK_HD void level_cost_row(const uint8_t* p, int ctx, uint16_t* table) {
    const int cost0 = ctx > 0 ? bit_cost(1, p[0]) : 0;
    const int cost_base = bit_cost(1, p[1]) + cost0;
    table[0] = (uint16_t)(bit_cost(0, p[1]) + cost0);
    for (int v = 1; v <= kMaxVarLevel; ++v) {
        int pattern = kLevelCodes[2 * (v - 1)], bits = kLevelCodes[2 * (v - 1) + 1], cost = 0;
        for (int i = 2; pattern; ++i) {
            if (pattern & 1) cost += bit_cost(bits & 1, p[i]);
            bits >>= 1;
            pattern >>= 1;
        }
        table[v] = (uint16_t)(cost_base + cost);
    }
}

// ---- transforms, quantisation ----
IK_HD void ftransform(const uint8_t* src, const uint8_t* ref, int16_t* out) {
    int tmp[16];
    for (int i = 0; i < 4; ++i, src += BPS, ref += BPS) {
        const int d0 = src[0] - ref[0], d1 = src[1] - ref[1], d2 = src[2] - ref[2], d3 = src[3] - ref[3];
        const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
        tmp[0 + i * 4] = (a0 + a1) * 8;
        tmp[1 + i * 4] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
        tmp[2 + i * 4] = (a0 - a1) * 8;
        tmp[3 + i * 4] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
    }
    for (int i = 0; i < 4; ++i) {
        const int a0 = tmp[0 + i] + tmp[12 + i], a1 = tmp[4 + i] + tmp[8 + i];
        const int a2 = tmp[4 + i] - tmp[8 + i], a3 = tmp[0 + i] - tmp[12 + i];
        out[0 + i] = (int16_t)((a0 + a1 + 7) >> 4);
        out[4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
        out[8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
        out[12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
    }
}

IK_HD void ftransform_wht(const int16_t* in, int16_t* out) {  // in: 16 blocks of 16, DC at in[16 n]
    int tmp[16];
    for (int i = 0; i < 4; ++i, in += 64) {
        const int a0 = in[0 * 16] + in[2 * 16], a1 = in[1 * 16] + in[3 * 16];
        const int a2 = in[1 * 16] - in[3 * 16], a3 = in[0 * 16] - in[2 * 16];
        tmp[0 + i * 4] = a0 + a1;
        tmp[1 + i * 4] = a3 + a2;
        tmp[2 + i * 4] = a3 - a2;
        tmp[3 + i * 4] = a0 - a1;
    }
    for (int i = 0; i < 4; ++i) {
        const int a0 = tmp[0 + i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
        const int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[0 + i] - tmp[8 + i];
        const int b0 = a0 + a1, b1 = a3 + a2, b2 = a3 - a2, b3 = a0 - a1;
        out[0 + i] = (int16_t)(b0 >> 1);
        out[4 + i] = (int16_t)(b1 >> 1);
        out[8 + i] = (int16_t)(b2 >> 1);
        out[12 + i] = (int16_t)(b3 >> 1);
    }
}

IK_HD void itransform_wht(const int16_t* in, int16_t* out) {  // out: block n's DC at out[16 n]
    int tmp[16];
    for (int i = 0; i < 4; ++i) {
        const int a0 = in[0 + i] + in[12 + i], a1 = in[4 + i] + in[8 + i];
        const int a2 = in[4 + i] - in[8 + i], a3 = in[0 + i] - in[12 + i];
        tmp[0 + i] = a0 + a1;
        tmp[8 + i] = a0 - a1;
        tmp[4 + i] = a3 + a2;
        tmp[12 + i] = a3 - a2;
    }
    for (int i = 0; i < 4; ++i) {
        const int dc = tmp[0 + i * 4] + 3;
        const int a0 = dc + tmp[3 + i * 4], a1 = tmp[1 + i * 4] + tmp[2 + i * 4];
        const int a2 = tmp[1 + i * 4] - tmp[2 + i * 4], a3 = dc - tmp[3 + i * 4];
        out[0] = (int16_t)((a0 + a1) >> 3);
        out[16] = (int16_t)((a3 + a2) >> 3);
        out[32] = (int16_t)((a0 - a1) >> 3);
        out[48] = (int16_t)((a3 - a2) >> 3);
        out += 64;
    }
}

IK_HD void itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst) {
    int C[16];
    for (int i = 0; i < 4; ++i) {
        const int a = in[i] + in[8 + i], b = in[i] - in[8 + i];
        const int c = ((in[4 + i] * 35468) >> 16) - (((in[12 + i] * 20091) >> 16) + in[12 + i]);
        const int d = (((in[4 + i] * 20091) >> 16) + in[4 + i]) + ((in[12 + i] * 35468) >> 16);
        C[4 * i + 0] = a + d;
        C[4 * i + 1] = b + c;
        C[4 * i + 2] = b - c;
        C[4 * i + 3] = a - d;
    }
    for (int i = 0; i < 4; ++i) {
        const int dc = C[i] + 4;
        const int a = dc + C[8 + i], b = dc - C[8 + i];
        const int c = ((C[4 + i] * 35468) >> 16) - (((C[12 + i] * 20091) >> 16) + C[12 + i]);
        const int d = (((C[4 + i] * 20091) >> 16) + C[4 + i]) + ((C[12 + i] * 35468) >> 16);
        dst[0 + i * BPS] = xclip8(ref[0 + i * BPS] + ((a + d) >> 3));
        dst[1 + i * BPS] = xclip8(ref[1 + i * BPS] + ((b + c) >> 3));
        dst[2 + i * BPS] = xclip8(ref[2 + i * BPS] + ((b - c) >> 3));
        dst[3 + i * BPS] = xclip8(ref[3 + i * BPS] + ((a - d) >> 3));
    }
}

IK_HD int quantize_block(int16_t* in, int16_t* out, const XMatrix& m) {
    int last = -1;
    for (int n = 0; n < 16; ++n) {
        const int j = zigzag(n);
        const int sign = in[j] < 0;
        const uint32_t coeff = (uint32_t)((sign ? -in[j] : in[j]) + m.sharpen[j]);
        if (coeff > m.zthresh[j]) {
            int level = (int)((coeff * m.iq[j] + m.bias[j]) >> QFIX);
            if (level > 2047) level = 2047;
            if (sign) level = -level;
            in[j] = (int16_t)(level * (int)m.q[j]);
            out[n] = (int16_t)level;
            if (level) last = n;
        } else {
            out[n] = 0;
            in[j] = 0;
        }
    }
    return last >= 0;
}

// ---- distortion ----
IK_HD int sse_wh(const uint8_t* a, const uint8_t* b, int w, int h) {
    int s = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const int d = a[x + y * BPS] - b[x + y * BPS];
            s += d * d;
        }
    return s;
}

IK_HD int ttransform(const uint8_t* in) {
    int sum = 0, tmp[16];
    for (int i = 0; i < 4; ++i, in += BPS) {
        const int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[1] - in[3], a3 = in[0] - in[2];
        tmp[0 + i * 4] = a0 + a1;
        tmp[1 + i * 4] = a3 + a2;
        tmp[2 + i * 4] = a3 - a2;
        tmp[3 + i * 4] = a0 - a1;
    }
    for (int i = 0; i < 4; ++i) {
        const int a0 = tmp[0 + i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
        const int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[0 + i] - tmp[8 + i];
        sum += kWeightY[i] * xabs(a0 + a1) + kWeightY[4 + i] * xabs(a3 + a2) + kWeightY[8 + i] * xabs(a3 - a2) +
               kWeightY[12 + i] * xabs(a0 - a1);
    }
    return sum;
}
IK_HD int disto4x4(const uint8_t* a, const uint8_t* b) { return xabs(ttransform(b) - ttransform(a)) >> 5; }

IK_HD int is_flat(const int16_t* levels, int num_blocks, int thresh) {
    int score = 0;
    while (num_blocks-- > 0) {
        for (int i = 1; i < 16; ++i) {
            score += levels[i] != 0;
            if (score > thresh) return 0;
        }
        levels += 16;
    }
    return 1;
}

// ---- rates (cost_enc.c GetResidualCost); lc: the image's level costs [type][band][ctx][68],
// pr: its coefficient probabilities [type][band][ctx][11] ----
IK_HD int residual_cost(const uint16_t* lc, const uint8_t* pr, int type, int first, int ctx0, const int16_t* c) {
    int last = -1;
    for (int n = 15; n >= 0; --n)
        if (c[n]) { last = n; break; }
    int n = first;
    const int p0 = pr[((type * 8 + n) * 3 + ctx0) * 11];
    if (last < 0) return bit_cost(0, p0);
    int cost = ctx0 == 0 ? bit_cost(1, p0) : 0;
    const uint16_t* t = lc + ((type * 8 + kEncBands[n]) * 3 + ctx0) * kLevelTab;
    for (; n < last; ++n) {
        const int v = xabs(c[n]);
        const int ctx = v >= 2 ? 2 : v;
        cost += kLevelFixedCosts[v] + t[v > kMaxVarLevel ? kMaxVarLevel : v];
        t = lc + ((type * 8 + kEncBands[n + 1]) * 3 + ctx) * kLevelTab;
    }
    const int v = xabs(c[n]);
    cost += kLevelFixedCosts[v] + t[v > kMaxVarLevel ? kMaxVarLevel : v];
    if (n < 15) cost += bit_cost(0, pr[((type * 8 + kEncBands[n + 1]) * 3 + (v == 1 ? 1 : 2)) * 11]);
    return cost;
}

// ---- predictors ----
IK_HD void fill(uint8_t* dst, int v, int size) {
    for (int j = 0; j < size; ++j)
        for (int i = 0; i < size; ++i) dst[i + j * BPS] = (uint8_t)v;
}
// NxN prediction of mode m (DC 0, TM 1, V 2, H 3); left / top may be null (frame edge);
// left[-1] is the corner
IK_HD void pred_nxn(uint8_t* dst, int m, const uint8_t* left, const uint8_t* top, int size) {
    if (m == 0) {
        const int shift = size == 16 ? 5 : 4;
        int DC = 0;
        if (top) {
            for (int j = 0; j < size; ++j) DC += top[j];
            if (left) for (int j = 0; j < size; ++j) DC += left[j];
            else DC += DC;
            DC = (DC + size) >> shift;
        } else if (left) {
            for (int j = 0; j < size; ++j) DC += left[j];
            DC += DC;
            DC = (DC + size) >> shift;
        } else {
            DC = 0x80;
        }
        fill(dst, DC, size);
    } else if (m == 1) {
        if (left && top) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = xclip8(left[y] + top[x] - left[-1]);
        } else if (left) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = left[y];
        } else if (top) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = top[x];
        } else {
            fill(dst, 129, size);
        }
    } else if (m == 2) {
        if (top) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = top[x];
        } else {
            fill(dst, 127, size);
        }
    } else {
        if (left) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = left[y];
        } else {
            fill(dst, 129, size);
        }
    }
}

// the 4x4 block (bx, by) of pred_nxn(.., m, .., 16)
IK_HD void pred16_block(uint8_t* dst, int m, const uint8_t* left, const uint8_t* top, int bx, int by) {
    const int x0 = 4 * bx, y0 = 4 * by;
    int v = 0;
    if (m == 0) {
        int DC = 0;
        if (top) {
            for (int j = 0; j < 16; ++j) DC += top[j];
            if (left) for (int j = 0; j < 16; ++j) DC += left[j];
            else DC += DC;
            DC = (DC + 16) >> 5;
        } else if (left) {
            for (int j = 0; j < 16; ++j) DC += left[j];
            DC += DC;
            DC = (DC + 16) >> 5;
        } else {
            DC = 0x80;
        }
        v = DC;
    }
    for (int y = y0; y < y0 + 4; ++y)
        for (int x = x0; x < x0 + 4; ++x) {
            int p;
            if (m == 0) p = v;
            else if (m == 1) p = (left && top) ? xclip8(left[y] + top[x] - left[-1]) : left ? left[y] : top ? top[x] : 129;
            else if (m == 2) p = top ? top[x] : 127;
            else p = left ? left[y] : 129;
            dst[x + y * BPS] = (uint8_t)p;
        }
}

IK_HD uint8_t avg3(int a, int b, int c) { return (uint8_t)((a + 2 * b + c + 2) >> 2); }
IK_HD uint8_t avg2(int a, int b) { return (uint8_t)((a + b + 1) >> 1); }

// intra-4 predictor from top[] (top[-1] corner, top[-2..-5] the left column, top[0..7]
// above and above-right); row stride S (the device builds it in registers with S = 4)
template <int S = BPS>
IK_HD void pred4(uint8_t* dst, int mode, const uint8_t* top) {
    const int X = top[-1], I = top[-2], J = top[-3], K = top[-4], L = top[-5];
    const int A = top[0], B = top[1], C = top[2], D = top[3], E = top[4], F = top[5], G = top[6], H = top[7];
#define DST(x, y) dst[(x) + (y) * S]
    switch (mode) {
    case 0: {
        const int dc = (4 + A + B + C + D + I + J + K + L) >> 3;
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) DST(x, y) = (uint8_t)dc;
        break;
    }
    case 1: {
        const int lf[4] = {I, J, K, L}, tp[4] = {A, B, C, D};
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) DST(x, y) = xclip8(lf[y] + tp[x] - X);
        break;
    }
    case 2:
        for (int y = 0; y < 4; ++y) {
            DST(0, y) = avg3(X, A, B);
            DST(1, y) = avg3(A, B, C);
            DST(2, y) = avg3(B, C, D);
            DST(3, y) = avg3(C, D, E);
        }
        break;
    case 3: {
        const uint8_t r[4] = {avg3(X, I, J), avg3(I, J, K), avg3(J, K, L), avg3(K, L, L)};
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) DST(x, y) = r[y];
        break;
    }
    case 4:
        DST(0, 3) = avg3(J, K, L);
        DST(0, 2) = DST(1, 3) = avg3(I, J, K);
        DST(0, 1) = DST(1, 2) = DST(2, 3) = avg3(X, I, J);
        DST(0, 0) = DST(1, 1) = DST(2, 2) = DST(3, 3) = avg3(A, X, I);
        DST(1, 0) = DST(2, 1) = DST(3, 2) = avg3(B, A, X);
        DST(2, 0) = DST(3, 1) = avg3(C, B, A);
        DST(3, 0) = avg3(D, C, B);
        break;
    case 5:
        DST(0, 0) = DST(1, 2) = avg2(X, A);
        DST(1, 0) = DST(2, 2) = avg2(A, B);
        DST(2, 0) = DST(3, 2) = avg2(B, C);
        DST(3, 0) = avg2(C, D);
        DST(0, 3) = avg3(K, J, I);
        DST(0, 2) = avg3(J, I, X);
        DST(0, 1) = DST(1, 3) = avg3(I, X, A);
        DST(1, 1) = DST(2, 3) = avg3(X, A, B);
        DST(2, 1) = DST(3, 3) = avg3(A, B, C);
        DST(3, 1) = avg3(B, C, D);
        break;
    case 6:
        DST(0, 0) = avg3(A, B, C);
        DST(1, 0) = DST(0, 1) = avg3(B, C, D);
        DST(2, 0) = DST(1, 1) = DST(0, 2) = avg3(C, D, E);
        DST(3, 0) = DST(2, 1) = DST(1, 2) = DST(0, 3) = avg3(D, E, F);
        DST(3, 1) = DST(2, 2) = DST(1, 3) = avg3(E, F, G);
        DST(3, 2) = DST(2, 3) = avg3(F, G, H);
        DST(3, 3) = avg3(G, H, H);
        break;
    case 7:
        DST(0, 0) = avg2(A, B);
        DST(1, 0) = DST(0, 2) = avg2(B, C);
        DST(2, 0) = DST(1, 2) = avg2(C, D);
        DST(3, 0) = DST(2, 2) = avg2(D, E);
        DST(0, 1) = avg3(A, B, C);
        DST(1, 1) = DST(0, 3) = avg3(B, C, D);
        DST(2, 1) = DST(1, 3) = avg3(C, D, E);
        DST(3, 1) = DST(2, 3) = avg3(D, E, F);
        DST(3, 2) = avg3(E, F, G);
        DST(3, 3) = avg3(F, G, H);
        break;
    case 8:
        DST(0, 0) = DST(2, 1) = avg2(I, X);
        DST(0, 1) = DST(2, 2) = avg2(J, I);
        DST(0, 2) = DST(2, 3) = avg2(K, J);
        DST(0, 3) = avg2(L, K);
        DST(3, 0) = avg3(A, B, C);
        DST(2, 0) = avg3(X, A, B);
        DST(1, 0) = DST(3, 1) = avg3(I, X, A);
        DST(1, 1) = DST(3, 2) = avg3(J, I, X);
        DST(1, 2) = DST(3, 3) = avg3(K, J, I);
        DST(1, 3) = avg3(L, K, J);
        break;
    default:
        DST(0, 0) = avg2(I, J);
        DST(2, 0) = DST(0, 1) = avg2(J, K);
        DST(2, 1) = DST(0, 2) = avg2(K, L);
        DST(1, 0) = avg3(I, J, K);
        DST(3, 0) = DST(1, 1) = avg3(J, K, L);
        DST(3, 1) = DST(1, 2) = avg3(K, L, L);
        DST(3, 2) = DST(2, 2) = DST(0, 3) = DST(1, 3) = DST(2, 3) = DST(3, 3) = (uint8_t)L;
        break;
    }
#undef DST
}

// ---- per-MB record the device hands to the host bitstream writer ----
struct alignas(16) XMB {
    uint8_t ymode;      // 0..3 i16 DC/TM/V/H, 4 = intra-4
    uint8_t uvmode;
    uint8_t seg;
    uint8_t pad;
    uint8_t bmodes[16];
    int16_t dc[16];     // i16: the Y2 levels (zigzag)
    int16_t ac[16][16]; // luma levels per block (raster block order), zigzag
    int16_t uv[8][16];  // U blocks 0..3, V 4..7
    uint8_t pad2[12];   // a whole number of 16-byte stores
};
static_assert(sizeof(XMB) == 832, "XMB is stored as 52 16-byte words");

// The token statistics of one MB (frame_enc.c RecordTokens, token_enc.c
// VP8RecordCoeffTokens' statistics side); nz contexts in/out like the iterator's.
IK_HD int record_stats(int bit, uint32_t* s) {
    uint32_t p = *s;
    if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
    p += 0x00010000u + (uint32_t)bit;
    *s = p;
    return bit;
}

// ST(slot, bit) records one statistic (and returns bit); TOK(bit, id) sees every token
// (id: TOKEN_ID + node, or 0x4000 | a fixed probability)
template <typename ST, typename TOK>
IK_HD int record_coeff(ST st, int type, int first, int ctx, const int16_t* coeffs, TOK tok) {
    int last = -1;
    for (int n = 15; n >= 0; --n)
        if (coeffs[n]) { last = n; break; }
    int n = first;
    uint32_t base = (uint32_t)(11 * (ctx + 3 * (n + 8 * type)));
    uint32_t s = base;  // the statistics row (== base: ids and slots coincide but for node 10)
    auto add = [&](int bit, uint32_t id, uint32_t slot) { tok(bit, id); return st(slot, bit); };
    if (!add(last >= 0, base + 0, s + 0)) return 0;
    while (n < 16) {
        const int c = coeffs[n++];
        const int sign = c < 0;
        const uint32_t v = (uint32_t)(sign ? -c : c);
        if (!add(v != 0, base + 1, s + 1)) {
            base = s = (uint32_t)(11 * (0 + 3 * (kEncBands[n] + 8 * type)));
            continue;
        }
        if (!add(v > 1, base + 2, s + 2)) {
            base = s = (uint32_t)(11 * (1 + 3 * (kEncBands[n] + 8 * type)));
        } else {
            if (!add(v > 4, base + 3, s + 3)) {
                if (add(v != 2, base + 4, s + 4)) add(v == 4, base + 5, s + 5);
            } else if (!add(v > 10, base + 6, s + 6)) {
                if (!add(v > 6, base + 7, s + 7)) {
                    tok(v == 6, 0x4000u | 159);
                } else {
                    tok(v >= 9, 0x4000u | 165);
                    tok(!(v & 1), 0x4000u | 145);
                }
            } else {
                constexpr uint8_t kCat3[] = {173, 148, 140, 0};
                constexpr uint8_t kCat4[] = {176, 155, 140, 135, 0};
                constexpr uint8_t kCat5[] = {180, 157, 141, 134, 130, 0};
                constexpr uint8_t kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};
                int mask;
                const uint8_t* tab;
                uint32_t residue = v - 3;
                if (residue < (8 << 1)) {
                    add(0, base + 8, s + 8);
                    add(0, base + 9, s + 9);
                    residue -= (8 << 0);
                    mask = 1 << 2;
                    tab = kCat3;
                } else if (residue < (8 << 2)) {
                    add(0, base + 8, s + 8);
                    add(1, base + 9, s + 9);
                    residue -= (8 << 1);
                    mask = 1 << 3;
                    tab = kCat4;
                } else if (residue < (8 << 3)) {  // (libwebp: node 10's bit counted at stats slot 9)
                    add(1, base + 8, s + 8);
                    add(0, base + 10, s + 9);
                    residue -= (8 << 2);
                    mask = 1 << 4;
                    tab = kCat5;
                } else {
                    add(1, base + 8, s + 8);
                    add(1, base + 10, s + 9);
                    residue -= (8 << 3);
                    mask = 1 << 10;
                    tab = kCat6;
                }
                while (mask) {
                    tok((residue & (uint32_t)mask) != 0, 0x4000u | *tab++);
                    mask >>= 1;
                }
            }
            base = s = (uint32_t)(11 * (2 + 3 * (kEncBands[n] + 8 * type)));
        }
        tok(sign, 0x4000u | 128);
        if (n == 16 || !add(n <= last, base + 0, s + 0)) return 1;
    }
    return 1;
}

// one MB's tokens in RecordTokens order; tnz/lnz: the iterator's top_nz[9] / left_nz[9]
template <typename ST, typename TOK>
IK_HD void record_mb(ST st, const XMB& m, int* tnz, int* lnz, TOK tok) {
    int first = 0, type = 3;
    if (m.ymode != 4) {
        const int ctx = tnz[8] + lnz[8];
        tnz[8] = lnz[8] = record_coeff(st, 1, 0, ctx, m.dc, tok);
        first = 1;
        type = 0;
    }
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) tnz[x] = lnz[y] = record_coeff(st, type, first, tnz[x] + lnz[y], m.ac[x + 4 * y], tok);
    for (int ch = 0; ch <= 2; ch += 2)
        for (int y = 0; y < 2; ++y)
            for (int x = 0; x < 2; ++x)
                tnz[4 + ch + x] = lnz[4 + ch + y] =
                    record_coeff(st, 2, 0, tnz[4 + ch + x] + lnz[4 + ch + y], m.uv[ch * 2 + x + y * 2], tok);
}

// FinalizeTokenProbas: the probabilities the stats say are worth their update cost
IK_HD int finalize_proba(uint32_t stats, int i) {
    const int nb = (int)(stats & 0xffff), total = (int)((stats >> 16) & 0xffff);
    const int upd = kCoeffUpdateProbs[i], old_p = kCoeffProbs0[i];
    const int new_p = nb ? (255 - nb * 255 / total) : 255;
    const int old_cost = nb * bit_cost(1, old_p) + (total - nb) * bit_cost(0, old_p) + bit_cost(0, upd);
    const int new_cost = nb * bit_cost(1, new_p) + (total - nb) * bit_cost(0, new_p) + bit_cost(1, upd) + 8 * 256;
    return old_cost > new_cost ? new_p : old_p;
}

}  // namespace vp8x
}  // namespace ik
