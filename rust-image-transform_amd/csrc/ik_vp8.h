// ik_vp8.h -- VP8 key-frame macroblock coding shared by the GPU encoder
// (ik_vp8.hip) and the host bitstream writer (ik_vp8_enc.cpp): the encode_image
// WebP branch (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp) done
// MI355X-side.  Bitstream semantics follow RFC 6386 as implemented by libwebp's
// decoder (the decoder every WebP consumer runs): intra predictors with the
// 127/129 frame-edge fill, the 4x4 top-right rules, the islow-free VP8 inverse
// DCT / WHT, and the coefficient token tree.  The forward transforms and the
// quantiser follow libwebp's encoder (FTransform, FTransformWHT, QFIX 17 with
// kBiasMatrices); mode decisions are rate-distortion with the bit costs of the
// default probabilities.
#pragma once
#include <cstdint>

#include "ik_vp8_tables.h"

#if defined(__HIPCC__)
#define IK_HD __host__ __device__ inline
#define IK_UNROLL _Pragma("unroll")
#else
#define IK_HD inline
#define IK_UNROLL _Pragma("GCC unroll 16")
#endif

namespace ik {
namespace vp8 {

// libwebp's mode numbering: 4x4 modes, and the 16x16 / chroma modes that share
// the values of their 4x4 counterparts (used as contexts by neighbouring B_PRED MBs)
enum { B_DC = 0, B_TM, B_VE, B_HE, B_RD, B_VR, B_LD, B_VL, B_HD, B_HU, NUM_BMODES };
enum { DC_PRED = B_DC, TM_PRED = B_TM, V_PRED = B_VE, H_PRED = B_HE, B_PRED = 10 };

constexpr int kBps = 32;  // stride of the per-MB work buffers

IK_HD int zigzag(int n) {
    constexpr uint8_t z[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
    return z[n];
}
IK_HD int izigzag(int j) {  // raster position -> zigzag index
    constexpr uint8_t iz[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
    return iz[j];
}
IK_HD int band(int n) {
    constexpr uint8_t b[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
    return b[n];
}
IK_HD int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
IK_HD constexpr int cost0(int p) { return kBitCost[p]; }         // 1/256 bit, coding 0 with P(0)=p/256
IK_HD constexpr int cost1(int p) { return kBitCost[256 - p]; }   // coding 1
IK_HD constexpr int costb(int p, int b) { return b ? cost1(p) : cost0(p); }
IK_HD const uint8_t* coef_probs(const uint8_t* probs, int type, int bnd, int ctx) {
    return probs + ((type * 8 + bnd) * 3 + ctx) * 11;
}

// ---- quantisation (dequant factors exactly as libwebp's decoder derives them) ----
struct QMat {
    int q[2];     // dequant step [dc, ac]
    int iq[2];    // (1 << 17) / q
    int bias[2];  // rounding bias, QFIX 17
};
struct QParams {
    QMat y1, y2, uv;
    int qindex, lambda, filter_level;
    int dq_uv_dc;
};
IK_HD int clipi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
IK_HD void make_qmat(QMat& m, int qdc, int qac, int bdc, int bac) {
    m.q[0] = qdc; m.q[1] = qac;
    m.iq[0] = (1 << 17) / qdc; m.iq[1] = (1 << 17) / qac;
    m.bias[0] = bdc << 9; m.bias[1] = bac << 9;  // libwebp BIAS(b) = b << (QFIX - 8)
}
// q: quantiser index 0..127; dq_uv_dc: chroma DC delta (libwebp: -4 * sns / 100)
IK_HD QParams make_qparams(int q, int dq_uv_dc) {
    QParams p{};
    p.qindex = q;
    p.dq_uv_dc = dq_uv_dc;
    const int y2ac = (kAcTable[q] * 101581) >> 16;
    make_qmat(p.y1, kDcTable[q], kAcTable[q], 96, 110);
    make_qmat(p.y2, kDcTable[q] * 2, y2ac < 8 ? 8 : y2ac, 96, 108);
    make_qmat(p.uv, kDcTable[clipi(q + dq_uv_dc, 0, 117)], kAcTable[q], 110, 115);
    const int qa = kAcTable[q];
    p.lambda = (3 * qa * qa) >> 7;
    if (p.lambda < 1) p.lambda = 1;
    // libwebp SetupFilterStrength, filter_strength 60, sharpness 0, one segment
    const int qstep = kAcTable[q] >> 2;
    const int base = qstep < 63 ? qstep : 63;
    int f = base * 300 / 256;
    p.filter_level = f < 2 ? 0 : (f > 63 ? 63 : f);
    return p;
}

// ---- transforms ----
// libwebp FTransform: residual (src - ref) -> 16 coefficients (raster order)
IK_HD void fdct4(const uint8_t* src, int ss, const uint8_t* ref, int rs, int16_t* out) {
    int tmp[16];
    for (int i = 0; i < 4; ++i) {
        const int d0 = src[i * ss + 0] - ref[i * rs + 0], d1 = src[i * ss + 1] - ref[i * rs + 1];
        const int d2 = src[i * ss + 2] - ref[i * rs + 2], d3 = src[i * ss + 3] - ref[i * rs + 3];
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
// libwebp FTransformWHT over the 16 luma DCs (dc[i] = DC of block i, raster)
IK_HD void fwht(const int16_t* dc, int16_t* out) {
    int tmp[16];
    for (int i = 0; i < 4; ++i) {
        const int a0 = dc[i * 4 + 0] + dc[i * 4 + 2], a1 = dc[i * 4 + 1] + dc[i * 4 + 3];
        const int a2 = dc[i * 4 + 1] - dc[i * 4 + 3], a3 = dc[i * 4 + 0] - dc[i * 4 + 2];
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
// decoder inverse WHT (libwebp TransformWHT): dequantised Y2 -> the 16 block DCs
IK_HD void iwht(const int16_t* in, int16_t* dc) {
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
        const int d = tmp[0 + i * 4] + 3;
        const int a0 = d + tmp[3 + i * 4], a1 = tmp[1 + i * 4] + tmp[2 + i * 4];
        const int a2 = tmp[1 + i * 4] - tmp[2 + i * 4], a3 = d - tmp[3 + i * 4];
        dc[i * 4 + 0] = (int16_t)((a0 + a1) >> 3);
        dc[i * 4 + 1] = (int16_t)((a3 + a2) >> 3);
        dc[i * 4 + 2] = (int16_t)((a0 - a1) >> 3);
        dc[i * 4 + 3] = (int16_t)((a3 - a2) >> 3);
    }
}
// decoder inverse DCT + add (libwebp TransformOne): dst = clip(pred + idct(in))
IK_HD int mul1(int a) { return ((a * 20091) >> 16) + a; }
IK_HD int mul2(int a) { return (a * 35468) >> 16; }
IK_HD void idct4_add(const int16_t* in, const uint8_t* pred, int ps, uint8_t* dst, int ds) {
    int tmp[16];
    for (int i = 0; i < 4; ++i) {  // vertical pass
        const int a = in[0 + i] + in[8 + i], b = in[0 + i] - in[8 + i];
        const int c = mul2(in[4 + i]) - mul1(in[12 + i]), d = mul1(in[4 + i]) + mul2(in[12 + i]);
        tmp[0 + i * 4] = a + d;
        tmp[1 + i * 4] = b + c;
        tmp[2 + i * 4] = b - c;
        tmp[3 + i * 4] = a - d;
    }
    for (int i = 0; i < 4; ++i) {  // horizontal pass
        const int dc = tmp[0 + i] + 4;
        const int a = dc + tmp[8 + i], b = dc - tmp[8 + i];
        const int c = mul2(tmp[4 + i]) - mul1(tmp[12 + i]), d = mul1(tmp[4 + i]) + mul2(tmp[12 + i]);
        dst[i * ds + 0] = (uint8_t)clip8(pred[i * ps + 0] + ((a + d) >> 3));
        dst[i * ds + 1] = (uint8_t)clip8(pred[i * ps + 1] + ((b + c) >> 3));
        dst[i * ds + 2] = (uint8_t)clip8(pred[i * ps + 2] + ((b - c) >> 3));
        dst[i * ds + 3] = (uint8_t)clip8(pred[i * ps + 3] + ((a - d) >> 3));
    }
}

// quantise coefficients [first, 16) in zigzag order; coef (raster) is replaced by
// its dequantised value; returns the zigzag index after the last nonzero level
// (== first when none)
IK_HD int quantize(int16_t* coef, int16_t* lv, const QMat& m, int first) {
    int last = first;
    for (int n = 0; n < first; ++n) lv[n] = 0;
    for (int n = first; n < 16; ++n) {
        const int j = zigzag(n);
        const int c = coef[j];
        const int s = c < 0;
        const int a = s ? -c : c;
        const int k = n > 0;
        int l = (int)(((unsigned)a * (unsigned)m.iq[k] + (unsigned)m.bias[k]) >> 17);
        if (l > 2047) l = 2047;
        lv[n] = (int16_t)(s ? -l : l);
        coef[j] = (int16_t)((s ? -l : l) * m.q[k]);
        if (l) last = n + 1;
    }
    return last;
}

// rate of one block's tokens (1/256 bit) under `probs`, given its first-coefficient
// context; levels in zigzag order
IK_HD int large_cost(int v, const uint8_t* p) {
    if (v <= 4) {
        int c = cost0(p[3]);
        if (v == 2) return c + cost0(p[4]);
        return c + cost1(p[4]) + costb(p[5], v == 4);
    }
    int c = cost1(p[3]);
    if (v <= 10) {
        c += cost0(p[6]);
        if (v <= 6) return c + cost0(p[7]) + costb(159, v - 5);
        return c + cost1(p[7]) + costb(165, (v - 7) >> 1) + costb(145, (v - 7) & 1);
    }
    c += cost1(p[6]);
    const int cat = v <= 18 ? 0 : (v <= 34 ? 1 : (v <= 66 ? 2 : 3));
    c += costb(p[8], cat >> 1) + costb(p[9 + (cat >> 1)], cat & 1);
    const int nb = cat == 3 ? 11 : 3 + cat;
    // extra bits: ~1 bit each at their (near-128) probabilities
    return c + nb * 256;
}
IK_HD int block_cost(const int16_t* lv, int first, int last, int ctx, int type, const uint8_t* probs) {
    int n = first;
    const uint8_t* p = coef_probs(probs, type, band(n), ctx);
    if (last <= first) return cost0(p[0]);
    int cost = 0;
    for (;;) {
        cost += cost1(p[0]);
        while (lv[n] == 0) {
            cost += cost0(p[1]);
            ++n;
            p = coef_probs(probs, type, band(n), 0);
        }
        cost += cost1(p[1]);
        const int v = lv[n] < 0 ? -lv[n] : lv[n];
        int nctx;
        if (v == 1) { cost += cost0(p[2]); nctx = 1; }
        else { cost += cost1(p[2]) + large_cost(v, p); nctx = 2; }
        cost += 256;  // sign
        ++n;
        if (n == 16) return cost;
        p = coef_probs(probs, type, band(n), nctx);
        if (n >= last) return cost + cost0(p[0]);
    }
}

// block_cost(lv, FIRST, last, ctx0, TYPE, kCoeffProbs0), restated position by
// position for levels held in registers: the cost of zigzag position n depends
// only on lv[n-1] (its context and whether an end-of-block flag precedes it) and
// lv[n], and with the default probabilities every probability is a compile-time
// constant once the loop is unrolled -- the three contexts become selects, no
// table loads.  Same value as block_cost (tests/test_vp8_host.py).
IK_HD int sel3(int c, int a0, int a1, int a2) { return c == 0 ? a0 : (c == 1 ? a1 : a2); }
template <int TYPE>
IK_HD int pc0(int b, int c, int k) { return cost0(kCoeffProbs0[((TYPE * 8 + b) * 3 + c) * 11 + k]); }
template <int TYPE>
IK_HD int pc1(int b, int c, int k) { return cost1(kCoeffProbs0[((TYPE * 8 + b) * 3 + c) * 11 + k]); }
template <int TYPE>
IK_HD int large_cost_fixed(int v, int b, int c) {
#define IK_C0(k) sel3(c, pc0<TYPE>(b, 0, k), pc0<TYPE>(b, 1, k), pc0<TYPE>(b, 2, k))
#define IK_C1(k) sel3(c, pc1<TYPE>(b, 0, k), pc1<TYPE>(b, 1, k), pc1<TYPE>(b, 2, k))
    if (v <= 4) {
        if (v == 2) return IK_C0(3) + IK_C0(4);
        return IK_C0(3) + IK_C1(4) + (v == 4 ? IK_C1(5) : IK_C0(5));
    }
    if (v <= 10) {
        if (v <= 6) return IK_C1(3) + IK_C0(6) + IK_C0(7) + costb(159, v - 5);
        return IK_C1(3) + IK_C0(6) + IK_C1(7) + costb(165, (v - 7) >> 1) + costb(145, (v - 7) & 1);
    }
    const int cat = v <= 18 ? 0 : (v <= 34 ? 1 : (v <= 66 ? 2 : 3));
    const int c8 = (cat >> 1) ? IK_C1(8) : IK_C0(8);
    const int c9 = (cat >> 1) ? ((cat & 1) ? IK_C1(10) : IK_C0(10)) : ((cat & 1) ? IK_C1(9) : IK_C0(9));
    const int nb = cat == 3 ? 11 : 3 + cat;
    return IK_C1(3) + IK_C1(6) + c8 + c9 + nb * 256;
#undef IK_C0
#undef IK_C1
}
template <int TYPE, int FIRST>
IK_HD int block_cost_fixed(const int16_t* lv, int last, int ctx0) {
    if (last <= FIRST)
        return sel3(ctx0, pc0<TYPE>(band(FIRST), 0, 0), pc0<TYPE>(band(FIRST), 1, 0), pc0<TYPE>(band(FIRST), 2, 0));
    int cost = 0, pc = ctx0;
    bool chk = true;  // an end-of-block flag is coded before this position
IK_UNROLL
    for (int n = FIRST; n < 16; ++n) {
        const int b = band(n);
        const int v = lv[n] < 0 ? -lv[n] : lv[n];
        if (n < last) {
            int c = chk ? sel3(pc, pc1<TYPE>(b, 0, 0), pc1<TYPE>(b, 1, 0), pc1<TYPE>(b, 2, 0)) : 0;
            if (v == 0) {
                c += sel3(pc, pc0<TYPE>(b, 0, 1), pc0<TYPE>(b, 1, 1), pc0<TYPE>(b, 2, 1));
            } else {
                c += sel3(pc, pc1<TYPE>(b, 0, 1), pc1<TYPE>(b, 1, 1), pc1<TYPE>(b, 2, 1)) + 256;
                if (v == 1) c += sel3(pc, pc0<TYPE>(b, 0, 2), pc0<TYPE>(b, 1, 2), pc0<TYPE>(b, 2, 2));
                else c += sel3(pc, pc1<TYPE>(b, 0, 2), pc1<TYPE>(b, 1, 2), pc1<TYPE>(b, 2, 2)) + large_cost_fixed<TYPE>(v, b, pc);
            }
            cost += c;
        } else if (n == last) {
            cost += sel3(pc, pc0<TYPE>(b, 0, 0), pc0<TYPE>(b, 1, 0), pc0<TYPE>(b, 2, 0));  // end of block
        }
        pc = v == 0 ? 0 : (v == 1 ? 1 : 2);
        chk = v != 0;
    }
    return cost;
}

// Token-cost rows for one block type under the default probabilities, per
// (band, ctx): {c1(p0), c0(p0), c0(p1), c1(p1) + 256 (sign), c0(p2), c1(p2), 0, 0,
// then c0(pk), c1(pk) for k = 3..10} -- what block_cost reads, as a table the
// GPU's position-parallel token cost gathers from LDS.
struct TokCostTab { uint16_t v[8][3][24]; };
constexpr TokCostTab make_tok_cost(int type) {
    TokCostTab t{};
    for (int b = 0; b < 8; ++b)
        for (int c = 0; c < 3; ++c) {
            const uint8_t* p = kCoeffProbs0 + ((type * 8 + b) * 3 + c) * 11;
            uint16_t* r = t.v[b][c];
            r[0] = (uint16_t)cost1(p[0]); r[1] = (uint16_t)cost0(p[0]); r[2] = (uint16_t)cost0(p[1]);
            r[3] = (uint16_t)(cost1(p[1]) + 256); r[4] = (uint16_t)cost0(p[2]); r[5] = (uint16_t)cost1(p[2]);
            for (int k = 3; k <= 10; ++k) { r[8 + 2 * (k - 3)] = (uint16_t)cost0(p[k]); r[9 + 2 * (k - 3)] = (uint16_t)cost1(p[k]); }
        }
    return t;
}
constexpr TokCostTab kTokCostI4 = make_tok_cost(3);
// large_cost(v, p) from a row's c0/c1 of p3..p10 (r16[2*(k-3) + bit])
IK_HD int large_cost_row(int v, const uint16_t* r16) {
#define IK_R(k, bit) (int)r16[2 * ((k) - 3) + (bit)]
    if (v <= 4) {
        if (v == 2) return IK_R(3, 0) + IK_R(4, 0);
        return IK_R(3, 0) + IK_R(4, 1) + IK_R(5, v == 4);
    }
    if (v <= 10) {
        if (v <= 6) return IK_R(3, 1) + IK_R(6, 0) + IK_R(7, 0) + costb(159, v - 5);
        return IK_R(3, 1) + IK_R(6, 0) + IK_R(7, 1) + costb(165, (v - 7) >> 1) + costb(145, (v - 7) & 1);
    }
    const int cat = v <= 18 ? 0 : (v <= 34 ? 1 : (v <= 66 ? 2 : 3));
    const int nb = cat == 3 ? 11 : 3 + cat;
    return IK_R(3, 1) + IK_R(6, 1) + IK_R(8, cat >> 1) + IK_R(9 + (cat >> 1), cat & 1) + nb * 256;
#undef IK_R
}

IK_HD constexpr int bmode_cost(int mode, int top, int left) {
    const uint8_t* p = kBModeProbs + (top * 10 + left) * 9;
    // libwebp kYModesIntra4 tree
    switch (mode) {
    case B_DC: return cost0(p[0]);
    case B_TM: return cost1(p[0]) + cost0(p[1]);
    case B_VE: return cost1(p[0]) + cost1(p[1]) + cost0(p[2]);
    default: break;
    }
    int c = cost1(p[0]) + cost1(p[1]) + cost1(p[2]);
    switch (mode) {
    case B_HE: return c + cost0(p[3]) + cost0(p[4]);
    case B_RD: return c + cost0(p[3]) + cost1(p[4]) + cost0(p[5]);
    case B_VR: return c + cost0(p[3]) + cost1(p[4]) + cost1(p[5]);
    case B_LD: return c + cost1(p[3]) + cost0(p[6]);
    case B_VL: return c + cost1(p[3]) + cost1(p[6]) + cost0(p[7]);
    case B_HD: return c + cost1(p[3]) + cost1(p[6]) + cost1(p[7]) + cost0(p[8]);
    default: return c + cost1(p[3]) + cost1(p[6]) + cost1(p[7]) + cost1(p[8]);
    }
}
struct BModeCostTab { uint16_t v[NUM_BMODES][NUM_BMODES][NUM_BMODES]; };  // [top][left][mode]
constexpr BModeCostTab make_bmode_cost() {
    BModeCostTab t{};
    for (int a = 0; a < NUM_BMODES; ++a)
        for (int l = 0; l < NUM_BMODES; ++l)
            for (int m = 0; m < NUM_BMODES; ++m) t.v[a][l][m] = (uint16_t)bmode_cost(m, a, l);
    return t;
}
constexpr BModeCostTab kBModeCost = make_bmode_cost();

IK_HD int ymode_cost(int m) {  // key-frame y mode: B_PRED / DC / V / H / TM
    if (m == B_PRED) return cost0(145);
    const int c = cost1(145);
    if (m == DC_PRED) return c + cost0(156) + cost0(163);
    if (m == V_PRED) return c + cost0(156) + cost1(163);
    if (m == H_PRED) return c + cost1(156) + cost0(128);
    return c + cost1(156) + cost1(128);
}
IK_HD int uvmode_cost(int m) {
    if (m == DC_PRED) return cost0(142);
    if (m == V_PRED) return cost1(142) + cost0(114);
    if (m == H_PRED) return cost1(142) + cost1(114) + cost0(183);
    return cost1(142) + cost1(114) + cost1(183);
}

// ---- predictors (libwebp dec.c), dst has its context at dst[-1], dst[-kBps] ----
IK_HD int avg3(int a, int b, int c) { return (a + 2 * b + c + 2) >> 2; }
IK_HD int avg2(int a, int b) { return (a + b + 1) >> 1; }

// 4x4 prediction of mode m for the block whose top-left pixel is at ctx (work
// buffer, stride kBps); writes pred[16] (stride 4)
IK_HD void pred4(int m, const uint8_t* d, uint8_t* pr) {
    const int X = d[-1 - kBps];
    const int A = d[0 - kBps], B = d[1 - kBps], C = d[2 - kBps], D = d[3 - kBps];
    const int E = d[4 - kBps], F = d[5 - kBps], G = d[6 - kBps], H = d[7 - kBps];
    const int I = d[-1], J = d[-1 + kBps], K = d[-1 + 2 * kBps], L = d[-1 + 3 * kBps];
#define P(x, y) pr[(x) + (y) * 4]
    switch (m) {
    case B_DC: {
        const int v = (A + B + C + D + I + J + K + L + 4) >> 3;
        for (int i = 0; i < 16; ++i) pr[i] = (uint8_t)v;
        break;
    }
    case B_TM: {
        const int top[4] = {A, B, C, D}, left[4] = {I, J, K, L};
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) P(x, y) = (uint8_t)clip8(top[x] + left[y] - X);
        break;
    }
    case B_VE: {
        const int v0 = avg3(X, A, B), v1 = avg3(A, B, C), v2 = avg3(B, C, D), v3 = avg3(C, D, E);
        for (int y = 0; y < 4; ++y) { P(0, y) = v0; P(1, y) = v1; P(2, y) = v2; P(3, y) = v3; }
        break;
    }
    case B_HE: {
        const int r[4] = {avg3(X, I, J), avg3(I, J, K), avg3(J, K, L), avg3(K, L, L)};
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) P(x, y) = (uint8_t)r[y];
        break;
    }
    case B_RD:
        P(0, 3) = avg3(J, K, L);
        P(1, 3) = P(0, 2) = avg3(I, J, K);
        P(2, 3) = P(1, 2) = P(0, 1) = avg3(X, I, J);
        P(3, 3) = P(2, 2) = P(1, 1) = P(0, 0) = avg3(A, X, I);
        P(3, 2) = P(2, 1) = P(1, 0) = avg3(B, A, X);
        P(3, 1) = P(2, 0) = avg3(C, B, A);
        P(3, 0) = avg3(D, C, B);
        break;
    case B_VR:
        P(0, 0) = P(1, 2) = avg2(X, A);
        P(1, 0) = P(2, 2) = avg2(A, B);
        P(2, 0) = P(3, 2) = avg2(B, C);
        P(3, 0) = avg2(C, D);
        P(0, 3) = avg3(K, J, I);
        P(0, 2) = avg3(J, I, X);
        P(0, 1) = P(1, 3) = avg3(I, X, A);
        P(1, 1) = P(2, 3) = avg3(X, A, B);
        P(2, 1) = P(3, 3) = avg3(A, B, C);
        P(3, 1) = avg3(B, C, D);
        break;
    case B_LD:
        P(0, 0) = avg3(A, B, C);
        P(1, 0) = P(0, 1) = avg3(B, C, D);
        P(2, 0) = P(1, 1) = P(0, 2) = avg3(C, D, E);
        P(3, 0) = P(2, 1) = P(1, 2) = P(0, 3) = avg3(D, E, F);
        P(3, 1) = P(2, 2) = P(1, 3) = avg3(E, F, G);
        P(3, 2) = P(2, 3) = avg3(F, G, H);
        P(3, 3) = avg3(G, H, H);
        break;
    case B_VL:
        P(0, 0) = avg2(A, B);
        P(1, 0) = P(0, 2) = avg2(B, C);
        P(2, 0) = P(1, 2) = avg2(C, D);
        P(3, 0) = P(2, 2) = avg2(D, E);
        P(0, 1) = avg3(A, B, C);
        P(1, 1) = P(0, 3) = avg3(B, C, D);
        P(2, 1) = P(1, 3) = avg3(C, D, E);
        P(3, 1) = P(2, 3) = avg3(D, E, F);
        P(3, 2) = avg3(E, F, G);
        P(3, 3) = avg3(F, G, H);
        break;
    case B_HD:
        P(0, 0) = P(2, 1) = avg2(I, X);
        P(0, 1) = P(2, 2) = avg2(J, I);
        P(0, 2) = P(2, 3) = avg2(K, J);
        P(0, 3) = avg2(L, K);
        P(3, 0) = avg3(A, B, C);
        P(2, 0) = avg3(X, A, B);
        P(1, 0) = P(3, 1) = avg3(I, X, A);
        P(1, 1) = P(3, 2) = avg3(J, I, X);
        P(1, 2) = P(3, 3) = avg3(K, J, I);
        P(1, 3) = avg3(L, K, J);
        break;
    default:  // B_HU
        P(0, 0) = avg2(I, J);
        P(2, 0) = P(0, 1) = avg2(J, K);
        P(2, 1) = P(0, 2) = avg2(K, L);
        P(1, 0) = avg3(I, J, K);
        P(3, 0) = P(1, 1) = avg3(J, K, L);
        P(3, 1) = P(1, 2) = avg3(K, L, L);
        P(3, 2) = P(2, 2) = P(0, 3) = P(1, 3) = P(2, 3) = P(3, 3) = L;
        break;
    }
#undef P
}

// pred4 restated as one tap descriptor per (mode, pixel) over the 13 context
// samples 0:X 1..8:A..H 9..12:I..L -- so lanes predicting different modes run the
// same instructions (the GPU kernel's lane = (mode, row)).  kind<<12 | i0<<8 | i1<<4 | i2.
enum { P4_CP = 0, P4_A2, P4_A3, P4_TM, P4_DC };
constexpr uint16_t p4d(int kind, int a, int b = 0, int c = 0) {
    return (uint16_t)(kind << 12 | a << 8 | b << 4 | c);
}
#define CP(a) p4d(P4_CP, a)
#define A2(a, b) p4d(P4_A2, a, b)
#define A3(a, b, c) p4d(P4_A3, a, b, c)
#define TM(x, y) p4d(P4_TM, 1 + (x), 9 + (y), 0)
#define DC p4d(P4_DC, 0)
constexpr uint16_t kPred4Tab[NUM_BMODES][16] = {
    // B_DC
    {DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC, DC},
    // B_TM
    {TM(0, 0), TM(1, 0), TM(2, 0), TM(3, 0), TM(0, 1), TM(1, 1), TM(2, 1), TM(3, 1),
     TM(0, 2), TM(1, 2), TM(2, 2), TM(3, 2), TM(0, 3), TM(1, 3), TM(2, 3), TM(3, 3)},
    // B_VE: avg3 of the top row around column x (X left of A)
    {A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5), A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5),
     A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5), A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5)},
    // B_HE
    {A3(0, 9, 10), A3(0, 9, 10), A3(0, 9, 10), A3(0, 9, 10), A3(9, 10, 11), A3(9, 10, 11), A3(9, 10, 11),
     A3(9, 10, 11), A3(10, 11, 12), A3(10, 11, 12), A3(10, 11, 12), A3(10, 11, 12), A3(11, 12, 12),
     A3(11, 12, 12), A3(11, 12, 12), A3(11, 12, 12)},
    // B_RD: avg3 along the down-right diagonal of L K J I X A B C D
    {A3(9, 0, 1), A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4), A3(10, 9, 0), A3(9, 0, 1), A3(0, 1, 2), A3(1, 2, 3),
     A3(11, 10, 9), A3(10, 9, 0), A3(9, 0, 1), A3(0, 1, 2), A3(12, 11, 10), A3(11, 10, 9), A3(10, 9, 0), A3(9, 0, 1)},
    // B_VR
    {A2(0, 1), A2(1, 2), A2(2, 3), A2(3, 4), A3(9, 0, 1), A3(0, 1, 2), A3(1, 2, 3), A3(2, 3, 4),
     A3(10, 9, 0), A2(0, 1), A2(1, 2), A2(2, 3), A3(11, 10, 9), A3(9, 0, 1), A3(0, 1, 2), A3(1, 2, 3)},
    // B_LD: avg3 along the down-left diagonal (H repeated)
    {A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5), A3(4, 5, 6), A3(2, 3, 4), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7),
     A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7), A3(6, 7, 8), A3(4, 5, 6), A3(5, 6, 7), A3(6, 7, 8), A3(7, 8, 8)},
    // B_VL
    {A2(1, 2), A2(2, 3), A2(3, 4), A2(4, 5), A3(1, 2, 3), A3(2, 3, 4), A3(3, 4, 5), A3(4, 5, 6),
     A2(2, 3), A2(3, 4), A2(4, 5), A3(5, 6, 7), A3(2, 3, 4), A3(3, 4, 5), A3(4, 5, 6), A3(6, 7, 8)},
    // B_HD
    {A2(9, 0), A3(9, 0, 1), A3(0, 1, 2), A3(1, 2, 3), A2(10, 9), A3(10, 9, 0), A2(9, 0), A3(9, 0, 1),
     A2(11, 10), A3(11, 10, 9), A2(10, 9), A3(10, 9, 0), A2(12, 11), A3(12, 11, 10), A2(11, 10), A3(11, 10, 9)},
    // B_HU
    {A2(9, 10), A3(9, 10, 11), A2(10, 11), A3(10, 11, 12), A2(10, 11), A3(10, 11, 12), A2(11, 12), A3(11, 12, 12),
     A2(11, 12), A3(11, 12, 12), CP(12), CP(12), CP(12), CP(12), CP(12), CP(12)},
};
#undef CP
#undef A2
#undef A3
#undef TM
#undef DC
IK_HD int p4_off(int i) { return i == 0 ? -1 - kBps : (i <= 8 ? i - 1 - kBps : -1 + (i - 9) * kBps); }
// pixel p (= y*4 + x) of pred4(m, d, .); dcv = the block's B_DC value
IK_HD int pred4_px(int m, int p, const uint8_t* d, int dcv) {
    const int t = kPred4Tab[m][p];
    const int kind = t >> 12;
    const int a = d[p4_off((t >> 8) & 15)], b = d[p4_off((t >> 4) & 15)], c = d[p4_off(t & 15)];
    switch (kind) {
    case P4_CP: return a;
    case P4_A2: return avg2(a, b);
    case P4_A3: return avg3(a, b, c);
    case P4_TM: return clip8(a + b - c);
    default: return dcv;
    }
}
IK_HD int pred4_dc(const uint8_t* d) {
    return (d[-kBps] + d[1 - kBps] + d[2 - kBps] + d[3 - kBps] + d[-1] + d[-1 + kBps] + d[-1 + 2 * kBps] +
            d[-1 + 3 * kBps] + 4) >> 3;
}

// NxN (16 luma / 8 chroma) prediction; mb_x/mb_y select libwebp's DC variants
IK_HD void pred_nxn(int m, int N, const uint8_t* d, int mb_x, int mb_y, uint8_t* pr) {
    if (m == DC_PRED) {
        int s = 0, v;
        const int sh = N == 16 ? 4 : 3;
        if (mb_x > 0 && mb_y > 0) {
            for (int i = 0; i < N; ++i) s += d[i - kBps] + d[-1 + i * kBps];
            v = (s + N) >> (sh + 1);
        } else if (mb_y > 0) {  // no left
            for (int i = 0; i < N; ++i) s += d[i - kBps];
            v = (s + (N >> 1)) >> sh;
        } else if (mb_x > 0) {  // no top
            for (int i = 0; i < N; ++i) s += d[-1 + i * kBps];
            v = (s + (N >> 1)) >> sh;
        } else {
            v = 0x80;
        }
        for (int i = 0; i < N * N; ++i) pr[i] = (uint8_t)v;
        return;
    }
    for (int y = 0; y < N; ++y)
        for (int x = 0; x < N; ++x) {
            int v;
            if (m == V_PRED) v = d[x - kBps];
            else if (m == H_PRED) v = d[-1 + y * kBps];
            else v = clip8(d[x - kBps] + d[-1 + y * kBps] - d[-1 - kBps]);  // TM
            pr[y * N + x] = (uint8_t)v;
        }
}

// One 4x4 block (bx, by) of the NxN prediction pred_nxn(m, N, ...) would write:
// the same values, computed for that block only (the GPU kernel's lanes each own
// one block of one mode).
IK_HD void pred_blk(int m, int N, const uint8_t* d, int mb_x, int mb_y, int bx, int by, uint8_t* pr) {
    if (m == DC_PRED) {
        int s = 0, v;
        const int sh = N == 16 ? 4 : 3;
        if (mb_x > 0 && mb_y > 0) {
            for (int i = 0; i < N; ++i) s += d[i - kBps] + d[-1 + i * kBps];
            v = (s + N) >> (sh + 1);
        } else if (mb_y > 0) {
            for (int i = 0; i < N; ++i) s += d[i - kBps];
            v = (s + (N >> 1)) >> sh;
        } else if (mb_x > 0) {
            for (int i = 0; i < N; ++i) s += d[-1 + i * kBps];
            v = (s + (N >> 1)) >> sh;
        } else {
            v = 0x80;
        }
        for (int i = 0; i < 16; ++i) pr[i] = (uint8_t)v;
        return;
    }
    const int x0 = bx * 4, y0 = by * 4;
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            int v;
            if (m == V_PRED) v = d[x0 + x - kBps];
            else if (m == H_PRED) v = d[-1 + (y0 + y) * kBps];
            else v = clip8(d[x0 + x - kBps] + d[-1 + (y0 + y) * kBps] - d[-1 - kBps]);
            pr[y * 4 + x] = (uint8_t)v;
        }
}

// ---- one macroblock, scalar (the reference encoder; the GPU kernel runs it per lane) ----
struct MBOut {
    uint8_t ymode, uvmode, skip, pad;
    uint8_t bmodes[16];
    int16_t lv[25][16];  // [0..15] Y (raster block order), [16..19] U, [20..23] V, [24] Y2; zigzag
};

// Context of one MB: source pixels and the unfiltered reconstruction around it.
struct MBCtx {
    int mb_x, mb_y, mb_w;
    uint8_t src_y[16 * 16], src_u[8 * 8], src_v[8 * 8];
    // work buffers: row -1 / column -1 context + the MB's reconstruction
    uint8_t y[17 * kBps], u[9 * kBps], v[9 * kBps];  // pixel (x,y) at [(y+1)*kBps + x + 1]
    uint8_t top_bmodes[4], left_bmodes[4];            // contexts for B_PRED mode coding
    uint8_t top_nz[9], left_nz[9];                    // [0..3] Y, [4..5] U, [6..7] V, [8] Y2
};

IK_HD int sse(const uint8_t* a, int as, const uint8_t* b, int bs, int w, int h) {
    int s = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const int d = a[y * as + x] - b[y * bs + x];
            s += d * d;
        }
    return s;
}

// i16 candidate: returns J = 256*SSE + lambda*R; fills levels/recon (16x16, stride 16)
IK_HD long long try_i16(const MBCtx& c, const QParams& q, const uint8_t* probs, int mode, int16_t lv[25][16],
                        uint8_t* rec) {
    uint8_t pr[256];
    const uint8_t* d = c.y + kBps + 1;
    pred_nxn(mode, 16, d, c.mb_x, c.mb_y, pr);
    int16_t coef[16][16], dc[16], y2[16], dcq[16];
    for (int b = 0; b < 16; ++b) {
        const int bx = (b & 3) * 4, by = (b >> 2) * 4;
        fdct4(c.src_y + by * 16 + bx, 16, pr + by * 16 + bx, 16, coef[b]);
        dc[b] = coef[b][0];
    }
    fwht(dc, y2);
    int rate = ymode_cost(mode);
    const int l2 = quantize(y2, lv[24], q.y2, 0);
    rate += block_cost(lv[24], 0, l2, c.top_nz[8] + c.left_nz[8], 1, probs);
    iwht(y2, dcq);
    int tnz[4] = {c.top_nz[0], c.top_nz[1], c.top_nz[2], c.top_nz[3]};
    int lnz[4] = {c.left_nz[0], c.left_nz[1], c.left_nz[2], c.left_nz[3]};
    for (int b = 0; b < 16; ++b) {
        const int bx = b & 3, by = b >> 2;
        const int last = quantize(coef[b], lv[b], q.y1, 1);
        rate += block_cost(lv[b], 1, last, tnz[bx] + lnz[by], 0, probs);
        tnz[bx] = lnz[by] = last > 1;
        coef[b][0] = dcq[b];
        idct4_add(coef[b], pr + by * 4 * 16 + bx * 4, 16, rec + by * 4 * 16 + bx * 4, 16);
    }
    const int dist = sse(c.src_y, 16, rec, 16, 16, 16);
    return 256ll * dist + (long long)q.lambda * rate;
}

IK_HD long long try_uv(const MBCtx& c, const QParams& q, const uint8_t* probs, int mode, int16_t lv[25][16],
                       uint8_t* rec_u, uint8_t* rec_v) {
    int rate = uvmode_cost(mode);
    int dist = 0;
    for (int ch = 0; ch < 2; ++ch) {
        uint8_t pr[64];
        const uint8_t* d = (ch ? c.v : c.u) + kBps + 1;
        const uint8_t* src = ch ? c.src_v : c.src_u;
        uint8_t* rec = ch ? rec_v : rec_u;
        pred_nxn(mode, 8, d, c.mb_x, c.mb_y, pr);
        int tnz[2] = {c.top_nz[4 + 2 * ch], c.top_nz[5 + 2 * ch]};
        int lnz[2] = {c.left_nz[4 + 2 * ch], c.left_nz[5 + 2 * ch]};
        for (int b = 0; b < 4; ++b) {
            const int bx = b & 1, by = b >> 1;
            int16_t coef[16];
            fdct4(src + by * 4 * 8 + bx * 4, 8, pr + by * 4 * 8 + bx * 4, 8, coef);
            int16_t* l = lv[16 + 4 * ch + b];
            const int last = quantize(coef, l, q.uv, 0);
            rate += block_cost(l, 0, last, tnz[bx] + lnz[by], 2, probs);
            tnz[bx] = lnz[by] = last > 0;
            idct4_add(coef, pr + by * 4 * 8 + bx * 4, 8, rec + by * 4 * 8 + bx * 4, 8);
        }
        dist += sse(src, 8, rec, 8, 8, 8);
    }
    return 256ll * dist + (long long)q.lambda * rate;
}

// Full RD decision for one MB; the chosen reconstruction is left in c.y/c.u/c.v
// (work-buffer interior).  `probs` = the coefficient probabilities used for rate.
IK_HD void encode_mb(MBCtx& c, const QParams& q, const uint8_t* probs, MBOut& o) {
    // --- luma 16x16 ---
    int16_t lv[25][16];
    uint8_t rec[256], best_rec[256];
    long long best = -1;
    int best_mode = DC_PRED;
    for (int m = 0; m < 4; ++m) {
        const int mode = m == 0 ? DC_PRED : (m == 1 ? V_PRED : (m == 2 ? H_PRED : TM_PRED));
        const long long j = try_i16(c, q, probs, mode, lv, rec);
        if (best < 0 || j < best) {
            best = j;
            best_mode = mode;
            for (int i = 0; i < 256; ++i) best_rec[i] = rec[i];
            for (int b = 0; b < 25; ++b)
                for (int i = 0; i < 16; ++i) o.lv[b][i] = lv[b][i];
        }
    }
    // --- luma 4x4 ---
    {
        uint8_t y4[17 * kBps];
        for (int i = 0; i < 17 * kBps; ++i) y4[i] = c.y[i];
        int16_t lv4[16][16];
        uint8_t bm[16];
        int tnz[4] = {c.top_nz[0], c.top_nz[1], c.top_nz[2], c.top_nz[3]};
        int lnz[4] = {c.left_nz[0], c.left_nz[1], c.left_nz[2], c.left_nz[3]};
        long long total = (long long)q.lambda * ymode_cost(B_PRED);
        bool ok = true;
        for (int b = 0; b < 16 && ok; ++b) {
            const int bx = b & 3, by = b >> 2;
            uint8_t* d = y4 + (by * 4 + 1) * kBps + bx * 4 + 1;
            const uint8_t* src = c.src_y + by * 4 * 16 + bx * 4;
            const int top = by ? bm[b - 4] : c.top_bmodes[bx];
            const int left = bx ? bm[b - 1] : c.left_bmodes[by];
            long long bj = -1;
            int bmode = 0, blast = 0;
            int16_t bl[16];
            uint8_t brec[16];
            for (int m = 0; m < NUM_BMODES; ++m) {
                uint8_t pr[16], r4[16];
                int16_t coef[16], l[16];
                pred4(m, d, pr);
                fdct4(src, 16, pr, 4, coef);
                const int last = quantize(coef, l, q.y1, 0);
                idct4_add(coef, pr, 4, r4, 4);
                const int rate = bmode_cost(m, top, left) + block_cost(l, 0, last, tnz[bx] + lnz[by], 3, probs);
                const long long j = 256ll * sse(src, 16, r4, 4, 4, 4) + (long long)q.lambda * rate;
                if (bj < 0 || j < bj) {
                    bj = j; bmode = m; blast = last;
                    for (int i = 0; i < 16; ++i) { bl[i] = l[i]; brec[i] = r4[i]; }
                }
            }
            total += bj;
            if (total >= best) ok = false;  // 16x16 already better
            bm[b] = (uint8_t)bmode;
            tnz[bx] = lnz[by] = blast > 0;
            for (int i = 0; i < 16; ++i) lv4[b][i] = bl[i];
            for (int y = 0; y < 4; ++y)
                for (int x = 0; x < 4; ++x) d[y * kBps + x] = brec[y * 4 + x];
        }
        if (ok && total < best) {
            best_mode = B_PRED;
            for (int b = 0; b < 16; ++b) {
                o.bmodes[b] = bm[b];
                for (int i = 0; i < 16; ++i) o.lv[b][i] = lv4[b][i];
            }
            for (int i = 0; i < 16; ++i) o.lv[24][i] = 0;
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) best_rec[y * 16 + x] = y4[(y + 1) * kBps + x + 1];
        }
    }
    o.ymode = (uint8_t)best_mode;
    if (best_mode != B_PRED)
        for (int b = 0; b < 16; ++b) o.bmodes[b] = (uint8_t)best_mode;
    for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) c.y[(y + 1) * kBps + x + 1] = best_rec[y * 16 + x];
    // --- chroma ---
    uint8_t ru[64], rv[64], bu[64], bv[64];
    int16_t lvc[25][16];
    long long bestc = -1;
    int best_uv = DC_PRED;
    for (int m = 0; m < 4; ++m) {
        const int mode = m == 0 ? DC_PRED : (m == 1 ? V_PRED : (m == 2 ? H_PRED : TM_PRED));
        const long long j = try_uv(c, q, probs, mode, lvc, ru, rv);
        if (bestc < 0 || j < bestc) {
            bestc = j;
            best_uv = mode;
            for (int i = 0; i < 64; ++i) { bu[i] = ru[i]; bv[i] = rv[i]; }
            for (int b = 16; b < 24; ++b)
                for (int i = 0; i < 16; ++i) o.lv[b][i] = lvc[b][i];
        }
    }
    o.uvmode = (uint8_t)best_uv;
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            c.u[(y + 1) * kBps + x + 1] = bu[y * 8 + x];
            c.v[(y + 1) * kBps + x + 1] = bv[y * 8 + x];
        }
    bool any = false;
    for (int b = 0; b < 25 && !any; ++b)
        for (int i = 0; i < 16; ++i)
            if (o.lv[b][i]) { any = true; break; }
    o.skip = any ? 0 : 1;
}

}  // namespace vp8
}  // namespace ik
