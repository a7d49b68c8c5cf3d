/*
 * vp8_modes.c -- ORACLE (test infrastructure only, see ik_oracle.h): a C restatement of
 * libwebp's method-4 macroblock decisions -- the second stage of the reference's WebP
 * coder (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp WebPEncode, config
 * defaults: method 4 = RD_OPT_BASIC, token buffer, one pass, sns 50, segments 4).
 *
 * libwebp is a C dependency absent from /root/reference.  Its published algorithm is
 * restated here (src/enc/quant_enc.c: SetupMatrices, ReconstructIntra16/4/UV,
 * PickBestIntra16/4/UV, CorrectDCValues; src/enc/cost_enc.c: VP8GetCostLuma16/4/UV,
 * VP8CalculateLevelCosts; src/dsp/enc.c: the predictors, transforms, SSE, TDisto,
 * QuantizeBlock; src/enc/frame_enc.c: VP8EncTokenLoop's probability refresh every
 * mb_count/8 macroblocks, RecordTokens, FinalizeTokenProbas; src/enc/token_enc.c:
 * VP8RecordCoeffTokens' statistics; src/enc/iterator_enc.c: the boundary and
 * non-zero-context bookkeeping).  Its cost tables come from libwebp's own read-only data
 * (vp8_enc_tables.h, tools/gen_vp8_tables.py).  The output -- every macroblock's luma
 * and chroma modes and the frame's final coefficient probabilities -- is pinned against
 * what libwebp writes into its bytes (tests/test_vp8_modes.py, via tests/vp8_parse.py), and
 * iko_vp8_encode adds the bitstream (filter levels, partition 0, the token partition,
 * RIFF) -- byte-identical to WebPEncodeRGB's output.
 * The segment map and segment quantisers are inputs (tests/oracle_vp8.py restates
 * that first stage).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ik_oracle.h"
#include "vp8_enc_tables.h"

#define BPS 32
#define QFIX 17
#define BIAS(b) ((b) << (QFIX - 8))
#define QUANTDIV(n, iQ, B) ((int)(((uint32_t)(n) * (iQ) + (B)) >> QFIX))
#define MAX_LEVEL 2047
#define MAX_VARIABLE_LEVEL 67
#define SHARPEN_BITS 11
#define RD_DISTO_MULT 256
#define FLATNESS_LIMIT_I16 10
#define FLATNESS_LIMIT_I4 3
#define FLATNESS_LIMIT_UV 2
#define FLATNESS_PENALTY 140
#define MULT_8B(a, b) (((a) * (b) + 128) >> 8)
#define DSHIFT 4
#define DSCALE 1
#define C1 7
#define C2 8
#define ERROR_DIFFUSION_QUALITY 98

typedef int64_t score_t;

static const uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const int kBiasMatrices[3][2] = {{96, 110}, {96, 108}, {110, 115}};

typedef struct {
    uint16_t q[16], iq[16], sharpen[16];
    uint32_t bias[16], zthresh[16];
} Matrix;

typedef struct {
    Matrix y1, y2, uv;
    int lambda_i4, lambda_i16, lambda_uv, lambda_mode, tlambda;
} SegQ;

typedef struct {
    score_t D, SD, H, R, score;
    int16_t y_dc_levels[16];
    int16_t y_ac_levels[16][16];
    int16_t uv_levels[4 + 4][16];
    int mode_i16;
    uint8_t modes_i4[16];
    int mode_uv;
    uint32_t nz;
    int8_t derr[2][3];
} ModeScore;

/* ---- probabilities and costs (cost_enc.c) ---- */
typedef struct {
    uint8_t coeffs[4][8][3][11];
    uint32_t stats[4][8][3][11];
    uint16_t level_cost[4][8][3][MAX_VARIABLE_LEVEL + 1];
    int dirty;
} Proba;

static int bit_cost(int bit, int p) { return !bit ? kEntropyCost[p] : kEntropyCost[255 - p]; }

static int variable_level_cost(int level, const uint8_t* probas) {
    int pattern = kLevelCodes[2 * (level - 1)], bits = kLevelCodes[2 * (level - 1) + 1], cost = 0, i;
    for (i = 2; pattern; ++i) {
        if (pattern & 1) cost += bit_cost(bits & 1, probas[i]);
        bits >>= 1;
        pattern >>= 1;
    }
    return cost;
}

static void calculate_level_costs(Proba* P) {
    if (!P->dirty) return;
    for (int t = 0; t < 4; ++t)
        for (int b = 0; b < 8; ++b)
            for (int c = 0; c < 3; ++c) {
                const uint8_t* p = P->coeffs[t][b][c];
                uint16_t* table = P->level_cost[t][b][c];
                const int cost0 = c > 0 ? bit_cost(1, p[0]) : 0;
                const int cost_base = bit_cost(1, p[1]) + cost0;
                table[0] = (uint16_t)(bit_cost(0, p[1]) + cost0);
                for (int v = 1; v <= MAX_VARIABLE_LEVEL; ++v) table[v] = (uint16_t)(cost_base + variable_level_cost(v, p));
            }
    P->dirty = 0;
}

static int level_cost(const uint16_t* table, int level) {
    return kLevelFixedCosts[level] + table[level > MAX_VARIABLE_LEVEL ? MAX_VARIABLE_LEVEL : level];
}

typedef struct {
    int first, last, type;
    const int16_t* coeffs;
} Residual;

static void set_residual(Residual* r, const int16_t* coeffs) {
    r->last = -1;
    for (int n = 15; n >= 0; --n)
        if (coeffs[n]) { r->last = n; break; }
    r->coeffs = coeffs;
}

static int residual_cost(const Proba* P, int ctx0, const Residual* r) {
    int n = r->first;
    const int p0 = P->coeffs[r->type][n][ctx0][0];
    const uint16_t* t = P->level_cost[r->type][kEncBands[n]][ctx0];
    int cost = ctx0 == 0 ? bit_cost(1, p0) : 0;
    if (r->last < 0) return bit_cost(0, p0);
    for (; n < r->last; ++n) {
        const int v = abs(r->coeffs[n]);
        const int ctx = v >= 2 ? 2 : v;
        cost += level_cost(t, v);
        t = P->level_cost[r->type][kEncBands[n + 1]][ctx];
    }
    {
        const int v = abs(r->coeffs[n]);
        cost += level_cost(t, v);
        if (n < 15) {
            const int b = kEncBands[n + 1];
            const int ctx = v == 1 ? 1 : 2;
            cost += bit_cost(0, P->coeffs[r->type][b][ctx][0]);
        }
    }
    return cost;
}

/* ---- token statistics (token_enc.c VP8RecordCoeffTokens, the stats side only) ---- */
static int record_stats(int bit, uint32_t* s) {
    uint32_t p = *s;
    if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
    p += 0x00010000u + (uint32_t)bit;
    *s = p;
    return bit;
}

/* the token sink (VP8TBuffer): bit 15 = the bit, bit 14 = a constant probability
 * (bits 0-7), else bits 0-13 = the index of the coefficient probability it is coded
 * with (TOKEN_ID + node); NULL while only the decisions are wanted */
static uint32_t* g_tok;
static size_t g_ntok, g_tcap;

static void put_token(uint32_t t) {
    if (!g_tok && !g_tcap) return;
    if (g_ntok == g_tcap) {
        g_tcap = g_tcap * 2 + 4096;
        g_tok = realloc(g_tok, g_tcap * sizeof(*g_tok));
    }
    g_tok[g_ntok++] = t;
}

static int add_token(int bit, uint32_t id, uint32_t* s) {
    put_token(((uint32_t)bit << 15) | id);
    return record_stats(bit, s);
}

static void add_const(int bit, int prob) { put_token(((uint32_t)bit << 15) | (1u << 14) | (uint32_t)prob); }

#define TOKEN_ID(t, b, ctx) (11u * ((ctx) + 3u * ((b) + 8u * (t))))
static const uint8_t kCat3[] = {173, 148, 140, 0};
static const uint8_t kCat4[] = {176, 155, 140, 135, 0};
static const uint8_t kCat5[] = {180, 157, 141, 134, 130, 0};
static const uint8_t kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};

static int record_coeff_tokens(Proba* P, int ctx, const Residual* r) {
    const int16_t* coeffs = r->coeffs;
    const int t = r->type, last = r->last;
    int n = r->first;
    uint32_t base_id = TOKEN_ID(t, n, ctx);
    uint32_t* s = P->stats[t][n][ctx];
    if (!add_token(last >= 0, base_id + 0, s + 0)) return 0;
    while (n < 16) {
        const int c = coeffs[n++];
        const int sign = c < 0;
        const uint32_t v = (uint32_t)(sign ? -c : c);
        if (!add_token(v != 0, base_id + 1, s + 1)) {
            base_id = TOKEN_ID(t, kEncBands[n], 0);
            s = P->stats[t][kEncBands[n]][0];
            continue;
        }
        if (!add_token(v > 1, base_id + 2, s + 2)) {
            base_id = TOKEN_ID(t, kEncBands[n], 1);
            s = P->stats[t][kEncBands[n]][1];
        } else {
            if (!add_token(v > 4, base_id + 3, s + 3)) {
                if (add_token(v != 2, base_id + 4, s + 4)) add_token(v == 4, base_id + 5, s + 5);
            } else if (!add_token(v > 10, base_id + 6, s + 6)) {
                if (!add_token(v > 6, base_id + 7, s + 7)) {
                    add_const(v == 6, 159);
                } else {
                    add_const(v >= 9, 165);
                    add_const(!(v & 1), 145);
                }
            } else {
                int mask;
                const uint8_t* tab;
                uint32_t residue = v - 3;
                if (residue < (8 << 1)) {
                    add_token(0, base_id + 8, s + 8);
                    add_token(0, base_id + 9, s + 9);
                    residue -= (8 << 0);
                    mask = 1 << 2;
                    tab = kCat3;
                } else if (residue < (8 << 2)) {
                    add_token(0, base_id + 8, s + 8);
                    add_token(1, base_id + 9, s + 9);
                    residue -= (8 << 1);
                    mask = 1 << 3;
                    tab = kCat4;
                } else if (residue < (8 << 3)) {  /* (libwebp records cat 5/6's node-10 bit at stats slot 9) */
                    add_token(1, base_id + 8, s + 8);
                    add_token(0, base_id + 10, s + 9);
                    residue -= (8 << 2);
                    mask = 1 << 4;
                    tab = kCat5;
                } else {
                    add_token(1, base_id + 8, s + 8);
                    add_token(1, base_id + 10, s + 9);
                    residue -= (8 << 3);
                    mask = 1 << 10;
                    tab = kCat6;
                }
                while (mask) {
                    add_const(!!(residue & (uint32_t)mask), *tab++);
                    mask >>= 1;
                }
            }
            base_id = TOKEN_ID(t, kEncBands[n], 2);
            s = P->stats[t][kEncBands[n]][2];
        }
        add_const(sign, 128);
        if (n == 16 || !add_token(n <= last, base_id + 0, s + 0)) return 1;
    }
    return 1;
}

static int calc_token_proba(int nb, int total) { return nb ? (255 - nb * 255 / total) : 255; }
static int branch_cost(int nb, int total, int p) { return nb * bit_cost(1, p) + (total - nb) * bit_cost(0, p); }

static void finalize_token_probas(Proba* P) {
    int has_changed = 0;
    for (int t = 0; t < 4; ++t)
        for (int b = 0; b < 8; ++b)
            for (int c = 0; c < 3; ++c)
                for (int p = 0; p < 11; ++p) {
                    const uint32_t stats = P->stats[t][b][c][p];
                    const int nb = (int)(stats & 0xffff), total = (int)((stats >> 16) & 0xffff);
                    const int i = ((t * 8 + b) * 3 + c) * 11 + p;
                    const int update_proba = kCoeffsUpdateProba[i], old_p = kCoeffsProba0[i];
                    const int new_p = calc_token_proba(nb, total);
                    const int old_cost = branch_cost(nb, total, old_p) + bit_cost(0, update_proba);
                    const int new_cost = branch_cost(nb, total, new_p) + bit_cost(1, update_proba) + 8 * 256;
                    const int use_new_p = old_cost > new_cost;
                    if (use_new_p) {
                        P->coeffs[t][b][c][p] = (uint8_t)new_p;
                        has_changed |= new_p != old_p;
                    } else {
                        P->coeffs[t][b][c][p] = (uint8_t)old_p;
                    }
                }
    P->dirty = has_changed;
}

/* ---- transforms, quantisation (dsp/enc.c) ---- */
static void ftransform(const uint8_t* src, const uint8_t* ref, int16_t* out) {
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

static void ftransform_wht(const int16_t* in, int16_t* out) {  /* in: the 16 blocks' [16] arrays */
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

static void itransform_wht(const int16_t* in, int16_t* out) {  /* out: block n's DC at out[16 n] */
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

static uint8_t clip8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
#define MUL1(a) ((((a) * 20091) >> 16) + (a))
#define MUL2(a) (((a) * 35468) >> 16)

static void itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst) {
    int C[16], *tmp = C;
    for (int i = 0; i < 4; ++i) {
        const int a = in[0] + in[8], b = in[0] - in[8];
        const int c = MUL2(in[4]) - MUL1(in[12]), d = MUL1(in[4]) + MUL2(in[12]);
        tmp[0] = a + d;
        tmp[1] = b + c;
        tmp[2] = b - c;
        tmp[3] = a - d;
        tmp += 4;
        in++;
    }
    tmp = C;
    for (int i = 0; i < 4; ++i) {
        const int dc = tmp[0] + 4;
        const int a = dc + tmp[8], b = dc - tmp[8];
        const int c = MUL2(tmp[4]) - MUL1(tmp[12]), d = MUL1(tmp[4]) + MUL2(tmp[12]);
        dst[0 + i * BPS] = clip8(ref[0 + i * BPS] + ((a + d) >> 3));
        dst[1 + i * BPS] = clip8(ref[1 + i * BPS] + ((b + c) >> 3));
        dst[2 + i * BPS] = clip8(ref[2 + i * BPS] + ((b - c) >> 3));
        dst[3 + i * BPS] = clip8(ref[3 + i * BPS] + ((a - d) >> 3));
        tmp++;
    }
}

static int quantize_block(int16_t in[16], int16_t out[16], const Matrix* m) {
    int last = -1;
    for (int n = 0; n < 16; ++n) {
        const int j = kZigzag[n];
        const int sign = in[j] < 0;
        const uint32_t coeff = (uint32_t)((sign ? -in[j] : in[j]) + m->sharpen[j]);
        if (coeff > m->zthresh[j]) {
            const uint32_t Q = m->q[j], iQ = m->iq[j], B = m->bias[j];
            int level = QUANTDIV(coeff, iQ, B);
            if (level > MAX_LEVEL) level = MAX_LEVEL;
            if (sign) level = -level;
            in[j] = (int16_t)(level * (int)Q);
            out[n] = (int16_t)level;
            if (level) last = n;
        } else {
            out[n] = 0;
            in[j] = 0;
        }
    }
    return last >= 0;
}

static int expand_matrix(Matrix* m, int type) {
    int sum = 0;
    for (int i = 0; i < 2; ++i) {
        const int bias = kBiasMatrices[type][i > 0];
        m->iq[i] = (uint16_t)((1 << QFIX) / m->q[i]);
        m->bias[i] = (uint32_t)BIAS(bias);
        m->zthresh[i] = ((1u << QFIX) - 1 - m->bias[i]) / m->iq[i];
    }
    for (int i = 2; i < 16; ++i) {
        m->q[i] = m->q[1];
        m->iq[i] = m->iq[1];
        m->bias[i] = m->bias[1];
        m->zthresh[i] = m->zthresh[1];
    }
    for (int i = 0; i < 16; ++i) {
        m->sharpen[i] = type == 0 ? (uint16_t)((kFreqSharpening[i] * m->q[i]) >> SHARPEN_BITS) : 0;
        sum += m->q[i];
    }
    return (sum + 8) >> 4;
}

static int clipi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

static void setup_matrices(SegQ* s, int q, int dq_uv_dc, int dq_uv_ac, int sns) {
    memset(s, 0, sizeof(*s));
    s->y1.q[0] = kDcTable[clipi(q, 0, 127)];
    s->y1.q[1] = kAcTable[clipi(q, 0, 127)];
    s->y2.q[0] = (uint16_t)(kDcTable[clipi(q, 0, 127)] * 2);
    s->y2.q[1] = (uint16_t)((kAcTable[clipi(q, 0, 127)] * 101581) >> 16);
    if (s->y2.q[1] < 8) s->y2.q[1] = 8;
    s->uv.q[0] = kDcTable[clipi(q + dq_uv_dc, 0, 117)];
    s->uv.q[1] = kAcTable[clipi(q + dq_uv_ac, 0, 127)];
    const int q_i4 = expand_matrix(&s->y1, 0), q_i16 = expand_matrix(&s->y2, 1), q_uv = expand_matrix(&s->uv, 2);
    s->lambda_i4 = (3 * q_i4 * q_i4) >> 7;
    s->lambda_i16 = 3 * q_i16 * q_i16;
    s->lambda_uv = (3 * q_uv * q_uv) >> 6;
    s->lambda_mode = (1 * q_i4 * q_i4) >> 7;
    s->tlambda = (sns * q_i4) >> 5;  /* method >= 4: tlambda_scale = sns_strength */
    if (s->lambda_i4 < 1) s->lambda_i4 = 1;
    if (s->lambda_i16 < 1) s->lambda_i16 = 1;
    if (s->lambda_uv < 1) s->lambda_uv = 1;
    if (s->lambda_mode < 1) s->lambda_mode = 1;
    /* (tlambda may be 0: then no spectral distortion) */
}

/* ---- distortion ---- */
static int sse_wh(const uint8_t* a, const uint8_t* b, int w, int h) {
    int s = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const int d = a[x + y * BPS] - b[x + y * BPS];
            s += d * d;
        }
    return s;
}

static int ttransform(const uint8_t* in, const uint16_t* w) {
    int sum = 0, tmp[16];
    for (int i = 0; i < 4; ++i, in += BPS) {
        const int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[1] - in[3], a3 = in[0] - in[2];
        tmp[0 + i * 4] = a0 + a1;
        tmp[1 + i * 4] = a3 + a2;
        tmp[2 + i * 4] = a3 - a2;
        tmp[3 + i * 4] = a0 - a1;
    }
    for (int i = 0; i < 4; ++i, ++w) {
        const int a0 = tmp[0 + i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
        const int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[0 + i] - tmp[8 + i];
        const int b0 = a0 + a1, b1 = a3 + a2, b2 = a3 - a2, b3 = a0 - a1;
        sum += w[0] * abs(b0) + w[4] * abs(b1) + w[8] * abs(b2) + w[12] * abs(b3);
    }
    return sum;
}

static int disto4x4(const uint8_t* a, const uint8_t* b) { return abs(ttransform(b, kWeightY) - ttransform(a, kWeightY)) >> 5; }

static int disto16x16(const uint8_t* a, const uint8_t* b) {
    int D = 0;
    for (int y = 0; y < 16 * BPS; y += 4 * BPS)
        for (int x = 0; x < 16; x += 4) D += disto4x4(a + x + y, b + x + y);
    return D;
}

static int is_flat(const int16_t* levels, int num_blocks, int thresh) {
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

static int is_flat_source16(const uint8_t* src) {
    for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x)
            if (src[x + y * BPS] != src[0]) return 0;
    return 1;
}

static void set_rd_score(int lambda, ModeScore* rd) { rd->score = (rd->R + rd->H) * lambda + RD_DISTO_MULT * (rd->D + rd->SD); }

static void init_score(ModeScore* rd) {
    rd->D = rd->SD = 0;
    rd->R = rd->H = 0;
    rd->nz = 0;
    rd->score = (score_t)1 << 62;  /* MAX_COST */
}

static void copy_score(ModeScore* dst, const ModeScore* src) {
    dst->D = src->D;
    dst->SD = src->SD;
    dst->R = src->R;
    dst->H = src->H;
    dst->nz = src->nz;
    dst->score = src->score;
}

static void add_score(ModeScore* dst, const ModeScore* src) {
    dst->D += src->D;
    dst->SD += src->SD;
    dst->R += src->R;
    dst->H += src->H;
    dst->nz |= src->nz;
    dst->score += src->score;
}

/* ---- predictors (dsp/enc.c): into a BPS-pitched size x size block ---- */
static void fill(uint8_t* dst, int v, int size) {
    for (int j = 0; j < size; ++j) memset(dst + j * BPS, v, (size_t)size);
}
static void vertical_pred(uint8_t* dst, const uint8_t* top, int size) {
    if (top) for (int j = 0; j < size; ++j) memcpy(dst + j * BPS, top, (size_t)size);
    else fill(dst, 127, size);
}
static void horizontal_pred(uint8_t* dst, const uint8_t* left, int size) {
    if (left) for (int j = 0; j < size; ++j) memset(dst + j * BPS, left[j], (size_t)size);
    else fill(dst, 129, size);
}
static void true_motion(uint8_t* dst, const uint8_t* left, const uint8_t* top, int size) {
    if (left) {
        if (top) {
            for (int y = 0; y < size; ++y)
                for (int x = 0; x < size; ++x) dst[x + y * BPS] = clip8(left[y] + top[x] - left[-1]);
        } else {
            horizontal_pred(dst, left, size);
        }
    } else {
        if (top) vertical_pred(dst, top, size);
        else fill(dst, 129, size);
    }
}
static void dc_mode(uint8_t* dst, const uint8_t* left, const uint8_t* top, int size, int round, int shift) {
    int DC = 0;
    if (top) {
        for (int j = 0; j < size; ++j) DC += top[j];
        if (left) for (int j = 0; j < size; ++j) DC += left[j];
        else DC += DC;
        DC = (DC + round) >> shift;
    } else if (left) {
        for (int j = 0; j < size; ++j) DC += left[j];
        DC += DC;
        DC = (DC + round) >> shift;
    } else {
        DC = 0x80;
    }
    fill(dst, DC, size);
}

/* mode m (DC 0, TM 1, V 2, H 3) of an NxN block */
static void pred_nxn(uint8_t* dst, int m, const uint8_t* left, const uint8_t* top, int size) {
    if (m == 0) dc_mode(dst, left, top, size, size, size == 16 ? 5 : 4);
    else if (m == 1) true_motion(dst, left, top, size);
    else if (m == 2) vertical_pred(dst, top, size);
    else horizontal_pred(dst, left, size);
}

#define AVG3(a, b, c) ((uint8_t)(((a) + 2 * (b) + (c) + 2) >> 2))
#define AVG2(a, b) (((a) + (b) + 1) >> 1)
#define DST(x, y) dst[(x) + (y) * BPS]

/* the 10 intra-4 predictors from top[] (top[-1] corner, top[-2..-5] left column I J K L,
 * top[0..7] above and above-right) */
static void pred4(uint8_t* dst, int mode, const uint8_t* top) {
    const int X = top[-1], I = top[-2], J = top[-3], K = top[-4], L = top[-5];
    const int A = top[0], B = top[1], C = top[2], D = top[3], E = top[4], F = top[5], G = top[6], H = top[7];
    switch (mode) {
    case 0: { /* DC */
        uint32_t dc = 4;
        for (int i = 0; i < 4; ++i) dc += top[i] + top[-5 + i];
        fill(dst, (int)(dc >> 3), 4);
        break;
    }
    case 1: /* TM */
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) DST(x, y) = clip8(top[-2 - y] + top[x] - X);
        break;
    case 2: { /* VE */
        const uint8_t v[4] = {AVG3(X, A, B), AVG3(A, B, C), AVG3(B, C, D), AVG3(C, D, E)};
        for (int y = 0; y < 4; ++y) memcpy(dst + y * BPS, v, 4);
        break;
    }
    case 3: /* HE */
        memset(dst + 0 * BPS, AVG3(X, I, J), 4);
        memset(dst + 1 * BPS, AVG3(I, J, K), 4);
        memset(dst + 2 * BPS, AVG3(J, K, L), 4);
        memset(dst + 3 * BPS, AVG3(K, L, L), 4);
        break;
    case 4: /* RD */
        DST(0, 3) = AVG3(J, K, L);
        DST(0, 2) = DST(1, 3) = AVG3(I, J, K);
        DST(0, 1) = DST(1, 2) = DST(2, 3) = AVG3(X, I, J);
        DST(0, 0) = DST(1, 1) = DST(2, 2) = DST(3, 3) = AVG3(A, X, I);
        DST(1, 0) = DST(2, 1) = DST(3, 2) = AVG3(B, A, X);
        DST(2, 0) = DST(3, 1) = AVG3(C, B, A);
        DST(3, 0) = AVG3(D, C, B);
        break;
    case 5: /* VR */
        DST(0, 0) = DST(1, 2) = (uint8_t)AVG2(X, A);
        DST(1, 0) = DST(2, 2) = (uint8_t)AVG2(A, B);
        DST(2, 0) = DST(3, 2) = (uint8_t)AVG2(B, C);
        DST(3, 0) = (uint8_t)AVG2(C, D);
        DST(0, 3) = AVG3(K, J, I);
        DST(0, 2) = AVG3(J, I, X);
        DST(0, 1) = DST(1, 3) = AVG3(I, X, A);
        DST(1, 1) = DST(2, 3) = AVG3(X, A, B);
        DST(2, 1) = DST(3, 3) = AVG3(A, B, C);
        DST(3, 1) = AVG3(B, C, D);
        break;
    case 6: /* LD */
        DST(0, 0) = AVG3(A, B, C);
        DST(1, 0) = DST(0, 1) = AVG3(B, C, D);
        DST(2, 0) = DST(1, 1) = DST(0, 2) = AVG3(C, D, E);
        DST(3, 0) = DST(2, 1) = DST(1, 2) = DST(0, 3) = AVG3(D, E, F);
        DST(3, 1) = DST(2, 2) = DST(1, 3) = AVG3(E, F, G);
        DST(3, 2) = DST(2, 3) = AVG3(F, G, H);
        DST(3, 3) = AVG3(G, H, H);
        break;
    case 7: /* VL */
        DST(0, 0) = (uint8_t)AVG2(A, B);
        DST(1, 0) = DST(0, 2) = (uint8_t)AVG2(B, C);
        DST(2, 0) = DST(1, 2) = (uint8_t)AVG2(C, D);
        DST(3, 0) = DST(2, 2) = (uint8_t)AVG2(D, E);
        DST(0, 1) = AVG3(A, B, C);
        DST(1, 1) = DST(0, 3) = AVG3(B, C, D);
        DST(2, 1) = DST(1, 3) = AVG3(C, D, E);
        DST(3, 1) = DST(2, 3) = AVG3(D, E, F);
        DST(3, 2) = AVG3(E, F, G);
        DST(3, 3) = AVG3(F, G, H);
        break;
    case 8: /* HD */
        DST(0, 0) = DST(2, 1) = (uint8_t)AVG2(I, X);
        DST(0, 1) = DST(2, 2) = (uint8_t)AVG2(J, I);
        DST(0, 2) = DST(2, 3) = (uint8_t)AVG2(K, J);
        DST(0, 3) = (uint8_t)AVG2(L, K);
        DST(3, 0) = AVG3(A, B, C);
        DST(2, 0) = AVG3(X, A, B);
        DST(1, 0) = DST(3, 1) = AVG3(I, X, A);
        DST(1, 1) = DST(3, 2) = AVG3(J, I, X);
        DST(1, 2) = DST(3, 3) = AVG3(K, J, I);
        DST(1, 3) = AVG3(L, K, J);
        break;
    default: /* HU */
        DST(0, 0) = (uint8_t)AVG2(I, J);
        DST(2, 0) = DST(0, 1) = (uint8_t)AVG2(J, K);
        DST(2, 1) = DST(0, 2) = (uint8_t)AVG2(K, L);
        DST(1, 0) = AVG3(I, J, K);
        DST(3, 0) = DST(1, 1) = AVG3(J, K, L);
        DST(3, 1) = DST(1, 2) = AVG3(K, L, L);
        DST(3, 2) = DST(2, 2) = DST(0, 3) = DST(1, 3) = DST(2, 3) = DST(3, 3) = (uint8_t)L;
        break;
    }
    (void)E; (void)F; (void)G; (void)H;
}

/* ---- the frame ---- */
typedef struct {
    int mb_w, mb_h;
    const uint8_t *Y, *U, *V;  /* padded source planes: mb_w*16 (8) wide */
    uint8_t *y_top, *uv_top;   /* reconstructed bottom rows of the MB row above (127 for row 0) */
    uint8_t y_left[17], u_left[9], v_left[9]; /* [0] = corner, [1..] = column */
    uint32_t* nz;              /* per MB column (+1 in front): packed non-zero bits */
    int top_nz[9], left_nz[9];
    int left_dc_nz;            /* left_nz[8] persists along the row */
    int8_t (*top_derr)[2][2];
    int8_t left_derr[2][2];
    uint8_t* preds;            /* (mb_w*4 + 1) x (mb_h*4 + 1), border = B_DC_PRED */
    int preds_w;
    Proba P;
    int use_derr;
} Frame;

#define PREDS(F, mx, my) ((F)->preds + ((my) * 4 + 1) * (F)->preds_w + (mx) * 4 + 1)

static void nz_to_bytes(Frame* F, int mx) {
    const uint32_t tnz = F->nz[1 + mx], lnz = F->nz[mx];
    int* t = F->top_nz;
    int* l = F->left_nz;
#define BIT(v, n) (((v) >> (n)) & 1)
    t[0] = BIT(tnz, 12); t[1] = BIT(tnz, 13); t[2] = BIT(tnz, 14); t[3] = BIT(tnz, 15);
    t[4] = BIT(tnz, 18); t[5] = BIT(tnz, 19); t[6] = BIT(tnz, 22); t[7] = BIT(tnz, 23);
    t[8] = BIT(tnz, 24);
    l[0] = BIT(lnz, 3); l[1] = BIT(lnz, 7); l[2] = BIT(lnz, 11); l[3] = BIT(lnz, 15);
    l[4] = BIT(lnz, 17); l[5] = BIT(lnz, 19); l[6] = BIT(lnz, 21); l[7] = BIT(lnz, 23);
    l[8] = F->left_dc_nz;
#undef BIT
}

static void bytes_to_nz(Frame* F, int mx) {
    const int* t = F->top_nz;
    const int* l = F->left_nz;
    uint32_t nz = 0;
    nz |= (uint32_t)((t[0] << 12) | (t[1] << 13) | (t[2] << 14) | (t[3] << 15));
    nz |= (uint32_t)((t[4] << 18) | (t[5] << 19) | (t[6] << 22) | (t[7] << 23));
    nz |= (uint32_t)(t[8] << 24);
    nz |= (uint32_t)((l[0] << 3) | (l[1] << 7) | (l[2] << 11));
    nz |= (uint32_t)((l[4] << 17) | (l[6] << 21));
    F->nz[1 + mx] = nz;
    F->left_dc_nz = l[8];
}

typedef struct {
    int mx, my;
    uint8_t yuv_in[BPS * 16];   /* Y at 0, U at 16, V at 24 */
    uint8_t pred16[4][BPS * 16];/* i16 predictions */
    uint8_t predc[4][BPS * 8];  /* chroma predictions, U at 0, V at 8 */
    uint8_t yuv_out[BPS * 16];  /* the chosen reconstruction */
    const SegQ* dqm;
    int seg;
} MB;

static int g_y2q1[4];
static int g_max_edge[4];  /* per segment: StoreMaxDelta's largest DC step of DC-only i16 MBs */

static int reconstruct_i16(Frame* F, MB* m, ModeScore* rd, uint8_t* out, int mode) {
    const uint8_t* ref = m->pred16[mode];
    const uint8_t* src = m->yuv_in;
    int16_t tmp[16][16], dc_tmp[16];
    uint32_t nz = 0;
    for (int n = 0; n < 16; ++n) {
        const int off = (n & 3) * 4 + (n >> 2) * 4 * BPS;
        ftransform(src + off, ref + off, tmp[n]);
    }
    ftransform_wht(tmp[0], dc_tmp);
    nz |= (uint32_t)quantize_block(dc_tmp, rd->y_dc_levels, &m->dqm->y2) << 24;
    for (int n = 0; n < 16; n += 2) {
        tmp[n][0] = tmp[n + 1][0] = 0;
        const int a = quantize_block(tmp[n], rd->y_ac_levels[n], &m->dqm->y1);
        const int b = quantize_block(tmp[n + 1], rd->y_ac_levels[n + 1], &m->dqm->y1);
        nz |= (uint32_t)(a | (b << 1)) << n;
    }
    itransform_wht(dc_tmp, tmp[0]);
    for (int n = 0; n < 16; ++n) {
        const int off = (n & 3) * 4 + (n >> 2) * 4 * BPS;
        itransform(ref + off, tmp[n], out + off);
    }
    (void)F;
    return (int)nz;
}

static int g_mx;  /* current column for the nz bookkeeping (single-threaded oracle) */

static int get_cost_luma16(Frame* F, const ModeScore* rd) {
    Residual r;
    int R = 0;
    nz_to_bytes(F, g_mx);
    r.first = 0; r.type = 1;
    set_residual(&r, rd->y_dc_levels);
    R += residual_cost(&F->P, F->top_nz[8] + F->left_nz[8], &r);
    r.first = 1; r.type = 0;
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const int ctx = F->top_nz[x] + F->left_nz[y];
            set_residual(&r, rd->y_ac_levels[x + y * 4]);
            R += residual_cost(&F->P, ctx, &r);
            F->top_nz[x] = F->left_nz[y] = r.last >= 0;
        }
    return R;
}

static int get_cost_uv(Frame* F, const ModeScore* rd) {
    Residual r;
    int R = 0;
    nz_to_bytes(F, g_mx);
    r.first = 0; r.type = 2;
    for (int ch = 0; ch <= 2; ch += 2)
        for (int y = 0; y < 2; ++y)
            for (int x = 0; x < 2; ++x) {
                const int ctx = F->top_nz[4 + ch + x] + F->left_nz[4 + ch + y];
                set_residual(&r, rd->uv_levels[ch * 2 + x + y * 2]);
                R += residual_cost(&F->P, ctx, &r);
                F->top_nz[4 + ch + x] = F->left_nz[4 + ch + y] = r.last >= 0;
            }
    return R;
}

static void pick_best_intra16(Frame* F, MB* m, ModeScore* rd) {
    const SegQ* dqm = m->dqm;
    const int lambda = dqm->lambda_i16, tlambda = dqm->tlambda;
    const uint8_t* src = m->yuv_in;
    uint8_t tmp_out[BPS * 16];
    ModeScore cur, best;
    int flat = is_flat_source16(src);
    init_score(&best);
    rd->mode_i16 = -1;
    for (int mode = 0; mode < 4; ++mode) {
        init_score(&cur);
        cur.mode_i16 = mode;
        cur.nz = (uint32_t)reconstruct_i16(F, m, &cur, tmp_out, mode);
        cur.D = sse_wh(src, tmp_out, 16, 16);
        cur.SD = tlambda ? MULT_8B(tlambda, disto16x16(src, tmp_out)) : 0;
        cur.H = kFixedCostsI16[mode];
        cur.R = get_cost_luma16(F, &cur);
        if (flat) {
            flat = is_flat(cur.y_ac_levels[0], 16, FLATNESS_LIMIT_I16);
            if (flat) {
                cur.D *= 2;
                cur.SD *= 2;
            }
        }
        set_rd_score(lambda, &cur);
        if (mode == 0 || cur.score < best.score) {
            best = cur;
            for (int y = 0; y < 16; ++y) memcpy(m->yuv_out + y * BPS, tmp_out + y * BPS, 16);
        }
    }
    *rd = best;
    set_rd_score(dqm->lambda_mode, rd);
    /* a blocky MB (only DCs non-zero) with fairly high distortion: record its largest
     * DC step for the filter strength (StoreMaxDelta) */
    if ((rd->nz & 0x100ffffu) == 0x1000000u && rd->D > 20 * dqm->y1.q[0]) {
        const int v0 = abs(rd->y_dc_levels[1]), v1 = abs(rd->y_dc_levels[2]), v2 = abs(rd->y_dc_levels[4]);
        int max_v = v1 > v0 ? v1 : v0;
        max_v = v2 > max_v ? v2 : max_v;
        if (max_v > g_max_edge[m->seg]) g_max_edge[m->seg] = max_v;
    }
}


static const int kTopLeftI4[16] = {17, 21, 25, 29, 13, 17, 21, 25, 9, 13, 17, 21, 5, 9, 13, 17};

/* returns 1 (and fills rd, m->yuv_out's luma) when intra-4 beats rd's intra-16 score */
static int pick_best_intra4(Frame* F, MB* m, ModeScore* rd, int max_i4_header_bits) {
    const SegQ* dqm = m->dqm;
    const int lambda = dqm->lambda_i4, tlambda = dqm->tlambda;
    uint8_t best_blocks[BPS * 16];
    uint8_t boundary[37];
    int total_header_bits = 0;
    ModeScore rd_best;
    if (max_i4_header_bits == 0) return 0;
    init_score(&rd_best);
    rd_best.H = 211;
    set_rd_score(dqm->lambda_mode, &rd_best);
    /* VP8IteratorStartI4 */
    for (int i = 0; i < 17; ++i) boundary[i] = F->y_left[16 - i];  /* y_left_[15 - i]: [0] = y_left_[15], [16] = corner */
    for (int i = 0; i < 16; ++i) boundary[17 + i] = F->y_top[m->mx * 16 + i];
    if (m->mx < F->mb_w - 1) {
        for (int i = 16; i < 20; ++i) boundary[17 + i] = F->y_top[m->mx * 16 + i];
    } else {
        for (int i = 16; i < 20; ++i) boundary[17 + i] = boundary[17 + 15];
    }
    nz_to_bytes(F, g_mx);
    uint8_t* preds = PREDS(F, m->mx, m->my);
    const int pw = F->preds_w;
    for (int i4 = 0; i4 < 16; ++i4) {
        uint8_t* top = boundary + kTopLeftI4[i4];
        const int bx = i4 & 3, by = i4 >> 2;
        const int off = bx * 4 + by * 4 * BPS;
        const uint8_t* src = m->yuv_in + off;
        const int left = bx == 0 ? preds[by * pw - 1] : rd->modes_i4[i4 - 1];
        const int topm = by == 0 ? preds[-pw + bx] : rd->modes_i4[i4 - 4];
        const uint16_t* mode_costs = kFixedCostsI4 + (topm * 10 + left) * 10;
        ModeScore rd_i4;
        int best_mode = -1;
        int16_t best_levels[16];
        uint8_t best_blk[BPS * 4];
        init_score(&rd_i4);
        for (int mode = 0; mode < 10; ++mode) {
            uint8_t pred[BPS * 4], out[BPS * 4];
            int16_t levels[16];
            ModeScore t;
            pred4(pred, mode, top);
            /* (src, pred and out all BPS-pitched) */
            init_score(&t);
            {
                int16_t tmp[16];
                ftransform(src, pred, tmp);
                t.nz = (uint32_t)quantize_block(tmp, levels, &dqm->y1) << i4;
                itransform(pred, tmp, out);
            }
            t.D = sse_wh(src, out, 4, 4);
            t.SD = tlambda ? MULT_8B(tlambda, disto4x4(src, out)) : 0;
            t.H = mode_costs[mode];
            t.R = (mode > 0 && is_flat(levels, 1, FLATNESS_LIMIT_I4)) ? FLATNESS_PENALTY : 0;
            set_rd_score(lambda, &t);
            if (best_mode >= 0 && t.score >= rd_i4.score) continue;
            {
                Residual r;
                r.first = 0; r.type = 3;
                set_residual(&r, levels);
                t.R += residual_cost(&F->P, F->top_nz[bx] + F->left_nz[by], &r);
            }
            set_rd_score(lambda, &t);
            if (best_mode < 0 || t.score < rd_i4.score) {
                copy_score(&rd_i4, &t);
                best_mode = mode;
                memcpy(best_levels, levels, sizeof(levels));
                for (int y = 0; y < 4; ++y) memcpy(best_blk + y * BPS, out + y * BPS, 4);
            }
        }
        set_rd_score(dqm->lambda_mode, &rd_i4);
        add_score(&rd_best, &rd_i4);
        if (rd_best.score >= rd->score) return 0;
        total_header_bits += (int)rd_i4.H;
        if (total_header_bits > max_i4_header_bits) return 0;
        for (int y = 0; y < 4; ++y) memcpy(best_blocks + off + y * BPS, best_blk + y * BPS, 4);
        memcpy(rd_best.y_ac_levels[i4], best_levels, sizeof(best_levels));
        rd->modes_i4[i4] = (uint8_t)best_mode;
        F->top_nz[bx] = F->left_nz[by] = rd_i4.nz ? 1 : 0;
        /* VP8IteratorRotateI4 */
        {
            const uint8_t* blk = best_blocks + off;
            for (int i = 0; i <= 3; ++i) top[-4 + i] = blk[i + 3 * BPS];
            if ((i4 & 3) != 3) {
                for (int i = 0; i <= 2; ++i) top[i] = blk[3 + (2 - i) * BPS];
            } else {
                for (int i = 0; i <= 3; ++i) top[i] = top[i + 4];
            }
        }
    }
    {
        uint8_t modes[16];
        memcpy(modes, rd->modes_i4, 16);
        copy_score(rd, &rd_best);
        memcpy(rd->modes_i4, modes, 16);
        memcpy(rd->y_ac_levels, rd_best.y_ac_levels, sizeof(rd->y_ac_levels));
    }
    for (int y = 0; y < 16; ++y) memcpy(m->yuv_out + y * BPS, best_blocks + y * BPS, 16);
    return 1;
}

static int quantize_single(int16_t* v, const Matrix* mtx) {
    int V = *v;
    const int sign = V < 0;
    if (sign) V = -V;
    if (V > (int)mtx->zthresh[0]) {
        const int qV = QUANTDIV(V, mtx->iq[0], mtx->bias[0]) * mtx->q[0];
        const int err = V - qV;
        *v = (int16_t)(sign ? -qV : qV);
        return (sign ? -err : err) >> DSCALE;
    }
    *v = 0;
    return (sign ? -V : V) >> DSCALE;
}

static void correct_dc_values(Frame* F, MB* m, const Matrix* mtx, int16_t tmp[][16], ModeScore* rd) {
    for (int ch = 0; ch <= 1; ++ch) {
        const int8_t* top = F->top_derr[m->mx][ch];
        const int8_t* left = F->left_derr[ch];
        int16_t(*c)[16] = &tmp[ch * 4];
        int err0, err1, err2, err3;
        c[0][0] = (int16_t)(c[0][0] + ((C1 * top[0] + C2 * left[0]) >> (DSHIFT - DSCALE)));
        err0 = quantize_single(&c[0][0], mtx);
        c[1][0] = (int16_t)(c[1][0] + ((C1 * top[1] + C2 * err0) >> (DSHIFT - DSCALE)));
        err1 = quantize_single(&c[1][0], mtx);
        c[2][0] = (int16_t)(c[2][0] + ((C1 * err0 + C2 * left[1]) >> (DSHIFT - DSCALE)));
        err2 = quantize_single(&c[2][0], mtx);
        c[3][0] = (int16_t)(c[3][0] + ((C1 * err1 + C2 * err2) >> (DSHIFT - DSCALE)));
        err3 = quantize_single(&c[3][0], mtx);
        rd->derr[ch][0] = (int8_t)err1;
        rd->derr[ch][1] = (int8_t)err2;
        rd->derr[ch][2] = (int8_t)err3;
    }
}

static int reconstruct_uv(Frame* F, MB* m, ModeScore* rd, uint8_t* out, int mode) {
    const uint8_t* ref = m->predc[mode];
    const uint8_t* src = m->yuv_in + 16;
    int16_t tmp[8][16];
    uint32_t nz = 0;
    for (int n = 0; n < 8; ++n) {
        const int off = (n & 1) * 4 + ((n >> 1) & 1) * 4 * BPS + (n >> 2) * 8;  /* VP8ScanUV */
        ftransform(src + off, ref + off, tmp[n]);
    }
    if (F->use_derr) correct_dc_values(F, m, &m->dqm->uv, tmp, rd);
    for (int n = 0; n < 8; n += 2) {
        const int a = quantize_block(tmp[n], rd->uv_levels[n], &m->dqm->uv);
        const int b = quantize_block(tmp[n + 1], rd->uv_levels[n + 1], &m->dqm->uv);
        nz |= (uint32_t)(a | (b << 1)) << n;
    }
    for (int n = 0; n < 8; ++n) {
        const int off = (n & 1) * 4 + ((n >> 1) & 1) * 4 * BPS + (n >> 2) * 8;
        itransform(ref + off, tmp[n], out + off);
    }
    return (int)(nz << 16);
}

static void pick_best_uv(Frame* F, MB* m, ModeScore* rd) {
    const int lambda = m->dqm->lambda_uv;
    const uint8_t* src = m->yuv_in + 16;
    uint8_t tmp_out[BPS * 8], best_out[BPS * 8];
    ModeScore best;
    rd->mode_uv = -1;
    init_score(&best);
    for (int mode = 0; mode < 4; ++mode) {
        ModeScore uv;
        init_score(&uv);
        uv.nz = (uint32_t)reconstruct_uv(F, m, &uv, tmp_out, mode);
        uv.D = sse_wh(src, tmp_out, 16, 8);
        uv.SD = 0;
        uv.H = kFixedCostsUV[mode];
        uv.R = get_cost_uv(F, &uv);
        if (mode > 0 && is_flat(uv.uv_levels[0], 8, FLATNESS_LIMIT_UV)) uv.R += FLATNESS_PENALTY * 8;
        set_rd_score(lambda, &uv);
        if (mode == 0 || uv.score < best.score) {
            copy_score(&best, &uv);
            rd->mode_uv = mode;
            memcpy(rd->uv_levels, uv.uv_levels, sizeof(rd->uv_levels));
            memcpy(rd->derr, uv.derr, sizeof(rd->derr));
            memcpy(best_out, tmp_out, sizeof(best_out));
        }
    }
    add_score(rd, &best);
    for (int y = 0; y < 8; ++y) memcpy(m->yuv_out + 16 + y * BPS, best_out + y * BPS, 16);
    if (F->use_derr) {
        for (int ch = 0; ch <= 1; ++ch) {
            int8_t* top = F->top_derr[m->mx][ch];
            int8_t* left = F->left_derr[ch];
            left[0] = rd->derr[ch][0];
            left[1] = (int8_t)((3 * rd->derr[ch][2]) >> 2);
            top[0] = rd->derr[ch][1];
            top[1] = (int8_t)(rd->derr[ch][2] - left[1]);
        }
    }
}

static void record_tokens(Frame* F, int is_i16, const ModeScore* rd) {
    Residual r;
    nz_to_bytes(F, g_mx);
    if (is_i16) {
        const int ctx = F->top_nz[8] + F->left_nz[8];
        r.first = 0; r.type = 1;
        set_residual(&r, rd->y_dc_levels);
        F->top_nz[8] = F->left_nz[8] = record_coeff_tokens(&F->P, ctx, &r);
        r.first = 1; r.type = 0;
    } else {
        r.first = 0; r.type = 3;
    }
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const int ctx = F->top_nz[x] + F->left_nz[y];
            set_residual(&r, rd->y_ac_levels[x + y * 4]);
            F->top_nz[x] = F->left_nz[y] = record_coeff_tokens(&F->P, ctx, &r);
        }
    r.first = 0; r.type = 2;
    for (int ch = 0; ch <= 2; ch += 2)
        for (int y = 0; y < 2; ++y)
            for (int x = 0; x < 2; ++x) {
                const int ctx = F->top_nz[4 + ch + x] + F->left_nz[4 + ch + y];
                set_residual(&r, rd->uv_levels[ch * 2 + x + y * 2]);
                F->top_nz[4 + ch + x] = F->left_nz[4 + ch + y] = record_coeff_tokens(&F->P, ctx, &r);
            }
    bytes_to_nz(F, g_mx);
}

/*
 * y, u, v: the YUV420 planes (w x h, (w+1)/2 x (h+1)/2, tightly packed); seg: per-MB
 * segment ids (after SimplifySegments); quant[4]: segment quantisers; dq_uv_dc / dq_uv_ac:
 * the chroma deltas; quality: the config quality (error diffusion when <= 98).
 * Out: ymode per MB (0..3 = i16 DC/TM/V/H, 4 = intra-4), bmodes (16 per MB, raster),
 * uvmode per MB, probas[1056]: the final coefficient probabilities.  Returns 0.
 */
int iko_vp8_modes(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, float quality,
                  const uint8_t* seg, const int* quant, int dq_uv_dc, int dq_uv_ac, uint8_t* ymode,
                  uint8_t* bmodes, uint8_t* uvmode, uint8_t* probas) {
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16, uw = (w + 1) / 2, uh = (h + 1) / 2;
    const int W = mb_w * 16, H = mb_h * 16;
    uint8_t* Y = malloc((size_t)W * H);
    uint8_t* U = malloc((size_t)W / 2 * H / 2);
    uint8_t* V = malloc((size_t)W / 2 * H / 2);
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) Y[(size_t)r * W + c] = y[(size_t)(r < h ? r : h - 1) * w + (c < w ? c : w - 1)];
    for (int r = 0; r < H / 2; ++r)
        for (int c = 0; c < W / 2; ++c) {
            const size_t s = (size_t)(r < uh ? r : uh - 1) * uw + (c < uw ? c : uw - 1);
            U[(size_t)r * (W / 2) + c] = u[s];
            V[(size_t)r * (W / 2) + c] = v[s];
        }
    Frame F;
    memset(&F, 0, sizeof(F));
    F.mb_w = mb_w;
    F.mb_h = mb_h;
    F.y_top = malloc((size_t)W + 4);
    F.uv_top = malloc((size_t)W);
    memset(F.y_top, 127, (size_t)W + 4);
    memset(F.uv_top, 127, (size_t)W);
    F.nz = calloc((size_t)mb_w + 1, sizeof(uint32_t));
    F.top_derr = calloc((size_t)mb_w, sizeof(*F.top_derr));
    F.preds_w = mb_w * 4 + 1;
    F.preds = calloc((size_t)F.preds_w * (mb_h * 4 + 1), 1);
    F.use_derr = quality <= ERROR_DIFFUSION_QUALITY;
    memcpy(F.P.coeffs, kCoeffsProba0, 1056);
    F.P.dirty = 1;
    SegQ segq[4];
    for (int s = 0; s < 4; ++s) setup_matrices(&segq[s], quant[s], dq_uv_dc, dq_uv_ac, 50);
    for (int s = 0; s < 4; ++s) {
        g_max_edge[s] = 0;
        g_y2q1[s] = segq[s].y2.q[1];
    }
    calculate_level_costs(&F.P);
    int max_count = (mb_w * mb_h) >> 3;
    if (max_count < 96) max_count = 96;  /* MIN_COUNT */
    int cnt = max_count;
    /* max_i4_header_bits_: 256 * 16 * 16 * limit^2 / 100^2, partition_limit 0 */
    const int max_i4_header_bits = 256 * 16 * 16;
    for (int my = 0; my < mb_h; ++my) {
        /* InitLeft */
        memset(F.y_left, 129, sizeof(F.y_left));
        memset(F.u_left, 129, sizeof(F.u_left));
        memset(F.v_left, 129, sizeof(F.v_left));
        F.y_left[0] = F.u_left[0] = F.v_left[0] = my > 0 ? 129 : 127;
        F.left_dc_nz = 0;
        F.nz[0] = 0;
        memset(F.left_derr, 0, sizeof(F.left_derr));
        for (int mx = 0; mx < mb_w; ++mx) {
            MB m;
            g_mx = mx;
            m.mx = mx;
            m.my = my;
            m.seg = seg[my * mb_w + mx];
            m.dqm = &segq[m.seg];
            for (int r = 0; r < 16; ++r) memcpy(m.yuv_in + r * BPS, Y + (size_t)(my * 16 + r) * W + mx * 16, 16);
            for (int r = 0; r < 8; ++r) {
                memcpy(m.yuv_in + 16 + r * BPS, U + (size_t)(my * 8 + r) * (W / 2) + mx * 8, 8);
                memcpy(m.yuv_in + 24 + r * BPS, V + (size_t)(my * 8 + r) * (W / 2) + mx * 8, 8);
            }
            if ((--cnt) < 0) {
                finalize_token_probas(&F.P);
                calculate_level_costs(&F.P);
                cnt = max_count;
            }
            /* predictions */
            {
                const uint8_t* left = mx ? F.y_left + 1 : NULL;
                const uint8_t* top = my ? F.y_top + mx * 16 : NULL;
                for (int md = 0; md < 4; ++md) pred_nxn(m.pred16[md], md, left, top, 16);
                uint8_t uvl[9 + 16], *ul = uvl + 1;  /* u_left (corner at -1) */
                uint8_t vvl[9], *vl = vvl + 1;
                memcpy(uvl, F.u_left, 9);
                memcpy(vvl, F.v_left, 9);
                const uint8_t* ut = my ? F.uv_top + mx * 16 : NULL;
                const uint8_t* vt = my ? F.uv_top + mx * 16 + 8 : NULL;
                for (int md = 0; md < 4; ++md) {
                    pred_nxn(m.predc[md], md, mx ? ul : NULL, ut, 8);
                    pred_nxn(m.predc[md] + 8, md, mx ? vl : NULL, vt, 8);
                }
            }
            ModeScore rd;
            memset(&rd, 0, sizeof(rd));
            pick_best_intra16(&F, &m, &rd);
            const int i4 = pick_best_intra4(&F, &m, &rd, max_i4_header_bits);
            pick_best_uv(&F, &m, &rd);
            uint8_t* pr = PREDS(&F, mx, my);
            const int idx = my * mb_w + mx;
            if (i4) {
                ymode[idx] = 4;
                for (int k = 0; k < 16; ++k) pr[(k >> 2) * F.preds_w + (k & 3)] = rd.modes_i4[k];
                memcpy(bmodes + (size_t)idx * 16, rd.modes_i4, 16);
            } else {
                ymode[idx] = (uint8_t)rd.mode_i16;
                for (int k = 0; k < 16; ++k) pr[(k >> 2) * F.preds_w + (k & 3)] = (uint8_t)rd.mode_i16;
                memset(bmodes + (size_t)idx * 16, rd.mode_i16, 16);
            }
            uvmode[idx] = (uint8_t)rd.mode_uv;
            record_tokens(&F, !i4, &rd);
            /* VP8IteratorSaveBoundary */
            if (mx < mb_w - 1) {
                for (int i = 0; i < 16; ++i) F.y_left[1 + i] = m.yuv_out[15 + i * BPS];
                for (int i = 0; i < 8; ++i) {
                    F.u_left[1 + i] = m.yuv_out[16 + 7 + i * BPS];
                    F.v_left[1 + i] = m.yuv_out[16 + 15 + i * BPS];
                }
                F.y_left[0] = F.y_top[mx * 16 + 15];
                F.u_left[0] = F.uv_top[mx * 16 + 7];
                F.v_left[0] = F.uv_top[mx * 16 + 8 + 7];
            }
            if (my < mb_h - 1) {
                memcpy(F.y_top + mx * 16, m.yuv_out + 15 * BPS, 16);
                memcpy(F.uv_top + mx * 16, m.yuv_out + 16 + 7 * BPS, 16);
            }
        }
    }
    finalize_token_probas(&F.P);
    memcpy(probas, F.P.coeffs, 1056);
    free(Y); free(U); free(V);
    free(F.y_top); free(F.uv_top); free(F.nz); free(F.top_derr); free(F.preds);
    return 0;
}

/* ---- the bitstream (libwebp utils/bit_writer_utils.c, enc/syntax_enc.c) ---- */
typedef struct {
    int32_t range, value;
    int run, nb_bits;
    uint8_t* buf;
    size_t pos, cap;
} BitWriter;

static void bw_init(BitWriter* bw) {
    memset(bw, 0, sizeof(*bw));
    bw->range = 255 - 1;
    bw->nb_bits = -8;
}

static void bw_byte(BitWriter* bw, uint8_t b) {
    if (bw->pos == bw->cap) {
        bw->cap = bw->cap * 2 + 1024;
        bw->buf = realloc(bw->buf, bw->cap);
    }
    bw->buf[bw->pos++] = b;
}

static void bw_flush(BitWriter* bw) {
    const int s = 8 + bw->nb_bits;
    const int32_t bits = bw->value >> s;
    bw->value -= bits << s;
    bw->nb_bits -= 8;
    if ((bits & 0xff) != 0xff) {
        if (bits & 0x100) {  /* carry into the bytes written */
            if (bw->pos > 0) bw->buf[bw->pos - 1]++;
        }
        for (; bw->run > 0; --bw->run) bw_byte(bw, (bits & 0x100) ? 0x00 : 0xff);
        bw_byte(bw, (uint8_t)(bits & 0xff));
    } else {
        bw->run++;  /* delay 0xff bytes, a carry may still come */
    }
}

static int norm_shift(int r) { int s = 0; while (((r + 1) << s) < 128) ++s; return s; }

static int bw_put(BitWriter* bw, int bit, int prob) {
    const int split = (bw->range * prob) >> 8;
    if (bit) {
        bw->value += split + 1;
        bw->range -= split + 1;
    } else {
        bw->range = split;
    }
    if (bw->range < 127) {
        const int shift = norm_shift(bw->range);
        bw->range = ((bw->range + 1) << shift) - 1;
        bw->value <<= shift;
        bw->nb_bits += shift;
        if (bw->nb_bits > 0) bw_flush(bw);
    }
    return bit;
}

static int bw_uniform(BitWriter* bw, int bit) {
    const int split = bw->range >> 1;
    if (bit) {
        bw->value += split + 1;
        bw->range -= split + 1;
    } else {
        bw->range = split;
    }
    if (bw->range < 127) {
        bw->range = ((bw->range + 1) << 1) - 1;
        bw->value <<= 1;
        bw->nb_bits += 1;
        if (bw->nb_bits > 0) bw_flush(bw);
    }
    return bit;
}

static void bw_bits(BitWriter* bw, uint32_t value, int nb) {
    for (uint32_t mask = 1u << (nb - 1); mask; mask >>= 1) bw_uniform(bw, (value & mask) != 0);
}

static void bw_signed(BitWriter* bw, int value, int nb) {
    if (!bw_uniform(bw, value != 0)) return;
    if (value < 0) bw_bits(bw, ((uint32_t)(-value) << 1) | 1u, nb + 1);
    else bw_bits(bw, (uint32_t)value << 1, nb + 1);
}

static void bw_finish(BitWriter* bw) {
    bw_bits(bw, 0, 9 - bw->nb_bits);
    bw->nb_bits = 0;
    bw_flush(bw);
}

static void put_le32(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }

/*
 * The whole WebP file libwebp writes (WebPEncodeRGB, method 4, lossy, no alpha) from the
 * YUV420 planes and the restated segment set-up (tests/oracle_vp8.py): seg (per MB),
 * num_segments / update_map / probs[3] (segment map), quant[4], fstr[4] (filter levels
 * before libwebp raises them after coding), dq_uv_dc / dq_uv_ac.  *out is malloc'd;
 * returns its size.
 */
long iko_vp8_encode(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, float quality,
                    const uint8_t* seg, int num_segments, int update_map, const int* probs, const int* quant,
                    const int* fstr, int dq_uv_dc, int dq_uv_ac, uint8_t** out) {
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16, n = mb_w * mb_h;
    uint8_t* ym = malloc((size_t)n);
    uint8_t* bm = malloc((size_t)n * 16);
    uint8_t* uvm = malloc((size_t)n);
    uint8_t probas[1056];
    g_ntok = 0;  /* the token sink on */
    g_tcap = 4096;
    g_tok = malloc(g_tcap * sizeof(*g_tok));
    iko_vp8_modes(y, u, v, w, h, quality, seg, quant, dq_uv_dc, dq_uv_ac, ym, bm, uvm, probas);
    /* VP8AdjustFilterStrength (no autofilter): each segment's level at least the one its
     * largest DC step needs (kLevelsFromDelta[sharpness 0] is the identity on 0..63) */
    int level[4], max_level = 0;
    for (int s = 0; s < 4; ++s) {
        const int delta = (g_max_edge[s] * g_y2q1[s]) >> 3;
        const int lv = delta < 63 ? delta : 63;
        level[s] = fstr[s] > lv ? fstr[s] : lv;
        if (level[s] > max_level) max_level = level[s];
    }
    /* partition 0: header + modes (GeneratePartition0) */
    BitWriter b0;
    bw_init(&b0);
    bw_uniform(&b0, 0);  /* colour space */
    bw_uniform(&b0, 0);  /* clamping */
    if (bw_uniform(&b0, num_segments > 1)) {
        bw_uniform(&b0, update_map);
        if (bw_uniform(&b0, 1)) {  /* segment data, absolute values */
            bw_uniform(&b0, 1);
            for (int s = 0; s < 4; ++s) bw_signed(&b0, quant[s], 7);
            for (int s = 0; s < 4; ++s) bw_signed(&b0, level[s], 6);
        }
        if (update_map)
            for (int s = 0; s < 3; ++s)
                if (bw_uniform(&b0, probs[s] != 255)) bw_bits(&b0, (uint32_t)probs[s], 8);
    }
    bw_uniform(&b0, 0);          /* normal (not simple) loop filter */
    bw_bits(&b0, (uint32_t)max_level, 6);
    bw_bits(&b0, 0, 3);          /* sharpness */
    bw_uniform(&b0, 0);          /* no lf deltas */
    bw_bits(&b0, 0, 2);          /* one token partition */
    bw_bits(&b0, (uint32_t)quant[0], 7);
    bw_signed(&b0, 0, 4);
    bw_signed(&b0, 0, 4);
    bw_signed(&b0, 0, 4);
    bw_signed(&b0, dq_uv_dc, 4);
    bw_signed(&b0, dq_uv_ac, 4);
    bw_uniform(&b0, 0);          /* no entropy refresh */
    for (int i = 0; i < 1056; ++i)
        if (bw_put(&b0, probas[i] != kCoeffsProba0[i], kCoeffsUpdateProba[i])) bw_bits(&b0, probas[i], 8);
    bw_uniform(&b0, 0);          /* no skip probability */
    {
        const int pw = mb_w * 4;
        uint8_t* pr = calloc((size_t)pw * mb_h * 4, 1);
        for (int i = 0; i < n; ++i) {
            const int mx = i % mb_w, my = i / mb_w;
            for (int k = 0; k < 16; ++k) pr[(my * 4 + (k >> 2)) * pw + mx * 4 + (k & 3)] = bm[(size_t)i * 16 + k];
        }
        for (int i = 0; i < n; ++i) {
            const int mx = i % mb_w, my = i / mb_w;
            if (update_map) {
                const int sg = seg[i];
                if (bw_put(&b0, sg >= 2, probs[0])) bw_put(&b0, sg & 1, probs[2]);
                else bw_put(&b0, sg & 1, probs[1]);
            }
            if (bw_put(&b0, ym[i] != 4, 145)) {
                const int mode = ym[i];
                if (bw_put(&b0, mode == 1 || mode == 3, 156)) bw_put(&b0, mode == 1, 128);
                else bw_put(&b0, mode == 2, 163);
            } else {
                for (int k = 0; k < 16; ++k) {
                    const int by = my * 4 + (k >> 2), bx = mx * 4 + (k & 3);
                    const int top = by > 0 ? pr[(by - 1) * pw + bx] : 0, left = bx > 0 ? pr[by * pw + bx - 1] : 0;
                    const uint8_t* p = kBModesProba + (top * 10 + left) * 9;
                    const int mode = bm[(size_t)i * 16 + k];
                    if (bw_put(&b0, mode != 0, p[0]))
                        if (bw_put(&b0, mode != 1, p[1]))
                            if (bw_put(&b0, mode != 2, p[2])) {
                                if (!bw_put(&b0, mode >= 6, p[3])) {
                                    if (bw_put(&b0, mode != 3, p[4])) bw_put(&b0, mode != 4, p[5]);
                                } else if (bw_put(&b0, mode != 6, p[6])) {
                                    if (bw_put(&b0, mode != 7, p[7])) bw_put(&b0, mode != 8, p[8]);
                                }
                            }
                }
            }
            const int uvmd = uvm[i];
            if (bw_put(&b0, uvmd != 0, 142))
                if (bw_put(&b0, uvmd != 2, 114)) bw_put(&b0, uvmd != 3, 183);
        }
        free(pr);
    }
    bw_finish(&b0);
    /* partition 1: the tokens with the final probabilities (VP8EmitTokens) */
    BitWriter b1;
    bw_init(&b1);
    for (size_t i = 0; i < g_ntok; ++i) {
        const uint32_t t = g_tok[i];
        const int bit = (int)((t >> 15) & 1);
        if (t & (1u << 14)) bw_put(&b1, bit, (int)(t & 0xffu));
        else bw_put(&b1, bit, probas[t & 0x3fffu]);
    }
    bw_finish(&b1);
    free(g_tok);
    g_tok = NULL; g_ntok = 0; g_tcap = 0;
    /* RIFF + VP8 chunk (PutWebPHeaders, PutVP8FrameHeader; profile 0: normal filter) */
    size_t vp8_size = 10 + b0.pos + b1.pos;
    const size_t pad = vp8_size & 1;
    vp8_size += pad;
    const size_t riff_size = 4 + 8 + vp8_size;
    const size_t total = 8 + riff_size;
    uint8_t* o = malloc(total);
    memcpy(o, "RIFF", 4);
    put_le32(o + 4, (uint32_t)riff_size);
    memcpy(o + 8, "WEBPVP8 ", 8);
    put_le32(o + 16, (uint32_t)vp8_size);
    {
        const uint32_t bits = 0u | (0u << 1) | (1u << 4) | ((uint32_t)b0.pos << 5);
        uint8_t* f = o + 20;
        f[0] = (uint8_t)bits; f[1] = (uint8_t)(bits >> 8); f[2] = (uint8_t)(bits >> 16);
        f[3] = 0x9d; f[4] = 0x01; f[5] = 0x2a;
        f[6] = (uint8_t)(w & 0xff); f[7] = (uint8_t)(w >> 8); f[8] = (uint8_t)(h & 0xff); f[9] = (uint8_t)(h >> 8);
    }
    memcpy(o + 30, b0.buf, b0.pos);
    memcpy(o + 30 + b0.pos, b1.buf, b1.pos);
    if (pad) o[30 + b0.pos + b1.pos] = 0;
    free(b0.buf); free(b1.buf);
    free(ym); free(bm); free(uvm);
    *out = o;
    return (long)total;
}
