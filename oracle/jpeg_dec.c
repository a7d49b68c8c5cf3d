/*
 * jpeg_dec.c -- CPU ORACLE: decode_image on a JPEG (reference src/transform.rs:31
 * -> image 0.25.8 -> zune-jpeg 0.4.21, Cargo.lock:3106-3109).
 *
 * TEST INFRASTRUCTURE ONLY (see ik_oracle.h): the checker for the GPU JPEG path.
 *
 * Entropy decoding (ITU T.81): baseline and extended sequential (SOF0/SOF1),
 * progressive (SOF2: DC first/refine, AC first/refine with EOB runs), restart
 * intervals, 8-bit, 1, 3 or 4 components -> dense quantised coefficient planes
 * (one plane of 8x8 blocks per component, MCU-padded, natural order).
 *
 * Reconstruction, two restatements over the same coefficients:
 *
 *   IKO_JPEG_LIBJPEG  libjpeg(-turbo) jidctint.c islow IDCT, jdsample.c "fancy"
 *                     h2v1 / h2v2 / h1v2 upsampling over the component's real
 *                     width/height (ceil(W h / hmax)), jdcolor.c YCbCr->RGB
 *                     (SCALEBITS 16).  PINNED: equal to Pillow's decoder
 *                     (libjpeg-turbo) on every stream of tests/test_oracle_jpeg.py,
 *                     which pins the entropy decoder above as well.
 *
 *   IKO_JPEG_ZUNE     zune-jpeg 0.4.21's published algorithm, restated:
 *                     - IDCT: idct/scalar.rs (and its AVX2 twin) -- stb_image's
 *                       fixed-point IDCT (stbi__idct_block: f2f = (int)(x*4096+0.5),
 *                       column pass + 512 >> 10), row pass + SCALE_BITS
 *                       (512 + 65536 + (128 << 17)) >> 17, clamp 0..255; a block
 *                       whose 63 AC coefficients are all zero takes the shortcut
 *                       clamp((dc >> 3) + 128) (not what the full path rounds to);
 *                     - upsampling: upsampler/scalar.rs -- separable, vertical first
 *                       (3 near + far + 2) >> 2 into i16, then horizontal
 *                       out[2i] = (3 in[i] + in[i-1] + 2) >> 2,
 *                       out[2i+1] = (3 in[i] + in[i+1] + 2) >> 2, out[0] = in[0],
 *                       out[2n-2] = (3 in[n-2] + in[n-1] + 2) >> 2, out[2n-1] = in[n-1],
 *                       over the MCU-padded component row (n = blocks * 8), the row
 *                       above/below replicated at the padded top/bottom;
 *                       other ratios replicate (upsample_generic);
 *                     - colour: color_convert/scalar.rs ycbcr_to_rgb_inner_16_scalar
 *                       in i16: r = y + ((45 cr') >> 5),
 *                       g = y - ((11 cb' + 23 cr') >> 5), b = y + ((113 cb') >> 6),
 *                       cb' = cb - 128, cr' = cr - 128, clamp 0..255.
 *                     PARITY UNPINNED: there is no zune-jpeg source, binary or output
 *                     in this environment (no Rust toolchain, no crate sources, no
 *                     network); the constants above are restated from the published
 *                     crate, the right-edge horizontal rule and the padded-edge
 *                     context are its code as recalled and the least certain parts.
 *
 * CMYK / YCCK (4 components; Adobe APP14 transform 0 / 2): both modes convert to
 * RGB8 as Pillow's decoder does -- Adobe CMYK is stored inverted (rawmode
 * "CMYK;I"), YCCK is YCbCr->RGB then inverted into CMY (libjpeg jdcolor.c
 * ycck_cmyk_convert), then Convert.c cmyk2rgb: R = nk - MULDIV255(C, nk),
 * nk = 255 - K.  Pinned against Pillow for CMYK in the libjpeg mode; zune-jpeg's
 * own CMYK->RGB is unpinned (assumed the same).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ik_oracle.h"

static const uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

typedef struct {
    int present;
    int maxcode[18], valptr[17], mincode[17];
    uint8_t vals[256];
} Huff;

typedef struct {
    int id, h, v, tq, td, ta;
    int bw, bh, dw, dh;  /* blocks (MCU-padded), real sample width/height */
    size_t blk0;
    int pred;
} Comp;

typedef struct {
    const uint8_t *p, *end;
    uint32_t acc;
    int nbits;
    int marker; /* a marker was hit: zeros are fed from here on */
} Bits;

typedef struct {
    const uint8_t *b, *end;
    uint16_t qt[4][64];
    Huff dc[4], ac[4];
    Comp c[4];
    int nc, W, H, hmax, vmax, mcux, mcuy, restart, progressive, adobe, adobe_transform, have_frame;
    int16_t *coef;
    size_t nblocks;
    int eobrun;
} Dec;

static int build_huff(const uint8_t *bits, const uint8_t *vals, int nvals, Huff *t) {
    memset(t, 0, sizeof(*t));
    memcpy(t->vals, vals, (size_t)nvals);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        t->valptr[l] = k;
        t->mincode[l] = code;
        code += bits[l - 1];
        k += bits[l - 1];
        t->maxcode[l] = bits[l - 1] ? code - 1 : -1;
        if (code > (1 << l)) return -1;
        code <<= 1;
    }
    t->maxcode[17] = 0x7fffffff;
    t->present = 1;
    return 0;
}

static void fill(Bits *br) {
    while (br->nbits <= 24) {
        int byte = 0;
        if (!br->marker && br->p < br->end) {
            byte = *br->p;
            if (byte == 0xFF) {
                const int nx = br->p + 1 < br->end ? br->p[1] : 0;
                if (nx == 0x00) {
                    br->p += 2;
                } else { /* a marker: stop, feed zeros */
                    br->marker = 1;
                    byte = 0;
                }
            } else {
                br->p++;
            }
        }
        br->acc |= (uint32_t)byte << (24 - br->nbits);
        br->nbits += 8;
    }
}

static int getbits(Bits *br, int n) {
    if (!n) return 0;
    fill(br);
    const int v = (int)(br->acc >> (32 - n));
    br->acc <<= n;
    br->nbits -= n;
    return v;
}

static int getbit(Bits *br) { return getbits(br, 1); }

static int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

static int decode_sym(Bits *br, const Huff *t) {
    if (!t->present) return -1;
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
        code = (code << 1) | getbit(br);
        if (code <= t->maxcode[l]) return t->vals[t->valptr[l] + code - t->mincode[l]];
    }
    return -1;
}

/* at a restart boundary: skip to the RSTn marker and reset the reader */
static void restart_reader(Bits *br) {
    const uint8_t *p = br->p;
    while (p + 1 < br->end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < br->end) p += 2;
    br->p = p;
    br->acc = 0;
    br->nbits = 0;
    br->marker = 0;
}

static int16_t *blockp(Dec *d, const Comp *c, int bx, int by) {
    return &d->coef[(c->blk0 + (size_t)by * c->bw + bx) * 64];
}

/* one block of a scan (T.81 F.2.2 / G.1.2) */
static int scan_block(Dec *d, Bits *br, Comp *c, int16_t *blk, int ss, int se, int ah, int al) {
    if (!d->progressive) {
        int t = decode_sym(br, &d->dc[c->td]);
        if (t < 0 || t > 11) return -1;
        c->pred += t ? extend(getbits(br, t), t) : 0;
        blk[0] = (int16_t)c->pred;
        for (int k = 1; k < 64;) {
            const int rs = decode_sym(br, &d->ac[c->ta]);
            if (rs < 0) return -1;
            const int r = rs >> 4, s = rs & 15;
            if (!s) {
                if (r != 15) break;
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return -1;
            blk[kZz[k]] = (int16_t)extend(getbits(br, s), s);
            ++k;
        }
        return 0;
    }
    if (ss == 0) { /* DC scan */
        if (ah == 0) {
            int t = decode_sym(br, &d->dc[c->td]);
            if (t < 0 || t > 11) return -1;
            c->pred += t ? extend(getbits(br, t), t) : 0;
            blk[0] = (int16_t)(c->pred * (1 << al));
        } else if (getbit(br)) {
            blk[0] |= (int16_t)(1 << al);
        }
        return 0;
    }
    if (ah == 0) { /* AC first */
        if (d->eobrun > 0) { --d->eobrun; return 0; }
        for (int k = ss; k <= se;) {
            const int rs = decode_sym(br, &d->ac[c->ta]);
            if (rs < 0) return -1;
            const int r = rs >> 4, s = rs & 15;
            if (!s) {
                if (r < 15) {
                    d->eobrun = (1 << r) - 1;
                    if (r) d->eobrun += getbits(br, r);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return -1;
            blk[kZz[k]] = (int16_t)(extend(getbits(br, s), s) * (1 << al));
            ++k;
        }
        return 0;
    }
    /* AC refine (jdphuff.c decode_mcu_AC_refine) */
    const int p1 = 1 << al, m1 = -1 * (1 << al);
    int k = ss;
    if (d->eobrun <= 0) {
        for (; k <= se;) {
            const int rs = decode_sym(br, &d->ac[c->ta]);
            if (rs < 0) return -1;
            int r = rs >> 4, s = rs & 15, v = 0;
            if (s) {
                if (s != 1) return -1;
                v = getbit(br) ? p1 : m1;
            } else if (r != 15) {
                d->eobrun = 1 << r;
                if (r) d->eobrun += getbits(br, r);
                break;
            }
            while (k <= se) {
                int16_t *cp = &blk[kZz[k]];
                if (*cp) {
                    if (getbit(br) && (*cp & p1) == 0) *cp = (int16_t)(*cp >= 0 ? *cp + p1 : *cp + m1);
                } else {
                    if (r == 0) {
                        if (v) *cp = (int16_t)v;
                        ++k;
                        break;
                    }
                    --r;
                }
                ++k;
            }
        }
    }
    if (d->eobrun > 0) {
        for (; k <= se; ++k) {
            int16_t *cp = &blk[kZz[k]];
            if (*cp && getbit(br) && (*cp & p1) == 0) *cp = (int16_t)(*cp >= 0 ? *cp + p1 : *cp + m1);
        }
        --d->eobrun;
    }
    return 0;
}

static int scan(Dec *d, const uint8_t *s, int len, const uint8_t **after) {
    const int ns = s[0];
    if (ns < 1 || ns > 4 || len < 1 + 2 * ns + 3) return -1;
    Comp *sc[4];
    for (int i = 0; i < ns; ++i) {
        const int id = s[1 + 2 * i];
        sc[i] = NULL;
        for (int k = 0; k < d->nc; ++k)
            if (d->c[k].id == id) sc[i] = &d->c[k];
        if (!sc[i]) return -1;
        sc[i]->td = s[2 + 2 * i] >> 4;
        sc[i]->ta = s[2 + 2 * i] & 15;
        if (sc[i]->td > 3 || sc[i]->ta > 3) return -1;
    }
    const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ah = s[3 + 2 * ns] >> 4, al = s[3 + 2 * ns] & 15;
    Bits br = {s + len, d->end, 0, 0, 0};
    for (int i = 0; i < ns; ++i) sc[i]->pred = 0;
    d->eobrun = 0;
    long mcu = 0;
    const int single = ns == 1;
    const long total = single ? (long)((sc[0]->dw + 7) / 8) * ((sc[0]->dh + 7) / 8) : (long)d->mcux * d->mcuy;
    const int sbw = single ? (sc[0]->dw + 7) / 8 : 0;
    for (; mcu < total; ++mcu) {
        if (d->restart && mcu && mcu % d->restart == 0) {
            restart_reader(&br);
            for (int i = 0; i < ns; ++i) sc[i]->pred = 0;
            d->eobrun = 0;
        }
        if (single) {
            const int bx = (int)(mcu % sbw), by = (int)(mcu / sbw);
            if (scan_block(d, &br, sc[0], blockp(d, sc[0], bx, by), ss, se, ah, al)) return -1;
        } else {
            const int mx = (int)(mcu % d->mcux), my = (int)(mcu / d->mcux);
            for (int i = 0; i < ns; ++i)
                for (int v = 0; v < sc[i]->v; ++v)
                    for (int h = 0; h < sc[i]->h; ++h)
                        if (scan_block(d, &br, sc[i], blockp(d, sc[i], mx * sc[i]->h + h, my * sc[i]->v + v), ss, se,
                                       ah, al))
                            return -1;
        }
    }
    /* continue after the entropy-coded data: the next marker that is not RSTn */
    const uint8_t *p = br.p;
    while (p + 1 < d->end && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
    *after = p;
    return 0;
}

static int parse(Dec *d) {
    const uint8_t *p = d->b;
    if (d->end - p < 4 || p[0] != 0xFF || p[1] != 0xD8) return -1;
    p += 2;
    while (p + 4 <= d->end) {
        if (p[0] != 0xFF) { ++p; continue; }
        const int m = p[1];
        if (m == 0xFF) { ++p; continue; }
        if (m == 0xD9) break;
        if (m >= 0xD0 && m <= 0xD7) { p += 2; continue; }
        const int len = (int)p[2] << 8 | p[3];
        if (len < 2 || p + 2 + len > d->end) return -1;
        const uint8_t *s = p + 4;
        const int n = len - 2;
        if (m == 0xDB) { /* DQT */
            for (int o = 0; o < n;) {
                const int pq = s[o] >> 4, tq = s[o] & 3;
                ++o;
                for (int k = 0; k < 64; ++k) {
                    d->qt[tq][kZz[k]] = pq ? (uint16_t)(s[o + 2 * k] << 8 | s[o + 2 * k + 1]) : s[o + k];
                }
                o += pq ? 128 : 64;
            }
        } else if (m == 0xC4) { /* DHT */
            for (int o = 0; o < n;) {
                const int tc = s[o] >> 4, th = s[o] & 3;
                int tot = 0;
                for (int k = 0; k < 16; ++k) tot += s[o + 1 + k];
                if (tot > 256 || build_huff(s + o + 1, s + o + 17, tot, tc ? &d->ac[th] : &d->dc[th])) return -1;
                o += 17 + tot;
            }
        } else if (m == 0xDD) {
            d->restart = (int)s[0] << 8 | s[1];
        } else if (m == 0xEE) {
            if (n >= 12 && !memcmp(s, "Adobe", 5)) { d->adobe = 1; d->adobe_transform = s[11]; }
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
            if (s[0] != 8) return -1;
            d->progressive = m == 0xC2;
            d->H = (int)s[1] << 8 | s[2];
            d->W = (int)s[3] << 8 | s[4];
            d->nc = s[5];
            if (!d->W || !d->H || (d->nc != 1 && d->nc != 3 && d->nc != 4)) return -1;
            d->hmax = d->vmax = 1;
            for (int i = 0; i < d->nc; ++i) {
                d->c[i].id = s[6 + 3 * i];
                d->c[i].h = s[7 + 3 * i] >> 4;
                d->c[i].v = s[7 + 3 * i] & 15;
                d->c[i].tq = s[8 + 3 * i] & 3;
                if (d->c[i].h < 1 || d->c[i].h > 4 || d->c[i].v < 1 || d->c[i].v > 4) return -1;
                if (d->c[i].h > d->hmax) d->hmax = d->c[i].h;
                if (d->c[i].v > d->vmax) d->vmax = d->c[i].v;
            }
            d->mcux = (d->W + 8 * d->hmax - 1) / (8 * d->hmax);
            d->mcuy = (d->H + 8 * d->vmax - 1) / (8 * d->vmax);
            size_t blocks = 0;
            for (int i = 0; i < d->nc; ++i) {
                Comp *c = &d->c[i];
                if (d->hmax % c->h || d->vmax % c->v) return -1;
                c->bw = d->mcux * c->h;
                c->bh = d->mcuy * c->v;
                c->dw = (d->W * c->h + d->hmax - 1) / d->hmax;
                c->dh = (d->H * c->v + d->vmax - 1) / d->vmax;
                c->blk0 = blocks;
                blocks += (size_t)c->bw * c->bh;
            }
            d->nblocks = blocks;
            d->coef = (int16_t *)calloc(blocks * 64, sizeof(int16_t));
            if (!d->coef) return -1;
            d->have_frame = 1;
        } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return -1; /* arithmetic / lossless / hierarchical */
        } else if (m == 0xDA) {
            if (!d->have_frame) return -1;
            const uint8_t *after;
            if (scan(d, s, n, &after)) return -1;
            p = after;
            continue;
        }
        p += 2 + len;
    }
    return d->have_frame ? 0 : -1;
}

/* ---- reconstruction: libjpeg(-turbo) ---- */
static int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
static uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

static void islow8(const int *i, int st, int *o) { /* jidctint.c butterfly, pre-descale */
    int z2 = i[2 * st], z3 = i[6 * st];
    int z1 = (z2 + z3) * 4433;
    int tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
    int tmp0 = (i[0] + i[4 * st]) * 8192, tmp1 = (i[0] - i[4 * st]) * 8192;
    const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = i[7 * st]; tmp1 = i[5 * st]; tmp2 = i[3 * st]; tmp3 = i[1 * st];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * 9633;
    tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    o[0] = t10 + tmp3; o[7] = t10 - tmp3; o[1] = t11 + tmp2; o[6] = t11 - tmp2;
    o[2] = t12 + tmp1; o[5] = t12 - tmp1; o[3] = t13 + tmp0; o[4] = t13 - tmp0;
}

static void idct_islow(const int *in, uint8_t *out, int stride) {
    int ws[64], o[8];
    for (int c = 0; c < 8; ++c) {
        if (!in[8 + c] && !in[16 + c] && !in[24 + c] && !in[32 + c] && !in[40 + c] && !in[48 + c] && !in[56 + c]) {
            for (int r = 0; r < 8; ++r) ws[r * 8 + c] = in[c] * 4;
            continue;
        }
        islow8(in + c, 8, o);
        for (int r = 0; r < 8; ++r) ws[r * 8 + c] = descale(o[r], 11);
    }
    for (int r = 0; r < 8; ++r) {
        const int *w = ws + r * 8;
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t dc = clamp8(descale(w[0], 5) + 128);
            for (int k = 0; k < 8; ++k) out[r * stride + k] = dc;
            continue;
        }
        islow8(w, 1, o);
        for (int k = 0; k < 8; ++k) out[r * stride + k] = clamp8(descale(o[k], 18) + 128);
    }
}

/* ---- reconstruction: zune-jpeg 0.4.21 (restated, unpinned) ---- */
static void zune8(const int *i, int st, int *x, int *t, int bias) {
    int p2 = i[2 * st], p3 = i[6 * st];
    int p1 = (p2 + p3) * 2217;
    int t2 = p1 + p3 * -7567, t3 = p1 + p2 * 3135;
    p2 = i[0];
    p3 = i[4 * st];
    int t0 = (p2 + p3) * 4096, t1 = (p2 - p3) * 4096;
    x[0] = t0 + t3 + bias; x[3] = t0 - t3 + bias; x[1] = t1 + t2 + bias; x[2] = t1 - t2 + bias;
    t0 = i[7 * st]; t1 = i[5 * st]; t2 = i[3 * st]; t3 = i[1 * st];
    p3 = t0 + t2;
    int p4 = t1 + t3;
    p1 = t0 + t3;
    p2 = t1 + t2;
    const int p5 = (p3 + p4) * 4816;
    t0 *= 1223; t1 *= 8410; t2 *= 12586; t3 *= 6149;
    p1 = p5 + p1 * -3685; p2 = p5 + p2 * -10497; p3 *= -8034; p4 *= -1597;
    t3 += p1 + p4; t2 += p2 + p3; t1 += p2 + p4; t0 += p1 + p3;
    t[0] = t0; t[1] = t1; t[2] = t2; t[3] = t3;
}

static void idct_zune(const int *in, uint8_t *out, int stride) {
    int ac = 0;
    for (int k = 1; k < 64; ++k) ac |= in[k];
    if (!ac) {
        const uint8_t v = clamp8((in[0] >> 3) + 128);
        for (int r = 0; r < 8; ++r)
            for (int k = 0; k < 8; ++k) out[r * stride + k] = v;
        return;
    }
    int ws[64], x[4], t[4];
    for (int c = 0; c < 8; ++c) {
        zune8(in + c, 8, x, t, 512);
        ws[c] = (x[0] + t[3]) >> 10; ws[8 + c] = (x[1] + t[2]) >> 10;
        ws[16 + c] = (x[2] + t[1]) >> 10; ws[24 + c] = (x[3] + t[0]) >> 10;
        ws[32 + c] = (x[3] - t[0]) >> 10; ws[40 + c] = (x[2] - t[1]) >> 10;
        ws[48 + c] = (x[1] - t[2]) >> 10; ws[56 + c] = (x[0] - t[3]) >> 10;
    }
    const int SCALE = 512 + 65536 + (128 << 17);
    for (int r = 0; r < 8; ++r) {
        zune8(ws + r * 8, 1, x, t, SCALE);
        uint8_t *o = out + r * stride;
        o[0] = clamp8((x[0] + t[3]) >> 17); o[1] = clamp8((x[1] + t[2]) >> 17);
        o[2] = clamp8((x[2] + t[1]) >> 17); o[3] = clamp8((x[3] + t[0]) >> 17);
        o[4] = clamp8((x[3] - t[0]) >> 17); o[5] = clamp8((x[2] - t[1]) >> 17);
        o[6] = clamp8((x[1] - t[2]) >> 17); o[7] = clamp8((x[0] - t[3]) >> 17);
    }
}

/* libjpeg fancy upsampling of component plane p (pw stride, real dw x dh) at (x, y) */
static int up_libjpeg(const uint8_t *p, int pw, int dw, int dh, int fh, int fv, int x, int y) {
    const int ow = dw * fh, oh = dh * fv;
    const int xs = x < ow ? x : ow - 1, ys = y < oh ? y : oh - 1;
#define ROW(r) (p + (size_t)((r) < 0 ? 0 : ((r) >= dh ? dh - 1 : (r))) * pw)
    if (fh == 1 && fv == 1) return ROW(ys)[xs];
    if (fh == 2 && fv == 1) {
        const uint8_t *ip = ROW(ys);
        const int X = xs >> 1;
        if (dw == 1) return ip[0];
        if (!(xs & 1)) return X == 0 ? ip[0] : (ip[X] * 3 + ip[X - 1] + 1) >> 2;
        return X == dw - 1 ? ip[X] : (ip[X] * 3 + ip[X + 1] + 2) >> 2;
    }
    if (fh == 2 && fv == 2) {
        const int Y = ys >> 1, X = xs >> 1;
        const uint8_t *i0 = ROW(Y), *i1 = ROW((ys & 1) ? Y + 1 : Y - 1);
        const int ths = i0[X] * 3 + i1[X];
        if (dw == 1) return (xs & 1) ? (ths * 4 + 7) >> 4 : (ths * 4 + 8) >> 4;
        if (!(xs & 1)) {
            if (X == 0) return (ths * 4 + 8) >> 4;
            return (ths * 3 + i0[X - 1] * 3 + i1[X - 1] + 8) >> 4;
        }
        if (X == dw - 1) return (ths * 4 + 7) >> 4;
        return (ths * 3 + i0[X + 1] * 3 + i1[X + 1] + 7) >> 4;
    }
    if (fh == 1 && fv == 2) {
        const int Y = ys >> 1, lower = ys & 1;
        const uint8_t *i0 = ROW(Y), *i1 = ROW(lower ? Y + 1 : Y - 1);
        return (i0[xs] * 3 + i1[xs] + (lower ? 2 : 1)) >> 2;
    }
    return ROW(ys / fv)[xs / fh];
#undef ROW
}

/* zune-jpeg upsampling over the MCU-padded plane (pw samples per row, ph rows) */
static int up_zune(const uint8_t *p, int pw, int ph, int fh, int fv, int x, int y) {
#define ZR(r) (p + (size_t)((r) < 0 ? 0 : ((r) >= ph ? ph - 1 : (r))) * pw)
    if (fh == 1 && fv == 1) return ZR(y)[x];
    if (fh == 2 && fv == 1) { /* upsample_horizontal */
        const uint8_t *ip = ZR(y);
        const int i = x >> 1, n = pw;
        if (x == 0) return ip[0];
        if (x == 1) return (ip[0] * 3 + ip[1] + 2) >> 2;
        if (x == 2 * n - 2) return (ip[n - 2] * 3 + ip[n - 1] + 2) >> 2;
        if (x == 2 * n - 1) return ip[n - 1];
        return (x & 1) ? (ip[i] * 3 + ip[i + 1] + 2) >> 2 : (ip[i] * 3 + ip[i - 1] + 2) >> 2;
    }
    if (fh == 1 && fv == 2) {
        const int Y = y >> 1;
        const uint8_t *i0 = ZR(Y), *i1 = ZR((y & 1) ? Y + 1 : Y - 1);
        return (i0[x] * 3 + i1[x] + 2) >> 2;
    }
    if (fh == 2 && fv == 2) { /* upsample_hv: upsample_vertical into i16, then upsample_horizontal */
        const int Y = y >> 1, n = pw, i = x >> 1;
        const uint8_t *i0 = ZR(Y), *i1 = ZR((y & 1) ? Y + 1 : Y - 1);
#define ZV(k) ((i0[k] * 3 + i1[k] + 2) >> 2)
        if (x == 0) return ZV(0);
        if (x == 1) return (ZV(0) * 3 + ZV(1) + 2) >> 2;
        if (x == 2 * n - 2) return (ZV(n - 2) * 3 + ZV(n - 1) + 2) >> 2;
        if (x == 2 * n - 1) return ZV(n - 1);
        return (x & 1) ? (ZV(i) * 3 + ZV(i + 1) + 2) >> 2 : (ZV(i) * 3 + ZV(i - 1) + 2) >> 2;
#undef ZV
    }
    return ZR(y / fv)[x / fh];
#undef ZR
}

static uint8_t muldiv255(int a, int b) {
    const int t = a * b + 128;
    return (uint8_t)(((t >> 8) + t) >> 8);
}

int iko_jpeg_decode(const uint8_t *bytes, size_t n, int mode, uint8_t **out, int *w, int *h, int *c) {
    Dec d;
    memset(&d, 0, sizeof(d));
    d.b = bytes;
    d.end = bytes + n;
    d.adobe_transform = -1;
    *out = NULL;
    if (parse(&d)) { free(d.coef); return -1; }
    const int nc = d.nc, W = d.W, H = d.H;
    /* IDCT every block of every component into MCU-padded planes */
    uint8_t *pl[4] = {0};
    for (int ci = 0; ci < nc; ++ci) {
        const Comp *cp = &d.c[ci];
        const int pw = cp->bw * 8;
        pl[ci] = (uint8_t *)malloc((size_t)pw * cp->bh * 8);
        if (!pl[ci]) return -1;
        const uint16_t *q = d.qt[cp->tq];
        for (int by = 0; by < cp->bh; ++by)
            for (int bx = 0; bx < cp->bw; ++bx) {
                const int16_t *blk = &d.coef[(cp->blk0 + (size_t)by * cp->bw + bx) * 64];
                int in[64];
                for (int k = 0; k < 64; ++k) in[k] = (int)blk[k] * (int)q[k];
                uint8_t *o = pl[ci] + (size_t)by * 8 * pw + (size_t)bx * 8;
                if (mode == IKO_JPEG_ZUNE) idct_zune(in, o, pw);
                else idct_islow(in, o, pw);
            }
    }
    const int oc = nc == 1 ? 1 : 3;
    uint8_t *img = (uint8_t *)malloc((size_t)W * H * oc);
    if (!img) return -1;
    int cs = nc == 1 ? 0 : 1; /* gray, YCbCr, RGB, CMYK, YCCK */
    if (nc == 3 && d.adobe && d.adobe_transform == 0) cs = 2;
    if (nc == 3 && !d.adobe && d.c[0].id == 'R' && d.c[1].id == 'G' && d.c[2].id == 'B') cs = 2;
    if (nc == 4) cs = d.adobe && d.adobe_transform == 2 ? 4 : 3;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int s[4];
            for (int ci = 0; ci < nc; ++ci) {
                const Comp *cp = &d.c[ci];
                const int fh = d.hmax / cp->h, fv = d.vmax / cp->v;
                s[ci] = mode == IKO_JPEG_ZUNE ? up_zune(pl[ci], cp->bw * 8, cp->bh * 8, fh, fv, x, y)
                                              : up_libjpeg(pl[ci], cp->bw * 8, cp->dw, cp->dh, fh, fv, x, y);
            }
            uint8_t *o = img + ((size_t)y * W + x) * oc;
            if (cs == 0) { o[0] = (uint8_t)s[0]; continue; }
            int r, g, b;
            if (cs == 2 || cs == 3) {
                r = s[0]; g = s[1]; b = s[2];
            } else if (mode == IKO_JPEG_ZUNE) {
                const int16_t cb = (int16_t)(s[1] - 128), cr = (int16_t)(s[2] - 128);
                r = s[0] + ((int16_t)(45 * cr) >> 5);
                g = s[0] - ((int16_t)(11 * cb + 23 * cr) >> 5);
                b = s[0] + ((int16_t)(113 * cb) >> 6);
            } else {
                const int cb = s[1] - 128, cr = s[2] - 128;
                r = s[0] + ((91881 * cr + 32768) >> 16);
                g = s[0] + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
                b = s[0] + ((116130 * cb + 32768) >> 16);
            }
            if (cs < 3) {
                o[0] = clamp8(r); o[1] = clamp8(g); o[2] = clamp8(b);
                continue;
            }
            /* CMYK / YCCK -> RGB (Pillow: Adobe CMYK is inverted; cmyk2rgb) */
            int cc, mm, yy;
            if (cs == 4) { cc = 255 - clamp8(r); mm = 255 - clamp8(g); yy = 255 - clamp8(b); }
            else { cc = r; mm = g; yy = b; }
            int k = s[3];
            if (d.adobe) { cc = 255 - cc; mm = 255 - mm; yy = 255 - yy; k = 255 - k; }
            const int nk = 255 - k;
            o[0] = clamp8(nk - muldiv255(cc, nk));
            o[1] = clamp8(nk - muldiv255(mm, nk));
            o[2] = clamp8(nk - muldiv255(yy, nk));
        }
    for (int ci = 0; ci < nc; ++ci) free(pl[ci]);
    free(d.coef);
    *out = img;
    *w = W;
    *h = H;
    *c = oc;
    return 0;
}
