// ik_vp8_enc.cpp -- host half of the GPU WebP encoder (see ik_vp8_enc.h): token
// statistics and coefficient-probability updates, the RFC 6386 boolean encoder,
// the key-frame header, per-MB mode coding, the token partition and the RIFF
// container.  Plain C++ (no HIP): tests/test_vp8_host.py builds it with the scalar
// macroblock reference (tools/vp8_cpu_check.cpp) to check the bitstream against
// libwebp's decoder without a GPU.
#include "ik_vp8_enc.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace ik {
namespace vp8 {
namespace {

constexpr size_t kPackHeader = 16;
constexpr uint32_t kPackMagicHost = 0x4b503856u;  // ik_vp8_gpu.h kPackMagic

// RFC 6386 section 7.3 boolean encoder, normalising a whole shift at a time.
// `range` holds range-1 (the split is then (range*prob)>>8); bytes whose value is
// 0xff are held back as a run until the next byte settles whether a carry
// ripples through them.
struct BoolEnc {
    std::vector<uint8_t> out;
    int32_t range = 254, value = 0;
    int nb_bits = -8, run = 0;
    void emit() {
        const int s = 8 + nb_bits;
        const int32_t bits = value >> s;
        value -= bits << s;
        nb_bits -= 8;
        if ((bits & 0xff) != 0xff) {
            if ((bits & 0x100) && !out.empty()) ++out.back();
            if (run) {
                out.insert(out.end(), (size_t)run, (bits & 0x100) ? 0x00 : 0xff);
                run = 0;
            }
            out.push_back((uint8_t)bits);
        } else {
            ++run;
        }
    }
    inline void put(int bit, int prob) {  // branch-free but for the byte emit
        const int32_t split = (range * prob) >> 8;
        value += (split + 1) & -bit;
        range = bit ? range - (split + 1) : split;
        // renormalise: shift so that range+1 >= 128 (shift 0 when it already is)
        const int shift = __builtin_clz((uint32_t)range + 1) - 24;
        range = ((range + 1) << shift) - 1;
        value <<= shift;
        nb_bits += shift;
        if (nb_bits > 0) emit();
    }
    void literal(int v, int n) {
        for (int i = n - 1; i >= 0; --i) put((v >> i) & 1, 128);
    }
    void flush() {  // pad with zero bits until every coded bit is in a byte
        const int pad = 9 - nb_bits;
        for (int i = 0; i < pad; ++i) put(0, 128);
        nb_bits = 0;
        emit();
    }
};

// Recorded token decisions: bit 15 = the bit, bits 0..10 = index into a 1312-entry
// probability table: 0..1055 the adapted node probabilities, 1056 + p the fixed
// probability p (extra bits, sign).
// Pass 1 builds this and the node counts in one walk of the residuals; the coding
// pass then only runs the boolean coder over it.
struct TokenSink {
    std::vector<uint16_t> toks;
    uint16_t* w = nullptr;            // write cursor into toks
    uint32_t (*counts)[2] = nullptr;  // [1056][2]
    // room for one more macroblock: 25 blocks x 16 coefficients x <= 24 decisions
    void reserve_mb() {
        const size_t used = w ? (size_t)(w - toks.data()) : 0, need = used + 25 * 16 * 24;
        if (toks.size() < need) {
            toks.resize(need * 2);
        }
        w = toks.data() + used;
    }
    size_t size() const { return (size_t)(w - toks.data()); }
    std::vector<size_t> row_end;  // token count at the end of each MB row
    inline void node(int idx, int b) {
        ++counts[idx][b];
        *w++ = (uint16_t)(idx | (b << 15));
    }
    inline void fixed(int prob, int b) { *w++ = (uint16_t)((1056 + prob) | (b << 15)); }
};

}  // namespace

int last_nz(const int16_t* lv, int first) {
    for (int n = 15; n >= first; --n)
        if (lv[n]) return n + 1;
    return first;
}

namespace {

// one block's tokens (libwebp GetCoeffs in reverse) from its compact form (u16
// nonzero mask + the nonzero levels; null = all zero); returns nz (any nonzero
// level at or after `first`)
int write_block(TokenSink& s, const uint8_t* blk, int first, int ctx, int type) {
    uint32_t cm = 0;
    const uint8_t* v = nullptr;
    if (blk) {
        uint16_t c;
        std::memcpy(&c, blk, 2);
        cm = c;
        v = blk + 2 + 2 * __builtin_popcount(cm & ((1u << first) - 1));  // levels before `first` are not coded
        cm &= ~((1u << first) - 1);
    }
    int n = first;
    auto base = [&](int nn, int c) { return ((type * 8 + band(nn)) * 3 + c) * 11; };
    int b = base(n, ctx);
    if (!cm) {
        s.node(b + 0, 0);
        return 0;
    }
    const int last = 32 - __builtin_clz(cm);
    for (;;) {
        s.node(b + 0, 1);
        while (!((cm >> n) & 1)) {
            s.node(b + 1, 0);
            ++n;
            b = base(n, 0);
        }
        s.node(b + 1, 1);
        int16_t lvn;
        std::memcpy(&lvn, v, 2);
        v += 2;
        const int val = lvn < 0 ? -lvn : lvn;
        int nctx;
        if (val == 1) {
            s.node(b + 2, 0);
            nctx = 1;
        } else {
            s.node(b + 2, 1);
            if (val <= 4) {
                s.node(b + 3, 0);
                if (val == 2) s.node(b + 4, 0);
                else { s.node(b + 4, 1); s.node(b + 5, val == 4); }
            } else if (val <= 10) {
                s.node(b + 3, 1);
                s.node(b + 6, 0);
                if (val <= 6) {
                    s.node(b + 7, 0);
                    s.fixed(159, val - 5);
                } else {
                    s.node(b + 7, 1);
                    s.fixed(165, (val - 7) >> 1);
                    s.fixed(145, (val - 7) & 1);
                }
            } else {
                s.node(b + 3, 1);
                s.node(b + 6, 1);
                static const uint8_t kCat3[] = {173, 148, 140, 0};
                static const uint8_t kCat4[] = {176, 155, 140, 135, 0};
                static const uint8_t kCat5[] = {180, 157, 141, 134, 130, 0};
                static const uint8_t kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};
                static const uint8_t* const kCat[4] = {kCat3, kCat4, kCat5, kCat6};
                const int cat = val <= 18 ? 0 : (val <= 34 ? 1 : (val <= 66 ? 2 : 3));
                s.node(b + 8, cat >> 1);
                s.node(b + 9 + (cat >> 1), cat & 1);
                const int extra = val - (3 + (8 << cat));
                const int nb = cat == 3 ? 11 : 3 + cat;
                for (int i = 0; i < nb; ++i) s.fixed(kCat[cat][i], (extra >> (nb - 1 - i)) & 1);
            }
            nctx = 2;
        }
        s.fixed(128, lvn < 0);  // sign
        ++n;
        if (n == 16) return 1;
        b = base(n, nctx);
        if (n >= last) {
            s.node(b + 0, 0);
            return 1;
        }
    }
}

// One MB of a compact stream (layout in ik_vp8_gpu.h): modes, and per block a
// pointer to its u16 coefficient mask + nonzero levels (null: all zero).
struct PackedMB {
    uint8_t ymode, uvmode, skip;
    const uint8_t* bmodes;  // 16 (B_PRED only)
    const uint8_t* blk[25];
};

// parse the record at p (bounded by end); returns the next record or null
const uint8_t* parse_mb(const uint8_t* p, const uint8_t* end, PackedMB& m) {
    if (end - p < 8) return nullptr;
    m.ymode = p[0];
    m.uvmode = p[1];
    m.skip = p[2];
    uint32_t nzmask;
    std::memcpy(&nzmask, p + 4, 4);
    p += 8;
    m.bmodes = nullptr;
    if (m.ymode == B_PRED) {
        if (end - p < 16) return nullptr;
        m.bmodes = p;
        p += 16;
    }
    for (int b = 0; b < 25; ++b) {
        m.blk[b] = nullptr;
        if (!((nzmask >> b) & 1)) continue;
        if (end - p < 2) return nullptr;
        uint16_t cm;
        std::memcpy(&cm, p, 2);
        const long n = 2 + 2 * __builtin_popcount(cm);
        if (end - p < n) return nullptr;
        m.blk[b] = p;
        p += n;
    }
    return p;
}

// all residual tokens of the frame, with the decoder's non-zero contexts
void write_tokens(TokenSink& s, int mb_w, int mb_h, const uint8_t* const* recs, const uint8_t* end, bool use_skip) {
    std::vector<uint8_t> top((size_t)mb_w * 9, 0);
    PackedMB m;
    for (int my = 0; my < mb_h; ++my) {
        uint8_t left[9] = {0};
        for (int mx = 0; mx < mb_w; ++mx) {
            parse_mb(recs[(size_t)my * mb_w + mx], end, m);  // validated by index_records
            uint8_t* t = &top[(size_t)mx * 9];
            const bool i4 = m.ymode == B_PRED;
            s.reserve_mb();
            if (use_skip && m.skip) {
                for (int i = 0; i < 8; ++i) t[i] = left[i] = 0;
                if (!i4) t[8] = left[8] = 0;
                continue;
            }
            int first = 0, ytype = 3;
            if (!i4) {
                const int nz = write_block(s, m.blk[24], 0, t[8] + left[8], 1);
                t[8] = left[8] = (uint8_t)nz;
                first = 1;
                ytype = 0;
            }
            for (int y = 0; y < 4; ++y)
                for (int x = 0; x < 4; ++x) {
                    const int nz = write_block(s, m.blk[y * 4 + x], first, t[x] + left[y], ytype);
                    t[x] = left[y] = (uint8_t)nz;
                }
            for (int ch = 0; ch < 2; ++ch)
                for (int y = 0; y < 2; ++y)
                    for (int x = 0; x < 2; ++x) {
                        const int nz = write_block(s, m.blk[16 + 4 * ch + y * 2 + x], 0,
                                                   t[4 + 2 * ch + x] + left[4 + 2 * ch + y], 2);
                        t[4 + 2 * ch + x] = left[4 + 2 * ch + y] = (uint8_t)nz;
                    }
        }
        s.row_end.push_back(s.size());
    }
}

// Code the token streams (the first partition, then the token partitions: MB row
// r -> partition r % K) with their boolean coders interleaved: each coder is one
// long dependency chain, so several side by side keep the core busy.  Streams
// are taken shortest first: positions [from, to) run on the A that are still
// that long.
struct Strm {
    const uint16_t* p;
    size_t n;
    BoolEnc* e;
};

template <int A>
void code_span(const Strm* st, size_t from, size_t to, const uint8_t* ptab) {
    BoolEnc e[A];  // coder state in locals (registers) for the span
    const uint16_t* p[A];
    for (int k = 0; k < A; ++k) { e[k] = std::move(*st[k].e); p[k] = st[k].p; }
    for (size_t i = from; i < to; ++i)
#pragma GCC unroll 8
        for (int k = 0; k < A; ++k) e[k].put(p[k][i] >> 15, ptab[p[k][i] & 0x7ff]);
    for (int k = 0; k < A; ++k) *st[k].e = std::move(e[k]);
}

void code_streams(Strm* st, int S, const uint8_t* ptab) {
    std::sort(st, st + S, [](const Strm& a, const Strm& b) { return a.n < b.n; });
    size_t done = 0;
    for (int j = 0; j < S; ++j) {
        const int A = S - j;
        const size_t to = st[j].n;
        if (to > done) {
            switch (A) {
            case 5: code_span<5>(st + j, done, to, ptab); break;
            case 4: code_span<4>(st + j, done, to, ptab); break;
            case 3: code_span<3>(st + j, done, to, ptab); break;
            case 2: code_span<2>(st + j, done, to, ptab); break;
            default: code_span<1>(st + j, done, to, ptab); break;
            }
            done = to;
        }
    }
}

// records first-partition decisions as fixed-probability tokens, so the header
// is coded side by side with the token partitions
struct RecEnc {
    std::vector<uint16_t> toks;
    void put(int bit, int prob) { toks.push_back((uint16_t)((1056 + prob) | (bit << 15))); }
    void literal(int v, int n) {
        for (int i = n - 1; i >= 0; --i) put((v >> i) & 1, 128);
    }
};

template <class E>
void put_bmode(E& e, int mode, int top, int left) {
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

void pack_mbs(const MBOut* mbs, size_t nmb, std::vector<uint8_t>& out) {
    out.assign(kPackHeader, 0);
    for (size_t i = 0; i < nmb; ++i) {
        const MBOut& o = mbs[i];
        uint32_t nzmask = 0;
        for (int b = 0; b < 25; ++b)
            for (int n = 0; n < 16; ++n)
                if (o.lv[b][n]) nzmask |= 1u << b;
        const uint8_t hdr[4] = {o.ymode, o.uvmode, o.skip, 0};
        out.insert(out.end(), hdr, hdr + 4);
        out.insert(out.end(), (const uint8_t*)&nzmask, (const uint8_t*)&nzmask + 4);
        if (o.ymode == B_PRED) out.insert(out.end(), o.bmodes, o.bmodes + 16);
        for (int b = 0; b < 25; ++b) {
            if (!((nzmask >> b) & 1)) continue;
            uint16_t cm = 0;
            for (int n = 0; n < 16; ++n) cm |= (uint16_t)((o.lv[b][n] != 0) << n);
            out.insert(out.end(), (const uint8_t*)&cm, (const uint8_t*)&cm + 2);
            for (int n = 0; n < 16; ++n)
                if (o.lv[b][n]) out.insert(out.end(), (const uint8_t*)&o.lv[b][n], (const uint8_t*)&o.lv[b][n] + 2);
        }
    }
    const uint32_t h[4] = {(uint32_t)out.size(), (uint32_t)nmb, kPackMagicHost, 0};
    std::memcpy(out.data(), h, sizeof(h));
}

QParams qparams_for_quality(float quality) { return make_qparams(quality_to_qindex(quality), -2); }

bool write_webp_packed(int width, int height, const QParams& q, const uint8_t* pack, size_t cap, int filter_level,
                       std::vector<uint8_t>& out) {
    const int mb_w = (width + 15) >> 4, mb_h = (height + 15) >> 4;
    const size_t nmb = (size_t)mb_w * mb_h;
    // 0. the records: validate the stream once, keep each MB's start
    uint32_t hdr[4];
    if (cap < sizeof(hdr)) return false;
    std::memcpy(hdr, pack, sizeof(hdr));
    if (hdr[2] != kPackMagicHost || hdr[1] != nmb || hdr[0] > cap || hdr[0] < sizeof(hdr)) return false;
    const uint8_t* end = pack + hdr[0];
    static thread_local std::vector<const uint8_t*> recs;
    recs.resize(nmb);
    size_t nskip = 0;
    {
        const uint8_t* r = pack + sizeof(hdr);
        PackedMB m;
        for (size_t i = 0; i < nmb; ++i) {
            recs[i] = r;
            r = parse_mb(r, end, m);
            if (!r) return false;
            // y: DC/TM/V/H (0..3) or B_PRED; uv: DC/TM/V/H
            if ((m.ymode > 3 && m.ymode != B_PRED) || m.uvmode > 3) return false;
            if (m.bmodes)
                for (int b = 0; b < 16; ++b)
                    if (m.bmodes[b] >= NUM_BMODES) return false;
            nskip += m.skip;
        }
        if (r != end) return false;
    }
    // 1. token statistics under the frame's structure -> adapted probabilities
    std::vector<uint32_t> cnt(1056 * 2, 0);
    const bool use_skip = nskip > 0;
    uint8_t probs[1056];
    std::memcpy(probs, kCoeffProbs0, sizeof(probs));
    TokenSink s;
    s.counts = reinterpret_cast<uint32_t(*)[2]>(cnt.data());
    s.toks.resize(nmb * 128);
    s.w = s.toks.data();
    write_tokens(s, mb_w, mb_h, recs.data(), end, use_skip);
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
    // 2. first partition: header + per-MB modes (recorded, coded in step 3)
    RecEnc h;
    h.literal(0, 1);  // color_space
    h.literal(0, 1);  // clamping_type
    h.literal(0, 1);  // segmentation_enabled
    h.literal(0, 1);  // filter_type: normal
    h.literal(filter_level < 0 ? q.filter_level : filter_level, 6);
    h.literal(0, 3);  // sharpness
    h.literal(0, 1);  // loop_filter_adj_enable
    // token partitions: 4 (2, 1 for frames of fewer MB rows)
    const int log2k = mb_h >= 4 ? 2 : (mb_h >= 2 ? 1 : 0), K = 1 << log2k;
    h.literal(log2k, 2);
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
            PackedMB m;
            parse_mb(recs[(size_t)my * mb_w + mx], end, m);
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
    // 3. the first partition and the token partitions, coded together
    std::vector<uint16_t> part[5];
    part[0].swap(h.toks);
    for (int r = 0; r < mb_h; ++r) {
        const size_t b0 = r ? s.row_end[r - 1] : 0, b1 = s.row_end[r];
        part[1 + r % K].insert(part[1 + r % K].end(), s.toks.data() + b0, s.toks.data() + b1);
    }
    BoolEnc t[5];
    for (int k = 0; k <= K; ++k) t[k].out.reserve(part[k].size() / 4 + 64);
    uint8_t ptab[1056 + 256];
    std::memcpy(ptab, probs, 1056);
    for (int i = 0; i < 256; ++i) ptab[1056 + i] = (uint8_t)i;
    Strm st[5];
    for (int k = 0; k <= K; ++k) st[k] = Strm{part[k].data(), part[k].size(), &t[k]};
    code_streams(st, K + 1, ptab);
    for (int k = 0; k <= K; ++k) t[k].flush();
    // 4. frame + container
    std::vector<uint8_t> vp8;
    const uint32_t first = (uint32_t)t[0].out.size();
    const uint32_t tag = 0u | (0u << 1) | (1u << 4) | (first << 5);  // key frame, v0, shown
    vp8.push_back((uint8_t)tag); vp8.push_back((uint8_t)(tag >> 8)); vp8.push_back((uint8_t)(tag >> 16));
    vp8.push_back(0x9d); vp8.push_back(0x01); vp8.push_back(0x2a);
    vp8.push_back((uint8_t)width); vp8.push_back((uint8_t)(width >> 8));
    vp8.push_back((uint8_t)height); vp8.push_back((uint8_t)(height >> 8));
    vp8.insert(vp8.end(), t[0].out.begin(), t[0].out.end());
    for (int k = 1; k < K; ++k) {  // sizes of all token partitions but the last, 3 bytes LE
        const uint32_t sz = (uint32_t)t[k].out.size();
        vp8.push_back((uint8_t)sz); vp8.push_back((uint8_t)(sz >> 8)); vp8.push_back((uint8_t)(sz >> 16));
    }
    for (int k = 1; k <= K; ++k) vp8.insert(vp8.end(), t[k].out.begin(), t[k].out.end());
    const uint32_t vsize = (uint32_t)vp8.size(), pad = vsize & 1;
    out.clear();
    out.reserve(20 + vsize + pad);
    out.insert(out.end(), {'R', 'I', 'F', 'F'});
    le32(out, 4 + 8 + vsize + pad);
    out.insert(out.end(), {'W', 'E', 'B', 'P', 'V', 'P', '8', ' '});
    le32(out, vsize);
    out.insert(out.end(), vp8.begin(), vp8.end());
    if (pad) out.push_back(0);
    return true;
}

void write_webp(int width, int height, const QParams& q, const MBOut* mbs, int filter_level,
                std::vector<uint8_t>& out) {
    const size_t nmb = (size_t)((width + 15) >> 4) * ((height + 15) >> 4);
    std::vector<uint8_t> pack;
    pack_mbs(mbs, nmb, pack);
    write_webp_packed(width, height, q, pack.data(), pack.size(), filter_level, out);
}

}  // namespace vp8
}  // namespace ik
