// ik_png_wave.h -- block-parallel DEFLATE decoding of one decoder lane by a whole
// wave (the GPU PNG decoder's decode pass, ik_png.hip k_png_wave; its CPU model is
// ik_png_model.cpp ikm_inflate_wave, CPU tests only).
//
// decode_image on a PNG (reference src/transform.rs:31 -> image 0.25.8 -> png 0.18)
// is zlib inflate of the IDAT stream.  ik_inflate.h cuts the stream into decoder
// lanes at block-start candidates (k_png_find) and verifies them by the chain
// check; a lane is whole DEFLATE blocks from a verified start up to the next
// candidate.  Here a lane is decoded by 64 sub-lanes at once:
//
//  * The block's Huffman codes go into lookup tables shared by the wave (LDS):
//    literal/length kLB = 10 bits (an entry holds one symbol, or two literals
//    whose codes fit the 10 bits together), distance kDB = 8 bits; longer codes
//    take a canonical decode from the code-length limits (rare).
//  * The block's body [p, range end) is split into 64 sub-ranges of an odd number
//    of 32-bit words (so the sub-lanes' reads of the staged window spread over the
//    LDS banks).  Sub-lane 0 starts on the body's first symbol.  Sub-lane j > 0
//    starts kWarmBits before its range on a guessed boundary and decodes (the
//    warm-up: Huffman codes resynchronise within a few symbols); its first symbol
//    boundary at or past its range start is START_j, the first at or past its
//    range end EXIT_j.  It writes its tokens (raw literal bytes, matches) into its
//    own piece of the lane's token region from START_j on.
//  * Fix rounds: a sub-lane whose START differs from its predecessor's EXIT
//    decodes again from that EXIT, until none differs (sub-lane 0 is exact, so the
//    chain is right from the left).  A verified end-of-block ends the block: the
//    next block's header is parsed there and the loop goes on, until a block
//    boundary at or past the lane's stop (ik_inflate.h decode_lane semantics:
//    exact hit = kLaneOk, passing it or a final block before it = kLaneMismatch).
//
// Token format (ik_inflate.h): 0x4000 | byte (a literal), 0x8000 | (len - 3) then
// dist - 1 (a match), 0xFFFE padding (no symbol: pieces are padded to 8 tokens).
// The expand pass reads a lane's pieces in order (PieceTab).
#pragma once
#include <stdint.h>

#include "ik_inflate.h"

namespace ik {
namespace wave {

// IK_KEEP(x, y): on the GPU, x and y are computed on every path here (an empty
// volatile asm uses them), so the selects after it stay selects -- the compiler
// would otherwise sink an arm's arithmetic into a branch of its own, and a wave
// whose sub-lanes take both arms runs both with exec-mask bookkeeping around them.
#if defined(__HIP_DEVICE_COMPILE__)
#define IK_KEEP(x, y) asm volatile("" ::"v"(x), "v"(y))
#else
#define IK_KEEP(x, y) ((void)0)
#endif

constexpr int kLB = 10;                 // literal/length table bits
constexpr int kDB = 8;                  // distance table bits
constexpr uint32_t kLM = (1u << kLB) - 1u, kDM = (1u << kDB) - 1u;
constexpr int kSub = 64;                // sub-lanes (one wave)
constexpr int kWarmBits = 256;          // warm-up before a guessed sub-range start
constexpr int kMinSubBits = 512;        // fewer sub-lanes for shorter ranges
// stream bits of one window of a block's body (LDS staging): 12 KiB keeps the
// wave's LDS at ~20 KB (8 waves per CU) at ~8 % more sub-lane steps than a
// window holding a whole ~18 KB block
constexpr uint64_t kWindowBits = 8ull * 12288;

// literal/length entry (u32):
//   bits 0..4   bits consumed by the entry's symbols (0: slow / invalid)
//   bits 5..6   kind: 0 literal(s), 1 length, 2 end of block, 3 slow (code longer than kLB, or invalid)
//   bit 7       two literals
//   bits 8..15  first literal          | length: extra bits (8..10)
//   bits 16..23 second literal         | length: base - 3
//   bits 24..27 the first symbol's code length
enum { kKLit = 0, kKLen = 1, kKEob = 2, kKSlow = 3 };
IK_HD uint32_t e_bits(uint32_t e) { return e & 31u; }
IK_HD uint32_t e_kind(uint32_t e) { return (e >> 5) & 3u; }
IK_HD bool e_two(uint32_t e) { return (e >> 7) & 1u; }
IK_HD uint32_t e_lit1(uint32_t e) { return (e >> 8) & 255u; }
IK_HD uint32_t e_lit2(uint32_t e) { return (e >> 16) & 255u; }
IK_HD uint32_t e_len1(uint32_t e) { return (e >> 24) & 15u; }
IK_HD uint32_t e_lextra(uint32_t e) { return (e >> 8) & 7u; }
IK_HD uint32_t e_lbase(uint32_t e) { return ((e >> 16) & 255u) + 3u; }
IK_HD uint32_t mk_lit(uint32_t L, uint32_t b) { return L | ((uint32_t)kKLit << 5) | (b << 8) | (L << 24); }
IK_HD uint32_t mk_lit2(uint32_t L1, uint32_t b1, uint32_t L2, uint32_t b2) {
    return (L1 + L2) | ((uint32_t)kKLit << 5) | (1u << 7) | (b1 << 8) | (b2 << 16) | (L1 << 24);
}
IK_HD uint32_t mk_len(uint32_t L, uint32_t base, uint32_t extra) {
    return L | ((uint32_t)kKLen << 5) | (extra << 8) | ((base - 3u) << 16) | (L << 24);
}
IK_HD uint32_t mk_eob(uint32_t L) { return L | ((uint32_t)kKEob << 5) | (L << 24); }
constexpr uint32_t kSlowEntry = (uint32_t)kKSlow << 5;

// distance entry (u32): bits 0..4 code length (0: slow / invalid), bit 5 slow,
// bits 8..11 extra bits, bits 16..31 base distance
IK_HD uint32_t d_len(uint32_t d) { return d & 31u; }
IK_HD bool d_slow(uint32_t d) { return (d >> 5) & 1u; }
IK_HD uint32_t d_extra(uint32_t d) { return (d >> 8) & 15u; }
IK_HD uint32_t d_base(uint32_t d) { return d >> 16; }
IK_HD uint32_t mk_dist(uint32_t D, uint32_t base, uint32_t extra) { return D | (extra << 8) | (base << 16); }
constexpr uint32_t kSlowDist = 1u << 5;

// One canonical code: the left-justified limits packed for infl::canon_len, and
// per length L (1..15) the first code (15 bits) | the rank of its first symbol << 16.
struct Code {
    uint32_t pk[8];
    uint32_t info[16];
};

// Build a code from lengths lens[0..n) (lengths <= 15).  syms (n entries): the
// symbols in canonical order (length, then value).  Returns 0, or -1 if the code
// is oversubscribed, or incomplete where DEFLATE (zlib) does not allow it (a
// dynamic literal/length code must be complete or a single code of length 1, a
// distance code may also be empty; `fixed`: the fixed codes, not checked).
// Serial (the GPU runs it on one lane).
template <class Lens, class Syms>
IK_HD int code_build(const Lens& lens, int n, bool is_dist, Code& C, Syms syms, bool fixed = false) {
    uint32_t cnt[16];
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int s = 0; s < n; ++s) cnt[lens[s] & 15u]++;
    int maxl = 0;
    for (int l = 15; l >= 1; --l)
        if (cnt[l]) { maxl = l; break; }
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left = (left << 1) - (int)cnt[l];
        if (left < 0) return -1;
    }
    if (fixed) {
        // the fixed codes (RFC 1951 3.2.6): the distance code uses 30 of its 32 codes
    } else if (maxl == 0) {
        if (!is_dist) return -1;
    } else if (left > 0 && maxl != 1) {
        return -1;  // incomplete (zlib accepts only a single length-1 code)
    }
    uint32_t lim[15], off[16], code = 0, rank = 0;
    off[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + (l > 1 ? cnt[l - 1] : 0u)) << 1;
        C.info[l] = (code & 0x7FFFu) | (rank << 16);
        lim[l - 1] = (code + cnt[l]) << (15 - l);
        off[l] = rank;
        rank += cnt[l];
    }
    C.info[0] = 0;
    infl::pack_limits(lim, C.pk);
    uint32_t pos[16];
    for (int l = 0; l < 16; ++l) pos[l] = off[l];
    for (int s = 0; s < n; ++s) {
        const uint32_t l = lens[s] & 15u;
        if (l) syms[pos[l]++] = (uint16_t)s;
    }
    return 0;
}

// canonical decode of the next 15 stream bits (v: bit 0 = the next bit): symbol and
// code length L, or L > 15 for no code
template <class CodeT, class Syms>
IK_HD int canon_sym(uint32_t v15, const CodeT& C, const Syms& syms, int& L) {
    const uint32_t c15 = infl::rev32(v15) >> 17;
    L = infl::canon_len(c15, C.pk);
    if (L > 15) return -1;
    const uint32_t inf = C.info[L];
    return (int)syms[(inf >> 16) + (c15 >> (15 - L)) - (inf & 0x7FFFu)];
}

// the entry of a symbol decoded from a code of length L (literal/length code)
IK_HD uint32_t lit_symbol_entry(int sym, uint32_t L) {
    if (sym < 256) return mk_lit(L, (uint32_t)sym);
    if (sym == 256) return mk_eob(L);
    if (sym > 285) return kSlowEntry;  // 286 / 287 (fixed code): invalid
    int base, extra;
    infl::len_code(sym - 257, base, extra);
    return mk_len(L, (uint32_t)base, (uint32_t)extra);
}
IK_HD uint32_t dist_symbol_entry(int sym, uint32_t D) {
    if (sym > 29) return kSlowDist;  // 30 / 31: invalid
    int base, extra;
    infl::dist_code(sym, base, extra);
    return mk_dist(D, (uint32_t)base, (uint32_t)extra);
}

// table entry e (the next kLB stream bits, bit 0 first)
template <class CodeT, class Syms>
IK_HD uint32_t lit_table_entry(uint32_t e, const CodeT& C, const Syms& syms) {
    int L;
    const int s = canon_sym(e, C, syms, L);  // (bits past kLB read as zero: a code longer than kLB shows L > kLB)
    if (L > kLB || s < 0) return kSlowEntry;
    if (s < 256 && L < kLB) {
        const uint32_t r = (uint32_t)(kLB - L);
        const uint32_t e2 = (e >> L) & ((1u << r) - 1u);
        int L2;
        const int s2 = canon_sym(e2, C, syms, L2);
        if (s2 >= 0 && s2 < 256 && L2 <= (int)r) return mk_lit2((uint32_t)L, (uint32_t)s, (uint32_t)L2, (uint32_t)s2);
    }
    return lit_symbol_entry(s, (uint32_t)L);
}
template <class CodeT, class Syms>
IK_HD uint32_t dist_table_entry(uint32_t e, const CodeT& C, const Syms& syms) {
    int D;
    const int s = canon_sym(e, C, syms, D);
    if (D > kDB || s < 0) return kSlowDist;
    return dist_symbol_entry(s, (uint32_t)D);
}

// the slow path: the symbol at the next 15 bits by the canonical decode (entries
// of the same format, one symbol; kSlowEntry / kSlowDist = no code: invalid)
template <class Syms>
IK_HD uint32_t lit_slow(uint64_t v, const Code& C, const Syms& syms) {
    int L;
    const int s = canon_sym((uint32_t)v & 0x7FFFu, C, syms, L);
    if (s < 0) return kSlowEntry;
    return lit_symbol_entry(s, (uint32_t)L);
}
template <class Syms>
IK_HD uint32_t dist_slow(uint64_t v, const Code& C, const Syms& syms) {
    int D;
    const int s = canon_sym((uint32_t)v & 0x7FFFu, C, syms, D);
    if (s < 0) return kSlowDist;
    return dist_symbol_entry(s, (uint32_t)D);
}

// Token output of one sub-lane: tokens go to p[0 .. cap) in groups of 8 (one
// 16-byte store each); the last group is padded with kTokPad.  put4 takes up to
// four tokens at once (a step's output).  The host form writes straight to p; the
// GPU's (ik_png.hip WaveOut) stages the open group in LDS.
struct SubOutHost {
    uint16_t* p;
    uint32_t cap;        // tokens (a multiple of 8)
    uint32_t n = 0;      // tokens put
    uint8_t* marks = nullptr;  // the model's step profile: flags per step (sub_decode's out.mark)
    uint32_t nmarks = 0;
    IK_HD void reset() { n = 0; }
    IK_HD void mark(uint32_t step, uint32_t f) {
        if (marks && step - 1 < nmarks) marks[step - 1] |= (uint8_t)f;
    }
    IK_HD void put4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        const uint32_t t[4] = {a, b, c, d};
        for (uint32_t i = 0; i < k; ++i) {
            if (n < cap) p[n] = (uint16_t)t[i];
            ++n;
        }
    }
    IK_HD void finish() {
        for (uint32_t i = n; i < ((n + 7u) & ~7u); ++i)
            if (i < cap) p[i] = (uint16_t)infl::kTokPad;
    }
};

// Result of one sub-lane pass (positions relative to the window's base bit).
struct SubRes {
    uint32_t start;   // first symbol boundary >= the range start (or where an exact start began)
    uint32_t exit;    // first symbol boundary >= the range end, or just past a verified end of block
    uint32_t out;     // output bytes from start to exit
    uint32_t ntok;    // tokens written
    int eob;          // an end-of-block code ended the pass (exit = just past it)
    int bad;          // an invalid code inside the range (corrupt, or an unsynchronised start)
    int over;         // the token region was too small
    uint32_t steps;   // loop iterations (profile)
};

// Decode one sub-lane.  Positions are bits relative to the window's base (32-bit
// arithmetic on the step's chain).  From bit p0 (a guessed boundary, or the exact
// one when p0 >= lo), symbols before `lo` are the warm-up (no output; invalid codes skip a
// bit, end-of-block codes are stepped over); from the first boundary >= lo (START)
// tokens go out until the first boundary >= hi (EXIT) or an end-of-block code.
// win(pos) = the 64 stream bits from pos (positions only grow, by at most 48 bits a
// step, after win.init(p0)); lit / dist = the shared tables; C / syms
// = the codes (the slow path).  One step decodes up to four literals (two table
// entries of one or two each) or one match; both are computed and selected, so
// the lanes of a wave stay together except on the rare slow codes.
template <class Win, class LitTab, class DistTab, class LSyms, class DSyms, class Out>
IK_HD void sub_decode(Win& win, uint32_t p0, uint32_t lo, uint32_t hi, const LitTab& lit, const DistTab& dist,
                      const Code& LC, const LSyms& lsyms, const Code& DC, const DSyms& dsyms, Out& out,
                      SubRes& r) {
    uint32_t pos = p0;
    win.init(p0);  // (the GPU's cursor keeps the stream bits around pos in registers)
    // START is the first boundary at or past lo: positions only grow, so a step is
    // past START iff pos >= lo.  The step's control is bitwise (no short-circuit
    // branches: on the GPU a wave's 64 sub-lanes take one path); the loop's only
    // exits are the range end and a verified end-of-block / invalid code.
    r.start = p0 >= lo ? p0 : ~0u;
    r.eob = 0;
    r.bad = 0;
    out.reset();
    uint32_t cnt = 0;
    uint32_t steps = 0;
    bool stop = pos >= hi;
    while (!stop) {
        ++steps;
        const bool started = pos >= lo;
        r.start = (started & (r.start == ~0u)) ? pos : r.start;
        const uint32_t limit = started ? hi : lo;
        const uint64_t v = win(pos);
        uint32_t e1 = lit[(uint32_t)v & kLM];
        const bool slow1 = e_kind(e1) == kKSlow;
        if (slow1) e1 = lit_slow(v, LC, lsyms);
        const uint32_t k1 = e_kind(e1), n1 = e_bits(e1), L1 = e_len1(e1);
        // literals: e1's one or two, then the next entry's (each taken only while
        // it starts before the limit)
        const bool isl = k1 == kKLit;
        const bool two1 = e_two(e1) & (pos + L1 < limit);
        const uint32_t c1 = two1 ? n1 : L1;
        const uint32_t e2 = lit[(uint32_t)(v >> c1) & kLM];
        const bool lit2 = ((uint32_t)isl & ((uint32_t)two1 | (uint32_t)!e_two(e1)) & (uint32_t)(pos + c1 < limit) &
                           (uint32_t)(e_kind(e2) == kKLit)) != 0u;
        const uint32_t L2 = e_len1(e2);
        const bool two2 = lit2 & e_two(e2) & (pos + c1 + L2 < limit);
        const uint32_t c2 = lit2 ? (two2 ? e_bits(e2) : L2) : 0u;
        // a match (computed for every symbol, used for a length code)
        const uint32_t le = e_lextra(e1);
        const uint32_t ll = e_lbase(e1) + ((uint32_t)(v >> n1) & ((1u << le) - 1u));
        const uint64_t vd = v >> (n1 + le);
        uint32_t d = dist[(uint32_t)vd & kDM];
        const bool isn = k1 == kKLen;
        const bool slow2 = isn & d_slow(d);
        if (slow2) d = dist_slow(vd, DC, dsyms);
        const bool bad = (k1 == kKSlow) | (isn & d_slow(d));
        const uint32_t D = d_len(d), de = d_extra(d);
        const uint32_t dd = d_base(d) + ((uint32_t)(vd >> D) & ((1u << de) - 1u));
        IK_KEEP(ll, dd);
        const bool eob = k1 == kKEob;
        const bool fin = started & (bad | eob);  // the pass ends here (no tokens)
        // tokens: literals a b c d (two1 / lit2 / two2 say which), or the match's two
        const uint32_t t1 = isl ? infl::kTokRaw | e_lit1(e1) : infl::kTokMatch | (ll - 3u);
        const uint32_t t2l = infl::kTokRaw | (two1 ? e_lit2(e1) : e_lit1(e2)), t2m = dd - 1u;
        IK_KEEP(t2l, t2m);
        const uint32_t t2 = isl ? t2l : t2m;
        const uint32_t t3 = infl::kTokRaw | (two1 ? e_lit1(e2) : e_lit2(e2));
        const uint32_t t4 = infl::kTokRaw | e_lit2(e2);
        const uint32_t nl = 1u + (two1 ? 1u : 0u) + (lit2 ? 1u : 0u) + (two2 ? 1u : 0u);
        const bool emit = started & !fin;
        const uint32_t k = !emit ? 0u : isl ? nl : isn ? 2u : 0u;
        out.mark(steps, (slow1 ? 1u : 0u) | (slow2 ? 2u : 0u) | (((out.n + k) ^ out.n) & ~7u ? 4u : 0u) |
                            (isn ? 8u : 0u) | (!started ? 16u : 0u));
        out.put4(t1, t2, t3, t4, k);
        cnt += !emit ? 0u : isl ? nl : isn ? ll : 0u;
        // (warm-up: an invalid code skips a bit; a verified invalid code stays put)
        const uint32_t adv_l = c1 + c2, adv_n = n1 + le + D + de;
        IK_KEEP(adv_l, adv_n);
        const uint32_t adv = isl ? adv_l : isn ? adv_n : eob ? n1 : 1u;
        pos += (fin & bad) ? 0u : adv;
        r.eob = fin & eob;
        r.bad = fin & bad;
        stop = fin | (pos >= hi);
    }
    if (r.start == ~0u) r.start = pos;  // (the range was crossed in one step: START = EXIT)
    r.exit = pos;
    r.out = cnt;
    r.ntok = out.n;
    r.over = ((out.n + 7u) & ~7u) > out.cap;  // (the padded last group must fit too)
    r.steps = steps;
}

// One lane's pieces for the expand pass, entry k = (base, vstart): piece k is the
// tokens [base, base + n) of the lane's token region, n = vstart[k+1] - vstart[k]
// (the last: the lane's token count - vstart), a multiple of 8 (padding included);
// vstart = its first index in the lane's virtual token stream (the pieces in order).
// A lane's table holds pieces_capacity(bits) entries: about one per 512 stream
// bits (a sub-lane's least range) and per block.
IK_HD uint32_t pieces_capacity(uint64_t bits) {
    const uint64_t c = bits / 512 + 64;
    return (uint32_t)(c < (1u << 24) ? c : (1u << 24));
}

// A block window's split into sub-ranges: nsub sub-lanes of `lw` words (odd, so
// the sub-lanes' LDS words fall on different banks), the last one ending at re.
struct Split {
    int nsub;
    uint32_t lw;      // words per sub-range
    uint32_t cap;     // token capacity per sub-lane (a multiple of 8)
};
IK_HD Split split_range(uint64_t bp, uint64_t re, bool big) {
    const uint64_t bits = re > bp ? re - bp : 1;
    uint64_t ns = bits / kMinSubBits;
    ns = ns < 1 ? 1 : ns > (uint64_t)kSub ? (uint64_t)kSub : ns;
    uint64_t lw = (bits + 32 * ns - 1) / (32 * ns);
    lw |= 1u;
    ns = (bits + 32 * lw - 1) / (32 * lw);  // (the odd rounding may need fewer)
    Split s;
    s.nsub = (int)(ns < 1 ? 1 : ns);
    s.lw = (uint32_t)lw;
    // a token costs >= 1 bit (big); image data ~0.23 tokens per bit, more in a sub-range's
    // compressible stretches: 0.375 leaves room for those without a second round
    const uint64_t c = (big ? 32 * lw : 12 * lw) + 32;
    s.cap = (uint32_t)((c + 7) & ~7ull);
    return s;
}
// The end of a block window from bp: the staging limit, the lane's stop, and --
// for a block after the lane's first -- the block's estimated end (a block's end is
// found only by decoding it: sub-lanes past it decode for nothing).  zlib ends a
// block when its symbol buffer fills, so consecutive blocks of an image hold about
// as many bits: the estimate is the previous block's length + 4 Kbit, for every
// window of the block (a block longer than that takes one more window of at least
// 16 Kbit; the model's sweep on bench frames: shorter estimates cost more in extra
// windows than they save).
#if !defined(__HIP_DEVICE_COMPILE__)
inline int64_t g_est_mul = 1024, g_est_add = 4096, g_min_tail = 16384;  // (model experiments)
#endif
IK_HD uint64_t block_end_estimate(uint64_t body, uint64_t prev_bits) {
#if !defined(__HIP_DEVICE_COMPILE__)
    return prev_bits ? body + prev_bits * (uint64_t)g_est_mul / 1024 + (uint64_t)g_est_add : 0;
#else
    return prev_bits ? body + prev_bits + 4096 : 0;
#endif
}
IK_HD uint64_t window_end(uint64_t bp, uint64_t stop_eff, uint64_t est_end) {
    uint64_t re = bp + kWindowBits < stop_eff ? bp + kWindowBits : stop_eff;
    if (est_end) {
#if !defined(__HIP_DEVICE_COMPILE__)
        const uint64_t e = est_end > bp + (uint64_t)g_min_tail ? est_end : bp + (uint64_t)g_min_tail;
#else
        const uint64_t e = est_end > bp + 16384 ? est_end : bp + 16384;
#endif
        if (e < re) re = e;
    }
    return re;
}

// a wave lane's token region: every window's sub-lanes at their full capacity
// (a quarter token per bit, plus each window's rounding; `big`: a token per bit,
// the bound, for a lane whose region overflowed)
IK_HD uint64_t region_capacity(uint64_t bits, bool big) {
    const uint64_t slack = (bits / kWindowBits + 2) * 3072 + 64;
    const uint64_t c = big ? bits + 32ull * pieces_capacity(bits) + slack : bits / 8 * 3 + slack;
    return (c + 7) & ~7ull;  // (regions start 16-byte aligned: whole groups of 8 tokens)
}

// statistics of the CPU model (ikm_inflate_wave)
struct Stats {
    uint64_t windows = 0, sub_passes = 0, redo_passes = 0, fix_rounds = 0, max_rounds = 0;
    uint64_t symbols_bits = 0, blocks = 0, slow = 0, steps = 0;
    uint64_t wave_steps = 0;  // the wave's latency: per pass, its longest sub-lane's steps
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // first passes' wave steps with any sub-lane: slow literal,
                                                  // slow distance, group store, match, warm-up; all steps
};

// Expand units: the expand pass runs one wave per unit -- a run of a lane's whole
// blocks -- rather than per lane, so that a lane of many blocks (64 KiB of stream)
// expands with the parallelism of one-block lanes.  A block starts a new unit unless
// the lane's current unit holds fewer than kUnitMinTok tokens (short blocks share a
// unit).  Unit record k of a lane, at the lane's piece-table slot k (a lane has no
// more units than pieces): (its first piece, the lane's output bytes before it).
#ifndef IK_UNIT_MIN_TOK
#define IK_UNIT_MIN_TOK 16384
#endif
constexpr uint32_t kUnitMinTok = IK_UNIT_MIN_TOK;
IK_HD bool unit_starts(uint32_t nunits, uint64_t written, uint64_t unit_v0) {
    return nunits == 0 || written - unit_v0 >= kUnitMinTok;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// The lane algorithm on the host (the CPU model; ik_png.hip k_png_wave runs the
// same steps with the 64 sub-lanes in parallel).  words: the stream (zero padded
// past nbits); region: the lane's token region (cap tokens).  Fills r (end_bit,
// out_len, status, final_block, blocks) and pt.
template <class WinFn, class Pieces>
inline void lane_host(WinFn win, uint64_t nbits, uint64_t start, uint64_t stop, bool big, uint16_t* region,
                      uint64_t cap, infl::LaneResult& r, Pieces& pt, Pieces& units, Stats* stats,
                      uint64_t warm = kWarmBits) {
    const uint32_t pcap = pieces_capacity((stop == ~0ull ? nbits : stop) - start);
    const uint64_t stop_eff = stop == ~0ull ? nbits : stop;
    uint64_t p = start, used = 0, total = 0, written = 0;
    uint64_t prev_bits = 0;  // the last block's body length (window_end)
    r.status = infl::kLaneCorrupt;
    r.final_block = 0;
    r.blocks = 0;
    r.iters = 0;
    pt.clear();
    units.clear();
    uint64_t unit_v0 = 0;  // the current unit's first token (virtual index)
    uint32_t lit[1u << kLB], dist[1u << kDB];
    uint16_t lsyms[288], dsyms[32];
    Code LC, DC;
    for (;;) {
        if (p >= stop) {
            r.status = p == stop ? infl::kLaneOk : infl::kLaneMismatch;
            break;
        }
        if (p + 3 > nbits) break;
        // this block's start: a split goes back to it
        const uint64_t blk_start = p, blk_total = total, blk_used = used, blk_written = written;
        const uint32_t blk_pieces = (uint32_t)pt.size(), blk_units = (uint32_t)units.size();
        const uint64_t blk_v0 = unit_v0;
        if (unit_starts((uint32_t)units.size(), written, unit_v0)) {  // (undone with the block on a split)
            units.push_back({(uint32_t)pt.size(), (uint32_t)total});
            unit_v0 = written;
        }
        const uint64_t h = win(p);
        const int bfinal = (int)(h & 1u), btype = (int)((h >> 1) & 3u);
        ++r.blocks;
        if (stats) ++stats->blocks;
        if (btype == 3) break;
        if (btype == 0) {  // stored: one piece of raw tokens
            uint64_t q = (p + 3 + 7) & ~7ull;
            const uint64_t lh = win(q);
            const uint32_t len = (uint32_t)lh & 0xFFFFu, nlen = (uint32_t)(lh >> 16) & 0xFFFFu;
            if ((len ^ 0xFFFFu) != nlen) break;
            q += 32;
            if (q + 8ull * len > nbits) break;
            if (stop != ~0ull && q + 8ull * len > stop) {  // the block passes the lane's stop: no tokens needed
                p = q + 8ull * len;
                r.status = infl::kLaneMismatch;
                break;
            }
            const uint32_t n8 = (len + 7u) & ~7u;
            if (used + n8 > cap) { r.status = infl::kLaneOverflow; break; }
            if (pt.size() >= pcap) {
                units.resize(blk_units);  // (the split lane ends before this block)
                r.status = p > start ? (int)infl::kLaneSplit : (int)infl::kLaneOverflow;
                break;
            }
            for (uint32_t i = 0; i < n8; ++i)
                region[used + i] = i < len ? (uint16_t)(infl::kTokRaw | ((uint32_t)win(q + 8ull * i) & 255u))
                                           : (uint16_t)infl::kTokPad;
            pt.push_back({(uint32_t)used, (uint32_t)written});
            used += n8;
            written += n8;
            total += len;
            p = q + 8ull * len;
        } else {
            // the block's codes (ik_inflate.h parse_dynamic validates like zlib)
            uint8_t lens[288 + 32];
            int nlen, ndist;
            uint64_t body;
            if (btype == 2) {
                infl::Bits b;
                b.init(reinterpret_cast<const uint32_t*>(win.words), p + 3, (nbits >> 5) + 4);
                infl::CodeInfo lci, dci;
                if (infl::parse_dynamic(b, lens, nlen, ndist, lci, dci)) break;
                for (int i = ndist - 1; i >= 0; --i) lens[288 + i] = lens[nlen + i];
                body = b.pos();
            } else {
                infl::fixed_lens(lens);
                nlen = 288;
                ndist = 30;
                body = p + 3;
            }
            if (code_build(lens, nlen, false, LC, lsyms, btype == 1) ||
                code_build(lens + 288, ndist, true, DC, dsyms, btype == 1))
                break;
            for (uint32_t e = 0; e < (1u << kLB); ++e) lit[e] = lit_table_entry(e, LC, lsyms);
            for (uint32_t e = 0; e < (1u << kDB); ++e) dist[e] = dist_table_entry(e, DC, dsyms);
            // the body, window by window (LDS holds kWindowBits of stream on the GPU)
            uint64_t bp = body;
            const uint64_t est_end = block_end_estimate(body, prev_bits);
            int done = 0;  // 1: block ended (p updated), 2: lane ends (status set), 3: corrupt / overflow
            while (!done) {
                if (bp >= stop_eff) {  // the block runs past the lane's stop
                    r.status = stop == ~0ull ? infl::kLaneCorrupt : infl::kLaneMismatch;
                    done = 2;
                    break;
                }
                const uint64_t re = window_end(bp, stop_eff, est_end);
                const Split sp = split_range(bp, re, big);
                if (used + (uint64_t)sp.nsub * sp.cap > cap) { r.status = infl::kLaneOverflow; done = 3; break; }
                if (stats) ++stats->windows;
                SubRes sr[kSub];
                // positions relative to the window's first bit bp
                struct RelWin {
                    WinFn& w;
                    uint64_t base;
                    void init(uint32_t) {}
                    uint64_t operator()(uint32_t rel) const { return w(base + rel); }
                } rwin{win, bp};
                uint32_t lo[kSub + 1];
                for (int j = 0; j < sp.nsub; ++j) lo[j] = 32u * sp.lw * (uint32_t)j;
                lo[sp.nsub] = (uint32_t)(re - bp);
                uint32_t pass_max = 0;
                std::vector<uint8_t> wmarks(stats ? 4096 : 0, 0);
                for (int j = 0; j < sp.nsub; ++j) {
                    SubOutHost o{region + used + (uint64_t)j * sp.cap, sp.cap};
                    std::vector<uint8_t> sm(wmarks.size(), 0);
                    o.marks = sm.data();
                    o.nmarks = (uint32_t)sm.size();
                    const uint32_t p0 = j == 0 ? 0u : (lo[j] >= warm ? lo[j] - (uint32_t)warm : 0u);
                    sub_decode(rwin, p0, lo[j], lo[j + 1], lit, dist, LC, lsyms, DC, dsyms, o, sr[j]);
                    o.finish();
                    if (stats) { ++stats->sub_passes; stats->steps += sr[j].steps; }
                    pass_max = sr[j].steps > pass_max ? sr[j].steps : pass_max;
                    for (size_t q = 0; q < sm.size(); ++q) wmarks[q] |= sm[q];
                }
                if (stats) {
                    stats->wave_steps += pass_max;
                    for (uint32_t q = 0; q < pass_max && q < wmarks.size(); ++q)
                        for (int b = 0; b < 5; ++b) stats->prof[b] += (wmarks[q] >> b) & 1u;
                    stats->prof[7] += pass_max;
                }
                // fix rounds: a sub-lane whose start is not its predecessor's exit decodes
                // again from that exit (all such at once), until the chain holds
                int v = 0, rounds = 0;
                for (;;) {
                    v = 0;
                    while (v + 1 < sp.nsub && !sr[v].eob && !sr[v].bad && sr[v + 1].start == sr[v].exit) ++v;
                    if (sr[v].eob || sr[v].bad || v + 1 == sp.nsub) break;
                    ++rounds;
                    uint32_t ex[kSub];
                    bool redo[kSub];
                    for (int j = 0; j < sp.nsub; ++j) {
                        ex[j] = sr[j].exit;
                        redo[j] = j > v && !sr[j - 1].eob && !sr[j - 1].bad && sr[j].start != sr[j - 1].exit;
                    }
                    uint32_t redo_max = 0;
                    for (int j = v + 1; j < sp.nsub; ++j) {
                        if (!redo[j]) continue;
                        SubOutHost o{region + used + (uint64_t)j * sp.cap, sp.cap};
                        sub_decode(rwin, ex[j - 1], lo[j], lo[j + 1], lit, dist, LC, lsyms, DC, dsyms, o, sr[j]);
                        o.finish();
                        if (stats) { ++stats->redo_passes; stats->steps += sr[j].steps; }
                        redo_max = sr[j].steps > redo_max ? sr[j].steps : redo_max;
                    }
                    if (stats) stats->wave_steps += redo_max;
                }
                if (stats) {
                    stats->fix_rounds += (uint64_t)rounds;
                    if ((uint64_t)rounds > stats->max_rounds) stats->max_rounds = (uint64_t)rounds;
                }
                bool over = false;
                for (int j = 0; j <= v; ++j) over = over || sr[j].over;
                if (over) {
                    r.status = infl::kLaneOverflow;
                    done = 3;
                    break;
                }
                if (pt.size() + (size_t)(v + 1) > pcap) {
                    // no room for this window's pieces: the lane ends at the block's start
                    // (whole blocks so far) and the chain check starts a new lane there
                    r.status = blk_start > start ? (int)infl::kLaneSplit : (int)infl::kLaneOverflow;
                    done = 4;
                    break;
                }
#ifdef IKM_WAVE_DEBUG
                for (int j = 0; j <= v; ++j) {
                    const uint16_t* q = region + used + (uint64_t)j * sp.cap;
                    uint64_t nb = 0;
                    for (uint32_t k = 0; k < ((sr[j].ntok + 7u) & ~7u); ++k) {
                        const uint32_t t = q[k];
                        if ((t & 0xFF00u) == infl::kTokRaw) ++nb;
                        else if ((t & 0xFF00u) == infl::kTokMatch) { nb += (t & 255u) + 3; ++k; }
                    }
                    if (nb != sr[j].out)
                        fprintf(stderr, "sub-lane %d of %d: tokens %u describe %llu bytes, counted %llu (start %llu exit %llu lo %llu hi %llu eob %d)\n",
                                j, sp.nsub, sr[j].ntok, (unsigned long long)nb, (unsigned long long)sr[j].out,
                                (unsigned long long)sr[j].start, (unsigned long long)sr[j].exit, (unsigned long long)lo[j],
                                (unsigned long long)lo[j + 1], sr[j].eob);
                }
#endif
                for (int j = 0; j <= v; ++j) {
                    pt.push_back({(uint32_t)(used + (uint64_t)j * sp.cap), (uint32_t)written});
                    written += (sr[j].ntok + 7u) & ~7u;
                    total += sr[j].out;
                    if (stats) stats->symbols_bits += sr[j].exit - sr[j].start;
                }
                // the next window's sub-lanes start past the last piece (its region's rest is free)
                used += (uint64_t)v * sp.cap + ((sr[v].ntok + 7u) & ~7u);
                if (sr[v].bad) { done = 3; break; }  // an invalid code on the verified chain: corrupt
                if (sr[v].eob) {
                    p = bp + sr[v].exit;
                    prev_bits = p - body;
                    done = 1;
                    break;
                }
                bp += sr[v].exit;  // the window ended inside the block: the next window
            }
            if (done == 4) {  // split: undo this block (its earlier windows' pieces and output)
                pt.resize(blk_pieces);
                units.resize(blk_units);
                unit_v0 = blk_v0;
                total = blk_total;
                used = blk_used;
                written = blk_written;
                p = blk_start;
                break;
            }
            if (done != 1) break;
        }
        if (bfinal) {
            r.final_block = 1;
            r.status = stop == ~0ull ? infl::kLaneOk : infl::kLaneMismatch;
            break;
        }
    }
    r.end_bit = p;
    r.out_len = total;
    r.ntok = (uint32_t)written;
    r.pieces = (uint32_t)pt.size();
}
#endif

}  // namespace wave
}  // namespace ik
