// ik_inflate.h -- DEFLATE (RFC 1951) decoding core shared by the GPU PNG decoder
// (ik_png.hip) and its host-side model (ik_png_model.cpp, CPU tests only).
//
// decode_image on a PNG (reference src/transform.rs:31 -> png 0.18 via image
// 0.25.8) spends nearly all its time in zlib inflate of the IDAT stream.  The
// stream is one serial bit sequence, so the GPU decoder cuts it into chunks and
// decodes them in parallel, rapidgzip-style:
//
//  1. find:  in every chunk, the first bit offset where a *dynamic* block header
//            parses and builds valid Huffman codes (a strong filter: BTYPE, HLIT/
//            HDIST ranges, a complete code-length code, code lengths that decode
//            to exactly HLIT+HDIST entries, complete literal/distance codes with an
//            end-of-block code).
//  2. decode: one decoder lane per candidate start decodes whole blocks until it
//            reaches the next candidate; it must land exactly on it (else the
//            candidate was not a real block start: it is dropped and the lane
//            decodes on next round).  The lane writes a token stream (literal
//            ranks, matches, each block's literal table) into its own region and
//            reports its output length -> prefix sums -> output offsets.
//  3. expand: each lane's tokens -> u16 symbols at its output offset: a literal
//            byte (< 256), or for a back-reference into bytes before the lane's
//            own output (written by its predecessor) a marker 0x8000 | index into
//            the 32 KiB window that precedes the lane's first output byte.
//            Markers copied within a lane keep their value (they name an absolute
//            position).  This pass holds no code tables, so it runs at full
//            occupancy, which hides the latency of its copies' loads.
//  4. resolve (before the PNG unfilter pass): a marker is replaced by the byte at
//            its window position, following chains through earlier lanes.
//
// Everything here is written once for both compilers: IK_HD functions run in the
// HIP kernels and in the CPU model that the CPU test suite checks against zlib.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define IK_HD __host__ __device__ __forceinline__
#define IK_HD_COLD __host__ __device__ __attribute__((noinline))
#define IK_UNROLL _Pragma("unroll")
#else
#define IK_UNROLL
#define IK_HD inline
#define IK_HD_COLD inline
#endif

// device code: stream / output pointers in the global address space, so loads
// and stores are global_* (vmcnt only) instead of flat_* (which also count in
// lgkmcnt and would make every LDS wait wait for memory too)
#if defined(__HIP_DEVICE_COMPILE__)
#define IK_GLOBAL __attribute__((address_space(1)))
#else
#define IK_GLOBAL
#endif

namespace ik {
namespace infl {

constexpr int kWindow = 32768;

// 32-bit little-endian words of the stream; pos = absolute bit position of the
// next bit.  The buffer must hold >= 4 zero words past the last stream word.
struct Bits {
    const uint32_t* w;
    uint64_t buf;
    int n;          // valid bits in buf
    uint64_t wi;    // next word index to load
    uint64_t wend;  // words that may be read (the stream and its zero padding)
    uint32_t nxt;   // prefetched word wi
    IK_HD void init(const uint32_t* words, uint64_t bit, uint64_t nwords) {
        w = words;
        wend = nwords;
        wi = bit >> 5;
        const uint32_t first = wi < wend ? w[wi] : 0u;
        n = 32 - (int)(bit & 31);
        buf = (uint64_t)(first >> (bit & 31));
        ++wi;
        nxt = wi < wend ? w[wi] : 0u;
    }
    IK_HD uint64_t pos() const { return (wi << 5) - (uint64_t)n; }
    IK_HD void refill() {
        if (n < 32) {
            buf |= (uint64_t)nxt << n;
            n += 32;
            ++wi;
            nxt = wi < wend ? w[wi] : 0u;  // never past the buffer, whatever a corrupt stream says
        }
    }
    IK_HD uint32_t peek(int k) const { return (uint32_t)buf & ((1u << k) - 1u); }
    IK_HD void drop(int k) {
        buf >>= k;
        n -= k;
    }
    IK_HD uint32_t get(int k) {  // k <= 25 after a refill
        refill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
};

// canonical-code bookkeeping of one code (lengths 0..15)
struct CodeInfo {
    uint16_t count[16];
    int max;
};

// RFC 1951 3.2.2 / zlib inftrees: 0 = ok, -1 = oversubscribed or incomplete
// (incomplete is accepted only for a code of at most one length-1... i.e. max <= 1
// as zlib does for literal/distance codes; `codes` = the code-length code, which
// must be complete)
IK_HD_COLD int code_check(const uint8_t* lens, int n, bool codes, CodeInfo& ci) {
    for (int i = 0; i < 16; ++i) ci.count[i] = 0;
    for (int i = 0; i < n; ++i) ci.count[lens[i]]++;
    ci.max = 0;
    for (int l = 15; l >= 1; --l)
        if (ci.count[l]) { ci.max = l; break; }
    if (ci.max == 0) return codes ? -1 : 0;  // no codes: only allowed for literal/distance (distance-free block)
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left <<= 1;
        left -= ci.count[l];
        if (left < 0) return -1;  // oversubscribed
    }
    if (left > 0 && (codes || ci.max != 1)) return -1;  // incomplete
    return 0;
}

IK_HD uint32_t rev_bits(uint32_t v, int k) {
    uint32_t r = 0;
    for (int i = 0; i < k; ++i) {
        r = (r << 1) | (v & 1u);
        v >>= 1;
    }
    return r;
}

IK_HD int len_base(int s) {  // length symbols 257..285
    // RFC 1951 3.2.5
    const int i = s - 257;
    if (i < 8) return 3 + i;
    if (i == 28) return 258;
    const int e = (i - 4) >> 2;
    return ((4 + ((i - 4) & 3)) << e) + 3;
}
IK_HD int len_extra(int s) {
    const int i = s - 257;
    if (i < 8 || i == 28) return 0;
    return (i - 4) >> 2;
}
IK_HD int dist_base(int d) {  // distance symbols 0..29
    if (d < 4) return 1 + d;
    const int e = (d - 2) >> 1;
    return ((2 + (d & 1)) << e) + 1;
}
IK_HD int dist_extra(int d) { return d < 4 ? 0 : (d - 2) >> 1; }

// the same tables without branches (selects), for the GPU's symbol loop:
// length code rank i = symbol - 257 (0..28), distance code d (0..29)
IK_HD void len_code(int i, int& base, int& extra) {
    const int e0 = (i - 4) >> 2, e = e0 < 0 ? 0 : e0;
    const bool small = i < 8, last = i == 28;
    extra = (small || last) ? 0 : e;
    base = small ? 3 + i : (last ? 258 : ((4 + ((i - 4) & 3)) << e) + 3);
}
IK_HD void dist_code(int d, int& base, int& extra) {
    const int e0 = (d - 2) >> 1, e = e0 < 0 ? 0 : e0;
    const bool small = d < 4;
    extra = small ? 0 : e;
    base = small ? 1 + d : ((2 + (d & 1)) << e) + 1;
}

// Parse a dynamic block header at b (after BFINAL/BTYPE) into code lengths,
// validating like zlib.  lens: 286 + 30 entries (literal/length then distance).
// Returns 0 or -1.
IK_HD_COLD int parse_dynamic(Bits& b, uint8_t* lens, int& nlen, int& ndist, CodeInfo& lci, CodeInfo& dci) {
    const int hlit = (int)b.get(5), hdist = (int)b.get(5), hclen = (int)b.get(4);
    nlen = hlit + 257;
    ndist = hdist + 1;
    if (nlen > 286 || ndist > 30) return -1;
    const int ncode = hclen + 4;
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint8_t cl[19];
    for (int i = 0; i < 19; ++i) cl[i] = 0;
    for (int i = 0; i < ncode; ++i) cl[order[i]] = (uint8_t)b.get(3);
    CodeInfo cci;
    if (code_check(cl, 19, true, cci)) return -1;
    // code-length code: lengths <= 7, decode with a direct 7-bit table
    uint8_t ctab_sym[128], ctab_len[128];
    {
        uint32_t next[8];
        uint32_t c = 0;
        for (int l = 1; l <= 7; ++l) {
            c = (c + (l > 1 ? cci.count[l - 1] : 0)) << 1;
            next[l] = c;
        }
        for (int i = 0; i < 128; ++i) ctab_len[i] = 0;
        for (int l = 1; l <= 7; ++l)
            for (int s = 0; s < 19; ++s) {
                if (cl[s] != l) continue;
                const uint32_t r = rev_bits(next[l]++, l);
                for (uint32_t i = r; i < 128; i += (1u << l)) { ctab_sym[i] = (uint8_t)s; ctab_len[i] = (uint8_t)l; }
            }
    }
    const int total = nlen + ndist;
    int i = 0;
    while (i < total) {
        b.refill();
        const uint32_t k = b.peek(7);
        const int l = ctab_len[k];
        if (!l) return -1;
        const int s = ctab_sym[k];
        b.drop(l);
        if (s < 16) {
            lens[i++] = (uint8_t)s;
        } else {
            int rep;
            uint8_t v = 0;
            if (s == 16) {
                if (i == 0) return -1;
                v = lens[i - 1];
                rep = 3 + (int)b.get(2);
            } else if (s == 17) {
                rep = 3 + (int)b.get(3);
            } else {
                rep = 11 + (int)b.get(7);
            }
            if (i + rep > total) return -1;
            while (rep--) lens[i++] = v;
        }
    }
    if (lens[256] == 0) return -1;  // no end-of-block code
    if (code_check(lens, nlen, false, lci)) return -1;
    if (code_check(lens + nlen, ndist, false, dci)) return -1;
    return 0;
}

// Fixed Huffman code lengths (RFC 1951 3.2.6)
IK_HD_COLD void fixed_lens(uint8_t* lens) {
    for (int i = 0; i < 144; ++i) lens[i] = 8;
    for (int i = 144; i < 256; ++i) lens[i] = 9;
    for (int i = 256; i < 280; ++i) lens[i] = 7;
    for (int i = 280; i < 288; ++i) lens[i] = 8;
    for (int i = 0; i < 30; ++i) lens[288 + i] = 5;
}

// Kraft sum of a dynamic header's code-length code, in units of 2^-7 (complete =
// 128).  `cl` holds the 3-bit code-length-code lengths from bit 0 (57 bits; bits
// past the ncode fields may be anything); `T` maps 9 bits (three lengths) to the
// sum of 2^(7 - len) over its nonzero lengths.  Shifting the ncode fields to the
// top of the word drops the absent ones and leaves zeros below, and as 64 = 1 mod
// 3, every field then starts at a bit = 1 (mod 3): seven aligned 9-bit groups from
// bit 1 cover them, absent lengths reading as 0 -- no mask by ncode.
template <class Tab>
IK_HD uint32_t cl_kraft_top(uint64_t cl, int ncode, Tab T) {
    const uint64_t x = cl << (64 - 3 * ncode);  // ncode 4..19: shift 52..7
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    return (uint32_t)T[(xl >> 1) & 511u] + T[(xl >> 10) & 511u] + T[(xl >> 19) & 511u] +
           T[((xl >> 28) | (xh << 4)) & 511u] + T[(xh >> 5) & 511u] + T[(xh >> 14) & 511u] + T[xh >> 23];
}

// The finder's full header check, streaming: decodes the code lengths with the
// caller's 128-entry code-length-code table (LDS; entry = symbol | length << 5)
// and keeps only running sums -- no length arrays -- rejecting as soon as the
// literal/length code is oversubscribed.  Accepts exactly what parse_dynamic
// accepts (complete codes, or a single length-1 code; an end-of-block code).
// `bits` = the 57 bits after the 17 header bits (the code-length code lengths).
template <class Tab>
IK_HD bool dynamic_header_ok(const uint32_t* words, uint64_t nbits, uint64_t bit, uint32_t hdr17, uint64_t bits,
                             Tab tab) {
    const int nlen = (int)((hdr17 >> 3) & 31u) + 257, ndist = (int)((hdr17 >> 8) & 31u) + 1;
    const int ncode = (int)((hdr17 >> 13) & 15u) + 4;
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint8_t cl[19];
    for (int i = 0; i < 19; ++i) cl[i] = 0;
    for (int i = 0; i < ncode; ++i) {
        cl[order[i]] = (uint8_t)((bits >> (3 * i)) & 7u);
        cnt[cl[order[i]]]++;
    }
    uint32_t next[8];
    uint32_t c = 0;
    for (int l = 1; l <= 7; ++l) {
        c = (c + (l > 1 ? cnt[l - 1] : 0)) << 1;
        next[l] = c;
    }
    for (int l = 1; l <= 7; ++l)
        for (int sym = 0; sym < 19; ++sym) {
            if (cl[sym] != l) continue;
            const uint32_t r = rev_bits(next[l]++, l);
            for (uint32_t i = r; i < 128; i += (1u << l)) tab[i] = (uint8_t)(sym | (l << 5));
        }
    Bits b;
    b.init(words, bit + 17 + 3 * (uint64_t)ncode, (nbits >> 5) + 4);
    const int total = nlen + ndist;
    int i = 0, prev = -1;
    uint32_t kl = 0, kd = 0;
    int maxl = 0, maxd = 0;
    bool eob = false;
    while (i < total) {
        b.refill();
        const uint32_t e = tab[b.peek(7)];
        const int l = (int)(e >> 5), sym = (int)(e & 31u);
        b.drop(l);
        int rep = 1, val = sym;
        if (sym == 16) {
            if (prev < 0) return false;
            val = prev;
            rep = 3 + (int)b.get(2);
        } else if (sym == 17) {
            val = 0;
            rep = 3 + (int)b.get(3);
        } else if (sym == 18) {
            val = 0;
            rep = 11 + (int)b.get(7);
        }
        if (i + rep > total) return false;
        if (val) {
            // the run's lengths split between the literal/length and distance codes
            const int nl = i < nlen ? (i + rep <= nlen ? rep : nlen - i) : 0;
            const int nd = rep - nl;
            if (nl) {
                kl += (uint32_t)nl << (15 - val);
                if (kl > 32768u) return false;
                if (val > maxl) maxl = val;
                if (i <= 256 && 256 < i + nl) eob = true;
            }
            if (nd) {
                kd += (uint32_t)nd << (15 - val);
                if (kd > 32768u) return false;
                if (val > maxd) maxd = val;
            }
        }
        i += rep;
        prev = val;
    }
    if (!eob) return false;
    if (kl != 32768u && !(maxl == 1 && kl == 16384u)) return false;
    if (kd != 0u && kd != 32768u && !(maxd == 1 && kd == 16384u)) return false;
    return true;
}

// dynamic_header_ok's test shaped for the GPU block search's flush (k_png_find),
// where 64 lanes check 64 candidates at once and the wave waits for its slowest
// lane: the code-length code is decoded canonically -- left-justified limits,
// first codes and rank offsets packed bytewise in registers, the symbols by rank 5
// bits each in two more -- so no 128-entry table is built per candidate and the
// loop's dependent chain touches memory once per 32 bits (the window word); one
// refill per code length (32 bits cover a code of <= 7 bits and its <= 7 repeat
// bits), the repeat codes decoded without branches.  Same accept set as
// dynamic_header_ok (the CPU model holds the two equal on every candidate of its
// streams).  Win: fetch(w) loads stream words w .. w + 31, word(k) reads the k-th.
IK_HD uint32_t rev32(uint32_t v);
template <class Win>
IK_HD bool dynamic_header_win(uint64_t p, uint32_t h, uint64_t bits, Win& win) {
    const int nlen = (int)((h >> 3) & 31u) + 257, ndist = (int)((h >> 8) & 31u) + 1;
    const int ncode = (int)((h >> 13) & 15u) + 4;
    // code-length code: count per length, then ranks in canonical (length, symbol) order
    constexpr uint8_t inv_order[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};
    uint64_t cnt = 0;  // byte L: codes of length L (L = 1..7)
IK_UNROLL
    for (int s = 0; s < 19; ++s) {
        const int i = inv_order[s];
        const uint32_t len = i < ncode ? (uint32_t)(bits >> (3 * i)) & 7u : 0u;
        if (len) cnt += 1ull << (8 * len);
    }
    uint64_t first = 0, offs = 0, lim = 0;  // bytes L: first code, rank of the first code, left-justified limit
    {
        uint32_t code = 0, rank = 0;
IK_UNROLL
        for (int L = 1; L <= 7; ++L) {
            const uint32_t cprev = L > 1 ? (uint32_t)(cnt >> (8 * (L - 1))) & 255u : 0u;
            const uint32_t cl = (uint32_t)(cnt >> (8 * L)) & 255u;
            code = (code + cprev) << 1;
            first |= (uint64_t)code << (8 * L);
            offs |= (uint64_t)rank << (8 * L);
            lim |= (uint64_t)((code + cl) << (7 - L)) << (8 * L);
            rank += cl;
        }
    }
    // the symbols by canonical rank, 5 bits each in two registers (ranks 0..11, 12..18):
    // a register select per code length, not an LDS round trip on the loop's chain
    uint64_t sy_lo = 0, sy_hi = 0;
    {
        uint64_t ctr = 0;  // byte L: symbols of length L placed so far
IK_UNROLL
        for (int s = 0; s < 19; ++s) {
            const int i = inv_order[s];
            const uint32_t len = i < ncode ? (uint32_t)(bits >> (3 * i)) & 7u : 0u;
            if (len) {
                const uint32_t r = ((uint32_t)(offs >> (8 * len)) & 255u) + ((uint32_t)(ctr >> (8 * len)) & 255u);
                if (r < 12) sy_lo |= (uint64_t)s << (5 * r);
                else sy_hi |= (uint64_t)s << (5 * (r - 12));
                ctr += 1ull << (8 * len);
            }
        }
    }
    const uint64_t bit = p + 17 + 3 * (uint64_t)ncode;
    uint64_t wb = bit >> 5;  // window base (word index)
    win.fetch(wb);
    uint64_t buf = (uint64_t)(win.word(0) >> (bit & 31));
    int n = 32 - (int)(bit & 31);
    uint32_t k = 1;  // next window word
    const int total = nlen + ndist;
    int i = 0, prev = -1;
    uint32_t kl = 0, kd = 0;
    int maxl = 0, maxd = 0;
    bool eob = false;
    // one refill per code length: 32 bits in the buffer cover a code (<= 7 bits) and
    // its repeat bits (<= 7); the repeat symbols are decoded without branches (the
    // lanes of a flush hold different symbols, so branches ran every path anyway)
    while (i < total) {
        if (n < 32) {
            if (k == 32) {
                wb += 32;
                win.fetch(wb);
                k = 0;
            }
            buf |= (uint64_t)win.word(k) << n;
            n += 32;
            ++k;
        }
        const uint32_t c = rev32((uint32_t)buf) >> 25;  // the next 7 bits, first bit as MSB
        int L = 1;
IK_UNROLL
        for (int l = 1; l < 7; ++l) L += c >= ((uint32_t)(lim >> (8 * l)) & 255u) ? 1 : 0;
        const uint32_t r = (c >> (7 - L)) - ((uint32_t)(first >> (8 * L)) & 255u) + ((uint32_t)(offs >> (8 * L)) & 255u);
        const int sym = (int)((r < 12 ? sy_lo >> (5 * r) : sy_hi >> (5 * (r - 12))) & 31u);
        const int xb = sym < 16 ? 0 : sym == 16 ? 2 : sym == 17 ? 3 : 7;  // repeat bits
        const int rep = sym < 16 ? 1 : (sym == 18 ? 11 : 3) + (int)((uint32_t)(buf >> L) & ((1u << xb) - 1u));
        buf >>= L + xb;
        n -= L + xb;
        const int val = sym < 16 ? sym : sym == 16 ? prev : 0;
        if ((sym == 16 && prev < 0) || i + rep > total) return false;
        // the run's lengths split between the literal/length and distance codes
        const int nl = i < nlen ? (i + rep <= nlen ? rep : nlen - i) : 0;
        const int nd = rep - nl;
        const uint32_t w = val ? 1u << (15 - val) : 0u;
        kl += (uint32_t)nl * w;
        kd += (uint32_t)nd * w;
        if (kl > 32768u || kd > 32768u) return false;
        maxl = nl && val > maxl ? val : maxl;
        maxd = nd && val > maxd ? val : maxd;
        eob = eob || (val && i <= 256 && 256 < i + nl);
        i += rep;
        prev = val;
    }
    if (!eob) return false;
    if (kl != 32768u && !(maxl == 1 && kl == 16384u)) return false;
    if (kd != 0u && kd != 32768u && !(maxd == 1 && kd == 16384u)) return false;
    return true;
}

// Is there a plausible dynamic block header at absolute bit `bit`?  (step 1)
IK_HD_COLD bool plausible_dynamic(const uint32_t* words, uint64_t nbits, uint64_t bit) {
    Bits b;
    b.init(words, bit, (nbits >> 5) + 4);
    b.refill();
    const uint32_t h = b.peek(17);  // BFINAL, BTYPE(2), HLIT(5), HDIST(5), HCLEN(4)
    if (((h >> 1) & 3u) != 2u) return false;
    if (((h >> 3) & 31u) > 29u || ((h >> 8) & 31u) > 29u) return false;
    b.drop(3);
    uint8_t lens[286 + 30];
    int nlen, ndist;
    CodeInfo lci, dci;
    return parse_dynamic(b, lens, nlen, ndist, lci, dci) == 0;
}


// ---- one decoder ("lane") ------------------------------------------------------
enum LaneStatus { kLaneOk = 0, kLaneMismatch = 1, kLaneCorrupt = 2 };
struct LaneResult {
    uint64_t end_bit;   // block boundary where the decoder stopped
    uint64_t out_len;   // bytes it decoded
    uint32_t ntok;      // tokens it wrote (decode pass)
    int status;         // LaneStatus (or kLaneOverflow)
    int final_block;    // it decoded the BFINAL block
    uint32_t iters;     // symbol-loop iterations (profile)
    uint32_t kcycles;   // GPU: clock ticks / 1024 from start to end (profile)
    uint32_t blocks;    // blocks decoded
    uint32_t pieces;    // wave decoder (ik_png_wave.h): token pieces written
    uint32_t kc_setup;  // wave decoder, profile: clock ticks / 1024 in block codes, tables and window staging
    uint32_t units;     // wave decoder: expand units recorded (ik_png_wave.h kUnitMinTok)
};

// Decode whole blocks from `start` (a block boundary) until a block boundary >=
// `stop` (exact hit: kLaneOk; passing it, or the final block before it:
// kLaneMismatch), or through the final block when stop == ~0.  EMIT: write u16
// symbols at out[obase + k] (literal bytes, or window markers for bytes before
// obase, see the file comment); obase < 0 = unknown (count pass).  out_cap
// bounds the lane's output (corrupt past it).
// value of the u16 stream at absolute position q after following window markers.
// lane_obase: output offsets of the image's decoders (ascending), n of them;
// page_lane[q >> page_shift] = the decoder that holds the page's first byte.
// Returns -1 on a malformed chain.  Each hop lands in a strictly earlier decoder
// (a marker points into the window before its decoder's first byte), so a chain
// has at most n hops: repetitive data can carry a byte back through every lane.
template <class U16, class Off, class Pages>
IK_HD int resolve_at(U16 u16, Off lane_obase, int n, Pages page_lane, int page_shift, int64_t q) {
    int lane = -1;
    for (int guard = 0; guard <= n; ++guard) {
        const uint32_t v = u16[q];
        if (v < 256u) return (int)v;
        if (!(v & 0x8000u)) return -1;
        // the decoder that wrote position q (the first hop: its page's decoder or a
        // later one; later hops: the same decoder or an earlier one)
        if (lane < 0) {
            lane = page_lane[q >> page_shift];
            while (lane + 1 < n && (int64_t)lane_obase[lane + 1] <= q) ++lane;
        } else {
            while (lane > 0 && (int64_t)lane_obase[lane] > q) --lane;
        }
        q = (int64_t)lane_obase[lane] - kWindow + (int64_t)(v & 0x7FFFu);
        if (q < 0) return -1;
    }
    return -1;
}


// ---- canonical decoding, code-length limits in registers --------------------
// The GPU decoder lanes keep per-code tables tiny so that many waves fit a CU:
// for each code (literal/length, distance) the 15 left-justified limits live in
// registers, and a few small per-length tables live in LDS.
//   lim[L-1] (L = 1..15): exclusive upper bound of the codes of length <= L, as
//   15-bit MSB-first values.  For the next 15 stream bits W (bit-reversed: the
//   first bit read is the MSB), the code length is 1 + #{L < 15 : W >= lim[L-1]};
//   W >= lim[14] is no code (an incomplete code's gap).
// Canonical order within a length is by symbol value, so for the literal/length
// code a length's codes are: its literals, then end-of-block, then length codes.
// Table memory per lane (u32 words; the GPU keeps word w of lane l at LDS word
// 64 w + l, so that lanes reading different words hit different banks):
//   [0..15]  linfo[L]: first code (15 bits) | #literals of length L (9) << 15
//                      | EOB has length L (1) << 24 | rank of its first length code (5) << 25
//   [16..31] dinfo[L]: first distance code (15 bits) | rank of its first distance code (5) << 16
//                      | rank of the first LITERAL of length L (9) << 21
//   bytes from word 32: lsyms[32] (length symbol - 257), dsyms[32]
// A literal is identified by its rank (0..255) in canonical order; the rank ->
// byte table of each block goes into the token stream (below), not into LDS.
constexpr int kCanonWords = 48;  // 192 bytes
struct CanonRegs {
    uint32_t lpk[8], dpk[8];  // limits minus one, packed in signed 16-bit pairs (canon_len)
};
IK_HD void pack_limits(const uint32_t (&lim)[15], uint32_t (&pk)[8]) {
    for (int k = 0; k < 7; ++k)
        pk[k] = ((lim[2 * k] - 1u) & 0xFFFFu) | (((lim[2 * k + 1] - 1u) & 0xFFFFu) << 16);
    pk[7] = (lim[14] - 1u) & 0xFFFFu;
}

IK_HD uint32_t rev32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(v);
#else
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    v = ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
    v = ((v >> 4) & 0x0F0F0F0Fu) | ((v & 0x0F0F0F0Fu) << 4);
    v = ((v >> 8) & 0x00FF00FFu) | ((v & 0x00FF00FFu) << 8);
    return (v >> 16) | (v << 16);
#endif
}

template <class Mem>
IK_HD uint8_t cm_byte(const Mem& m, int i) { return (uint8_t)(m[32 + (i >> 2)] >> (8 * (i & 3))); }

// ---- token stream ---------------------------------------------------------------
// The decode pass writes each lane's output as u16 tokens into the lane's own
// region (its output offset is not known yet); the expand pass turns them into
// the u16 symbol stream (bytes, window markers) at the lane's output offset.
//   0x0000..0x00FF      a literal of a Huffman block: its canonical rank
//   0x4000 | byte       a literal of a stored block
//   0x8000 | (len - 3)  a match, followed by one token: distance - 1
//   0xFFFF              block start: 0xFFFE pads to a multiple of 8 tokens, then
//                       128 tokens hold the block's literal table (256 bytes:
//                       byte r = the literal of rank r)
constexpr uint32_t kTokRaw = 0x4000u, kTokMatch = 0x8000u, kTokTable = 0xFFFFu, kTokPad = 0xFFFEu;
constexpr uint32_t kTokTableLen = 128;
constexpr uint32_t kTokSlack = 16;  // tokens a region holds past its capacity check (padding)

// Token region capacity of a lane over `bits` compressed bits: a quarter token
// per bit (image data runs ~8 bits per token), or with `exact` the true bound
// (a token costs at least one bit: a literal >= 1, a match's two >= 2) -- for
// the lanes that overflowed the first.  Multiple of 8, plus a block's table.
IK_HD uint32_t tok_capacity(uint64_t bits, bool exact) {
    uint64_t c = (exact ? bits : bits / 4) + 2 * kTokTableLen + 64;
    if (c > 0x7FFFFFF0ull) c = 0x7FFFFFF0ull;
    return (uint32_t)((c + 7) & ~7ull);
}

// Token output of one lane: `p` = its region (16-byte aligned).  Complete groups
// of 8 tokens are held back (pending, at most two: a decode step adds up to three
// tokens and the GPU flushes every four steps, so up to twelve tokens -- two groups
// -- complete between flushes) and stored by flush(): the GPU decoder flushes only
// at its input ring's refill points, so that the wait there covers exactly the
// ring's DMA (see ik_png.hip WinLds::tick).
struct TokOut {
    IK_GLOBAL uint16_t* p;
    uint64_t p0 = 0, p1 = 0, q0 = 0, q1 = 0;
    uint32_t ppos = 0, qpos = 0;
    int npend = 0;
    IK_HD void group(uint32_t pos, uint64_t lo, uint64_t hi) {
        if (npend == 0) {
            p0 = lo;
            p1 = hi;
            ppos = pos;
        } else {
            q0 = lo;
            q1 = hi;
            qpos = pos;
        }
        ++npend;
    }
    IK_HD void store1(uint32_t pos, uint64_t lo, uint64_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 v = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
        *reinterpret_cast<IK_GLOBAL u4*>(p + pos) = v;  // one 16-byte store
#else
        for (int k = 0; k < 4; ++k) {
            p[pos + k] = (uint16_t)(lo >> (16 * k));
            p[pos + 4 + k] = (uint16_t)(hi >> (16 * k));
        }
#endif
    }
    // stores the pending groups; returns how many (0, 1, 2)
    IK_HD int flush() {
        const int n = npend;
        if (n >= 1) store1(ppos, p0, p1);
        if (n >= 2) store1(qpos, q0, q1);
        npend = 0;
        return n;
    }
    IK_HD void table_byte(uint32_t tpos, int rank, uint8_t v) const {
        reinterpret_cast<IK_GLOBAL uint8_t*>(p + tpos)[rank] = v;
    }
};

// Build both codes' limits and tables (lens: literal/length lengths [0, nlen),
// distance lengths at 288..); the literal table goes to the token stream at tpos.
template <class Mem>
IK_HD_COLD void canon_build(const uint8_t* lens, int nlen, int ndist, CanonRegs& R, Mem m, TokOut& out,
                            uint32_t tpos) {
    // literal/length code
    uint32_t cnt[16], first[16], llim[15], dlim[15];
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int s = 0; s < nlen; ++s) cnt[lens[s]]++;
    uint32_t code = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1;
        first[l] = code;
        llim[l - 1] = (first[l] + cnt[l]) << (15 - l);
    }
    for (int i = 0; i < 16; ++i) m[32 + i] = 0;  // lsyms, dsyms
    uint32_t litr = 0, lenr = 0;
    uint32_t lrank_of[16];
    lrank_of[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        uint32_t nl = 0, nlen_codes = 0, eob = 0;
        for (int s = 0; s < nlen && s < 286; ++s) {
            if (lens[s] != l) continue;
            if (s < 256) {
                out.table_byte(tpos, (int)(litr + nl), (uint8_t)s);
                ++nl;
            } else if (s == 256) {
                eob = 1;
            } else {
                const int w = (int)(lenr + nlen_codes);
                if (w < 32)
                    m[32 + w / 4] = (m[32 + w / 4] & ~(255u << (8 * (w & 3)))) | ((uint32_t)(s - 257) << (8 * (w & 3)));
                ++nlen_codes;
            }
        }
        m[l] = (first[l] & 0x7FFFu) | (nl << 15) | (eob << 24) | (lenr << 25);
        lrank_of[l] = litr;
        litr += nl;
        lenr += nlen_codes;
    }
    // distance code
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int s = 0; s < ndist; ++s) cnt[lens[288 + s]]++;
    code = 0;
    uint32_t dr = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1;
        dlim[l - 1] = (code + cnt[l]) << (15 - l);
        m[16 + l] = (code & 0x7FFFu) | (dr << 16) | (lrank_of[l] << 21);
        for (int s = 0; s < ndist; ++s) {
            if (lens[288 + s] != l) continue;
            const int w = 32 + (int)dr;
            if (dr < 32) m[32 + w / 4] = (m[32 + w / 4] & ~(255u << (8 * (w & 3)))) | ((uint32_t)s << (8 * (w & 3)));
            ++dr;
        }
    }
    m[0] = 0;
    m[16] = 0;
    pack_limits(llim, R.lpk);
    pack_limits(dlim, R.dpk);
}

// code length for a 15-bit window; 16 = no code.  pk[k] holds lim[2k]-1 and
// lim[2k+1]-1 as two signed 16-bit halves (pk[7]: lim[14]-1), so one packed
// 16-bit subtract compares the window with two limits at once and the sign bits
// count the limits at or below it (v_pk_sub_i16 + v_bcnt).
IK_HD int canon_len(uint32_t c15, const uint32_t (&pk)[8]) {
    uint32_t at_or_below = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    typedef short s2 __attribute__((ext_vector_type(2)));
    const s2 x = {(short)c15, (short)c15};
    uint32_t d[7];
    IK_UNROLL
    for (int k = 0; k < 7; ++k)
        d[k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, pk[k]) - x);  // lim - 1 - c15 < 0  <=>  lim <= c15
    // the sign bits sit in bytes 1 and 3: v_perm_b32 gathers those bytes of two
    // differences into one word, so one AND and one popcount count four limits
    IK_UNROLL
    for (int k = 0; k < 6; k += 2)
        at_or_below += (uint32_t)__builtin_popcount(__builtin_amdgcn_perm(d[k], d[k + 1], 0x07050301u) & 0x80808080u);
    at_or_below += (uint32_t)__builtin_popcount(d[6] & 0x80008000u);
#else
    for (int k = 0; k < 7; ++k) {
        at_or_below += (int16_t)(pk[k] & 0xFFFFu) - (int)c15 < 0 ? 1u : 0u;
        at_or_below += (int16_t)(pk[k] >> 16) - (int)c15 < 0 ? 1u : 0u;
    }
#endif
    return (int)c15 > (int16_t)(pk[7] & 0xFFFFu) ? 16 : 1 + (int)at_or_below;
}

// Input window of the hot loop on the host (the CPU model): the three words
// holding the next 64+ bits.  The GPU decoder's window is ik_png.hip WinLds (an
// LDS ring filled by DMA); both offer init / tick / bits64 / advance / pos.
struct Win {
    const uint32_t* w;
    uint32_t wend, pos;  // streams under 2^32 bits (the host checks)
    IK_HD uint32_t rd(uint32_t i) const { return i < wend ? w[i] : 0u; }
    IK_HD void init(const uint32_t* words, uint32_t nwords, uint32_t bit) {
        w = words;
        wend = nwords;
        pos = bit;
    }
    uint32_t it = 0;
    IK_HD void tick(TokOut& o) {  // every 4 steps, as the GPU's ring refill (ik_png.hip WinLds::tick)
        if (++it % 4u) return;
        o.flush();
    }
    // x0 / x1 / x2 for a slide of 0 / 1 / 2 words, by masks: a ternary chain
    // becomes an indexed private array on the GPU (scratch memory)
    IK_HD static uint32_t sel3(uint32_t m1, uint32_t m2, uint32_t x0, uint32_t x1, uint32_t x2) {
        return (x0 & ~m1) | (x1 & m1 & ~m2) | (x2 & m2);
    }
    IK_HD uint64_t bits64() const {  // the next 64 stream bits
        const uint32_t wi = pos >> 5, sh = pos & 31u;
        const uint64_t lo = (uint64_t)rd(wi) | ((uint64_t)rd(wi + 1) << 32);
        return sh ? (lo >> sh) | ((uint64_t)rd(wi + 2) << (64 - sh)) : lo;
    }
    IK_HD void advance(uint32_t k) { pos += k; }
};

enum { kLaneOverflow = 3 };  // LaneStatus: the token region was too small
// LaneStatus of the wave decoder (ik_png_wave.h): the lane decoded whole blocks up to
// end_bit (a block boundary before its stop) and has no room for more pieces; the
// chain check starts a new lane there (ik_png_plan.h)
enum { kLaneSplit = 4 };

// Decoder lane, decode pass: whole blocks from `start` (a block boundary) up to
// `stop`, as decode_lane, writing the token stream (TokOut, capacity tcap tokens
// + kTokSlack) and counting the output bytes.  m: this lane's table memory
// (kCanonWords).  first: lane 0 (no distance may reach before its output).
// The symbol loop computes the literal and the match decoding of every symbol
// and selects -- a wave's 64 lanes hold both kinds in nearly every step, so
// branching would run both paths anyway, plus the mask bookkeeping -- and keeps
// the rare cases (end of block, invalid codes, full region) in one branch.
template <class WinT, class Mem>
IK_HD void decode_lane_tok(const uint32_t* words, uint64_t nbits, uint64_t start, uint64_t stop, Mem m, TokOut& out,
                           uint32_t tcap, bool first, uint64_t out_cap, LaneResult& r, WinT W) {
    const uint64_t nwords = (nbits >> 5) + 4;
    Bits b;
    b.init(words, start, nwords);
    const uint64_t plimit = nbits + 64;  // decoding past the stream's padding: corrupt
    uint64_t cnt = 0;
    uint32_t tc = 0;
    uint64_t h0 = 0, h1 = 0;  // the last 8 tokens (newest in the top 16 bits of h1)
    r.status = kLaneCorrupt;
    r.final_block = 0;
    r.iters = 0;
    r.blocks = 0;
    uint8_t lens[288 + 32];
    CanonRegs R;
    auto tput = [&](uint32_t v) {
        h0 = (h0 >> 16) | (h1 << 48);
        h1 = (h1 >> 16) | ((uint64_t)v << 48);
        ++tc;
        if ((tc & 7u) == 0) out.group(tc - 8, h0, h1);
    };
    for (;;) {
        const uint64_t p = b.pos();
        if (p >= stop) {
            r.status = p == stop ? kLaneOk : kLaneMismatch;
            break;
        }
        if (p + 3 > nbits) break;
        b.refill();
        const uint32_t hdr = b.peek(3);
        b.drop(3);
        const int bfinal = (int)(hdr & 1u), btype = (int)(hdr >> 1);
        if (btype == 0) {  // stored
            b.drop(b.n & 7);
            const uint32_t len = b.get(16), nlen = b.get(16);
            if ((len ^ 0xFFFFu) != nlen) break;
            if (cnt + len > out_cap) break;
            if (b.pos() + 8ull * len > nbits) break;
            if ((uint64_t)tc + len > tcap) { r.status = kLaneOverflow; break; }
            for (uint32_t i = 0; i < len; ++i) {
                tput(kTokRaw | b.get(8));
                out.flush();
            }
            cnt += len;
        } else if (btype == 3) {
            break;
        } else {
            int nlen, ndist;
            if (btype == 2) {
                CodeInfo lci, dci;
                Bits hb = b;  // out-of-line parser on a copy: the hot state stays in registers
                const int prc = parse_dynamic(hb, lens, nlen, ndist, lci, dci);
                b = hb;
                if (prc) break;
                for (int i = ndist - 1; i >= 0; --i) lens[288 + i] = lens[nlen + i];
            } else {
                fixed_lens(lens);
                nlen = 288;
                ndist = 30;
            }
            if (tc + kTokTableLen + 8 > tcap) { r.status = kLaneOverflow; break; }
            tput(kTokTable);
            while (tc & 7u) tput(kTokPad);
            out.flush();
            {
                CanonRegs t;
                canon_build(lens, nlen, ndist, t, m, out, tc);
                R = t;
#if defined(__HIP_DEVICE_COMPILE__)
                // R comes back through the stack (canon_build is out of line): take
                // it into registers here, so the loop below holds no waits for those
                // loads -- a wait on the memory counter inside the loop would also
                // wait for the input ring's latest DMA, which the compiler cannot see
                asm volatile("" ::"v"(R.lpk[0]), "v"(R.lpk[1]), "v"(R.lpk[2]), "v"(R.lpk[3]), "v"(R.lpk[4]),
                             "v"(R.lpk[5]), "v"(R.lpk[6]), "v"(R.lpk[7]), "v"(R.dpk[0]), "v"(R.dpk[1]), "v"(R.dpk[2]),
                             "v"(R.dpk[3]), "v"(R.dpk[4]), "v"(R.dpk[5]), "v"(R.dpk[6]), "v"(R.dpk[7]));
#endif
            }
            tc += kTokTableLen;
            W.init((const IK_GLOBAL uint32_t*)words, (uint32_t)nwords, (uint32_t)b.pos());
            ++r.blocks;
            int code = 0;  // why the symbol loop ended: 1 end of block, 2 corrupt, 3 token region full
            for (;;) {
                ++r.iters;
                W.tick(out);
                const uint64_t v = W.bits64();
                // literal/length code
                const uint32_t c15 = rev32((uint32_t)v) >> 17;
                const int L = canon_len(c15, R.lpk);
                const int Lc = L > 15 ? 15 : L;
                const uint32_t info = m[Lc];
                const uint32_t i = (c15 >> (15 - Lc)) - (info & 0x7FFFu);
                const uint32_t nl = (info >> 15) & 0x1FFu;
                const bool lit = i < nl;
                const uint32_t eob = (info >> 24) & 1u;
                const uint32_t lr = ((info >> 25) & 31u) + (i - nl - eob);  // length code rank
                int lb, le;
                len_code((int)cm_byte(m, (int)(lr < 28u ? lr : 28u)), lb, le);
                const uint64_t v1 = v >> Lc;
                const int ll = lb + (int)((uint32_t)v1 & ((1u << le) - 1u));
                // distance code (computed for literals too, and not used)
                const uint64_t v2 = v1 >> le;
                const uint32_t c15d = rev32((uint32_t)v2) >> 17;
                const int D = canon_len(c15d, R.dpk);
                const int Dc = D > 15 ? 15 : D;
                const uint32_t dinfo = m[16 + Dc];
                const uint32_t di = ((c15d >> (15 - Dc)) - (dinfo & 0x7FFFu)) + ((dinfo >> 16) & 31u);
                int db, de;
                dist_code((int)cm_byte(m, 32 + (int)(di < 29u ? di : 29u)), db, de);
                const int dist = db + (int)((uint32_t)(v2 >> Dc) & ((1u << de) - 1u));
                // a second literal right behind a literal, decoded in the same step (about
                // 92 % of the steps on image data): the bits after the first code, the same
                // canonical decode; taken only when it is a literal (anything else -- a
                // length, end of block, an invalid code -- is the next step's first symbol)
                const uint32_t c15b = rev32((uint32_t)v1) >> 17;
                const int L2 = canon_len(c15b, R.lpk);
                const int Lc2 = L2 > 15 ? 15 : L2;
                const uint32_t info2 = m[Lc2];
                const uint32_t i2 = (c15b >> (15 - Lc2)) - (info2 & 0x7FFFu);
                const bool dbl = lit && L2 <= 15 && i2 < ((info2 >> 15) & 0x1FFu);
                // and a third behind the second, the same way
                const uint32_t c15c = rev32((uint32_t)(v1 >> Lc2)) >> 17;
                const int L3 = canon_len(c15c, R.lpk);
                const int Lc3 = L3 > 15 ? 15 : L3;
                const uint32_t info3 = m[Lc3];
                const uint32_t i3 = (c15c >> (15 - Lc3)) - (info3 & 0x7FFFu);
                const bool tri = dbl && L3 <= 15 && i3 < ((info3 >> 15) & 0x1FFu);
                // and a fourth (at most 60 bits for the four: within the 64-bit window)
                const uint32_t c15q = rev32((uint32_t)((v1 >> Lc2) >> Lc3)) >> 17;
                const int L4 = canon_len(c15q, R.lpk);
                const int Lc4 = L4 > 15 ? 15 : L4;
                const uint32_t info4 = m[Lc4];
                const uint32_t i4 = (c15q >> (15 - Lc4)) - (info4 & 0x7FFFu);
                const bool quad = tri && L4 <= 15 && i4 < ((info4 >> 15) & 0x1FFu);
                // the rare cases, one branch and one exit
                const bool eobk = !lit && eob && i == nl;
                const bool odd = L > 15 || (uint64_t)W.pos > plimit ||
                                 (!lit && !eobk && (lr > 28u || D > 15 || di > 29u || (first && (int64_t)cnt < dist)));
                if (odd || eobk || tc + 4 > tcap || cnt + 258 > out_cap) {
                    code = odd ? 2 : eobk ? 1 : tc + 4 > tcap ? 3
                         : cnt + (lit ? (quad ? 4u : tri ? 3u : dbl ? 2u : 1u) : (uint64_t)ll) > out_cap ? 2 : 0;
                    if (code) {
                        if (code == 1) W.advance((uint32_t)Lc);
                        break;
                    }
                }
                // one token (literal rank), two (two literal ranks; match length,
                // distance) or three (three literal ranks), without branches; three
                // tokens complete at most one group of 8
                const uint32_t t1 = lit ? ((m[16 + Lc] >> 21) & 0x1FFu) + i : (kTokMatch | (uint32_t)(ll - 3));
                const uint32_t t2 = lit ? ((m[16 + Lc2] >> 21) & 0x1FFu) + i2 : (uint32_t)(dist - 1);
                const uint32_t t3 = ((m[16 + Lc3] >> 21) & 0x1FFu) + i3;
                const uint32_t t4 = ((m[16 + Lc4] >> 21) & 0x1FFu) + i4;
                const bool two = !lit || dbl;
                const uint64_t a0 = (h0 >> 16) | (h1 << 48), a1 = (h1 >> 16) | ((uint64_t)t1 << 48);
                const uint64_t b0 = (a0 >> 16) | (a1 << 48), b1 = (a1 >> 16) | ((uint64_t)t2 << 48);
                const uint64_t e0 = (b0 >> 16) | (b1 << 48), e1 = (b1 >> 16) | ((uint64_t)t3 << 48);
                const uint64_t f0 = (e0 >> 16) | (e1 << 48), f1 = (e1 >> 16) | ((uint64_t)t4 << 48);
                const uint32_t tc1 = tc + 1;
                const bool g1 = (tc1 & 7u) == 0, g2 = two && ((tc1 + 1) & 7u) == 0, g3 = tri && ((tc1 + 2) & 7u) == 0,
                           g4 = quad && ((tc1 + 3) & 7u) == 0;
                if (g1 || g2 || g3 || g4)
                    out.group(g1 ? tc1 - 8 : g2 ? tc1 - 7 : g3 ? tc1 - 6 : tc1 - 5, g1 ? a0 : g2 ? b0 : g3 ? e0 : f0,
                              g1 ? a1 : g2 ? b1 : g3 ? e1 : f1);
                h0 = quad ? f0 : tri ? e0 : two ? b0 : a0;
                h1 = quad ? f1 : tri ? e1 : two ? b1 : a1;
                tc = quad ? tc1 + 3 : tri ? tc1 + 2 : two ? tc1 + 1 : tc1;
                cnt += lit ? (quad ? 4u : tri ? 3u : dbl ? 2u : 1u) : (uint64_t)ll;
                W.advance(lit ? (uint32_t)(Lc + (dbl ? Lc2 : 0) + (tri ? Lc3 : 0) + (quad ? Lc4 : 0))
                              : (uint32_t)(Lc + le + Dc + de));
            }
            const bool bad = code == 2, full = code == 3;
            out.flush();
            if (full) { r.status = kLaneOverflow; break; }
            if (bad) break;
            b.init(words, W.pos, nwords);
        }
        if (b.pos() > nbits + 64) break;
        if (bfinal) {
            r.final_block = 1;
            r.status = stop == ~0ull ? kLaneOk : kLaneMismatch;
            break;
        }
    }
    const uint32_t ntok = tc;
    out.flush();
    while (tc & 7u) tput(kTokPad);  // the last group, padded (capacity has kTokSlack)
    out.flush();
    r.end_bit = b.pos();
    r.out_len = cnt;
    r.ntok = ntok;
}

// Expand pass: a verified lane's tokens -> u16 symbols at out[obase ..): literal
// bytes, and for copies from before the lane's first byte window markers (0x8000
// | index into the 32 KiB before obase; copied markers keep their value).  The
// last 8 symbols live in two 64-bit registers (h0: distances 8..5, h1: 4..1,
// newest in the top 16 bits), which serve every copy with distance <= 8 and are
// written out as one aligned 16-byte store each time the output position
// reaches a multiple of 8 -- copies from farther back read stored symbols.
// Returns 0, or -1 if the tokens do not make out_len bytes.
template <class TokIn, class Out>
IK_HD int expand_lane(TokIn& tin, uint32_t ntok, Out out, int64_t obase, uint64_t out_len) {
    uint64_t cnt = 0;
    uint64_t h0 = 0, h1 = 0;
    auto put = [&](uint32_t v) {
        h0 = (h0 >> 16) | (h1 << 48);
        h1 = (h1 >> 16) | ((uint64_t)v << 48);
        ++cnt;
        const int64_t g = obase + (int64_t)cnt;
        if ((g & 7) == 0) {
            if ((int64_t)cnt >= 8) {
                out.store16(g - 8, h0, h1);
            } else {  // the group starts before this lane's first symbol: only ours
                for (int64_t q = g - (int64_t)cnt; q < g; ++q) {
                    const int dq = (int)(g - q);  // distance 1..7
                    const uint32_t hv = (uint32_t)((dq <= 4 ? h1 >> (16 * (4 - dq)) : h0 >> (16 * (8 - dq)))) & 0xFFFFu;
                    out.store1(q, (uint16_t)hv);
                }
            }
        }
    };
    auto hist = [&](int d) -> uint32_t {  // the symbol d back (1..8)
        return (uint32_t)((d <= 4 ? h1 >> (16 * (4 - d)) : h0 >> (16 * (8 - d)))) & 0xFFFFu;
    };
    bool have_tab = false;
    int rc = 0;
    for (uint32_t t = 0; t < ntok;) {
        const uint32_t v = tin.next();
        ++t;
        if (v < 256u) {  // a Huffman literal (rank)
            if (!have_tab || cnt >= out_len) { rc = -1; break; }
            put(tin.table(v));
            continue;
        }
        if ((v & 0xFF00u) == kTokRaw) {
            if (cnt >= out_len) { rc = -1; break; }
            put(v & 0xFFu);
            continue;
        }
        if (v == kTokPad) continue;  // the padding of a wave decoder's piece (ik_png_wave.h)
        if (v == kTokTable) {
            while (t & 7u) { (void)tin.next(); ++t; }
            tin.set_table(t);
            have_tab = true;
            t += kTokTableLen;
            tin.seek(t);
            continue;
        }
        if ((v & 0xFF00u) != kTokMatch || t >= ntok) { rc = -1; break; }
        const int ll = (int)(v & 0xFFu) + 3;
        const int dist = (int)tin.next() + 1;
        ++t;
        if (cnt + (uint64_t)ll > out_len) { rc = -1; break; }
        int q = 0;
        // sources before this lane's first symbol (window markers), or in the
        // history registers (distance <= 8: the registers roll as we copy)
        while (q < ll) {
            const int64_t sk = (int64_t)cnt - dist;
            if (sk < 0) put(0x8000u | (uint32_t)(kWindow + sk));
            else if (dist <= 8) put(hist(dist));
            else break;
            ++q;
        }
        // distance > 8: every source is at least 8 back, so already stored; in
        // groups of up to min(8, dist - 8) the loads go out together
        const int G = dist - 8 < 8 ? dist - 8 : 8;
        while (q < ll) {
            const int n = ll - q < G ? ll - q : G;
            const int64_t s0 = obase + (int64_t)cnt - dist;
            uint32_t vv[8];
            IK_UNROLL
            for (int t2 = 0; t2 < 8; ++t2) vv[t2] = t2 < n ? (uint32_t)out.load(s0 + t2) : 0u;
            IK_UNROLL
            for (int t2 = 0; t2 < 8; ++t2)
                if (t2 < n) put(vv[t2]);
            q += n;
        }
    }
    // the symbols after the last multiple of 8 are still only in the history
    const int64_t g = obase + (int64_t)cnt;
    const int64_t q0 = g - (int64_t)(g & 7) > obase ? g - (int64_t)(g & 7) : obase;
    for (int64_t q = q0; q < g; ++q) out.store1(q, (uint16_t)hist((int)(g - q)));
    return rc == 0 && cnt == out_len ? 0 : -1;
}

// Output of the expand pass: u16 symbols in global memory (or a host buffer).
struct U16Out {
    IK_GLOBAL uint16_t* p;
    IK_HD uint16_t load(int64_t i) const { return p[i]; }
    IK_HD void store1(int64_t i, uint16_t v) const { p[i] = v; }
    IK_HD void store16(int64_t i, uint64_t lo, uint64_t hi) const {  // 8 symbols at i (a multiple of 8)
        IK_GLOBAL uint64_t* q = reinterpret_cast<IK_GLOBAL uint64_t*>(p + i);
        q[0] = lo;
        q[1] = hi;
    }
};

// Token input of the expand pass on the host (the GPU's reads 16-byte groups
// ahead: ik_png.hip TokInDev).
struct TokInHost {
    const uint16_t* p;
    uint32_t t = 0, tab = 0;
    IK_HD uint32_t next() { return p[t++]; }
    IK_HD void seek(uint32_t pos) { t = pos; }
    IK_HD void set_table(uint32_t pos) { tab = pos; }  // the block's literal table is at token pos
    IK_HD uint32_t table(uint32_t rank) const { return reinterpret_cast<const uint8_t*>(p + tab)[rank]; }
};

}  // namespace infl
}  // namespace ik
