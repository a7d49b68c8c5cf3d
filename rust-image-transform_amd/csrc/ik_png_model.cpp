// ik_png_model.cpp -- CPU model of the GPU PNG inflate (TEST INFRASTRUCTURE: built
// into libik_pngmodel.so for the CPU test suite, never linked into the product).
//
// Runs the exact chunked algorithm of ik_png.hip / ik_png_decode.cpp -- candidate
// search per chunk, decode rounds (token streams) with the chain check, expand
// with window markers, marker resolution -- on the CPU with the same ik_inflate.h code, so that the
// tests can compare it with zlib on many streams without a GPU.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "ik_crc.h"
#include "ik_inflate.h"
#include "ik_png_gather.h"
#include "ik_png_plan.h"
#include "ik_png_wave.h"
#include "ik_unfilter.h"

using namespace ik;

namespace {
// the window of infl::dynamic_header_win over host words (the GPU's is LDS, k_png_find)
struct HostWin {
    const uint32_t* W;
    uint64_t wend;
    uint32_t w[32];
    void fetch(uint64_t base) {
        for (int k = 0; k < 32; ++k) w[k] = base + k < wend ? W[base + k] : 0u;
    }
    uint32_t word(uint32_t k) const { return w[k]; }
};
// 9 bits (three code-length-code lengths) -> sum of 2^(7 - len) (k_png_find's s_kraft)
struct KraftTab {
    uint8_t t[512];
    KraftTab() {
        for (int v = 0; v < 512; ++v) {
            uint32_t k = 0;
            for (int f = 0; f < 3; ++f) {
                const uint32_t l = ((uint32_t)v >> (3 * f)) & 7u;
                k += l ? (128u >> l) : 0u;
            }
            t[v] = (uint8_t)k;
        }
    }
};
const KraftTab g_kraft;
const uint8_t* const kraft_tab = g_kraft.t;

// the GPU block search (k_png_find) restated: per chunk, the first bit offset whose
// dynamic header passes every check; cand[0] = the first block.  Returns the
// candidates found, or < 0 if two of the checks disagree.
int find_candidates(const std::vector<uint32_t>& words, uint64_t nbits, size_t chunk_bytes, std::vector<int64_t>& cand) {
    const uint64_t cbits = (uint64_t)chunk_bytes * 8;
    const uint64_t nchunks = (nbits + cbits - 1) / cbits;
    cand.assign(nchunks, -1);
    cand[0] = 16;
    int found = 0;
    for (uint64_t c = 1; c < nchunks; ++c) {
        const uint64_t e = (c + 1) * cbits < nbits ? (c + 1) * cbits : nbits;
        for (uint64_t p = c * cbits; p < e; ++p) {
            // the GPU finder's filters: BTYPE/HLIT/HDIST, complete code-length code, streaming check
            const uint64_t wi = p >> 5;
            const uint64_t v = ((uint64_t)words[wi] | ((uint64_t)words[wi + 1] << 32)) >> (p & 31);
            const uint32_t h = (uint32_t)v;
            if (((h >> 1) & 3u) != 2u || ((h >> 3) & 31u) > 29u || ((h >> 8) & 31u) > 29u) continue;
            const int ncode = (int)((h >> 13) & 15u) + 4;
            const uint64_t q = p + 17, qi = q >> 5;
            const uint32_t sh = (uint32_t)(q & 31);
            const uint64_t lo = (uint64_t)words[qi] | ((uint64_t)words[qi + 1] << 32), hi = words[qi + 2];
            const uint64_t bits = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
            int kraft = 0, nz = 0;
            for (int i = 0; i < ncode; ++i) {
                const int l = (int)((bits >> (3 * i)) & 7u);
                if (l) { kraft += 128 >> l; ++nz; }
            }
            if ((infl::cl_kraft_top(bits, ncode, kraft_tab) == 128u) != (kraft == 128 && nz)) return -10;
            if (kraft != 128 || !nz) continue;
            uint8_t tab[128];
            const bool fast = infl::dynamic_header_ok(words.data(), nbits, p, h, bits, tab);
            if (fast != infl::plausible_dynamic(words.data(), nbits, p)) return -9;  // the checks must agree
            HostWin hw{words.data(), (nbits >> 5) + 4, {}};
            if (fast != infl::dynamic_header_win(p, h, bits, hw)) return -11;  // (the GPU search's check)
            if (fast) {
                cand[c] = (int64_t)p;
                ++found;
                break;
            }
        }
    }
    return found;
}

}  // namespace

extern "C" {

// zlib stream -> inflated bytes through the chunked parallel algorithm.
// stats (10 ints): chunks, candidates, lanes, rounds, markers, dropped
// candidates, zlib header bits, status of the chain check, token region overflows
int ikm_inflate_chunked(const uint8_t* z, size_t zlen, size_t chunk_bytes, uint8_t* out, size_t out_cap,
                        uint64_t* out_len, int* stats) {
    for (int i = 0; i < 10; ++i) stats[i] = 0;
    if (zlen < 2) return -1;
    if ((z[0] & 15) != 8 || ((z[0] << 8) | z[1]) % 31 || (z[1] & 0x20)) return -1;  // CM=8, FCHECK, no FDICT
    const uint64_t nbits = (uint64_t)zlen * 8;
    std::vector<uint32_t> words((zlen + 3) / 4 + 8, 0);
    std::memcpy(words.data(), z, zlen);
    const uint64_t cbits = (uint64_t)chunk_bytes * 8;
    const uint64_t nchunks = (nbits + cbits - 1) / cbits;
    std::vector<int64_t> cand;
    int found = find_candidates(words, nbits, chunk_bytes, cand);
    if (found < 0) return found;
    stats[0] = (int)nchunks;
    stats[1] = found;
    stats[6] = 16;
    pngplan::Lanes L;
    pngplan::build(cand, L);
    const size_t nl0 = L.start.size();
    uint32_t cm[infl::kCanonWords];
    // token regions: capacity from the lane's compressed bits (as the GPU path),
    // grown when a lane overflows
    std::vector<std::vector<uint16_t>> tok(L.start.size());
    int st;
    int overflows = 0;
    for (;;) {
        for (size_t i = 0; i < L.start.size(); ++i) {
            if (!L.dirty[i]) continue;
            const uint64_t bits = (L.stop[i] == ~0ull ? nbits : L.stop[i]) - L.start[i];
            const uint32_t cap = infl::tok_capacity(bits, L.big[i] != 0);
            tok[i].assign((size_t)cap + infl::kTokSlack, 0);
            infl::TokOut to{tok[i].data()};
            infl::decode_lane_tok(words.data(), nbits, L.start[i], L.stop[i], cm, to, cap, i == 0, out_cap, L.res[i],
                                  infl::Win{});
            if (L.res[i].status == infl::kLaneOverflow) {
                ++overflows;
                if (L.big[i]) {
                    // past the large region too: garbage from a false start, or a
                    // stream of tiny blocks (their tables); the chain check decides
                    L.res[i].status = infl::kLaneCorrupt;
                } else {
                    L.big[i] = 1;
                    continue;  // still dirty: again with the large region
                }
            }
            L.dirty[i] = 0;
        }
        if (getenv("IKM_DEBUG"))
            for (size_t i = 0; i < L.start.size(); ++i)
                fprintf(stderr, "lane %zu start %llu stop %llu end %llu len %llu tok %u status %d final %d\n", i,
                        (unsigned long long)L.start[i], (unsigned long long)L.stop[i],
                        (unsigned long long)L.res[i].end_bit, (unsigned long long)L.res[i].out_len, L.res[i].ntok,
                        L.res[i].status, L.res[i].final_block);
        bool pending = false;
        for (size_t i = 0; i < L.start.size(); ++i) pending = pending || L.dirty[i];
        if (pending) continue;  // overflowed lanes first
        // the chain check drops successors: keep the per-lane vectors in step
        std::vector<uint64_t> before(L.start);
        st = pngplan::check(L);
        if (L.start.size() != before.size()) {
            std::vector<std::vector<uint16_t>> t2;
            for (size_t i = 0, k = 0; i < before.size(); ++i)
                if (k < L.start.size() && L.start[k] == before[i]) {
                    t2.push_back(std::move(tok[i]));
                    ++k;
                }
            tok.swap(t2);
        }
        if (st != 1) break;
    }
    stats[8] = overflows;
    stats[2] = (int)L.start.size();
    stats[3] = L.rounds;
    stats[5] = (int)(nl0 - L.start.size());
    stats[7] = st;
    if (st) return -2;
    std::vector<int64_t> obase;
    uint64_t total;
    pngplan::offsets(L, obase, &total);
    if (total > out_cap) return -3;
    std::vector<uint16_t> u16(total + 16);
    for (size_t i = 0; i < L.start.size(); ++i) {
        infl::TokInHost tin{tok[i].data()};
        if (infl::expand_lane(tin, L.res[i].ntok, infl::U16Out{u16.data()}, obase[i], L.res[i].out_len)) return -4;
    }
    // page -> decoder table (as the host builds it for the GPU resolve pass)
    const int shift = 12;
    std::vector<int> pages((total >> shift) + 1);
    for (size_t pg = 0, ln = 0; pg < pages.size(); ++pg) {
        while (ln + 1 < obase.size() && (uint64_t)obase[ln + 1] <= (pg << shift)) ++ln;
        pages[pg] = (int)ln;
    }
    int markers = 0;
    for (uint64_t q = 0; q < total; ++q) {
        if (u16[q] >= 256) ++markers;
        const int v = infl::resolve_at(u16.data(), obase.data(), (int)obase.size(), pages.data(), shift, (int64_t)q);
        if (v < 0) return -5;
        out[q] = (uint8_t)v;
    }
    stats[4] = markers;
    *out_len = total;
    return 0;
}

// The same stream through the wave decoder's algorithm (ik_png_wave.h: one lane
// = whole blocks decoded by up to 64 self-synchronising sub-lanes with shared
// lookup tables, its tokens in pieces), then the unchanged expand / resolve.
// stats (20 x u64): chunks, candidates, lanes, rounds, overflows, windows, sub-lane
// passes, redo passes, fix rounds, most fix rounds of one window, blocks, decoded
// symbol bits, chain-check status, token-region tokens used, markers, sub-lane steps,
// wave steps (the passes' longest sub-lanes), expand units.  IKM_WARM / IKM_EST:
// warm-up and block-end estimate overrides (the model's sweeps).
int ikm_inflate_wave(const uint8_t* z, size_t zlen, size_t chunk_bytes, uint8_t* out, size_t out_cap,
                     uint64_t* out_len, uint64_t* stats) {
    for (int i = 0; i < 20; ++i) stats[i] = 0;
    if (const char* e = getenv("IKM_EST")) {  // model experiments: mul/1024, add, min tail (bits)
        long a = 1024, b = 4096, c = 16384;
        if (sscanf(e, "%ld,%ld,%ld", &a, &b, &c) == 3) { wave::g_est_mul = a; wave::g_est_add = b; wave::g_min_tail = c; }
    }
    if (zlen < 2) return -1;
    if ((z[0] & 15) != 8 || ((z[0] << 8) | z[1]) % 31 || (z[1] & 0x20)) return -1;
    const uint64_t nbits = (uint64_t)zlen * 8;
    std::vector<uint32_t> words((zlen + 3) / 4 + 8, 0);
    std::memcpy(words.data(), z, zlen);
    std::vector<int64_t> cand;
    const int found = find_candidates(words, nbits, chunk_bytes, cand);
    if (found < 0) return found;
    stats[0] = cand.size();
    stats[1] = (uint64_t)found;
    struct W {
        const uint32_t* words;
        uint64_t nw;
        uint64_t operator()(uint64_t pos) const {
            const uint64_t wi = pos >> 5;
            const uint32_t sh = (uint32_t)(pos & 31);
            auto rd = [&](uint64_t i) -> uint64_t { return i < nw ? words[i] : 0u; };
            const uint64_t lo = rd(wi) | (rd(wi + 1) << 32);
            return sh ? (lo >> sh) | (rd(wi + 2) << (64 - sh)) : lo;
        }
    } win{words.data(), (nbits >> 5) + 1};
    pngplan::Lanes L;
    pngplan::build(cand, L);
    // tokens and pieces by lane start (the chain check drops and splits lanes)
    std::map<uint64_t, std::vector<uint16_t>> tok;
    std::map<uint64_t, std::vector<std::pair<uint32_t, uint32_t>>> pieces;  // (base, vstart)
    std::map<uint64_t, std::vector<std::pair<uint32_t, uint32_t>>> units;   // (first piece, output before it)
    wave::Stats ws;
    int st, overflows = 0;
    for (;;) {
        for (size_t i = 0; i < L.start.size(); ++i) {
            if (!L.dirty[i]) continue;
            const uint64_t end = L.stop[i] == ~0ull ? nbits : L.stop[i];
            const uint64_t cap = wave::region_capacity(end > L.start[i] ? end - L.start[i] : 0, L.big[i] != 0);
            std::vector<uint16_t>& t = tok[L.start[i]];
            t.assign(cap, 0);
            static const uint64_t warm = getenv("IKM_WARM") ? strtoull(getenv("IKM_WARM"), nullptr, 10) : wave::kWarmBits;
            wave::lane_host(win, nbits, L.start[i], L.stop[i], L.big[i] != 0, t.data(), cap, L.res[i],
                            pieces[L.start[i]], units[L.start[i]], &ws, warm);
            if (L.res[i].status == infl::kLaneOverflow) {
                ++overflows;
                if (L.big[i]) {
                    L.res[i].status = infl::kLaneCorrupt;
                } else {
                    L.big[i] = 1;
                    continue;
                }
            }
            L.dirty[i] = 0;
        }
        if (getenv("IKM_DEBUG"))
            for (size_t i = 0; i < L.start.size(); ++i)
                fprintf(stderr, "lane %zu start %llu stop %llu end %llu len %llu pieces %u status %d final %d\n", i,
                        (unsigned long long)L.start[i], (unsigned long long)L.stop[i],
                        (unsigned long long)L.res[i].end_bit, (unsigned long long)L.res[i].out_len,
                        (unsigned)pieces[L.start[i]].size(),
                        L.res[i].status, L.res[i].final_block);
        bool pending = false;
        for (size_t i = 0; i < L.start.size(); ++i) pending = pending || L.dirty[i];
        if (pending) continue;
        st = pngplan::check(L);
        if (st != 1) break;
    }
    stats[2] = L.start.size();
    stats[3] = (uint64_t)L.rounds;
    stats[4] = (uint64_t)overflows;
    stats[5] = ws.windows;
    stats[6] = ws.sub_passes;
    stats[7] = ws.redo_passes;
    stats[8] = ws.fix_rounds;
    stats[9] = ws.max_rounds;
    stats[10] = ws.blocks;
    stats[11] = ws.symbols_bits;
    stats[12] = (uint64_t)(int64_t)st;
    stats[15] = ws.steps;
    stats[16] = ws.wave_steps;
    if (getenv("IKM_PROF"))
        fprintf(stderr, "[model] first-pass wave steps %llu: any slow literal %.1f%%, slow distance %.1f%%, group store "
                "%.1f%%, match %.1f%%, warm-up %.1f%%\n", (unsigned long long)ws.prof[7],
                100.0 * ws.prof[0] / ws.prof[7], 100.0 * ws.prof[1] / ws.prof[7], 100.0 * ws.prof[2] / ws.prof[7],
                100.0 * ws.prof[3] / ws.prof[7], 100.0 * ws.prof[4] / ws.prof[7]);
    if (st) return -2;
    std::vector<int64_t> obase;
    uint64_t total;
    pngplan::offsets(L, obase, &total);
    if (total > out_cap) return -3;
    std::vector<uint16_t> u16(total + 16);
    // the expand units (ik_png_wave.h kUnitMinTok): each unit's pieces in order, as
    // the GPU expand pass reads them, expanded at the unit's output offset (window
    // markers for copies before the unit); the resolve tables are per unit
    std::vector<int64_t> uob;
    for (size_t i = 0; i < L.start.size(); ++i) {
        const std::vector<std::pair<uint32_t, uint32_t>>& pt = pieces[L.start[i]];
        const std::vector<std::pair<uint32_t, uint32_t>>& ut = units[L.start[i]];
        const std::vector<uint16_t>& t = tok[L.start[i]];
        if (ut.empty() && L.res[i].out_len) return -4;
        for (size_t u = 0; u < ut.size(); ++u) {
            const uint32_t p0 = ut[u].first, p1 = u + 1 < ut.size() ? ut[u + 1].first : (uint32_t)pt.size();
            const uint64_t o0 = ut[u].second, o1 = u + 1 < ut.size() ? ut[u + 1].second : L.res[i].out_len;
            if (p0 > p1 || p1 > pt.size() || o0 > o1) return -4;
            std::vector<uint16_t> cat;
            for (uint32_t k = p0; k < p1; ++k) {
                const uint32_t n = (k + 1 < pt.size() ? pt[k + 1].second : L.res[i].ntok) - pt[k].second;
                cat.insert(cat.end(), t.begin() + pt[k].first, t.begin() + pt[k].first + n);
            }
            stats[13] += cat.size();
            stats[17] += 1;
            for (size_t q = 0; q + 1 < cat.size(); ++q) {  // match profile: near (<= 1024 back) / far, their lengths
                const uint32_t v = cat[q];
                if ((v & 0xFF00u) != infl::kTokMatch) continue;
                const uint32_t len = (v & 255u) + 3, d = (uint32_t)cat[q + 1] + 1;
                stats[d <= 1024 ? 18 : 19] += 1;
                if (getenv("IKM_PROF")) {
                    static uint64_t hist[8] = {0};
                    hist[d <= 4 ? 0 : d <= 64 ? 1 : d <= 1024 ? 2 : d <= 16384 ? 3 : d <= 16388 ? 4 : 5] += 1;
                    hist[6] += len;
                    hist[7] += 1;
                    if ((hist[7] & ((1u << 16) - 1)) == 0)
                        fprintf(stderr, "[model] matches %llu: d<=4 %llu, <=64 %llu, <=1024 %llu, <=16384 %llu, 16385-16388 %llu, "
                                "farther %llu; mean length %.1f\n", (unsigned long long)hist[7], (unsigned long long)hist[0],
                                (unsigned long long)hist[1], (unsigned long long)hist[2], (unsigned long long)hist[3],
                                (unsigned long long)hist[4], (unsigned long long)hist[5], (double)hist[6] / hist[7]);
                }
                ++q;
            }
            cat.resize(cat.size() + 16, (uint16_t)infl::kTokPad);
            infl::TokInHost tin{cat.data()};
            const int64_t ob = obase[i] + (int64_t)o0;
            uob.push_back(ob);
            if (infl::expand_lane(tin, (uint32_t)(cat.size() - 16), infl::U16Out{u16.data()}, ob, o1 - o0)) {
                if (getenv("IKM_DEBUG"))
                    fprintf(stderr, "lane %zu unit %zu/%zu expand failed: tokens %zu, out %llu\n", i, u, ut.size(),
                            cat.size() - 16, (unsigned long long)(o1 - o0));
                return -4;
            }
        }
    }
    obase.swap(uob);
    const int shift = 12;
    std::vector<int> pages((total >> shift) + 1);
    for (size_t pg = 0, ln = 0; pg < pages.size(); ++pg) {
        while (ln + 1 < obase.size() && (uint64_t)obase[ln + 1] <= (pg << shift)) ++ln;
        pages[pg] = (int)ln;
    }
    uint64_t markers = 0;
    for (uint64_t q = 0; q < total; ++q) {
        if (u16[q] >= 256) ++markers;
        const int v = infl::resolve_at(u16.data(), obase.data(), (int)obase.size(), pages.data(), shift, (int64_t)q);
        if (v < 0) return -5;
        out[q] = (uint8_t)v;
    }
    stats[14] = markers;
    *out_len = total;
    return 0;
}

// The upload gather pass (ik_png.hip k_png_gather + k_png_crc_check) on the host:
// the same plan (ik_png_gather.h), the same per-thread split (256 B per thread,
// bytes until the destination is word aligned, then words), the same tree join of
// the 256 partial CRCs and the same chunk check.  file: a whole PNG file as
// uploaded at raw offset `raw_off` (the destination alignment follows z_off).
// Writes the assembled zlib stream + `tail` zero bytes to stream[z_off ..];
// bad[k] = 1 for each IDAT chunk whose CRC does not match; returns the number of
// IDAT chunks (-1 on a malformed chunk walk).
int ikm_gather_check(const uint8_t* file, size_t len, uint64_t z_off, uint32_t tail, uint8_t* stream, size_t cap,
                     int* bad, int bad_cap) {
    auto be32 = [](const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; };
    std::vector<std::pair<uint64_t, uint32_t>> idat;
    size_t pos = 8;
    while (pos + 12 <= len) {
        const uint32_t n = be32(file + pos);
        if (n > len - pos - 12) return -1;
        if (!std::memcmp(file + pos + 4, "IDAT", 4) && n) idat.emplace_back((uint64_t)(pos + 8), n);
        if (!std::memcmp(file + pos + 4, "IEND", 4)) break;
        pos += 12 + n;
    }
    std::vector<PngGatherPiece> pieces;
    std::vector<PngCrcChunk> chunks;
    png_gather_plan(0, idat, z_off, tail, 0, pieces, chunks);
    uint32_t t[1024], x2n[32], level[8];
    for (uint32_t i = 0; i < 256; ++i) t[i] = crc::table_entry(i);
    for (int sl = 1; sl < 4; ++sl)
        for (int i = 0; i < 256; ++i) t[256 * sl + i] = (t[256 * (sl - 1) + i] >> 8) ^ t[t[256 * (sl - 1) + i] & 255u];
    crc::x2n_table(x2n);
    for (int k = 0; k < 8; ++k) level[k] = crc::x8n((uint64_t)256 << k, x2n);
    std::vector<uint32_t> piece_crc(2 * pieces.size());
    for (size_t b = 0; b < pieces.size(); ++b) {
        const PngGatherPiece& P = pieces[b];
        if (P.dst + P.len > cap) return -1;
        uint32_t sc[256], sl[256];
        for (uint32_t tid = 0; tid < 256; ++tid) {
            const uint32_t b0 = 256u * tid;
            const uint32_t n = P.len > b0 ? (P.len - b0 < 256u ? P.len - b0 : 256u) : 0u;
            uint32_t c = ~0u;
            uint8_t* dp = stream + P.dst + b0;
            if (n && P.src == kPngNoSrc) {
                std::memset(dp, 0, n);
            } else if (n) {
                const uint8_t* sp = file + P.src + b0;
                uint32_t i = 0;
                const uint32_t mis = (uint32_t)((P.dst + b0) & 3u);
                const uint32_t pre = mis ? (4u - mis < n ? 4u - mis : n) : 0u;
                for (; i < pre; ++i) { dp[i] = sp[i]; c = crc::step_byte(c, sp[i], t); }
                for (; i + 4 <= n; i += 4) {
                    uint32_t v;
                    std::memcpy(&v, sp + i, 4);
                    std::memcpy(dp + i, &v, 4);
                    c = crc::step_word(c, v, t);
                }
                for (; i < n; ++i) { dp[i] = sp[i]; c = crc::step_byte(c, sp[i], t); }
            }
            sc[tid] = ~c;
            sl[tid] = n;
        }
        for (int k = 0; k < 8; ++k) {
            const int stride = 1 << k;
            for (int tid = 0; tid < 256; tid += 2 * stride) {
                const uint32_t rl = sl[tid + stride];
                if (!rl) continue;
                const uint32_t op = rl == (256u << k) ? level[k] : crc::x8n(rl, x2n);
                sc[tid] = crc::combine_op(sc[tid], sc[tid + stride], op);
                sl[tid] += rl;
            }
        }
        piece_crc[2 * b] = sc[0];
        piece_crc[2 * b + 1] = sl[0];
    }
    uint32_t cidat = ~0u;
    for (const char ch : {'I', 'D', 'A', 'T'}) cidat = crc::step_byte(cidat, (uint8_t)ch, t);
    cidat = ~cidat;
    for (size_t k = 0; k < chunks.size(); ++k) {
        uint32_t c = cidat;
        for (uint32_t p = chunks[k].piece0; p < chunks[k].piece0 + chunks[k].npieces; ++p)
            c = crc::combine_op(c, piece_crc[2 * p], crc::x8n(piece_crc[2 * p + 1], x2n));
        if ((int)k < bad_cap) bad[k] = c != be32(file + chunks[k].crc_at);
    }
    return (int)chunks.size();
}

// finished CRC-32 of data split into pieces / 256-B runs and joined (ik_crc.h), for
// direct comparison with zlib.crc32
uint32_t ikm_crc32_joined(const uint8_t* data, size_t len, size_t run) {
    uint32_t t[1024], x2n[32];
    for (uint32_t i = 0; i < 256; ++i) t[i] = crc::table_entry(i);
    for (int sl = 1; sl < 4; ++sl)
        for (int i = 0; i < 256; ++i) t[256 * sl + i] = (t[256 * (sl - 1) + i] >> 8) ^ t[t[256 * (sl - 1) + i] & 255u];
    crc::x2n_table(x2n);
    uint32_t acc = 0;
    for (size_t o = 0; o < len; o += run) {
        const size_t n = len - o < run ? len - o : run;
        uint32_t c = ~0u;
        size_t i = 0;
        for (; i + 4 <= n; i += 4) {
            uint32_t v;
            std::memcpy(&v, data + o + i, 4);
            c = crc::step_word(c, v, t);
        }
        for (; i < n; ++i) c = crc::step_byte(c, data[o + i], t);
        acc = crc::combine_op(acc, ~c, crc::x8n(n, x2n));
    }
    return acc;
}

// the candidate test alone at one bit position (for the filter-strength test)
int ikm_plausible_dynamic(const uint8_t* z, size_t zlen, uint64_t bit) {
    std::vector<uint32_t> words((zlen + 3) / 4 + 8, 0);
    std::memcpy(words.data(), z, zlen);
    return infl::plausible_dynamic(words.data(), (uint64_t)zlen * 8, bit) ? 1 : 0;
}

}  // extern "C"

// unfilter_word (ik_unfilter.h, the GPU's word-at-a-time row filters for 4- and
// 8-byte pixels) against png's byte-wise definition, exhaustively: every (a, b, c)
// byte triple under every filter type, four different triples per word (so a
// carry or borrow between bytes shows up), raw bytes from a fixed sequence.
// Returns the number of mismatching bytes.
extern "C" long ikm_unfilter_word_check(void) {
    auto ref = [](int ft, int x, int a, int b, int c) {
        int p = 0;
        if (ft == 1) p = a;
        else if (ft == 2) p = b;
        else if (ft == 3) p = (a + b) >> 1;
        else if (ft == 4) {
            const int pa = std::abs(b - c), pb = std::abs(a - c), pc = std::abs(a + b - 2 * c);
            p = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
        }
        return (x + p) & 255;
    };
    long bad = 0;
    uint32_t seq = 12345u;
    for (int ft = 0; ft <= 4; ++ft) {
        const uint32_t ms = ft == 1 ? ~0u : 0u, mu = ft == 2 ? ~0u : 0u, mv = ft == 3 ? ~0u : 0u, mp = ft == 4 ? ~0u : 0u;
        for (uint32_t t = 0; t < (1u << 24); t += 4) {
            uint32_t A = 0, B = 0, C = 0, X = 0;
            int av[4], bv[4], cv[4], xv[4];
            for (int k = 0; k < 4; ++k) {
                const uint32_t q = (t + (uint32_t)k * 0x40404u + (uint32_t)k) & 0xFFFFFFu;  // a different triple per byte
                av[k] = (int)(q & 255u);
                bv[k] = (int)((q >> 8) & 255u);
                cv[k] = (int)((q >> 16) & 255u);
                seq = seq * 1103515245u + 12345u;
                xv[k] = (int)((seq >> 16) & 255u);
                A |= (uint32_t)av[k] << (8 * k);
                B |= (uint32_t)bv[k] << (8 * k);
                C |= (uint32_t)cv[k] << (8 * k);
                X |= (uint32_t)xv[k] << (8 * k);
            }
            const uint32_t got = ik::unfilter_word(X, A, B, C, ms, mu, mv, mp);
            for (int k = 0; k < 4; ++k)
                bad += (int)((got >> (8 * k)) & 255u) != ref(ft, xv[k], av[k], bv[k], cv[k]);
        }
    }
    return bad;
}

// infl::cl_kraft_top (the block search's Kraft sum with the absent code-length
// lengths shifted out) against the plain sum over the ncode lengths, on pseudo-
// random 57-bit fields with random garbage above them.  Returns the mismatches.
extern "C" long ikm_cl_kraft_check(long n) {
    uint8_t T[512];
    for (int v = 0; v < 512; ++v) {
        uint32_t k = 0;
        for (int f = 0; f < 3; ++f) {
            const uint32_t l = ((uint32_t)v >> (3 * f)) & 7u;
            k += l ? (128u >> l) : 0u;
        }
        T[v] = (uint8_t)k;
    }
    uint64_t x = 0x9E3779B97F4A7C15ull;
    long bad = 0;
    for (long t = 0; t < n; ++t) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        uint64_t cl = x;
        if (t & 1) cl &= 0x1249249249249249ull * 3;  // many short lengths: sums near 128 more often
        for (int ncode = 4; ncode <= 19; ++ncode) {
            uint32_t ref = 0;
            for (int i = 0; i < ncode; ++i) {
                const uint32_t l = (uint32_t)(cl >> (3 * i)) & 7u;
                ref += l ? (128u >> l) : 0u;
            }
            if (infl::cl_kraft_top(cl, ncode, (const uint8_t*)T) != ref) ++bad;
        }
    }
    return bad;
}
