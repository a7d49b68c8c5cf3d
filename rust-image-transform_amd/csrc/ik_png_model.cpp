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
#include <vector>

#include "ik_inflate.h"
#include "ik_png_plan.h"

using namespace ik;

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
    std::vector<int64_t> cand(nchunks, -1);
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
            if (kraft != 128 || !nz) continue;
            uint8_t tab[128];
            const bool fast = infl::dynamic_header_ok(words.data(), nbits, p, h, bits, tab);
            if (fast != infl::plausible_dynamic(words.data(), nbits, p)) return -9;  // the two checks must agree
            if (fast) {
                cand[c] = (int64_t)p;
                ++found;
                break;
            }
        }
    }
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

// the candidate test alone at one bit position (for the filter-strength test)
int ikm_plausible_dynamic(const uint8_t* z, size_t zlen, uint64_t bit) {
    std::vector<uint32_t> words((zlen + 3) / 4 + 8, 0);
    std::memcpy(words.data(), z, zlen);
    return infl::plausible_dynamic(words.data(), (uint64_t)zlen * 8, bit) ? 1 : 0;
}

}  // extern "C"
