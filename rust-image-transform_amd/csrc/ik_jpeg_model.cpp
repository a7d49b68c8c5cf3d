// ik_jpeg_model.cpp -- CPU model of the GPU self-synchronising JPEG entropy decoder
// (TEST INFRASTRUCTURE: built into libik_jpegmodel.so for the CPU test suite, never
// linked into the product).
//
// Runs the algorithm of ik_jpeg.hip's k_jsync_* kernels -- unstuffing, the sync
// pass with its warm-up, the fix rounds, the per-interval bases, the decode pass --
// on the CPU with the same ik_jpeg_sync.h code, and compares the coefficients with
// a plain serial decode of the same scan (interval by interval from its exact
// start), so that the tests can check the parallel machinery on many streams
// without a GPU and report how many lanes the warm-up synchronised.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ik_jpeg_sync.h"

using namespace ik;
using namespace ik::jsync;

namespace {

const uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    int maxcode[18] = {}, valptr[17] = {}, mincode[17] = {};
    uint8_t vals[256] = {};
    uint8_t look_len[512] = {}, look_val[512] = {};
};

bool build(const uint8_t* bits, const uint8_t* vals, int nvals, Huff& t) {
    t = Huff();
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
    code = 0;
    k = 0;
    for (int l = 1; l <= 9; ++l) {
        for (int i = 0; i < bits[l - 1]; ++i, ++k, ++code)
            for (int f = 0; f < (1 << (9 - l)); ++f) {
                t.look_len[(code << (9 - l)) | f] = (uint8_t)l;
                t.look_val[(code << (9 - l)) | f] = vals[k];
            }
        code <<= 1;
    }
    t.present = true;
    return true;
}

// the product's table layout (ik_jpeg_decode.cpp Decoder::tables)
void tables(const Huff* dc, const Huff* ac, JpegHuffTables& t) {
    std::memset(&t, 0, sizeof(t));
    for (int k = 0; k < 8; ++k) {
        const Huff& h = k < 4 ? dc[k] : ac[k - 4];
        for (int i = 0; i < 512; ++i) t.look[k][i] = (uint16_t)(h.look_len[i] << 8 | h.look_val[i]);
        std::memcpy(t.maxcode[k], h.maxcode, sizeof(h.maxcode));
        std::memcpy(t.valptr[k], h.valptr, sizeof(h.valptr));
        std::memcpy(t.mincode[k], h.mincode, sizeof(h.mincode));
        std::memcpy(t.vals[k], h.vals, sizeof(h.vals));
        int carry = 0;
        for (int l = 1; l <= 16; ++l) {
            if (h.maxcode[l] >= 0) carry = (h.maxcode[l] + 1) << (16 - l);
            t.lj[k][l] = carry;
        }
        if (k < 4) continue;
        for (int i = 0; i < 512; ++i) {
            const int L = h.look_len[i], rs = h.look_val[i], r = rs >> 4, sz = rs & 15;
            if (!L || !sz || L + sz > 9) continue;
            const int v = (i >> (9 - L - sz)) & ((1 << sz) - 1);
            const int val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;
            if (val < -128 || val > 127) continue;
            t.fast_ac[k - 4][i] = (int16_t)(val * 256 + r * 16 + L + sz);
        }
    }
}

struct Comp {
    int id = 0, h = 1, v = 1, td = 0, ta = 0, bw = 0, bh = 0, dw = 0, dh = 0;
    long long blk0 = 0;
};

// a baseline single-scan JPEG, parsed far enough for the entropy decoder
struct Jpeg {
    Huff dc[4], ac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, restart = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    long long nblocks = 0;
    std::vector<int> order;
    const uint8_t* scan = nullptr;
    size_t scan_len = 0;
    bool parse(const uint8_t* b, size_t n) {
        size_t p = 2;
        auto be16 = [&](size_t q) { return (int)b[q] << 8 | b[q + 1]; };
        while (p + 4 <= n) {
            if (b[p] != 0xFF) { ++p; continue; }
            const int m = b[p + 1];
            if (m == 0xFF) { ++p; continue; }
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7)) { p += 2; continue; }
            const int len = be16(p + 2);
            const uint8_t* s = b + p + 4;
            const uint8_t* se = b + p + 2 + len;
            if (m == 0xC4) {
                while (s < se) {
                    const int tc = s[0] >> 4, th = s[0] & 15;
                    int total = 0;
                    for (int i = 0; i < 16; ++i) total += s[1 + i];
                    if (!build(s + 1, s + 17, total, tc ? ac[th] : dc[th])) return false;
                    s += 17 + total;
                }
            } else if (m == 0xDD) {
                restart = be16(p + 4);
            } else if (m == 0xC0 || m == 0xC1) {
                H = be16(p + 5);
                W = be16(p + 7);
                const int nc = s[5];
                comps.resize(nc);
                for (int i = 0; i < nc; ++i) {
                    comps[i].id = s[6 + 3 * i];
                    comps[i].h = s[7 + 3 * i] >> 4;
                    comps[i].v = s[7 + 3 * i] & 15;
                    hmax = std::max(hmax, comps[i].h);
                    vmax = std::max(vmax, comps[i].v);
                }
                mcux = (W + 8 * hmax - 1) / (8 * hmax);
                mcuy = (H + 8 * vmax - 1) / (8 * vmax);
                for (auto& c : comps) {
                    c.bw = mcux * c.h;
                    c.bh = mcuy * c.v;
                    c.dw = (W * c.h + hmax - 1) / hmax;
                    c.dh = (H * c.v + vmax - 1) / vmax;
                    c.blk0 = nblocks;
                    nblocks += (long long)c.bw * c.bh;
                }
            } else if (m == 0xC2) {
                return false;  // progressive: not this decoder's
            } else if (m == 0xDA) {
                const int ns = s[0];
                for (int i = 0; i < ns; ++i) {
                    for (int k = 0; k < (int)comps.size(); ++k)
                        if (comps[k].id == s[1 + 2 * i]) {
                            comps[k].td = s[2 + 2 * i] >> 4;
                            comps[k].ta = s[2 + 2 * i] & 15;
                            order.push_back(k);
                        }
                }
                scan = se;
                // the scan ends at the first marker that is not RSTn (or stuffing)
                size_t q = (size_t)(se - b);
                while (q + 1 < n && !(b[q] == 0xFF && b[q + 1] != 0x00 && b[q + 1] != 0xFF &&
                                      !(b[q + 1] >= 0xD0 && b[q + 1] <= 0xD7)))
                    ++q;
                scan_len = (q + 1 < n ? q : n) - (size_t)(se - b);
                return true;
            }
            p += 2 + len;
        }
        return false;
    }
};

struct Model {
    Jpeg J;
    JpegHuffTables T;
    std::vector<uint32_t> words;
    std::vector<long long> ivl;
    std::vector<int> ivl_lane;
    Scan S{};
    long long total_mcu = 0;

    bool setup() {
        tables(J.dc, J.ac, T);
        const bool single = J.order.size() == 1;
        int bpm = 0;
        for (size_t i = 0; i < J.order.size(); ++i) {
            const Comp& c = J.comps[J.order[i]];
            const int nb = single ? 1 : c.h * c.v;
            for (int k = 0; k < nb; ++k) {
                if (bpm >= kMaxBPM) return false;
                S.comp_of[bpm] = (int)i;
                S.bx_of[bpm] = single ? 0 : k % c.h;
                S.by_of[bpm] = single ? 0 : k / c.h;
                ++bpm;
            }
            S.h[i] = c.h; S.v[i] = c.v; S.bw[i] = c.bw; S.td[i] = c.td; S.ta[i] = c.ta + 4;
            S.td[i] = c.td;
            S.blk0[i] = c.blk0;
        }
        // (S.ta holds the table index 4..7 in the combined table: see block())
        for (size_t i = 0; i < J.order.size(); ++i) S.ta[i] = J.comps[J.order[i]].ta;
        const Comp& c0 = J.comps[J.order[0]];
        const int sbw = (c0.dw + 7) / 8, sbh = (c0.dh + 7) / 8;
        total_mcu = single ? (long long)sbw * sbh : (long long)J.mcux * J.mcuy;
        S.bpm = bpm;
        S.mcux = J.mcux;
        S.single = single;
        S.single_bw = sbw;
        S.total_blocks = total_mcu * bpm;
        S.ivl_blocks = J.restart ? (long long)J.restart * bpm : S.total_blocks;
        // unstuff, byte by byte (the GPU's rule)
        std::vector<uint8_t> out;
        ivl.assign(1, 0);
        const uint8_t* b = J.scan;
        const size_t n = J.scan_len;
        for (size_t i = 0; i < n; ++i) {
            const int prev = i ? b[i - 1] : -1, cur = b[i], next = i + 1 < n ? b[i + 1] : -1;
            if (unstuff_bad(cur, next, i + 1 == n)) return false;
            if (unstuff_rst(cur, next)) ivl.push_back((long long)out.size() * 8);
            if (unstuff_keep(prev, cur, next, i + 1 == n)) out.push_back((uint8_t)cur);
        }
        const long long nbits = (long long)out.size() * 8;
        ivl.push_back(nbits);
        const long long want_ivl = J.restart ? (total_mcu + J.restart - 1) / J.restart : 1;
        if ((long long)ivl.size() - 1 != want_ivl) return false;
        words.assign((out.size() + 3) / 4 + kPadWords, 0u);
        for (size_t i = 0; i < out.size(); ++i) words[i >> 2] |= (uint32_t)out[i] << (24 - 8 * (i & 3));
        ivl_lane.assign(ivl.size(), 0);
        for (size_t k = 0; k + 1 < ivl.size(); ++k) {
            const long long bits = ivl[k + 1] - ivl[k];
            const int nl = bits > 0 ? (int)((bits + S.L - 1) / S.L) : 1;
            ivl_lane[k + 1] = ivl_lane[k] + nl;
        }
        S.words = words.data();
        S.ivl = ivl.data();
        S.nivl = (int)ivl.size() - 1;
        S.ivl_lane = ivl_lane.data();
        S.tabs = &T;
        return true;
    }
};

}  // namespace

extern "C" {

// Decode the scan of a baseline JPEG both ways and report:
// stats[0] lanes, [1] lanes inconsistent after the sync pass, [2] fix rounds,
// [3] blocks decoded by the sync pass + fix rounds (incl. warm-up), [4] total
// blocks, [5] 1 if the parallel coefficients equal the serial decode's,
// [6] intervals, [7] lanes re-decoded over all fix rounds, [8] longest fix chain.
// coef_out (may be null): the parallel decode's coefficients ([block][64]).
// Returns 0, or -1 when the stream is not a single-scan baseline JPEG the model takes.
int ikm_jsync_decode(const uint8_t* jpeg, size_t n, int lane_bits, int warm_bits, int16_t* coef_out, size_t coef_cap,
                     long long* stats) {
    Model M;
    M.S.L = lane_bits > 0 ? lane_bits : kLaneBits;
    M.S.W = warm_bits >= 0 ? warm_bits : kWarmBits;
    if (!M.J.parse(jpeg, n) || M.J.order.size() != M.J.comps.size() || !M.setup()) return -1;
    const Scan& S = M.S;
    const JpegHuffTables& T = M.T;
    const int nl = M.ivl_lane.back();
    // lane -> (interval, index)
    std::vector<int> lane_ivl(nl), lane_q(nl);
    for (int k = 0; k < S.nivl; ++k)
        for (int l = M.ivl_lane[k]; l < M.ivl_lane[k + 1]; ++l) { lane_ivl[l] = k; lane_q[l] = l - M.ivl_lane[k]; }
    long long decoded = 0;
    // 1. sync pass
    std::vector<LaneRec> R(nl);
    for (int l = 0; l < nl; ++l) {
        const LaneGeom g = lane_geom(S, lane_ivl[l], lane_q[l]);
        run_lane(S, T, kZz, g, warm_start(S, g), R[l]);
        decoded += R[l].work;
    }
    auto consistent = [&](int l) {
        if (lane_q[l] == 0) return true;
        return R[l - 1].exit != 0 && R[l].start == R[l - 1].exit;
    };
    long long bad0 = 0;
    for (int l = 0; l < nl; ++l) bad0 += !consistent(l);
    // 2. fix rounds (each reads the previous round's records)
    int rounds = 0;
    long long redone = 0;
    for (;;) {
        std::vector<int> todo;
        for (int l = 0; l < nl; ++l)
            if (!consistent(l) && R[l - 1].exit != 0) todo.push_back(l);
        if (todo.empty()) break;
        ++rounds;
        std::vector<LaneRec> prevR = R;
        for (int l : todo) {
            const LaneGeom g = lane_geom(S, lane_ivl[l], lane_q[l]);
            run_lane(S, T, kZz, g, prevR[l - 1].exit, R[l]);
            decoded += R[l].work;
            ++redone;
        }
        if (rounds > nl + 2) return -2;
    }
    // 3. bases per interval (cut the end padding's blocks), errors
    std::vector<long long> base(nl);
    std::vector<int> cnt(nl);
    std::vector<int> dcb(4 * (size_t)nl);
    bool ok = true;
    for (int k = 0; k < S.nivl && ok; ++k) {
        const long long want = k + 1 < S.nivl ? S.ivl_blocks : S.total_blocks - (long long)k * S.ivl_blocks;
        long long b = 0;
        int dc[4] = {0, 0, 0, 0};
        for (int l = M.ivl_lane[k]; l < M.ivl_lane[k + 1]; ++l) {
            if (!consistent(l)) { ok = false; break; }
            base[l] = (long long)k * S.ivl_blocks + b;
            for (int c = 0; c < 4; ++c) { dcb[4 * l + c] = dc[c]; dc[c] += R[l].dc[c]; }
            long long take = std::min<long long>(R[l].nblk, want - b);
            if (take < 0) take = 0;
            // a bad code within the interval's real blocks is an error
            if (R[l].err && R[l].err - 1 < take) { ok = false; break; }
            cnt[l] = (int)take;
            b += take;
        }
        if (b != want) ok = false;
    }
    // 4. decode pass
    std::vector<int16_t> par((size_t)M.J.nblocks * 64, 0);
    for (int l = 0; l < nl && ok; ++l) {
        if (!cnt[l]) continue;
        Bits br;
        const LaneGeom g = lane_geom(S, lane_ivl[l], lane_q[l]);
        br.init(S.words, st_bit(R[l].start), g.e);
        int j = st_j(R[l].start);
        int pred[4];
        for (int c = 0; c < 4; ++c) pred[c] = dcb[4 * l + c];
        for (int i = 0; i < cnt[l]; ++i) {
            const long long bi = block_index(S, base[l] + i);
            int16_t* blk = &par[(size_t)bi * 64];
            const int c = S.comp_of[j];
            int diff;
            if (!block<true>(br, T, kZz, S.td[c], S.ta[c], &diff, blk)) { ok = false; break; }
            pred[c] += diff;
            blk[0] = (int16_t)pred[c];
            j = j + 1 == S.bpm ? 0 : j + 1;
        }
    }
    // serial reference: every interval from its exact start
    std::vector<int16_t> ser((size_t)M.J.nblocks * 64, 0);
    bool sok = true;
    for (int k = 0; k < S.nivl && sok; ++k) {
        const long long want = k + 1 < S.nivl ? S.ivl_blocks : S.total_blocks - (long long)k * S.ivl_blocks;
        Bits br;
        br.init(S.words, (uint64_t)S.ivl[k], (uint64_t)S.ivl[k + 1]);
        int pred[4] = {0, 0, 0, 0};
        for (long long i = 0; i < want; ++i) {
            const long long b = (long long)k * S.ivl_blocks + i;
            const int j = (int)(b % S.bpm);
            const int c = S.comp_of[j];
            int16_t* blk = &ser[(size_t)block_index(S, b) * 64];
            int diff;
            if (!block<true>(br, T, kZz, S.td[c], S.ta[c], &diff, blk)) { sok = false; break; }
            pred[c] += diff;
            blk[0] = (int16_t)pred[c];
        }
    }
    if (stats) {
        stats[0] = nl;
        stats[1] = bad0;
        stats[2] = rounds;
        stats[3] = decoded;
        stats[4] = S.total_blocks;
        stats[5] = ok && sok && par == ser;
        stats[6] = S.nivl;
        stats[7] = redone;
        stats[8] = M.ivl_lane.back();
    }
    if (coef_out && ok) std::memcpy(coef_out, par.data(), std::min(coef_cap, par.size()) * sizeof(int16_t));
    return ok ? 0 : 1;
}

}  // extern "C"
