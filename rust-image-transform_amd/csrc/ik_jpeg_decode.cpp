// ik_jpeg_decode.cpp -- JPEG branch of decode_image (reference src/transform.rs:31 ->
// image 0.25.8 -> zune-jpeg 0.4.21, Cargo.lock:3106), host half.
//
// The host parses the markers and runs the Huffman entropy decoder into a dense
// block-coefficient image (quantised int16, natural order, one plane of 8x8
// blocks per component): baseline sequential (SOF0/SOF1, interleaved or not) and
// progressive (SOF2: DC first/refine, AC first/refine with EOB runs), restart
// intervals, 8-bit, 1 (gray -> L8), 3 (YCbCr -> Rgb8, or RGB for Adobe
// transform 0) or 4 components (CMYK / YCCK -> Rgb8).  Reconstruction --
// dequantise, IDCT, chroma upsampling, colour conversion -- runs on the GPU
// (ik_jpeg.hip) straight into the device image, by default as zune-jpeg 0.4.21
// does it (restated, parity unpinned: no crate sources or outputs here; equal to
// oracle/jpeg_dec.c), or as libjpeg-turbo does (bit-exact with Pillow) --
// ik_set_jpeg_reconstruction.  Arithmetic-coded, lossless, hierarchical and
// 12-bit JPEGs report IK_ERR_UNSUPPORTED.
#include <algorithm>
#include <thread>
#include <memory>
#include <atomic>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {
namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct HuffTable {
    bool present = false;
    // canonical decode: maxcode[l], valptr[l], mincode[l]; plus a 9-bit lookahead
    int maxcode[18] = {}, valptr[17] = {}, mincode[17] = {};
    uint8_t vals[256] = {};
    uint8_t look_len[512] = {}, look_val[512] = {};
};

bool build_huff(const uint8_t* bits, const uint8_t* vals, int nvals, HuffTable& t) {
    t = HuffTable();
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
    // lookahead for codes up to 9 bits
    code = 0;
    k = 0;
    for (int l = 1; l <= 9; ++l) {
        for (int i = 0; i < bits[l - 1]; ++i, ++k, ++code) {
            const int shift = 9 - l;
            for (int f = 0; f < (1 << shift); ++f) {
                t.look_len[(code << shift) | f] = (uint8_t)l;
                t.look_val[(code << shift) | f] = vals[k];
            }
        }
        code <<= 1;
    }
    t.present = true;
    return true;
}

struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc = 0;
    int n = 0;
    bool marker_hit = false;
    void fill() {
        while (n <= 56) {
            uint8_t b = 0;
            if (!marker_hit && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const uint8_t nx = p + 1 < end ? p[1] : 0;
                    if (nx == 0x00) { p += 2; }
                    else { marker_hit = true; b = 0; }  // feed zeros past a marker
                } else {
                    ++p;
                }
            }
            acc |= (uint64_t)b << (56 - n);
            n += 8;
        }
    }
    inline int peek(int k) { if (n < k) fill(); return (int)(acc >> (64 - k)); }
    inline void skip(int k) { acc <<= k; n -= k; }
    inline int get(int k) { if (!k) return 0; const int v = peek(k); skip(k); return v; }
    void reset_at_marker() { acc = 0; n = 0; marker_hit = false; }
};

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

int decode_symbol(BitReader& br, const HuffTable& t) {
    const int look = br.peek(9);
    const int l = t.look_len[look];
    if (l) { br.skip(l); return t.look_val[look]; }
    int code = br.peek(16);
    for (int len = 10; len <= 16; ++len) {
        const int c = code >> (16 - len);
        if (t.maxcode[len] >= 0 && c <= t.maxcode[len] && c >= t.mincode[len]) {
            br.skip(len);
            return t.vals[t.valptr[len] + c - t.mincode[len]];
        }
    }
    return -1;
}

struct Component {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0;    // blocks across/down, padded to whole MCUs
    int dw = 0, dh = 0;    // downsampled width/height (libjpeg downsampled_width/height)
    size_t blk0 = 0;       // first block in the coefficient image
    int pred = 0;
};

const char* const kFmtErr = "Format error decoding Jpeg";

// Restart-free baseline scans on the GPU (self-synchronising decoding, run_seq);
// IK_JPEG_SEQ=0 keeps them on the host entropy decoder.
bool seq_enabled() {
    static const bool on = [] {
        const char* e = getenv("IK_JPEG_SEQ");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}
constexpr size_t kSeqMinBytes = 32 << 10;  // smaller scans: the host decoder is faster

// Progressive scans with restart intervals on the GPU (k_jpeg_prog);
// IK_JPEG_PROG=0 keeps them on the host entropy decoder.
bool prog_enabled() {
    static const bool on = [] {
        const char* e = getenv("IK_JPEG_PROG");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}

struct Decoder {
    const uint8_t* b;
    const uint8_t* end;
    uint16_t qt[4][64] = {};
    HuffTable dc[4], ac[4];
    std::vector<Component> comps;
    int width = 0, height = 0, restart = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool have_frame = false, progressive = false, adobe = false;
    int adobe_transform = -1;
    std::vector<int16_t> coef;  // [block][64], natural order, quantised (host-decoded scans only)
    size_t nblocks = 0;
    int eobrun = 0;
    // GPU entropy decoding of a baseline scan with restart intervals: the scan is
    // recorded here (segment starts = first byte after each RSTn) instead of decoded
    bool try_gpu = false, deferred = false, need_host = false, scanned = false;
    const uint8_t* gpu_data = nullptr;
    std::vector<unsigned> gpu_segs;
    JpegScanArgs gpu_scan{};
    // progressive scans with restart intervals, recorded for k_jpeg_prog (all of
    // the image's scans, in order: one the GPU cannot take sends the image to the
    // host decoder, or keeps it there from the first scan on)
    struct ProgScan {
        JpegScanArgs a;
        std::vector<unsigned> segs;
        JpegHuffTables tabs;
    };
    std::vector<ProgScan> prog;
    bool prog_host = false;
    // baseline scan without restart markers (self-synchronising GPU decoding)
    bool seq = false;
    std::vector<uint32_t> seq_words;  // unstuffed scan, big-endian words
    JpegSeqArgs seq_args{};

    void ensure_coef() {
        if (coef.empty()) coef.assign(nblocks * 64, 0);
    }

    int16_t* block(const Component& c, int bx, int by) { return &coef[(c.blk0 + (size_t)by * c.bw + bx) * 64]; }

    int frame(const uint8_t* s, int m) {
        if (have_frame) return fail(IK_ERR_TRANSFORM, "%s: duplicate SOF", kFmtErr);
        if (s[0] != 8) return fail(IK_ERR_UNSUPPORTED, "%d-bit JPEG is not supported", s[0]);
        progressive = m == 0xC2;
        height = (int)s[1] << 8 | s[2];
        width = (int)s[3] << 8 | s[4];
        const int nc = s[5];
        if (!width || !height) return fail(IK_ERR_TRANSFORM, "%s: zero dimension", kFmtErr);
        if (nc != 1 && nc != 3 && nc != 4)
            return fail(IK_ERR_UNSUPPORTED, "JPEG with %d components is not supported", nc);
        // image's default Limits: max_alloc 512 MiB of decoded bytes (L8: 1 per pixel, Rgb8: 3)
        if ((uint64_t)width * height * (nc == 1 ? 1u : 3u) > (512ull << 20))
            return fail(IK_ERR_TRANSFORM, "Limits are exceeded");
        comps.resize(nc);
        for (int i = 0; i < nc; ++i) {
            comps[i].id = s[6 + 3 * i];
            comps[i].h = s[7 + 3 * i] >> 4;
            comps[i].v = s[7 + 3 * i] & 15;
            comps[i].tq = s[8 + 3 * i] & 3;
            if (comps[i].h < 1 || comps[i].h > 4 || comps[i].v < 1 || comps[i].v > 4)
                return fail(IK_ERR_TRANSFORM, "%s: bad sampling factors", kFmtErr);
            hmax = std::max(hmax, comps[i].h);
            vmax = std::max(vmax, comps[i].v);
        }
        for (auto& c : comps)
            if (hmax % c.h || vmax % c.v)
                return fail(IK_ERR_UNSUPPORTED, "fractional JPEG chroma sampling is not supported");
        mcux = (width + 8 * hmax - 1) / (8 * hmax);
        mcuy = (height + 8 * vmax - 1) / (8 * vmax);
        size_t blocks = 0;
        for (auto& c : comps) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.dw = (width * c.h + hmax - 1) / hmax;
            c.dh = (height * c.v + vmax - 1) / vmax;
            c.blk0 = blocks;
            blocks += (size_t)c.bw * c.bh;
        }
        nblocks = blocks;
        have_frame = true;
        return IK_OK;
    }

    // one block of one scan (ITU T.81 F.2.2 / G.1.2; libjpeg jdhuff.c / jdphuff.c)
    int block_baseline(BitReader& br, Component& c, int16_t* blk) {
        const int t = decode_symbol(br, dc[c.td]);
        if (t < 0 || t > 11) return fail(IK_ERR_TRANSFORM, "%s: bad DC code", kFmtErr);
        c.pred += t ? extend(br.get(t), t) : 0;
        blk[0] = (int16_t)c.pred;
        for (int k = 1; k < 64;) {
            const int rs = decode_symbol(br, ac[c.ta]);
            if (rs < 0) return fail(IK_ERR_TRANSFORM, "%s: bad AC code", kFmtErr);
            const int r = rs >> 4, sz = rs & 15;
            if (!sz) {
                if (r != 15) break;  // EOB
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return fail(IK_ERR_TRANSFORM, "%s: AC overflow", kFmtErr);
            blk[kZigzag[k]] = (int16_t)extend(br.get(sz), sz);
            ++k;
        }
        return IK_OK;
    }
    int block_dc_first(BitReader& br, Component& c, int16_t* blk, int Al) {
        const int t = decode_symbol(br, dc[c.td]);
        if (t < 0 || t > 11) return fail(IK_ERR_TRANSFORM, "%s: bad DC code", kFmtErr);
        c.pred += t ? extend(br.get(t), t) : 0;
        blk[0] = (int16_t)(c.pred * (1 << Al));
        return IK_OK;
    }
    void block_dc_refine(BitReader& br, int16_t* blk, int Al) {
        if (br.get(1)) blk[0] = (int16_t)(blk[0] | (1 << Al));
    }
    int block_ac_first(BitReader& br, const Component& c, int16_t* blk, int Ss, int Se, int Al) {
        if (eobrun > 0) { --eobrun; return IK_OK; }
        for (int k = Ss; k <= Se; ++k) {
            const int rs = decode_symbol(br, ac[c.ta]);
            if (rs < 0) return fail(IK_ERR_TRANSFORM, "%s: bad AC code", kFmtErr);
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
                k += r;
                if (k > Se) return fail(IK_ERR_TRANSFORM, "%s: AC overflow", kFmtErr);
                blk[kZigzag[k]] = (int16_t)(extend(br.get(sz), sz) * (1 << Al));
            } else if (r == 15) {
                k += 15;
            } else {
                eobrun = 1 << r;
                if (r) eobrun += br.get(r);
                --eobrun;
                break;
            }
        }
        return IK_OK;
    }
    int block_ac_refine(BitReader& br, const Component& c, int16_t* blk, int Ss, int Se, int Al) {
        const int p1 = 1 << Al, m1 = -1 * (1 << Al);
        auto refine = [&](int16_t* co) {
            if (br.get(1) && (*co & p1) == 0) *co = (int16_t)(*co >= 0 ? *co + p1 : *co + m1);
        };
        int k = Ss;
        if (eobrun == 0) {
            for (; k <= Se; ++k) {
                const int rs = decode_symbol(br, ac[c.ta]);
                if (rs < 0) return fail(IK_ERR_TRANSFORM, "%s: bad AC code", kFmtErr);
                int r = rs >> 4, sz = rs & 15, val = 0;
                if (sz) {
                    if (sz != 1) return fail(IK_ERR_TRANSFORM, "%s: bad AC refinement", kFmtErr);
                    val = br.get(1) ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += br.get(r);
                    break;  // the rest of the band goes to the EOB-run pass below
                }
                // skip r zero-history coefficients, refining the nonzero ones passed
                do {
                    int16_t* co = blk + kZigzag[k];
                    if (*co != 0) refine(co);
                    else if (--r < 0) break;
                    ++k;
                } while (k <= Se);
                if (val) {
                    if (k > Se) return fail(IK_ERR_TRANSFORM, "%s: AC overflow", kFmtErr);
                    blk[kZigzag[k]] = (int16_t)val;
                }
            }
        }
        if (eobrun > 0) {
            for (; k <= Se; ++k) {
                int16_t* co = blk + kZigzag[k];
                if (*co != 0) refine(co);
            }
            --eobrun;
        }
        return IK_OK;
    }

    // Record a baseline scan for k_jpeg_huff: find its restart markers (the end of
    // the scan is the first other marker).  False (decode on the host) when the
    // marker count does not match the MCU count.
    bool defer_scan(const std::vector<int>& order, const uint8_t* data, const uint8_t*& next) {
        const bool single = order.size() == 1;
        const Component& c0 = comps[order[0]];
        const int single_bw = (c0.dw + 7) / 8, single_bh = (c0.dh + 7) / 8;
        const long long total_mcu = single ? (long long)single_bw * single_bh : (long long)mcux * mcuy;
        const long long want = (total_mcu + restart - 1) / restart;
        gpu_segs.assign(1, 0u);
        const uint8_t* q = data;
        while (q + 1 < end) {
            if (q[0] != 0xFF) {  // to the next 0xFF (memchr: entropy-coded data holds ~1 in 256 bytes)
                const void* f = std::memchr(q, 0xFF, (size_t)(end - 1 - q));
                if (!f) { q = end - 1; break; }
                q = static_cast<const uint8_t*>(f);
            }
            const uint8_t m = q[1];
            if (m == 0x00) { q += 2; continue; }
            if (m == 0xFF) { ++q; continue; }
            if (m >= 0xD0 && m <= 0xD7) {
                if ((long long)gpu_segs.size() >= want) break;  // a marker past the last interval: let the host judge
                gpu_segs.push_back((unsigned)(q + 2 - data));
                q += 2;
                continue;
            }
            break;
        }
        if ((long long)gpu_segs.size() != want || (size_t)(end - data) > 0xffffffffu) return false;
        JpegScanArgs& a = gpu_scan;
        a = JpegScanArgs{};
        a.size = (long long)(end - data);
        a.n_seg = (int)want;
        a.restart = restart;
        a.total_mcu = total_mcu;
        a.mcux = mcux;
        a.single = single ? 1 : 0;
        a.single_bw = single_bw;
        a.ns = (int)order.size();
        for (int i = 0; i < a.ns; ++i) {
            const Component& c = comps[order[i]];
            a.h[i] = c.h; a.v[i] = c.v; a.bw[i] = c.bw; a.td[i] = c.td; a.ta[i] = c.ta;
            a.blk0[i] = (long long)c.blk0;
        }
        gpu_data = data;
        deferred = true;
        next = q;
        return true;
    }

    // Record a progressive scan with restart intervals for k_jpeg_prog, as
    // defer_scan records a baseline one; a.data holds the scan's offset in the file.
    bool defer_prog(const std::vector<int>& order, int kind, int Ss, int Se, int Al, const uint8_t* data,
                    const uint8_t*& next) {
        const uint8_t* nx = next;
        std::vector<unsigned> keep;
        keep.swap(gpu_segs);
        const bool ok = defer_scan(order, data, nx);
        deferred = false;  // (defer_scan's single-scan record is not used)
        ProgScan ps;
        ps.segs.swap(gpu_segs);
        gpu_segs.swap(keep);
        if (!ok) return false;
        ps.a = gpu_scan;
        ps.a.data = reinterpret_cast<const uint8_t*>((uintptr_t)(data - b));
        ps.a.kind = kind;
        ps.a.Ss = Ss;
        ps.a.Se = Se;
        ps.a.Al = Al;
        tables(ps.tabs);
        prog.push_back(std::move(ps));
        next = nx;
        return true;
    }

    // Record a baseline scan without restart markers for k_jpeg_seq_*: unstuff it
    // (0xFF 0x00 -> 0xFF) up to the first marker into big-endian words.
    bool defer_seq(const std::vector<int>& order, const uint8_t* data, const uint8_t*& next) {
        const bool single = order.size() == 1;
        int bpm = 0;
        JpegSeqArgs a{};
        for (size_t i = 0; i < order.size(); ++i) {
            const Component& c = comps[order[i]];
            const int nb = single ? 1 : c.h * c.v;
            for (int k = 0; k < nb; ++k) {
                if (bpm >= kSeqMaxBPM) return false;
                a.comp_of[bpm] = (int)i;
                a.bx_of[bpm] = single ? 0 : k % c.h;
                a.by_of[bpm] = single ? 0 : k / c.h;
                ++bpm;
            }
            a.h[i] = c.h; a.v[i] = c.v; a.bw[i] = c.bw; a.td[i] = c.td; a.ta[i] = c.ta;
            a.blk0[i] = (long long)c.blk0;
        }
        const Component& c0 = comps[order[0]];
        const int single_bw = (c0.dw + 7) / 8, single_bh = (c0.dh + 7) / 8;
        const long long total_mcu = single ? (long long)single_bw * single_bh : (long long)mcux * mcuy;
        std::vector<uint8_t> clean;
        clean.reserve((size_t)(end - data));
        const uint8_t* q = data;
        while (q < end) {
            if (q[0] != 0xFF) {  // the run up to the next 0xFF in one copy
                const void* f = std::memchr(q, 0xFF, (size_t)(end - q));
                const uint8_t* r = f ? static_cast<const uint8_t*>(f) : end;
                clean.insert(clean.end(), q, r);
                q = r;
                continue;
            }
            if (q + 1 < end && q[1] == 0x00) { clean.push_back(0xFF); q += 2; continue; }
            if (q + 1 >= end) { clean.push_back(0xFF); ++q; continue; }  // a lone 0xFF at the end: stuffed, as on the host
            break;  // a marker: the scan ends (the host feeds zeros from here)
        }
        if (clean.size() < kSeqMinBytes) return false;
        // zero words past the end: a decoder (the GPU lanes, the host frontier walk)
        // may start a block just before nbits and read one whole block of zero bits
        // from there, at most 16 + 11 + 63 (16 + 10) bits, plus peek32's next word
        constexpr size_t kSeqPadWords = (16 + 11 + 63 * (16 + 10) + 31) / 32 + 2;
        const size_t nw = (clean.size() + 3) / 4 + kSeqPadWords;
        seq_words.assign(nw, 0u);
        const size_t nfull = clean.size() / 4;
        for (size_t i = 0; i < nfull; ++i) {  // big-endian words, four bytes at a time
            uint32_t v;
            std::memcpy(&v, clean.data() + 4 * i, 4);
            seq_words[i] = __builtin_bswap32(v);
        }
        for (size_t i = 4 * nfull; i < clean.size(); ++i) seq_words[i >> 2] |= (uint32_t)clean[i] << (24 - 8 * (i & 3));
        a.nbits = (long long)clean.size() * 8;
        // bits per lane (IK_JPEG_SEQ_L, a multiple of 32): 2048, not 8192 -- four times
        // the lanes, each round a quarter as long; the host walk stays small
        // (loadtest restart-free 645 -> 1,061 requests/s, configs[2] restart-free
        // 7,757 -> 14,901 MPix/s, profiles/r03am_jpeg_seq_lane_bits.txt)
        static const int kL = [] {
            const char* e = getenv("IK_JPEG_SEQ_L");
            const int v = e ? atoi(e) : 2048;
            return v < 1024 ? 1024 : (v > 65536 ? 65536 : v & ~31);
        }();
        a.L = kL;
        a.nsub = (int)std::max<long long>(1, (a.nbits + a.L - 1) / a.L);
        a.bpm = bpm;
        a.mcux = mcux;
        a.single = single ? 1 : 0;
        a.single_bw = single_bw;
        a.total_blocks = total_mcu * bpm;
        seq_args = a;
        seq = true;
        deferred = true;
        next = q;
        return true;
    }

    void tables(JpegHuffTables& t) const {
        std::memset(&t, 0, sizeof(t));
        for (int k = 0; k < 8; ++k) {
            const HuffTable& h = k < 4 ? dc[k] : ac[k - 4];
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
            for (int i = 0; i < 512; ++i) {  // run/size code and its magnitude bits in one lookup
                const int L = h.look_len[i], rs = h.look_val[i], r = rs >> 4, sz = rs & 15;
                if (!L || !sz || L + sz > 9) continue;
                const int v = (i >> (9 - L - sz)) & ((1 << sz) - 1);
                const int val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;
                if (val < -128 || val > 127) continue;
                t.fast_ac[k - 4][i] = (int16_t)(val * 256 + r * 16 + L + sz);
            }
        }
    }

    int scan(const uint8_t* s, const uint8_t* se, const uint8_t*& next) {
        if (!have_frame) return fail(IK_ERR_TRANSFORM, "%s: SOS before SOF", kFmtErr);
        const int ns = s[0];
        if (ns < 1 || ns > (int)comps.size() || se - s < 1 + 2 * ns + 3)
            return fail(IK_ERR_TRANSFORM, "%s: bad SOS", kFmtErr);
        std::vector<int> order(ns);
        for (int i = 0; i < ns; ++i) {
            const int cid = s[1 + 2 * i];
            int k = -1;
            for (int j = 0; j < (int)comps.size(); ++j) if (comps[j].id == cid) k = j;
            if (k < 0) return fail(IK_ERR_TRANSFORM, "%s: bad scan component", kFmtErr);
            comps[k].td = s[2 + 2 * i] >> 4;
            comps[k].ta = s[2 + 2 * i] & 15;
            if (comps[k].td > 3 || comps[k].ta > 3) return fail(IK_ERR_TRANSFORM, "%s: bad table id", kFmtErr);
            order[i] = k;
        }
        const int Ss = s[1 + 2 * ns], Se = s[2 + 2 * ns], Ah = s[3 + 2 * ns] >> 4, Al = s[3 + 2 * ns] & 15;
        // kind: 0 baseline, 1 DC first, 2 DC refine, 3 AC first, 4 AC refine
        int kind = 0;
        if (progressive) {
            if (Ss == 0) {
                if (Se != 0) return fail(IK_ERR_TRANSFORM, "%s: bad progressive DC scan", kFmtErr);
                kind = Ah ? 2 : 1;
            } else {
                if (Se < Ss || Se > 63 || ns != 1) return fail(IK_ERR_TRANSFORM, "%s: bad progressive AC scan", kFmtErr);
                kind = Ah ? 4 : 3;
            }
            if (Al > 13) return fail(IK_ERR_TRANSFORM, "%s: bad successive approximation", kFmtErr);
        }
        for (int i = 0; i < ns; ++i) {
            const Component& c = comps[order[i]];
            const bool need_dc = kind == 0 || kind == 1, need_ac = kind == 0 || kind >= 3;
            if ((need_dc && !dc[c.td].present) || (need_ac && !ac[c.ta].present))
                return fail(IK_ERR_TRANSFORM, "%s: missing Huffman table", kFmtErr);
        }
        if (deferred) {  // a second scan: the whole image goes through the host decoder
            need_host = true;
            return IK_OK;
        }
        if (try_gpu && progressive && !prog_host && prog_enabled()) {
            scanned = true;
            if (restart > 0 && defer_prog(order, kind, Ss, Se, Al, se, next)) return IK_OK;
            if (!prog.empty()) {  // a later scan the GPU cannot take: all scans on the host
                need_host = true;
                return IK_OK;
            }
            prog_host = true;  // the first scan: this and every later one on the host
        }
        const bool first_scan = !scanned;
        scanned = true;
        if (try_gpu && first_scan && kind == 0 && restart > 0 && ns == (int)comps.size() && defer_scan(order, se, next))
            return IK_OK;
        if (try_gpu && first_scan && kind == 0 && restart == 0 && ns == (int)comps.size() && seq_enabled() &&
            defer_seq(order, se, next))
            return IK_OK;
        ensure_coef();
        for (auto& c : comps) c.pred = 0;
        eobrun = 0;
        BitReader br{se, end};
        const bool single = ns == 1;
        const Component& c0 = comps[order[0]];
        const int single_bw = (c0.dw + 7) / 8, single_bh = (c0.dh + 7) / 8;
        const long total_mcu = single ? (long)single_bw * single_bh : (long)mcux * mcuy;
        auto do_block = [&](Component& c, int16_t* blk) -> int {
            switch (kind) {
            case 0: return block_baseline(br, c, blk);
            case 1: return block_dc_first(br, c, blk, Al);
            case 2: block_dc_refine(br, blk, Al); return IK_OK;
            case 3: return block_ac_first(br, c, blk, Ss, Se, Al);
            default: return block_ac_refine(br, c, blk, Ss, Se, Al);
            }
        };
        for (long mcu = 0; mcu < total_mcu; ++mcu) {
            if (restart && mcu > 0 && mcu % restart == 0) {
                // expect RSTn: realign to the marker, reset predictors and EOB run
                const uint8_t* q = br.p;
                while (q + 1 < end && !(q[0] == 0xFF && q[1] >= 0xD0 && q[1] <= 0xD7)) ++q;
                if (q + 1 >= end) return fail(IK_ERR_TRANSFORM, "%s: missing restart marker", kFmtErr);
                br.p = q + 2;
                br.reset_at_marker();
                for (auto& c : comps) c.pred = 0;
                eobrun = 0;
            }
            if (single) {
                Component& c = comps[order[0]];
                const int st = do_block(c, block(c, (int)(mcu % single_bw), (int)(mcu / single_bw)));
                if (st) return st;
                continue;
            }
            const int mx = (int)(mcu % mcux), my = (int)(mcu / mcux);
            for (int oi = 0; oi < ns; ++oi) {
                Component& c = comps[order[oi]];
                for (int by = 0; by < c.v; ++by)
                    for (int bx = 0; bx < c.h; ++bx) {
                        const int st = do_block(c, block(c, mx * c.h + bx, my * c.v + by));
                        if (st) return st;
                    }
            }
        }
        next = br.p;
        return IK_OK;
    }

    int parse() {
        const uint8_t* p = b + 2;
        auto be16 = [](const uint8_t* q) { return (int)q[0] << 8 | q[1]; };
        for (;;) {
            while (p < end && *p != 0xFF) ++p;  // tolerate garbage between segments
            while (p < end && *p == 0xFF) ++p;
            if (p >= end || *p == 0xD9) {
                if (scanned) return IK_OK;  // EOI (or a stream cut after its last scan)
                return fail(IK_ERR_TRANSFORM, "%s: no SOS", kFmtErr);
            }
            const uint8_t m = *p++;
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
            if (p + 2 > end) return fail(IK_ERR_TRANSFORM, "%s: truncated", kFmtErr);
            const int len = be16(p);
            if (len < 2 || p + len > end) return fail(IK_ERR_TRANSFORM, "%s: bad segment length", kFmtErr);
            const uint8_t* s = p + 2;
            const uint8_t* se = p + len;
            if (m == 0xDB) {  // DQT
                while (s < se) {
                    const int pq = s[0] >> 4, tq = s[0] & 15;
                    if (tq > 3 || s + 1 + (pq ? 128 : 64) > se) return fail(IK_ERR_TRANSFORM, "%s: bad DQT", kFmtErr);
                    ++s;
                    for (int i = 0; i < 64; ++i) qt[tq][kZigzag[i]] = pq ? (uint16_t)be16(s + 2 * i) : s[i];
                    s += pq ? 128 : 64;
                }
            } else if (m == 0xC4) {  // DHT
                while (s < se) {
                    const int tc = s[0] >> 4, th = s[0] & 15;
                    if (th > 3 || tc > 1 || s + 17 > se) return fail(IK_ERR_TRANSFORM, "%s: bad DHT", kFmtErr);
                    int total = 0;
                    for (int i = 0; i < 16; ++i) total += s[1 + i];
                    if (total > 256 || s + 17 + total > se) return fail(IK_ERR_TRANSFORM, "%s: bad DHT", kFmtErr);
                    if (!build_huff(s + 1, s + 17, total, tc ? ac[th] : dc[th]))
                        return fail(IK_ERR_TRANSFORM, "%s: bad Huffman table", kFmtErr);
                    s += 17 + total;
                }
            } else if (m == 0xDD) {  // DRI
                if (len < 4) return fail(IK_ERR_TRANSFORM, "%s: bad DRI", kFmtErr);
                restart = be16(s);
            } else if (m == 0xEE) {  // APP14 Adobe
                if (len >= 14 && !std::memcmp(s, "Adobe", 5)) { adobe = true; adobe_transform = s[11]; }
            } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  // SOF0 / SOF1 / SOF2
                if (len < 8) return fail(IK_ERR_TRANSFORM, "%s: bad SOF", kFmtErr);
                const int st = frame(s, m);
                if (st) return st;
            } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                return fail(IK_ERR_UNSUPPORTED, "arithmetic / lossless / hierarchical JPEG (SOF%d) is not supported",
                            m - 0xC0);
            } else if (m == 0xDA) {  // SOS: entropy-coded data follows the header
                const uint8_t* next = se;
                const int st = scan(s, se, next);
                if (st) return st;
                if (need_host) return IK_OK;
                p = next;
                continue;
            }
            p += len;
        }
    }
};

}  // namespace

std::atomic<int> g_jpeg_recon{-1};  // -1: not yet read from IK_JPEG_RECON

namespace {

int jpeg_recon() {
    int m = g_jpeg_recon.load();
    if (m < 0) {
        const char* e = getenv("IK_JPEG_RECON");
        m = e && !strcmp(e, "libjpeg") ? IK_JPEG_RECON_LIBJPEG : IK_JPEG_RECON_ZUNE;
        int expected = -1;
        g_jpeg_recon.compare_exchange_strong(expected, m);
        m = g_jpeg_recon.load();
    }
    return m;
}

// reconstruction geometry of a parsed stream; returns the plane bytes it needs
size_t make_geom(const Decoder& d, JpegGeom& g) {
    const int nc = (int)d.comps.size();
    int colorspace = nc == 1 ? 0 : 1;  // gray / YCbCr
    if (nc == 3 && d.adobe && d.adobe_transform == 0) colorspace = 2;  // Adobe RGB-coded
    if (nc == 3 && !d.adobe && d.comps[0].id == 'R' && d.comps[1].id == 'G' && d.comps[2].id == 'B') colorspace = 2;
    if (nc == 4) colorspace = d.adobe && d.adobe_transform == 2 ? 4 : 3;  // YCCK / CMYK
    g = JpegGeom{};
    g.adobe = d.adobe ? 1 : 0;
    g.recon = jpeg_recon();
    g.ncomp = nc;
    g.W = d.width;
    g.H = d.height;
    g.hmax = d.hmax;
    g.vmax = d.vmax;
    g.colorspace = colorspace;
    size_t plane_bytes = 0;
    for (int i = 0; i < nc; ++i) {
        const Component& c = d.comps[i];
        g.h[i] = c.h; g.v[i] = c.v; g.bw[i] = c.bw; g.bh[i] = c.bh; g.dw[i] = c.dw; g.dh[i] = c.dh;
        g.blk0[i] = (long long)c.blk0;
        g.plane0[i] = (long long)plane_bytes;
        plane_bytes += (size_t)c.bw * 8 * c.bh * 8;
    }
    g.nblocks = (long long)d.nblocks;
    return plane_bytes;
}

void qtables(const Decoder& d, uint16_t q[256]) {
    std::memset(q, 0, 256 * sizeof(uint16_t));
    for (int i = 0; i < (int)d.comps.size(); ++i) std::memcpy(&q[i * 64], d.qt[d.comps[i].tq], 64 * sizeof(uint16_t));
}

inline size_t up256(size_t x) { return (x + 255) / 256 * 256; }

// Host decoder over the unstuffed words from an arbitrary (bit, MCU phase) state:
// the frontier walk below uses it on the few lanes the GPU rounds leave unsynced.
struct HostSeq {
    const Decoder& d;
    const JpegSeqArgs& a;
    const uint32_t* w;
    uint32_t peek32(unsigned long long pos) const {
        const size_t i = (size_t)(pos >> 5);
        const uint64_t buf = ((uint64_t)w[i] << 32) | w[i + 1];
        return (uint32_t)((buf << (pos & 31)) >> 32);
    }
    int sym(unsigned long long& pos, const HuffTable& t) const {
        const uint32_t win = peek32(pos);
        const int look = (int)(win >> 23);
        if (t.look_len[look]) { pos += t.look_len[look]; return t.look_val[look]; }
        const int code = (int)(win >> 16);
        for (int len = 10; len <= 16; ++len) {
            const int c = code >> (16 - len);
            if (t.maxcode[len] >= 0 && c <= t.maxcode[len] && c >= t.mincode[len]) {
                pos += len;
                return t.vals[t.valptr[len] + c - t.mincode[len]];
            }
        }
        return -1;
    }
    int get(unsigned long long& pos, int n) const {
        if (!n) return 0;
        const int v = (int)(peek32(pos) >> (32 - n));
        pos += n;
        return v;
    }
    bool block(unsigned long long& pos, int c) const {
        const int t = sym(pos, d.dc[a.td[c]]);
        if (t < 0 || t > 11) return false;
        (void)get(pos, t);
        for (int k = 1; k < 64;) {
            const int rs = sym(pos, d.ac[a.ta[c]]);
            if (rs < 0) return false;
            const int r = rs >> 4, sz = rs & 15;
            if (!sz) {
                if (r != 15) break;
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return false;
            (void)get(pos, sz);
            ++k;
        }
        return true;
    }
    // lane u from (bit, j): the first block start at or past its end; false on a bad code
    bool lane(int u, unsigned long long& bit, int& j) const {
        const unsigned long long end = (unsigned long long)(u + 1) * (unsigned long long)a.L;
        while (bit < end && bit < (unsigned long long)a.nbits) {
            if (!block(bit, a.comp_of[j])) return false;
            j = j + 1 == a.bpm ? 0 : j + 1;
        }
        return true;
    }
};

// Self-synchronising GPU decoding of a scan recorded by defer_seq into the
// coefficient image dcoef (pre-zeroed).
//  1. GPU rounds: every lane decodes from its guessed first block start (bit, MCU
//     phase) to its end; the state there is the next lane's new guess.  Most lanes
//     synchronise in the first round.
//  2. Frontier walk on the host: from the first lane whose guess changed (its new
//     guess is exact), decode lane by lane until the walk meets the GPU's chain
//     again, then jump to the next changed lane -- only the unsynchronised stretches
//     are decoded serially.
//  3. A GPU round on the corrected starts must change nothing; its block counts and
//     DC sums give the bases (host prefix sums) for the decode pass.
// IK_OK, or 1: inconsistent (bad data) -> host decoder.
// device bytes run_seq needs (part of the caller's scratch: no hipMalloc/hipFree,
// which would synchronise the device under concurrent decodes)
size_t seq_bytes(const Decoder& d) {
    const size_t ns = (size_t)d.seq_args.nsub;
    return up256(d.seq_words.size() * 4) + 2 * up256(8 * ns) + 3 * up256(4 * ns) + up256(16 * ns) + up256(8 * ns) +
           up256(16 * ns) + up256(4 * ns) + 256;
}

int run_seq(const Decoder& d, const uint8_t* dtabs, int16_t* dcoef, uint8_t* dev, hipStream_t s) {
    const JpegSeqArgs& base = d.seq_args;
    const int ns = base.nsub;
    const size_t wbytes = d.seq_words.size() * 4;
    const size_t o_sb = up256(wbytes), o_nbit = o_sb + up256(8ull * ns), o_sj = o_nbit + up256(8ull * ns);
    const size_t o_nj = o_sj + up256(4ull * ns), o_nb = o_nj + up256(4ull * ns), o_dc = o_nb + up256(4ull * ns);
    const size_t o_bb = o_dc + up256(16ull * ns), o_db = o_bb + up256(8ull * ns), o_fg = o_db + up256(16ull * ns);
    const size_t o_fl = o_fg + up256(4ull * ns);
    static const bool timing = getenv("IK_JPEG_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<unsigned long long> S(ns), G(ns);
    std::vector<int> Sj(ns, 0), Gj(ns, 0), flags(ns, 0);
    for (int t = 0; t < ns; ++t) S[t] = (unsigned long long)t * base.L;  // guess: a block starts at each cut
    int rc = copy_h2d_2d(dev, wbytes, reinterpret_cast<const uint8_t*>(d.seq_words.data()), wbytes, wbytes, 1, s);
    if (rc) return rc;
    JpegSeqArgs a = base;
    a.words = reinterpret_cast<const uint32_t*>(dev);
    a.tabs = reinterpret_cast<const JpegHuffTables*>(dtabs);
    a.start_bit = reinterpret_cast<const unsigned long long*>(dev + o_sb);
    a.start_j = reinterpret_cast<const int*>(dev + o_sj);
    a.next_bit = reinterpret_cast<unsigned long long*>(dev + o_nbit);
    a.next_j = reinterpret_cast<int*>(dev + o_nj);
    a.nblocks = reinterpret_cast<int*>(dev + o_nb);
    a.dcsum = reinterpret_cast<int*>(dev + o_dc);
    a.flags = reinterpret_cast<int*>(dev + o_fg);
    a.changed = reinterpret_cast<int*>(dev + o_fl);
    a.err = reinterpret_cast<int*>(dev + o_fl + 4);
    a.coef = dcoef;
    a.lanes = jpeg_lanes_for(ns);
    // one GPU round on the starts S: new guesses into G, flags; returns the changed count or < 0
    auto round = [&]() -> int {
        int changed = 0;
        int r = copy_h2d_2d(dev + o_sb, 8ull * ns, reinterpret_cast<const uint8_t*>(S.data()), 8ull * ns, 8ull * ns, 1, s);
        if (!r) r = copy_h2d_2d(dev + o_sj, 4ull * ns, reinterpret_cast<const uint8_t*>(Sj.data()), 4ull * ns, 4ull * ns, 1, s);
        if (r) return -1;
        hipError_t e = hipMemsetAsync(a.changed, 0, 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(a.flags, 0, 4ull * ns, s);
        if (e == hipSuccess) e = launch_jpeg_seq_sync(a, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&changed, a.changed, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { hip_fail(e, "jpeg seq sync"); return -1; }
        if (changed) {
            r = copy_d2h_2d(reinterpret_cast<uint8_t*>(G.data()), 8ull * ns, dev + o_nbit, 8ull * ns, 8ull * ns, 1, s);
            if (!r) r = copy_d2h_2d(reinterpret_cast<uint8_t*>(Gj.data()), 4ull * ns, dev + o_nj, 4ull * ns, 4ull * ns, 1, s);
            if (!r) r = copy_d2h_2d(reinterpret_cast<uint8_t*>(flags.data()), 4ull * ns, dev + o_fg, 4ull * ns, 4ull * ns, 1, s);
            if (r) return -1;
            G[0] = 0;
            Gj[0] = 0;
            flags[0] = 0;
        }
        return changed;
    };
    // round 1 from the naive guesses; round 2 from its results (most already exact),
    // so that the walk below meets a chain whose starts are mostly right
    // (IK_JPEG_SEQ_ROUNDS: GPU rounds before the walk, default 2; each round fixes
    // at least one more lane of every unsynchronised stretch)
    static const int max_rounds = [] {
        const char* e = getenv("IK_JPEG_SEQ_ROUNDS");
        const int v = e ? atoi(e) : 2;
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    int changed = round();
    int walked = 0, rounds_run = 1;
    if (changed < 0) return 1;
    while (changed > 0 && rounds_run < max_rounds) {
        S = G;
        Sj = Gj;
        changed = round();
        ++rounds_run;
        if (changed < 0) return 1;
    }
    if (changed > 0) {
        // lanes before the first changed one are consistent from lane 0, so that
        // lane's new guess is exact; walk from there
        const HostSeq hs{d, base, d.seq_words.data()};
        std::vector<unsigned long long> T = S;
        std::vector<int> Tj = Sj;
        int u = 1;
        while (u < ns && !flags[u]) ++u;
        while (u < ns) {
            unsigned long long bit = G[u];
            int j = Gj[u];
            T[u] = bit;
            Tj[u] = j;
            // walk until the walked state equals the GPU's guess for a lane whose own
            // guess did not change (from there the GPU chain is consistent)
            for (;;) {
                if (!hs.lane(u, bit, j)) return 1;
                ++walked;
                ++u;
                if (u >= ns) break;
                T[u] = bit;
                Tj[u] = j;
                if (!flags[u] && bit == S[u] && j == Sj[u]) break;
            }
            while (u < ns && !flags[u]) ++u;  // consistent stretch: keep the GPU's starts
        }
        S = T;
        Sj = Tj;
        changed = round();  // verification: nothing may change now
        if (changed != 0) return 1;
    }
    if (timing)
        fprintf(stderr, "[jpeg seq] %d lanes, %d per wave, %d lanes walked on the host, %.2f ms\n", ns, a.lanes, walked,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    // prefix sums on the host (a few thousand lanes)
    std::vector<int> nb(ns), dc(4ull * ns);
    rc = copy_d2h_2d(reinterpret_cast<uint8_t*>(nb.data()), 4ull * ns, dev + o_nb, 4ull * ns, 4ull * ns, 1, s);
    if (!rc) rc = copy_d2h_2d(reinterpret_cast<uint8_t*>(dc.data()), 16ull * ns, dev + o_dc, 16ull * ns, 16ull * ns, 1, s);
    if (rc) return rc;
    long long acc = 0;
    for (int t = 0; t < ns; ++t) acc += nb[t];
    if (acc < base.total_blocks) return 1;  // a real block failed to decode: the host decoder decides
    if (acc > base.total_blocks) {  // blocks decoded from the padding past the final block: drop them
        long long excess = acc - base.total_blocks;
        for (int t = ns - 1; t >= 0 && excess > 0; --t) {
            const long long take = std::min<long long>(nb[t], excess);
            nb[t] -= (int)take;
            excess -= take;
        }
        rc = copy_h2d_2d(dev + o_nb, 4ull * ns, reinterpret_cast<const uint8_t*>(nb.data()), 4ull * ns, 4ull * ns, 1, s);
        if (rc) return rc;
    }
    std::vector<long long> bb(ns);
    std::vector<int> db(4ull * ns);
    acc = 0;
    int dacc[4] = {0, 0, 0, 0};
    for (int t = 0; t < ns; ++t) {
        bb[t] = acc;
        acc += nb[t];
        for (int c = 0; c < 4; ++c) { db[4 * t + c] = dacc[c]; dacc[c] += dc[4 * t + c]; }
    }
    rc = copy_h2d_2d(dev + o_bb, 8ull * ns, reinterpret_cast<const uint8_t*>(bb.data()), 8ull * ns, 8ull * ns, 1, s);
    if (!rc) rc = copy_h2d_2d(dev + o_db, 16ull * ns, reinterpret_cast<const uint8_t*>(db.data()), 16ull * ns, 16ull * ns, 1, s);
    if (rc) return rc;
    a.block_base = reinterpret_cast<const long long*>(dev + o_bb);
    a.dc_base = reinterpret_cast<const int*>(dev + o_db);
    int err = 0;
    hipError_t e = hipMemsetAsync(a.err, 0, 4, s);
    if (e == hipSuccess) e = launch_jpeg_seq_decode(a, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&err, a.err, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "jpeg seq decode");
    return err ? 1 : IK_OK;
}

// try_gpu: baseline scans with restart intervals are entropy-decoded on the GPU
// (k_jpeg_huff), restart-free baseline scans by self-synchronising decoding
// (k_jpeg_seq_*), progressive scans with restart intervals scan by scan
// (k_jpeg_prog); anything else, and any stream the GPU finds a bad code in, goes
// through the host decoder
// process-wide: JPEG streams whose entropy decoding ran on the GPU / on the host
std::atomic<unsigned long long> g_jpeg_gpu_streams{0}, g_jpeg_host_streams{0};

int decode_jpeg_impl(const uint8_t* bytes, size_t n, ik_image** out, bool try_gpu) {
    static const bool timing = getenv("IK_JPEG_TIMING") != nullptr;  // dev: phase times to stderr
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = timing ? now() : 0;
    Decoder d;
    d.b = bytes;
    d.end = bytes + n;
    d.try_gpu = try_gpu;
    int st = d.parse();
    if (st) return st;
    if (d.need_host) return decode_jpeg_impl(bytes, n, out, false);  // several scans: all on the host
    const int nc = (int)d.comps.size();
    JpegGeom g;
    const size_t plane_bytes = make_geom(d, g);

    // device scratch: [qtables 4x64 u16][coefficients][planes][GPU entropy decoding:
    // tables, error flag, segment starts, scan bytes]
    const size_t qbytes = 256 * sizeof(uint16_t);
    const size_t cbytes = d.nblocks * 64 * sizeof(int16_t);
    const bool gpu = d.deferred;
    const bool seq = d.seq;
    const size_t tbytes = gpu ? (sizeof(JpegHuffTables) + 255) / 256 * 256 : 0;
    const size_t sbytes = gpu && !seq ? (d.gpu_segs.size() * sizeof(unsigned) + 255) / 256 * 256 : 0;
    const size_t dbytes = gpu && !seq ? (size_t)d.gpu_scan.size : 0;
    std::vector<uint16_t> q(256, 0);
    qtables(d, q.data());
    const double t1 = timing ? now() : 0;
    ik_image* img = nullptr;
    st = alloc_image((uint32_t)d.width, (uint32_t)d.height, nc == 1 ? 1u : 3u, &img);
    if (st) return st;
    const double t2 = timing ? now() : 0;
    const size_t pl_off = qbytes + (cbytes + 255) / 256 * 256;
    const size_t t_off = pl_off + (plane_bytes + 255) / 256 * 256;
    const size_t e_off = t_off + tbytes, s_off = e_off + 256, d_off = s_off + sbytes;
    const size_t q_off = up256(d_off + dbytes + 1024);  // the restart bit reader fetches 64-B chunks past the end
    // progressive scans on the GPU: [the file (+ reader slack)][error flag][per scan:
    // tables, interval starts], staged in one host buffer and copied at once
    const bool prog = !d.prog.empty();
    std::vector<uint8_t> pstage;
    std::vector<size_t> ptab_off, pseg_off;
    size_t p_err = 0;
    if (prog) {
        size_t o = up256(n + 1024);
        p_err = o;
        o += 256;
        for (const auto& ps : d.prog) {
            ptab_off.push_back(o);
            o += up256(sizeof(JpegHuffTables));
            pseg_off.push_back(o);
            o += up256(ps.segs.size() * sizeof(unsigned));
        }
        pstage.assign(o, 0);
        std::memcpy(pstage.data(), bytes, n);
        for (size_t k = 0; k < d.prog.size(); ++k) {
            std::memcpy(pstage.data() + ptab_off[k], &d.prog[k].tabs, sizeof(JpegHuffTables));
            std::memcpy(pstage.data() + pseg_off[k], d.prog[k].segs.data(), d.prog[k].segs.size() * sizeof(unsigned));
        }
    }
    uint8_t* dev = scratch(q_off + (gpu && seq ? seq_bytes(d) : 0) + pstage.size());
    if (!dev) { ik_image_free(img); return fail(IK_ERR_DEVICE, "cannot allocate device scratch"); }
    hipStream_t s = thread_stream();
    st = copy_h2d_2d(dev, qbytes, reinterpret_cast<const uint8_t*>(q.data()), qbytes, qbytes, 1, s);
    if (!st && gpu && seq) {
        JpegHuffTables tabs;
        d.tables(tabs);
        st = copy_h2d_2d(dev + t_off, sizeof(tabs), reinterpret_cast<const uint8_t*>(&tabs), sizeof(tabs),
                         sizeof(tabs), 1, s);
        if (!st && hipMemsetAsync(dev + qbytes, 0, cbytes, s) != hipSuccess) st = fail(IK_ERR_DEVICE, "memset");
        if (!st) st = run_seq(d, dev + t_off, reinterpret_cast<int16_t*>(dev + qbytes), dev + q_off, s);
        if (st == 1) {  // not resolved on the GPU: the host decoder decides
            ik_image_free(img);
            return decode_jpeg_impl(bytes, n, out, false);
        }
    } else if (!st && gpu) {
        JpegHuffTables tabs;
        d.tables(tabs);
        st = copy_h2d_2d(dev + t_off, sizeof(tabs), reinterpret_cast<const uint8_t*>(&tabs), sizeof(tabs),
                         sizeof(tabs), 1, s);
        if (!st)
            st = copy_h2d_2d(dev + s_off, sbytes, reinterpret_cast<const uint8_t*>(d.gpu_segs.data()),
                             d.gpu_segs.size() * sizeof(unsigned), d.gpu_segs.size() * sizeof(unsigned), 1, s);
        if (!st && dbytes) st = copy_h2d_2d(dev + d_off, dbytes, d.gpu_data, dbytes, dbytes, 1, s);
        if (!st) {
            hipError_t e = hipMemsetAsync(dev + qbytes, 0, cbytes, s);
            if (e == hipSuccess) e = hipMemsetAsync(dev + e_off, 0, sizeof(int), s);
            JpegScanArgs a = d.gpu_scan;
            a.data = dev + d_off;
            a.seg = reinterpret_cast<const unsigned*>(dev + s_off);
            a.tabs = reinterpret_cast<const JpegHuffTables*>(dev + t_off);
            a.coef = reinterpret_cast<int16_t*>(dev + qbytes);
            a.err = reinterpret_cast<int*>(dev + e_off);
            if (e == hipSuccess) e = launch_jpeg_huff(a, s);
            int err = 0;
            if (e == hipSuccess) e = hipMemcpyAsync(&err, dev + e_off, sizeof(int), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) { ik_image_free(img); return hip_fail(e, "jpeg entropy decode"); }
            if (err) {  // a bad code somewhere: the host decoder reports it
                ik_image_free(img);
                return decode_jpeg_impl(bytes, n, out, false);
            }
        }
    } else if (!st && prog) {
        uint8_t* pb = dev + q_off;
        st = copy_h2d_2d(pb, pstage.size(), pstage.data(), pstage.size(), pstage.size(), 1, s);
        if (!st) {
            hipError_t e = hipMemsetAsync(dev + qbytes, 0, cbytes, s);
            int* d_err = reinterpret_cast<int*>(pb + p_err);
            for (size_t k = 0; k < d.prog.size() && e == hipSuccess; ++k) {
                JpegScanArgs a = d.prog[k].a;
                a.data = pb + (size_t)(uintptr_t)a.data;  // the scan's offset in the file
                a.seg = reinterpret_cast<const unsigned*>(pb + pseg_off[k]);
                a.tabs = reinterpret_cast<const JpegHuffTables*>(pb + ptab_off[k]);
                a.coef = reinterpret_cast<int16_t*>(dev + qbytes);
                a.err = d_err;
                e = launch_jpeg_prog(a, s);
            }
            int err = 0;
            if (e == hipSuccess) e = hipMemcpyAsync(&err, d_err, sizeof(int), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) { ik_image_free(img); return hip_fail(e, "jpeg progressive entropy decode"); }
            if (err) {  // a bad code somewhere: the host decoder reports it
                ik_image_free(img);
                return decode_jpeg_impl(bytes, n, out, false);
            }
        }
    } else if (!st && cbytes) {
        st = copy_h2d_2d(dev + qbytes, cbytes, reinterpret_cast<const uint8_t*>(d.coef.data()), cbytes, cbytes, 1, s);
    }
    if (st) { ik_image_free(img); return st; }
    const double t3 = timing ? now() : 0;
    g.qt = reinterpret_cast<const uint16_t*>(dev);
    g.coef = reinterpret_cast<const int16_t*>(dev + qbytes);
    g.planes = dev + pl_off;
    hipError_t e = launch_jpeg_reconstruct(g, img->d, img->pitch, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { ik_image_free(img); return hip_fail(e, "jpeg reconstruct"); }
    if (timing)
        fprintf(stderr, "[jpeg] %s: parse %.2f alloc %.2f entropy/upload %.2f reconstruct %.2f ms\n",
                gpu || prog ? "gpu entropy" : "host entropy", t1 - t0, t2 - t1, t3 - t2, now() - t3);
    (gpu || prog ? g_jpeg_gpu_streams : g_jpeg_host_streams) += 1;
    *out = img;
    return IK_OK;
}

}  // namespace

int decode_jpeg_batch(const uint8_t* const* bytes, const size_t* lens, int n, ik_image** outs, int* status,
                      std::string* msgs) {
    // 1. parse every stream (host threads); restart-interval baseline scans are deferred
    std::vector<std::unique_ptr<Decoder>> ds(n);
    std::vector<int> st(n, IK_OK);
    auto note = [&](int i) {
        if (st[i] && msgs) {
            char buf[512];
            ik_last_error(buf, sizeof(buf));
            msgs[i] = buf;
        }
    };
    parallel_for(n, 0, [&](int i) {
        ds[i].reset(new Decoder());
        ds[i]->b = bytes[i];
        ds[i]->end = bytes[i] + lens[i];
        ds[i]->try_gpu = true;
        st[i] = ds[i]->parse();
        note(i);
    });
    std::vector<int> gpu_idx, host_idx, seq_idx;
    for (int i = 0; i < n; ++i) {
        outs[i] = nullptr;
        if (st[i]) continue;
        if (ds[i]->deferred && !ds[i]->need_host && !ds[i]->seq) gpu_idx.push_back(i);
        else if ((ds[i]->seq || !ds[i]->prog.empty()) && !ds[i]->need_host) seq_idx.push_back(i);  // one by one, GPU
        else host_idx.push_back(i);
    }
    // 2. the deferred scans: one device allocation, one Huffman launch over all of them.
    // Layout: [args][error flags][every image's quantisation + Huffman tables and
    // interval starts][every image's scan bytes][every image's coefficients and
    // planes].  The tables go up in one copy from a pinned block filled by the pool;
    // scan bytes already in page-locked memory (ik_host_alloc) are DMAed in place, the
    // rest through a pinned block the pool fills -- all asynchronous on the stream,
    // ordered before the launch (before: four synchronous staged copies per image).
    const int m = (int)gpu_idx.size();
    if (m) {
        struct Lay { size_t q, t, sg, dt, coef, pl, end; JpegGeom g; };
        std::vector<Lay> lay(m);
        const size_t o_args = 256, o_err = o_args + up256(sizeof(JpegScanArgs) * m);
        size_t total = o_err + up256(sizeof(int) * m);
        const size_t o_small = total;
        for (int k = 0; k < m; ++k) {  // tables and interval starts
            const Decoder& d = *ds[gpu_idx[k]];
            Lay& L = lay[k];
            L.q = total;
            L.t = L.q + 512;
            L.sg = L.t + up256(sizeof(JpegHuffTables));
            total = L.sg + up256(d.gpu_segs.size() * sizeof(unsigned));
        }
        const size_t small_bytes = total - o_small;
        for (int k = 0; k < m; ++k) {  // scan bytes
            lay[k].dt = total;
            total += up256((size_t)ds[gpu_idx[k]]->gpu_scan.size + 1024);  // 64-B chunk fetches past the end
        }
        for (int k = 0; k < m; ++k) {  // coefficients and planes
            const Decoder& d = *ds[gpu_idx[k]];
            Lay& L = lay[k];
            const size_t pb = make_geom(d, L.g);
            L.coef = total;
            L.pl = L.coef + up256(d.nblocks * 64 * sizeof(int16_t));
            L.end = L.pl + up256(pb);
            total = L.end;
        }
        // the batch's device work area: a grow-only per-thread arena (hipFree would
        // synchronise the whole device under concurrent batches)
        hipStream_t s = thread_stream();
        uint8_t* dev = scratch_slot(1, total);
        int rc = dev ? IK_OK : fail(IK_ERR_DEVICE, "cannot allocate the JPEG batch work area");
        uint8_t* hsmall = rc ? nullptr : pinned_slot(1, small_bytes);
        if (!rc && !hsmall) rc = IK_ERR_NOMEM;
        std::vector<char> in_place(m, 0);
        std::vector<size_t> st_off(m, 0);
        size_t st_total = 0;
        for (int k = 0; k < m && !rc; ++k) {
            const Decoder& d = *ds[gpu_idx[k]];
            in_place[k] = host_pinned(d.gpu_data, (size_t)d.gpu_scan.size) ? 1 : 0;
            if (!in_place[k]) {
                st_off[k] = st_total;
                st_total += up256((size_t)d.gpu_scan.size);
            }
        }
        uint8_t* hdata = !rc && st_total ? pinned_slot(2, st_total) : nullptr;
        if (!rc && st_total && !hdata) rc = IK_ERR_NOMEM;
        std::vector<JpegScanArgs> args(m);
        int max_seg = 0;
        if (!rc) {
            parallel_for(m, 0, [&](int k) {
                const Decoder& d = *ds[gpu_idx[k]];
                const Lay& L = lay[k];
                qtables(d, reinterpret_cast<uint16_t*>(hsmall + (L.q - o_small)));
                d.tables(*reinterpret_cast<JpegHuffTables*>(hsmall + (L.t - o_small)));
                std::memcpy(hsmall + (L.sg - o_small), d.gpu_segs.data(), d.gpu_segs.size() * sizeof(unsigned));
                if (!in_place[k]) std::memcpy(hdata + st_off[k], d.gpu_data, (size_t)d.gpu_scan.size);
            });
            hipError_t e = hipMemcpyAsync(dev + o_small, hsmall, small_bytes, hipMemcpyHostToDevice, s);
            for (int k = 0; k < m && e == hipSuccess; ++k) {
                const Decoder& d = *ds[gpu_idx[k]];
                const size_t db = (size_t)d.gpu_scan.size;
                if (db)
                    e = hipMemcpyAsync(dev + lay[k].dt, in_place[k] ? d.gpu_data : hdata + st_off[k], db,
                                       hipMemcpyHostToDevice, s);
            }
            if (e != hipSuccess) rc = hip_fail(e, "jpeg batch upload");
        }
        for (int k = 0; k < m && !rc; ++k) {
            const Decoder& d = *ds[gpu_idx[k]];
            const Lay& L = lay[k];
            JpegScanArgs& a = args[k];
            a = d.gpu_scan;
            a.data = dev + L.dt;
            a.seg = reinterpret_cast<const unsigned*>(dev + L.sg);
            a.tabs = reinterpret_cast<const JpegHuffTables*>(dev + L.t);
            a.coef = reinterpret_cast<int16_t*>(dev + L.coef);
            a.err = reinterpret_cast<int*>(dev + o_err) + k;
            max_seg = std::max(max_seg, a.n_seg);
        }
        const size_t hdr = o_small;
        std::vector<int> errs(m, 0);
        if (!rc) {  // (synchronous: also the point where the async uploads above are ordered before the launch)
            rc = copy_h2d_2d(dev + o_args, sizeof(JpegScanArgs) * m, reinterpret_cast<const uint8_t*>(args.data()),
                             sizeof(JpegScanArgs) * m, sizeof(JpegScanArgs) * m, 1, s);
        }
        if (!rc) {
            // No zeroing of the coefficient images where the decoder stores every
            // block whole: an interleaved scan covers every block of its image.  A
            // one-component scan covers only the blocks of the component's own size;
            // when its sampling factors pad the component to more (a gray image with
            // H = V = 2), the padding blocks are zeroed so that no stale scratch
            // reaches the reconstruction, even where the crop drops it.
            hipError_t e = hipMemsetAsync(dev + o_err, 0, sizeof(int) * m, s);
            for (int k = 0; k < m && e == hipSuccess; ++k)
                if (args[k].single && (size_t)args[k].total_mcu < ds[gpu_idx[k]]->nblocks)
                    e = hipMemsetAsync(dev + lay[k].coef, 0, ds[gpu_idx[k]]->nblocks * 64 * sizeof(int16_t), s);
            EvPair& ev = thread_events(2);
            if (e == hipSuccess && ev.a) e = hipEventRecord(ev.a, s);
            if (e == hipSuccess)
                e = launch_jpeg_huff_batch(reinterpret_cast<const JpegScanArgs*>(dev + o_args), m, max_seg, s);
            if (e == hipSuccess && ev.b) e = hipEventRecord(ev.b, s);
            if (e == hipSuccess) e = hipMemcpyAsync(errs.data(), dev + o_err, sizeof(int) * m, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "jpeg batch entropy decode");
            if (!rc) {  // ik_batch_last_timing: the launch's time and algorithmic bytes
                double scan = 0, coef = 0, lanes = 0;
                for (int k = 0; k < m; ++k) {
                    scan += (double)args[k].size;
                    coef += (double)ds[gpu_idx[k]]->nblocks * 64 * sizeof(int16_t);
                    lanes += args[k].n_seg;
                }
                const int d = current_device();
                batch_timing_add(d, kBtJpegHuffMs, ev_pair_ms(ev));
                batch_timing_add(d, kBtJpegScanBytes, scan);
                batch_timing_add(d, kBtJpegCoefBytes, coef);
                batch_timing_add(d, kBtJpegImages, m);
                batch_timing_add(d, kBtJpegLanes, lanes);
            }
        }
        // 3. reconstruction of every image the GPU decoded cleanly
        for (int k = 0; k < m && !rc; ++k) {
            const int i = gpu_idx[k];
            if (errs[k]) { host_idx.push_back(i); continue; }
            const Decoder& d = *ds[i];
            JpegGeom g = lay[k].g;
            g.qt = reinterpret_cast<const uint16_t*>(dev + lay[k].q);
            g.coef = reinterpret_cast<const int16_t*>(dev + lay[k].coef);
            g.planes = dev + lay[k].pl;
            ik_image* img = nullptr;
            st[i] = alloc_image((uint32_t)d.width, (uint32_t)d.height, d.comps.size() == 1 ? 1u : 3u, &img);
            if (st[i]) continue;
            hipError_t e = launch_jpeg_reconstruct(g, img->d, img->pitch, s);
            if (e != hipSuccess) { ik_image_free(img); st[i] = hip_fail(e, "jpeg reconstruct"); continue; }
            outs[i] = img;
        }
        hipError_t e = rc ? hipSuccess : hipStreamSynchronize(s);
        if (rc || e != hipSuccess) {  // the batch as a whole failed on the device: each image on its own path
            for (int k = 0; k < m; ++k) {
                const int i = gpu_idx[k];
                if (outs[i]) { ik_image_free(outs[i]); outs[i] = nullptr; }
                if (!errs[k]) host_idx.push_back(i);
                st[i] = IK_OK;
            }
        } else {
            for (int k = 0; k < m; ++k)
                if (outs[gpu_idx[k]]) g_jpeg_gpu_streams += 1;
        }
        (void)hdr;
    }
    // 4. everything else: the single-image path with host entropy decoding
    // restart-free baseline scans: self-synchronising GPU decoding, one stream per host thread
    const int nh = (int)host_idx.size();
    host_idx.insert(host_idx.end(), seq_idx.begin(), seq_idx.end());
    parallel_for((int)host_idx.size(), 0, [&](int k) {
        const int i = host_idx[k];
        st[i] = decode_jpeg_impl(bytes[i], lens[i], &outs[i], k >= nh);
        note(i);
    });
    int first = IK_OK;
    for (int i = 0; i < n; ++i) {
        if (status) status[i] = st[i];
        if (st[i] && !first) first = st[i];
    }
    return first;
}

int decode_jpeg_device(const uint8_t* bytes, size_t n, ik_image** out) {
    static const bool gpu = [] {
        const char* e = getenv("IK_JPEG_GPU_ENTROPY");
        return !(e && !strcmp(e, "0"));
    }();
    return decode_jpeg_impl(bytes, n, out, gpu);
}

}  // namespace ik

namespace ik {
int jpeg_recon_mode() { return jpeg_recon(); }
}  // namespace ik

extern "C" {

int ik_set_jpeg_reconstruction(int mode) {
    if (mode != IK_JPEG_RECON_LIBJPEG && mode != IK_JPEG_RECON_ZUNE)
        return ik::fail(IK_ERR_INVALID, "bad JPEG reconstruction mode %d", mode);
    (void)ik::jpeg_recon_mode();
    ik::g_jpeg_recon.store(mode);
    return IK_OK;
}

int ik_get_jpeg_reconstruction(void) { return ik::jpeg_recon_mode(); }

int ik_jpeg_counters(unsigned long long* out) {
    if (!out) return ik::fail(IK_ERR_INVALID, "null pointer");
    out[0] = ik::g_jpeg_gpu_streams.load();
    out[1] = ik::g_jpeg_host_streams.load();
    return IK_OK;
}

}  // extern "C"
