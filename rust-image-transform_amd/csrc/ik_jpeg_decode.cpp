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
#include <array>
#include <mutex>
#include <condition_variable>
#include <map>

#include "../../include/imagekit_hip.h"
#include "ik_png.h"
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

// Baseline scans go to the self-synchronising GPU decoder (ik_jsync.hip) from this
// size up; smaller ones are faster on the host entropy decoder.
constexpr size_t kJsyncMinBytes = 4 << 10;
// lanes a batch's self-synchronising decoding aims for (about what the chip holds at once)
constexpr long long kJsyncLanes = 512 << 10;

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
    // a baseline scan for the self-synchronising GPU decoder (ik_jsync.hip): its
    // entropy-coded bytes (stuffed, with any RSTn markers) and geometry
    bool js = false;
    const uint8_t* js_data = nullptr;
    size_t js_len = 0;
    long long js_nivl = 0;  // restart intervals the frame must have
    jsync::Scan js_scan{};  // geometry (device pointers filled at launch)

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

    // Record a baseline scan for the self-synchronising GPU decoder: its bytes run
    // to the file's final EOI marker (the GPU's unstuffing flags any other marker
    // inside them, and counts the restart markers against the frame's intervals;
    // either mismatch sends the image to the host decoder, which reports png's --
    // zune-jpeg's -- error).
    bool defer_jsync(const std::vector<int>& order, const uint8_t* data, const uint8_t*& next) {
        const bool single = order.size() == 1;
        jsync::Scan a{};
        int bpm = 0;
        for (size_t i = 0; i < order.size(); ++i) {
            const Component& c = comps[order[i]];
            const int nb = single ? 1 : c.h * c.v;
            for (int k = 0; k < nb; ++k) {
                if (bpm >= jsync::kMaxBPM) return false;
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
        // the scan's end: the last FF D9 of the file (trailing bytes after EOI are
        // ignored, as the parser ignores them), else the file's end
        const uint8_t* e = end;
        for (const uint8_t* q = end - 2; q >= data && q >= end - 4096; --q)
            if (q[0] == 0xFF && q[1] == 0xD9) { e = q; break; }
        if ((size_t)(e - data) < kJsyncMinBytes) return false;
        a.bpm = bpm;
        a.mcux = mcux;
        a.single = single ? 1 : 0;
        a.single_bw = single_bw;
        a.total_blocks = total_mcu * bpm;
        a.ivl_blocks = restart ? (long long)restart * bpm : a.total_blocks;
        a.L = jsync::kLaneBits;
        a.W = jsync::kWarmBits;
        js_scan = a;
        js_nivl = restart ? (total_mcu + restart - 1) / restart : 1;
        js_data = data;
        js_len = (size_t)(e - data);
        js = true;
        deferred = true;
        next = e;
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
        if (try_gpu && first_scan && kind == 0 && ns == (int)comps.size() && defer_jsync(order, se, next))
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

// process-wide: JPEG streams whose entropy decoding ran on the GPU / on the host
std::atomic<unsigned long long> g_jpeg_gpu_streams{0}, g_jpeg_host_streams{0};

}  // namespace

// ---- the upload stage's JPEG areas (JpegUpload) ------------------------------------
struct JpegArea {
    int device = 0;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    uint8_t* pin = nullptr;  // staging for files the caller did not pin
    size_t pin_cap = 0;
    hipEvent_t ev = nullptr;
    bool busy = false;
};

namespace {
constexpr int kJpegAreas = 2;
struct JpegAreaPool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<JpegArea*> areas;
};
std::mutex g_jarea_mu;
std::map<int, JpegAreaPool*> g_jarea_pools;
JpegAreaPool& jarea_pool(int device) {
    std::lock_guard<std::mutex> lk(g_jarea_mu);
    JpegAreaPool*& p = g_jarea_pools[device];
    if (!p) p = new JpegAreaPool();
    return *p;
}
// an idle area of the device (waits while the batches ahead hold both), as a
// shared_ptr whose deleter hands it back
std::shared_ptr<JpegArea> jarea_acquire(int device) {
    JpegAreaPool& P = jarea_pool(device);
    std::unique_lock<std::mutex> lk(P.mu);
    JpegArea* got = nullptr;
    while (!got) {
        for (JpegArea* a : P.areas)
            if (!a->busy) { got = a; break; }
        if (!got && (int)P.areas.size() < kJpegAreas) {
            got = new JpegArea();
            got->device = device;
            if (hipEventCreateWithFlags(&got->ev, hipEventDisableTiming) != hipSuccess) got->ev = nullptr;
            P.areas.push_back(got);
        }
        if (!got) P.cv.wait(lk);
    }
    got->busy = true;
    return std::shared_ptr<JpegArea>(got, [](JpegArea* a) {
        JpegAreaPool& Q = jarea_pool(a->device);
        {
            std::lock_guard<std::mutex> l2(Q.mu);
            a->busy = false;
        }
        Q.cv.notify_all();
    });
}
}  // namespace

int jpeg_upload_begin(const uint8_t* const* bytes, const size_t* lens, int n, JpegUpload& up) {
    up = JpegUpload();
    if (n <= 0) return IK_OK;
    std::vector<size_t> off(n), soff(n, (size_t)-1);
    size_t total = 0, stotal = 0;
    for (int i = 0; i < n; ++i) {
        off[i] = total;
        total += up256(lens[i] + 64);
        if (!host_pinned(bytes[i], lens[i])) { soff[i] = stotal; stotal += up256(lens[i]); }
    }
    std::shared_ptr<JpegArea> A = jarea_acquire(current_device());
    if (!A->ev) return IK_OK;  // (no event: the kernel stage copies the scans itself)
    // grow an idle area (nothing pending reads it: it was handed back after its batch's decode)
    if (total > A->cap) {
        if (A->dev) { (void)hipFree(A->dev); mem_stat(kMemUploadDev, -(int64_t)A->cap); }
        A->dev = nullptr;
        A->cap = 0;
        if (hipMalloc((void**)&A->dev, total + total / 8) != hipSuccess) { A->dev = nullptr; return IK_OK; }
        A->cap = total + total / 8;
        mem_stat(kMemUploadDev, (int64_t)A->cap);
    }
    if (stotal > A->pin_cap) {
        if (A->pin) { (void)hipHostFree(A->pin); mem_stat(kMemUploadPinned, -(int64_t)A->pin_cap); }
        A->pin = nullptr;
        A->pin_cap = 0;
        if (hipHostMalloc((void**)&A->pin, stotal + stotal / 8, hipHostMallocDefault) != hipSuccess) {
            A->pin = nullptr;
            return IK_OK;
        }
        A->pin_cap = stotal + stotal / 8;
        mem_stat(kMemUploadPinned, (int64_t)A->pin_cap);
    }
    if (stotal)
        parallel_for(n, 0, [&](int i) {
            if (soff[i] != (size_t)-1) std::memcpy(A->pin + soff[i], bytes[i], lens[i]);
        });
    hipStream_t s = thread_stream();
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; ++i)
        e = hipMemcpyAsync(A->dev + off[i], soff[i] == (size_t)-1 ? bytes[i] : A->pin + soff[i], lens[i],
                           hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(A->ev, s);
    static const bool timing = getenv("IK_TIMING") != nullptr;
    if (timing)
        fprintf(stderr, "[jpeg-upload] %d files, %.1f MB (%.1f MB staged) queued at t=%.1f ms\n", n, total / 1e6, stotal / 1e6,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count() -
                    1e3 * (double)(long long)(std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() / 1000) * 1000);
    if (e != hipSuccess) {  // the kernel stage copies the scans itself
        (void)hipStreamSynchronize(s);
        return IK_OK;
    }
    for (int i = 0; i < n; ++i) up.dev[bytes[i]] = A->dev + off[i];
    up.n = n;
    up.ev = A->ev;
    up.area = std::move(A);
    return IK_OK;
}

// ik_shutdown: the JPEG upload areas (no batch is in flight)
void jpeg_shutdown() {
    std::vector<JpegAreaPool*> ps;
    {
        std::lock_guard<std::mutex> lk(g_jarea_mu);
        for (auto& kv : g_jarea_pools) ps.push_back(kv.second);
    }
    for (JpegAreaPool* P : ps) {
        std::lock_guard<std::mutex> lk(P->mu);
        for (JpegArea* a : P->areas) {
            (void)hipSetDevice(a->device);
            if (a->dev) { (void)hipFree(a->dev); mem_stat(kMemUploadDev, -(int64_t)a->cap); }
            if (a->pin) { (void)hipHostFree(a->pin); mem_stat(kMemUploadPinned, -(int64_t)a->pin_cap); }
            if (a->ev) (void)hipEventDestroy(a->ev);
            delete a;
        }
        P->areas.clear();
    }
}

namespace {

#ifdef IK_JPEG_DUMP
std::mutex g_jdump_mu;
std::vector<std::array<std::vector<uint8_t>, 7>> g_jdump;  // per image of the last batch
#endif

// The baseline scans of a batch (ds[idx[k]]->js), all through the self-synchronising
// GPU decoder at once (ik_jsync.hip; algorithm ik_jpeg_sync.h):
//   1. upload: every scan's bytes (DMAed in place when page-locked, else staged),
//      Huffman and quantisation tables, the unstuffing chunk table -- one small copy
//   2. unstuffing on the GPU, then the interval tables come back (a few KB)
//   3. lanes: per image, each interval cut into pieces of lane_bits (host)
//   4. the sync pass, the fix rounds (one over all lanes, then the settle kernel's
//      per image until no lane changes), bases, the decode pass -- no host round trip
//   5. reconstruction of every image (IDCT, upsampling, colour)
// An image the GPU finds inconsistent (a stray marker, a restart count that does
// not match the frame, lanes that never synchronise, a bad code) goes to host_idx:
// the host decoder decides and reports the reference's errors.
static void jsync_batch(std::vector<std::unique_ptr<Decoder>>& ds, const std::vector<int>& idx, ik_image** outs,
                        std::vector<int>& st, std::vector<int>& host_idx, const uint8_t* const* files,
                        const JpegUpload* up) {
    using namespace jsync;
    const int m = (int)idx.size();
    if (!m) return;
    static const bool timing = getenv("IK_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    constexpr int kChunkBytes = 4096;
    // ---- layout ----
    struct Lay {
        size_t scan, out, ivl, qt, tab, coef, pl;
        long long lanes_max, lane0;
        int chunk0, nchunks, ivl0;
        JpegGeom g;
    };
    std::vector<Lay> lay(m);
    // scans the upload stage already put on the device (JpegUpload) are read where
    // they lie: no scratch copy is laid out for them
    std::vector<const uint8_t*> on_dev(m, nullptr);
    if (up && up->n)
        for (int k = 0; k < m; ++k) {
            auto it = up->dev.find(files[idx[k]]);
            if (it != up->dev.end()) on_dev[k] = it->second + (ds[idx[k]]->js_data - files[idx[k]]);
        }
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += up256(bytes); return r; };
    const size_t o_img = take(sizeof(JsImageDev) * m);
    int nchunks = 0, nivl_total = 0;
    long long lanes_max = 0;
    // lane length: 1,024 bits, longer for large batches (up to 4,096) while the batch
    // still has ~kJsyncLanes lanes -- a longer lane costs the sync pass less warm-up
    // per bit and the fix rounds about as many rounds (ik_jpeg_model.cpp on the
    // bench's 4096^2 frames: sync + fix work 2.8x the scan at 1,024, 1.7x at 4,096)
    long long batch_bits = 0;
    for (int k = 0; k < m; ++k) batch_bits += 8ll * (long long)ds[idx[k]]->js_len;
    const int lane_bits = (int)std::min<long long>(4 * kLaneBits,
                                                   std::max<long long>(1, batch_bits / kJsyncLanes / kLaneBits) * kLaneBits);
    for (int k = 0; k < m; ++k) {
        const Decoder& d = *ds[idx[k]];
        Lay& L = lay[k];
        L.chunk0 = nchunks;
        L.nchunks = (int)((d.js_len + kChunkBytes - 1) / kChunkBytes);
        nchunks += L.nchunks;
        L.ivl0 = nivl_total;
        nivl_total += (int)d.js_nivl + 1;
        L.lane0 = lanes_max;
        L.lanes_max = ((long long)(8 * d.js_len) / lane_bits + d.js_nivl + 1 + 255) & ~255ll;
        lanes_max += L.lanes_max;
    }
    const size_t o_chunks = take(sizeof(int2) * nchunks);
    for (int k = 0; k < m; ++k) lay[k].tab = take(sizeof(JpegHuffTables));
    for (int k = 0; k < m; ++k) lay[k].qt = take(512);
    const size_t small_end = o;  // [images | chunks | tables | qt]: one upload
    const size_t o_status = take(sizeof(int) * m), o_totals = take(sizeof(uint32_t) * 2 * m);
    const size_t o_ivl = take(sizeof(long long) * nivl_total);  // contiguous: one read-back
    const size_t small2_end = o;  // [status | totals | ivl]: one read-back
    const size_t o_counts = take(sizeof(uint2) * nchunks);
    const size_t o_scans = take(sizeof(Scan) * m);
    const size_t o_ivlane = take(sizeof(int) * nivl_total);
    const size_t o_wgs = take(sizeof(int2) * (size_t)(lanes_max / 256));
    const size_t tab2_bytes = o - o_scans;  // [scans | ivl_lane | wgs]: the second upload
    const size_t o_changed = take(256);
    const size_t o_recs = take(sizeof(LaneRec) * (size_t)lanes_max);
    const size_t o_bases = take(sizeof(LaneBase) * (size_t)lanes_max);
    const size_t o_cs = take(jsync_chunk_scratch_bytes(lanes_max));
    const size_t o_items = take(sizeof(JpegReconItem) * m);  // the reconstruction launches' image table
    for (int k = 0; k < m; ++k) {
        const Decoder& d = *ds[idx[k]];
        Lay& L = lay[k];
        L.scan = on_dev[k] ? 0 : take(d.js_len + 64);
        L.out = take(d.js_len + 4 * kPadWords + 8);
        const size_t pb = make_geom(d, L.g);
        L.coef = take(d.nblocks * 64 * sizeof(int16_t));
        L.pl = take(pb);
    }
    hipStream_t s = thread_stream();
    uint8_t* dev = scratch_slot(1, o);
    const size_t pin_bytes = std::max(std::max(small_end, sizeof(JpegReconItem) * m + 256),
                                      std::max(small2_end - o_status, tab2_bytes)) + up256(sizeof(int) * m) + 256;
    uint8_t* hp = dev ? pinned_slot(1, pin_bytes) : nullptr;
    auto fail_all = [&](const char* why) {
        (void)why;
        for (int k = 0; k < m; ++k) host_idx.push_back(idx[k]);
    };
    if (!dev || !hp) { fail_all("memory"); return; }
    const double tm_layout = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    (void)hipStreamSynchronize(s);  // the pinned block is free
    // Small transfers between hp and the device go through a copy kernel on this
    // stream that reads or writes the pinned block directly (ik_png_decode.cpp Xfer):
    // SDMA copies queue behind the next batch's scan upload on the same engine --
    // ~12 ms per transfer with configs[2]'s 683 MB batches in flight.
    uint8_t* hp_dev = nullptr;
    if (hipHostGetDevicePointer((void**)&hp_dev, hp, 0) != hipSuccess) hp_dev = nullptr;
    auto h2d = [&](uint8_t* d, size_t off, size_t n) -> hipError_t {  // hp[off, off + n) -> d
        if (!n) return hipSuccess;
        if (!hp_dev) return hipMemcpyAsync(d, hp + off, n, hipMemcpyHostToDevice, s);
        return launch_copy_words(reinterpret_cast<const uint32_t*>(hp_dev + off), reinterpret_cast<uint32_t*>(d),
                                 (n + 3) / 4, s);
    };
    auto d2h = [&](size_t off, const uint8_t* d, size_t n) -> hipError_t {  // d -> hp[off, off + n)
        if (!n) return hipSuccess;
        if (!hp_dev) return hipMemcpyAsync(hp + off, d, n, hipMemcpyDeviceToHost, s);
        return launch_copy_words(reinterpret_cast<const uint32_t*>(d), reinterpret_cast<uint32_t*>(hp_dev + off),
                                 (n + 3) / 4, s);
    };
    const double tm_sync = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // ---- 1. upload ----
    {
        JsImageDev* I = reinterpret_cast<JsImageDev*>(hp + o_img);
        int2* ch = reinterpret_cast<int2*>(hp + o_chunks);
        for (int k = 0; k < m; ++k) {
            const Decoder& d = *ds[idx[k]];
            const Lay& L = lay[k];
            JsImageDev& J = I[k];
            J = JsImageDev{};
            J.scan = dev + L.scan;
            J.scan_len = (long long)d.js_len;
            J.out = dev + L.out;
            J.ivl = reinterpret_cast<long long*>(dev + o_ivl) + L.ivl0;
            J.ivl_cap = (int)d.js_nivl + 1;
            J.chunk0 = L.chunk0;
            J.nchunks = L.nchunks;
            J.totals = reinterpret_cast<uint32_t*>(dev + o_totals) + 2 * k;
            J.status = reinterpret_cast<int*>(dev + o_status) + k;
            for (int c = 0; c < L.nchunks; ++c) ch[L.chunk0 + c] = make_int2(k, c);
        }
        parallel_for(m, 0, [&](int k) {
            const Decoder& d = *ds[idx[k]];
            d.tables(*reinterpret_cast<JpegHuffTables*>(hp + lay[k].tab));
            qtables(d, reinterpret_cast<uint16_t*>(hp + lay[k].qt));
        });
    }
    // the scan bytes: where the upload stage put them (JpegUpload), else DMAed in
    // place from page-locked memory, else through pinned staging
    std::vector<char> in_place(m, 0);
    std::vector<size_t> st_off(m, 0);
    size_t st_total = 0;
    for (int k = 0; k < m; ++k) {
        const Decoder& d = *ds[idx[k]];
        if (on_dev[k]) continue;
        in_place[k] = host_pinned(d.js_data, d.js_len) ? 1 : 0;
        if (!in_place[k]) { st_off[k] = st_total; st_total += up256(d.js_len); }
    }
    for (int k = 0; k < m; ++k)
        if (on_dev[k]) reinterpret_cast<JsImageDev*>(hp + o_img)[k].scan = on_dev[k];
    uint8_t* hdata = st_total ? pinned_slot(2, st_total) : nullptr;
    if (st_total && !hdata) { fail_all("memory"); return; }
    if (st_total)
        parallel_for(m, 0, [&](int k) {
            if (!in_place[k]) std::memcpy(hdata + st_off[k], ds[idx[k]]->js_data, ds[idx[k]]->js_len);
        });
    const double tm_tables = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    double tm_upwait = -1;  // (IK_TIMING: how long the upload stage's DMA still had to run)
    if (timing && up && up->n && up->ev) {
        const auto tw = std::chrono::steady_clock::now();
        if (hipEventQuery(up->ev) != hipSuccess) (void)hipEventSynchronize(up->ev);
        tm_upwait = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
    }
    hipError_t e = h2d(dev, 0, small_end);
    for (int k = 0; k < m && e == hipSuccess; ++k) {
        const Decoder& d = *ds[idx[k]];
        if (on_dev[k]) continue;
        e = hipMemcpyAsync(dev + lay[k].scan, in_place[k] ? d.js_data : hdata + st_off[k], d.js_len,
                           hipMemcpyHostToDevice, s);
    }
    if (e == hipSuccess && up && up->n && up->ev) e = hipStreamWaitEvent(s, up->ev, 0);
    if (e == hipSuccess) e = hipMemsetAsync(dev + o_status, 0, small2_end - o_status, s);
    // ---- 2. unstuffing; the interval tables back ----
    if (e == hipSuccess)
        e = launch_jsync_unstuff(reinterpret_cast<JsImageDev*>(dev + o_img), m,
                                 reinterpret_cast<const int2*>(dev + o_chunks), nchunks,
                                 reinterpret_cast<uint2*>(dev + o_counts), s);
    if (e == hipSuccess) e = d2h(0, dev + o_status, small2_end - o_status);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { (void)hip_fail(e, "jpeg unstuff"); fail_all("device"); return; }
    const double t_unstuff = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // ---- 3. lanes ----
    std::vector<int> ok(m, 0), hstatus(m);
    std::vector<int> ivl_lane((size_t)nivl_total, 0);
    std::vector<int2> wgs;
    std::vector<Scan> scans(m);
    long long lanes_used = 0;
    {
        const int* hst = reinterpret_cast<const int*>(hp);
        const uint32_t* tot = reinterpret_cast<const uint32_t*>(hp + (o_totals - o_status));
        const long long* hivl = reinterpret_cast<const long long*>(hp + (o_ivl - o_status));
        for (int k = 0; k < m; ++k) {
            const Decoder& d = *ds[idx[k]];
            Lay& L = lay[k];
            if (hst[k] || (long long)tot[2 * k + 1] + 1 != d.js_nivl) continue;  // stray marker / wrong restart count
            const long long* iv = hivl + L.ivl0;
            int* il = ivl_lane.data() + L.ivl0;
            bool good = true;
            il[0] = 0;
            for (long long q = 0; q < d.js_nivl; ++q) {
                const long long bits = iv[q + 1] - iv[q];
                if (bits < 0) { good = false; break; }
                il[q + 1] = il[q] + (int)std::max<long long>(1, (bits + lane_bits - 1) / lane_bits);
            }
            if (!good || il[d.js_nivl] > L.lanes_max) continue;
            ok[k] = 1;
            const int nl = il[d.js_nivl];
            lanes_used += nl;
            for (int w = 0; w < nl; w += 256) wgs.push_back(make_int2(k, w));
            Scan& S = scans[k];
            S = d.js_scan;
            S.L = lane_bits;
            S.words = reinterpret_cast<const uint32_t*>(dev + L.out);
            S.ivl = reinterpret_cast<const long long*>(dev + o_ivl) + L.ivl0;
            S.nivl = (int)d.js_nivl;
            S.lane0 = L.lane0;
            S.ivl_lane = reinterpret_cast<const int*>(dev + o_ivlane) + L.ivl0;
            S.tabs = reinterpret_cast<const JpegHuffTables*>(dev + L.tab);
            S.coef = reinterpret_cast<int16_t*>(dev + L.coef);
        }
    }
    for (int k = 0; k < m; ++k)
        if (!ok[k]) host_idx.push_back(idx[k]);
    const int nwg = (int)wgs.size();
    if (!nwg) return;
    std::memcpy(hp, scans.data(), sizeof(Scan) * m);
    std::memcpy(hp + (o_ivlane - o_scans), ivl_lane.data(), sizeof(int) * nivl_total);
    std::memcpy(hp + (o_wgs - o_scans), wgs.data(), sizeof(int2) * nwg);
    const Scan* d_scans = reinterpret_cast<const Scan*>(dev + o_scans);
    const int2* d_wgs = reinterpret_cast<const int2*>(dev + o_wgs);
    LaneRec* d_recs = reinterpret_cast<LaneRec*>(dev + o_recs);
    int* d_status = reinterpret_cast<int*>(dev + o_status);
    int* d_changed = reinterpret_cast<int*>(dev + o_changed);
    // ---- 4. sync, fix rounds, bases, decode ----
    EvPair& ev = thread_events(2);
    e = h2d(dev + o_scans, 0, tab2_bytes);
    if (e == hipSuccess) ev_record(ev.a, s);
    if (e == hipSuccess) e = launch_jsync_sync(d_scans, d_wgs, nwg, d_recs, s);
    if (e == hipSuccess) e = hipMemsetAsync(d_changed, 0, sizeof(int), s);
    if (e == hipSuccess) e = launch_jsync_fix(d_scans, m, d_wgs, nwg, d_recs, d_changed, s);
    if (e == hipSuccess)
        e = launch_jsync_bases_decode(d_scans, m, d_wgs, nwg, d_recs, reinterpret_cast<LaneBase*>(dev + o_bases),
                                      dev + o_cs, d_status, s);
    if (e == hipSuccess) ev_record(ev.b, s);
    int rounds = 0;  // the settle kernel's most rounds over the batch's images
    if (e == hipSuccess) e = d2h(0, reinterpret_cast<const uint8_t*>(d_status), sizeof(int) * m);
    if (e == hipSuccess) e = d2h(up256(sizeof(int) * m), reinterpret_cast<const uint8_t*>(d_changed), sizeof(int));
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) {
        std::memcpy(hstatus.data(), hp, sizeof(int) * m);
        std::memcpy(&rounds, hp + up256(sizeof(int) * m), sizeof(int));
    }
    if (e != hipSuccess) {
        if (e != hipSuccess) (void)hip_fail(e, "jpeg entropy decode");
        for (int k = 0; k < m; ++k)
            if (ok[k]) host_idx.push_back(idx[k]);
        return;
    }
#ifdef IK_JPEG_DUMP  // dev experiment: every image's unstuffed words, lane tables and coefficients
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_jdump_mu);
        g_jdump.assign(m, {});
        for (int k = 0; k < m; ++k) {
            if (!ok[k]) continue;
            const Decoder& d = *ds[idx[k]];
            const Lay& L = lay[k];
            const int nl = ivl_lane[L.ivl0 + d.js_nivl];
            auto get = [&](int what, const void* src, size_t bytes) {
                g_jdump[k][what].resize(bytes);
                (void)hipMemcpy(g_jdump[k][what].data(), src, bytes, hipMemcpyDeviceToHost);
            };
            get(0, dev + L.out, d.js_len);
            get(1, dev + o_ivl + sizeof(long long) * L.ivl0, sizeof(long long) * (d.js_nivl + 1));
            get(2, dev + o_recs + sizeof(LaneRec) * L.lane0, sizeof(LaneRec) * nl);
            get(3, dev + o_bases + sizeof(LaneBase) * L.lane0, sizeof(LaneBase) * nl);
            get(4, dev + L.coef, d.nblocks * 64 * sizeof(int16_t));
            g_jdump[k][5].resize(sizeof(int) * (d.js_nivl + 1));
            std::memcpy(g_jdump[k][5].data(), ivl_lane.data() + L.ivl0, sizeof(int) * (d.js_nivl + 1));
            g_jdump[k][6].resize(sizeof(int) * 2);
            std::memcpy(g_jdump[k][6].data(), &hstatus[k], sizeof(int));
            std::memcpy(g_jdump[k][6].data() + sizeof(int), &rounds, sizeof(int));
        }
    }
#endif
    {  // ik_batch_last_timing: the decoding launches' time and algorithmic bytes
        double scan = 0, coef = 0;
        for (int k = 0; k < m; ++k)
            if (ok[k]) {
                scan += (double)ds[idx[k]]->js_len;
                coef += (double)ds[idx[k]]->nblocks * 64 * sizeof(int16_t);
            }
        const int d = current_device();
        batch_timing_add(d, kBtJpegHuffMs, ev_pair_ms(ev));
        batch_timing_add(d, kBtJpegScanBytes, scan);
        batch_timing_add(d, kBtJpegCoefBytes, coef);
        batch_timing_add(d, kBtJpegImages, (double)(lanes_used ? std::count(ok.begin(), ok.end(), 1) : 0));
        batch_timing_add(d, kBtJpegLanes, (double)lanes_used);
    }
    // ---- 5. reconstruction: every image in three launches ----
    {
        JpegReconItem* items = reinterpret_cast<JpegReconItem*>(hp);
        int mi = 0, max_w = 0, max_h = 0;
        long long max_blocks = 0;
        bool any_fast = false, any_slow = false;
        for (int k = 0; k < m; ++k) {
            if (!ok[k]) continue;
            const int i = idx[k];
            if (hstatus[k]) { host_idx.push_back(i); continue; }
            const Decoder& d = *ds[i];
            JpegGeom g = lay[k].g;
            g.qt = reinterpret_cast<const uint16_t*>(dev + lay[k].qt);
            g.coef = reinterpret_cast<const int16_t*>(dev + lay[k].coef);
            g.planes = dev + lay[k].pl;
            ik_image* img = nullptr;
            st[i] = alloc_image((uint32_t)d.width, (uint32_t)d.height, d.comps.size() == 1 ? 1u : 3u, &img);
            if (st[i]) continue;
            outs[i] = img;
            const bool fast = jpeg_zune_fast(g);
            items[mi++] = JpegReconItem{g, img->d, img->pitch, fast ? 1 : 0, 0};
            max_blocks = std::max(max_blocks, g.nblocks);
            max_w = std::max(max_w, g.W);
            max_h = std::max(max_h, g.H);
            any_fast = any_fast || fast;
            any_slow = any_slow || !fast;
        }
        const JpegReconItem* d_items = reinterpret_cast<const JpegReconItem*>(dev + o_items);
        e = h2d(dev + o_items, 0, sizeof(JpegReconItem) * mi);
        if (e == hipSuccess) e = launch_jpeg_reconstruct_batch(d_items, mi, max_blocks, max_w, max_h, any_fast, any_slow, true, s);
        if (e != hipSuccess) (void)hip_fail(e, "jpeg reconstruct");
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    for (int k = 0; k < m; ++k) {
        const int i = idx[k];
        if (!ok[k] || hstatus[k] || !outs[i]) continue;
        if (e != hipSuccess) {  // the device failed: the host decoder takes them
            ik_image_free(outs[i]);
            outs[i] = nullptr;
            st[i] = IK_OK;
            host_idx.push_back(i);
            continue;
        }
        g_jpeg_gpu_streams += 1;
    }
    if (timing)
        fprintf(stderr, "[jsync] %d images, %lld lanes, %d fix rounds: layout %.2f, sync %.2f, tables %.2f, upload wait %.2f, "
                "unstuff %.2f ms, total %.2f ms\n", m, lanes_used, rounds, tm_layout, tm_sync, tm_tables, tm_upwait, t_unstuff,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

}  // namespace
int decode_jpeg_batch(const uint8_t* const* bytes, const size_t* lens, int n, ik_image** outs, int* status,
                      std::string* msgs, const JpegUpload* up);
namespace {

// try_gpu: baseline scans go through the self-synchronising GPU decoder (the batch
// path with one image), progressive scans with restart intervals scan by scan
// (k_jpeg_prog); anything else, and any stream the GPU finds inconsistent, goes
// through the host decoder
int decode_jpeg_impl(const uint8_t* bytes, size_t n, ik_image** out, bool try_gpu) {
    static const bool timing = getenv("IK_TIMING") != nullptr;  // dev: phase times to stderr
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = timing ? now() : 0;
    Decoder d;
    d.b = bytes;
    d.end = bytes + n;
    d.try_gpu = try_gpu;
    int st = d.parse();
    if (st) return st;
    if (d.need_host) return decode_jpeg_impl(bytes, n, out, false);  // several scans: all on the host
    if (d.js) {
        int status = IK_OK;
        std::string msg;
        st = decode_jpeg_batch(&bytes, &n, 1, out, &status, &msg, nullptr);
        if (st && !msg.empty()) return fail(st, "%s", msg.c_str());
        return st;
    }
    const int nc = (int)d.comps.size();
    JpegGeom g;
    const size_t plane_bytes = make_geom(d, g);

    // device scratch: [qtables 4x64 u16][coefficients][planes][progressive scans]
    const size_t qbytes = 256 * sizeof(uint16_t);
    const size_t cbytes = d.nblocks * 64 * sizeof(int16_t);
    std::vector<uint16_t> q(256, 0);
    qtables(d, q.data());
    const double t1 = timing ? now() : 0;
    ik_image* img = nullptr;
    st = alloc_image((uint32_t)d.width, (uint32_t)d.height, nc == 1 ? 1u : 3u, &img);
    if (st) return st;
    const double t2 = timing ? now() : 0;
    const size_t pl_off = qbytes + (cbytes + 255) / 256 * 256;
    const size_t q_off = pl_off + (plane_bytes + 255) / 256 * 256;
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
    uint8_t* dev = scratch(q_off + pstage.size());
    if (!dev) { ik_image_free(img); return fail(IK_ERR_DEVICE, "cannot allocate device scratch"); }
    hipStream_t s = thread_stream();
    st = copy_h2d_2d(dev, qbytes, reinterpret_cast<const uint8_t*>(q.data()), qbytes, qbytes, 1, s);
    if (!st && prog) {
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
                prog ? "gpu entropy" : "host entropy", t1 - t0, t2 - t1, t3 - t2, now() - t3);
    (prog ? g_jpeg_gpu_streams : g_jpeg_host_streams) += 1;
    *out = img;
    return IK_OK;
}

}  // namespace

int decode_jpeg_batch(const uint8_t* const* bytes, const size_t* lens, int n, ik_image** outs, int* status,
                      std::string* msgs, const JpegUpload* up) {
    // 1. parse every stream (host threads); baseline scans are deferred to the GPU
    std::vector<std::unique_ptr<Decoder>> ds(n);
    std::vector<int> st(n, IK_OK);
    auto note = [&](int i) {
        if (st[i] && msgs) {
            char buf[512];
            ik_last_error(buf, sizeof(buf));
            msgs[i] = buf;
        }
    };
    static const bool timing = getenv("IK_TIMING") != nullptr;
    const auto tp0 = std::chrono::steady_clock::now();
    parallel_for(n, 0, [&](int i) {
        ds[i].reset(new Decoder());
        ds[i]->b = bytes[i];
        ds[i]->end = bytes[i] + lens[i];
        ds[i]->try_gpu = true;
        st[i] = ds[i]->parse();
        note(i);
    });
    if (timing)
        fprintf(stderr, "[jpeg-batch] %d streams parsed in %.2f ms\n", n,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count());
    std::vector<int> js_idx, host_idx, prog_idx;
    for (int i = 0; i < n; ++i) {
        outs[i] = nullptr;
        if (st[i]) continue;
        if (ds[i]->js && !ds[i]->need_host) js_idx.push_back(i);
        else if (!ds[i]->prog.empty() && !ds[i]->need_host) prog_idx.push_back(i);  // one by one, GPU
        else host_idx.push_back(i);
    }
    // 2. the baseline scans: the self-synchronising GPU decoder over all of them at once
    jsync_batch(ds, js_idx, outs, st, host_idx, bytes, up);
    // 3. everything else: progressive scans with restart intervals on the GPU image by
    // image, the rest (and anything the GPU found inconsistent) with host entropy decoding
    const int nh = (int)host_idx.size();
    host_idx.insert(host_idx.end(), prog_idx.begin(), prog_idx.end());
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

int decode_jpeg_device(const uint8_t* bytes, size_t n, ik_image** out) { return decode_jpeg_impl(bytes, n, out, true); }

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

#ifdef IK_JPEG_DUMP
// dev experiment: part `what` of image i of the last self-synchronising batch
// (0 unstuffed bytes, 1 interval bits, 2 lane records, 3 lane bases, 4 coefficients,
// 5 interval lanes, 6 status and fix rounds); returns its size
extern "C" long long ik_dev_jpeg_dump(int i, int what, uint8_t* out, size_t cap) {
    std::lock_guard<std::mutex> lk(ik::g_jdump_mu);
    if (i < 0 || i >= (int)ik::g_jdump.size() || what < 0 || what > 6) return -1;
    const auto& v = ik::g_jdump[i][what];
    if (out) std::memcpy(out, v.data(), std::min(cap, v.size()));
    return (long long)v.size();
}
#endif
