// ik_jpeg_sync.h -- self-synchronising parallel Huffman decoding of baseline JPEG
// scans, shared by the GPU kernels (ik_jpeg.hip k_jsync_*) and their CPU model
// (ik_jpeg_model.cpp, CPU tests only).
//
// decode_image on a JPEG (reference src/transform.rs:31 -> image 0.25.8 ->
// zune-jpeg 0.4.21) spends its time in the entropy decoding of the scan: one
// serial bit sequence per restart interval (ITU T.81 F.2.2).  Huffman codes
// resynchronise: a decoder started at an arbitrary bit soon lands on the true
// block boundaries with the true block-in-MCU phase.  So every interval (the whole
// scan when there are no restart markers) is cut into lanes of kLaneBits bits and
// decoded by thousands of lanes at once (Weissenberger & Schmidt's scheme, with
// a warm-up instead of a first blind round):
//
//  0. unstuff: the entropy-coded bytes lose their stuffing (FF 00 -> FF) and
//     restart markers; each interval starts at a known bit with the DC
//     predictions at zero and block phase 0 (k_jsync_unstuff_*).
//  1. sync: lane q of an interval decodes from kWarmBits before its own range
//     (from a guessed block start, phase 0) up to the first block starting at or
//     after its range start -- its START state (bit, phase) -- then on to the first
//     block starting at or after its range end -- its EXIT state -- counting the
//     blocks in between and summing their DC differences per component.  The
//     first lane of an interval starts exactly at the interval start.
//  2. fix rounds: lane q is consistent when its START equals lane q-1's EXIT.
//     Each round re-decodes every inconsistent lane from its predecessor's EXIT
//     (no warm-up: that state is exact once the predecessor is), until a round
//     changes nothing.  Consistency propagates from the interval starts, so the
//     rounds needed are the longest run of lanes the warm-up did not synchronise.
//  3. bases: block counts and DC sums -> per-lane block index and DC prediction
//     (prefix sums within each interval); blocks counted past an interval's known
//     block count come from its end padding and are cut.
//  4. decode: every lane decodes its blocks again from its START with those
//     bases and writes the coefficients.
#pragma once
#include <stdint.h>

#ifndef IK_HD
#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define IK_HD __host__ __device__ __forceinline__
#else
#define IK_HD inline
#endif
#endif
#ifndef IK_GLOBAL
#if defined(__HIP_DEVICE_COMPILE__)
#define IK_GLOBAL __attribute__((address_space(1)))
#else
#define IK_GLOBAL
#endif
#endif

namespace ik {

// Baseline Huffman tables: 4 DC then 4 AC, canonical form plus a 9-bit lookahead
// (look = length << 8 | value, length 0 = longer code).
struct JpegHuffTables {
    uint16_t look[8][512];
    int maxcode[8][18], valptr[8][17], mincode[8][17];
    int lj[8][17];  // left-justified 16-bit bound of the codes up to each length (carried over empty lengths)
    uint8_t vals[8][256];
    // AC codes whose code + magnitude bits fit the 9-bit lookahead, decoded in one
    // lookup (entry: value << 8 | run << 4 | bits; 0 = take the general path)
    int16_t fast_ac[4][512];
};

namespace jsync {

constexpr int kMaxBPM = 10;       // blocks per MCU at most (T.81 B.2.3)
constexpr int kLaneBits = 1024;   // a lane's range (bits of unstuffed data), default
constexpr int kWarmBits = 1024;   // decoded before the range from a guessed start, default

// A state at a block start: its first bit, the block's index in the MCU and a
// valid flag; 0 = no state (a bad code on the way)
IK_HD uint64_t st_pack(uint64_t bit, int j) { return bit | (uint64_t)j << 48 | 1ull << 63; }
IK_HD uint64_t st_bit(uint64_t s) { return s & ((1ull << 48) - 1); }
IK_HD int st_j(uint64_t s) { return (int)((s >> 48) & 15); }

// one scan of one image, as the sync kernels see it
struct Scan {
    const IK_GLOBAL uint32_t* words;  // unstuffed data, big-endian words, >= kPadWords zero words past nbits
    const IK_GLOBAL long long* ivl;   // [nivl + 1] interval start bits (ivl[nivl] = nbits)
    int nivl;
    long long lane0;                  // the scan's first lane in the batch's lane arrays
    const IK_GLOBAL int* ivl_lane;    // [nivl + 1] first lane of each interval, relative to lane0
    long long ivl_blocks;             // blocks per interval (restart * bpm), the last one takes the rest
    int L, W;                         // lane bits, warm-up bits
    long long total_blocks;
    int bpm;
    int comp_of[kMaxBPM], bx_of[kMaxBPM], by_of[kMaxBPM];  // per block of an MCU: scan component, offset
    int mcux, single, single_bw;
    int h[4], v[4], bw[4], td[4], ta[4];
    long long blk0[4];
    const JpegHuffTables* tabs;
    int16_t* coef;                    // [block][64] natural order
};
// zero words a decoder may read past the data: one block of zero bits (16 + 11 + 63 * (16 + 10)),
// plus the reader's three-word window
constexpr int kPadWords = (16 + 11 + 63 * (16 + 10) + 31) / 32 + 4;

// per-lane results of the sync and fix passes
struct LaneRec {
    uint64_t start, exit;  // states (st_pack)
    int nblk;              // blocks starting in the lane's range
    int err;               // 0, or 1 + blocks decoded before a bad code
    int dc[4];             // DC differences summed per scan component
    int work;              // blocks decoded, the warm-up included (a cost measure)
    int pad;
};

// per-lane block base and DC predictions (the bases pass), the decode pass's input
struct LaneBase {
    long long block;  // the scan's block index of the lane's first block
    int count;        // blocks the lane decodes (cut at its interval's end)
    int dc[4];        // DC predictions before its first block
    int head;         // (bases pass scratch: a segment head at or before the lane in its chunk)
};

// the interval holding lane r of a scan (r < S.ivl_lane[S.nivl]): the last k
// with ivl_lane[k] <= r
IK_HD int lane_interval(const Scan& S, int r) {
    int lo = 0, hi = S.nivl - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S.ivl_lane[mid] <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// MSB-first reader over the unstuffed words; bits at or past `end` read as zero
// (the interval's end: the host decoder feeds zeros at a marker)
// (a block never advances more than 27 bits between two peeks, so the window
// moves one word at a time, and the word after it is loaded a step ahead)
struct Bits {
    const IK_GLOBAL uint32_t* w;
    uint64_t pos, end;
    uint64_t buf;  // words [idx, idx + 1]
    uint32_t nxt;  // word idx + 2
    long long idx;
    IK_HD void init(const IK_GLOBAL uint32_t* words, uint64_t p, uint64_t e) {
        w = words;
        pos = p;
        end = e;
        idx = (long long)(p >> 5);
        buf = (uint64_t)w[idx] << 32 | w[idx + 1];
        nxt = w[idx + 2];
    }
    IK_HD uint32_t peek32() {
        const long long i = (long long)(pos >> 5);
        if (i != idx) {
            if (i == idx + 1) {
                buf = buf << 32 | nxt;
            } else {
                buf = (uint64_t)w[i] << 32 | w[i + 1];
            }
            nxt = w[i + 2];
            idx = i;
        }
        uint32_t v = (uint32_t)((buf << (pos & 31)) >> 32);
        if (pos + 32 > end) v = pos >= end ? 0u : v & ~(0xFFFFFFFFu >> (uint32_t)(end - pos));
        return v;
    }
};

IK_HD int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

IK_HD int sym(Bits& br, const JpegHuffTables& T, int t) {
    const uint32_t win = br.peek32();
    const int lv = T.look[t][win >> 23];
    if (lv >> 8) {
        br.pos += (uint32_t)lv >> 8;
        return lv & 0xff;
    }
    const int code = (int)(win >> 16);
    int len = 10;
    for (int l = 10; l <= 16; ++l) len += code >= T.lj[t][l];
    if (len > 16) return -1;
    br.pos += (uint32_t)len;
    const int c = code >> (16 - len);
    return T.vals[t][T.valptr[t][len] + c - T.mincode[t][len]];
}

IK_HD int getbits(Bits& br, int n) {
    if (!n) return 0;
    const uint32_t v = br.peek32() >> (32 - n);
    br.pos += (uint32_t)n;
    return (int)v;
}

// One block (T.81 F.2.2.1-2): the DC difference into *dcdiff; the AC levels into
// blk (natural order, zz maps zigzag -> natural) when kStore, else skipped.
// false on a bad code.  (A template flag, not a null test: an LDS block at
// address 0 is a valid pointer the compiler may still treat as null.)
template <bool kStore, typename Blk>
IK_HD bool block(Bits& br, const JpegHuffTables& T, const uint8_t* zz, int td, int ta, int* dcdiff, Blk blk) {
    const int t = sym(br, T, td);
    if (t < 0 || t > 11) return false;
    *dcdiff = t ? extend(getbits(br, t), t) : 0;
    for (int k = 1; k < 64;) {
        const int fa = T.fast_ac[ta][br.peek32() >> 23];
        if (fa) {  // a short run/size code and its magnitude in one lookup
            k += (fa >> 4) & 15;
            br.pos += (uint32_t)(fa & 15);
            if (k > 63) return false;
            if (kStore) blk[zz[k]] = (int16_t)(fa >> 8);
            ++k;
            continue;
        }
        const int rs = sym(br, T, 4 + ta);
        if (rs < 0) return false;
        const int r = rs >> 4, sz = rs & 15;
        if (!sz) {
            if (r != 15) break;  // EOB
            k += 16;
            continue;
        }
        k += r;
        if (k > 63) return false;
        const int val = extend(getbits(br, sz), sz);
        if (kStore) blk[zz[k]] = (int16_t)val;
        ++k;
    }
    return true;
}

// Unstuffing of the entropy-coded bytes b[0, n) of a scan (everything between the
// SOS header and the marker that ends the scan), byte by byte from its neighbours
// so that a GPU thread can decide any byte alone -- the same stream the host
// decoder's reader sees (ik_jpeg_decode.cpp BitReader, libjpeg jdhuff.c):
//   FF 00  -> FF (the 00 is stuffing)
//   FF Dn  -> nothing; a restart marker: the next interval starts here
//   FF FF  -> the first FF is fill before a marker: nothing
//   a lone FF as the last byte -> FF (as the host reader: stuffed)
IK_HD bool unstuff_keep(int prev, int cur, int next, bool last) {
    if (cur == 0xFF) return last || next == 0x00;
    if (prev == 0xFF && (cur == 0x00 || (cur >= 0xD0 && cur <= 0xD7))) return false;
    return true;
}
IK_HD bool unstuff_rst(int cur, int next) { return cur == 0xFF && next >= 0xD0 && next <= 0xD7; }
// a marker other than RSTn inside the range (bad data: the host decoder decides)
IK_HD bool unstuff_bad(int cur, int next, bool last) {
    return cur == 0xFF && !last && next != 0x00 && next != 0xFF && !(next >= 0xD0 && next <= 0xD7);
}

// the lane's range [lo, hi) and its interval's [s, e)
struct LaneGeom {
    uint64_t lo, hi, s, e;
    int q;  // index in the interval (0: starts exactly at s)
};

IK_HD LaneGeom lane_geom(const Scan& S, int ivl, int q) {
    LaneGeom g;
    g.s = (uint64_t)S.ivl[ivl];
    g.e = (uint64_t)S.ivl[ivl + 1];
    g.q = q;
    g.lo = g.s + (uint64_t)q * (uint64_t)S.L;
    const uint64_t hi = g.lo + (uint64_t)S.L;
    g.hi = hi < g.e ? hi : g.e;
    return g;
}

// Decode from `from` (a state) over the blocks that start before g.hi: blocks that
// start before g.lo are skipped (the warm-up), the state at the first block start
// >= g.lo becomes r.start, the blocks from there on are counted, and the state at
// the first block start >= g.hi becomes r.exit.  A bad code ends the lane (r.err;
// r.exit = 0, and r.start = 0 if it came before g.lo).
IK_HD void run_lane(const Scan& S, const JpegHuffTables& T, const uint8_t* zz, const LaneGeom& g, uint64_t from,
                    LaneRec& r) {
    r.start = r.exit = 0;
    r.nblk = 0;
    r.err = 0;
    r.work = 0;
    for (int c = 0; c < 4; ++c) r.dc[c] = 0;
    Bits br;
    br.init(S.words, st_bit(from), g.e);
    int j = st_j(from);
    bool counting = false;
    // the DC sums in four registers (an array indexed by the component would live
    // in scratch memory on the GPU)
    int dc0 = 0, dc1 = 0, dc2 = 0, dc3 = 0;
    for (;;) {
        if (!counting && br.pos >= g.lo) {
            counting = true;
            r.start = st_pack(br.pos, j);
        }
        if (br.pos >= g.hi) {
            r.exit = st_pack(br.pos, j);
            break;
        }
        const int c = S.comp_of[j];
        int diff;
        if (!block<false>(br, T, zz, S.td[c], S.ta[c], &diff, (int16_t*)nullptr)) {
            r.err = 1 + r.nblk;
            if (counting) ++r.nblk;  // the block started in the range (a padding block at an interval end)
            break;
        }
        ++r.work;
        if (counting) {
            ++r.nblk;
            const int d = diff;
            dc0 += c == 0 ? d : 0;
            dc1 += c == 1 ? d : 0;
            dc2 += c == 2 ? d : 0;
            dc3 += c == 3 ? d : 0;
        }
        j = j + 1 == S.bpm ? 0 : j + 1;
    }
    r.dc[0] = dc0;
    r.dc[1] = dc1;
    r.dc[2] = dc2;
    r.dc[3] = dc3;
}

// the sync pass's starting state for lane q: the interval start for q = 0, else a
// guessed block start (phase 0) kWarmBits before the range, not before the interval
IK_HD uint64_t warm_start(const Scan& S, const LaneGeom& g) {
    if (g.q == 0) return st_pack(g.s, 0);
    const uint64_t w = g.lo - g.s > (uint64_t)S.W ? g.lo - (uint64_t)S.W : g.s;
    return st_pack(w, 0);
}

// coefficient block of the scan's block b (decode order)
IK_HD long long block_index(const Scan& S, long long b) {
    const long long mcu = b / S.bpm;
    const int j = (int)(b - mcu * S.bpm);
    const int c = S.comp_of[j];
    if (S.single) return S.blk0[c] + (mcu / S.single_bw) * S.bw[c] + (mcu % S.single_bw);
    const long long my = mcu / S.mcux, mx = mcu - my * S.mcux;
    return S.blk0[c] + (my * S.v[c] + S.by_of[j]) * S.bw[c] + mx * S.h[c] + S.bx_of[j];
}

}  // namespace jsync
}  // namespace ik
