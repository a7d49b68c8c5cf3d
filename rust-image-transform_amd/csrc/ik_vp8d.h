// ik_vp8d.h -- the WebP (VP8 lossy) decoder of decode_image (reference src/transform.rs:31
// -> image 0.25.8 load_from_memory_with_format -> WebP).  RFC 6386 key-frame decoding with
// the pixels of libwebp's WebPDecodeRGB, which the tests pin it to (fancy chroma
// upsampling, libwebp's fixed-point YUV -> RGB).  Shared by the host (RIFF / frame
// header and partition 0: segments, filter, quantisers, probabilities, every MB's
// modes; ik_vp8d_host.cpp) and the GPU (token partitions, reconstruction + loop filter,
// colour; ik_vp8d.hip).
#pragma once
#include <cstdint>

#include "ik_vp8x.h"

namespace ik {
namespace vp8d {

using namespace ::ik::vp8;
using ::ik::vp8x::xclip8;

// ---- boolean decoder: libwebp bit_reader's arithmetic (value window, range - 1,
// bits = valid bits below the 8-bit window), so that running out of data sets eof
// at the same symbol as VP8GetBit does.  Src supplies big-endian words / bytes of
// the stream at byte offsets.
struct BitReader {
    uint64_t value;
    uint32_t range;  // range - 1, in [126, 254]
    int bits;
    int eof;
    uint32_t pos, end;  // byte offsets of the next unread byte and the end
};

template <class Src>
IK_HD void br_load(BitReader& br, const Src& s) {
    if (br.pos + 4 <= br.end) {
        br.value = (br.value << 32) | s.be32(br.pos);
        br.pos += 4;
        br.bits += 32;
    } else if (br.pos < br.end) {
        br.value = (br.value << 8) | s.byte(br.pos);
        br.pos += 1;
        br.bits += 8;
    } else if (!br.eof) {
        br.value <<= 8;
        br.bits += 8;
        br.eof = 1;
    } else {
        br.bits = 0;
    }
}
template <class Src>
IK_HD void br_init(BitReader& br, const Src& s, uint32_t start, uint32_t end) {
    br.value = 0;
    br.range = 255 - 1;
    br.bits = -8;
    br.eof = 0;
    br.pos = start;
    br.end = end;
    br_load(br, s);
}
IK_HD int log2_floor(uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
    return 31 - __clz(v);
#else
    return 31 - __builtin_clz(v);
#endif
}
template <class Src>
IK_HD int br_bit(BitReader& br, const Src& s, int prob) {
    uint32_t range = br.range;
    if (br.bits < 0) br_load(br, s);
    const int pos = br.bits;
    const uint32_t split = (range * (uint32_t)prob) >> 8;
    const uint32_t value = (uint32_t)(br.value >> pos);
    int bit;
    if (value > split) {
        range -= split;
        br.value -= (uint64_t)(split + 1) << pos;
        bit = 1;
    } else {
        range = split + 1;
        bit = 0;
    }
    const int shift = 7 ^ log2_floor(range);
    range <<= shift;
    br.bits -= shift;
    br.range = range - 1;
    return bit;
}
template <class Src>
IK_HD int br_value(BitReader& br, const Src& s, int n) {  // VP8GetValue: n bits, MSB first
    int v = 0;
    while (n-- > 0) v |= br_bit(br, s, 0x80) << n;
    return v;
}
template <class Src>
IK_HD int br_signed_value(BitReader& br, const Src& s, int n) {  // VP8GetSignedValue
    const int v = br_value(br, s, n);
    return br_bit(br, s, 0x80) ? -v : v;
}

struct HostSrc {  // the stream in host memory
    const uint8_t* b;
    IK_HD uint32_t byte(uint32_t i) const { return b[i]; }
    IK_HD uint32_t be32(uint32_t i) const {
        return (uint32_t)b[i] << 24 | (uint32_t)b[i + 1] << 16 | (uint32_t)b[i + 2] << 8 | b[i + 3];
    }
};

// ---- what partition 0 and the headers hand to the device ----
struct DMB {  // one macroblock's modes (libwebp ParseIntraMode)
    uint8_t is_i4, ymode, uvmode, seg;  // ymode / uvmode: DC 0, TM 1, V 2, H 3
    uint8_t skip, pad[3];               // skip: the MB's skip flag (when the frame codes them)
    uint8_t bmodes[16];                 // intra-4 sub-block modes, raster order (i16: ymode)
};
static_assert(sizeof(DMB) == 24, "DMB layout");

struct DSeg {  // per segment: VP8ParseQuant's matrices; PrecomputeFilterStrengths [i16, i4]
    int16_t y1[2], y2[2], uv[2];  // [0] DC, [1] AC
    uint8_t limit[2], ilevel[2], hev[2], pad[2];
};

// one frame: geometry, filter, token partitions (offsets into the file bytes),
// segments and coefficient probabilities ([type][band][ctx] rows of 11, padded to 16)
struct alignas(16) DFrame {
    int32_t w, h, mb_w, mb_h;
    int32_t filter_type;  // 0 none, 1 simple, 2 normal (libwebp dec->filter_type_)
    int32_t num_parts;
    int32_t use_skip;
    int32_t pad0;
    uint32_t part_off[8], part_end[8];
    DSeg seg[4];
    uint8_t proba[4 * 8 * 3 * 16];
};

// ---- reconstruction helpers (BPS-pitched, as ik_vp8x.h) ----
// the 4x4 block (bx, by) of the size x size prediction of mode m (DC 0, TM 1, V 2, H 3)
// from top[0..size) / left[0..size) / left[-1] (the corner; the caller supplies the
// frame-edge values 127 / 129, so only DC needs has_top / has_left: libwebp's
// DC16NoTop / NoLeft / NoTopLeft)
IK_HD void pred_block(uint8_t* dst, int m, const uint8_t* left, int left_step, const uint8_t* top, int corner,
                      int size, int has_top, int has_left, int bx, int by) {
    int dc = 0;
    if (m == 0) {
        const int shift = size == 16 ? 4 : 3;
        int s = 0;
        if (has_top)
            for (int j = 0; j < size; ++j) s += top[j];
        if (has_left)
            for (int j = 0; j < size; ++j) s += left[j * left_step];
        if (has_top && has_left) dc = (s + size) >> (shift + 1);
        else if (has_top || has_left) dc = (s + (size >> 1)) >> shift;
        else dc = 0x80;
    }
    for (int y = 4 * by; y < 4 * by + 4; ++y)
        for (int x = 4 * bx; x < 4 * bx + 4; ++x) {
            int p;
            if (m == 0) p = dc;
            else if (m == 1) p = xclip8(left[y * left_step] + top[x] - corner);
            else if (m == 2) p = top[x];
            else p = left[y * left_step];
            dst[(x - 4 * bx) + (y - 4 * by) * vp8x::BPS] = (uint8_t)p;
        }
}

// ---- loop filter (libwebp dsp/dec.c): one line across an edge at p (q0), step
// between its samples; thresh2 = 2 * thresh + 1 ----
IK_HD int sclip1(int v) { return v < -128 ? -128 : v > 127 ? 127 : v; }  // VP8ksclip1
IK_HD int sclip2(int v) { return v < -16 ? -16 : v > 15 ? 15 : v; }      // VP8ksclip2
IK_HD int uclip(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }         // VP8kclip1
IK_HD int iabs(int v) { return v < 0 ? -v : v; }

IK_HD void do_filter2(uint8_t* p, int step) {
    const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
    const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
    p[-step] = (uint8_t)uclip(p0 + a2);
    p[0] = (uint8_t)uclip(q0 - a1);
}
IK_HD void do_filter4(uint8_t* p, int step) {
    const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
    const int a = 3 * (q0 - p0);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
    p[-2 * step] = (uint8_t)uclip(p1 + a3);
    p[-step] = (uint8_t)uclip(p0 + a2);
    p[0] = (uint8_t)uclip(q0 - a1);
    p[step] = (uint8_t)uclip(q1 - a3);
}
IK_HD void do_filter6(uint8_t* p, int step) {
    const int p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
    const int q0 = p[0], q1 = p[step], q2 = p[2 * step];
    const int a = sclip1(3 * (q0 - p0) + sclip1(p1 - q1));
    const int a1 = (27 * a + 63) >> 7, a2 = (18 * a + 63) >> 7, a3 = (9 * a + 63) >> 7;
    p[-3 * step] = (uint8_t)uclip(p2 + a3);
    p[-2 * step] = (uint8_t)uclip(p1 + a2);
    p[-step] = (uint8_t)uclip(p0 + a1);
    p[0] = (uint8_t)uclip(q0 - a1);
    p[step] = (uint8_t)uclip(q1 - a2);
    p[2 * step] = (uint8_t)uclip(q2 - a3);
}
IK_HD int hev(const uint8_t* p, int step, int t) {
    return iabs(p[-2 * step] - p[-step]) > t || iabs(p[step] - p[0]) > t;
}
IK_HD int needs_filter(const uint8_t* p, int step, int t2) {
    return 4 * iabs(p[-step] - p[0]) + iabs(p[-2 * step] - p[step]) <= t2;
}
IK_HD int needs_filter2(const uint8_t* p, int step, int t2, int it) {
    const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
    const int q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
    if (4 * iabs(p0 - q0) + iabs(p1 - q1) > t2) return 0;
    return iabs(p3 - p2) <= it && iabs(p2 - p1) <= it && iabs(p1 - p0) <= it && iabs(q3 - q2) <= it &&
           iabs(q2 - q1) <= it && iabs(q1 - q0) <= it;
}
// FilterLoop26 (macroblock edges) / FilterLoop24 (inner edges) on one line
IK_HD void filter_line(uint8_t* p, int step, int t2, int it, int hev_t, bool mb_edge) {
    if (!needs_filter2(p, step, t2, it)) return;
    if (hev(p, step, hev_t)) do_filter2(p, step);
    else if (mb_edge) do_filter6(p, step);
    else do_filter4(p, step);
}
IK_HD void simple_line(uint8_t* p, int step, int t2) {
    if (needs_filter(p, step, t2)) do_filter2(p, step);
}

// ---- colour (libwebp yuv.h, YUV_FIX2 = 6) ----
IK_HD int mult_hi(int v, int c) { return (v * c) >> 8; }
IK_HD int yuv_clip8(int v) { return (v & ~((256 << 6) - 1)) == 0 ? (v >> 6) : v < 0 ? 0 : 255; }
IK_HD int yuv_r(int y, int v) { return yuv_clip8(mult_hi(y, 19077) + mult_hi(v, 26149) - 14234); }
IK_HD int yuv_g(int y, int u, int v) {
    return yuv_clip8(mult_hi(y, 19077) - mult_hi(u, 6419) - mult_hi(v, 13320) + 8708);
}
IK_HD int yuv_b(int y, int u) { return yuv_clip8(mult_hi(y, 19077) + mult_hi(u, 33050) - 17685); }

// The fancy upsampler's chroma for output column c (libwebp UPSAMPLE_FUNC, per
// channel): near / far are the chroma rows weighted 3 / 1 vertically, len the width
IK_HD int fancy_chroma(const uint8_t* near, const uint8_t* far, int c, int len) {
    if (c == 0) return (3 * near[0] + far[0] + 2) >> 2;
    if (!(len & 1) && c == len - 1) {
        const int k = (len - 1) >> 1;
        return (3 * near[k] + far[k] + 2) >> 2;
    }
    const int x = (c + 1) >> 1;  // pair (x - 1, x)
    const int s = near[x - 1] + near[x] + far[x - 1] + far[x] + 8;
    if (c & 1) return (((s + 2 * (near[x] + far[x - 1])) >> 3) + near[x - 1]) >> 1;
    return (((s + 2 * (near[x - 1] + far[x])) >> 3) + near[x]) >> 1;
}

}  // namespace vp8d
}  // namespace ik
