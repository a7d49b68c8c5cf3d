// ik_vp8x_host.cpp -- the exact WebP coder's host half (encode_image's WebP branch,
// reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp WebPEncodeRGB): libwebp's
// segment analysis and macroblock decisions run on the GPU (ik_vp8_analysis.hip,
// ik_vp8x.hip); here the epoch/diagonal schedule, the segment set-up, and the
// bitstream: the tokens in RecordTokens order with the final probabilities, libwebp's
// boolean coder, partition 0 (header, segment map, modes), the filter levels libwebp
// raises after coding, and the RIFF container -- the same file WebPEncodeRGB writes
// (tests/test_gpu_vp8x.py; the model is oracle/vp8_modes.c).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"
#include "ik_vp8_gpu.h"
#include "ik_vp8x_gpu.h"

namespace ik {

namespace {

using namespace vp8x;

// ---- libwebp's boolean coder (utils/bit_writer_utils.c) ----
struct BitWriter {
    int32_t range = 255 - 1, value = 0;
    int run = 0, nb_bits = -8;
    std::vector<uint8_t> buf;

    void flush() {
        const int s = 8 + nb_bits;
        const int32_t bits = value >> s;
        value -= bits << s;
        nb_bits -= 8;
        if ((bits & 0xff) != 0xff) {
            if ((bits & 0x100) && !buf.empty()) buf.back()++;  // carry into the bytes written
            for (; run > 0; --run) buf.push_back((bits & 0x100) ? 0x00 : 0xff);
            buf.push_back((uint8_t)(bits & 0xff));
        } else {
            run++;  // 0xff bytes wait: a carry may still come
        }
    }
    int put(int bit, int prob) {
        const int split = (range * prob) >> 8;
        if (bit) {
            value += split + 1;
            range -= split + 1;
        } else {
            range = split;
        }
        if (range < 127) {
            int shift = 0;
            while (((range + 1) << shift) < 128) ++shift;
            range = ((range + 1) << shift) - 1;
            value <<= shift;
            nb_bits += shift;
            if (nb_bits > 0) flush();
        }
        return bit;
    }
    int uniform(int bit) {
        const int split = range >> 1;
        if (bit) {
            value += split + 1;
            range -= split + 1;
        } else {
            range = split;
        }
        if (range < 127) {
            range = ((range + 1) << 1) - 1;
            value <<= 1;
            nb_bits += 1;
            if (nb_bits > 0) flush();
        }
        return bit;
    }
    void bits(uint32_t v, int nb) {
        for (uint32_t mask = 1u << (nb - 1); mask; mask >>= 1) uniform((v & mask) != 0);
    }
    void sbits(int v, int nb) {
        if (!uniform(v != 0)) return;
        if (v < 0) bits(((uint32_t)(-v) << 1) | 1u, nb + 1);
        else bits((uint32_t)v << 1, nb + 1);
    }
    void finish() {
        bits(0, 9 - nb_bits);
        nb_bits = 0;
        flush();
    }
};

void put_le32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// The WebP file of one image from the device's decisions.
void write_file(int w, int h, const XMB* mbs, const uint8_t* probas, const ik_vp8_segment_header& hd,
                const int* max_edge, const XSeg* segs, std::vector<uint8_t>& out) {
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16;
    // the token partition, in RecordTokens order, with the final probabilities
    BitWriter b1;
    {
        std::vector<int> top((size_t)mb_w * 9, 0);
        for (int my = 0; my < mb_h; ++my) {
            int left[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int mx = 0; mx < mb_w; ++mx) {
                record_mb([](uint32_t, int bit) { return bit; }, mbs[my * mb_w + mx], &top[(size_t)mx * 9], left,
                          [&](int bit, uint32_t id) {
                    if (id & 0x4000u) b1.put(bit, (int)(id & 0xffu));
                    else b1.put(bit, probas[id]);
                });
            }
        }
        b1.finish();
    }
    // VP8AdjustFilterStrength: each segment's level at least what its DC-only MBs' largest
    // step needs (kLevelsFromDelta[sharpness 0] is the identity on 0..63)
    int level[4], max_level = 0;
    for (int s = 0; s < 4; ++s) {
        const int delta = (max_edge[s] * segs[s].y2.q[1]) >> 3;
        const int lv = delta < 63 ? delta : 63;
        level[s] = hd.fstrength[s] > lv ? hd.fstrength[s] : lv;
        if (level[s] > max_level) max_level = level[s];
    }
    // partition 0
    BitWriter b0;
    b0.uniform(0);  // colour space
    b0.uniform(0);  // clamping
    if (b0.uniform(hd.num_segments > 1)) {
        b0.uniform(hd.update_map);
        if (b0.uniform(1)) {
            b0.uniform(1);  // absolute values
            for (int s = 0; s < 4; ++s) b0.sbits(hd.quant[s], 7);
            for (int s = 0; s < 4; ++s) b0.sbits(level[s], 6);
        }
        if (hd.update_map)
            for (int s = 0; s < 3; ++s)
                if (b0.uniform(hd.probs[s] != 255)) b0.bits((uint32_t)hd.probs[s], 8);
    }
    b0.uniform(0);  // normal loop filter
    b0.bits((uint32_t)max_level, 6);
    b0.bits(0, 3);  // sharpness
    b0.uniform(0);  // no lf deltas
    b0.bits(0, 2);  // one token partition
    b0.bits((uint32_t)hd.quant[0], 7);
    b0.sbits(0, 4);
    b0.sbits(0, 4);
    b0.sbits(0, 4);
    b0.sbits(hd.dq_uv_dc, 4);
    b0.sbits(hd.dq_uv_ac, 4);
    b0.uniform(0);  // no entropy refresh
    for (int i = 0; i < 1056; ++i)
        if (b0.put(probas[i] != kCoeffProbs0[i], kCoeffUpdateProbs[i])) b0.bits(probas[i], 8);
    b0.uniform(0);  // no skip probability
    for (int i = 0; i < mb_w * mb_h; ++i) {
        const int mx = i % mb_w, my = i / mb_w;
        const XMB& m = mbs[i];
        if (hd.update_map) {
            if (b0.put(m.seg >= 2, hd.probs[0])) b0.put(m.seg & 1, hd.probs[2]);
            else b0.put(m.seg & 1, hd.probs[1]);
        }
        if (b0.put(m.ymode != 4, 145)) {
            const int mode = m.ymode;
            if (b0.put(mode == 1 || mode == 3, 156)) b0.put(mode == 1, 128);
            else b0.put(mode == 2, 163);
        } else {
            for (int k = 0; k < 16; ++k) {
                const int bx = k & 3, by = k >> 2;
                const int top = by ? m.bmodes[k - 4] : (my ? mbs[i - mb_w].bmodes[12 + bx] : 0);
                const int left = bx ? m.bmodes[k - 1] : (mx ? mbs[i - 1].bmodes[by * 4 + 3] : 0);
                const uint8_t* p = kBModeProbs + (top * 10 + left) * 9;
                const int mode = m.bmodes[k];
                if (b0.put(mode != 0, p[0]))
                    if (b0.put(mode != 1, p[1]))
                        if (b0.put(mode != 2, p[2])) {
                            if (!b0.put(mode >= 6, p[3])) {
                                if (b0.put(mode != 3, p[4])) b0.put(mode != 4, p[5]);
                            } else if (b0.put(mode != 6, p[6])) {
                                if (b0.put(mode != 7, p[7])) b0.put(mode != 8, p[8]);
                            }
                        }
            }
        }
        if (b0.put(m.uvmode != 0, 142))
            if (b0.put(m.uvmode != 2, 114)) b0.put(m.uvmode != 3, 183);
    }
    b0.finish();
    // RIFF + VP8 chunk (profile 0: normal filter)
    size_t vp8_size = 10 + b0.buf.size() + b1.buf.size();
    const size_t pad = vp8_size & 1;
    vp8_size += pad;
    const size_t riff_size = 4 + 8 + vp8_size;
    out.assign(8 + riff_size, 0);
    uint8_t* o = out.data();
    std::memcpy(o, "RIFF", 4);
    put_le32(o + 4, (uint32_t)riff_size);
    std::memcpy(o + 8, "WEBPVP8 ", 8);
    put_le32(o + 16, (uint32_t)vp8_size);
    const uint32_t bits = (1u << 4) | ((uint32_t)b0.buf.size() << 5);
    o[20] = (uint8_t)bits;
    o[21] = (uint8_t)(bits >> 8);
    o[22] = (uint8_t)(bits >> 16);
    o[23] = 0x9d;
    o[24] = 0x01;
    o[25] = 0x2a;
    o[26] = (uint8_t)(w & 0xff);
    o[27] = (uint8_t)(w >> 8);
    o[28] = (uint8_t)(h & 0xff);
    o[29] = (uint8_t)(h >> 8);
    std::memcpy(o + 30, b0.buf.data(), b0.buf.size());
    std::memcpy(o + 30 + b0.buf.size(), b1.buf.data(), b1.buf.size());
}

// The call's schedule, cached per thread for its geometry: epochs at libwebp's
// probability refreshes; tickets in (epoch, diagonal, image) order, each epoch's folds
// after its MBs.  Diagonals are found by one counting pass per epoch.
struct XSchedule {
    int w = 0, h = 0, n = 0;
    std::vector<int> bounds;
    std::vector<uint64_t> tasks;
    int grid = 0;
};

const XSchedule& exact_schedule(int w, int h, int n) {
    static thread_local XSchedule sc;
    if (sc.w == w && sc.h == h && sc.n == n) return sc;
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16, nmb = mb_w * mb_h;
    const int M = (nmb >> 3) < 96 ? 96 : (nmb >> 3);
    sc.bounds.assign(1, 0);
    for (int k = M; k < nmb; k += M + 1) sc.bounds.push_back(k);
    sc.bounds.push_back(nmb);
    sc.tasks.clear();
    sc.tasks.reserve((size_t)n * (nmb + sc.bounds.size()));
    int widest = 1;
    std::vector<int> first, list;
    for (size_t e = 0; e + 1 < sc.bounds.size(); ++e) {
        const int k0 = sc.bounds[e], k1 = sc.bounds[e + 1];
        // (an epoch that starts mid-row holds MBs of smaller diagonals in its next row)
        int d0 = 1 << 30, d1 = -1;
        for (int k = k0; k < k1; ++k) {
            d0 = std::min(d0, k % mb_w + 2 * (k / mb_w));
            d1 = std::max(d1, k % mb_w + 2 * (k / mb_w));
        }
        first.assign((size_t)(d1 - d0 + 2), 0);  // counting sort of the epoch's MBs by diagonal
        for (int k = k0; k < k1; ++k) ++first[(size_t)(k % mb_w + 2 * (k / mb_w) - d0 + 1)];
        for (size_t d = 1; d < first.size(); ++d) first[d] += first[d - 1];
        list.assign((size_t)(k1 - k0), 0);
        std::vector<int> at(first.begin(), first.end() - 1);
        for (int k = k0; k < k1; ++k) list[(size_t)at[(size_t)(k % mb_w + 2 * (k / mb_w) - d0)]++] = k;
        const uint64_t ep = (uint64_t)e << 48;
        for (int d = 0; d <= d1 - d0; ++d) {
            const int a = first[(size_t)d], b = first[(size_t)d + 1];
            widest = std::max(widest, (b - a) * n);
            for (int i = 0; i < n; ++i)
                for (int j = a; j < b; ++j) sc.tasks.push_back(ep | ((uint64_t)i << 32) | (uint32_t)list[(size_t)j]);
        }
        for (int i = 0; i < n; ++i) sc.tasks.push_back((1ull << 63) | ep | ((uint64_t)i << 32));
    }
    // resident workgroups: the widest diagonal's MBs (every workgroup more would hold
    // LDS and registers that another batch's decode kernels beside the coder lose)
    // (IK_VP8X_GRID: a multiple of that, e.g. 0.5 -- dev A/B)
    static const double mul = getenv("IK_VP8X_GRID") ? atof(getenv("IK_VP8X_GRID")) : 1.0;
    const int want = std::max(1, (int)(std::max(mul, 0.05) * widest));
    sc.grid = (int)std::min<size_t>(std::min(want, 2048), sc.tasks.size());
    sc.w = w;
    sc.h = h;
    sc.n = n;
    return sc;
}

// libwebp VP8SetSegmentParams' quantiser for a segment alpha (-127..127) at quality q:
// the pow() is the host's (the same libm call libwebp makes)
void segment_quant_table(float quality, int* qtab) {
    const double amp = 0.9 * 50 / 100. / 128.;  // SNS_TO_DQ, sns 50
    const double Q = quality / 100.;
    const double linear_c = (Q < 0.75) ? Q * (2. / 3.) : 2. * Q - 1.;
    const double c_base = pow(linear_c, 1 / 3.);
    for (int s = -127; s <= 127; ++s) {
        const int v = (int)(127. * (1. - pow(c_base, 1. - amp * s)));
        qtab[s + 127] = v < 0 ? 0 : (v > 127 ? 127 : v);
    }
}

}  // namespace

// n images of w x h YUV420 planes on the device (yuv_stride bytes apart) -> the WebP
// files libwebp's WebPEncodeRGB writes at this quality.  Device work on the thread's
// coder stream (ordered after its main stream, which produced the planes): segment
// analysis, set-up, ONE persistent launch for every decision and statistics fold,
// the records back; then the files on the host.
int webp_encode_exact(const uint8_t* d_yuv, size_t yuv_stride, int n, int w, int h, int quality,
                      std::vector<std::vector<uint8_t>>& outs) {
    if (n < 1 || n > 65535 || w < 1 || h < 1 || w > 16383 || h > 16383)
        return fail(IK_ERR_INVALID, "bad WebP shape %dx%d x %d", w, h, n);
    hipStream_t ts = thread_stream();
    if (!ts) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    // the coder's stream: the highest priority, so its launch is dispatched ahead of
    // another batch's decode kernels; ordered after the caller's stream by an event
    hipStream_t s = ts;
    hipEvent_t ev = nullptr;
    if (thread_prio_stream(&s, &ev) && s != ts) {
        IK_HIP(hipEventRecord(ev, ts));
        IK_HIP(hipStreamWaitEvent(s, ev, 0));
    } else {
        s = ts;
    }
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16, nmb = mb_w * mb_h;
    const float q = (float)quality;
    const XSchedule& sc = exact_schedule(w, h, n);
    const int nep = (int)sc.bounds.size() - 1;
    // device buffers (one allocation, 256-byte aligned parts); the hand-off words first,
    // zeroed by one memset per call
    size_t off = 0;
    auto part = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t sync_words = 4 + (size_t)n * nmb + 2ull * n * nep;
    const size_t o_sync = part(4 * sync_words);
    const size_t sync_bytes = off;
    const size_t o_alpha = part((size_t)nmb * n), o_uva = part((size_t)nmb * n * 2), o_kseg = part((size_t)nmb * n);
    const size_t o_rec = part(sizeof(vp8::SegRecord) * n), o_hdr = part(sizeof(ik_vp8_segment_header) * n);
    const size_t o_mbs = part(sizeof(XMB) * nmb * n), o_edges = part(sizeof(XEdge) * nmb * n);
    const size_t o_seg = part((size_t)nmb * n), o_segs = part(sizeof(XSeg) * 4 * n);
    const size_t o_lc = part(2ull * kCostRows * kLevelTab * n), o_pr = part(1056ull * n), o_st = part(4ull * 1056 * n);
    const size_t o_me = part(16ull * n);
    const size_t o_qtab = part(4 * 255), o_bounds = part(4 * sc.bounds.size()), o_tasks = part(8 * sc.tasks.size());
    uint8_t* d = scratch_slot(kScratchExact, off);
    if (!d) return fail(IK_ERR_DEVICE, "cannot allocate the exact coder's work area (%zu bytes)", off);
    // the constants: quantiser table, epoch bounds, tickets (through pinned staging)
    const size_t const_bytes = off - o_qtab;
    uint8_t* hc = pinned_slot(kPinnedExactIn, const_bytes);
    if (!hc) return IK_ERR_NOMEM;
    segment_quant_table(q, reinterpret_cast<int*>(hc));
    std::memcpy(hc + (o_bounds - o_qtab), sc.bounds.data(), 4 * sc.bounds.size());
    std::memcpy(hc + (o_tasks - o_qtab), sc.tasks.data(), 8 * sc.tasks.size());
    IK_HIP(hipMemcpyAsync(d + o_qtab, hc, const_bytes, hipMemcpyHostToDevice, s));
    IK_HIP(hipMemsetAsync(d + o_sync, 0, sync_bytes, s));
    XArgs a{};
    a.yuv = d_yuv;
    a.yuv_stride = yuv_stride;
    a.w = w;
    a.h = h;
    a.mb_w = mb_w;
    a.mb_h = mb_h;
    a.mbs = (XMB*)(d + o_mbs);
    a.edges = (XEdge*)(d + o_edges);
    a.seg = d + o_seg;
    a.segs = (XSeg*)(d + o_segs);
    a.lc = (uint16_t*)(d + o_lc);
    a.pr = d + o_pr;
    a.stats = (uint32_t*)(d + o_st);
    a.max_edge = (int*)(d + o_me);
    a.use_derr = q <= 98.f;  // ERROR_DIFFUSION_QUALITY
    XRun r{};
    r.tasks = (const uint64_t*)(d + o_tasks);
    r.ntasks = (uint32_t)sc.tasks.size();
    r.nep = (uint32_t)nep;
    r.bounds = (const int*)(d + o_bounds);
    r.sync = (uint32_t*)(d + o_sync);
    r.done = r.sync + 4;
    r.cnt = r.done + (size_t)n * nmb;
    r.ready = r.cnt + (size_t)n * nep;
    // 1. segment analysis (ik_vp8_analysis.hip), 2. set-up, 3. every decision and fold
    IK_HIP(vp8::launch_vp8_analysis(d_yuv, yuv_stride, n, w, h, d + o_alpha, (uint16_t*)(d + o_uva), d + o_kseg,
                                    (vp8::SegRecord*)(d + o_rec), s));
    IK_HIP(launch_vp8x_setup(a, (const vp8::SegRecord*)(d + o_rec), d + o_kseg, (const int*)(d + o_qtab),
                             (ik_vp8_segment_header*)(d + o_hdr), n, s));
    IK_HIP(launch_vp8x_run(a, r, sc.grid, s));
    // 4. the records back (~830 B per MB), the final probabilities, the filter-edge
    // maxima, the headers and the error word; the files on the host
    const size_t rec_bytes = sizeof(XMB) * (size_t)nmb * n;
    const size_t o_hpr = rec_bytes, o_hme = o_hpr + 1056ull * n, o_hhd = o_hme + 16ull * n;
    const size_t o_herr = o_hhd + sizeof(ik_vp8_segment_header) * n, hbytes = o_herr + 16;
    uint8_t* hp = pinned_slot(kPinnedExactOut, hbytes);
    if (!hp) return IK_ERR_NOMEM;
    IK_HIP(hipMemcpyAsync(hp, d + o_mbs, rec_bytes, hipMemcpyDeviceToHost, s));
    IK_HIP(hipMemcpyAsync(hp + o_hpr, d + o_pr, 1056ull * n, hipMemcpyDeviceToHost, s));
    IK_HIP(hipMemcpyAsync(hp + o_hme, d + o_me, 16ull * n, hipMemcpyDeviceToHost, s));
    IK_HIP(hipMemcpyAsync(hp + o_hhd, d + o_hdr, sizeof(ik_vp8_segment_header) * n, hipMemcpyDeviceToHost, s));
    IK_HIP(hipMemcpyAsync(hp + o_herr, d + o_sync, 8, hipMemcpyDeviceToHost, s));
    IK_HIP(hipStreamSynchronize(s));
    uint32_t err_word = 0;
    std::memcpy(&err_word, hp + o_herr + 4, 4);
    if (err_word) return fail(IK_ERR_DEVICE, "exact WebP coder: a dependency wait timed out on the device");
    const XMB* mbs = reinterpret_cast<const XMB*>(hp);
    const uint8_t* pr = hp + o_hpr;
    const int* me = reinterpret_cast<const int*>(hp + o_hme);
    const ik_vp8_segment_header* hdr = reinterpret_cast<const ik_vp8_segment_header*>(hp + o_hhd);
    outs.resize(n);
    parallel_for(n, n < 16 ? n : 16, [&](int i) {
        XSeg segs[4];
        for (int sg = 0; sg < 4; ++sg) segs[sg] = setup_segment(hdr[i].quant[sg], hdr[i].dq_uv_dc, hdr[i].dq_uv_ac, 50);
        write_file(w, h, mbs + (size_t)nmb * i, pr + (size_t)1056 * i, hdr[i], me + (size_t)4 * i, segs, outs[i]);
    });
    return IK_OK;
}


// The exact coder's first two stages alone (ik_vp8_analyze_device): libwebp's segment
// analysis and the segment set-up on the device, the final segment map and headers
// into host memory; on the calling thread's stream, waits.
int vp8_analyze_setup(const uint8_t* d_yuv, size_t yuv_stride, int n, int w, int h, float quality, uint8_t* seg,
                      ik_vp8_segment_header* hdr) {
    hipStream_t s = thread_stream();
    if (!s) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    const int mb_w = (w + 15) / 16, mb_h = (h + 15) / 16, nmb = mb_w * mb_h;
    size_t off = 0;
    auto part = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_alpha = part((size_t)nmb * n), o_uva = part((size_t)nmb * n * 2), o_kseg = part((size_t)nmb * n);
    const size_t o_rec = part(sizeof(vp8::SegRecord) * n), o_hdr = part(sizeof(ik_vp8_segment_header) * n);
    const size_t o_seg = part((size_t)nmb * n), o_segs = part(sizeof(XSeg) * 4 * n);
    const size_t o_lc = part(2ull * kCostRows * kLevelTab * n), o_pr = part(1056ull * n), o_st = part(4ull * 1056 * n);
    const size_t o_me = part(16ull * n), o_qtab = part(4 * 255);
    uint8_t* d = scratch_slot(kScratchExact, off);
    if (!d) return fail(IK_ERR_DEVICE, "cannot allocate the segment analysis' work area (%zu bytes)", off);
    uint8_t* hc = pinned_slot(kPinnedExactIn, 4 * 255);
    if (!hc) return IK_ERR_NOMEM;
    segment_quant_table(quality, reinterpret_cast<int*>(hc));
    IK_HIP(hipMemcpyAsync(d + o_qtab, hc, 4 * 255, hipMemcpyHostToDevice, s));
    XArgs a{};
    a.yuv = d_yuv;
    a.yuv_stride = yuv_stride;
    a.w = w;
    a.h = h;
    a.mb_w = mb_w;
    a.mb_h = mb_h;
    a.seg = d + o_seg;
    a.segs = (XSeg*)(d + o_segs);
    a.lc = (uint16_t*)(d + o_lc);
    a.pr = d + o_pr;
    a.stats = (uint32_t*)(d + o_st);
    a.max_edge = (int*)(d + o_me);
    IK_HIP(vp8::launch_vp8_analysis(d_yuv, yuv_stride, n, w, h, d + o_alpha, (uint16_t*)(d + o_uva), d + o_kseg,
                                    (vp8::SegRecord*)(d + o_rec), s));
    IK_HIP(launch_vp8x_setup(a, (const vp8::SegRecord*)(d + o_rec), d + o_kseg, (const int*)(d + o_qtab),
                             (ik_vp8_segment_header*)(d + o_hdr), n, s));
    IK_HIP(hipMemcpyAsync(seg, d + o_seg, (size_t)nmb * n, hipMemcpyDeviceToHost, s));
    IK_HIP(hipMemcpyAsync(hdr, d + o_hdr, sizeof(ik_vp8_segment_header) * n, hipMemcpyDeviceToHost, s));
    IK_HIP(hipStreamSynchronize(s));
    return IK_OK;
}

}  // namespace ik

using namespace ik;

extern "C" int ik_webp_encode_exact_device(const uint8_t* dev_yuv, size_t yuv_stride, uint32_t n, uint32_t w,
                                           uint32_t h, int quality, uint8_t** outs, size_t* out_lens) {
    IK_API_ENTER();
    if (!dev_yuv || !outs || !out_lens) return fail(IK_ERR_INVALID, "null pointer");
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    const size_t ysz = (size_t)w * h + 2 * (size_t)((w + 1) / 2) * ((h + 1) / 2);
    if (n > 1 && yuv_stride < ysz) return fail(IK_ERR_INVALID, "image stride %zu under the planes' %zu bytes", yuv_stride, ysz);
    std::vector<std::vector<uint8_t>> files;
    if (int rc = webp_encode_exact(dev_yuv, yuv_stride, (int)n, (int)w, (int)h, q, files)) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        outs[i] = (uint8_t*)malloc(files[i].size() ? files[i].size() : 1);
        if (!outs[i]) {
            for (uint32_t j = 0; j < i; ++j) {
                free(outs[j]);
                outs[j] = nullptr;
                out_lens[j] = 0;
            }
            return fail(IK_ERR_NOMEM, "out of host memory");
        }
        std::memcpy(outs[i], files[i].data(), files[i].size());
        out_lens[i] = files[i].size();
    }
    return IK_OK;
}
