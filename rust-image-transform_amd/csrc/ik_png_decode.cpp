// ik_png_decode.cpp -- decode_image on PNG streams with the GPU doing the inflate
// and the unfiltering (reference src/transform.rs:31 -> image 0.25.8 ->
// png 0.18).  Kernels: ik_png.hip; algorithm: ik_inflate.h / ik_png_plan.h.
//
// Per batch of streams:
//   host   chunk walk + CRC check of every chunk (png verifies CRCs), IHDR;
//          the IDAT payloads of all streams -> one pinned buffer -> one H2D copy
//   GPU    k_png_find (block-start candidates per 16 KiB chunk)
//   GPU    k_png_decode rounds (token streams + output lengths); the host checks
//          the lane chain after each (a false candidate is dropped and its
//          predecessor decodes on)
//   GPU    k_png_expand (tokens -> u16 symbols + window markers), k_png_resolve
//          (filtered rows into the image, markers followed), k_png_unfilter
// The GPU path covers 8- and 16-bit, non-interlaced, non-palette streams
// without tRNS (png's EXPAND leaves those samples as they are); everything else,
// and any stream the GPU finds inconsistent, goes through the host decoder, whose
// error messages are png's.  The zlib Adler-32 is not verified, as png 0.18 does
// not by default (CRCs cover the data).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/imagekit_hip.h"
#include "ik_png.h"
#include "ik_png_plan.h"
#include "ik_runtime.h"

namespace ik {

namespace {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
size_t up256(size_t v) { return (v + 255) & ~size_t(255); }

struct PngJob {
    int idx = -1;                                   // stream index in the batch
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, bpp = 0, ch = 0;       // bytes per pixel, image channels
    std::vector<std::pair<const uint8_t*, uint32_t>> idat;
    size_t zlen = 0;                                 // IDAT payload bytes (zlib stream)
    uint64_t raw_total = 0;
    int rowbytes = 0;
    // device layout (offsets into the batch work area)
    size_t o_words = 0, o_u16 = 0, o_ft = 0;
    size_t z_off = 0;                                // offset of the stream in the pinned buffer
    uint64_t nbits = 0;
    int chunk0 = 0, nchunks = 0;                     // its chunks in the batch chunk table
    pngplan::Lanes lanes;
    int state = 0;                                   // 0 running, 1 verified, -1 host fallback
    ik_image* img = nullptr;
};

// png 0.18 + image's EXPAND: which streams the GPU path decodes.  Returns false
// for streams that must go to the host decoder (which also produces png's
// errors for malformed ones).
bool parse_png(const uint8_t* b, size_t n, PngJob& J) {
    if (n < 8 || std::memcmp(b, "\x89PNG\r\n\x1a\n", 8)) return false;
    size_t pos = 8;
    bool ihdr = false, trns = false;
    int interlace = 0;
    while (pos + 12 <= n) {
        const uint32_t len = be32(b + pos);
        if (len > n - pos - 12) return false;
        const uint8_t* type = b + pos + 4;
        const uint8_t* data = b + pos + 8;
        // (IDAT CRCs are checked while the payload is staged: decode_png_batch)
        if (std::memcmp(type, "IDAT", 4) && png_chunk_crc(type, data, len) != be32(data + len)) return false;
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13 || ihdr) return false;
            J.w = be32(data);
            J.h = be32(data + 4);
            J.depth = data[8];
            J.ctype = data[9];
            interlace = data[12];
            ihdr = true;
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns = true;
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (len) J.idat.emplace_back(data, len);
            J.zlen += len;
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    if (!ihdr || J.idat.empty() || !J.w || !J.h || interlace || trns) return false;
    if (J.depth != 8 && J.depth != 16) return false;
    int spp;
    switch (J.ctype) {
    case 0: spp = 1; break;
    case 2: spp = 3; break;
    case 4: spp = 2; break;
    case 6: spp = 4; break;
    default: return false;  // palette: host
    }
    J.ch = spp;
    J.bpp = spp * J.depth / 8;
    if (J.depth == 16) return false;  // 16-bit samples: host (see decode_png)
    const uint64_t rb = (uint64_t)J.w * J.bpp;
    // image's default limit: 512 MiB of decoded pixels
    if (rb * J.h > (512ull << 20) || rb > 0x7FFFFFF0ull) return false;
    J.rowbytes = (int)rb;
    J.raw_total = (rb + 1) * J.h;
    // zlib header: CM 8, window <= 32 KiB, FCHECK, no preset dictionary
    const uint8_t* z0 = J.idat[0].first;
    uint8_t cmf, flg;
    if (J.idat[0].second >= 2) { cmf = z0[0]; flg = z0[1]; }
    else if (J.idat.size() > 1) { cmf = z0[0]; flg = J.idat[1].first[0]; }
    else return false;
    if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 || (flg & 0x20)) return false;
    return true;
}

struct HostTables {
    std::vector<int> chunk_img, chunk_idx, pages, xst;
    std::vector<int64_t> cand, obase;
    std::vector<PngLaneDev> lanes;
    std::vector<std::pair<int, int>> who;
    std::vector<infl::LaneResult> res;
    std::vector<int2> rows;
};

// Small host<->device transfers of the kernel phase (lane tables, offsets, row and
// page tables, per-lane results) go through a copy kernel on the compute stream
// that reads or writes pinned host memory directly, not through SDMA copies: those
// queue behind any multi-GB stream upload on the same engine (another batch's, with
// batches in flight), measured at 8-10 ms per table.  One pinned region per batch
// (bump-allocated), so no transfer overwrites one a pending kernel still reads.
struct Xfer {
    uint8_t* pin = nullptr;   // host view
    uint8_t* dpin = nullptr;  // the same memory as the device addresses it
    size_t cap = 0, used = 0;
    hipStream_t s = nullptr;
    bool init(size_t bytes, hipStream_t st) {
        s = st;
        used = 0;
        pin = pinned_slot(3, bytes);
        void* dp = nullptr;
        if (pin && hipHostGetDevicePointer(&dp, pin, 0) != hipSuccess) dp = nullptr;
        dpin = reinterpret_cast<uint8_t*>(dp);
        cap = dpin ? bytes : 0;
        return dpin != nullptr;
    }
    size_t take(size_t n) {  // offset of a fresh region, or ~0 when the area is used up
        n = (n + 255) & ~size_t(255);
        if (used + n > cap) return ~size_t(0);
        const size_t o = used;
        used += n;
        return o;
    }
    hipError_t h2d(void* dev, const void* host, size_t n) {
        if (!n) return hipSuccess;
        const size_t o = take(n + 4);
        if (o == ~size_t(0))  // (more decode rounds than the area was sized for) the copy engine
            return copy_h2d_2d(reinterpret_cast<uint8_t*>(dev), n, reinterpret_cast<const uint8_t*>(host), n, n, 1, s)
                       ? hipErrorUnknown : hipSuccess;
        std::memcpy(pin + o, host, n);
        return launch_copy_words(reinterpret_cast<const uint32_t*>(dpin + o), reinterpret_cast<uint32_t*>(dev),
                                 (n + 3) / 4, s);
    }
    // (synchronises the stream)
    hipError_t d2h(void* host, const void* dev, size_t n) {
        if (!n) return hipSuccess;
        const size_t o = take(n + 4);
        hipError_t e = hipSuccess;
        size_t done = 0;
        if (o != ~size_t(0)) {
            e = launch_copy_words(reinterpret_cast<const uint32_t*>(dev), reinterpret_cast<uint32_t*>(dpin + o), n / 4, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) std::memcpy(host, pin + o, n & ~size_t(3));
            done = n & ~size_t(3);
        }
        if (e == hipSuccess && done < n) {  // a tail under one word, or no room: the copy engine
            e = hipMemcpyAsync(reinterpret_cast<uint8_t*>(host) + done, reinterpret_cast<const uint8_t*>(dev) + done,
                               n - done, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
        }
        return e;
    }
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the last batch's stage times on this thread (ik_png_last_timing): host parse +
// staging, then device ms of find / count (all rounds) / emit / resolve / unfilter
// from HIP events on the thread's stream, wall ms, rounds, lanes, streams sent to
// the GPU, streams the GPU decoded (verified), streams the host decoder took,
// tokens the verified lanes wrote (the decode pass's output, the expand pass's input)
thread_local double t_png_timing[13];
// process-wide: PNG streams decoded by the GPU path / by the host decoder
std::atomic<unsigned long long> g_png_gpu_streams{0}, g_png_host_streams{0};
struct Events {
    hipEvent_t e[12] = {};
    bool ok = false;
    Events() {
        ok = true;
        for (auto& x : e) ok = ok && hipEventCreate(&x) == hipSuccess;
    }
};
Events& events() {
    static thread_local Events ev;
    return ev;
}
float ev_ms(int a, int b) {
    float ms = 0;
    if (!events().ok || hipEventElapsedTime(&ms, events().e[a], events().e[b]) != hipSuccess) return 0;
    return ms;
}

}  // namespace

namespace {
std::atomic<long long> g_png_gpu_min{-2};  // -2: not read yet; -1: GPU path off
long long png_gpu_min() {
    long long v = g_png_gpu_min.load();
    if (v == -2) {
        const char* e = getenv("IK_PNG_GPU");
        const char* m = getenv("IK_PNG_GPU_MIN");
        v = (e && !strcmp(e, "0")) ? -1 : (m ? (long long)strtoull(m, nullptr, 10) : (256ll << 10));
        long long expect = -2;
        g_png_gpu_min.compare_exchange_strong(expect, v);
        v = g_png_gpu_min.load();
    }
    return v;
}
}  // namespace

bool png_gpu_enabled(size_t raw_bytes) {
    const long long v = png_gpu_min();
    return v >= 0 && (long long)raw_bytes >= v;
}

int decode_png_batch(const uint8_t* const* bytes, const size_t* lens, int n, ik_image** outs, int* status,
                     std::string* msgs) {
    static const bool timing = getenv("IK_PNG_TIMING") != nullptr;
    const double t0 = now_ms();
    for (double& v : t_png_timing) v = 0;
    Events& ev = events();
    auto rec = [&](int k, hipStream_t st) { if (ev.ok) (void)hipEventRecord(ev.e[k], st); };
    // a stream the GPU path gives up on: the host decoder takes it (and gives png's
    // error if the stream is malformed); IK_PNG_TIMING says why
    auto reject = [&](PngJob& j, const char* why) {
        j.state = -1;
        if (timing) fprintf(stderr, "[png] stream %d (%ux%u) -> host decoder: %s\n", j.idx, j.w, j.h, why);
    };
    double count_dev = 0;
    std::vector<PngJob> jobs(n);
    std::vector<char> gpu(n, 0);
    parallel_for(n, 0, [&](int i) {
        outs[i] = nullptr;
        status[i] = IK_OK;
        jobs[i].idx = i;
        gpu[i] = parse_png(bytes[i], lens[i], jobs[i]) && png_gpu_enabled(jobs[i].raw_total);
    });
    std::vector<PngJob*> J;
    for (int i = 0; i < n; ++i)
        if (gpu[i]) J.push_back(&jobs[i]);
    const int m = (int)J.size();
    hipStream_t s = thread_stream();
    int rc = IK_OK;
    const uint64_t cbits = kPngChunkBytes * 8;
    if (m) {
        // ---- device layout ----
        constexpr size_t kPad = 512;  // zero bytes past each stream (Bits::wend, the LDS ring's DMAs)
        size_t total = 0, zbytes = 0;
        int nchunks = 0;
        for (PngJob* j : J) {
            j->z_off = zbytes;
            zbytes += ((j->zlen + 3) & ~size_t(3)) + kPad;  // the zero padding travels with the stream
            j->nbits = (uint64_t)j->zlen * 8;
            j->nchunks = (int)((j->nbits - 16 + cbits - 1) / cbits);
            j->chunk0 = nchunks;
            nchunks += j->nchunks;
            j->o_words = total;
            total += up256(((j->zlen + 3) & ~size_t(3)) + kPad);
            j->o_u16 = total;
            total += up256(2 * (j->raw_total + 64));
            j->o_ft = total;
            total += up256(j->h);
        }
        const size_t o_imgs = total;
        total += up256(sizeof(PngImgDev) * m);
        const size_t o_ctab = total;
        total += up256(sizeof(int) * 2 * nchunks);
        const size_t o_cand = total;
        total += up256(sizeof(int64_t) * nchunks);
        const size_t o_err = total;
        total += up256(sizeof(int) * m);
        const size_t o_dyn = total;  // lane tables, results, obase, rows, subtables: sized per round below
        // the work area: lane tables (bounded by the chunk count), row / page
        // tables, unfilter class descriptors, and the token area: a quarter token
        // per compressed bit for every first-round lane, plus half again for lanes
        // that decode again (a dropped successor, an overflow)
        size_t max_lanes = 0;
        uint64_t tok_total = 0;
        for (PngJob* j : J) {
            max_lanes += (size_t)j->nchunks;
            tok_total += infl::tok_capacity(j->nbits, false) + (uint64_t)j->nchunks * (infl::tok_capacity(0, false) +
                                                                                       infl::kTokSlack);
        }
        tok_total += tok_total / 2 + 64;
        size_t dyn = up256(sizeof(PngLaneDev) * max_lanes) + up256(sizeof(infl::LaneResult) * max_lanes) +
                     up256(sizeof(int64_t) * max_lanes) + up256(2 * sizeof(int) * max_lanes) +
                     up256(sizeof(PngImgDev) * m);
        size_t nrows = 0, npages = 0, nbands = 0, ngroups = 0;
        for (PngJob* j : J) {
            nrows += j->h;
            npages += (j->raw_total >> kPngPageShift) + 1;
            nbands += ((size_t)j->h + 63) / 64;
            ngroups += (size_t)png_unfilter_groups((int)j->h);
        }
        // unfilter: band-group table + per-image band offsets (staged), then one
        // progress counter per band and one ticket per class (zeroed)
        const size_t unf_tab = up256(sizeof(int2) * ngroups) + up256(sizeof(int) * m);
        const size_t unf_zero = up256(sizeof(unsigned) * (nbands + 8));
        dyn += up256(sizeof(int2) * nrows) + up256(sizeof(int) * npages) + unf_tab + unf_zero + up256(2 * tok_total);
        uint8_t* dev = rc ? nullptr : scratch_slot(2, o_dyn + dyn);
        if (!rc && !dev) rc = fail(IK_ERR_DEVICE, "cannot allocate the PNG batch work area (%zu bytes)", o_dyn + dyn);
        PngLaneDev* d_lanes = nullptr;
        infl::LaneResult* d_res = nullptr;
        int64_t* d_obase = nullptr;
        int* d_xst = nullptr;
        PngImgDev* d_cls = nullptr;
        int2* d_rows = nullptr;
        int* d_pages = nullptr;
        uint8_t* d_unf = nullptr;
        uint16_t* d_tok = nullptr;
        if (!rc) {
            size_t o = o_dyn;
            d_lanes = reinterpret_cast<PngLaneDev*>(dev + o);
            o += up256(sizeof(PngLaneDev) * max_lanes);
            d_res = reinterpret_cast<infl::LaneResult*>(dev + o);
            o += up256(sizeof(infl::LaneResult) * max_lanes);
            d_obase = reinterpret_cast<int64_t*>(dev + o);
            o += up256(sizeof(int64_t) * max_lanes);
            d_xst = reinterpret_cast<int*>(dev + o);
            o += up256(2 * sizeof(int) * max_lanes);
            d_cls = reinterpret_cast<PngImgDev*>(dev + o);
            o += up256(sizeof(PngImgDev) * m);
            d_rows = reinterpret_cast<int2*>(dev + o);
            o += up256(sizeof(int2) * nrows);
            d_pages = reinterpret_cast<int*>(dev + o);
            o += up256(sizeof(int) * npages);
            d_unf = dev + o;
            o += unf_tab + unf_zero;
            d_tok = reinterpret_cast<uint16_t*>(dev + o);
        }
        uint64_t tok_used = 0;
        Xfer X;
        if (!rc && !X.init(2 * sizeof(PngLaneDev) * max_lanes + sizeof(infl::LaneResult) * max_lanes +
                               sizeof(int64_t) * (max_lanes + nchunks) + 2 * sizeof(int) * max_lanes +
                               sizeof(int2) * (nrows + ngroups) + sizeof(int) * (npages + 2 * m) +
                               3 * sizeof(PngImgDev) * m + (64u << 10), s))
            rc = fail(IK_ERR_NOMEM, "cannot allocate pinned PNG transfer area");
        // phases: staging + upload + block search under the device's upload gate,
        // the decode kernels on under its kernel gate (ik_runtime.h), so that
        // concurrent batches take the GPU in turn
        gate_enter(kGateUpload);
        // with the device free, each stream's block search runs as soon as its copy
        // lands; with another batch's kernels running, the searches wait for the
        // kernel gate (sharing the CUs with those kernels slows both)
        const bool early = gate_try_enter(kGateKernels);
        // ---- image descriptors and the chunk table (before any stream lands) ----
        std::vector<PngImgDev> hd(m);
        // the large host tables are kept per thread between batches (clear() keeps
        // the capacity): fresh multi-MB vectors cost page faults every batch
        static thread_local HostTables ht;
        std::vector<int>& hchunk_img = ht.chunk_img;
        std::vector<int>& hchunk_idx = ht.chunk_idx;
        hchunk_img.assign(nchunks, 0);
        hchunk_idx.assign(nchunks, 0);
        for (int k = 0; k < m && !rc; ++k) {
            PngJob& j = *J[k];
            PngImgDev& d = hd[k];
            d.words = reinterpret_cast<const uint32_t*>(dev + j.o_words);
            d.bit0 = 16;
            d.nbits = j.nbits;
            d.u16 = reinterpret_cast<uint16_t*>(dev + j.o_u16);
            d.raw_total = j.raw_total;
            d.rowbytes = j.rowbytes;
            d.H = (int)j.h;
            d.bpp = j.bpp;
            d.ft = dev + j.o_ft;
            for (int c = 0; c < j.nchunks; ++c) {
                hchunk_img[j.chunk0 + c] = k;
                hchunk_idx[j.chunk0 + c] = c;
            }
        }
        if (!rc) rc = copy_h2d_2d(dev + o_ctab, sizeof(int) * nchunks, reinterpret_cast<const uint8_t*>(hchunk_img.data()),
                                  sizeof(int) * nchunks, sizeof(int) * nchunks, 1, s);
        if (!rc) rc = copy_h2d_2d(dev + o_ctab + sizeof(int) * nchunks, sizeof(int) * nchunks,
                                  reinterpret_cast<const uint8_t*>(hchunk_idx.data()), sizeof(int) * nchunks,
                                  sizeof(int) * nchunks, 1, s);
        if (!rc) rc = copy_h2d_2d(dev + o_imgs, sizeof(PngImgDev) * m, reinterpret_cast<const uint8_t*>(hd.data()),
                                  sizeof(PngImgDev) * m, sizeof(PngImgDev) * m, 1, s);
        const PngImgDev* d_imgs = reinterpret_cast<const PngImgDev*>(dev + o_imgs);
        const int* d_cimg = reinterpret_cast<const int*>(dev + o_ctab);
        const int* d_cidx = d_cimg + nchunks;
        int64_t* d_cand = reinterpret_cast<int64_t*>(dev + o_cand);
        uint8_t* pin = rc ? nullptr : pinned_slot(1, zbytes + 64);
        if (!rc && !pin) rc = fail(IK_ERR_NOMEM, "cannot allocate pinned PNG staging");
        // IDAT payloads -> pinned (host threads), CRC-checked on the way (png
        // verifies every chunk's CRC).  Each stream's H2D copy goes out on the copy
        // stream as soon as it is staged, and its block search on the compute stream
        // as soon as the copy has landed (an event), so the PCIe transfer overlaps
        // the staging of the later streams and the search the transfer
        hipStream_t sc = rc ? nullptr : thread_copy_stream();
        if (!rc && !sc) rc = fail(IK_ERR_DEVICE, "cannot create the PNG copy stream");
        static thread_local std::vector<hipEvent_t> landed;
        while (!rc && (int)landed.size() < m) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                rc = fail(IK_ERR_DEVICE, "cannot create PNG upload events");
                break;
            }
            landed.push_back(e);
        }
        // (the workers below see their own thread_local vector: pass the caller's)
        hipEvent_t* const ev_landed = landed.data();
        std::vector<char> crc_bad(m, 0);
        std::atomic<int> up_err{0};
        std::atomic<long long> t_copy_calls{0};  // dev timing: us spent inside hipMemcpyAsync
        const double t_stage0 = now_ms();
        double t_stage1 = t_stage0;
        if (!rc) {
            rec(0, s);
            // the first streams go up in pieces of <= kPiece bytes, so the PCIe transfer
            // starts after one piece is staged instead of after whole 35-MB streams
            // (measured: 5.5 ms from a batch's start to its first copy); the thread
            // that finishes a stream's last piece records its event, launches its
            // block search and then checks its CRCs; whole streams check their CRCs
            // while staging, as before
            constexpr size_t kPiece = size_t(4) << 20;
            constexpr int kPieced = 2;
            struct Piece { int k; size_t lo, n; };
            std::vector<Piece> pieces;
            std::vector<std::vector<size_t>> seg_off(m);  // logical start of each IDAT segment (pieced streams)
            std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[m]);
            for (int k = 0; k < m; ++k) {
                const PngJob& j = *J[k];
                const size_t tot = ((j.zlen + 3) & ~size_t(3)) + kPad;
                const size_t piece = k < kPieced ? kPiece : tot;
                int np = 0;
                for (size_t lo = 0; lo < tot; lo += piece, ++np) pieces.push_back(Piece{k, lo, std::min(piece, tot - lo)});
                left[k] = np;
                if (np > 1) {
                    size_t o = 0;
                    for (auto& seg : j.idat) { seg_off[k].push_back(o); o += seg.second; }
                }
            }
            parallel_for((int)pieces.size(), 0, [&, s, sc](int pi) {
                const Piece P = pieces[pi];
                const int k = P.k;
                const PngJob& j = *J[k];
                const bool whole = P.lo == 0 && seg_off[k].empty();
                uint8_t* d = pin + j.z_off + P.lo;
                if (whole) {
                    for (auto& seg : j.idat) {
                        if (png_chunk_crc(seg.first - 4, seg.first, seg.second) != be32(seg.first + seg.second)) crc_bad[k] = 1;
                        std::memcpy(d, seg.first, seg.second);
                        d += seg.second;
                    }
                    std::memset(d, 0, pin + j.z_off + P.n - d);
                } else {
                    const std::vector<size_t>& so = seg_off[k];
                    size_t lo = P.lo, n = P.n;
                    size_t si = (size_t)(std::upper_bound(so.begin(), so.end(), lo) - so.begin()) - 1;
                    while (n && lo < j.zlen) {
                        const size_t in = lo - so[si], c = std::min(n, (size_t)j.idat[si].second - in);
                        std::memcpy(d, j.idat[si].first + in, c);
                        d += c; lo += c; n -= c; ++si;
                    }
                    if (n) std::memset(d, 0, n);
                }
                // one plain copy per piece (no memset kernel ahead of it, which would
                // wait for a CU while other kernels run)
                const double tc0 = timing ? now_ms() : 0.0;
                hipError_t e = hipMemcpyAsync(dev + j.o_words + P.lo, pin + j.z_off + P.lo, P.n, hipMemcpyHostToDevice, sc);
                if (timing) t_copy_calls += (long long)(1000.0 * (now_ms() - tc0));
                if (left[k].fetch_sub(1) == 1) {  // the stream is all queued
                    if (early) {
                        if (e == hipSuccess) e = hipEventRecord(ev_landed[k], sc);
                        if (e == hipSuccess) e = hipStreamWaitEvent(s, ev_landed[k], 0);
                        if (e == hipSuccess)
                            e = launch_png_find(d_imgs, d_cimg + j.chunk0, d_cidx + j.chunk0, j.nchunks, cbits,
                                                d_cand + j.chunk0, s);
                    }
                    if (!whole)
                        for (auto& seg : j.idat)
                            if (png_chunk_crc(seg.first - 4, seg.first, seg.second) != be32(seg.first + seg.second))
                                crc_bad[k] = 1;
                }
                if (e != hipSuccess) up_err = (int)e;
            });
            t_stage1 = now_ms();
            gate_leave(kGateUpload);
            if (!early) {  // all copies are on sc: one event after the last, then one search launch
                gate_enter(kGateKernels);
                hipError_t e = hipEventRecord(ev_landed[0], sc);
                if (e == hipSuccess) e = hipStreamWaitEvent(s, ev_landed[0], 0);
                if (e == hipSuccess) e = launch_png_find(d_imgs, d_cimg, d_cidx, nchunks, cbits, d_cand, s);
                if (e != hipSuccess) up_err = (int)e;
            }
            rec(1, s);
        }
        if (!rc && up_err) rc = hip_fail((hipError_t)up_err.load(), "PNG stream upload / block search");
        for (int k = 0; k < m; ++k)
            if (crc_bad[k]) J[k]->state = -1;  // the host decoder reports png's CRC error
        const double t1 = now_ms();
        // ---- candidates ----
        std::vector<int64_t>& cand = ht.cand;
        cand.assign(nchunks, 0);
        if (!rc) {
            hipError_t e = X.d2h(cand.data(), d_cand, sizeof(int64_t) * nchunks);
            if (e != hipSuccess) rc = hip_fail(e, "PNG block search");
        }
        gate_leave(kGateUpload);   // (error paths)
        gate_enter(kGateKernels);
        const double t_gate = now_ms();
        const double t2 = now_ms();
        double mk[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // dev timing marks (IK_PNG_TIMING)
        for (PngJob* j : J) {
            std::vector<int64_t> c(cand.begin() + j->chunk0, cand.begin() + j->chunk0 + j->nchunks);
            pngplan::build(c, j->lanes);
        }
        // ---- decode rounds: token streams; the host checks the lane chain ----
        int rounds = 0, dropped = 0, overflows = 0;
        std::vector<PngLaneDev>& hl = ht.lanes;
        std::vector<std::pair<int, int>>& who = ht.who;  // (job, lane) of each launched lane
        std::vector<infl::LaneResult>& hres = ht.res;
        hl.clear();
        who.clear();
        hres.clear();
        while (!rc) {
            hl.clear();
            who.clear();
            for (int k = 0; k < m; ++k) {
                PngJob& j = *J[k];
                if (j.state) continue;
                pngplan::Lanes& LL = j.lanes;
                for (size_t i = 0; i < LL.start.size(); ++i) {
                    if (!LL.dirty[i]) continue;
                    const uint64_t end = LL.stop[i] == ~0ull ? j.nbits : LL.stop[i];
                    const uint32_t cap = infl::tok_capacity(end > LL.start[i] ? end - LL.start[i] : 0, LL.big[i] != 0);
                    if (cap > LL.tcap[i]) {  // a (larger) region from the area
                        const uint64_t need = cap + infl::kTokSlack;
                        if (tok_used + need > tok_total) { reject(j, "token area full"); break; }  // host decoder
                        LL.tbase[i] = tok_used;
                        LL.tcap[i] = cap;
                        tok_used += need;
                    }
                    PngLaneDev L{};
                    L.start = LL.start[i];
                    L.stop = LL.stop[i];
                    L.tbase = LL.tbase[i];
                    L.ntok = LL.tcap[i];
                    L.img = (uint32_t)k;
                    L.first = i == 0;
                    hl.push_back(L);
                    who.emplace_back(k, (int)i);
                }
            }
            // lanes of a job that just fell back are dropped from the launch
            if (!hl.empty()) {
                size_t w = 0;
                for (size_t t = 0; t < hl.size(); ++t)
                    if (J[who[t].first]->state == 0) { hl[w] = hl[t]; who[w] = who[t]; ++w; }
                hl.resize(w);
                who.resize(w);
            }
            if (hl.empty()) break;
            if (hl.size() > max_lanes) { rc = fail(IK_ERR_DEVICE, "PNG lane table overflow"); break; }
            const size_t lb = sizeof(PngLaneDev) * hl.size();
            if (X.h2d(d_lanes, hl.data(), lb) != hipSuccess) { rc = fail(IK_ERR_DEVICE, "PNG lane table upload"); break; }
            hres.resize(hl.size());
            if (!mk[0]) mk[0] = now_ms();  // plan built, lanes uploaded (first round)
            rec(2, s);
            hipError_t e = launch_png_decode(d_imgs, d_lanes, (int)hl.size(), d_tok, d_res, s);
            rec(3, s);
            if (e == hipSuccess) e = X.d2h(hres.data(), d_res, sizeof(infl::LaneResult) * hl.size());
            if (e != hipSuccess) { rc = hip_fail(e, "PNG inflate (decode)"); break; }
            count_dev += ev_ms(2, 3);
            ++rounds;
            std::vector<char> again(m, 0);  // a job with overflowed lanes: those first, then the check
            for (size_t t = 0; t < hl.size(); ++t) {
                pngplan::Lanes& LL = J[who[t].first]->lanes;
                const int i = who[t].second;
                LL.res[i] = hres[t];
                LL.dirty[i] = 0;
                if (hres[t].status == infl::kLaneOverflow) {
                    ++overflows;
                    if (LL.big[i]) {
                        LL.res[i].status = infl::kLaneCorrupt;  // past the exact bound too (see tok_capacity)
                    } else {
                        LL.big[i] = 1;
                        LL.dirty[i] = 1;
                        again[who[t].first] = 1;
                    }
                }
            }
            for (int k = 0; k < m; ++k) {
                PngJob& j = *J[k];
                if (j.state || again[k]) continue;
                const size_t before = j.lanes.start.size();
                const int st = pngplan::check(j.lanes);
                dropped += (int)(before - j.lanes.start.size());
                if (st == 0) j.state = 1;
                else if (st < 0) reject(j, "lane chain check");
            }
        }
        const double t3 = now_ms();
        // ---- offsets, output images, expand, resolve, unfilter ----
        std::vector<int64_t>& hob = ht.obase;
        std::vector<int>& hpages = ht.pages;
        hob.clear();
        hpages.clear();
        hl.clear();
        size_t npg = 0;                        // page-table entries so far
        std::vector<std::pair<int, size_t>> pj;  // (job, its first entry in hob) of every verified job
        for (int k = 0; k < m && !rc; ++k) {
            PngJob& j = *J[k];
            if (j.state != 1) continue;
            std::vector<int64_t> ob;
            uint64_t tot = 0;
            pngplan::offsets(j.lanes, ob, &tot);
            if (tot != j.raw_total) { reject(j, "image data length"); continue; }  // png's error
            if (alloc_image(j.w, j.h, (uint32_t)j.bpp, &j.img)) { reject(j, "image allocation"); continue; }
            hd[k].obase = d_obase + hob.size();
            hd[k].page_lane = d_pages + npg;  // (the page table itself is built while expand runs)
            hd[k].nlanes = (int)ob.size();
            pj.emplace_back(k, hob.size());
            npg += (j.raw_total >> kPngPageShift) + 1;
            hd[k].dst = j.img->d;
            hd[k].pitch = j.img->pitch;
            for (size_t i = 0; i < ob.size(); ++i) t_png_timing[12] += (double)j.lanes.res[i].ntok;
            for (size_t i = 0; i < ob.size(); ++i) {
                PngLaneDev L{};
                L.tbase = j.lanes.tbase[i];
                L.obase = ob[i];
                L.out_len = j.lanes.res[i].out_len;
                L.ntok = j.lanes.res[i].ntok;
                L.img = (uint32_t)k;
                L.first = i == 0;
                hl.push_back(L);
            }
            hob.insert(hob.end(), ob.begin(), ob.end());
        }
        mk[1] = now_ms();  // offsets, images, page tables, lane table built
        std::vector<int2>& hrows = ht.rows;
        std::vector<int>& hxst = ht.xst;
        hrows.clear();
        hxst.clear();
        std::vector<int> herr(m, 0);
        if (!rc && !hl.empty()) {
            // expand goes out first; the resolve pass's page and row tables are built
            // on the host while it runs (stream order puts their uploads after it)
            const size_t lb = sizeof(PngLaneDev) * hl.size();
            hipError_t ue = X.h2d(d_lanes, hl.data(), lb);
            if (ue == hipSuccess) ue = X.h2d(d_obase, hob.data(), sizeof(int64_t) * hob.size());
            if (ue == hipSuccess) ue = X.h2d(dev + o_imgs, hd.data(), sizeof(PngImgDev) * m);
            if (ue == hipSuccess) ue = hipMemsetAsync(dev + o_err, 0, sizeof(int) * m, s);
            if (ue != hipSuccess) rc = hip_fail(ue, "PNG expand tables");
            hxst.resize(2 * hl.size());
            mk[2] = now_ms();  // lane tables uploaded
            if (!rc) {
                hipError_t e = hipSuccess;
                rec(4, s);
                if (e == hipSuccess) e = launch_png_expand(d_imgs, d_lanes, (int)hl.size(), d_tok, d_xst, s);
                rec(5, s);
                // page -> decoder that holds the page's first byte (resolve's lane lookup)
                for (const auto& q : pj) {
                    const PngJob& j = *J[q.first];
                    const int64_t* ob = hob.data() + q.second;
                    const size_t nl = (size_t)hd[q.first].nlanes;
                    for (uint64_t pg = 0, ln = 0; pg <= (j.raw_total >> kPngPageShift); ++pg) {
                        while (ln + 1 < nl && (uint64_t)ob[ln + 1] <= (pg << kPngPageShift)) ++ln;
                        hpages.push_back((int)ln);
                    }
                    for (uint32_t y = 0; y < j.h; ++y) hrows.push_back(make_int2(q.first, (int)y));
                }
                if (e == hipSuccess) e = X.h2d(d_pages, hpages.data(), sizeof(int) * hpages.size());
                if (e == hipSuccess) e = X.h2d(d_rows, hrows.data(), sizeof(int2) * hrows.size());
                if (e == hipSuccess) e = launch_png_resolve(d_imgs, d_rows, (int)hrows.size(),
                                                            reinterpret_cast<int*>(dev + o_err), s);
                rec(6, s);
                // unfilter: one launch per bytes-per-pixel class, over that class's
                // images; a workgroup per 16 bands, its (image, group) by ticket
                if (e == hipSuccess) {
                    std::vector<PngImgDev> cls;
                    std::vector<int2> groups;
                    std::vector<int> pbase;
                    struct Range { int bpp, img0, grp0; };
                    std::vector<Range> ranges;
                    int band0 = 0;
                    for (int bpp : {1, 2, 3, 4, 6, 8}) {
                        const Range r{bpp, (int)cls.size(), (int)groups.size()};
                        for (int k = 0; k < m; ++k)
                            if (J[k]->state == 1 && hd[k].bpp == bpp) {
                                for (int g = 0; g < png_unfilter_groups(hd[k].H); ++g)
                                    groups.push_back(make_int2((int)cls.size() - r.img0, g));
                                pbase.push_back(band0);
                                band0 += (hd[k].H + 63) / 64;
                                cls.push_back(hd[k]);
                            }
                        if ((int)cls.size() > r.img0) ranges.push_back(r);
                    }
                    const size_t gb = up256(sizeof(int2) * ngroups);
                    std::vector<uint8_t> tabs(unf_tab, 0);
                    std::memcpy(tabs.data(), groups.data(), sizeof(int2) * groups.size());
                    std::memcpy(tabs.data() + gb, pbase.data(), sizeof(int) * pbase.size());
                    e = X.h2d(d_unf, tabs.data(), unf_tab);
                    unsigned* d_prog = reinterpret_cast<unsigned*>(d_unf + unf_tab);
                    unsigned* d_ticket = d_prog + nbands;
                    if (e == hipSuccess) e = hipMemsetAsync(d_prog, 0, unf_zero, s);
                    if (e == hipSuccess) e = X.h2d(d_cls, cls.data(), sizeof(PngImgDev) * cls.size());
                    const int2* d_groups = reinterpret_cast<const int2*>(d_unf);
                    const int* d_pbase = reinterpret_cast<const int*>(d_unf + gb);
                    for (size_t r = 0; r < ranges.size() && e == hipSuccess; ++r) {
                        const int g1 = r + 1 < ranges.size() ? ranges[r + 1].grp0 : (int)groups.size();
                        const int g0 = ranges[r].grp0, i0 = ranges[r].img0;
                        e = launch_png_unfilter(d_cls + i0, d_groups + g0, g1 - g0, d_pbase + i0, d_prog,
                                                d_ticket + r, ranges[r].bpp, s);
                    }
                }
                rec(7, s);
                if (e == hipSuccess) e = X.d2h(hxst.data(), d_xst, 2 * sizeof(int) * hl.size());
                if (e == hipSuccess) e = X.d2h(herr.data(), dev + o_err, sizeof(int) * m);
                mk[3] = now_ms();  // expand .. unfilter done
                if (e != hipSuccess) rc = hip_fail(e, "PNG inflate (expand) / unfilter");
                if (!rc) {
                    t_png_timing[3] = ev_ms(4, 5);
                    t_png_timing[4] = ev_ms(5, 6);
                    t_png_timing[5] = ev_ms(6, 7);
                }
            }
            if (!rc) {
                size_t t = 0;
                for (int k = 0; k < m; ++k) {
                    PngJob& j = *J[k];
                    if (j.state != 1) continue;
                    const bool rows_ok = herr[k] == 0;
                    bool lanes_ok = true;
                    for (size_t i = 0; i < j.lanes.start.size(); ++i, ++t) lanes_ok = lanes_ok && hxst[2 * t] == 0;
                    if (!rows_ok || !lanes_ok) reject(j, !lanes_ok ? "expand status" : "row filter bytes");
                }
            }
        }
        gate_leave(kGateUpload);   // (error paths)
        gate_leave(kGateKernels);  // unless the caller pinned it (transform_part: resize + encode next)
        if (timing && !hl.empty()) {  // per-lane profile of the last decode round and the expand pass
            double si = 0, sc = 0, sx = 0, mi = 0, mc = 0, mx = 0, sb = 0, mb = 0;
            for (size_t t = 0; t < hres.size(); ++t) {
                si += hres[t].iters; sc += hres[t].kcycles; sb += hres[t].blocks;
                mi = std::max(mi, (double)hres[t].iters); mc = std::max(mc, (double)hres[t].kcycles);
                mb = std::max(mb, (double)hres[t].blocks);
            }
            for (size_t t = 0; 2 * t + 1 < hxst.size(); ++t) {
                sx += hxst[2 * t + 1];
                mx = std::max(mx, (double)hxst[2 * t + 1]);
            }
            const double n1 = (double)std::max<size_t>(1, hres.size()), n2 = (double)std::max<size_t>(1, hxst.size() / 2);
            fprintf(stderr, "[png] decode lanes %zu: iters mean %.0f max %.0f, blocks mean %.2f max %.0f, kcycles mean %.0f "
                    "max %.0f (%.0f cycles/iter); expand kcycles mean %.0f max %.0f\n", hres.size(), si / n1, mi, sb / n1,
                    mb, sc / n1, mc, 1024.0 * sc / std::max(1.0, si), sx / n2, mx);
        }
        t_png_timing[0] = t1 - t0;
        t_png_timing[1] = ev_ms(0, 1);
        t_png_timing[2] = count_dev;
        t_png_timing[7] = rounds;
        t_png_timing[8] = (double)hl.size();
        t_png_timing[9] = m;
        if (timing)
            fprintf(stderr, "[png] t=%.1f %d streams (%d on the GPU): stage %.2f ms, find %.2f ms (kernel gate at +%.2f), "
                    "decode %.2f ms (%d rounds, %d dropped, %d overflows), expand+resolve+unfilter %.2f ms; staging "
                    "loop %.2f ms (early %d), in hipMemcpyAsync %.2f ms summed\n",
                    fmod(t0, 1e5), n, m, t1 - t0, t2 - t1, t_gate - t0, t3 - t2, rounds, dropped, overflows, now_ms() - t3,
                    t_stage1 - t_stage0, (int)early, 1e-3 * (double)t_copy_calls.load());
        if (timing)
            fprintf(stderr, "[png] host: plan+lanes %.2f, (decode rounds) .. tables %.2f, rows+uploads %.2f, "
                    "(expand..unfilter) %.2f, after %.2f ms\n", mk[0] - t2, mk[1] - t3, mk[2] - mk[1], mk[3] - mk[2],
                    now_ms() - mk[3]);
        for (int k = 0; k < m; ++k) {
            PngJob& j = *J[k];
            if (!rc && j.state == 1) {
                outs[j.idx] = j.img;
                j.img = nullptr;
            } else {
                if (j.img) { ik_image_free(j.img); j.img = nullptr; }
                gpu[j.idx] = 0;  // host decoder below
            }
        }
        if (rc) {  // the device path failed as a whole: every stream on the host
            for (int k = 0; k < m; ++k) gpu[J[k]->idx] = 0;
        }
    }
    // ---- host decoder: streams outside the GPU path, and GPU rejects ----
    std::vector<int> host;
    for (int i = 0; i < n; ++i)
        if (!gpu[i]) host.push_back(i);
    t_png_timing[11] = (double)host.size();
    t_png_timing[10] = (double)(n - (int)host.size());
    g_png_gpu_streams += (unsigned long long)(n - (int)host.size());
    g_png_host_streams += (unsigned long long)host.size();
    parallel_for((int)host.size(), 0, [&](int k) {
        const int i = host[k];
        thread_local std::vector<uint8_t> px;
        uint32_t w = 0, h = 0, c = 0, dep = 1;
        int st = decode_png(bytes[i], lens[i], w, h, c, px, &dep);
        if (!st) st = dep == 2 ? ik_image_from_host16(reinterpret_cast<const uint16_t*>(px.data()), w, h, c, &outs[i])
                               : ik_image_from_host(px.data(), w, h, c, &outs[i]);
        if (px.capacity() > (128u << 20)) std::vector<uint8_t>().swap(px);
        status[i] = st;
        if (st && msgs) {
            char buf[512];
            ik_last_error(buf, sizeof(buf));
            msgs[i] = buf;
        }
    });
    t_png_timing[6] = now_ms() - t0;
    if (timing) fprintf(stderr, "[png] decode_png_batch returns at t=%.1f\n", fmod(now_ms(), 1e5));
    int first = IK_OK;
    for (int i = 0; i < n; ++i)
        if (status[i] && !first) first = status[i];
    return first;
}

}  // namespace ik

extern "C" int ik_png_counters(unsigned long long* out) {
    out[0] = ik::g_png_gpu_streams.load();
    out[1] = ik::g_png_host_streams.load();
    return IK_OK;
}

extern "C" int ik_png_last_timing(double* out, int n) {
    for (int i = 0; i < n && i < 13; ++i) out[i] = ik::t_png_timing[i];
    return IK_OK;
}

extern "C" int ik_set_png_gpu_min(long long min_raw_bytes) {
    (void)ik::png_gpu_min();
    ik::g_png_gpu_min.store(min_raw_bytes < 0 ? -1 : min_raw_bytes);
    return IK_OK;
}
