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
// The GPU path covers non-interlaced 8-bit streams of every colour type, palette
// and gray streams of 1/2/4 bits, and tRNS (png's EXPAND: k_png_px); 16-bit and
// interlaced streams, and any stream the GPU finds inconsistent, go through the
// host decoder, whose error messages are png's.  The zlib Adler-32 is not verified, as png 0.18 does
// not by default (CRCs cover the data).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
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
#include "ik_png_wave.h"
#include "ik_runtime.h"

namespace ik {

namespace {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
size_t up256(size_t v) { return (v + 255) & ~size_t(255); }

struct PngJob {
    int idx = -1;                                   // stream index in the batch
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, bpp = 0, ch = 0;       // bytes per pixel, image channels
    std::vector<std::pair<uint64_t, uint32_t>> idat;  // non-empty IDAT payloads: (file offset, length)
    size_t zlen = 0;                                 // IDAT payload bytes (zlib stream)
    uint64_t raw_total = 0;
    int rowbytes = 0;
    // layout: the file in the upload area's raw part, its zlib stream in the
    // stream part, its staging copy (inputs the caller did not pin); the kernel
    // stage's u16 symbols and filter types
    size_t raw_off = 0, z_off = 0, stage_off = 0;
    size_t o_u16 = 0, o_ft = 0;
    uint64_t nbits = 0;
    int chunk0 = 0, nchunks = 0;                     // its chunks in the batch chunk table
    pngplan::Lanes lanes;
    int state = 0;                                   // 0 running, 1 verified, -1 host fallback
    ik_image* img = nullptr;
    // png's EXPAND (palette -> RGB(A), gray below 8 bits -> 8 bits, tRNS -> alpha):
    // the unfiltered rows land in `rows` (rowbytes wide) and k_png_px writes the
    // expanded pixels (out_c channels) into img
    bool expand = false;
    int out_c = 0;
    PngPxDev px{};
    ik_image* rows = nullptr;
};

// One chunk as parse_chunks sees it: its type, its data where the host can read
// it (null for an IDAT payload of a device-resident file), the file offset of its
// length field, whether its stored CRC matches (IDAT payload CRCs are checked on
// the GPU by the gather pass instead), and its first data bytes.
struct ChunkRef {
    const uint8_t* type;
    const uint8_t* data;
    uint32_t len;
    uint64_t off;
    bool crc_ok;
    const uint8_t* head;
};

// the chunks of a PNG file in host memory, as png walks them: while 12 bytes
// remain, stop after IEND; false on a length past the end of the file
bool host_chunks(const uint8_t* b, size_t n, std::vector<ChunkRef>& out) {
    out.clear();
    if (n < 8 || std::memcmp(b, "\x89PNG\r\n\x1a\n", 8)) return false;
    size_t pos = 8;
    while (pos + 12 <= n) {
        const uint32_t len = be32(b + pos);
        if (len > n - pos - 12) return false;
        const uint8_t* type = b + pos + 4;
        const uint8_t* data = b + pos + 8;
        const bool idat = !std::memcmp(type, "IDAT", 4) && len;
        out.push_back(ChunkRef{type, data, len, pos, idat || png_chunk_crc(type, data, len) == be32(data + len), data});
        pos += 12 + len;
        if (!std::memcmp(type, "IEND", 4)) break;
    }
    return true;
}

// the chunks of a device-resident file from its walk (k_png_walk): non-IDAT chunk
// contents from the side area (type + data + CRC)
bool walk_chunks(const PngWalkRec* R, int nrec, const uint8_t* side, std::vector<ChunkRef>& out) {
    out.clear();
    if (nrec < 0) return false;
    for (int k = 0; k < nrec; ++k) {
        const PngWalkRec& r = R[k];
        if (r.side != ~0u) {
            const uint8_t* t = side + r.side;
            out.push_back(ChunkRef{t, t + 4, r.len, r.off, png_chunk_crc(t, t + 4, r.len) == be32(t + 4 + r.len), t + 4});
        } else {
            out.push_back(ChunkRef{r.type, nullptr, r.len, r.off, true, r.head});
        }
    }
    return true;
}

// png 0.18 + image's EXPAND: which streams the GPU path decodes.  Returns false
// for streams that must go to the host decoder (which also produces png's
// errors for malformed ones).
bool parse_chunks(const std::vector<ChunkRef>& C, PngJob& J) {
    bool ihdr = false, trns = false;
    int interlace = 0;
    std::vector<uint8_t> plte;
    const uint8_t* trns_data = nullptr;
    size_t trns_len = 0;
    const uint8_t* zh[2] = {nullptr, nullptr};  // first payload bytes of the first two IDATs
    uint32_t zl0 = 0;
    for (const ChunkRef& c : C) {
        const uint8_t* type = c.type;
        const uint8_t* data = c.data;
        const uint32_t len = c.len;
        if (!c.crc_ok) return false;
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13 || ihdr || !data) return false;
            J.w = be32(data);
            J.h = be32(data + 4);
            J.depth = data[8];
            J.ctype = data[9];
            interlace = data[12];
            ihdr = true;
        } else if (!std::memcmp(type, "tRNS", 4)) {
            if (!data && len) return false;
            trns = true;
            trns_data = data;
            trns_len = len;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (!data && len) return false;
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (len) {
                if (J.idat.empty()) { zh[0] = c.head; zl0 = len; }
                else if (J.idat.size() == 1) zh[1] = c.head;
                J.idat.emplace_back(c.off + 8, len);
            }
            J.zlen += len;
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
    }
    if (!ihdr || J.idat.empty() || !J.w || !J.h || interlace) return false;
    // 8-bit L / LA / RGB / RGBA as they are; palette (1/2/4/8 bits), gray below 8
    // bits and tRNS through png's EXPAND on the GPU (k_png_px); 16-bit: host
    int spp;
    switch (J.ctype) {
    case 0: spp = 1; break;
    case 2: spp = 3; break;
    case 3: spp = 1; break;
    case 4: spp = 2; break;
    case 6: spp = 4; break;
    default: return false;
    }
    const bool low = J.depth == 1 || J.depth == 2 || J.depth == 4;
    const bool d16 = J.depth == 16;
    if (!(J.depth == 8 || (d16 && J.ctype != 3) || (low && (J.ctype == 0 || J.ctype == 3)))) return false;
    if (trns && J.ctype != 0 && J.ctype != 2 && J.ctype != 3) return false;  // (png rejects those)
    J.ch = spp;
    const uint64_t bits_pp = (uint64_t)spp * J.depth;
    J.bpp = (int)((bits_pp + 7) / 8);
    const uint64_t rb = ((uint64_t)J.w * bits_pp + 7) / 8;
    // (16-bit: the big-endian samples become native u16 in k_png_px, with tRNS alpha 0 / 65535)
    J.expand = J.ctype == 3 || low || trns || d16;
    J.out_c = spp;
    if (J.expand) {
        PngPxDev& X = J.px;
        X.w = (int)J.w;
        X.h = (int)J.h;
        X.depth = J.depth;
        X.ctype = J.ctype;
        X.key = -1;
        if (J.ctype == 3) {
            if (plte.empty() || plte.size() % 3 || plte.size() > 768) return false;
            J.out_c = trns_len ? 4 : 3;
            const size_t np = plte.size() / 3;
            for (size_t i = 0; i < 256; ++i) {
                const uint32_t r = i < np ? plte[3 * i] : 0, g = i < np ? plte[3 * i + 1] : 0, bl = i < np ? plte[3 * i + 2] : 0;
                const uint32_t a = i < trns_len ? trns_data[i] : 255u;
                X.pal[i] = r | g << 8 | bl << 16 | a << 24;
            }
        } else if (J.ctype == 0) {
            J.out_c = trns_len >= 2 ? 2 : 1;
            if (trns_len >= 2) X.key = (int)((trns_data[0] << 8) | trns_data[1]);
            X.scale = J.depth == 1 ? 255 : J.depth == 2 ? 85 : J.depth == 4 ? 17 : 1;
        } else if (J.ctype == 2) {  // RGB + tRNS
            if (trns_len < 6) { J.expand = d16; }
            else {
                J.out_c = 4;
                X.key_rgb[0] = (trns_data[0] << 8) | trns_data[1];
                X.key_rgb[1] = (trns_data[2] << 8) | trns_data[3];
                X.key_rgb[2] = (trns_data[4] << 8) | trns_data[5];
                X.key = 0;
            }
        }
        X.out_c = J.out_c;
    }
    // image's default limit: 512 MiB of decoded (expanded) pixel bytes
    if ((uint64_t)J.w * J.h * J.out_c * (d16 ? 2 : 1) > (512ull << 20) || rb > 0x7FFFFFF0ull) return false;
    J.rowbytes = (int)rb;
    J.raw_total = (rb + 1) * J.h;
    // zlib header: CM 8, window <= 32 KiB, FCHECK, no preset dictionary
    uint8_t cmf, flg;
    if (zl0 >= 2) { cmf = zh[0][0]; flg = zh[0][1]; }
    else if (J.idat.size() > 1) { cmf = zh[0][0]; flg = zh[1][0]; }
    else return false;
    if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 || (flg & 0x20)) return false;
    return true;
}

struct HostTables {
    std::vector<int> chunk_img, chunk_idx, pages, xst;
    std::vector<int64_t> cand, obase;
    std::vector<PngLaneDev> lanes;
    std::vector<std::pair<int, int>> who;
    std::vector<uint32_t> order;
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
        if (o == ~size_t(0) && getenv("IK_TIMING"))
            fprintf(stderr, "[png] transfer area full: a %zu-byte copy takes the copy engine\n", n);
        if (o == ~size_t(0))  // (more decode rounds than the area was sized for) the copy engine
            return copy_h2d_2d(reinterpret_cast<uint8_t*>(dev), n, reinterpret_cast<const uint8_t*>(host), n, n, 1, s)
                       ? hipErrorUnknown : hipSuccess;
        std::memcpy(pin + o, host, n);
        return launch_copy_words(reinterpret_cast<const uint32_t*>(dpin + o), reinterpret_cast<uint32_t*>(dev),
                                 (n + 3) / 4, s);
    }
    // d2h in two halves: start queues the copy kernel (its data lands in the pinned
    // region returned in *off), finish waits for the event recorded after it and
    // copies out -- so work queued between the two (the next batch's block search)
    // runs while the host waits for nothing but the copy
    hipError_t d2h_start(const void* dev, size_t n, size_t* off, hipEvent_t ev) {
        const size_t o = take(n + 4);
        if (o == ~size_t(0) || (n & 3) || !ev) { *off = ~size_t(0); return hipSuccess; }
        hipError_t e = launch_copy_words(reinterpret_cast<const uint32_t*>(dev), reinterpret_cast<uint32_t*>(dpin + o),
                                         n / 4, s);
        if (e == hipSuccess) e = hipEventRecord(ev, s);
        *off = o;
        return e;
    }
    hipError_t d2h_finish(void* host, const void* dev, size_t n, size_t off, hipEvent_t ev) {
        if (off == ~size_t(0)) return d2h(host, dev, n);  // (no room / odd size: the synchronous path)
        hipError_t e = hipEventSynchronize(ev);
        if (e == hipSuccess) std::memcpy(host, pin + off, n);
        return e;
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
        if (o == ~size_t(0) && getenv("IK_TIMING"))
            fprintf(stderr, "[png] transfer area full: a %zu-byte copy takes the copy engine\n", n);
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

// the last batch's stage times (ik_png_last_timing, per device): see the header
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

#ifdef IK_PNG_DUMP
namespace {
std::mutex g_dump_mu;
std::vector<std::vector<uint8_t>> g_dump;  // per image of the last batch: H rows of rowbytes, then H filter types
}  // namespace
template <typename JV, typename HV>
static void png_dump_store(const JV& J, const HV& hd, int m) {
    std::lock_guard<std::mutex> lk(g_dump_mu);
    g_dump.assign(m, std::vector<uint8_t>());
    for (int k = 0; k < m; ++k) {
        if (J[k]->state != 1 || J[k]->idx < 0 || J[k]->idx >= m) continue;
        const auto& I = hd[k];
        std::vector<uint8_t>& o = g_dump[J[k]->idx];
        o.resize((size_t)I.H * I.rowbytes + I.H);
        (void)hipMemcpy2D(o.data(), I.rowbytes, I.dst, I.pitch, I.rowbytes, I.H, hipMemcpyDeviceToHost);
        (void)hipMemcpy(o.data() + (size_t)I.H * I.rowbytes, I.ft, I.H, hipMemcpyDeviceToHost);
    }
}
#endif

bool png_gpu_enabled(size_t raw_bytes) {
    const long long v = png_gpu_min();
    return v >= 0 && (long long)raw_bytes >= v;
}

// ---- upload areas ----------------------------------------------------------------
// A batch's upload stage fills an area of device memory -- the PNG files exactly
// as the caller holds them (raw), the zlib streams assembled from their IDAT
// payloads (+ zero padding), the gather plan, per-piece CRCs and per-stream CRC
// flags -- that its kernel stage reads until its decode rounds end.  Two areas
// per device: the next batch's upload (PCIe + the gather pass) runs while the
// current batch's kernels read the other one.
namespace {
struct UploadArea {
    int device = 0;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    uint8_t* pin = nullptr;  // pinned: the plan tables, and staging for inputs the caller did not pin
    size_t pin_cap = 0;
    // upload issued, file DMAs done, gather + CRC done, block search done, block
    // search started (the block search waits on [2], the kernel stage on [3])
    hipEvent_t ev[5] = {};
    bool busy = false;
};
constexpr int kUploadAreas = 2;
struct AreaPool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<UploadArea*> areas;
};
std::mutex g_area_mu;
std::map<int, AreaPool*> g_area_pools;
AreaPool& area_pool(int device) {
    std::lock_guard<std::mutex> lk(g_area_mu);
    AreaPool*& p = g_area_pools[device];
    if (!p) p = new AreaPool();
    return *p;
}
UploadArea* acquire_area(int device) {
    AreaPool& P = area_pool(device);
    std::unique_lock<std::mutex> lk(P.mu);
    for (;;) {
        for (UploadArea* a : P.areas)
            if (!a->busy) { a->busy = true; return a; }
        if ((int)P.areas.size() < kUploadAreas) {
            auto* a = new UploadArea();
            a->device = device;
            for (hipEvent_t& e : a->ev)
                if (hipEventCreate(&e) != hipSuccess) e = nullptr;
            a->busy = true;
            P.areas.push_back(a);
            return a;
        }
        P.cv.wait(lk);
    }
}
void release_area(UploadArea*& a) {
    if (!a) return;
    AreaPool& P = area_pool(a->device);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        a->busy = false;
    }
    P.cv.notify_all();
    a = nullptr;
}
// grow an idle area (nothing pending reads it: it was released after its batch's
// decode rounds synchronised)
bool area_reserve(UploadArea* a, size_t dev_bytes, size_t pin_bytes) {
    if (dev_bytes > a->cap) {
        if (a->dev) { (void)hipFree(a->dev); mem_stat(kMemUploadDev, -(int64_t)a->cap); }
        a->dev = nullptr;
        a->cap = 0;
        const size_t want = dev_bytes + dev_bytes / 8;
        if (hipMalloc((void**)&a->dev, want) != hipSuccess) { a->dev = nullptr; return false; }
        a->cap = want;
        mem_stat(kMemUploadDev, (int64_t)want);
    }
    if (pin_bytes > a->pin_cap) {
        if (a->pin) { (void)hipHostFree(a->pin); mem_stat(kMemUploadPinned, -(int64_t)a->pin_cap); }
        a->pin = nullptr;
        a->pin_cap = 0;
        const size_t want = std::max<size_t>(pin_bytes + pin_bytes / 8, 1u << 20);
        if (hipHostMalloc((void**)&a->pin, want, hipHostMallocDefault) != hipSuccess) { a->pin = nullptr; return false; }
        a->pin_cap = want;
        mem_stat(kMemUploadPinned, (int64_t)want);
    }
    return true;
}

}  // namespace

// ik_shutdown: the upload areas' device and pinned buffers and events (no batch is
// in flight: the stage threads have ended)
void png_shutdown() {
    std::vector<AreaPool*> ps;
    {
        std::lock_guard<std::mutex> lk(g_area_mu);
        for (auto& kv : g_area_pools) ps.push_back(kv.second);
    }
    for (AreaPool* P : ps) {
        std::lock_guard<std::mutex> lk(P->mu);
        for (UploadArea* a : P->areas) {
            (void)hipSetDevice(a->device);
            if (a->dev) { (void)hipFree(a->dev); mem_stat(kMemUploadDev, -(int64_t)a->cap); }
            if (a->pin) { (void)hipHostFree(a->pin); mem_stat(kMemUploadPinned, -(int64_t)a->pin_cap); }
            for (hipEvent_t e : a->ev)
                if (e) (void)hipEventDestroy(e);
            delete a;
        }
        P->areas.clear();
    }
}

namespace {
// the last batch's stage times per device (ik_png_last_timing)
std::mutex g_timing_mu;
std::map<int, std::vector<double>> g_timing;
}  // namespace

// the upload stage's hand-off to the kernel stage
struct PngBatchState {
    int device = 0;
    int n = 0;
    std::vector<PngJob> jobs;
    std::vector<char> gpu;
    std::vector<PngJob*> J;
    UploadArea* area = nullptr;
    int rc = IK_OK;
    size_t o_zs = 0, o_err = 0;  // area offsets: assembled streams, per-stream CRC flags
    size_t o_ftab = 0, o_fimg = 0, o_cand = 0;  // the block search's chunk table, stream descriptors, candidates
    int nchunks = 0;
    bool find_launched = false;
    int pinned_streams = 0;
    bool dev = false;  // the files are the caller's device copies (PngUpload::dev)
    double t0 = 0, t_host = 0;
    ~PngBatchState() { release_area(area); }
};

// The decode pass: the wave decoder (ik_png_wave.h, k_png_wave: a wave per lane,
// 64 self-synchronising sub-lanes over shared lookup tables) by default;
// IK_PNG_DECODE=lane selects round 4's one-thread-per-lane canonical decoder
// (k_png_decode, token streams with literal tables) for A/B runs.
// The direct-rows expand (IK_PNG_DIRECT=1: expand writes the rows and filter types
// itself and lists the window markers for k_png_marks, so no pass reads the u16
// symbols back whole).  Measured slower on the bench frames and not the default:
// their 164 M markers per 64 frames (3.8 % of the bytes, near every unit start) cost
// expand 3.9 ms of list writes and byte stores and k_png_marks 3.1 ms, against the
// resolve pass's 4.3 ms (profiles/r05_ab_notes.md).
static bool png_direct_rows() {
    static const bool v = getenv("IK_PNG_DIRECT") != nullptr;
    return v;
}

bool png_find_beside_decode() {
    static const bool v = getenv("IK_FIND_BESIDE") != nullptr;
    return v;
}

static bool png_wave_decoder() {
    static const bool v = [] {
        const char* e = getenv("IK_PNG_DECODE");
        return !(e && !strcmp(e, "lane"));
    }();
    return v;
}

// The search chunk: one decoder lane starts at (about) each chunk's first block.
// The wave decoder's lanes run 64 sub-lanes over each block, so a lane can span
// several blocks: 64 KiB chunks (~7 blocks of image data) take a quarter of the
// block searches of 16 KiB and a quarter of the lane starts (window markers, chain
// links) at the same decode parallelism; the one-thread lane decoder keeps 16 KiB.
// IK_PNG_CHUNK_KB overrides (A/B runs).
static uint64_t png_chunk_bytes() {
    static const uint64_t v = [] {
        const char* e = getenv("IK_PNG_CHUNK_KB");
        const long kb = e ? atol(e) : 0;
        if (kb >= 4 && kb <= 4096) return (uint64_t)kb << 10;
        return png_wave_decoder() ? (uint64_t)kPngWaveChunkBytes : kPngChunkBytes;
    }();
    return v;
}

int png_upload_begin(const uint8_t* const* bytes, const size_t* lens, int n, PngUpload& up) {
    static const bool timing = getenv("IK_TIMING") != nullptr;
    auto st = std::make_shared<PngBatchState>();
    up.st = st;
    up.bytes = bytes;
    up.lens = lens;
    up.n = n;
    PngBatchState& S = *st;
    S.device = current_device();
    S.n = n;
    S.t0 = now_ms();
    S.jobs.assign(n, PngJob());
    S.gpu.assign(n, 0);
    S.dev = up.dev;
    hipStream_t sc = thread_copy_stream();
    if (!sc) { S.rc = fail(IK_ERR_DEVICE, "cannot create the PNG copy stream"); return IK_OK; }
    if (up.dev) {
        // the files are in device memory: the GPU walks their chunks into pinned
        // memory (records + the small chunks' contents), the host plans from that
        const size_t o_rec = 0, o_side = up256(sizeof(PngWalkRec) * kPngWalkRecs * (size_t)n);
        const size_t o_n = o_side + up256((size_t)kPngWalkSide * n);
        const size_t o_files = o_n + up256(sizeof(int) * n);
        const size_t wbytes = o_files + 2 * sizeof(uint64_t) * n;
        uint8_t* wp = pinned_slot(6, wbytes);
        void* wd = nullptr;
        if (!wp || hipHostGetDevicePointer(&wd, wp, 0) != hipSuccess || !wd) {
            S.rc = fail(IK_ERR_NOMEM, "cannot allocate the PNG chunk-walk area");
            return IK_OK;
        }
        uint8_t* wdev = reinterpret_cast<uint8_t*>(wd);
        uint64_t* files = reinterpret_cast<uint64_t*>(wp + o_files);
        for (int i = 0; i < n; ++i) {
            files[i] = (uint64_t)(uintptr_t)bytes[i];
            files[n + i] = lens[i];
        }
        int* cnt = reinterpret_cast<int*>(wp + o_n);
        hipError_t e = launch_png_walk(reinterpret_cast<const uint64_t*>(wdev + o_files),
                                       reinterpret_cast<const uint64_t*>(wdev + o_files) + n, n,
                                       reinterpret_cast<PngWalkRec*>(wdev + o_rec), wdev + o_side,
                                       reinterpret_cast<int*>(wdev + o_n), sc);
        if (e == hipSuccess) e = hipStreamSynchronize(sc);
        if (e != hipSuccess) { S.rc = hip_fail(e, "PNG chunk walk"); return IK_OK; }
        const PngWalkRec* recs = reinterpret_cast<const PngWalkRec*>(wp + o_rec);
        const uint8_t* side = wp + o_side;
        parallel_for(n, 0, [&](int i) {
            S.jobs[i].idx = i;
            thread_local std::vector<ChunkRef> cr;
            // (a file shorter than the signature, or without it, goes to the host decoder)
            S.gpu[i] = lens[i] >= 8 && up.heads && !std::memcmp(up.heads[i], "\x89PNG\r\n\x1a\n", 8) &&
                       walk_chunks(recs + (size_t)i * kPngWalkRecs, cnt[i], side + (size_t)i * kPngWalkSide, cr) &&
                       parse_chunks(cr, S.jobs[i]) && png_gpu_enabled(S.jobs[i].raw_total);
        });
    } else {
        parallel_for(n, 0, [&](int i) {
            S.jobs[i].idx = i;
            thread_local std::vector<ChunkRef> cr;
            S.gpu[i] = host_chunks(bytes[i], lens[i], cr) && parse_chunks(cr, S.jobs[i]) &&
                       png_gpu_enabled(S.jobs[i].raw_total);
        });
    }
    for (int i = 0; i < n; ++i)
        if (S.gpu[i]) S.J.push_back(&S.jobs[i]);
    const int m = (int)S.J.size();
    if (!m) return IK_OK;
    constexpr size_t kPad = 512;  // zero bytes past each stream (Bits::wend, the LDS ring's DMAs)
    // ---- layout of the area: [raw files][streams][pieces][chunks][piece CRCs][flags] ----
    size_t raw = 0, zs = 0, stage = 0;
    std::vector<PngGatherPiece> pieces;
    std::vector<PngCrcChunk> chunks;
    std::vector<char> pinned(m, 0);
    for (int k = 0; k < m; ++k) {
        PngJob& j = *S.J[k];
        j.z_off = zs;
        zs += up256(((j.zlen + 3) & ~size_t(3)) + kPad);
        if (S.dev) {  // the gather pass reads the caller's device copy (raw base 0)
            j.raw_off = (uint64_t)(uintptr_t)bytes[j.idx];
            continue;
        }
        j.raw_off = raw;
        raw += up256(lens[j.idx] + 4);  // (+4: the gather pass reads whole words)
        pinned[k] = host_pinned(bytes[j.idx], lens[j.idx]);
        if (!pinned[k]) {
            j.stage_off = stage;
            stage += up256(lens[j.idx]);
        }
        S.pinned_streams += pinned[k];
    }
    for (int k = 0; k < m; ++k) {
        const PngJob& j = *S.J[k];
        const uint32_t tail = (uint32_t)((((j.zlen + 3) & ~size_t(3)) + kPad) - j.zlen);
        png_gather_plan(j.raw_off, j.idat, raw + j.z_off, tail, (uint32_t)k, pieces, chunks);
    }
    // the block search's chunks (chunk 0 starts at the first block): png_chunk_bytes() of stream each
    const uint64_t cbits = png_chunk_bytes() * 8;
    int nchunks = 0;
    for (PngJob* j : S.J) {
        j->nbits = (uint64_t)j->zlen * 8;
        j->nchunks = (int)((j->nbits - 16 + cbits - 1) / cbits);
        j->chunk0 = nchunks;
        nchunks += j->nchunks;
    }
    S.nchunks = nchunks;
    // (the pieces' dst offsets are area offsets: the stream area follows the raw one)
    S.o_zs = raw;
    const size_t o_pieces = raw + up256(zs);
    const size_t o_chunks = o_pieces + up256(sizeof(PngGatherPiece) * pieces.size());
    S.o_ftab = o_chunks + up256(sizeof(PngCrcChunk) * chunks.size());
    S.o_fimg = S.o_ftab + up256(2 * sizeof(int) * nchunks);
    const size_t o_pcrc = S.o_fimg + up256(sizeof(PngImgDev) * m);
    S.o_err = o_pcrc + up256(2 * sizeof(uint32_t) * pieces.size());
    S.o_cand = S.o_err + up256(sizeof(int) * m);
    const size_t dev_bytes = S.o_cand + up256(sizeof(int64_t) * nchunks);
    const size_t tab_bytes = o_pcrc - o_pieces;  // pieces, chunks, search chunk table, search descriptors
    S.area = acquire_area(S.device);  // waits while two earlier batches' kernel stages hold both areas
    UploadArea* A = S.area;
    if (!area_reserve(A, dev_bytes, tab_bytes + stage)) {
        S.rc = fail(IK_ERR_DEVICE, "cannot allocate the PNG upload area (%zu device bytes)", dev_bytes);
        return IK_OK;  // the kernel stage sends every stream to the host decoder
    }
    // the upload goes out under the device's upload gate: concurrent batches take
    // PCIe in turn (ik_runtime.h)
    gate_enter(kGateUpload);
    std::atomic<int> err{0};
    if (A->ev[0]) (void)hipEventRecord(A->ev[0], sc);
    // files the caller pinned (ik_host_alloc / ik_host_register) go straight from
    // its memory; the others through the area's pinned staging (host memcpy only:
    // the CRCs are the GPU's)
    for (int k = 0; k < m; ++k) {
        if (S.dev || !pinned[k]) continue;
        const PngJob& j = *S.J[k];
        if (hipMemcpyAsync(A->dev + j.raw_off, bytes[j.idx], lens[j.idx], hipMemcpyHostToDevice, sc) != hipSuccess)
            err = 1;
    }
    std::vector<int> staged;
    for (int k = 0; k < m; ++k)
        if (!S.dev && !pinned[k]) staged.push_back(k);
    uint8_t* stg = A->pin + tab_bytes;
    parallel_for((int)staged.size(), 0, [&, sc](int q) {
        const PngJob& j = *S.J[staged[q]];
        std::memcpy(stg + j.stage_off, bytes[j.idx], lens[j.idx]);
        if (hipMemcpyAsync(A->dev + j.raw_off, stg + j.stage_off, lens[j.idx], hipMemcpyHostToDevice, sc) != hipSuccess)
            err = 1;
    });
    if (A->ev[1]) (void)hipEventRecord(A->ev[1], sc);
    std::memcpy(A->pin, pieces.data(), sizeof(PngGatherPiece) * pieces.size());
    std::memcpy(A->pin + (o_chunks - o_pieces), chunks.data(), sizeof(PngCrcChunk) * chunks.size());
    {
        int* ft = reinterpret_cast<int*>(A->pin + (S.o_ftab - o_pieces));
        PngImgDev* fi = reinterpret_cast<PngImgDev*>(A->pin + (S.o_fimg - o_pieces));
        for (int k = 0; k < m; ++k) {
            const PngJob& j = *S.J[k];
            PngImgDev d{};
            d.words = reinterpret_cast<const uint32_t*>(A->dev + S.o_zs + j.z_off);
            d.bit0 = 16;
            d.nbits = j.nbits;
            fi[k] = d;
            for (int c = 0; c < j.nchunks; ++c) {
                ft[j.chunk0 + c] = k;
                ft[nchunks + j.chunk0 + c] = c;
            }
        }
    }
    hipError_t e = hipMemcpyAsync(A->dev + o_pieces, A->pin, tab_bytes, hipMemcpyHostToDevice, sc);
    if (e == hipSuccess) e = hipMemsetAsync(A->dev + S.o_err, 0, sizeof(int) * m, sc);
    if (e == hipSuccess)
        e = launch_png_gather(S.dev ? 0 : (uintptr_t)A->dev, A->dev, reinterpret_cast<const PngGatherPiece*>(A->dev + o_pieces),
                              (int)pieces.size(), reinterpret_cast<uint32_t*>(A->dev + o_pcrc), sc);
    if (e == hipSuccess)
        e = launch_png_crc_check(S.dev ? 0 : (uintptr_t)A->dev, reinterpret_cast<const PngCrcChunk*>(A->dev + o_chunks), (int)chunks.size(),
                                 reinterpret_cast<const uint32_t*>(A->dev + o_pcrc),
                                 reinterpret_cast<int*>(A->dev + S.o_err), sc);
    if (e == hipSuccess && A->ev[2]) e = hipEventRecord(A->ev[2], sc);
    if (e == hipSuccess && !A->ev[2]) e = hipStreamSynchronize(sc);  // (no event: the stage waits here)
    gate_leave(kGateUpload);
    if (e != hipSuccess || err) S.rc = hip_fail(e != hipSuccess ? e : hipErrorUnknown, "PNG upload / gather");
    S.t_host = now_ms() - S.t0;
    if (timing)
        fprintf(stderr, "[png] upload t=%.1f: %d streams (%d pinned), %zu pieces, %zu IDAT chunks, host %.2f ms\n",
                fmod(S.t0, 1e5), m, S.pinned_streams, pieces.size(), chunks.size(), S.t_host);
    return IK_OK;
}

// the block search of a batch whose upload was issued: on stream s, once the
// upload (with its gather + CRC pass) has landed; once per batch
static void png_find_launch(PngBatchState& S, hipStream_t s) {
    if (S.find_launched || S.rc || !S.area || S.J.empty()) return;
    UploadArea* A = S.area;
    const uint64_t cbits = png_chunk_bytes() * 8;
    hipError_t e = A->ev[2] ? hipStreamWaitEvent(s, A->ev[2], 0) : hipSuccess;
    if (e == hipSuccess && A->ev[4]) e = hipEventRecord(A->ev[4], s);
    const int* ft = reinterpret_cast<const int*>(A->dev + S.o_ftab);
    if (e == hipSuccess)
        e = launch_png_find(reinterpret_cast<const PngImgDev*>(A->dev + S.o_fimg), ft, ft + S.nchunks, S.nchunks, cbits,
                            reinterpret_cast<int64_t*>(A->dev + S.o_cand), s);
    if (e == hipSuccess && A->ev[3]) e = hipEventRecord(A->ev[3], s);
    if (e == hipSuccess && !A->ev[3]) e = hipStreamSynchronize(s);
    if (e != hipSuccess) S.rc = hip_fail(e, "PNG block search");
    S.find_launched = true;
}

bool png_upload_landed(const PngUpload& up) {
    if (!up.st || !up.st->area) return false;
    hipEvent_t e = up.st->area->ev[2];
    return e && hipEventQuery(e) == hipSuccess;
}

void png_find_prelaunch(PngUpload& up, hipStream_t s) {
    if (up.st) png_find_launch(*up.st, s);
}

// Decode lanes in launch order.  All lanes of a batch run in one round (two waves
// per SIMD), and a wave lasts as long as its longest lane, so the kernel ends with
// the slowest waves -- the longest blocks, ~20 % past the mean lane
// (IK_TIMING: 8,729 mean / 10,171 max steps).  Lanes sorted by compressed
// length, longest first, fill the first half of the waves; the second half takes
// the shortest first, so wave i and wave W/2 + i -- which the dispatcher puts on
// the same SIMD, one round of waves apart -- pair a long group with a short one
// and the long wave runs alone once its partner is done.  The kernel reads lane
// order[slot] at launch slot `slot` and writes that lane's result in place, so the
// lane table and its results keep job order.  Returns false (no order table) for
// small launches.
static bool order_lanes(const std::vector<PngLaneDev>& hl, const std::vector<PngJob*>& J,
                        std::vector<uint32_t>& order) {
    const size_t n = hl.size();
    if (n < 2 * 64) return false;
    // counting sort on the length in 512-bit buckets, longest first: O(n), as this
    // sits on the host between the decode rounds
    constexpr uint32_t kBuckets = 1024;
    thread_local std::vector<uint16_t> key;
    thread_local std::vector<uint32_t> cnt;
    key.resize(n);
    cnt.assign(kBuckets + 1, 0);
    for (size_t t = 0; t < n; ++t) {
        const PngLaneDev& L = hl[t];
        const uint64_t end = L.stop == ~0ull ? J[L.img]->nbits : L.stop;
        const uint64_t len = end > L.start ? end - L.start : 0;
        const uint32_t b = kBuckets - 1 - (uint32_t)std::min<uint64_t>(len >> 9, kBuckets - 1);  // longest -> 0
        key[t] = (uint16_t)b;
        ++cnt[b + 1];
    }
    for (uint32_t b = 0; b < kBuckets; ++b) cnt[b + 1] += cnt[b];
    // sorted rank r -> launch slot: ranks [0, nlong) in order, then the rest reversed
    const size_t waves = (n + 63) / 64, nlong = std::min(n, (waves + 1) / 2 * 64);
    order.resize(n);
    for (size_t t = 0; t < n; ++t) {
        const size_t r = cnt[key[t]]++;
        order[r < nlong ? r : n - 1 - (r - nlong)] = (uint32_t)t;
    }
    return true;
}

// token region of a lane of `bits` compressed bits (its capacity in tokens)
static uint64_t lane_tok_capacity(uint64_t bits, bool big) {
    return png_wave_decoder() ? wave::region_capacity(bits, big) : infl::tok_capacity(bits, big);
}

int png_decode_finish(PngUpload& up, ik_image** outs, int* status, std::string* msgs) {
    static const bool timing = getenv("IK_TIMING") != nullptr;
    const bool wavedec = png_wave_decoder();
    const double t0 = now_ms();
    double tim[kPngTimingFields] = {};
    Events& ev = events();
    auto rec = [&](int k, hipStream_t st) { if (ev.ok) (void)hipEventRecord(ev.e[k], st); };
    auto reject = [&](PngJob& j, const char* why) {
        j.state = -1;
        if (timing) fprintf(stderr, "[png] stream %d (%ux%u) -> host decoder: %s\n", j.idx, j.w, j.h, why);
    };
    PngBatchState& S = *up.st;
    const uint8_t* const* bytes = up.bytes;
    const size_t* lens = up.lens;
    const int n = up.n;
    for (int i = 0; i < n; ++i) {
        outs[i] = nullptr;
        status[i] = IK_OK;
    }
    double count_dev = 0;
    std::vector<PngJob*>& J = S.J;
    std::vector<char>& gpu = S.gpu;
    const int m = (int)J.size();
    hipStream_t s = thread_stream();
    int rc = S.rc;
    UploadArea* A = S.area;
    if (m && !rc) {
        // ---- the kernel stage's work area (this thread's) ----
        size_t total = 0;
        const int nchunks = S.nchunks;
        for (PngJob* j : J) {
            j->o_u16 = total;
            total += up256(2 * (j->raw_total + 64));
            j->o_ft = total;
            total += up256(j->h);
        }
        const size_t o_imgs = total;
        total += up256(sizeof(PngImgDev) * m);
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
            // (the wave decoder may split lanes at block boundaries: room for more)
            max_lanes += (size_t)j->nchunks + (wavedec ? (size_t)j->nchunks / 4 + 16 : 0);
            tok_total += lane_tok_capacity(j->nbits, false) + (uint64_t)j->nchunks * (lane_tok_capacity(0, false) +
                                                                                      infl::kTokSlack);
        }
        tok_total += tok_total / 2 + 64;
        // the wave decoder's piece tables: per lane wave::pieces_capacity(its bits) entries, handed out as
        // the token regions are (a lane decoded again over a longer range gets a larger one)
        uint64_t pieces_total = 0;
        if (wavedec) {
            for (PngJob* j : J) pieces_total += wave::pieces_capacity(j->nbits) + 64ull * (uint64_t)j->nchunks;
            pieces_total += pieces_total / 2 + 4096;
        }
        const size_t pieces_bytes = up256(sizeof(uint2) * pieces_total);  // (twice: pieces, unit records)
        size_t dyn = up256(sizeof(PngLaneDev) * max_lanes) + up256(sizeof(infl::LaneResult) * max_lanes) +
                     up256(sizeof(int64_t) * max_lanes) + up256(2 * sizeof(int) * max_lanes) +
                     up256(sizeof(uint32_t) * max_lanes) + up256(sizeof(PngImgDev) * m);
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
        dyn += up256(sizeof(int2) * nrows) + up256(sizeof(int) * npages) + unf_tab + unf_zero + 2 * pieces_bytes +
               up256(2 * tok_total);
        uint8_t* dev = scratch_slot(2, o_dyn + dyn);
        if (!dev) rc = fail(IK_ERR_DEVICE, "cannot allocate the PNG batch work area (%zu bytes)", o_dyn + dyn);
        PngLaneDev* d_lanes = nullptr;
        infl::LaneResult* d_res = nullptr;
        int64_t* d_obase = nullptr;
        int* d_xst = nullptr;
        uint32_t* d_order = nullptr;
        PngImgDev* d_cls = nullptr;
        int2* d_rows = nullptr;
        int* d_pages = nullptr;
        uint8_t* d_unf = nullptr;
        uint2* d_pieces = nullptr;
        uint2* d_units = nullptr;  // the wave decoder's expand-unit records (slots parallel to d_pieces)
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
            d_order = reinterpret_cast<uint32_t*>(dev + o);
            o += up256(sizeof(uint32_t) * max_lanes);
            d_cls = reinterpret_cast<PngImgDev*>(dev + o);
            o += up256(sizeof(PngImgDev) * m);
            d_rows = reinterpret_cast<int2*>(dev + o);
            o += up256(sizeof(int2) * nrows);
            d_pages = reinterpret_cast<int*>(dev + o);
            o += up256(sizeof(int) * npages);
            d_unf = dev + o;
            o += unf_tab + unf_zero;
            d_pieces = pieces_bytes ? reinterpret_cast<uint2*>(dev + o) : nullptr;
            o += pieces_bytes;
            d_units = pieces_bytes ? reinterpret_cast<uint2*>(dev + o) : nullptr;
            o += pieces_bytes;
            d_tok = reinterpret_cast<uint16_t*>(dev + o);
        }
        uint64_t tok_used = 0;
        // the small transfers go through the pinned area by copy kernels on this stream:
        // one that falls back to the copy engine queues behind the next batch's PCIe
        // upload (2.25 GB on the bench) and stalls this kernel stage for its length.
        // The expand units' status (2 ints each): a unit holds kUnitMinTok tokens or
        // ends its lane
        const size_t max_units = wavedec ? (size_t)(tok_total / wave::kUnitMinTok) + max_lanes + 16 : 0;
        Xfer X;
        if (!rc && !X.init(2 * sizeof(PngLaneDev) * max_lanes + sizeof(infl::LaneResult) * max_lanes +
                               sizeof(int64_t) * (max_lanes + nchunks) + 3 * sizeof(int) * max_lanes +
                               2 * sizeof(int) * max_units +
                               sizeof(int2) * (nrows + ngroups) + sizeof(int) * (npages + 4 * m) +
                               3 * sizeof(PngImgDev) * m + 2 * sizeof(int) * nchunks + (64u << 10), s))
            rc = fail(IK_ERR_NOMEM, "cannot allocate pinned PNG transfer area");
        // the kernels run under the device's kernel gate (ik_runtime.h)
        gate_enter(kGateKernels);
        // ---- image descriptors ----
        std::vector<PngImgDev> hd(m);
        // the large host tables are kept per thread between batches (clear() keeps
        // the capacity): fresh multi-MB vectors cost page faults every batch
        static thread_local HostTables ht;
        for (int k = 0; k < m && !rc; ++k) {
            PngJob& j = *J[k];
            PngImgDev& d = hd[k];
            d.words = reinterpret_cast<const uint32_t*>(A->dev + S.o_zs + j.z_off);
            d.bit0 = 16;
            d.nbits = j.nbits;
            d.u16 = reinterpret_cast<uint16_t*>(dev + j.o_u16);
            d.raw_total = j.raw_total;
            d.rowbytes = j.rowbytes;
            d.H = (int)j.h;
            d.bpp = j.bpp;
            d.ft = dev + j.o_ft;
        }
        const PngImgDev* d_imgs = reinterpret_cast<const PngImgDev*>(dev + o_imgs);
        // ---- the block search: launched here unless the kernel stage launched it
        // beside the previous batch's unfilter (PngUpload::on_next_search); its
        // candidates come from the upload area ----
        hipError_t e = rc ? hipSuccess : X.h2d(dev + o_imgs, hd.data(), sizeof(PngImgDev) * m);
        const bool pre = S.find_launched;
        if (!rc && e == hipSuccess) {
            png_find_launch(S, s);
            rc = S.rc;
        }
        if (!rc && e == hipSuccess && A->ev[3]) e = hipStreamWaitEvent(s, A->ev[3], 0);
#ifdef IK_FIND_PROF
        {
            (void)hipStreamSynchronize(s);
            unsigned long long pf[8] = {};
            if (png_find_prof_read(pf) == hipSuccess && pf[5])
                fprintf(stderr, "[find-prof] waves %llu: cycles/wave %.0f, flush cycles/wave %.0f (%.1f%%), flushes/wave %.2f, "
                        "steps/wave %.1f, candidates/wave %.1f, kernel %.2f ms\n", pf[5], (double)pf[0] / pf[5],
                        (double)pf[1] / pf[5], 100.0 * pf[1] / std::max(1.0, (double)pf[0]), (double)pf[2] / pf[5],
                        (double)pf[3] / pf[5], (double)pf[4] / pf[5], ev_ms(8, 9));
        }
#endif
        std::vector<int64_t>& cand = ht.cand;
        cand.assign(nchunks, 0);
        std::vector<int> crc_err(m, 0);
        if (!rc && e == hipSuccess) e = X.d2h(cand.data(), A->dev + S.o_cand, sizeof(int64_t) * nchunks);
        if (!rc && e == hipSuccess) {
            e = launch_copy_words(reinterpret_cast<const uint32_t*>(A->dev + S.o_err),
                                  reinterpret_cast<uint32_t*>(dev + o_err), (size_t)m, s);
            if (e == hipSuccess) e = X.d2h(crc_err.data(), dev + o_err, sizeof(int) * m);
        }
        if (!rc && e != hipSuccess) rc = hip_fail(e, "PNG block search");
        for (int k = 0; k < m; ++k)
            if (crc_err[k]) reject(*J[k], "IDAT CRC");  // the host decoder reports png's CRC error
        const double t1 = now_ms();
        tim[15] = t1 - t0;  // from the stage's start until the candidates are back (upload wait + search)
        const double t2 = now_ms();
        double mk[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // dev timing marks (IK_TIMING)
        // the lane plans, one job per pool task (the decode waits on this host work)
        parallel_for(m, 0, [&](int k) {
            PngJob* j = J[k];
            std::vector<int64_t> c(cand.begin() + j->chunk0, cand.begin() + j->chunk0 + j->nchunks);
            pngplan::build(c, j->lanes);
        });
        // ---- decode rounds: token streams; the host checks the lane chain ----
        int rounds = 0, dropped = 0, overflows = 0;
        bool search_done = false;  // the next batch's block search was handed to the hook
        std::vector<PngLaneDev>& hl = ht.lanes;
        std::vector<std::pair<int, int>>& who = ht.who;  // (job, lane) of each launched lane
        std::vector<infl::LaneResult>& hres = ht.res;
        std::vector<uint32_t>& lane_order = ht.order;  // launch slot -> lane (order_lanes)
        hl.clear();
        who.clear();
        hres.clear();
        // first round, in parallel: every lane of every live job is new, and the token
        // area was sized for all of them, so each job's lanes and token regions go to
        // fixed offsets (prefix sums over the jobs) and the jobs fill their parts at once
        bool first_built = false;
        uint64_t p_used = 0;  // piece-table entries handed out (the wave decoder)
        {
            std::vector<size_t> l0(m + 1, 0);
            std::vector<uint64_t> t0(m + 1, 0), q0(m + 1, 0);
            for (int k = 0; k < m; ++k) {
                const PngJob& j = *J[k];
                const pngplan::Lanes& LL = j.lanes;
                size_t nl = 0;
                uint64_t need = 0, pneed = 0;
                if (!j.state)
                    for (size_t i = 0; i < LL.start.size(); ++i) {
                        if (!LL.dirty[i]) continue;
                        const uint64_t end = LL.stop[i] == ~0ull ? j.nbits : LL.stop[i];
                        const uint64_t bits = end > LL.start[i] ? end - LL.start[i] : 0;
                        const uint32_t cap = (uint32_t)lane_tok_capacity(bits, LL.big[i] != 0);
                        ++nl;
                        if (cap > LL.tcap[i]) need += cap + infl::kTokSlack;
                        if (wavedec && wave::pieces_capacity(bits) > LL.pcap[i]) pneed += wave::pieces_capacity(bits);
                    }
                l0[k + 1] = l0[k] + nl;
                t0[k + 1] = t0[k] + need;
                q0[k + 1] = q0[k] + pneed;
            }
            if (tok_used + t0[m] <= tok_total && l0[m] <= max_lanes && p_used + q0[m] <= pieces_total) {
                hl.resize(l0[m]);
                who.resize(l0[m]);
                parallel_for(m, 0, [&](int k) {
                    PngJob& j = *J[k];
                    if (j.state) return;
                    pngplan::Lanes& LL = j.lanes;
                    size_t t = l0[k];
                    uint64_t tu = tok_used + t0[k], pu = p_used + q0[k];
                    for (size_t i = 0; i < LL.start.size(); ++i) {
                        if (!LL.dirty[i]) continue;
                        const uint64_t end = LL.stop[i] == ~0ull ? j.nbits : LL.stop[i];
                        const uint64_t bits = end > LL.start[i] ? end - LL.start[i] : 0;
                        const uint32_t cap = (uint32_t)lane_tok_capacity(bits, LL.big[i] != 0);
                        if (cap > LL.tcap[i]) {
                            LL.tbase[i] = tu;
                            LL.tcap[i] = cap;
                            tu += cap + infl::kTokSlack;
                        }
                        if (wavedec && wave::pieces_capacity(bits) > LL.pcap[i]) {
                            LL.pslot[i] = (int64_t)pu;
                            LL.pcap[i] = wave::pieces_capacity(bits);
                            pu += LL.pcap[i];
                        }
                        PngLaneDev L{};
                        L.start = LL.start[i];
                        L.stop = LL.stop[i];
                        L.tbase = LL.tbase[i];
                        L.ntok = LL.tcap[i];
                        L.img = (uint32_t)k;
                        L.first = i == 0;
                        L.big = LL.big[i] ? 1u : 0u;
                        L.pbase = LL.pslot[i] < 0 ? 0 : (uint64_t)LL.pslot[i];
                        L.npieces = LL.pcap[i];
                        hl[t] = L;
                        who[t] = {k, (int)i};
                        ++t;
                    }
                });
                tok_used += t0[m];
                p_used += q0[m];
                first_built = true;
            }
        }
        while (!rc) {
            if (!first_built) {
                hl.clear();
                who.clear();
                for (int k = 0; k < m; ++k) {
                    PngJob& j = *J[k];
                    if (j.state) continue;
                    pngplan::Lanes& LL = j.lanes;
                    for (size_t i = 0; i < LL.start.size(); ++i) {
                        if (!LL.dirty[i]) continue;
                        const uint64_t end = LL.stop[i] == ~0ull ? j.nbits : LL.stop[i];
                        const uint32_t cap = (uint32_t)lane_tok_capacity(end > LL.start[i] ? end - LL.start[i] : 0,
                                                                         LL.big[i] != 0);
                        if (cap > LL.tcap[i]) {  // a (larger) region from the area
                            const uint64_t need = cap + infl::kTokSlack;
                            if (tok_used + need > tok_total) { reject(j, "token area full"); break; }  // host decoder
                            LL.tbase[i] = tok_used;
                            LL.tcap[i] = cap;
                            tok_used += need;
                        }
                        const uint32_t pneed = wavedec ? wave::pieces_capacity(end > LL.start[i] ? end - LL.start[i] : 0) : 0;
                        if (pneed > LL.pcap[i]) {
                            if (p_used + pneed > pieces_total) { reject(j, "piece tables full"); break; }  // host decoder
                            LL.pslot[i] = (int64_t)p_used;
                            LL.pcap[i] = pneed;
                            p_used += pneed;
                        }
                        PngLaneDev L{};
                        L.start = LL.start[i];
                        L.stop = LL.stop[i];
                        L.tbase = LL.tbase[i];
                        L.ntok = LL.tcap[i];
                        L.img = (uint32_t)k;
                        L.first = i == 0;
                        L.big = LL.big[i] ? 1u : 0u;
                        L.pbase = LL.pslot[i] < 0 ? 0 : (uint64_t)LL.pslot[i];
                        L.npieces = LL.pcap[i];
                        hl.push_back(L);
                        who.emplace_back(k, (int)i);
                    }
                }
            }
            first_built = false;
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
            const bool ordered = order_lanes(hl, J, lane_order);
            const size_t lb = sizeof(PngLaneDev) * hl.size();
            if (X.h2d(d_lanes, hl.data(), lb) != hipSuccess ||
                (ordered && X.h2d(d_order, lane_order.data(), sizeof(uint32_t) * hl.size()) != hipSuccess)) {
                rc = fail(IK_ERR_DEVICE, "PNG lane table upload");
                break;
            }
            hres.resize(hl.size());
            if (!mk[0]) mk[0] = now_ms();  // plan built, lanes uploaded (first round)
            rec(2, s);
            // (IK_FIND_BESIDE: the next batch's block search beside this decode, on another queue)
            if (!search_done && png_find_beside_decode() && up.on_next_search && ev.ok) {
                (void)hipEventRecord(ev.e[11], s);
                up.on_next_search(ev.e[11]);
                search_done = true;
            }
            hipError_t e2 = wavedec ? launch_png_wave(d_imgs, d_lanes, ordered ? d_order : nullptr, (int)hl.size(), d_tok,
                                                      d_pieces, d_units, d_res, s)
                                    : launch_png_decode(d_imgs, d_lanes, ordered ? d_order : nullptr, (int)hl.size(), d_tok,
                                                        d_res, s);
            rec(3, s);
            // the lane results come back behind the decode; the next batch's block
            // search (the stage executor's hook) queues behind that copy, so it runs
            // while this thread checks the lane chain and plans expand / resolve
            size_t roff = ~size_t(0);
            const size_t rbytes = sizeof(infl::LaneResult) * hl.size();
            if (e2 == hipSuccess) e2 = X.d2h_start(d_res, rbytes, &roff, ev.ok ? ev.e[10] : nullptr);
            if (e2 == hipSuccess && !search_done && up.on_next_search) {
                up.on_next_search(nullptr);
                search_done = true;
            }
            if (e2 == hipSuccess) e2 = X.d2h_finish(hres.data(), d_res, rbytes, roff, ev.ok ? ev.e[10] : nullptr);
            if (e2 != hipSuccess) { rc = hip_fail(e2, "PNG inflate (decode)"); break; }
            count_dev += ev_ms(2, 3);
#ifdef IK_WAVE_PROF
            if (wavedec) {
                unsigned long long pf[8] = {};
                if (png_wave_prof_read(pf) == hipSuccess && pf[7])
                    fprintf(stderr, "[wave-prof] lanes %llu: kcycles/lane total %.0f, codes %.0f (lengths %.0f), tables %.0f, "
                            "staging %.0f, first passes %.0f, fix rounds %.0f, rest %.0f\n", pf[7], pf[0] / 1024.0 / pf[7],
                            pf[6] / 1024.0 / pf[7],
                            pf[1] / 1024.0 / pf[7], pf[2] / 1024.0 / pf[7], pf[3] / 1024.0 / pf[7], pf[4] / 1024.0 / pf[7],
                            pf[5] / 1024.0 / pf[7],
                            ((double)pf[0] - pf[1] - pf[2] - pf[3] - pf[4] - pf[5]) / 1024.0 / pf[7]);
            }
#endif
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
        // the compressed streams are read for the last time (every decode round's
        // results were synchronised): the next batch may upload into the area
        (void)hipStreamSynchronize(s);
        {
            float ms = 0;
            if (A->ev[3] && A->ev[4] && hipEventElapsedTime(&ms, A->ev[4], A->ev[3]) == hipSuccess) tim[13] = ms;
            if (A->ev[0] && A->ev[2] && hipEventElapsedTime(&ms, A->ev[0], A->ev[2]) == hipSuccess) tim[1] = ms;
            if (A->ev[1] && A->ev[2] && hipEventElapsedTime(&ms, A->ev[1], A->ev[2]) == hipSuccess) tim[14] = ms;
        }
        tim[16] = pre ? 1.0 : 0.0;
        release_area(S.area);
        const double t3 = now_ms();
        // ---- offsets, output images, expand, resolve, unfilter ----
        std::vector<int64_t>& hob = ht.obase;
        std::vector<int>& hpages = ht.pages;
        hob.clear();
        hpages.clear();
        hl.clear();
        size_t npg = 0;                        // page-table entries so far
        std::vector<std::pair<int, size_t>> pj;  // (job, its first entry in hob) of every verified job
        // the wave decoder's expand units (ik_png_wave.h unit_starts): numbered lane by
        // lane; an image's units are contiguous from uimg[k]
        uint32_t nunits = 0;
        std::vector<uint32_t> uimg(m, 0);
        for (int k = 0; k < m && !rc; ++k) {
            PngJob& j = *J[k];
            if (j.state != 1) continue;
            std::vector<int64_t> ob;
            uint64_t tot = 0;
            pngplan::offsets(j.lanes, ob, &tot);
            if (tot != j.raw_total) { reject(j, "image data length"); continue; }  // png's error
            if (wavedec) {
                bool units_ok = true;
                for (size_t i = 0; i < ob.size(); ++i) units_ok = units_ok && j.lanes.res[i].units > 0;
                if (!units_ok) { reject(j, "expand units"); continue; }
            }
            if (j.expand) {  // unfiltered rows in a row image, then k_png_px into the output image
                if (alloc_image((uint32_t)j.rowbytes, j.h, 1, &j.rows) ||
                alloc_image(j.w, j.h, (uint32_t)j.out_c, &j.img, j.depth == 16 ? 2 : 1)) {
                    reject(j, "image allocation");
                    continue;
                }
            } else if (alloc_image(j.w, j.h, (uint32_t)j.bpp, &j.img)) {
                reject(j, "image allocation");
                continue;
            }
            hd[k].obase = d_obase + hob.size();  // (the wave decoder's: its unit table, set below)
            hd[k].page_lane = d_pages + npg;  // (the page table itself is built while expand runs)
            hd[k].nlanes = (int)ob.size();
            uimg[k] = nunits;
            pj.emplace_back(k, hob.size());
            npg += (j.raw_total >> kPngPageShift) + 1;
            hd[k].dst = j.expand ? j.rows->d : j.img->d;
            hd[k].pitch = j.expand ? j.rows->pitch : j.img->pitch;
            hd[k].flags = reinterpret_cast<const int*>(dev + o_err) + k;
            for (size_t i = 0; i < ob.size(); ++i) tim[12] += (double)j.lanes.res[i].ntok;
            for (size_t i = 0; i < ob.size(); ++i) {
                PngLaneDev L{};
                L.tbase = j.lanes.tbase[i];
                L.obase = ob[i];
                L.out_len = j.lanes.res[i].out_len;
                L.ntok = j.lanes.res[i].ntok;
                L.img = (uint32_t)k;
                L.first = i == 0;
                if (wavedec) {  // the tokens are the lane's pieces (piece table at its slot), expanded by units
                    L.pbase = (uint64_t)j.lanes.pslot[i];
                    L.npieces = j.lanes.res[i].pieces;
                    L.ubase = nunits;
                    L.uimg = uimg[k];
                    L.nunits = j.lanes.res[i].units;
                    nunits += L.nunits;
                }
                hl.push_back(L);
            }
            if (wavedec) hd[k].nlanes = (int)(nunits - uimg[k]);
            hob.insert(hob.end(), ob.begin(), ob.end());
        }
        // the units' tables: offsets (resolve's lane_obase), unit -> lane, expand status
        int64_t* d_uob = nullptr;
        uint32_t* d_ulane = nullptr;
        int* d_uxst = nullptr;
        // and the direct-rows expand's marker list (png_direct_rows): a slot per 16 output bytes
        PngMarks marks;
        if (!rc && wavedec && nunits) {
            uint64_t raw_sum = 0;
            for (const auto& q : pj) raw_sum += J[q.first]->raw_total;
            // (at least 64 K entries per sub-list: a small batch's few units each take one)
            const uint64_t mcap =
                png_direct_rows() ? std::min<uint64_t>(std::max<uint64_t>(raw_sum / 16, 65536ull * kMarkLists), 0xFFFFFF00ull) : 0;
            const size_t b0 = up256(sizeof(int64_t) * nunits), b1 = up256(sizeof(uint32_t) * nunits);
            const size_t b2 = up256(2 * sizeof(int) * nunits),
                         b3 = mcap ? up256(sizeof(uint32_t) * kMarkLists) + up256(sizeof(uint64_t) * mcap) : 0;
            uint8_t* ua = scratch_slot(5, b0 + b1 + b2 + b3);
            if (!ua) {
                rc = fail(IK_ERR_DEVICE, "cannot allocate the PNG expand-unit tables (%u units)", nunits);
            } else {
                d_uob = reinterpret_cast<int64_t*>(ua);
                d_ulane = reinterpret_cast<uint32_t*>(ua + b0);
                d_uxst = reinterpret_cast<int*>(ua + b0 + b1);
                for (const auto& q : pj) hd[q.first].obase = d_uob + uimg[q.first];
                if (mcap) {
                    marks.count = reinterpret_cast<uint32_t*>(ua + b0 + b1 + b2);
                    marks.list = reinterpret_cast<uint64_t*>(ua + b0 + b1 + b2 + up256(sizeof(uint32_t) * kMarkLists));
                    marks.cap = (uint32_t)mcap;
                }
            }
        }
        const size_t nexp = wavedec ? (size_t)nunits : hl.size();  // expand waves: units, or lanes
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
            if (ue == hipSuccess && marks.count) ue = hipMemsetAsync(marks.count, 0, sizeof(uint32_t) * kMarkLists, s);
            if (ue != hipSuccess) rc = hip_fail(ue, "PNG expand tables");
            hxst.resize(2 * nexp);
            mk[2] = now_ms();  // lane tables uploaded
            // the next batch's block search (VALU-bound) beside this batch's expand,
            // resolve and unfilter, which run at a raised wave priority (ik_png.hip
            // raise_priority): the stage executor's hook
            if (!rc && !search_done && up.on_next_search) {
                up.on_next_search(nullptr);
                search_done = true;
            }
            if (!rc) {
                hipError_t e3 = hipSuccess;
                rec(4, s);
                if (wavedec) {
                    // the units' tables and page tables (k_png_units), then one wave per unit
                    if (e3 == hipSuccess) e3 = launch_png_units(d_imgs, d_lanes, (int)hl.size(), d_units, d_ulane, s);
                    if (e3 == hipSuccess)
                        e3 = launch_png_expand(d_imgs, d_lanes, (int)nunits, d_tok, d_uxst, s, d_pieces, d_units, d_ulane,
                                               marks);
                } else if (e3 == hipSuccess) {
                    e3 = launch_png_expand(d_imgs, d_lanes, (int)hl.size(), d_tok, d_xst, s);
                }
                rec(5, s);
                // page -> decoder that holds the page's first byte (resolve's lane lookup;
                // the wave decoder's units: k_png_units built it)
                for (const auto& q : pj) {
                    const PngJob& j = *J[q.first];
                    if (!wavedec) {
                        const int64_t* ob = hob.data() + q.second;
                        const size_t nl = (size_t)hd[q.first].nlanes;
                        for (uint64_t pg = 0, ln = 0; pg <= (j.raw_total >> kPngPageShift); ++pg) {
                            while (ln + 1 < nl && (uint64_t)ob[ln + 1] <= (pg << kPngPageShift)) ++ln;
                            hpages.push_back((int)ln);
                        }
                    }
                    for (uint32_t y = 0; y < j.h; ++y) hrows.push_back(make_int2(q.first, (int)y));
                }
                if (e3 == hipSuccess && !wavedec) e3 = X.h2d(d_pages, hpages.data(), sizeof(int) * hpages.size());
                if (e3 == hipSuccess) e3 = X.h2d(d_rows, hrows.data(), sizeof(int2) * hrows.size());
                if (e3 == hipSuccess)
                    e3 = marks.list ? launch_png_marks(d_imgs, marks, d_rows, (int)hrows.size(), reinterpret_cast<int*>(dev + o_err), s)
                                    : launch_png_resolve(d_imgs, d_rows, (int)hrows.size(), reinterpret_cast<int*>(dev + o_err), s);
                rec(6, s);
#ifdef IK_PNG_DUMP  // dev experiment: every image's filtered rows and filter types before the unfilter
                if (e3 == hipSuccess) {
                    (void)hipStreamSynchronize(s);
                    png_dump_store(J, hd, m);
                }
#endif
                // unfilter (+ png's EXPAND), as a step of its own: the direct-rows path whose
                // marker list overflowed runs resolve and this again (below)
                auto unfilter_all = [&](hipError_t e3) -> hipError_t {
                    // unfilter: one launch per bytes-per-pixel class, over that class's
                    // images; a workgroup per 16 bands, its (image, group) by ticket
                    if (e3 == hipSuccess) {
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
                        e3 = X.h2d(d_unf, tabs.data(), unf_tab);
                        unsigned* d_prog = reinterpret_cast<unsigned*>(d_unf + unf_tab);
                        unsigned* d_ticket = d_prog + nbands;
                        if (e3 == hipSuccess) e3 = hipMemsetAsync(d_prog, 0, unf_zero, s);
                        if (e3 == hipSuccess) e3 = X.h2d(d_cls, cls.data(), sizeof(PngImgDev) * cls.size());
                        const int2* d_groups = reinterpret_cast<const int2*>(d_unf);
                        const int* d_pbase = reinterpret_cast<const int*>(d_unf + gb);
                        // RGBA8 images of None / Sub / Up rows take the scan path, the others
                        // the diagonal kernel; each skips the other's images, so the diagonal
                        // one runs beside, on this thread's high-priority stream (fork / join
                        // by events): 1.3 + 1.9 ms in turn -> 1.8-2.0 ms together
                        static thread_local hipEvent_t fork_ev = nullptr, join_ev = nullptr;
                        if (!fork_ev && (hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming) != hipSuccess ||
                                         hipEventCreateWithFlags(&join_ev, hipEventDisableTiming) != hipSuccess))
                            fork_ev = join_ev = nullptr;
                        hipStream_t side = nullptr;
                        hipEvent_t side_ev = nullptr;
                        if (fork_ev && !thread_prio_stream(&side, &side_ev)) side = nullptr;
                        for (size_t r = 0; r < ranges.size() && e3 == hipSuccess; ++r) {
                            const int g1 = r + 1 < ranges.size() ? ranges[r + 1].grp0 : (int)groups.size();
                            const int g0 = ranges[r].grp0, i0 = ranges[r].img0;
                            const int i1 = r + 1 < ranges.size() ? ranges[r + 1].img0 : (int)cls.size();
                            const bool fork = side && ranges[r].bpp == 4;
                            if (fork) {
                                e3 = hipEventRecord(fork_ev, s);
                                if (e3 == hipSuccess) e3 = hipStreamWaitEvent(side, fork_ev, 0);
                            }
                            if (e3 == hipSuccess)
                                e3 = launch_png_unfilter(d_cls + i0, d_groups + g0, g1 - g0, d_pbase + i0, d_prog,
                                                         d_ticket + r, ranges[r].bpp, fork ? side : s);
                            if (e3 == hipSuccess && ranges[r].bpp == 4) e3 = launch_png_unfilter_su(d_cls + i0, i1 - i0, s);
                            if (fork && e3 == hipSuccess) {
                                e3 = hipEventRecord(join_ev, side);
                                if (e3 == hipSuccess) e3 = hipStreamWaitEvent(s, join_ev, 0);
                            }
                        }
                    }
                    // png's EXPAND for the palette / low-bit / tRNS images
                    for (int k = 0; k < m && e3 == hipSuccess; ++k) {
                        PngJob& j = *J[k];
                        if (j.state != 1 || !j.expand || !j.rows) continue;
                        j.px.src = j.rows->d;
                        j.px.sp = j.rows->pitch;
                        j.px.dst = j.img->d;
                        j.px.dp = j.img->pitch;
                        e3 = launch_png_px(j.px, s);
                    }
                    return e3;
                };
                e3 = unfilter_all(e3);
                rec(7, s);
#ifdef IK_EXP_PROF
                {
                    (void)hipStreamSynchronize(s);
                    unsigned long long pf[8] = {};
                    if (png_exp_prof_read(pf) == hipSuccess && pf[0])
                        fprintf(stderr, "[exp-prof] waves %zu: kcycles/wave %.0f: token wait %.0f, scan %.0f, literals %.0f, "
                                "matches %.0f, stores+sync %.0f, loop %.0f; batches/wave %.1f\n", nexp,
                                pf[0] / 1024.0 / nexp, pf[6] / 1024.0 / nexp, pf[1] / 1024.0 / nexp, pf[2] / 1024.0 / nexp,
                                pf[3] / 1024.0 / nexp, pf[4] / 1024.0 / nexp, pf[5] / 1024.0 / nexp, (double)pf[7] / nexp);
                }
#endif
#ifdef IK_UNF_PROF
                {
                    (void)hipStreamSynchronize(s);
                    unsigned long long pf[8] = {};
                    if (png_unf_prof_read(pf) == hipSuccess && pf[7])
                        fprintf(stderr, "[unf-prof] waves %llu: cycles/wave above %.0f, fetch-issue %.0f, steps %.0f, publish "
                                "%.0f, landed %.0f; unfilter %.2f ms\n", pf[7], (double)pf[0] / pf[7], (double)pf[1] / pf[7],
                                (double)pf[2] / pf[7], (double)pf[3] / pf[7], (double)pf[4] / pf[7], ev_ms(6, 7));
                }
#endif
                uint32_t nmarks = 0, mcnt[kMarkLists];
                bool mover = false;
                if (e3 == hipSuccess && marks.count) {
                    e3 = X.d2h(mcnt, marks.count, sizeof(mcnt));
                    for (uint32_t q = 0; q < kMarkLists; ++q) {
                        nmarks += mcnt[q];
                        mover = mover || mcnt[q] > marks.cap / kMarkLists;
                    }
                }
                if (e3 == hipSuccess && mover) {
                    // the marker list overflowed (runs of copies across units, e.g. a flat
                    // image): the rows from the u16 symbols after all, then the unfilter again
                    if (timing) fprintf(stderr, "[png] %u window markers > list %u: resolve pass\n", nmarks, marks.cap);
                    e3 = hipMemsetAsync(dev + o_err, 0, sizeof(int) * m, s);
                    if (e3 == hipSuccess)
                        e3 = launch_png_resolve(d_imgs, d_rows, (int)hrows.size(), reinterpret_cast<int*>(dev + o_err), s);
                    e3 = unfilter_all(e3);
                }
                if (timing && marks.count) fprintf(stderr, "[png] window markers %u (list %u)\n", nmarks, marks.cap);
                if (e3 == hipSuccess) e3 = X.d2h(hxst.data(), wavedec ? d_uxst : d_xst, 2 * sizeof(int) * nexp);
                if (e3 == hipSuccess) e3 = X.d2h(herr.data(), dev + o_err, sizeof(int) * m);
                mk[3] = now_ms();  // expand .. unfilter done
                if (e3 != hipSuccess) rc = hip_fail(e3, "PNG inflate (expand) / unfilter");
                if (!rc) {
                    tim[3] = ev_ms(4, 5);
                    tim[4] = ev_ms(5, 6);
                    tim[5] = ev_ms(6, 7);
                }
            }
            if (!rc) {
                size_t t = 0;
                for (int k = 0; k < m; ++k) {
                    PngJob& j = *J[k];
                    if (j.state != 1) continue;
                    const bool rows_ok = (herr[k] & 3) == 0;  // (bit 4: Average / Paeth rows, not an error)
                    bool lanes_ok = true;
                    for (size_t i = 0; i < j.lanes.start.size(); ++i) {
                        const uint32_t nu = wavedec ? j.lanes.res[i].units : 1u;  // expand waves of this lane
                        for (uint32_t u = 0; u < nu; ++u, ++t) {
                            lanes_ok = lanes_ok && hxst[2 * t] == 0;
                            if (timing && hxst[2 * t] != 0) {
                                const infl::LaneResult& q = j.lanes.res[i];
                                fprintf(stderr, "[png] stream %d lane %zu/%zu unit %u/%u: expand failed (start %llu stop %llu "
                                        "end %llu out %llu tokens %u pieces %u blocks %u status %d)\n", j.idx, i,
                                        j.lanes.start.size(), u, nu, (unsigned long long)j.lanes.start[i],
                                        (unsigned long long)j.lanes.stop[i], (unsigned long long)q.end_bit,
                                        (unsigned long long)q.out_len, q.ntok, q.pieces, q.blocks, q.status);
                            }
                        }
                    }
                    if (!rows_ok || !lanes_ok) reject(j, !lanes_ok ? "expand status" : "row filter bytes");
                }
            }
        }
        gate_leave(kGateKernels);  // unless the caller pinned it (transform_part: resize + encode next)
        if (timing && !hl.empty()) {  // per-lane profile of the last decode round and the expand pass
            double si = 0, sc = 0, sx = 0, mi = 0, mc = 0, mx = 0, sb = 0, mb = 0, ss = 0;
            for (size_t t = 0; t < hres.size(); ++t) {
                si += hres[t].iters; sc += hres[t].kcycles; sb += hres[t].blocks; ss += hres[t].kc_setup;
                mi = std::max(mi, (double)hres[t].iters); mc = std::max(mc, (double)hres[t].kcycles);
                mb = std::max(mb, (double)hres[t].blocks);
            }
            for (size_t t = 0; 2 * t + 1 < hxst.size(); ++t) {
                sx += hxst[2 * t + 1];
                mx = std::max(mx, (double)hxst[2 * t + 1]);
            }
            const double n1 = (double)std::max<size_t>(1, hres.size()), n2 = (double)std::max<size_t>(1, hxst.size() / 2);
            fprintf(stderr, "[png] decode lanes %zu: iters mean %.0f max %.0f, blocks mean %.2f max %.0f, kcycles mean %.0f "
                    "max %.0f (%.0f cycles/iter; setup kcycles mean %.0f); expand kcycles mean %.0f max %.0f\n",
                    hres.size(), si / n1, mi, sb / n1, mb, sc / n1, mc, 1024.0 * sc / std::max(1.0, si), ss / n1, sx / n2,
                    mx);
        }
        tim[0] = S.t_host;
        tim[2] = count_dev;
        tim[7] = rounds;
        tim[8] = (double)hl.size();
        tim[9] = m;
        if (timing)
            fprintf(stderr, "[png] t=%.1f %d streams (%d on the GPU): upload host %.2f ms, upload device %.2f ms (gather "
                    "%.2f), waited+find %.2f ms (find %.2f), decode %.2f ms (%d rounds, %d dropped, %d overflows), "
                    "expand+resolve+unfilter %.2f ms\n",
                    fmod(t0, 1e5), n, m, tim[0], tim[1], tim[14], t1 - t0, tim[13], t3 - t2, rounds, dropped, overflows,
                    now_ms() - t3);
        if (timing)
            fprintf(stderr, "[png] host: plan+lanes %.2f, (decode rounds) .. tables %.2f, rows+uploads %.2f, "
                    "(expand..unfilter) %.2f, after %.2f ms\n", mk[0] - t2, mk[1] - t3, mk[2] - mk[1], mk[3] - mk[2],
                    now_ms() - mk[3]);
    }
    release_area(S.area);  // (error paths)
    if (m) {
        (void)hipStreamSynchronize(s);  // the row images are read
        for (int k = 0; k < m; ++k) {
            PngJob& j = *J[k];
            if (j.rows) { ik_image_free(j.rows); j.rows = nullptr; }
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
    tim[11] = (double)host.size();
    tim[10] = (double)(n - (int)host.size());
    g_png_gpu_streams += (unsigned long long)(n - (int)host.size());
    g_png_host_streams += (unsigned long long)host.size();
    parallel_for((int)host.size(), 0, [&](int k) {
        const int i = host[k];
        thread_local std::vector<uint8_t> px;
        uint32_t w = 0, h = 0, c = 0, dep = 1;
        // a device-resident file comes back to host memory for the host decoder
        std::vector<uint8_t> hb;
        const uint8_t* src = bytes[i];
        if (up.dev) {
            hb.resize(lens[i]);
            if (lens[i] && hipMemcpy(hb.data(), bytes[i], lens[i], hipMemcpyDeviceToHost) != hipSuccess) {
                status[i] = hip_fail(hipErrorUnknown, "PNG device input copy");
                if (msgs) msgs[i] = "PNG device input copy failed";
                return;
            }
            src = hb.data();
        }
        int st = decode_png(src, lens[i], w, h, c, px, &dep);
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
    tim[6] = now_ms() - t0;
    if (m) {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        g_timing[S.device].assign(tim, tim + kPngTimingFields);
    }
    if (timing) fprintf(stderr, "[png] decode_png_batch returns at t=%.1f\n", fmod(now_ms(), 1e5));
    up.st.reset();
    int first = IK_OK;
    for (int i = 0; i < n; ++i)
        if (status[i] && !first) first = status[i];
    return first;
}

int decode_png_batch(const uint8_t* const* bytes, const size_t* lens, int n, ik_image** outs, int* status,
                     std::string* msgs) {
    PngUpload up;
    png_upload_begin(bytes, lens, n, up);
    return png_decode_finish(up, outs, status, msgs);
}

}  // namespace ik

extern "C" int ik_png_counters(unsigned long long* out) {
    out[0] = ik::g_png_gpu_streams.load();
    out[1] = ik::g_png_host_streams.load();
    return IK_OK;
}

extern "C" int ik_png_last_timing(double* out, int n) {
    if (!out) return ik::fail(IK_ERR_INVALID, "null pointer");
    std::vector<double> t;
    {
        std::lock_guard<std::mutex> lk(ik::g_timing_mu);
        auto it = ik::g_timing.find(ik::current_device());
        if (it != ik::g_timing.end()) t = it->second;
    }
    for (int i = 0; i < n; ++i) out[i] = i < (int)t.size() ? t[i] : 0.0;
    return IK_OK;
}

extern "C" int ik_set_png_gpu_min(long long min_raw_bytes) {
    (void)ik::png_gpu_min();
    ik::g_png_gpu_min.store(min_raw_bytes < 0 ? -1 : min_raw_bytes);
    return IK_OK;
}

#ifdef IK_PNG_DUMP
// dev experiment: image i of the last GPU PNG batch before its unfilter (rows, then filter types)
extern "C" long long ik_dev_png_dump(int i, uint8_t* out, size_t cap) {
    std::lock_guard<std::mutex> lk(ik::g_dump_mu);
    if (i < 0 || i >= (int)ik::g_dump.size()) return -1;
    const auto& v = ik::g_dump[i];
    if (out) std::memcpy(out, v.data(), std::min(cap, v.size()));
    return (long long)v.size();
}
#endif
