// ik_host.cpp -- the C ABI of libimagekit_hip.so (include/imagekit_hip.h).
//
// Mirrors reference src/transform.rs: decode_image (:27-43), resize_image
// (:62-90), encode_image (:113-150) with the error mapping of src/lib.rs:34-52
// (every failure is a status + thread-local message, never a panic).  Pixels
// stay device-resident between the three calls; only compressed bytes cross
// PCIe (plus the small planes/coefficients handed to the host entropy coders).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <tuple>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <deque>

#include "../../include/imagekit_hip.h"
#include "ik_png.h"
#include "ik_runtime.h"

namespace ik {

static thread_local std::string t_err;
static thread_local int t_device = -1;

int fail(int status, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_err = buf;
    return status;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(IK_ERR_DEVICE, "HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
}

int current_device() {
    if (t_device < 0) {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) d = 0;
        t_device = d;
    }
    return t_device;
}

DeviceGuard::DeviceGuard(int device) : prev(current_device()) {
    if (device != prev) {
        t_device = device;
        (void)hipSetDevice(device);
    }
}
DeviceGuard::~DeviceGuard() {
    if (t_device != prev) {
        t_device = prev;
        (void)hipSetDevice(prev);
    }
}

// Per-thread HIP resources: a non-blocking stream per device, pinned staging
// arenas and grow-only device arenas.  Worker threads are persistent (ik_pool.cpp),
// so these live as long as the process; a caller's own thread releases its set
// when it exits.
namespace {
struct Arena {
    uint8_t* p = nullptr;
    size_t cap = 0;
    int device = 0;
};
struct ThreadRes {
    std::map<int, hipStream_t> streams, copy_streams, prio_streams;
    std::map<int, hipEvent_t> prio_events;
    std::map<std::pair<int, int>, Arena> dev;  // (device, slot)
    Arena pinned[11];
    void release() {
        for (auto& kv : streams) (void)hipStreamSynchronize(kv.second);
        for (auto& kv : copy_streams) (void)hipStreamSynchronize(kv.second);
        for (auto& kv : prio_streams) (void)hipStreamSynchronize(kv.second);
        for (auto& kv : dev) {
            if (!kv.second.p) continue;
            (void)hipSetDevice(kv.second.device);
            (void)hipFree(kv.second.p);
            mem_stat(kMemArenaDev, -(int64_t)kv.second.cap);
        }
        for (Arena& a : pinned)
            if (a.p) {
                (void)hipHostFree(a.p);
                mem_stat(kMemArenaPinned, -(int64_t)a.cap);
            }
        for (auto& kv : streams) (void)hipStreamDestroy(kv.second);
        for (auto& kv : copy_streams) (void)hipStreamDestroy(kv.second);
        for (auto& kv : prio_streams) (void)hipStreamDestroy(kv.second);
        for (auto& kv : prio_events) (void)hipEventDestroy(kv.second);
        streams.clear();
        copy_streams.clear();
        prio_streams.clear();
        prio_events.clear();
        dev.clear();
        for (Arena& a : pinned) a = Arena();
    }
    // a caller's own thread that exits releases its set here; workers and stage
    // threads release theirs before they end (ik_shutdown), and after ik_shutdown
    // the process's main thread holds none, so nothing is left to a destructor that
    // runs during process exit
    ~ThreadRes() { release(); }
};
ThreadRes& tres() {
    static thread_local ThreadRes r;
    return r;
}
}  // namespace

void release_thread_resources() { tres().release(); }

namespace {
std::mutex g_bt_mu;
// per device: the batches in the decode and post stages, the last one finished
std::map<int, std::vector<double>> g_bt_dec, g_bt_post, g_bt_last;
bool bt_post_field(int f) { return f >= kBtResizeMs && f < kBtHostWallMs; }
bool bt_host_field(int f) { return f >= kBtHostWallMs; }
thread_local bool t_bt_active = false;  // inside a stage's batch (BatchTimingScope)
// per device (an event records only on its own device's streams); the events are
// left to the runtime: a thread-exit destructor may run at process exit
struct ThreadEvents {
    std::map<int, std::array<EvPair, 4>> p;
};

// the lifetime lock (ApiGuard): shared by callers, exclusive for teardown, and
// writer-preferring -- a waiting teardown holds back new callers, so callers that
// keep calling (a server's request threads) cannot starve it
struct LifeLock {
    std::mutex mu;
    std::condition_variable cv;
    int readers = 0, writers_waiting = 0;
    bool writer = false;
    void lock_shared() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !writer && writers_waiting == 0; });
        ++readers;
    }
    void unlock_shared() {
        std::lock_guard<std::mutex> lk(mu);
        if (--readers == 0) cv.notify_all();
    }
    void lock() {
        std::unique_lock<std::mutex> lk(mu);
        ++writers_waiting;
        cv.wait(lk, [&] { return !writer && readers == 0; });
        --writers_waiting;
        writer = true;
    }
    void unlock() {
        std::lock_guard<std::mutex> lk(mu);
        writer = false;
        cv.notify_all();
    }
};
LifeLock g_life;
std::atomic<bool> g_closed{false};
thread_local int t_api_depth = 0;
thread_local bool t_internal = false;
}  // namespace

ApiGuard::ApiGuard() {
    if (t_internal) return;
    if (t_api_depth++ == 0) {
        g_life.lock_shared();
        held = true;
    }
    closed = g_closed.load(std::memory_order_acquire);
}
ApiGuard::~ApiGuard() {
    if (t_internal) return;
    if (--t_api_depth == 0 && held) g_life.unlock_shared();
}
void mark_internal_thread() { t_internal = true; }

namespace {
std::atomic<int64_t> g_mem[kMemStats];
}  // namespace
void mem_stat(int which, int64_t delta) { g_mem[which].fetch_add(delta, std::memory_order_relaxed); }

BatchTimingScope::BatchTimingScope() : prev(t_bt_active) { t_bt_active = true; }
BatchTimingScope::~BatchTimingScope() { t_bt_active = prev; }

void ev_record(hipEvent_t e, hipStream_t s) {
    if (e && hipEventRecord(e, s) != hipSuccess) (void)hipGetLastError();
}

void batch_timing_reset(int device, bool post) {
    std::lock_guard<std::mutex> lk(g_bt_mu);
    (post ? g_bt_post : g_bt_dec)[device].assign(kBtFields, 0.0);
}
void batch_timing_commit(int device, bool post) {
    std::lock_guard<std::mutex> lk(g_bt_mu);
    std::vector<double>& src = (post ? g_bt_post : g_bt_dec)[device];
    std::vector<double>& dst = g_bt_last[device];
    src.resize(kBtFields, 0.0);
    dst.resize(kBtFields, 0.0);
    for (int f = 0; f < kBtFields; ++f)
        if (!bt_host_field(f) && bt_post_field(f) == post) dst[(size_t)f] = src[(size_t)f];
}
void batch_timing_host(int device, double wall_ms, double core_ms, double images) {
    std::lock_guard<std::mutex> lk(g_bt_mu);
    std::vector<double>& dst = g_bt_last[device];
    dst.resize(kBtFields, 0.0);
    dst[kBtHostWallMs] = wall_ms;
    dst[kBtHostCoreMs] = core_ms;
    dst[kBtHostImages] = images;
}
void batch_timing_add(int device, int field, double v) {
    if (!t_bt_active) return;
    std::lock_guard<std::mutex> lk(g_bt_mu);
    std::vector<double>& t = (bt_post_field(field) ? g_bt_post : g_bt_dec)[device];
    if (t.size() < (size_t)kBtFields) t.resize(kBtFields, 0.0);
    t[(size_t)field] += v;
}
EvPair& thread_events(int which) {
    static thread_local ThreadEvents te;
    EvPair& e = te.p[current_device()][which & 3];
    if (!e.a && hipEventCreate(&e.a) != hipSuccess) e.a = nullptr;
    if (!e.b && hipEventCreate(&e.b) != hipSuccess) e.b = nullptr;
    return e;
}
float ev_pair_ms(const EvPair& e) {
    float ms = 0;
    if (!e.a || !e.b || hipEventElapsedTime(&ms, e.a, e.b) != hipSuccess) return 0.f;
    return ms;
}

hipStream_t thread_stream() {
    ThreadRes& r = tres();
    const int d = current_device();
    auto it = r.streams.find(d);
    if (it != r.streams.end()) return it->second;
    (void)hipSetDevice(d);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    r.streams[d] = s;
    return s;
}

// The upload stream (PCIe copies of whole batches: 2.25 GB on the bench, ~42 ms)
// at the lowest stream priority: a stream of another priority never shares its
// hardware queue, so no kernel of another stage waits in queue order behind a
// batch's DMA (GPU_MAX_HW_QUEUES is 4: same-priority streams share queues).
hipStream_t thread_copy_stream() {
    ThreadRes& r = tres();
    const int d = current_device();
    auto it = r.copy_streams.find(d);
    if (it != r.copy_streams.end()) return it->second;
    (void)hipSetDevice(d);
    hipStream_t s = nullptr;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
    // (the priority other than the default one: the lowest if it is not the default)
    const int prio = least != 0 ? least : greatest;
    if (getenv("IK_TIMING")) fprintf(stderr, "[streams] priority range %d..%d: upload stream at %d\n", least, greatest, prio);
    if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio) != hipSuccess &&
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return nullptr;
    r.copy_streams[d] = s;
    return s;
}

bool thread_prio_stream(hipStream_t* out, hipEvent_t* ev) {
    ThreadRes& r = tres();
    const int d = current_device();
    auto it = r.prio_streams.find(d);
    if (it == r.prio_streams.end()) {
        (void)hipSetDevice(d);
        hipStream_t s = nullptr;
        hipEvent_t e = nullptr;
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
        if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(s);
            return false;
        }
        it = r.prio_streams.emplace(d, s).first;
        r.prio_events[d] = e;
    }
    *out = it->second;
    *ev = r.prio_events[d];
    return true;
}

uint8_t* pinned_slot(int slot, size_t bytes) {
    Arena& a = tres().pinned[slot];
    if (bytes <= a.cap) return a.p;
    if (a.p) {
        (void)hipStreamSynchronize(thread_stream());  // no copy may still read the old buffer
        auto cs = tres().copy_streams.find(current_device());
        if (cs != tres().copy_streams.end()) (void)hipStreamSynchronize(cs->second);
        auto ps = tres().prio_streams.find(current_device());
        if (ps != tres().prio_streams.end()) (void)hipStreamSynchronize(ps->second);
        (void)hipHostFree(a.p);
        mem_stat(kMemArenaPinned, -(int64_t)a.cap);
    }
    a.p = nullptr;
    a.cap = 0;
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    const hipError_t e = hipHostMalloc((void**)&a.p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
        a.p = nullptr;
        fail(IK_ERR_NOMEM, "hipHostMalloc(%zu bytes): %s", want, hipGetErrorString(e));
        return nullptr;
    }
    a.cap = want;
    mem_stat(kMemArenaPinned, (int64_t)want);
    return a.p;
}

// Caller-pinned ranges (ik_host_alloc / ik_host_register): inputs inside one are
// DMAed in place.  Keyed by start address; the ranges never overlap.
namespace {
struct PinnedRange {
    size_t n = 0;
    bool owned = false;  // ik_host_alloc (hipHostFree) vs ik_host_register (hipHostUnregister)
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinnedRange> g_pins;
}  // namespace

bool host_pinned(const void* p, size_t n) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.upper_bound(a);
    if (it == g_pins.begin()) return false;
    --it;
    return a >= it->first && a - it->first <= it->second.n && n <= it->second.n - (a - it->first);
}

// Host <-> device copies of pageable memory go through a per-thread pinned
// staging buffer with stream-ordered async copies on the thread's stream.  (A
// synchronous hipMemcpy* from pageable memory is issued on the null stream, and
// a non-blocking stream is not ordered after its DMA.)
static uint8_t* staging(size_t bytes) { return pinned_slot(0, bytes); }

int copy_h2d_2d(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                size_t height, hipStream_t s) {
    const size_t chunk_rows = height ? (size_t)((64u << 20) / (width ? width : 1)) + 1 : 1;
    for (size_t y0 = 0; y0 < height; y0 += chunk_rows) {
        const size_t rows = height - y0 < chunk_rows ? height - y0 : chunk_rows;
        uint8_t* st = staging(rows * width);
        if (!st) return IK_ERR_NOMEM;  // pinned_slot recorded the error
        for (size_t y = 0; y < rows; ++y) std::memcpy(st + y * width, src + (y0 + y) * spitch, width);
        IK_HIP(hipMemcpy2DAsync(dst + y0 * dpitch, dpitch, st, width, width, rows, hipMemcpyHostToDevice, s));
        IK_HIP(hipStreamSynchronize(s));
    }
    return IK_OK;
}

int copy_d2h_2d(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                size_t height, hipStream_t s) {
    const size_t chunk_rows = height ? (size_t)((64u << 20) / (width ? width : 1)) + 1 : 1;
    for (size_t y0 = 0; y0 < height; y0 += chunk_rows) {
        const size_t rows = height - y0 < chunk_rows ? height - y0 : chunk_rows;
        uint8_t* st = staging(rows * width);
        if (!st) return IK_ERR_NOMEM;  // pinned_slot recorded the error
        IK_HIP(hipMemcpy2DAsync(st, width, src + y0 * spitch, spitch, width, rows, hipMemcpyDeviceToHost, s));
        IK_HIP(hipStreamSynchronize(s));
        for (size_t y = 0; y < rows; ++y) std::memcpy(dst + (y0 + y) * dpitch, st + y * width, width);
    }
    return IK_OK;
}

// Per-thread, per-device device scratch (grown with hipMalloc; never the
// stream-ordered allocator).  Valid until the next scratch() call on this thread.
uint8_t* scratch_slot(int slot, size_t bytes) {
    const int d = current_device();
    Arena& a = tres().dev[{d, slot}];
    a.device = d;
    if (bytes <= a.cap) return a.p;
    if (a.p) {
        (void)hipStreamSynchronize(thread_stream());
        auto ps = tres().prio_streams.find(d);
        if (ps != tres().prio_streams.end()) (void)hipStreamSynchronize(ps->second);
        (void)hipFree(a.p);
        mem_stat(kMemArenaDev, -(int64_t)a.cap);
    }
    a.p = nullptr;
    a.cap = 0;
    // grow geometrically so a run of slightly larger requests does not re-allocate each time
    size_t want = bytes < (4u << 20) ? (4u << 20) : bytes + bytes / 8;
    (void)hipSetDevice(d);
    if (hipMalloc((void**)&a.p, want) != hipSuccess) return nullptr;
    a.cap = want;
    mem_stat(kMemArenaDev, (int64_t)want);
    return a.p;
}

uint8_t* scratch(size_t bytes) { return scratch_slot(0, bytes); }

size_t pitch_for(uint32_t w, uint32_t c) { return ((size_t)w * c + 255) & ~size_t(255); }

// Device image blocks are recycled per device: hipFree synchronises the whole
// device, which would serialise every thread's stream under request load.  A
// freed block is kept (up to kPoolBytes per device) and handed to the next image
// that fits in it; every API call has synchronised its own stream before it
// returns, so a block is idle when it comes back.
namespace {
// 32 GiB of the 288 GB: two 64-frame 4096^2 batches in flight hold 8 GiB of decoded
// frames; at 4 GiB the pool overflowed every batch, and each hipFree of an
// overflowing block stalled the whole device (and every concurrent batch)
constexpr size_t kPoolBytes = size_t(32) << 30;
struct ImagePool {
    std::mutex mu;
    std::multimap<size_t, uint8_t*> free_blocks;
    size_t held = 0;
};
std::mutex g_ipool_mu;
std::map<int, ImagePool*> g_ipools;
ImagePool& image_pool(int device) {
    std::lock_guard<std::mutex> lk(g_ipool_mu);
    ImagePool*& p = g_ipools[device];
    if (!p) p = new ImagePool();
    return *p;
}
size_t block_size(size_t bytes) {  // 64 KiB granules: images of similar sizes share blocks
    return (bytes + (size_t(64) << 10) - 1) & ~((size_t(64) << 10) - 1);
}
}  // namespace

int alloc_image(uint32_t w, uint32_t h, uint32_t c, ik_image** out, uint32_t depth) {
    auto* img = new ik_image();
    img->w = w; img->h = h; img->c = c; img->depth = depth;
    img->pitch = pitch_for(w, c * depth);
    img->device = current_device();
    (void)hipSetDevice(img->device);
    // + 16 bytes: the fused kernel's 8-byte lane loads may touch the pitch tail
    const size_t need = block_size(img->pitch * (size_t)(h ? h : 1) + 16);
    ImagePool& pool = image_pool(img->device);
    {
        std::lock_guard<std::mutex> lk(pool.mu);
        auto it = pool.free_blocks.lower_bound(need);
        if (it != pool.free_blocks.end() && it->first <= 2 * need) {  // reuse a block at most twice the size
            img->d = it->second;
            img->block = it->first;
            pool.held -= it->first;
            pool.free_blocks.erase(it);
            mem_stat(kMemImageFree, -(int64_t)img->block);
        }
    }
    if (!img->d) {
        hipError_t e = hipMalloc(&img->d, need);
        if (e != hipSuccess) { delete img; return hip_fail(e, "hipMalloc(image)"); }
        img->block = need;
    }
    mem_stat(kMemImageLive, (int64_t)img->block);
    *out = img;
    return IK_OK;
}

void webp_gamma_tables(uint16_t g2l[256], int l2g[33]) {
    // libwebp picture_csp_enc.c InitGammaTables: kGamma 0.80, kGammaFix 12, kGammaTabFix 7
    const double scale = (double)(1 << 7) / ((1 << 12) - 1);
    const double norm = 1. / 255.;
    for (int v = 0; v <= 255; ++v) g2l[v] = (uint16_t)(pow(norm * v, 0.80) * ((1 << 12) - 1) + .5);
    for (int v = 0; v <= 32; ++v) l2g[v] = (int)(255. * pow(scale * v, 1. / 0.80) + .5);
}

namespace {
std::atomic<int> g_resize_mode{-1};  // -1 = not yet read from IK_RESIZE_MODE
}  // namespace

int resize_mode() {
    int m = g_resize_mode.load();
    if (m < 0) {
        const char* e = getenv("IK_RESIZE_MODE");
        m = (e && (!strcmp(e, "fma") || !strcmp(e, "1"))) ? IK_RESIZE_FMA : IK_RESIZE_EXACT;
        int expected = -1;
        g_resize_mode.compare_exchange_strong(expected, m);
        m = g_resize_mode.load();
    }
    return m;
}

namespace {
std::mutex g_consts_mu;
std::map<int, DeviceConsts*> g_consts;
}  // namespace

const DeviceConsts* device_consts(int device) {
    std::mutex& mu = g_consts_mu;
    std::map<int, DeviceConsts*>& m = g_consts;
    std::lock_guard<std::mutex> lk(mu);
    auto it = m.find(device);
    if (it != m.end()) return it->second;
    uint16_t g2l[256];
    int l2g[33];
    webp_gamma_tables(g2l, l2g);
    uint32_t hf[4 * 256];
    jpeg_huff_u32(hf);
    auto* dc = new DeviceConsts();
    (void)hipSetDevice(device);
    if (hipMalloc(&dc->gamma_to_lin, sizeof(g2l)) != hipSuccess ||
        hipMalloc(&dc->lin_to_gamma, sizeof(l2g)) != hipSuccess ||
        hipMalloc(&dc->jpeg_huff, sizeof(hf)) != hipSuccess ||
        hipMemcpy(dc->gamma_to_lin, g2l, sizeof(g2l), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dc->lin_to_gamma, l2g, sizeof(l2g), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dc->jpeg_huff, hf, sizeof(hf), hipMemcpyHostToDevice) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {  // order before non-blocking streams
        delete dc;
        return nullptr;
    }
    m[device] = dc;
    return dc;
}

// Run the device front end of encode_image and hand its output to the host
// entropy stage.  WebP: to_rgb8 + RGB->YUV420 on the GPU, libwebp VP8 coding of
// those planes on the host.  JPEG: to_rgb8 + YCbCr + FDCT + quantise on the GPU,
// baseline Huffman coding on the host.  AVIF: to_rgba8 + YCbCr 4:4:4 on the GPU,
// AV1 coding by libavif/aom on the host.
int encode_device_front(const uint8_t* dev, uint32_t w, uint32_t h, uint32_t c, size_t pitch, int fmt, int quality,
                        EncodePrep& p, std::vector<uint8_t>& out) {
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    p.fmt = fmt;
    p.q = q;
    p.w = w;
    p.h = h;
    p.done = true;  // unless a host coder is left to run (encode_host_back)
    hipStream_t s = thread_stream();
    if (!s) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    if (fmt == IK_FORMAT_WEBP) {
        if (w > 16383 || h > 16383) return fail(IK_ERR_TRANSFORM, "WebP dimensions %ux%u exceed 16383", w, h);
        const DeviceConsts* dc = device_consts(current_device());
        if (!dc) return fail(IK_ERR_DEVICE, "cannot upload WebP tables");
        const size_t uvw = (w + 1) / 2, uvh = (h + 1) / 2;
        const size_t bytes = (size_t)w * h + 2 * uvw * uvh;
        if (default_webp_encoder() == IK_WEBP_EXACT) {  // (read once: a concurrent switch cannot mix paths)
            uint8_t* dyuv = scratch(bytes);
            if (!dyuv) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
            hipError_t e = launch_webp_yuv420(dev, (int)w, (int)h, (int)c, pitch, 0, dyuv, 0, 1,
                                              dc->gamma_to_lin, dc->lin_to_gamma, s);
            if (e != hipSuccess) return hip_fail(e, "webp yuv420");
            std::vector<std::vector<uint8_t>> files;
            if (int rc = webp_encode_exact(dyuv, 0, 1, (int)w, (int)h, q, files)) return rc;
            out.swap(files[0]);
            return IK_OK;
        }
        // the colour kernel writes the planes straight into pinned host memory: no
        // copy-engine transfer, which would queue behind another batch's stream upload
        uint8_t* hp = pinned_slot(4, bytes);
        void* dhp = nullptr;
        if (!hp || hipHostGetDevicePointer(&dhp, hp, 0) != hipSuccess || !dhp)
            return fail(IK_ERR_NOMEM, "cannot map pinned WebP planes");
        hipError_t e = launch_webp_yuv420(dev, (int)w, (int)h, (int)c, pitch, 0, reinterpret_cast<uint8_t*>(dhp), 0, 1,
                                          dc->gamma_to_lin, dc->lin_to_gamma, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "webp yuv420");
        p.planes.assign(hp, hp + bytes);
        p.done = false;  // libwebp's VP8 coding of the planes: encode_host_back
        return IK_OK;
    }
    if (fmt == IK_FORMAT_JPEG) {
        if (w > 65535 || h > 65535) return fail(IK_ERR_TRANSFORM, "JPEG dimensions %ux%u exceed 65535", w, h);
        uint8_t qt[128];
        jpeg_quant_tables(q, qt);
        const size_t nmcu = (size_t)((w + 7) / 8) * ((h + 7) / 8);
        const size_t cbytes = nmcu * 3 * 64 * sizeof(int16_t);
        const DeviceConsts* dc = device_consts(current_device());
        if (!dc) return fail(IK_ERR_DEVICE, "cannot upload JPEG tables");
        // [qtables 256][coefficients][Huffman work: words + staging][stuffed stream][length]
        const size_t cap = jpeg_enc_cap((int)w, (int)h);
        const size_t c_off = 256, w_off = c_off + (cbytes + 255) / 256 * 256;
        const size_t o_off = w_off + 2 * cap, l_off = o_off + cap;
        uint8_t* dq = scratch(l_off + 256);
        if (!dq) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
        int16_t* dcoef = (int16_t*)(dq + c_off);
        int rc = copy_h2d_2d(dq, 128, qt, 128, 128, 1, s);
        if (rc) return rc;
        hipError_t e = launch_jpeg_coeffs(dev, (int)w, (int)h, (int)c, pitch, 0, dq, dcoef, 0, 1, s);
        if (e != hipSuccess) return hip_fail(e, "jpeg coefficients");
        JpegEncArgs a{};
        a.coef = dcoef;
        a.coef_img_stride = 0;
        a.nmcu = (int)nmcu;
        a.huff = dc->jpeg_huff;
        a.work = dq + w_off;
        a.work_img_bytes = 2 * cap;
        a.words_bytes = cap;
        a.out = dq + o_off;
        a.out_img_stride = cap;
        a.out_cap = cap;
        a.out_len = reinterpret_cast<uint32_t*>(dq + l_off);
        e = launch_jpeg_huff_enc(a, 1, s);
        if (e != hipSuccess) return hip_fail(e, "jpeg huffman");
        uint32_t len = 0;
        rc = copy_d2h_2d(reinterpret_cast<uint8_t*>(&len), 4, dq + l_off, 4, 4, 1, s);
        if (rc) return rc;
        if (len == 0xffffffffu) {  // does not fit the GPU coder's buffer: host coder
            std::vector<int16_t> coef(nmcu * 3 * 64);
            rc = copy_d2h_2d((uint8_t*)coef.data(), cbytes, (const uint8_t*)dcoef, cbytes, cbytes, 1, s);
            if (rc) return rc;
            jpeg_write(coef.data(), (int)w, (int)h, qt, out);
            return IK_OK;
        }
        jpeg_header((int)w, (int)h, qt, out);
        const size_t hdr = out.size();
        out.resize(hdr + len + 2);
        if (len) rc = copy_d2h_2d(out.data() + hdr, len, dq + o_off, len, len, 1, s);
        if (rc) return rc;
        out[hdr + len] = 0xFF;
        out[hdr + len + 1] = 0xD9;
        return IK_OK;
    }
    if (fmt == IK_FORMAT_AVIF) {
        // image 0.25.8 AvifEncoder::new_with_speed_quality(out, 4, q) (src/transform.rs:140-145)
        const size_t n = (size_t)w * h;
        uint8_t* dp = scratch(4 * n + 256);
        if (!dp) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
        int* dflag = reinterpret_cast<int*>(dp + 4 * n + 128 - ((4 * n) & 127));
        hipError_t e = launch_avif_yuv444(dev, (int)w, (int)h, (int)c, pitch, 0, dp, 0, dflag, 1, s);
        if (e != hipSuccess) return hip_fail(e, "avif yuv444");
        p.planes.resize(4 * n);
        int transparent = 0;
        int rc = copy_d2h_2d(p.planes.data(), 4 * n, dp, 4 * n, 4 * n, 1, s);
        if (!rc) rc = copy_d2h_2d(reinterpret_cast<uint8_t*>(&transparent), 4, reinterpret_cast<const uint8_t*>(dflag), 4, 4, 1, s);
        if (rc) return rc;
        p.transparent = transparent != 0;
        p.done = false;  // AV1 coding by libavif: encode_host_back
        return IK_OK;
    }
    return fail(IK_ERR_INVALID, "unknown ImageFormat %d", fmt);
}

int encode_host_back(EncodePrep& p, std::vector<uint8_t>& out) {
    if (p.done) return IK_OK;
    p.done = true;
    if (p.fmt == IK_FORMAT_WEBP) {
        const size_t uvw = (p.w + 1) / 2, uvh = (p.h + 1) / 2;
        const uint8_t* Y = p.plane_data();
        return webp_encode_yuv420(Y, Y + (size_t)p.w * p.h, Y + (size_t)p.w * p.h + uvw * uvh, (int)p.w, (int)p.h,
                                  (float)p.q, out);
    }
    if (p.fmt == IK_FORMAT_AVIF) return avif_encode_yuv444(p.plane_data(), p.transparent, (int)p.w, (int)p.h, p.q, 4, out);
    return fail(IK_ERR_INVALID, "unknown ImageFormat %d", p.fmt);
}

int encode_device_image(const uint8_t* dev, uint32_t w, uint32_t h, uint32_t c, size_t pitch, int fmt, int quality,
                        std::vector<uint8_t>& out) {
    EncodePrep p;
    const int rc = encode_device_front(dev, w, h, c, pitch, fmt, quality, p, out);
    return rc ? rc : encode_host_back(p, out);
}

// the front half of ik_encode on a handle (u16 images are rescaled to u8 first,
// as to_rgb8 / to_rgba8 do)
int encode_image_front(const ik_image* img, int fmt, int quality, EncodePrep& p, std::vector<uint8_t>& out) {
    if (!img) return fail(IK_ERR_INVALID, "null pointer");
    if (img->w == 0 || img->h == 0) return fail(IK_ERR_TRANSFORM, "cannot encode an empty image");
    DeviceGuard g(img->device);
    if (img->depth != 2) return encode_device_front(img->d, img->w, img->h, img->c, img->pitch, fmt, quality, p, out);
    ik_image* u8 = nullptr;
    int st = alloc_image(img->w, img->h, img->c, &u8);
    if (st) return st;
    hipError_t e = launch_u16_to_u8(img->d, img->pitch, u8->d, u8->pitch, (int)(img->w * img->c), (int)img->h,
                                    thread_stream());
    st = e == hipSuccess ? encode_device_front(u8->d, u8->w, u8->h, u8->c, u8->pitch, fmt, quality, p, out)
                         : hip_fail(e, "u16 -> u8");
    if (e == hipSuccess && !st) (void)hipStreamSynchronize(thread_stream());  // u8 is read before it is freed
    ik_image_free(u8);
    return st;
}

}  // namespace ik

using namespace ik;

extern "C" {

const char* ik_version(void) { return "imagekit-hip 0.1.0 (gfx950)"; }

int ik_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(IK_ERR_INVALID, "null pointer");
    *out = nullptr;
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable);
    if (e != hipSuccess) return fail(IK_ERR_NOMEM, "hipHostMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pins[(uintptr_t)p] = PinnedRange{bytes, true};
    *out = p;
    return IK_OK;
}

int ik_host_free(void* p) {
    if (!p) return IK_OK;
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pins.find((uintptr_t)p);
        if (it == g_pins.end() || !it->second.owned) return fail(IK_ERR_INVALID, "not an ik_host_alloc pointer");
        g_pins.erase(it);
    }
    IK_HIP(hipHostFree(p));
    return IK_OK;
}

int ik_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return fail(IK_ERR_INVALID, "empty range");
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pins.upper_bound((uintptr_t)p + bytes - 1);
        if (it != g_pins.begin()) {
            --it;
            if (it->first + it->second.n > (uintptr_t)p) return fail(IK_ERR_INVALID, "range overlaps a pinned range");
        }
    }
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
    if (e != hipSuccess) return fail(IK_ERR_NOMEM, "hipHostRegister(%zu bytes): %s", bytes, hipGetErrorString(e));
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pins[(uintptr_t)p] = PinnedRange{bytes, false};
    return IK_OK;
}

int ik_host_unregister(void* p) {
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pins.find((uintptr_t)p);
        if (it == g_pins.end() || it->second.owned) return fail(IK_ERR_INVALID, "not an ik_host_register range");
        g_pins.erase(it);
    }
    IK_HIP(hipHostUnregister(p));
    return IK_OK;
}

size_t ik_last_error(char* buf, size_t cap) {
    const std::string& e = t_err;
    if (buf && cap) {
        size_t n = e.size() < cap - 1 ? e.size() : cap - 1;
        std::memcpy(buf, e.data(), n);
        buf[n] = 0;
    }
    return e.size();
}

int ik_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// How host threads wait for the GPU.  HIP's default (hipDeviceScheduleAuto) spins
// the waiting thread on the CPU; the batch paths have several threads waiting on
// device work at once (stage threads, lane checks) while the host coders (libwebp)
// need every core of the quota, so the library asks for blocking waits
// (hipDeviceScheduleBlockingSync: the thread sleeps until the GPU signals).
// IK_SYNC=spin keeps the spinning.  Applied once per visible device, process-wide.
static void apply_sync_mode(int ndev) {
    static std::once_flag once;
    std::call_once(once, [ndev] {
        const char* e = getenv("IK_SYNC");
        if (e && !strcmp(e, "spin")) return;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) cur = 0;
        for (int d = 0; d < ndev; ++d) {
            if (hipSetDevice(d) != hipSuccess) continue;
            const hipError_t r = hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
            if (r != hipSuccess && getenv("IK_TIMING"))
                fprintf(stderr, "[init] device %d: blocking sync not set (%s)\n", d, hipGetErrorString(r));
        }
        (void)hipSetDevice(cur);
    });
}

int ik_init(int device) {
    IK_API_ENTER();
    int n = 0;
    IK_HIP(hipGetDeviceCount(&n));
    apply_sync_mode(n);
    if (device >= n) return fail(IK_ERR_INVALID, "device %d out of range (%d devices)", device, n);
    if (device < 0) {  // every visible GPU (or IK_DEVICES): one process, many devices
        if (int rc = sched_configure(nullptr, 0)) return rc;
        device = sched_phys(0);
    }
    t_device = device;
    IK_HIP(hipSetDevice(current_device()));
    if (!thread_stream()) return fail(IK_ERR_DEVICE, "cannot create HIP stream");
    return IK_OK;
}

int ik_init_devices(const int* devices, int n) {
    IK_API_ENTER();
    if (!devices || n <= 0) return fail(IK_ERR_INVALID, "empty device list");
    if (int rc = sched_configure(devices, n)) return rc;
    return ik_init(sched_phys(0));
}

int ik_logical_device_count(void) { return sched_multi() ? sched_count() : 0; }

int ik_logical_device_stats(uint32_t logical, uint64_t* jobs, uint64_t* cost_done, uint64_t* outstanding) {
    IK_API_ENTER();
    if (!sched_multi()) return fail(IK_ERR_INVALID, "multi-device dispatch is not enabled");
    return sched_stats(logical, jobs, cost_done, outstanding);
}

uint64_t ik_request_cost(const uint8_t* bytes, size_t len, int64_t w, int64_t h, int fmt) {
    return request_cost(bytes, len, w, h, fmt);
}

void ik_schedule_plan(const uint64_t* costs, uint32_t n, uint32_t ndev, const uint64_t* outstanding,
                      uint32_t* assign) {
    if (!costs || !assign || !ndev) return;
    sched_plan(costs, n, ndev, outstanding, assign);
}

uint32_t ik_schedule_split(const uint64_t* costs, uint32_t n, uint32_t ndev, const uint64_t* outstanding,
                           uint32_t min_batch, uint32_t* part_lo, uint32_t* part_dev) {
    if (!costs || !part_lo || !part_dev || !ndev) return 0;
    std::vector<uint64_t> out(ndev, 0);
    if (outstanding) std::copy(outstanding, outstanding + ndev, out.begin());
    return sched_split(costs, n, ndev, min_batch, out.data(), part_lo, part_dev);
}

int ik_image_from_host(const uint8_t* pixels, uint32_t width, uint32_t height, uint32_t channels,
                       ik_image** out) {
    IK_API_ENTER();
    if (!out || (!pixels && width && height)) return fail(IK_ERR_INVALID, "null pointer");
    if (channels < 1 || channels > 4) return fail(IK_ERR_INVALID, "channels must be 1..4");
    ik_image* img = nullptr;
    int st = alloc_image(width, height, channels, &img);
    if (st) return st;
    if (width && height) {
        const size_t row = (size_t)width * channels;
        int rc = copy_h2d_2d(img->d, img->pitch, pixels, row, row, height, thread_stream());
        if (rc) { ik_image_free(img); return rc; }
    }
    *out = img;
    return IK_OK;
}

int ik_image_from_host16(const uint16_t* pixels, uint32_t width, uint32_t height, uint32_t channels,
                         ik_image** out) {
    IK_API_ENTER();
    if (!out || (!pixels && width && height)) return fail(IK_ERR_INVALID, "null pointer");
    if (channels < 1 || channels > 4) return fail(IK_ERR_INVALID, "channels must be 1..4");
    ik_image* img = nullptr;
    int st = alloc_image(width, height, channels, &img, 2);
    if (st) return st;
    if (width && height) {
        const size_t row = (size_t)width * channels * 2;
        int rc = copy_h2d_2d(img->d, img->pitch, reinterpret_cast<const uint8_t*>(pixels), row, row, height,
                             thread_stream());
        if (rc) { ik_image_free(img); return rc; }
    }
    *out = img;
    return IK_OK;
}

int ik_image_depth(const ik_image* img) { return img ? (int)img->depth : 0; }

int ik_image_wrap_device(uint8_t* dev_pixels, uint32_t width, uint32_t height, uint32_t channels,
                         size_t pitch, ik_image** out) {
    IK_API_ENTER();
    if (!out || !dev_pixels) return fail(IK_ERR_INVALID, "null pointer");
    if (channels < 1 || channels > 4) return fail(IK_ERR_INVALID, "channels must be 1..4");
    if (pitch < (size_t)width * channels) return fail(IK_ERR_INVALID, "pitch smaller than a row");
    auto* img = new ik_image();
    img->w = width; img->h = height; img->c = channels; img->pitch = pitch;
    img->d = dev_pixels; img->owned = false; img->device = current_device();
    *out = img;
    return IK_OK;
}

int ik_image_info(const ik_image* img, uint32_t* w, uint32_t* h, uint32_t* c) {
    if (!img) return fail(IK_ERR_INVALID, "null image");
    if (w) *w = img->w;
    if (h) *h = img->h;
    if (c) *c = img->c;
    return IK_OK;
}

int ik_image_to_host(const ik_image* img, uint8_t* dst, size_t cap) {
    IK_API_ENTER();
    if (!img || !dst) return fail(IK_ERR_INVALID, "null pointer");
    const size_t row = (size_t)img->w * img->c * img->depth;
    if (cap < row * img->h) return fail(IK_ERR_INVALID, "destination too small");
    if (!row || !img->h) return IK_OK;
    DeviceGuard g(img->device);
    return copy_d2h_2d(dst, row, img->d, img->pitch, row, img->h, thread_stream());
}

void ik_image_free(ik_image* img) {
    IK_API_ENTER_VOID();
    if (!img) return;
    if (img->owned && img->d) {
        ImagePool& pool = image_pool(img->device);
        bool kept = false;
        if (img->block) {
            mem_stat(kMemImageLive, -(int64_t)img->block);
            std::lock_guard<std::mutex> lk(pool.mu);
            if (pool.held + img->block <= kPoolBytes) {
                pool.free_blocks.emplace(img->block, img->d);
                pool.held += img->block;
                kept = true;
                mem_stat(kMemImageFree, (int64_t)img->block);
            }
        }
        if (!kept) {
            DeviceGuard g(img->device);
            (void)hipFree(img->d);
        }
    }
    delete img;
}

void ik_buf_free(uint8_t* buf) { free(buf); }

// imageops::resize(image, nw, nh, filter)
int ik_resize_exact(const ik_image* img, uint32_t nw, uint32_t nh, int filter, ik_image** out) {
    IK_API_ENTER();
    if (!img || !out) return fail(IK_ERR_INVALID, "null pointer");
    if (filter < 0 || filter > 4) return fail(IK_ERR_INVALID, "unknown filter %d", filter);
    if (nw == 0 || nh == 0) return fail(IK_ERR_INVALID, "zero output dimension");
    DeviceGuard g(img->device);
    ik_image* o = nullptr;
    int st = alloc_image(nw, nh, img->c, &o, img->depth);
    if (st) return st;
    hipStream_t s = thread_stream();
    const size_t orow = (size_t)nw * img->c * img->depth;
    if (img->w == 0 || img->h == 0) {  // "nothing to sample from": blank image
        hipError_t e = hipMemset2DAsync(o->d, o->pitch, 0, orow, nh, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { ik_image_free(o); return hip_fail(e, "blank image"); }
        *out = o;
        return IK_OK;
    }
    if (nw == img->w && nh == img->h) {  // copy instead of resampling
        hipError_t e = hipMemcpy2DAsync(o->d, o->pitch, img->d, img->pitch, orow, nh, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { ik_image_free(o); return hip_fail(e, "copy image"); }
        *out = o;
        return IK_OK;
    }
    int rc;
    if (img->depth == 2) {  // 16-bit: the two-pass path over u16 samples
        ResizePlan* plan = get_resize_plan(current_device(), (int)img->w, (int)img->h, (int)img->c, (int)nw, (int)nh,
                                           filter, 1);
        float* tmp = plan ? (float*)scratch(sizeof(float) * (size_t)nh * img->w * img->c) : nullptr;
        if (!plan || !tmp) rc = fail(IK_ERR_DEVICE, "cannot set up the 16-bit resize");
        else {
            hipError_t e = launch_resize16(*plan, img->d, img->pitch, o->d, o->pitch, tmp, s);
            rc = e == hipSuccess ? IK_OK : hip_fail(e, "resize (16-bit)");
        }
    } else {
        rc = ik_resize_batch_device(img->d, img->w, img->h, img->c, img->pitch, 0, 1, nw, nh, filter,
                                    o->d, o->pitch, 0, s);
    }
    if (rc == IK_OK) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "resize");
    }
    if (rc) { ik_image_free(o); return rc; }
    *out = o;
    return IK_OK;
}

static uint32_t f32_as_u32(float v) {
    if (!(v > 0.0f)) return 0;
    if (v >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

}  // extern "C"

namespace ik {

// The output size of src/transform.rs:62-90 + DynamicImage::resize for a w x h
// image and the request's (w, h) options (-1 = None; not both None)
int resize_target(uint32_t W, uint32_t H, int64_t w, int64_t h, uint32_t* onw, uint32_t* onh) {
    if (w > 0xFFFFFFFFll || h > 0xFFFFFFFFll) return fail(IK_ERR_INVALID, "dimension exceeds u32");
    uint32_t tw, th;
    if (w >= 0) tw = (uint32_t)w;
    else tw = f32_as_u32(roundf((float)W * ((float)(uint32_t)h / (float)H)));
    if (h >= 0) th = (uint32_t)h;
    else th = f32_as_u32(roundf((float)H * ((float)(uint32_t)w / (float)W)));
    if (tw < 1) tw = 1;
    if (th < 1) th = 1;
    uint32_t nw = tw, nh = th;
    if (!(tw == W && th == H)) {
        const double wr = (double)tw / (double)W, hr = (double)th / (double)H;
        const double r = wr < hr ? wr : hr;
        double fw = std::round((double)W * r), fh = std::round((double)H * r);
        unsigned long long rw = fw < 1 ? 1 : (unsigned long long)fw;
        unsigned long long rh = fh < 1 ? 1 : (unsigned long long)fh;
        if (rw > 0xFFFFFFFFull || rh > 0xFFFFFFFFull) return fail(IK_ERR_INVALID, "dimension overflow");
        nw = (uint32_t)rw; nh = (uint32_t)rh;
    }
    *onw = nw;
    *onh = nh;
    return IK_OK;
}

// encode_image's device front end for n same-geometry 8-bit images going to WebP
// through libwebp: ONE colour-conversion launch over per-image base pointers,
// writing every image's YUV420 planes straight into pinned host memory; prep[i]
// gets the planes for encode_host_back.  Returns IK_ERR_UNSUPPORTED (nothing
// done) when the per-image path applies instead (the GPU VP8 encoder, > 16383).
// Page-locked blocks shared by the requests of a batched colour launch: a pool of
// free blocks (process-wide); a block goes back when its last holder drops it.
// Best fit (the smallest free block that holds the request, at most twice its
// size, so a small group does not take the block a large one needs), and at most
// kPinnedPoolBytes kept: a block returned past that goes back to the runtime.
namespace {
constexpr size_t kPinnedPoolBytes = size_t(2) << 30;
std::mutex g_pblk_mu;
std::multimap<size_t, uint8_t*> g_pblk_free;  // capacity -> block
size_t g_pblk_held = 0;
}  // namespace
static std::shared_ptr<uint8_t> pinned_block(size_t bytes) {
    uint8_t* p = nullptr;
    size_t cap = 0;
    {
        std::lock_guard<std::mutex> lk(g_pblk_mu);
        auto it = g_pblk_free.lower_bound(bytes);
        if (it != g_pblk_free.end() && it->first <= 2 * bytes) {
            cap = it->first;
            p = it->second;
            g_pblk_held -= cap;
            g_pblk_free.erase(it);
        }
    }
    if (!p) {
        cap = bytes;
        if (hipHostMalloc((void**)&p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    }
    return std::shared_ptr<uint8_t>(p, [cap](uint8_t* q) {
        {
            std::lock_guard<std::mutex> lk(g_pblk_mu);
            if (g_pblk_held + cap <= kPinnedPoolBytes) {
                g_pblk_free.emplace(cap, q);
                g_pblk_held += cap;
                return;
            }
        }
        (void)hipHostFree(q);
    });
}

// The exact coder for a same-geometry group (IK_WEBP_EXACT): one batched colour launch
// into device memory, then the whole group through webp_encode_exact -- the files
// are final, no host coder runs.
static int webp_exact_group(const std::vector<ik_image*>& imgs, int quality, std::vector<std::vector<uint8_t>*>& outs) {
    const size_t n = imgs.size();
    const ik_image* i0 = imgs[0];
    DeviceGuard g(i0->device);
    const DeviceConsts* dc = device_consts(current_device());
    if (!dc) return fail(IK_ERR_DEVICE, "cannot upload WebP tables");
    const uint32_t w = i0->w, h = i0->h;
    const size_t uvw = (w + 1) / 2, uvh = (h + 1) / 2, bytes = (size_t)w * h + 2 * uvw * uvh;
    const size_t stride = (bytes + 255) & ~size_t(255);
    hipStream_t s = thread_stream();
    uint8_t* dyuv = scratch(stride * n + 16 * n + 256);
    if (!dyuv) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
    std::vector<uint64_t> htab(n);
    for (size_t i = 0; i < n; ++i) htab[i] = (uint64_t)(uintptr_t)imgs[i]->d;
    uint64_t* dtab = reinterpret_cast<uint64_t*>(dyuv + stride * n);
    hipError_t e = hipMemcpyAsync(dtab, htab.data(), 8 * n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = launch_webp_yuv420(nullptr, (int)w, (int)h, (int)i0->c, i0->pitch, 0, dyuv, stride, (int)n,
                               dc->gamma_to_lin, dc->lin_to_gamma, s, dtab);
    if (e != hipSuccess) return hip_fail(e, "webp yuv420 (exact group)");
    std::vector<std::vector<uint8_t>> files;
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    if (int rc = webp_encode_exact(dyuv, stride, (int)n, (int)w, (int)h, q, files)) return rc;
    for (size_t i = 0; i < n; ++i) outs[i]->swap(files[i]);
    return IK_OK;
}

int webp_front_group(const std::vector<ik_image*>& imgs, int quality, std::vector<EncodePrep*>& prep) {
    const size_t n = imgs.size();
    if (!n) return IK_OK;
    const ik_image* i0 = imgs[0];
    if (i0->w > 16383 || i0->h > 16383 || i0->depth != 1)  // (the caller chose the libwebp coder)
        return IK_ERR_UNSUPPORTED;
    DeviceGuard g(i0->device);
    const DeviceConsts* dc = device_consts(current_device());
    if (!dc) return fail(IK_ERR_DEVICE, "cannot upload WebP tables");
    const uint32_t w = i0->w, h = i0->h;
    const size_t uvw = (w + 1) / 2, uvh = (h + 1) / 2, bytes = (size_t)w * h + 2 * uvw * uvh;
    const size_t stride = (bytes + 255) & ~size_t(255);
    std::shared_ptr<uint8_t> blk = pinned_block(stride * n + 16 * n + 256);
    uint8_t* hp = blk.get();
    void* dhp = nullptr;
    if (!hp || hipHostGetDevicePointer(&dhp, hp, 0) != hipSuccess || !dhp)
        return fail(IK_ERR_NOMEM, "cannot map pinned WebP planes");
    uint64_t* dtab = reinterpret_cast<uint64_t*>(scratch_slot(3, sizeof(uint64_t) * n));
    if (!dtab) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
    hipStream_t s = thread_stream();
    (void)hipStreamSynchronize(s);  // nothing pending reads the pinned area
    uint64_t* htab = reinterpret_cast<uint64_t*>(hp + stride * n);
    for (size_t i = 0; i < n; ++i) htab[i] = (uint64_t)(uintptr_t)imgs[i]->d;
    hipError_t e = launch_copy_words(reinterpret_cast<const uint32_t*>(reinterpret_cast<uint8_t*>(dhp) + stride * n),
                                     reinterpret_cast<uint32_t*>(dtab), 2 * n, s);
    if (e == hipSuccess)
        e = launch_webp_yuv420(nullptr, (int)w, (int)h, (int)i0->c, i0->pitch, 0, reinterpret_cast<uint8_t*>(dhp), stride,
                               (int)n, dc->gamma_to_lin, dc->lin_to_gamma, s, dtab);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "webp yuv420 (batched)");
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    for (size_t i = 0; i < n; ++i) {
        EncodePrep& p = *prep[i];
        p.fmt = IK_FORMAT_WEBP;
        p.q = q;
        p.w = w;
        p.h = h;
        p.pin_block = blk;
        p.pin_planes = hp + stride * i;
        p.done = false;
    }
    return IK_OK;
}

// imageops::resize over n 8-bit images of one geometry (same W, H, C, pitch) in
// ONE fused launch: the kernel reads each image's base pointer from a table, so
// the images may sit anywhere.  Same arithmetic as ik_resize_exact, per image.
// Returns IK_ERR_UNSUPPORTED (nothing allocated) when the geometry needs the
// two-kernel fallback; the caller then resizes image by image.
// encode_image's JPEG branch for a group of same-size 8-bit images (one quality),
// batched: one coefficient launch (to_rgb8 + YCbCr + FDCT + quantise) and one
// Huffman launch over all of them, writing the stuffed streams and their lengths
// straight into pinned host memory -- instead of a launch pair and two blocking
// copies per image, which serialised 256 small launches per configs[2] batch.
// Images whose stream does not fit the GPU coder's buffer are coded by the
// single-image path (its host fallback).  out[i] gets the finished JPEG bytes.
int jpeg_front_group(const std::vector<ik_image*>& imgs, int quality, std::vector<std::vector<uint8_t>*>& out) {
    const size_t n = imgs.size();
    if (!n) return IK_OK;
    const ik_image* i0 = imgs[0];
    if (i0->w > 65535 || i0->h > 65535 || i0->depth != 1) return IK_ERR_UNSUPPORTED;
    DeviceGuard g(i0->device);
    const DeviceConsts* dc = device_consts(current_device());
    if (!dc) return fail(IK_ERR_DEVICE, "cannot upload JPEG tables");
    const int q = quality < 1 ? 1 : (quality > 100 ? 100 : quality);
    const uint32_t w = i0->w, h = i0->h;
    uint8_t qt[128];
    jpeg_quant_tables(q, qt);
    std::vector<uint8_t> hdr;
    jpeg_header((int)w, (int)h, qt, hdr);
    const size_t nmcu = (size_t)((w + 7) / 8) * ((h + 7) / 8);
    const size_t cimg = ((nmcu * 3 * 64 * sizeof(int16_t)) + 255) & ~size_t(255);  // coefficients per image
    const size_t cap = jpeg_enc_cap((int)w, (int)h);
    hipStream_t s = thread_stream();
    // sub-batches bound the device and pinned memory (2 cap + coefficients per image)
    constexpr size_t kSub = 64;
    for (size_t b0 = 0; b0 < n; b0 += kSub) {
        const size_t m = std::min(kSub, n - b0);
        // device: [qt 256][src table][coefficients][Huffman work]; pinned: [streams][lengths][qt + table staging]
        const size_t o_tab = 256, o_coef = o_tab + ((sizeof(uint64_t) * m + 255) & ~size_t(255));
        const size_t o_work = o_coef + cimg * m;
        uint8_t* dv = scratch_slot(4, o_work + 2 * cap * m);
        const size_t p_len = cap * m, p_stage = p_len + ((sizeof(uint32_t) * m + 255) & ~size_t(255));
        uint8_t* hp = pinned_slot(5, p_stage + 256 + sizeof(uint64_t) * m);
        void* dhp = nullptr;
        if (!dv || !hp || hipHostGetDevicePointer(&dhp, hp, 0) != hipSuccess || !dhp)
            return fail(IK_ERR_NOMEM, "cannot allocate the batched JPEG encoder's buffers");
        uint8_t* dh = reinterpret_cast<uint8_t*>(dhp);
        (void)hipStreamSynchronize(s);  // nothing pending reads the pinned area
        std::memcpy(hp + p_stage, qt, 128);
        uint64_t* htab = reinterpret_cast<uint64_t*>(hp + p_stage + 256);
        for (size_t i = 0; i < m; ++i) htab[i] = (uint64_t)(uintptr_t)imgs[b0 + i]->d;
        EvPair& ev = thread_events(1);
        hipError_t e = launch_copy_words(reinterpret_cast<const uint32_t*>(dh + p_stage), reinterpret_cast<uint32_t*>(dv),
                                         32, s);
        if (e == hipSuccess) ev_record(ev.a, s);
        if (e == hipSuccess)
            e = launch_copy_words(reinterpret_cast<const uint32_t*>(dh + p_stage + 256),
                                  reinterpret_cast<uint32_t*>(dv + o_tab), 2 * m, s);
        if (e == hipSuccess)
            e = launch_jpeg_coeffs(nullptr, (int)w, (int)h, (int)i0->c, i0->pitch, 0, dv,
                                   reinterpret_cast<int16_t*>(dv + o_coef), cimg / sizeof(int16_t), (int)m, s,
                                   reinterpret_cast<const uint64_t*>(dv + o_tab));
        if (e == hipSuccess) {
            JpegEncArgs a{};
            a.coef = reinterpret_cast<const int16_t*>(dv + o_coef);
            a.coef_img_stride = cimg / sizeof(int16_t);
            a.nmcu = (int)nmcu;
            a.huff = dc->jpeg_huff;
            a.work = dv + o_work;
            a.work_img_bytes = 2 * cap;
            a.words_bytes = cap;
            a.out = dh;
            a.out_img_stride = cap;
            a.out_cap = cap;
            a.out_len = reinterpret_cast<uint32_t*>(dh + p_len);
            e = launch_jpeg_huff_enc(a, (int)m, s);
        }
        if (e == hipSuccess) ev_record(ev.b, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "jpeg encode (batched)");
        batch_timing_add(current_device(), kBtJpegEncMs, ev_pair_ms(ev));
        batch_timing_add(current_device(), kBtJpegEncImages, (double)m);
        const uint32_t* lens = reinterpret_cast<const uint32_t*>(hp + p_len);
        for (size_t i = 0; i < m; ++i) {
            std::vector<uint8_t>& o = *out[b0 + i];
            if (lens[i] == 0xffffffffu) {  // past the GPU coder's buffer: the single-image path (host coder)
                EncodePrep pp;
                if (int rc = encode_device_front(imgs[b0 + i]->d, w, h, i0->c, i0->pitch, IK_FORMAT_JPEG, q, pp, o))
                    return rc;
                continue;
            }
            o.assign(hdr.begin(), hdr.end());
            o.insert(o.end(), hp + cap * i, hp + cap * i + lens[i]);
            o.push_back(0xFF);
            o.push_back(0xD9);
        }
    }
    return IK_OK;
}

int resize_group(const std::vector<ik_image*>& src, uint32_t nw, uint32_t nh, int filter, std::vector<ik_image*>& out) {
    const size_t n = src.size();
    out.assign(n, nullptr);
    if (!n) return IK_OK;
    const ik_image* s0 = src[0];
    DeviceGuard g(s0->device);
    ResizePlan* plan = get_resize_plan(current_device(), (int)s0->w, (int)s0->h, (int)s0->c, (int)nw, (int)nh, filter,
                                       (int)n);
    if (!plan) return fail(IK_ERR_DEVICE, "cannot build resize plan");
    if (plan->slots == 0 || !resize_fused_fits(s0->pitch, s0->h) || (s0->pitch & 7)) return IK_ERR_UNSUPPORTED;
    std::vector<uint64_t> tab(2 * n);
    for (size_t i = 0; i < n; ++i) {
        const int st = alloc_image(nw, nh, s0->c, &out[i]);
        if (st) {
            for (ik_image*& o : out) { ik_image_free(o); o = nullptr; }
            return st;
        }
        tab[i] = (uint64_t)(uintptr_t)src[i]->d;
        tab[n + i] = (uint64_t)(uintptr_t)out[i]->d;
    }
    hipStream_t s = thread_stream();
    uint64_t* dtab = reinterpret_cast<uint64_t*>(scratch_slot(3, sizeof(uint64_t) * 2 * n));
    // the pointer table goes up through a copy kernel reading pinned memory (a
    // copy-engine transfer would queue behind another batch's stream upload)
    uint8_t* ht = pinned_slot(5, 16 * n);
    void* dht = nullptr;
    int rc = IK_OK;
    if (!dtab) rc = fail(IK_ERR_DEVICE, "cannot allocate device scratch");
    else if (!ht || hipHostGetDevicePointer(&dht, ht, 0) != hipSuccess || !dht)
        rc = fail(IK_ERR_NOMEM, "cannot map pinned resize table");
    if (!rc) {
        (void)hipStreamSynchronize(s);  // the previous table is read
        std::memcpy(ht, tab.data(), 16 * n);
        const hipError_t e = launch_copy_words(reinterpret_cast<const uint32_t*>(dht), reinterpret_cast<uint32_t*>(dtab),
                                               4 * n, s);
        if (e != hipSuccess) rc = hip_fail(e, "resize table upload");
    }
    if (!rc) {
        EvPair& ev = thread_events(0);
        ev_record(ev.a, s);
        hipError_t e = launch_resize(*plan, nullptr, s0->pitch, 0, nullptr, out[0]->pitch, 0, (int)n, nullptr, s, dtab,
                                     dtab + n);
        if (e == hipSuccess) ev_record(ev.b, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "resize (batched)");
        if (!rc) {
            const int d = current_device();
            batch_timing_add(d, kBtResizeMs, ev_pair_ms(ev));
            batch_timing_add(d, kBtResizeBytes, (double)n * s0->c * ((double)s0->w * s0->h + (double)nw * nh));
            batch_timing_add(d, kBtResizeImages, (double)n);
        }
    }
    if (rc)
        for (ik_image*& o : out) { ik_image_free(o); o = nullptr; }
    return rc;
}

}  // namespace ik

extern "C" {

// src/transform.rs:62-90 then DynamicImage::resize (image 0.25.8):
// (nw,nh) == dims -> clone; else resize_dimensions(..., fill=false) (aspect FIT,
// f64, round, max 1) -> imageops::resize.
int ik_resize(ik_image* img, int64_t w, int64_t h, int filter, ik_image** out) {
    IK_API_ENTER();
    if (!img || !out) return fail(IK_ERR_INVALID, "null pointer");
    if (w < 0 && h < 0) { *out = img; return IK_OK; }
    uint32_t nw, nh;
    const int st = resize_target(img->w, img->h, w, h, &nw, &nh);
    if (st) return st;
    return ik_resize_exact(img, nw, nh, filter, out);
}

int ik_encode(const ik_image* img, int fmt, int quality, uint8_t** out, size_t* out_len) {
    IK_API_ENTER();
    if (!img || !out || !out_len) return fail(IK_ERR_INVALID, "null pointer");
    std::vector<uint8_t> bytes;
    EncodePrep prep;
    int st = encode_image_front(img, fmt, quality, prep, bytes);
    if (!st) st = encode_host_back(prep, bytes);
    if (st) return st;
    *out = (uint8_t*)malloc(bytes.size() ? bytes.size() : 1);
    if (!*out) return fail(IK_ERR_NOMEM, "out of host memory");
    std::memcpy(*out, bytes.data(), bytes.size());
    *out_len = bytes.size();
    return IK_OK;
}

}  // extern "C"

namespace ik {

// decode_image: image::guess_format + load_from_memory_with_format; formats the
// reference build compiles in (Cargo.toml:20: jpeg, png, webp; avif = encoder only)
static int decode_one(const uint8_t* bytes, size_t len, ik_image** out, int* fmt_out) {
    if (!out) return fail(IK_ERR_INVALID, "null pointer");
    if (!bytes && len) return fail(IK_ERR_INVALID, "null bytes");
    const Sniffed f = guess_format(bytes, len);
    if (f == Sniffed::Unknown) return fail(IK_ERR_TRANSFORM, "The image format could not be determined");
    uint32_t w = 0, h = 0, c = 0;
    // host-decoded pixels: a per-thread buffer (with the PNG decoder's own it
    // trades places, so neither is page-faulted in again per image); released
    // after images over 128 MiB
    thread_local std::vector<uint8_t> px;
    struct Trim {
        ~Trim() { if (px.capacity() > (128u << 20)) std::vector<uint8_t>().swap(px); }
    } trim;
    int st;
    ik_image* img = nullptr;
    switch (f) {
    case Sniffed::Png: {  // GPU inflate + unfilter when the stream allows, else the host decoder
        std::string msg;
        const uint8_t* const bp[1] = {bytes};
        st = decode_png_batch(bp, &len, 1, &img, &st, &msg);
        if (st) return fail(st, "%s", msg.c_str());
        break;
    }
    case Sniffed::Jpeg: st = decode_jpeg_device(bytes, len, &img); break;
    case Sniffed::WebP:  // lossy on the GPU when it covers the file, else libwebp on the host
        st = decode_webp_device(bytes, len, &img);
        if (st == kVp8dHost) {
            if (webp_decode_mode() == 2)
                return fail(IK_ERR_TRANSFORM, "IK_WEBP_DECODE=gpu: the GPU WebP decoder leaves this file to libwebp");
            st = decode_webp(bytes, len, w, h, c, px);
        }
        break;
    default:
        return fail(IK_ERR_TRANSFORM, "The image format %s is not supported", format_name(f));
    }
    if (st) return st;
    if (!img) {
        st = ik_image_from_host(px.data(), w, h, c, &img);
        if (st) return st;
    }
    *out = img;
    if (fmt_out) {
        *fmt_out = f == Sniffed::WebP ? IK_FORMAT_WEBP
                 : f == Sniffed::Jpeg ? IK_FORMAT_JPEG
                 : f == Sniffed::Avif ? IK_FORMAT_AVIF : -1;
    }
    return IK_OK;
}

static std::string last_error_str() { return t_err; }

// decode_image over a batch on the calling thread's device; per-item status and
// message (the decoder's own, as TransformError(e.to_string()) carries it).  up:
// the batch's PNG streams' upload, already issued (png_upload_begin), or null
// sniff: null, or a host copy of each item's first bytes (sniff_len(i) of them) when
// bytes holds device addresses for the PNG items (device-resident inputs: every
// other item is a host copy already)
static size_t sniff_len(const uint8_t* const* sniff, const uint8_t* const* bytes, const size_t* lens, uint32_t i) {
    return sniff && sniff[i] != bytes[i] ? std::min<size_t>(lens[i], 64) : lens[i];
}

int decode_batch_dev(const uint8_t* const* bytes, const size_t* lens, uint32_t n, ik_image** outs, int* fmts,
                     int* st, std::string* msg, int threads, PngUpload* up = nullptr,
                     const uint8_t* const* sniff = nullptr, const JpegUpload* jup = nullptr) {
    std::vector<const uint8_t*> jb, pb, ph;
    std::vector<size_t> jl, pl;
    std::vector<uint32_t> ji, pi, other;
    for (uint32_t i = 0; i < n; ++i) {
        outs[i] = nullptr;
        st[i] = IK_OK;
        if (fmts) fmts[i] = -1;
        if (!bytes[i] && lens[i]) { st[i] = fail(IK_ERR_INVALID, "null bytes"); msg[i] = t_err; continue; }
        const Sniffed f = guess_format(sniff ? sniff[i] : bytes[i], sniff_len(sniff, bytes, lens, i));
        if (f == Sniffed::Jpeg) {
            jb.push_back(bytes[i]);
            jl.push_back(lens[i]);
            ji.push_back(i);
            if (fmts) fmts[i] = IK_FORMAT_JPEG;
        } else if (f == Sniffed::Png) {
            pb.push_back(bytes[i]);
            pl.push_back(lens[i]);
            ph.push_back(sniff ? sniff[i] : bytes[i]);
            pi.push_back(i);
        } else {
            other.push_back(i);
        }
    }
    if (!pi.empty()) {  // every PNG of the batch through one set of GPU launches
        std::vector<ik_image*> po(pi.size(), nullptr);
        std::vector<int> ps(pi.size(), IK_OK);
        std::vector<std::string> pm(pi.size());
        if (up && up->n == (int)pi.size()) {
            png_decode_finish(*up, po.data(), ps.data(), pm.data());
        } else {
            PngUpload u;
            u.dev = sniff != nullptr;  // (device-resident inputs: the PNG items are device addresses)
            u.heads = ph.data();
            png_upload_begin(pb.data(), pl.data(), (int)pi.size(), u);
            png_decode_finish(u, po.data(), ps.data(), pm.data());
        }
        for (size_t k = 0; k < pi.size(); ++k) {
            outs[pi[k]] = po[k];
            st[pi[k]] = ps[k];
            msg[pi[k]] = pm[k];
        }
    }
    parallel_for((int)other.size(), threads, [&](int k) {  // PNG / WebP / unknown: host decoders, in parallel
        const uint32_t i = other[k];
        st[i] = decode_one(bytes[i], lens[i], &outs[i], fmts ? &fmts[i] : nullptr);
        if (st[i]) msg[i] = t_err;
    });
    if (!ji.empty()) {
        std::vector<ik_image*> jo(ji.size(), nullptr);
        std::vector<int> js(ji.size(), IK_OK);
        std::vector<std::string> jm(ji.size());
        decode_jpeg_batch(jb.data(), jl.data(), (int)ji.size(), jo.data(), js.data(), jm.data(), jup);
        for (size_t k = 0; k < ji.size(); ++k) {
            outs[ji[k]] = jo[k];
            st[ji[k]] = js[k];
            msg[ji[k]] = jm[k];
        }
    }
    int first = IK_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (st[i] && !first) first = st[i];
    return first;
}

}  // namespace ik (reopened for the ABI below)
extern "C" {

int ik_decode(const uint8_t* bytes, size_t len, ik_image** out, int* fmt_out) {
    IK_API_ENTER();
    if (!sched_multi()) return decode_one(bytes, len, out, fmt_out);
    // several devices: the least-loaded one decodes (the image stays there)
    const uint64_t cost = request_cost(bytes, len, -1, -1, IK_FORMAT_JPEG);
    const int ld = sched_acquire(cost);
    int st;
    {
        DeviceGuard g(sched_phys(ld));
        st = decode_one(bytes, len, out, fmt_out);
    }
    sched_release(ld, cost);
    return st;
}

int ik_decode_batch(const uint8_t* const* bytes, const size_t* lens, uint32_t n, ik_image** outs, int* fmts,
                    int* status) {
    IK_API_ENTER();
    if (!bytes || !lens || !outs || !n) return fail(IK_ERR_INVALID, "bad batch");
    std::vector<int> st(n, IK_OK);
    std::vector<std::string> msg(n);
    int first;
    if (sched_multi()) {
        uint64_t cost = 0;
        for (uint32_t i = 0; i < n; ++i) cost += request_cost(bytes[i], lens[i], -1, -1, IK_FORMAT_JPEG);
        const int ld = sched_acquire(cost);
        {
            DeviceGuard g(sched_phys(ld));
            first = decode_batch_dev(bytes, lens, n, outs, fmts, st.data(), msg.data(), 0);
        }
        sched_release(ld, cost);
    } else {
        first = decode_batch_dev(bytes, lens, n, outs, fmts, st.data(), msg.data(), 0);
    }
    uint32_t fi = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (status) status[i] = st[i];
        if (st[i] && fi == 0 && first && st[fi] == IK_OK) fi = i;
    }
    if (first) {
        for (fi = 0; fi < n && !st[fi]; ++fi) {}
        return fail(first, "input %u: %s", fi, msg[fi].c_str());
    }
    return IK_OK;
}

int ik_set_resize_mode(int mode) {
    if (mode != IK_RESIZE_EXACT && mode != IK_RESIZE_FMA) return fail(IK_ERR_INVALID, "bad resize mode %d", mode);
    (void)resize_mode();
    g_resize_mode.store(mode);
    return IK_OK;
}

int ik_get_resize_mode(void) { return resize_mode(); }

}  // extern "C"

namespace ik {

// ---- batched transforms: a four-stage pipeline per device -------------------------
// ik_transform_batch(_submit) -- the handlers of src/lib.rs:175-191 serving many
// requests -- runs each batch through four stages, each on its own threads, so
// that consecutive batches overlap on one device:
//   upload   (one thread per device)  the PNG streams' upload: parse, DMA of the
//            files (in place when the caller pinned them), the GPU gather + CRC
//            pass, and the JPEG files' DMA, on the upload thread's copy stream
//            (png_upload_begin, jpeg_upload_begin)
//   decode   (one thread per device)  the PNG decode kernels once that upload has
//            landed, JPEG entropy decoding and reconstruction, host decoders for
//            the rest (transform_decode_phase)
//   post     (one thread per device)  one resize launch per geometry group, the
//            encoders' device front ends (transform_post_phase), on its own stream:
//            batch k's resize runs beside batch k+1's decode kernels
//   host     (the device's worker pool)  the host coders (libwebp / libavif) and
//            the output buffers (transform_host_phase)
// so batch k+1's PCIe upload runs under batch k's kernels, and batch k's libwebp
// beside both.  With several logical devices (ik_init(-1) / IK_DEVICES) each has
// its own stages; a batch goes whole to the least-loaded device, or is split into
// parts of at least IK_MIN_DEVICE_BATCH (64) requests over several devices -- the
// inflate kernels' time hardly depends on how many frames a launch holds, so
// small parts would only add launches.
struct HostPhase {
    std::vector<uint32_t> idx;
    std::vector<EncodePrep> prep;
    std::vector<std::vector<uint8_t>> bytes_out;
    int threads = 0;
    double t_resize = 0, t_front = 0;
    // the decode stage's results, for the post stage: decoded images, status, message
    std::vector<ik_image*> imgs;
    std::vector<int> ds;
    std::vector<std::string> dm;
};

// the PNG requests among idx (decode_batch_dev takes the same ones, in the same order)
static void png_items(const uint8_t* const* bytes, const size_t* lens, const uint8_t* const* sniff,
                      const std::vector<uint32_t>& idx, std::vector<const uint8_t*>& pb, std::vector<size_t>& pl,
                      std::vector<const uint8_t*>& ph) {
    pb.clear();
    pl.clear();
    ph.clear();
    for (uint32_t i : idx)
        if ((bytes[i] || !lens[i]) &&
            guess_format(sniff ? sniff[i] : bytes[i], sniff_len(sniff, bytes, lens, i)) == Sniffed::Png) {
            pb.push_back(bytes[i]);
            pl.push_back(lens[i]);
            ph.push_back(sniff ? sniff[i] : bytes[i]);
        }
}

// the JPEG requests among idx, host inputs only (device-resident batches copy
// their non-PNG items to the host first)
static void jpeg_items(const uint8_t* const* bytes, const size_t* lens, const std::vector<uint32_t>& idx,
                       std::vector<const uint8_t*>& jb, std::vector<size_t>& jl) {
    jb.clear();
    jl.clear();
    for (uint32_t i : idx)
        if (bytes[i] && guess_format(bytes[i], lens[i]) == Sniffed::Jpeg) {
            jb.push_back(bytes[i]);
            jl.push_back(lens[i]);
        }
}

// Device half, decode stage: decode (GPU where the stream allows; the PNG upload
// already issued when up is given) under the device's kernel gate; the images,
// statuses and messages go to hp.imgs / ds / dm for the post stage
static void transform_decode_phase(const uint8_t* const* bytes, const size_t* lens, HostPhase& hp, PngUpload* up,
                                   const uint8_t* const* sniff = nullptr, const JpegUpload* jup = nullptr) {
    const std::vector<uint32_t>& idx = hp.idx;
    const uint32_t m = (uint32_t)idx.size();
    hp.imgs.assign(m, nullptr);
    hp.ds.assign(m, IK_OK);
    hp.dm.assign(m, std::string());
    if (!m) return;
    std::vector<const uint8_t*> b(m), sn(sniff ? m : 0);
    std::vector<size_t> l(m);
    for (uint32_t k = 0; k < m; ++k) {
        b[k] = bytes[idx[k]];
        l[k] = lens[idx[k]];
        if (sniff) sn[k] = sniff[idx[k]];
    }
    static const bool timing = getenv("IK_TIMING") != nullptr;  // dev: per-stage sums to stderr
    const auto tg0 = std::chrono::steady_clock::now();
    gate_pin(kGateKernels, true);
    const auto tg1 = std::chrono::steady_clock::now();
    batch_timing_reset(current_device(), false);
    BatchTimingScope bts;
    decode_batch_dev(b.data(), l.data(), m, hp.imgs.data(), nullptr, hp.ds.data(), hp.dm.data(), hp.threads, up,
                     sniff ? sn.data() : nullptr, jup);
    batch_timing_commit(current_device(), false);
    gate_pin(kGateKernels, false);
    if (timing)
        fprintf(stderr, "[device_phase] gate wait %.2f ms, decode %.2f ms\n",
                std::chrono::duration<double, std::milli>(tg1 - tg0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tg1).count());
}

// IK_WEBP_AUTO: smallest same-geometry group that the exact GPU coder takes
constexpr size_t kAutoExactMinGroup = 32;

// Device half, post stage: resize, the encoders' device front ends (under the
// post gate, so a batch's resize runs beside the next batch's decode kernels);
// request i's status / message land in st[i] / errs[i]
static void transform_post_phase(const int64_t* w, const int64_t* h, const int* fmt, const int* quality, int filter,
                                 int* st, std::string* errs, HostPhase& hp) {
    const std::vector<uint32_t>& idx = hp.idx;
    const int threads = hp.threads;
    const uint32_t m = (uint32_t)idx.size();
    if (!m) return;
    std::vector<ik_image*>& imgs = hp.imgs;
    std::vector<int>& ds = hp.ds;
    std::vector<std::string>& dm = hp.dm;
    static const bool timing = getenv("IK_TIMING") != nullptr;
    gate_pin(kGatePost, true);
    gate_enter(kGatePost);
    batch_timing_reset(current_device(), true);
    BatchTimingScope bts;
    std::mutex tmu;
    double& t_resize = hp.t_resize;
    double& t_front = hp.t_front;
    hp.prep.assign(m, EncodePrep());
    hp.bytes_out.assign(m, std::vector<uint8_t>());
    std::vector<EncodePrep>& prep = hp.prep;
    std::vector<std::vector<uint8_t>>& bytes_out = hp.bytes_out;
    // requests whose decoded images share a geometry and an output size resize in
    // one launch (resize_group); the rest, image by image below
    std::vector<ik_image*> rsz(m, nullptr);
    std::vector<char> fronted(m, 0);  // encode front end already run (batched WebP colour conversion)
    {
        std::map<std::tuple<uint32_t, uint32_t, uint32_t, size_t, int, uint32_t, uint32_t>, std::vector<uint32_t>> groups;
        for (uint32_t k = 0; k < m; ++k) {
            const uint32_t i = idx[k];
            if (ds[k] || !imgs[k] || imgs[k]->depth != 1 || (w[i] < 0 && h[i] < 0)) continue;
            uint32_t nw, nh;
            if (resize_target(imgs[k]->w, imgs[k]->h, w[i], h[i], &nw, &nh)) continue;
            if (nw == imgs[k]->w && nh == imgs[k]->h) continue;
            groups[std::make_tuple(imgs[k]->w, imgs[k]->h, imgs[k]->c, imgs[k]->pitch, imgs[k]->device, nw, nh)]
                .push_back(k);
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (auto& kv : groups) {
            if (kv.second.size() < 2) continue;
            std::vector<ik_image*> src, out;
            for (uint32_t k : kv.second) src.push_back(imgs[k]);
            if (resize_group(src, std::get<5>(kv.first), std::get<6>(kv.first), filter, out) != IK_OK) continue;
            for (size_t j = 0; j < out.size(); ++j) rsz[kv.second[j]] = out[j];
            // the group's WebP requests of one quality: one colour-conversion launch;
            // its JPEG requests of one quality: one coefficient + one Huffman launch
            std::map<int, std::vector<uint32_t>> byq, jbyq;
            for (uint32_t k : kv.second) {
                if (fmt[idx[k]] == IK_FORMAT_WEBP) byq[quality[idx[k]]].push_back(k);
                if (fmt[idx[k]] == IK_FORMAT_JPEG) jbyq[quality[idx[k]]].push_back(k);
            }
            const int webp_enc = default_webp_encoder();  // read once for the batch's groups (AUTO: exact)
            for (auto& qv : byq) {
                if (qv.second.size() < 2) continue;
                std::vector<ik_image*> im;
                std::vector<EncodePrep*> pp;
                for (uint32_t k : qv.second) { im.push_back(rsz[k]); pp.push_back(&prep[k]); }
                // AUTO: the GPU coder from kAutoExactMinGroup frames of one geometry on (its
                // chain of macroblock steps costs about the same for 2 frames as for 64; a
                // mixed-size stream's small groups code faster on the host threads:
                // configs[3]'s loadtest 2,106 vs 1,224 requests/s)
                const bool exact = webp_enc == IK_WEBP_EXACT ||
                                   (webp_enc == IK_WEBP_AUTO && qv.second.size() >= kAutoExactMinGroup);
                if (exact && im[0]->depth == 1 && im[0]->w <= 16383 && im[0]->h <= 16383) {
                    std::vector<std::vector<uint8_t>*> oo;
                    for (uint32_t k : qv.second) oo.push_back(&bytes_out[k]);
                    if (webp_exact_group(im, qv.first, oo) == IK_OK)
                        for (uint32_t k : qv.second) {
                            fronted[k] = 1;
                            prep[k].fmt = IK_FORMAT_WEBP;
                            prep[k].done = true;  // the files are final: no host coder
                        }
                    continue;
                }
                if (webp_front_group(im, qv.first, pp) == IK_OK)
                    for (uint32_t k : qv.second) fronted[k] = 1;
            }
            for (auto& qv : jbyq) {
                if (qv.second.size() < 2) continue;
                std::vector<ik_image*> im;
                std::vector<std::vector<uint8_t>*> oo;
                for (uint32_t k : qv.second) { im.push_back(rsz[k]); oo.push_back(&bytes_out[k]); }
                if (jpeg_front_group(im, qv.first, oo) == IK_OK)
                    for (uint32_t k : qv.second) {
                        fronted[k] = 1;
                        prep[k].fmt = IK_FORMAT_JPEG;
                        prep[k].done = true;  // the bytes are final: no host coder
                    }
            }
        }
        t_resize += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    parallel_for((int)m, threads, [&](int k) {
        const uint32_t i = idx[k];
        if (ds[k]) { st[i] = ds[k]; errs[i] = dm[k]; return; }
        ik_image* rs = rsz[k];
        const auto t0 = std::chrono::steady_clock::now();
        int r = rs ? IK_OK : ik_resize(imgs[k], w[i], h[i], filter, &rs);
        const auto t1 = std::chrono::steady_clock::now();
        if (!r && !fronted[k]) r = encode_image_front(rs, fmt[i], quality[i], prep[k], bytes_out[k]);
        if (timing) {
            const auto t2 = std::chrono::steady_clock::now();
            std::lock_guard<std::mutex> lk(tmu);
            t_resize += std::chrono::duration<double, std::milli>(t1 - t0).count();
            t_front += std::chrono::duration<double, std::milli>(t2 - t1).count();
        }
        if (r) { errs[i] = last_error_str(); st[i] = r; prep[k].done = true; }
        if (rs && rs != imgs[k]) ik_image_free(rs);
        ik_image_free(imgs[k]);
        imgs[k] = nullptr;
    });
    batch_timing_commit(current_device(), true);
    gate_pin(kGatePost, false);
    std::vector<ik_image*>().swap(hp.imgs);
    std::vector<int>().swap(hp.ds);
    std::vector<std::string>().swap(hp.dm);
}

static void transform_host_phase(uint8_t** outs, size_t* out_lens, int* st, std::string* errs, HostPhase& hp) {
    static const bool timing = getenv("IK_TIMING") != nullptr;
    const std::vector<uint32_t>& idx = hp.idx;
    const uint32_t m = (uint32_t)idx.size();
    std::vector<EncodePrep>& prep = hp.prep;
    std::vector<std::vector<uint8_t>>& bytes_out = hp.bytes_out;
    std::mutex tmu;
    double t_back = 0;
    std::atomic<int64_t> cpu_ns{0};  // thread CPU time of the coders (core budget)
    std::atomic<int> coded{0};
    const auto tw0 = std::chrono::steady_clock::now();
    const double tg = timing ? std::chrono::duration<double, std::milli>(
                                   std::chrono::steady_clock::now().time_since_epoch()).count() : 0.0;
    auto thread_cpu_ns = [] {
        timespec ts{};
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
        return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
    };
    parallel_for((int)m, hp.threads, [&](int k) {
        const uint32_t i = idx[k];
        if (st[i]) return;
        const auto t0 = std::chrono::steady_clock::now();
        const int64_t c0 = thread_cpu_ns();
        if (!prep[k].done) coded.fetch_add(1);  // a host coder runs (libwebp / libavif)
        int r = encode_host_back(prep[k], bytes_out[k]);
        cpu_ns.fetch_add(thread_cpu_ns() - c0);
        std::vector<uint8_t>().swap(prep[k].planes);
        prep[k].pin_block.reset();  // (the batch's pinned plane block goes back to its pool with the last)
        prep[k].pin_planes = nullptr;
        if (!r) {
            outs[i] = (uint8_t*)malloc(bytes_out[k].size() ? bytes_out[k].size() : 1);
            if (!outs[i]) r = fail(IK_ERR_NOMEM, "out of host memory");
            else {
                std::memcpy(outs[i], bytes_out[k].data(), bytes_out[k].size());
                out_lens[i] = bytes_out[k].size();
            }
        }
        if (timing) {
            std::lock_guard<std::mutex> lk(tmu);
            t_back += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        if (r) { errs[i] = last_error_str(); st[i] = r; }
    });
    batch_timing_host(current_device(),
                      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count(),
                      (double)cpu_ns.load() * 1e-6, (double)coded.load());
    if (timing)
        fprintf(stderr, "[transform_batch] t=%.1f..%.1f %u requests on device %d: resize %.1f ms, encode front %.1f ms, "
                "host coders %.1f ms (summed)\n", fmod(tg, 1e5), fmod(std::chrono::duration<double, std::milli>(
                std::chrono::steady_clock::now().time_since_epoch()).count(), 1e5), m, current_device(), hp.t_resize,
                hp.t_front, t_back);
}

namespace {

// one submitted batch (a ticket): its parts run on one or more devices
struct Ticket {
    uint32_t n = 0;
    uint8_t** outs = nullptr;
    size_t* out_lens = nullptr;
    int* status = nullptr;
    std::vector<int> st;
    std::vector<std::string> errs;
    std::mutex mu;
    std::condition_variable cv;
    int pending = 0;
    // device-resident inputs (ik_transform_batch_submit_device): the request array
    // the stages read (PNG items: the caller's device addresses; others: host
    // copies), the host copies, and each item's sniff bytes
    std::vector<const uint8_t*> eff, sniff;
    std::vector<std::vector<uint8_t>> hcopy;
    std::vector<uint8_t> heads;
};

// one device's share of a ticket
struct BatchPart {
    std::shared_ptr<Ticket> t;
    const uint8_t* const* bytes = nullptr;
    const size_t* lens = nullptr;
    const int64_t* w = nullptr;
    const int64_t* h = nullptr;
    const int* fmt = nullptr;
    const int* quality = nullptr;
    int filter = 0;
    HostPhase hp;
    std::vector<const uint8_t*> pb;  // its PNG inputs (the upload stage's batch)
    std::vector<size_t> pl;
    std::vector<const uint8_t*> ph;  // their first bytes in host memory
    const uint8_t* const* sniff = nullptr;  // device-resident inputs (Ticket::sniff), else null
    PngUpload up;
    std::vector<const uint8_t*> jb;  // its JPEG inputs in host memory
    std::vector<size_t> jl;
    JpegUpload jup;  // their device copies (the upload stage's JPEG DMA)
    int logical = -1;  // logical device (multi-device dispatch), -1 = none
    uint64_t cost = 0;
};

class StageExec {
public:
    StageExec(int device, Pool* host_pool) : dev_(device), pool_(host_pool) {
        for (int k = 0; k < kStages; ++k) th_[k] = std::thread([this, k] { loop(k); });  // live until stop()
    }
    // ik_shutdown: the stages finish what is queued (upload, then decode, then post), then end
    void stop() {
        for (int k = 0; k < kStages; ++k) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                done_[k] = true;
            }
            cv_.notify_all();
            th_[k].join();
        }
    }
    void submit(std::shared_ptr<BatchPart> p) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_[0].push_back(std::move(p));
        }
        cv_.notify_all();
    }

private:
    void loop(int stage) {
        mark_internal_thread();  // the library's own thread: no lifetime lock (ApiGuard)
        ik_init(dev_);  // this thread's streams, staging and scratch live on dev_
        for (;;) {
            std::shared_ptr<BatchPart> p;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return done_[stage] || !q_[stage].empty(); });
                if (q_[stage].empty()) break;  // stopped, nothing left
                p = std::move(q_[stage].front());
                q_[stage].pop_front();
            }
            if (stage == 0) {
                png_items(p->bytes, p->lens, p->sniff, p->hp.idx, p->pb, p->pl, p->ph);
                p->up.dev = p->sniff != nullptr;
                p->up.heads = p->ph.data();
                if (!p->pb.empty()) png_upload_begin(p->pb.data(), p->pl.data(), (int)p->pb.size(), p->up);
                if (!p->sniff) {
                    jpeg_items(p->bytes, p->lens, p->hp.idx, p->jb, p->jl);
                    if (!p->jb.empty()) jpeg_upload_begin(p->jb.data(), p->jl.data(), (int)p->jb.size(), p->jup);
                }
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    q_[1].push_back(std::move(p));
                }
                cv_.notify_all();
                continue;
            }
            if (stage == 2) {
                // resize + the encoders' device front ends, beside the next batch's decode
                Ticket& t = *p->t;
                transform_post_phase(p->w, p->h, p->fmt, p->quality, p->filter, t.st.data(), t.errs.data(), p->hp);
                pool_->post([p] {
                    Ticket& tk = *p->t;
                    transform_host_phase(tk.outs, tk.out_lens, tk.st.data(), tk.errs.data(), p->hp);
                    p->hp = HostPhase();
                    if (p->logical >= 0) sched_release(p->logical, p->cost);
                    std::lock_guard<std::mutex> lk(tk.mu);
                    if (--tk.pending == 0) tk.cv.notify_all();
                });
                continue;
            }
            // the next queued batch's block search goes out on this stream between
            // this batch's decode rounds and its expand
            p->up.on_next_search = [this](hipEvent_t after) {
                std::shared_ptr<BatchPart> nx;
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    if (!q_[1].empty()) nx = q_[1].front();
                }
                if (!nx || nx->pb.empty()) return;
                // On the kernel stream itself, between this batch's decode rounds and its
                // expand (it covers the host planning there), once the next batch's
                // upload has landed (else its own kernel stage launches it).  Beside
                // expand / resolve / unfilter it only slows them: a stream on another
                // hardware queue measured 63-69 vs 61-62 ms per step (the search took
                // resolve from 3.6 to 13-19 ms; profiles/r03n_find_*.json).
                if (!png_upload_landed(nx->up)) return;
                hipStream_t fs = png_find_beside_decode() ? thread_copy_stream() : thread_stream();
                if (after && hipStreamWaitEvent(fs, after, 0) != hipSuccess) return;
                png_find_prelaunch(nx->up, fs);
            };
            transform_decode_phase(p->bytes, p->lens, p->hp, p->pb.empty() ? nullptr : &p->up, p->sniff, &p->jup);
            p->up = PngUpload();
            p->jup = JpegUpload();  // (the decode has returned: its area is free again)
            {
                std::lock_guard<std::mutex> lk(mu_);
                q_[2].push_back(std::move(p));
            }
            cv_.notify_all();
        }
        release_thread_resources();
    }
    int dev_;
    Pool* pool_;
    std::mutex mu_;
    std::condition_variable cv_;
    static constexpr int kStages = 3;  // upload, decode, post (resize + device front ends)
    std::deque<std::shared_ptr<BatchPart>> q_[kStages];
    bool done_[kStages] = {false, false, false};
    std::thread th_[kStages];
};

std::mutex g_stage_mu;
std::map<int, StageExec*> g_stages;

// the stages of a logical device, or (single-device mode) of physical device
// `phys` (-1: the calling thread's device)
StageExec& stage_exec(int logical, int phys) {
    const int dev = phys >= 0 ? phys : current_device();
    const int key = logical >= 0 ? 1000 + logical : dev;
    std::lock_guard<std::mutex> lk(g_stage_mu);
    StageExec*& e = g_stages[key];
    if (!e) e = logical >= 0 ? new StageExec(sched_phys(logical), &sched_pool(logical))
                             : new StageExec(dev, &device_pool(dev));
    return *e;
}

std::mutex g_async_mu;
std::map<uint64_t, std::shared_ptr<Ticket>> g_async;
uint64_t g_async_next = 1;

}  // namespace

// ik_shutdown's device-memory part: pooled image blocks, the batched colour
// launches' pinned blocks, the per-device constant tables
static void memory_shutdown() {
    {
        std::lock_guard<std::mutex> lk(g_ipool_mu);
        for (auto& kv : g_ipools) {
            std::lock_guard<std::mutex> lk2(kv.second->mu);
            (void)hipSetDevice(kv.first);
            for (auto& b : kv.second->free_blocks) {
                (void)hipFree(b.second);
                mem_stat(kMemImageFree, -(int64_t)b.first);
            }
            kv.second->free_blocks.clear();
            kv.second->held = 0;
        }
    }
    {
        std::lock_guard<std::mutex> lk(g_pblk_mu);
        for (auto& b : g_pblk_free) (void)hipHostFree(b.second);
        g_pblk_free.clear();
        g_pblk_held = 0;
    }
    std::lock_guard<std::mutex> lk(g_consts_mu);
    for (auto& kv : g_consts) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second->gamma_to_lin);
        (void)hipFree(kv.second->lin_to_gamma);
        (void)hipFree(kv.second->jpeg_huff);
        delete kv.second;
    }
    g_consts.clear();
}

// ik_shutdown: wait for every submitted batch, end the stage threads and the
// worker pools (each releases its streams and arenas), then free what the
// library holds, all while the HIP runtime is alive
int shutdown_all(bool close) {
    // exclusive: every caller still inside the library returns first (ApiGuard);
    // nested entry points called from here see depth > 0 and take nothing
    std::unique_lock<LifeLock> life(g_life);
    ++t_api_depth;
    if (close) g_closed.store(true, std::memory_order_release);
    std::vector<std::shared_ptr<Ticket>> ts;
    {
        std::lock_guard<std::mutex> lk(g_async_mu);
        for (auto& kv : g_async) ts.push_back(kv.second);
    }
    for (auto& t : ts) {
        std::unique_lock<std::mutex> lk(t->mu);
        t->cv.wait(lk, [&] { return t->pending == 0; });
    }
    std::vector<StageExec*> st;
    {
        std::lock_guard<std::mutex> lk(g_stage_mu);
        for (auto& kv : g_stages) st.push_back(kv.second);
        g_stages.clear();
    }
    for (StageExec* e : st) {
        e->stop();
        delete e;
    }
    pools_shutdown();
    const int dev = t_device;
    png_shutdown();
    jpeg_shutdown();
    plans_shutdown();
    memory_shutdown();
    release_thread_resources();
    if (dev >= 0) (void)hipSetDevice(dev);
    --t_api_depth;
    return IK_OK;
}

namespace {

int min_device_batch() {
    static const int v = [] {
        const char* e = getenv("IK_MIN_DEVICE_BATCH");
        const int x = e && *e ? atoi(e) : 64;
        return x < 1 ? 1 : x;
    }();
    return v;
}

}  // namespace
}  // namespace ik

extern "C" {

}  // extern "C"

namespace ik {
namespace {

// the parts of a ticket to the stage executors.  bytes / sniff: the request array
// the stages read (Ticket::eff / sniff for device-resident inputs); phys >= 0:
// the inputs live on that physical device, so the batch goes whole to it
int submit_parts(const std::shared_ptr<Ticket>& t, const uint8_t* const* bytes, const uint8_t* const* sniff,
                 int phys, const size_t* lens, uint32_t n, const int64_t* w, const int64_t* h, const int* fmt,
                 const int* quality, int filter, int threads, uint64_t* ticket) {
    auto make_part = [&](uint32_t lo, uint32_t hi) {
        auto p = std::make_shared<BatchPart>();
        p->t = t;
        p->bytes = bytes; p->lens = lens; p->w = w; p->h = h; p->fmt = fmt; p->quality = quality;
        p->sniff = sniff;
        p->filter = filter;
        p->hp.threads = threads;
        for (uint32_t i = lo; i < hi; ++i) p->hp.idx.push_back(i);
        return p;
    };
    auto cost_of = [&](uint32_t i) {
        return request_cost(sniff ? sniff[i] : bytes[i], sniff_len(sniff, bytes, lens, i), w[i], h[i], fmt[i]);
    };
    std::vector<std::shared_ptr<BatchPart>> parts;
    if (!sched_multi()) {
        parts.push_back(make_part(0, n));  // to the stages of `phys` (the inputs' device) or the caller's device
    } else if (phys >= 0) {
        auto p = make_part(0, n);
        for (uint32_t i = 0; i < n; ++i) p->cost += cost_of(i);
        p->logical = sched_acquire_on(phys, p->cost);
        if (p->logical < 0) return fail(IK_ERR_INVALID, "the inputs are on device %d, which serves no logical device", phys);
        parts.push_back(p);
    } else {
        // whole parts of >= IK_MIN_DEVICE_BATCH requests (sched_split's bounds), each to the
        // least-loaded device by the live counters
        const uint32_t nd = (uint32_t)sched_count();
        std::vector<uint64_t> costs(n), out(nd, 0);
        for (uint32_t i = 0; i < n; ++i) costs[i] = cost_of(i);
        std::vector<uint32_t> lo(nd + 1), dev(nd);
        const uint32_t P = sched_split(costs.data(), n, nd, (uint32_t)min_device_batch(), out.data(), lo.data(), dev.data());
        for (uint32_t q = 0; q < P; ++q) {
            auto p = make_part(lo[q], lo[q + 1]);
            for (uint32_t i : p->hp.idx) p->cost += costs[i];
            p->logical = sched_acquire(p->cost);
            parts.push_back(p);
        }
    }
    t->pending = (int)parts.size();
    {
        std::lock_guard<std::mutex> lk(g_async_mu);
        *ticket = g_async_next++;
        g_async[*ticket] = t;
    }
    for (auto& p : parts) {
        const int ld = p->logical;
        stage_exec(ld, ld >= 0 ? -1 : phys).submit(std::move(p));
    }
    return IK_OK;
}

std::shared_ptr<Ticket> new_ticket(uint32_t n, uint8_t** outs, size_t* out_lens, int* status) {
    auto t = std::make_shared<Ticket>();
    t->n = n;
    t->outs = outs;
    t->out_lens = out_lens;
    t->status = status;
    t->st.assign(n, IK_OK);
    t->errs.assign(n, std::string());
    for (uint32_t i = 0; i < n; ++i) { outs[i] = nullptr; out_lens[i] = 0; }
    return t;
}

}  // namespace
}  // namespace ik

extern "C" {

int ik_transform_batch_submit(const uint8_t* const* bytes, const size_t* lens, uint32_t n, const int64_t* w,
                              const int64_t* h, const int* fmt, const int* quality, int filter, int threads,
                              uint8_t** outs, size_t* out_lens, int* status, uint64_t* ticket) {
    IK_API_ENTER();
    if (!bytes || !lens || !w || !h || !fmt || !quality || !outs || !out_lens || !n || !ticket)
        return fail(IK_ERR_INVALID, "bad batch");
    auto t = new_ticket(n, outs, out_lens, status);
    return submit_parts(t, bytes, nullptr, -1, lens, n, w, h, fmt, quality, filter, threads, ticket);
}

int ik_transform_batch_submit_device(const uint8_t* const* dev_bytes, const size_t* lens, uint32_t n,
                                     const int64_t* w, const int64_t* h, const int* fmt, const int* quality,
                                     int filter, int threads, uint8_t** outs, size_t* out_lens, int* status,
                                     uint64_t* ticket) {
    IK_API_ENTER();
    if (!dev_bytes || !lens || !w || !h || !fmt || !quality || !outs || !out_lens || !n || !ticket)
        return fail(IK_ERR_INVALID, "bad batch");
    // every input must be device memory of one device (the batch runs there)
    int phys = -1;
    for (uint32_t i = 0; i < n; ++i) {
        if (!lens[i]) continue;
        if (!dev_bytes[i]) return fail(IK_ERR_INVALID, "input %u: null bytes", i);
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, dev_bytes[i]) != hipSuccess || at.type != hipMemoryTypeDevice) {
            (void)hipGetLastError();
            return fail(IK_ERR_INVALID, "input %u is not device memory", i);
        }
        if (phys < 0) phys = at.device;
        else if (phys != at.device) return fail(IK_ERR_INVALID, "inputs on devices %d and %d", phys, at.device);
    }
    if (phys < 0) phys = current_device();
    auto t = new_ticket(n, outs, out_lens, status);
    t->eff.assign(dev_bytes, dev_bytes + n);
    t->sniff.assign(n, nullptr);
    t->hcopy.resize(n);
    t->heads.assign(64 * (size_t)n, 0);
    {
        DeviceGuard g(phys);
        // the first 64 bytes of every file, through pinned memory
        const size_t o_files = (64 * (size_t)n + 255) & ~size_t(255);
        uint8_t* pin = pinned_slot(7, o_files + 2 * sizeof(uint64_t) * n);
        void* dp = nullptr;
        if (!pin || hipHostGetDevicePointer(&dp, pin, 0) != hipSuccess || !dp)
            return fail(IK_ERR_NOMEM, "cannot allocate pinned memory for the input headers");
        uint64_t* files = reinterpret_cast<uint64_t*>(pin + o_files);
        for (uint32_t i = 0; i < n; ++i) {
            files[i] = (uint64_t)(uintptr_t)dev_bytes[i];
            files[n + i] = dev_bytes[i] ? lens[i] : 0;
        }
        hipStream_t s = thread_stream();
        const uint64_t* df = reinterpret_cast<const uint64_t*>(reinterpret_cast<uint8_t*>(dp) + o_files);
        IK_HIP(launch_copy_heads(df, df + n, (int)n, reinterpret_cast<uint8_t*>(dp), s));
        IK_HIP(hipStreamSynchronize(s));
        std::memcpy(t->heads.data(), pin, 64 * (size_t)n);
        // PNG files stay where they are (the upload stage walks and gathers them on
        // the GPU); any other item comes back to host memory for its host-side parse
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t* hd = t->heads.data() + 64 * (size_t)i;
            if (!dev_bytes[i] || guess_format(hd, std::min<size_t>(lens[i], 64)) == Sniffed::Png) {
                t->sniff[i] = dev_bytes[i] ? hd : nullptr;
                continue;
            }
            t->hcopy[i].resize(lens[i]);
            IK_HIP(hipMemcpy(t->hcopy[i].data(), dev_bytes[i], lens[i], hipMemcpyDeviceToHost));
            t->eff[i] = t->sniff[i] = t->hcopy[i].data();
        }
    }
    // the batch runs where its inputs are: on a logical device of `phys`, or (single-
    // device mode) on the stages of `phys` whatever the calling thread's device is
    return submit_parts(t, t->eff.data(), t->sniff.data(), phys, lens, n, w, h, fmt, quality, filter, threads, ticket);
}

int ik_memory_stats(uint64_t* out, int n) {
    if (!out || n <= 0) return fail(IK_ERR_INVALID, "bad stats buffer");
    for (int i = 0; i < n; ++i) out[i] = i < kMemStats ? (uint64_t)std::max<int64_t>(0, g_mem[i].load()) : 0;
    return IK_OK;
}

int ik_shutdown(void) { return shutdown_all(false); }
int ik_close(void) { return shutdown_all(true); }

int ik_batch_last_timing(double* out, int n) {
    if (!out || n <= 0) return fail(IK_ERR_INVALID, "bad timing buffer");
    const int d = current_device();
    std::lock_guard<std::mutex> lk(g_bt_mu);
    auto it = g_bt_last.find(d);
    for (int i = 0; i < n; ++i) out[i] = it != g_bt_last.end() && i < (int)it->second.size() ? it->second[(size_t)i] : 0.0;
    return IK_OK;
}

int ik_transform_batch_wait(uint64_t ticket) {
    IK_API_ENTER();
    std::shared_ptr<Ticket> t;
    {
        std::lock_guard<std::mutex> lk(g_async_mu);
        auto it = g_async.find(ticket);
        if (it == g_async.end()) return fail(IK_ERR_INVALID, "unknown batch ticket %llu", (unsigned long long)ticket);
        t = it->second;
        g_async.erase(it);
    }
    {
        std::unique_lock<std::mutex> lk(t->mu);
        t->cv.wait(lk, [&] { return t->pending == 0; });
    }
    int first = IK_OK;
    uint32_t first_i = 0;
    for (uint32_t i = 0; i < t->n; ++i) {
        if (t->status) t->status[i] = t->st[i];
        if (t->st[i] && !first) { first = t->st[i]; first_i = i; }
    }
    if (first) return fail(first, "item %u: %s", first_i, t->errs[first_i].c_str());
    return IK_OK;
}

int ik_transform_batch(const uint8_t* const* bytes, const size_t* lens, uint32_t n, const int64_t* w,
                       const int64_t* h, const int* fmt, const int* quality, int filter, int threads, uint8_t** outs,
                       size_t* out_lens, int* status) {
    IK_API_ENTER();
    uint64_t ticket = 0;
    if (int rc = ik_transform_batch_submit(bytes, lens, n, w, h, fmt, quality, filter, threads, outs, out_lens, status,
                                           &ticket))
        return rc;
    return ik_transform_batch_wait(ticket);
}

static int transform_here(const uint8_t* bytes, size_t len, int64_t w, int64_t h, int fmt, int quality,
                          int filter, uint8_t** out, size_t* out_len) {
    ik_image* img = nullptr;
    int st = decode_one(bytes, len, &img, nullptr);
    if (st) return st;
    ik_image* rs = nullptr;
    st = ik_resize(img, w, h, filter, &rs);
    if (st) { ik_image_free(img); return st; }
    st = ik_encode(rs, fmt, quality, out, out_len);
    if (rs != img) ik_image_free(rs);
    ik_image_free(img);
    return st;
}

int ik_transform(const uint8_t* bytes, size_t len, int64_t w, int64_t h, int fmt, int quality,
                 int filter, uint8_t** out, size_t* out_len) {
    IK_API_ENTER();
    if (!sched_multi()) return transform_here(bytes, len, w, h, fmt, quality, filter, out, out_len);
    // several devices: queue the request to the least-loaded device's workers
    const uint64_t cost = request_cost(bytes, len, w, h, fmt);
    const int ld = sched_acquire(cost);
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    int st = IK_OK;
    std::string msg;
    sched_pool(ld).post([&] {
        const int r = transform_here(bytes, len, w, h, fmt, quality, filter, out, out_len);
        std::string m = r ? last_error_str() : std::string();
        std::lock_guard<std::mutex> lk(mu);
        st = r;
        msg.swap(m);
        done = true;
        cv.notify_all();
    });
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done; });
    }
    sched_release(ld, cost);
    if (st) return fail(st, "%s", msg.c_str());
    return IK_OK;
}

int ik_resize_batch_device(const uint8_t* dev_src, uint32_t W, uint32_t H, uint32_t C,
                           size_t src_pitch, size_t src_image_stride, uint32_t n, uint32_t nw,
                           uint32_t nh, int filter, uint8_t* dev_dst, size_t dst_pitch,
                           size_t dst_image_stride, void* hip_stream) {
    IK_API_ENTER();
    if (!dev_src || !dev_dst) return fail(IK_ERR_INVALID, "null device pointer");
    if (C < 1 || C > 4 || !W || !H || !nw || !nh || !n) return fail(IK_ERR_INVALID, "bad geometry");
    if (filter < 0 || filter > 4) return fail(IK_ERR_INVALID, "unknown filter %d", filter);
    if (src_pitch < (size_t)W * C || dst_pitch < (size_t)nw * C) return fail(IK_ERR_INVALID, "pitch too small");
    if ((src_pitch & 7) || ((uintptr_t)dev_src & 7)) return fail(IK_ERR_INVALID, "source rows must be 8-byte aligned");
    if (C == 4 && (((uintptr_t)dev_dst & 3) || (dst_pitch & 3) || (dst_image_stride & 3)))
        return fail(IK_ERR_INVALID, "RGBA destination rows must be 4-byte aligned");
    if (n > 1 && (src_image_stride < src_pitch * H || dst_image_stride < dst_pitch * nh))
        return fail(IK_ERR_INVALID, "image stride too small");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : thread_stream();
    ResizePlan* plan = get_resize_plan(current_device(), (int)W, (int)H, (int)C, (int)nw, (int)nh, filter, (int)n);
    if (!plan) return fail(IK_ERR_DEVICE, "cannot build resize plan");
    float* tmp = nullptr;
    if (plan->slots == 0 || !resize_fused_fits(src_pitch, H)) {
        tmp = (float*)scratch(sizeof(float) * (size_t)n * nh * W * C);
        if (!tmp) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
    }
    hipError_t e = launch_resize(*plan, dev_src, src_pitch, src_image_stride, dev_dst, dst_pitch,
                                 dst_image_stride, (int)n, tmp, s);
    if (e != hipSuccess) return hip_fail(e, "resize kernel launch");
    return IK_OK;
}

const char* ik_resize_kernel_name(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter) {
    if (C < 1 || C > 4 || !W || !H || !nw || !nh || filter < 0 || filter > 4) return nullptr;
    ResizePlan* plan = get_resize_plan(current_device(), (int)W, (int)H, (int)C, (int)nw, (int)nh, filter, 1);
    return plan ? resize_kernel_name(*plan, (size_t)W * C) : nullptr;
}

int ik_webp_yuv420_device(const uint8_t* dev_src, uint32_t w, uint32_t h, uint32_t C, size_t pitch,
                          uint8_t* dev_yuv, void* hip_stream) {
    IK_API_ENTER();
    if (!dev_src || !dev_yuv || !w || !h || C < 1 || C > 4) return fail(IK_ERR_INVALID, "bad arguments");
    const DeviceConsts* dc = device_consts(current_device());
    if (!dc) return fail(IK_ERR_DEVICE, "cannot upload WebP tables");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : thread_stream();
    IK_HIP(launch_webp_yuv420(dev_src, (int)w, (int)h, (int)C, pitch, 0, dev_yuv, 0, 1,
                              dc->gamma_to_lin, dc->lin_to_gamma, s));
    return IK_OK;
}

int ik_jpeg_coeffs_device(const uint8_t* dev_src, uint32_t w, uint32_t h, uint32_t C, size_t pitch,
                          int quality, int16_t* dev_coef, void* hip_stream) {
    IK_API_ENTER();
    if (!dev_src || !dev_coef || !w || !h || C < 1 || C > 4) return fail(IK_ERR_INVALID, "bad arguments");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : thread_stream();
    uint8_t qt[128];
    jpeg_quant_tables(quality < 1 ? 1 : quality > 100 ? 100 : quality, qt);
    uint8_t* dq = scratch(128);
    if (!dq) return fail(IK_ERR_DEVICE, "cannot allocate device scratch");
    if (int rc = copy_h2d_2d(dq, 128, qt, 128, 128, 1, s)) return rc;
    IK_HIP(launch_jpeg_coeffs(dev_src, (int)w, (int)h, (int)C, pitch, 0, dq, dev_coef, 0, 1, s));
    IK_HIP(hipStreamSynchronize(s));
    return IK_OK;
}

int ik_dev_alloc(size_t bytes, void** dev_ptr) {
    if (!dev_ptr) return fail(IK_ERR_INVALID, "null pointer");
    (void)hipSetDevice(current_device());
    IK_HIP(hipMalloc(dev_ptr, bytes ? bytes : 1));
    return IK_OK;
}
int ik_dev_free(void* p) { IK_HIP(hipFree(p)); return IK_OK; }
int ik_memcpy_h2d(void* d, const void* h, size_t n) {
    IK_API_ENTER();
    IK_HIP(hipDeviceSynchronize());
    return copy_h2d_2d((uint8_t*)d, n, (const uint8_t*)h, n, n, n ? 1 : 0, thread_stream());
}
int ik_memcpy_d2h(void* h, const void* d, size_t n) {
    IK_API_ENTER();
    IK_HIP(hipDeviceSynchronize());
    return copy_d2h_2d((uint8_t*)h, n, (const uint8_t*)d, n, n, n ? 1 : 0, thread_stream());
}
int ik_dev_synchronize(void) { IK_HIP(hipDeviceSynchronize()); return IK_OK; }

}  // extern "C"
