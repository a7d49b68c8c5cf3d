// ik_pool.cpp -- persistent host workers and the multi-device work queue of
// libimagekit_hip.so.
//
// The reference runs one synchronous transform per tokio worker thread
// (src/main.rs:20, handlers src/lib.rs:175-191 / :281-297), so a drop-in is
// called from up to `nproc` threads at once.  Two things follow:
//
//  - Workers are PERSISTENT.  Each worker thread owns per-device HIP resources in
//    thread-local storage (a stream, pinned staging, device scratch); a pool
//    thread keeps them for the life of the process, so a batch call reuses them
//    instead of creating (and leaking) them per call.  parallel_for hands work
//    to the pool of the calling thread's device and the caller takes part, so
//    nested calls from a worker can never deadlock.
//
//  - One process can drive several GPUs (ik_init(-1), IK_DEVICES).  Requests go
//    to LOGICAL devices (IK_DEVICES=0,0 maps two onto device 0, for tests) by
//    least outstanding cost: each request's cost is an estimate in bytes of the
//    work it brings (encoded input + decoded pixels + an encoder weight per
//    output pixel), added to the chosen device's counter on submission and
//    removed on completion.  Each logical device has its own worker pool.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {

namespace {

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    if (!e || !*e) return dflt;
    const int v = atoi(e);
    return v > 0 ? v : dflt;
}

}  // namespace

int default_threads() {
    static const int t = env_int("IK_THREADS", (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    return t;
}

// ---- phase gates -----------------------------------------------------------------
namespace {
std::mutex& gate_mutex(int device, int which) {
    static std::mutex m[64][3];
    return m[(unsigned)device % 64u][(unsigned)which % 3u];
}
struct GateState {
    bool held[3] = {false, false, false}, pinned[3] = {false, false, false};
    int dev[3] = {0, 0, 0};
};
thread_local GateState t_gate;
}  // namespace

void gate_enter(int which) {
    if (t_gate.held[which]) return;
    const int d = current_device();
    gate_mutex(d, which).lock();
    t_gate.held[which] = true;
    t_gate.dev[which] = d;
}

bool gate_try_enter(int which) {
    if (t_gate.held[which]) return true;
    const int d = current_device();
    if (!gate_mutex(d, which).try_lock()) return false;
    t_gate.held[which] = true;
    t_gate.dev[which] = d;
    return true;
}

bool gate_held_any() { return t_gate.held[kGateKernels] || t_gate.held[kGateUpload] || t_gate.held[kGatePost]; }

void gate_leave(int which) {
    if (!t_gate.held[which] || t_gate.pinned[which]) return;
    gate_mutex(t_gate.dev[which], which).unlock();
    t_gate.held[which] = false;
}

void gate_pin(int which, bool on) {
    t_gate.pinned[which] = on;
    if (!on) gate_leave(which);
}

// ---- Pool ----------------------------------------------------------------------
Pool::Pool(int device, int max_threads) : device_(device), max_threads_(std::max(1, max_threads)) {}

void Pool::ensure(int nthreads) {
    // called with mu_ held; workers live until stop() (ik_shutdown)
    nthreads = std::min(nthreads, max_threads_);
    while (nthreads_ < nthreads) {
        threads_.emplace_back([this] { loop(); });
        ++nthreads_;
    }
}

void Pool::stop() {
    std::vector<std::thread> ts;
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
        ts.swap(threads_);
    }
    cv_.notify_all();
    for (std::thread& t : ts) t.join();
    std::lock_guard<std::mutex> lk(mu_);
    nthreads_ = 0;
    stop_ = false;
}

void Pool::loop() {
    // bulk host work (staging copies, libwebp / libavif coding) runs here: a lower
    // priority than the callers' own threads, which launch the kernels and plan
    // the next launch -- on a CPU-limited host those must not wait behind it
    static const int nice_v = env_int("IK_WORKER_NICE", 19);
    if (nice_v > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice_v);
    mark_internal_thread();  // the library's own thread: no lifetime lock (ApiGuard)
    ik_init(device_);  // this worker's stream / staging / scratch live on device_
    for (;;) {
        std::function<void()> task;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) break;  // stopped, nothing left to run
            task = std::move(q_.front().fn);
            q_.pop_front();
            ++busy_;
        }
        task();
        std::lock_guard<std::mutex> lk(mu_);
        --busy_;
    }
    release_thread_resources();  // while the runtime is alive (not a thread-exit destructor)
}

void Pool::post(std::function<void()> task) { post_tagged(std::move(task), nullptr); }

void Pool::post_tagged(std::function<void()> task, const void* tag) {
    // work for a caller inside a GPU phase (it holds a phase gate: an upload or a
    // kernel stage) goes to the front of the queue: behind another batch's bulk
    // host work (libwebp) it would keep the GPU phase -- and the device -- waiting
    const bool urgent = gate_held_any();
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (urgent) q_.push_front(Task{std::move(task), tag});
        else q_.push_back(Task{std::move(task), tag});
        ensure(busy_ + (int)q_.size());
    }
    cv_.notify_one();
}

// A finished parallel_for's helpers still queued would do nothing when run, but
// they count as work in ensure(): left there, every later call would see them and
// start more threads (each with its own stream and arenas) -- the pool crept
// towards its cap under batch load.  Remove them.
void Pool::withdraw(const void* tag) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = q_.begin(); it != q_.end();) {
        if (it->tag == tag) it = q_.erase(it);
        else ++it;
    }
}

namespace {
struct ForState {
    std::atomic<int> next{0};
    int n = 0;
    const std::function<void(int)>* fn = nullptr;
    std::mutex mu;
    std::condition_variable cv;
    int done = 0;
    void work() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            (*fn)(i);
            std::lock_guard<std::mutex> lk(mu);
            if (++done == n) cv.notify_all();
        }
    }
};
}  // namespace

void Pool::parallel_for(int n, int threads, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (threads <= 0) threads = default_threads();
    threads = std::min(threads, n);
    if (threads <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    auto st = std::make_shared<ForState>();
    st->n = n;
    st->fn = &fn;
    // helpers: a helper dequeued after every index was claimed returns at once and
    // never touches fn; the caller always works too, so progress never depends on
    // a free worker (nested parallel_for from a worker is safe)
    for (int t = 1; t < threads; ++t) post_tagged([st] { st->work(); }, st.get());
    st->work();
    {
        std::unique_lock<std::mutex> lk(st->mu);
        st->cv.wait(lk, [&] { return st->done == st->n; });
    }
    withdraw(st.get());
}

namespace {
std::mutex g_dpool_mu;
std::map<int, Pool*> g_dpools;  // never freed: a Pool& handed out stays valid
}  // namespace

Pool& device_pool(int device) {
    std::lock_guard<std::mutex> lk(g_dpool_mu);
    Pool*& p = g_dpools[device];
    if (!p) p = new Pool(device, env_int("IK_MAX_WORKERS", 256));
    return *p;
}

void parallel_for(int n, int threads, const std::function<void(int)>& fn) {
    device_pool(current_device()).parallel_for(n, threads, fn);
}

// ---- multi-device scheduler ------------------------------------------------------
namespace {
struct Logical {
    int phys = 0;
    std::atomic<uint64_t> outstanding{0}, jobs{0}, cost_done{0};
    Pool* pool = nullptr;
};
struct Sched {
    std::mutex mu;                      // guards picks (read-modify of the counters)
    std::vector<std::unique_ptr<Logical>> devs;
    bool multi = false;
};
Sched& sched() {
    static Sched s;
    return s;
}
}  // namespace

int sched_configure(const int* devices, int n) {
    Sched& s = sched();
    std::lock_guard<std::mutex> lk(s.mu);
    int nvis = 0;
    if (hipGetDeviceCount(&nvis) != hipSuccess) nvis = 0;
    std::vector<int> ids;
    if (devices && n > 0) {
        ids.assign(devices, devices + n);
    } else if (const char* e = getenv("IK_DEVICES")) {
        for (const char* p = e; *p;) {
            char* endp = nullptr;
            const long v = strtol(p, &endp, 10);
            if (endp == p) { ++p; continue; }
            ids.push_back((int)v);
            p = endp;
        }
    } else {
        for (int d = 0; d < nvis; ++d) ids.push_back(d);
    }
    if (ids.empty()) return fail(IK_ERR_INVALID, "no devices for multi-device dispatch");
    for (int d : ids)
        if (d < 0 || d >= nvis) return fail(IK_ERR_INVALID, "device %d out of range (%d devices)", d, nvis);
    if (s.multi && s.devs.size() == ids.size()) {
        bool same = true;
        for (size_t i = 0; i < ids.size(); ++i) same = same && s.devs[i]->phys == ids[i];
        if (same) return IK_OK;
    }
    if (s.multi) return fail(IK_ERR_INVALID, "multi-device dispatch is already configured differently");
    const int per = env_int("IK_WORKERS_PER_DEVICE", std::max(2, default_threads()));
    for (size_t i = 0; i < ids.size(); ++i) {
        auto L = std::make_unique<Logical>();
        L->phys = ids[i];
        L->pool = new Pool(ids[i], per);  // one pool per LOGICAL device
        s.devs.push_back(std::move(L));
    }
    s.multi = true;
    return IK_OK;
}

void pools_shutdown() {
    Sched& s = sched();
    {
        std::lock_guard<std::mutex> lk(s.mu);
        for (auto& L : s.devs) L->pool->stop();
        // (the Logical records stay allocated: a caller may still hold a pool
        // reference; a later ik_init(-1) configures afresh)
        for (auto& L : s.devs) (void)L.release();
        s.devs.clear();
        s.multi = false;
    }
    std::vector<Pool*> ps;
    {
        std::lock_guard<std::mutex> lk(g_dpool_mu);
        for (auto& kv : g_dpools) ps.push_back(kv.second);
    }
    for (Pool* p : ps) p->stop();
}

bool sched_multi() { return sched().multi; }
int sched_count() { return (int)sched().devs.size(); }
int sched_phys(int ld) { return sched().devs[ld]->phys; }
Pool& sched_pool(int ld) { return *sched().devs[ld]->pool; }

// least outstanding cost; ties to the lowest index
int sched_acquire(uint64_t cost) {
    Sched& s = sched();
    std::lock_guard<std::mutex> lk(s.mu);
    int best = 0;
    uint64_t bv = UINT64_MAX;
    for (size_t i = 0; i < s.devs.size(); ++i) {
        const uint64_t v = s.devs[i]->outstanding.load();
        if (v < bv) { bv = v; best = (int)i; }
    }
    s.devs[best]->outstanding += cost;
    s.devs[best]->jobs += 1;
    return best;
}

int sched_acquire_on(int phys, uint64_t cost) {
    Sched& s = sched();
    std::lock_guard<std::mutex> lk(s.mu);
    int best = -1;
    uint64_t bv = UINT64_MAX;
    for (size_t i = 0; i < s.devs.size(); ++i) {
        if (s.devs[i]->phys != phys) continue;
        const uint64_t v = s.devs[i]->outstanding.load();
        if (v < bv) { bv = v; best = (int)i; }
    }
    if (best >= 0) {
        s.devs[best]->outstanding += cost;
        s.devs[best]->jobs += 1;
    }
    return best;
}

void sched_release(int ld, uint64_t cost) {
    Logical& L = *sched().devs[ld];
    L.outstanding -= cost;
    L.cost_done += cost;
}

// A batch's split over nd logical devices: P = min(nd, n / min_batch) (at least 1)
// contiguous parts of n/P requests (lo[0..P] their bounds), each placed in turn on
// the device with the least outstanding cost (outstanding: nd entries, updated),
// as submit_parts does with the live counters
uint32_t sched_split(const uint64_t* costs, uint32_t n, uint32_t nd, uint32_t min_batch, uint64_t* outstanding,
                     uint32_t* lo, uint32_t* dev) {
    if (!nd || !n) return 0;
    const uint32_t P = std::max<uint32_t>(1, std::min<uint32_t>(nd, n / std::max<uint32_t>(1, min_batch)));
    for (uint32_t q = 0; q <= P; ++q) lo[q] = (uint32_t)((uint64_t)n * q / P);
    for (uint32_t q = 0; q < P; ++q) {
        uint64_t c = 0;
        for (uint32_t i = lo[q]; i < lo[q + 1]; ++i) c += costs[i];
        uint32_t best = 0;
        for (uint32_t d = 1; d < nd; ++d)
            if (outstanding[d] < outstanding[best]) best = d;
        dev[q] = best;
        outstanding[best] += c;
    }
    return P;
}

void sched_plan(const uint64_t* costs, uint32_t n, uint32_t ndev, const uint64_t* outstanding, uint32_t* assign) {
    // longest processing time first: the largest request goes to the least-loaded device
    std::vector<uint64_t> load(ndev, 0);
    if (outstanding) std::copy(outstanding, outstanding + ndev, load.begin());
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return costs[a] > costs[b]; });
    for (uint32_t i : order) {
        uint32_t best = 0;
        for (uint32_t d = 1; d < ndev; ++d)
            if (load[d] < load[best]) best = d;
        assign[i] = best;
        load[best] += costs[i];
    }
}

// partition a batch over the logical devices, accounting the costs as outstanding
void sched_acquire_batch(const uint64_t* costs, uint32_t n, uint32_t* assign) {
    Sched& s = sched();
    std::lock_guard<std::mutex> lk(s.mu);
    const uint32_t nd = (uint32_t)s.devs.size();
    std::vector<uint64_t> out(nd);
    for (uint32_t d = 0; d < nd; ++d) out[d] = s.devs[d]->outstanding.load();
    sched_plan(costs, n, nd, out.data(), assign);
    for (uint32_t i = 0; i < n; ++i) {
        s.devs[assign[i]]->outstanding += costs[i];
        s.devs[assign[i]]->jobs += 1;
    }
}

int sched_stats(uint32_t ld, uint64_t* jobs, uint64_t* cost_done, uint64_t* outstanding) {
    Sched& s = sched();
    if (ld >= s.devs.size()) return fail(IK_ERR_INVALID, "logical device %u out of range", ld);
    if (jobs) *jobs = s.devs[ld]->jobs.load();
    if (cost_done) *cost_done = s.devs[ld]->cost_done.load();
    if (outstanding) *outstanding = s.devs[ld]->outstanding.load();
    return IK_OK;
}

// ---- request cost ------------------------------------------------------------------
namespace {
inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
inline uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
inline uint32_t le24(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16; }
}  // namespace

bool sniff_dims(const uint8_t* b, size_t n, uint32_t& w, uint32_t& h, uint32_t& c) {
    w = h = 0;
    c = 4;
    if (!b) return false;
    switch (guess_format(b, n)) {
    case Sniffed::Png:
        if (n < 33 || std::memcmp(b + 12, "IHDR", 4)) return false;
        w = be32(b + 16);
        h = be32(b + 20);
        c = b[25] == 0 ? 1 : b[25] == 4 ? 2 : b[25] == 2 ? 3 : 4;
        if (b[24] == 16) c *= 2;
        return true;
    case Sniffed::Jpeg: {
        size_t p = 2;
        while (p + 9 < n) {
            if (b[p] != 0xFF) { ++p; continue; }
            const uint8_t m = b[p + 1];
            if (m == 0xFF) { ++p; continue; }
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) { p += 2; continue; }
            const size_t len = (size_t)b[p + 2] << 8 | b[p + 3];
            if ((m >= 0xC0 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                h = (uint32_t)b[p + 5] << 8 | b[p + 6];
                w = (uint32_t)b[p + 7] << 8 | b[p + 8];
                c = b[p + 9] == 1 ? 1 : 3;
                return true;
            }
            p += 2 + len;
        }
        return false;
    }
    case Sniffed::WebP:
        if (n >= 30 && !std::memcmp(b + 12, "VP8 ", 4)) {
            w = le16(b + 26) & 0x3FFF;
            h = le16(b + 28) & 0x3FFF;
            c = 3;
            return true;
        }
        if (n >= 25 && !std::memcmp(b + 12, "VP8L", 4)) {
            const uint32_t v = (uint32_t)b[21] | (uint32_t)b[22] << 8 | (uint32_t)b[23] << 16 | (uint32_t)b[24] << 24;
            w = (v & 0x3FFF) + 1;
            h = ((v >> 14) & 0x3FFF) + 1;
            return true;
        }
        if (n >= 30 && !std::memcmp(b + 12, "VP8X", 4)) {
            w = le24(b + 24) + 1;
            h = le24(b + 27) + 1;
            return true;
        }
        return false;
    default: return false;
    }
}

uint64_t request_cost(const uint8_t* b, size_t n, int64_t w, int64_t h, int fmt) {
    uint32_t W, H, C;
    uint64_t decoded = sniff_dims(b, n, W, H, C) ? (uint64_t)W * H * C : (uint64_t)n * 4;
    // output pixels: the aspect-fit target when both sides are given is at most w*h
    uint64_t out_px;
    if (w < 0 && h < 0) out_px = decoded / std::max<uint32_t>(C, 1);
    else if (w >= 0 && h >= 0) out_px = (uint64_t)std::max<int64_t>(w, 1) * std::max<int64_t>(h, 1);
    else {
        const int64_t s = std::max<int64_t>(w >= 0 ? w : h, 1);
        out_px = (uint64_t)s * s;
    }
    // encoder weight per output pixel (host entropy coding, bytes-equivalent):
    // libwebp VP8 ~ 64, JPEG (GPU Huffman) ~ 4, AV1 at speed 4 ~ 4096
    const uint64_t wgt = fmt == IK_FORMAT_AVIF ? 4096 : fmt == IK_FORMAT_WEBP ? 64 : 4;
    return (uint64_t)n + decoded + out_px * wgt;
}

}  // namespace ik
