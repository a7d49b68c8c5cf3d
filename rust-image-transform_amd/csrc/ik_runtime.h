// ik_runtime.h -- host runtime internals of libimagekit_hip.so (not part of the ABI).
#pragma once
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <unordered_map>

#include "ik_internal.h"

struct ik_image {
    uint32_t w = 0, h = 0, c = 0;  // c interleaved channels
    uint32_t depth = 1;            // bytes per sample: 1 (8-bit) or 2 (16-bit, native-endian u16)
    size_t pitch = 0;              // bytes between rows on the device (multiple of 256)
    uint8_t* d = nullptr;          // device pixels
    bool owned = true;
    int device = 0;
    size_t block = 0;              // bytes of the pooled allocation behind d (owned images)
};

namespace ik {

// thread-local error message + status (ik_last_error)
int fail(int status, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
#define IK_HIP(call)                                    \
    do {                                                \
        hipError_t _e = (call);                         \
        if (_e != hipSuccess) return hip_fail(_e, #call); \
    } while (0)

int current_device();
// make `device` the calling thread's device for the guard's lifetime (an image's
// stages run on the device that holds its pixels)
struct DeviceGuard {
    int prev;
    explicit DeviceGuard(int device);
    ~DeviceGuard();
};

// ---- persistent host workers (ik_pool.cpp) ----
int default_threads();  // IK_THREADS, else min(16, cores)
class Pool {
public:
    Pool(int device, int max_threads);
    // fn(i) for i in [0, n) on up to `threads` threads (the caller included; 0 =
    // default_threads()); returns when every call has returned
    void parallel_for(int n, int threads, const std::function<void(int)>& fn);
    void post(std::function<void()> task);  // run on a worker (device already selected)
    int device() const { return device_; }
    // ik_shutdown: run what is queued, then end and join every worker (each
    // releases its streams and arenas first); the pool takes work again after
    void stop();

private:
    struct Task {
        std::function<void()> fn;
        const void* tag;  // parallel_for helpers: their ForState (withdrawn once it is done)
    };
    void post_tagged(std::function<void()> task, const void* tag);
    void withdraw(const void* tag);
    void ensure(int nthreads);
    void loop();
    int device_, max_threads_;
    int nthreads_ = 0, busy_ = 0;
    bool stop_ = false;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task> q_;
    std::vector<std::thread> threads_;
};
Pool& device_pool(int device);  // the persistent workers of a physical device
// fn(i) for i in [0, n) on the calling thread's device pool (and the caller)
void parallel_for(int n, int threads, const std::function<void(int)>& fn);

// Figures of the last batch each device's kernel stages ran (ik_batch_last_timing):
// device ms from HIP events on the stage's stream and the algorithmic bytes of the
// same launches.  Two records per device, one per stage: the decode stage's fields
// (kBtJpeg* up to kBtJpegLanes) and the post stage's (resize, JPEG encoder); each is
// reset when its stage starts a batch and summed over that batch's launches.
enum BatchTimingField {
    kBtJpegHuffMs = 0,   // JPEG entropy decoding launches (restart intervals / self-sync)
    kBtJpegScanBytes,    // entropy-coded bytes they read
    kBtJpegCoefBytes,    // int16 coefficients they wrote
    kBtJpegImages,
    kBtJpegLanes,        // decoder lanes (restart intervals or self-sync subsequences)
    kBtResizeMs,         // grouped resize launches
    kBtResizeBytes,      // C*W*H in + C*w*h out per image
    kBtResizeImages,
    kBtJpegEncMs,        // batched JPEG encoder (coefficients + Huffman) launches
    kBtJpegEncImages,
    kBtHostWallMs,       // the host coder stage (libwebp / libavif): wall ms of the batch
    kBtHostCoreMs,       // its thread CPU ms summed over the requests (core-ms)
    kBtHostImages,       // requests it coded
    kBtFields
};
// the host coder stage's record of the batch it just finished (set directly: that
// stage runs on the device's worker pool after the post stage committed)
void batch_timing_host(int device, double wall_ms, double core_ms, double images);
void batch_timing_reset(int device, bool post);
void batch_timing_commit(int device, bool post);  // the stage is done: its fields become the last batch's
void batch_timing_add(int device, int field, double v);
// a pair of events on the calling thread (timing one launch sequence); ms between them
struct EvPair {
    hipEvent_t a = nullptr, b = nullptr;
};
EvPair& thread_events(int which);  // which < 4
float ev_pair_ms(const EvPair& e);

// A scope in which batch_timing_add records (the decode and post stages of a
// batch set it on their thread); work outside one -- a single-image ik_decode, a
// pool worker's own resize -- adds nothing to ik_batch_last_timing
struct BatchTimingScope {
    bool prev;
    BatchTimingScope();
    ~BatchTimingScope();
};
// record a timing-only event: a failure is ignored (the pair then reads 0 ms) and
// never changes the caller's path
void ev_record(hipEvent_t e, hipStream_t s);

// The library's lifetime against ik_shutdown / ik_close: every public
// entry point holds the lifetime lock shared for its call (ApiGuard; nested calls
// on one thread take it once), shutdown takes it exclusively, so teardown never
// runs under a caller that is still inside the library (e.g. a daemon thread of
// a server during interpreter exit).  Threads the library owns (pool workers,
// stage threads, pipeline workers) are marked internal and never take it:
// shutdown waits for them while it holds the lock.  After ik_close, entry points
// that take it return IK_ERR_INVALID.
struct ApiGuard {
    bool held = false, closed = false;
    ApiGuard();
    ~ApiGuard();
};
void mark_internal_thread();
#define IK_API_ENTER()                                                                        \
    ::ik::ApiGuard ik_api_guard_;                                                             \
    if (ik_api_guard_.closed) return ::ik::fail(IK_ERR_INVALID, "the library is closed (ik_close)")
#define IK_API_ENTER_VOID()          \
    ::ik::ApiGuard ik_api_guard_;    \
    if (ik_api_guard_.closed) return

// Bytes the library holds, by pool (ik_memory_stats): device image blocks in use
// and kept free for reuse, the per-thread device and pinned arenas, the PNG / JPEG
// upload areas (device, pinned), the cached resize plans' device tables
enum MemStat {
    kMemImageLive = 0, kMemImageFree, kMemArenaDev, kMemArenaPinned, kMemUploadDev, kMemUploadPinned,
    kMemPlans, kMemStats
};
void mem_stat(int which, int64_t delta);

// ik_shutdown: stop and join every pool's workers (device and logical pools);
// multi-device dispatch is unconfigured
void pools_shutdown();
// release the calling thread's streams and arenas (synchronised first); a later
// call on this thread creates them again
void release_thread_resources();
void png_shutdown();    // the PNG upload areas (ik_png_decode.cpp)
void plans_shutdown();  // the cached resize plans (ik_plan.cpp)

// multi-device dispatch (ik_init(-1) / IK_DEVICES): logical devices, least outstanding cost
int sched_configure(const int* devices, int n);
bool sched_multi();
int sched_count();
int sched_phys(int logical);
Pool& sched_pool(int logical);
int sched_acquire(uint64_t cost);
// the least-loaded logical device on physical device `phys` (-1: none)
int sched_acquire_on(int phys, uint64_t cost);
void sched_release(int logical, uint64_t cost);
void sched_acquire_batch(const uint64_t* costs, uint32_t n, uint32_t* assign);
void sched_plan(const uint64_t* costs, uint32_t n, uint32_t ndev, const uint64_t* outstanding, uint32_t* assign);
uint32_t sched_split(const uint64_t* costs, uint32_t n, uint32_t nd, uint32_t min_batch, uint64_t* outstanding,
                     uint32_t* lo, uint32_t* dev);
int sched_stats(uint32_t logical, uint64_t* jobs, uint64_t* cost_done, uint64_t* outstanding);
// header-only dimension sniff (PNG IHDR, JPEG SOFn, WebP VP8/VP8L/VP8X); c = bytes per pixel
bool sniff_dims(const uint8_t* b, size_t n, uint32_t& w, uint32_t& h, uint32_t& c);
uint64_t request_cost(const uint8_t* b, size_t n, int64_t w, int64_t h, int fmt);

hipStream_t thread_stream();  // per-thread, per-device non-blocking stream
hipStream_t thread_copy_stream();  // a second one, for uploads that overlap the first's kernels
// a third, at the highest priority, and an event to order it after the first (the
// exact WebP coder's launches); false if it cannot be made
bool thread_prio_stream(hipStream_t* s, hipEvent_t* ev);
size_t pitch_for(uint32_t w, uint32_t c);
uint8_t* scratch(size_t bytes);  // per-thread device scratch, valid until the next call
// per-thread, per-device grow-only device arenas for batch work (slot 1: JPEG
// batch decode, slot 2: PNG batch decode); valid until the next call with that slot
uint8_t* scratch_slot(int slot, size_t bytes);
uint8_t* pinned_slot(int slot, size_t bytes);  // per-thread grow-only pinned host arenas (slots 0..10)
// the exact WebP coder's arenas: its device work area; its constants in, its records out
constexpr int kScratchExact = 8, kPinnedExactIn = 8, kPinnedExactOut = 9;
// the WebP (VP8) decoder's: its device work area and its staged file + headers
constexpr int kScratchVp8d = 9, kPinnedVp8d = 10;
int copy_h2d_2d(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                size_t height, hipStream_t s);
int copy_d2h_2d(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                size_t height, hipStream_t s);
int alloc_image(uint32_t w, uint32_t h, uint32_t c, ik_image** out, uint32_t depth = 1);

// per-device constant tables (WebP gamma tables)
struct DeviceConsts {
    uint16_t* gamma_to_lin = nullptr;  // [256]
    int* lin_to_gamma = nullptr;       // [33]
    uint32_t* jpeg_huff = nullptr;     // [4][256] standard Huffman tables (k_jpeg_huff_enc)
};
const DeviceConsts* device_consts(int device);
void webp_gamma_tables(uint16_t g2l[256], int l2g[33]);

// host entropy stages (ik_codec.cpp)
int webp_encode_yuv420(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h,
                       float quality, std::vector<uint8_t>& out);
void jpeg_quant_tables(int quality, uint8_t qt[128]);
int avif_encode_yuv444(const uint8_t* planes /* Y, U, V, A */, bool has_alpha, int w, int h, int quality,
                       int speed, std::vector<uint8_t>& out);
void jpeg_write(const int16_t* coef, int w, int h, const uint8_t qt[128], std::vector<uint8_t>& out);
void jpeg_header(int w, int h, const uint8_t qt[128], std::vector<uint8_t>& out);  // SOI .. SOS
void jpeg_huff_u32(uint32_t t[4 * 256]);  // ldc, lac, cdc, cac: code << 8 | size

// the WebP coder encode_image uses unless ik_set_webp_encoder / IK_WEBP_ENCODER says
// otherwise (ik_webp_gpu.cpp)
constexpr int kDefaultWebpEncoder = IK_WEBP_AUTO;
int default_webp_encoder();
// the exact coder (ik_vp8x_host.cpp): libwebp's files from n device YUV420 images
int webp_encode_exact(const uint8_t* d_yuv, size_t yuv_stride, int n, int w, int h, int quality,
                      std::vector<std::vector<uint8_t>>& outs);
// its first stages alone (ik_vp8_analyze_device): segment analysis and set-up on the
// device, the segment map and headers into host memory
int vp8_analyze_setup(const uint8_t* d_yuv, size_t yuv_stride, int n, int w, int h, float quality, uint8_t* seg,
                      ik_vp8_segment_header* hdr);

// host decoders (ik_decode.cpp): tightly packed 8-bit pixels
enum class Sniffed { Png, Jpeg, Gif, WebP, Tiff, Bmp, Ico, Hdr, Avif, OpenExr, Qoi, Farbfeld, Pnm, Dds, Unknown };
Sniffed guess_format(const uint8_t* b, size_t n);
const char* format_name(Sniffed f);
// depth (optional): 16-bit streams decode to native-endian u16 samples (*depth = 2);
// without it they are unsupported
int decode_png(const uint8_t* b, size_t n, uint32_t& w, uint32_t& h, uint32_t& c, std::vector<uint8_t>& px,
               uint32_t* depth = nullptr);
uint32_t png_chunk_crc(const uint8_t* type, const uint8_t* data, size_t len);  // CRC-32 of type + data
// PNG on the GPU (ik_png_decode.cpp + ik_png.hip): inflate + unfilter of n streams
// in one set of launches, straight into new device images; streams the GPU path
// does not cover (or that fail on it) go through decode_png.  Per-stream status
// and message; returns the first failure.
int decode_png_batch(const uint8_t* const* b, const size_t* lens, int n, ik_image** outs, int* status,
                     std::string* msgs);
// decode_png_batch as two stages, so that one batch's upload (PCIe + the GPU
// gather / CRC pass, on the calling thread's copy stream) runs under the previous
// batch's kernels: png_upload_begin parses the streams and issues the upload
// (returns once issued); png_decode_finish, on the kernel stage's thread, runs the
// decode kernels once the upload has landed.  The input arrays stay valid until
// finish returns; every begin is finished exactly once.
struct PngBatchState;
struct PngUpload {
    const uint8_t* const* bytes = nullptr;
    const size_t* lens = nullptr;
    int n = 0;
    std::shared_ptr<PngBatchState> st;
    // dev: bytes[i] are device addresses on the calling thread's device (the
    // caller's files already in HBM), heads[i] a host copy of each file's first 8
    // bytes; the upload then walks the chunks on the GPU and gathers from there
    bool dev = false;
    const uint8_t* const* heads = nullptr;
    // called by png_decode_finish once the batch's decode rounds are done (argument:
    // an event to wait for first, or null): the stage executor launches the next
    // batch's block search there, on the kernel stream before this batch's expand
    // (beside the unfilter instead it doubled the unfilter: profiles/r04k_*)
    std::function<void(hipEvent_t)> on_next_search;
};
int png_upload_begin(const uint8_t* const* b, const size_t* lens, int n, PngUpload& up);
int png_decode_finish(PngUpload& up, ik_image** outs, int* status, std::string* msgs);
// the block search of an issued upload, on stream s (after the upload lands);
// png_decode_finish then only waits for it.  Kernel-stage thread only.
void png_find_prelaunch(PngUpload& up, hipStream_t s);
bool png_find_beside_decode();  // IK_FIND_BESIDE: the next batch's block search beside the decode (experiment)
bool png_upload_landed(const PngUpload& up);  // its upload + gather pass have completed (nothing to wait for)
constexpr int kPngTimingFields = 17;  // ik_png_last_timing
// caller-pinned host memory (ik_host_alloc / ik_host_register): [p, p + n) lies
// inside one such range, so DMAs may read it in place
bool host_pinned(const void* p, size_t n);
bool png_gpu_enabled(size_t raw_bytes);  // IK_PNG_GPU / IK_PNG_GPU_MIN policy
int decode_webp(const uint8_t* b, size_t n, uint32_t& w, uint32_t& h, uint32_t& c, std::vector<uint8_t>& px);
// WebP lossy ("VP8 ", no alpha, no animation) on the GPU (ik_vp8d_host.cpp + ik_vp8d.hip):
// the host parses the headers and partition 0, the device decodes the tokens,
// reconstructs, loop-filters and converts to RGB straight into a new device image.
// Returns kVp8dHost (nothing recorded) for files it leaves to decode_webp: other
// WebP kinds, anything its parser finds unusual, data that runs out.
constexpr int kVp8dHost = -1000;
int decode_webp_device(const uint8_t* b, size_t n, ik_image** out);
// IK_WEBP_DECODE (read per call): 0 "host" (libwebp only), 2 "gpu" (every size; a file
// the GPU path leaves to the host is an error instead: the tests' proof that it ran),
// 1 otherwise (auto: the GPU path from 3 MPix, where it is faster than libwebp)
int webp_decode_mode();

// JPEG: host entropy decode + GPU reconstruction straight into a new device image
// (ik_jpeg_decode.cpp + ik_jpeg.hip)
int decode_jpeg_device(const uint8_t* b, size_t n, ik_image** out);
// A batch's JPEG files DMAed to the device by the upload stage (ik_host.cpp
// StageExec), so that the kernel stage's self-synchronising decoder reads their
// scans where they lie instead of copying them in its own time.  The files of the
// batch in one device area (two per device, as the PNG upload areas), DMAed in
// place when the caller pinned them, else through pinned staging; `ev` marks the
// DMAs' end on the upload thread's stream.  Dropping the JpegUpload (after the
// batch's decode returned) frees the area for the next batch.
struct JpegArea;
struct JpegUpload {
    int n = 0;
    std::unordered_map<const uint8_t*, const uint8_t*> dev;  // host file -> its device copy
    hipEvent_t ev = nullptr;
    std::shared_ptr<JpegArea> area;
};
int jpeg_upload_begin(const uint8_t* const* b, const size_t* lens, int n, JpegUpload& up);
void jpeg_shutdown();  // ik_shutdown: the JPEG upload areas
// n streams at once: baseline scans entropy-decoded together by the self-
// synchronising GPU decoder; per-stream status (outs[i] null on failure); returns
// the first failure.  up: the files' device copies (jpeg_upload_begin), or null
int decode_jpeg_batch(const uint8_t* const* b, const size_t* lens, int n, ik_image** outs, int* status,
                      std::string* msgs /* [n] or null: per-stream error message */,
                      const JpegUpload* up = nullptr);

// device-side stage helpers used by ik_encode and the pipeline
int encode_device_image(const uint8_t* dev, uint32_t w, uint32_t h, uint32_t c, size_t pitch,
                        int fmt, int quality, std::vector<uint8_t>& out);
// encode_image in two halves: the device front end (colour conversion, FDCT and
// Huffman coding for JPEG) leaves either the final bytes (done) or the planes the
// host coder takes (WebP YUV420, AVIF YUV444 + alpha); the back end runs that
// host coder (libwebp / libavif) and touches no device
struct EncodePrep {
    int fmt = -1, q = 0;
    uint32_t w = 0, h = 0;
    bool done = false, transparent = false;
    std::vector<uint8_t> planes;
    // or the planes in a shared page-locked block written by a batched colour
    // launch (webp_front_group): no copy into `planes`; the block returns to its
    // pool when the last request holding it is coded
    std::shared_ptr<uint8_t> pin_block;
    const uint8_t* pin_planes = nullptr;
    const uint8_t* plane_data() const { return pin_planes ? pin_planes : planes.data(); }
};
int encode_device_front(const uint8_t* dev, uint32_t w, uint32_t h, uint32_t c, size_t pitch, int fmt, int quality,
                        EncodePrep& p, std::vector<uint8_t>& out);
int encode_image_front(const ik_image* img, int fmt, int quality, EncodePrep& p, std::vector<uint8_t>& out);
int encode_host_back(EncodePrep& p, std::vector<uint8_t>& out);

// resize_image's output size (src/transform.rs:62-90 + DynamicImage::resize) and
// a one-launch resize of same-geometry 8-bit images (ik_host.cpp)
int resize_target(uint32_t W, uint32_t H, int64_t w, int64_t h, uint32_t* nw, uint32_t* nh);
int resize_group(const std::vector<ik_image*>& src, uint32_t nw, uint32_t nh, int filter, std::vector<ik_image*>& out);

// Per-device phase gates (ik_pool.cpp).  Concurrent batch calls on one device
// take its GPU phases in turn: kGateUpload covers a PNG batch's staging, H2D and
// block search, kGateKernels the decode kernels, kGatePost the resize and the
// encoders' device front ends (so one batch's resize runs beside the next batch's
// decode kernels).  A batch's host phases (libwebp / libavif coding) run outside
// all three, beside the next batch's kernels; its small kernels never queue
// behind another batch's long ones.  gate_pin keeps a gate held across
// gate_leave (a caller that spans several phases).
enum { kGateUpload = 0, kGateKernels = 1, kGatePost = 2 };
void gate_enter(int which);
bool gate_try_enter(int which);  // true if now held (or gates are off)
bool gate_held_any();            // this thread holds one of its device's gates
void gate_leave(int which);
void gate_pin(int which, bool on);

}  // namespace ik
