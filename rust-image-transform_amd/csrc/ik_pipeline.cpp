// ik_pipeline.cpp -- batched transform over device-resident images (the
// throughput path behind the /img and /upload handlers, src/lib.rs:175-191 and
// :281-297, when many requests are in flight).
//
// Per batch: ONE resize launch over the whole batch (k_resize_fused, pixels HBM ->
// LDS -> HBM), ONE colour-convert launch (WebP YUV420 planes or JPEG quantised
// coefficients), one D2H copy of the small planes into pinned memory, then the host
// entropy stage (libwebp VP8 / AV1 / the JPEG segments the GPU Huffman coder wrote;
// with the exact WebP coder, ik_vp8x.hip's one launch per batch) over a
// persistent thread pool, one image per task -- the reference runs one
// synchronous transform per tokio worker (src/main.rs:20), so per-image serial
// entropy coding across cores is the same structure.  submit / collect keep two
// batches in flight, so the host stage of one overlaps the device stage of the
// next; run = submit + collect.
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {
namespace {

class CoderPool {
public:
    explicit CoderPool(int n) {
        for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    ~CoderPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    // run fn(i) for i in [0, n) on the workers (and the caller), wait for all
    void run(int n, const std::function<void(int)>& fn) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_ == n_; });
        fn_ = nullptr;
    }

private:
    void work() {
        for (;;) {
            const int i = next_.fetch_add(1);
            if (i >= n_) return;
            (*fn_)(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (++done_ == n_) done_cv_.notify_all();
        }
    }
    void loop() {
        mark_internal_thread();  // the library's own thread: no lifetime lock (ApiGuard)
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (gen_ != seen && fn_ != nullptr); });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, done_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace
}  // namespace ik

struct ik_pipeline {
    int device = 0;
    hipStream_t stream = nullptr;   // resize + colour convert (+ host copies)
    hipStream_t stream2 = nullptr;  // (spare stream, kept for the ABI's event layout)
    uint32_t W = 0, H = 0, C = 0, nw = 0, nh = 0, max_batch = 0;
    int filter = 4, fmt = 1, quality = 80;
    uint8_t* d_resized = nullptr;
    size_t r_pitch = 0, r_img_stride = 0;
    uint8_t* d_stage = nullptr;  // per slot: YUV planes or int16 coefficients, per image
    size_t stage_bytes = 0;
    uint8_t* d_qt = nullptr;
    uint8_t qt[128];
    float* d_tmp = nullptr;      // naive resize path only
    int webp_enc = IK_WEBP_LIBWEBP;  // IK_WEBP_EXACT: the exact GPU coder in the collect stage
    uint8_t* d_jwork = nullptr;      // JPEG: k_jpeg_huff_enc work (2 * jcap per image)
    size_t jcap = 0;
    std::vector<uint8_t> jpeg_hdr;   // SOI .. SOS for this geometry and quality
    // Two slots: the device stage of batch k+1 (enqueued by submit) runs while
    // the host entropy stage of batch k (collect) works from its slot.  The
    // resized images are shared (stream order); each slot has its own stage
    // planes on the device, so the exact WebP coder of batch k (collect) reads its
    // slot's planes while the resize of batch k+1 runs.
    struct Slot {
        uint8_t* h_stage = nullptr;       // pinned planes / coefficients
        uint8_t* h_jpeg = nullptr;        // pinned entropy-coded JPEG segments (k_jpeg_huff_enc), jcap apart
        uint32_t* h_jlen = nullptr;       // their lengths
        int* d_aflag = nullptr;           // AVIF: per image, 1 when any alpha < 255 (k_avif_yuv444)
        int* h_aflag = nullptr;           // their pinned copies
        // resize start / end, colour end, stage end, copies end, stage start
        hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        uint8_t* d_stage = nullptr;       // this slot's part of ik_pipeline::d_stage
        uint32_t n = 0;
        bool exact = false;  // WebP: the exact GPU coder codes this slot's planes in collect
    } slot[2];
    int head = 0, inflight = 0;
    double ms[4] = {0, 0, 0, 0};
    uint32_t last_n = 0;
    ik::CoderPool* pool = nullptr;
    std::vector<std::vector<uint8_t>> outs;
    std::vector<int> status;
};

using namespace ik;

namespace {

int check_batch(const ik_pipeline* p, const uint8_t* dev_src, size_t src_pitch, size_t src_image_stride, uint32_t n) {
    if (!p || !dev_src || !n || n > p->max_batch) return fail(IK_ERR_INVALID, "bad batch");
    if (src_pitch < (size_t)p->W * p->C || (src_pitch & 7) || ((uintptr_t)dev_src & 7))
        return fail(IK_ERR_INVALID, "source rows must be 8-byte aligned and >= W*C");
    if (n > 1 && src_image_stride < src_pitch * p->H) return fail(IK_ERR_INVALID, "image stride too small");
    if (!resize_fused_fits(src_pitch, p->H) && !p->d_tmp)  // (created for tightly packed rows under 2 GiB)
        return fail(IK_ERR_INVALID, "source image over 2 GiB at this pitch: use ik_resize_batch_device");
    return IK_OK;
}

// device stage of one batch on the pipeline's stream, events into slot s; with
// copy_out, also the D2H of what the host stage needs (no synchronisation)
int enqueue(ik_pipeline* p, ik_pipeline::Slot& s, const uint8_t* dev_src, size_t src_pitch, size_t src_image_stride,
            uint32_t n, bool copy_out) {
    IK_HIP(hipSetDevice(p->device));
    ResizePlan* plan = get_resize_plan(p->device, (int)p->W, (int)p->H, (int)p->C, (int)p->nw, (int)p->nh,
                                       p->filter, (int)p->max_batch);
    if (!plan) return fail(IK_ERR_DEVICE, "cannot build resize plan");
    s.exact = p->fmt == IK_FORMAT_WEBP && p->webp_enc == IK_WEBP_EXACT;
    s.n = n;
    IK_HIP(hipEventRecord(s.ev[0], p->stream));
    IK_HIP(launch_resize(*plan, dev_src, src_pitch, src_image_stride, p->d_resized, p->r_pitch,
                         p->r_img_stride, (int)n, p->d_tmp, p->stream));
    IK_HIP(hipEventRecord(s.ev[1], p->stream));
    // the slot's stage planes were last read two batches back (collected before
    // this submit: the host stage waited for them)
    if (p->fmt == IK_FORMAT_AVIF) {
        IK_HIP(launch_avif_yuv444(p->d_resized, (int)p->nw, (int)p->nh, (int)p->C, p->r_pitch, p->r_img_stride,
                                  s.d_stage, p->stage_bytes, s.d_aflag, (int)n, p->stream));
    } else if (p->fmt == IK_FORMAT_WEBP) {
        const DeviceConsts* dc = device_consts(p->device);
        IK_HIP(launch_webp_yuv420(p->d_resized, (int)p->nw, (int)p->nh, (int)p->C, p->r_pitch,
                                  p->r_img_stride, s.d_stage, p->stage_bytes, (int)n,
                                  dc->gamma_to_lin, dc->lin_to_gamma, p->stream));
    } else {
        IK_HIP(launch_jpeg_coeffs(p->d_resized, (int)p->nw, (int)p->nh, (int)p->C, p->r_pitch,
                                  p->r_img_stride, p->d_qt, (int16_t*)s.d_stage,
                                  p->stage_bytes / sizeof(int16_t), (int)n, p->stream));
    }
    IK_HIP(hipEventRecord(s.ev[2], p->stream));
    {
        IK_HIP(hipEventRecord(s.ev[5], p->stream));
        if (copy_out && p->fmt == IK_FORMAT_JPEG) {  // Huffman coding on the GPU, straight into pinned memory
            JpegEncArgs ja{};
            ja.coef = reinterpret_cast<const int16_t*>(s.d_stage);
            ja.coef_img_stride = p->stage_bytes / sizeof(int16_t);
            ja.nmcu = (int)(((p->nw + 7) / 8) * ((p->nh + 7) / 8));
            ja.huff = device_consts(p->device)->jpeg_huff;
            ja.work = p->d_jwork;
            ja.work_img_bytes = 2 * p->jcap;
            ja.words_bytes = p->jcap;
            ja.out = s.h_jpeg;
            ja.out_img_stride = p->jcap;
            ja.out_cap = p->jcap;
            ja.out_len = s.h_jlen;
            IK_HIP(launch_jpeg_huff_enc(ja, (int)n, p->stream));
        }
        IK_HIP(hipEventRecord(s.ev[3], p->stream));
        if (copy_out && p->fmt != IK_FORMAT_JPEG && !s.exact)
            IK_HIP(hipMemcpyAsync(s.h_stage, s.d_stage, p->stage_bytes * n, hipMemcpyDeviceToHost, p->stream));
        if (copy_out && p->fmt == IK_FORMAT_AVIF)
            IK_HIP(hipMemcpyAsync(s.h_aflag, s.d_aflag, sizeof(int) * n, hipMemcpyDeviceToHost, p->stream));
        IK_HIP(hipEventRecord(s.ev[4], p->stream));
    }
    return IK_OK;
}

int finish_device(ik_pipeline* p, ik_pipeline::Slot& s) {
    IK_HIP(hipEventSynchronize(s.ev[4]));
    float a = 0, b = 0, c = 0;
    IK_HIP(hipEventElapsedTime(&a, s.ev[0], s.ev[1]));
    IK_HIP(hipEventElapsedTime(&b, s.ev[1], s.ev[2]));
    IK_HIP(hipEventElapsedTime(&c, s.ev[5], s.ev[3]));
    p->ms[0] = a;
    p->ms[1] = b;
    p->ms[2] = 0.0;
    (void)c;
    p->last_n = s.n;
    return IK_OK;
}

// host entropy stage of a finished slot; bytes back to back into out
int host_stage(ik_pipeline* p, const ik_pipeline::Slot& s, uint8_t* out, size_t out_cap, size_t* out_sizes) {
    const uint32_t n = s.n;
    const auto t0 = std::chrono::steady_clock::now();
    p->outs.resize(n);
    p->status.assign(n, 0);
    std::vector<std::string> errs(n);
    if (s.exact) {  // libwebp's decisions on the GPU for the whole batch, the files on the host
        DeviceGuard g(p->device);
        if (int rc = webp_encode_exact(s.d_stage, p->stage_bytes, (int)n, (int)p->nw, (int)p->nh, p->quality, p->outs))
            return rc;
    }
    p->pool->run(s.exact ? 0 : (int)n, [&](int i) {
        const uint8_t* st = s.h_stage + p->stage_bytes * (size_t)i;
        if (p->fmt == IK_FORMAT_AVIF) {
            // image 0.25.8 AvifEncoder::new_with_speed_quality(out, 4, q) (src/transform.rs:140-145)
            p->status[i] = avif_encode_yuv444(st, s.h_aflag[i] != 0, (int)p->nw, (int)p->nh, p->quality, 4,
                                              p->outs[i]);
            if (p->status[i]) {
                char buf[256];
                ik_last_error(buf, sizeof(buf));
                errs[i] = buf;
            }
        } else if (p->fmt == IK_FORMAT_WEBP) {
            const size_t ys = (size_t)p->nw * p->nh, uvs = (size_t)((p->nw + 1) / 2) * ((p->nh + 1) / 2);
            p->status[i] = webp_encode_yuv420(st, st + ys, st + ys + uvs, (int)p->nw, (int)p->nh,
                                              (float)p->quality, p->outs[i]);
            if (p->status[i]) {
                char buf[256];
                ik_last_error(buf, sizeof(buf));
                errs[i] = buf;
            }
        } else if (s.h_jlen[i] != 0xffffffffu) {  // GPU-coded segment: header + bytes + EOI
            const uint32_t len = s.h_jlen[i];
            std::vector<uint8_t>& o = p->outs[i];
            o.resize(p->jpeg_hdr.size() + len + 2);
            std::memcpy(o.data(), p->jpeg_hdr.data(), p->jpeg_hdr.size());
            std::memcpy(o.data() + p->jpeg_hdr.size(), s.h_jpeg + p->jcap * (size_t)i, len);
            o[o.size() - 2] = 0xFF;
            o[o.size() - 1] = 0xD9;
        } else {  // did not fit the GPU coder's buffer: coefficients back, host coder
            std::vector<int16_t> coef(p->stage_bytes / sizeof(int16_t));
            if (hipMemcpy(coef.data(), s.d_stage + p->stage_bytes * (size_t)i, p->stage_bytes,
                          hipMemcpyDeviceToHost) != hipSuccess) {
                p->status[i] = IK_ERR_DEVICE;
                errs[i] = "coefficient copy failed";
                return;
            }
            jpeg_write(coef.data(), (int)p->nw, (int)p->nh, p->qt, p->outs[i]);
        }
    });
    p->ms[3] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    size_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (p->status[i]) return fail(p->status[i], "image %u: %s", i, errs[i].c_str());
        if (out_sizes) out_sizes[i] = p->outs[i].size();
        if (out) {
            if (off + p->outs[i].size() > out_cap) return fail(IK_ERR_INVALID, "output buffer too small");
            std::memcpy(out + off, p->outs[i].data(), p->outs[i].size());
        }
        off += p->outs[i].size();
    }
    return IK_OK;
}

}  // namespace

extern "C" {

namespace {
int pipeline_create(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter, int fmt, int quality,
                    uint32_t max_batch, int threads, ik_pipeline* p);
}  // namespace

int ik_pipeline_create(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter,
                       int fmt, int quality, uint32_t max_batch, int threads, ik_pipeline** out) {
    IK_API_ENTER();
    if (!out || !W || !H || !nw || !nh || !max_batch || C < 1 || C > 4) return fail(IK_ERR_INVALID, "bad geometry");
    if (fmt != IK_FORMAT_WEBP && fmt != IK_FORMAT_JPEG && fmt != IK_FORMAT_AVIF)
        return fail(IK_ERR_INVALID, "unknown ImageFormat %d", fmt);
    auto* p = new ik_pipeline();
    const int rc = pipeline_create(W, H, C, nw, nh, filter, fmt, quality, max_batch, threads, p);
    if (rc) {  // release whatever was allocated before the failure
        ik_pipeline_destroy(p);
        return rc;
    }
    *out = p;
    // EXACT, or AUTO with batches of 32+ frames (the rule of a batch's same-geometry
    // groups, ik_host.cpp kAutoExactMinGroup)
    const int enc = default_webp_encoder();
    if (fmt == IK_FORMAT_WEBP && (enc == IK_WEBP_EXACT || (enc == IK_WEBP_AUTO && max_batch >= 32)))
        return ik_pipeline_set_webp_encoder(p, IK_WEBP_EXACT);
    return IK_OK;
}

}  // extern "C"

namespace {
int pipeline_create(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter, int fmt, int quality,
                    uint32_t max_batch, int threads, ik_pipeline* p) {
    p->device = current_device();
    IK_HIP(hipSetDevice(p->device));
    p->W = W; p->H = H; p->C = C; p->nw = nw; p->nh = nh; p->max_batch = max_batch;
    p->filter = filter; p->fmt = fmt;
    p->quality = quality < 1 ? 1 : quality > 100 ? 100 : quality;
    IK_HIP(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    IK_HIP(hipStreamCreateWithFlags(&p->stream2, hipStreamNonBlocking));
    for (auto& sl : p->slot)
        for (auto& e : sl.ev) IK_HIP(hipEventCreate(&e));
    p->r_pitch = pitch_for(nw, C);
    p->r_img_stride = p->r_pitch * nh;
    IK_HIP(hipMalloc(&p->d_resized, p->r_img_stride * max_batch + 16));
    if (fmt == IK_FORMAT_WEBP) {
        const size_t uvw = (nw + 1) / 2, uvh = (nh + 1) / 2;
        p->stage_bytes = (size_t)nw * nh + 2 * uvw * uvh;
    } else if (fmt == IK_FORMAT_AVIF) {  // Y, U, V, A planes (4:4:4), 256-B aligned per image
        p->stage_bytes = (4 * (size_t)nw * nh + 255) & ~(size_t)255;
        for (auto& sl : p->slot) {
            IK_HIP(hipMalloc(&sl.d_aflag, sizeof(int) * max_batch));
            IK_HIP(hipHostMalloc(&sl.h_aflag, sizeof(int) * max_batch, hipHostMallocDefault));
        }
    } else {
        p->stage_bytes = (size_t)((nw + 7) / 8) * ((nh + 7) / 8) * 3 * 64 * sizeof(int16_t);
        jpeg_quant_tables(p->quality, p->qt);
        jpeg_header((int)nw, (int)nh, p->qt, p->jpeg_hdr);
        p->jcap = jpeg_enc_cap((int)nw, (int)nh);
        IK_HIP(hipMalloc(&p->d_jwork, 2 * p->jcap * max_batch));
        for (auto& sl : p->slot) {
            IK_HIP(hipHostMalloc(&sl.h_jpeg, p->jcap * max_batch, hipHostMallocDefault));
            IK_HIP(hipHostMalloc(&sl.h_jlen, sizeof(uint32_t) * max_batch, hipHostMallocDefault));
        }
        if (!device_consts(p->device)) return fail(IK_ERR_DEVICE, "cannot upload JPEG tables");
        IK_HIP(hipMalloc(&p->d_qt, 128));
        if (int rc = copy_h2d_2d(p->d_qt, 128, p->qt, 128, 128, 1, p->stream)) return rc;
    }
    IK_HIP(hipMalloc(&p->d_stage, 2 * p->stage_bytes * max_batch));
    p->slot[0].d_stage = p->d_stage;
    p->slot[1].d_stage = p->d_stage + p->stage_bytes * max_batch;
    for (auto& sl : p->slot) IK_HIP(hipHostMalloc(&sl.h_stage, p->stage_bytes * max_batch, hipHostMallocDefault));
    ResizePlan* plan = get_resize_plan(p->device, (int)W, (int)H, (int)C, (int)nw, (int)nh, filter, (int)max_batch);
    if (!plan) return fail(IK_ERR_DEVICE, "cannot build resize plan");
    if (plan->slots == 0 || !resize_fused_fits((size_t)W * C, H))  // naive path: its intermediate rows
        IK_HIP(hipMalloc(&p->d_tmp, sizeof(float) * (size_t)max_batch * nh * W * C));
    if (threads <= 0) {
        threads = (int)std::thread::hardware_concurrency();
        if (threads > 16) threads = 16;
        if (threads < 1) threads = 1;
    }
    p->pool = new CoderPool(threads - 1);  // the calling thread works too
    if (fmt == IK_FORMAT_WEBP && !device_consts(p->device)) return fail(IK_ERR_DEVICE, "cannot upload WebP tables");
    return IK_OK;
}
}  // namespace

extern "C" {

int ik_pipeline_set_webp_encoder(ik_pipeline* p, int encoder) {
    IK_API_ENTER();
    if (!p) return fail(IK_ERR_INVALID, "null pipeline");
    if (encoder != IK_WEBP_LIBWEBP && encoder != IK_WEBP_EXACT) return fail(IK_ERR_INVALID, "bad WebP encoder %d", encoder);
    if (p->fmt != IK_FORMAT_WEBP) return fail(IK_ERR_INVALID, "not a WebP pipeline");
    if (p->inflight) return fail(IK_ERR_INVALID, "batches in flight: collect them first");
    if (encoder == IK_WEBP_EXACT && (p->nw > 16383 || p->nh > 16383))
        return fail(IK_ERR_TRANSFORM, "WebP dimensions exceed 16383");
    p->webp_enc = encoder;
    return IK_OK;
}

int ik_pipeline_run_device(ik_pipeline* p, const uint8_t* dev_src, size_t src_pitch,
                           size_t src_image_stride, uint32_t n) {
    IK_API_ENTER();
    if (int rc = check_batch(p, dev_src, src_pitch, src_image_stride, n)) return rc;
    if (p->inflight) return fail(IK_ERR_INVALID, "batches in flight: collect them first");
    if (int rc = enqueue(p, p->slot[0], dev_src, src_pitch, src_image_stride, n, false)) return rc;
    return finish_device(p, p->slot[0]);
}

int ik_pipeline_submit(ik_pipeline* p, const uint8_t* dev_src, size_t src_pitch, size_t src_image_stride,
                       uint32_t n) {
    IK_API_ENTER();
    if (int rc = check_batch(p, dev_src, src_pitch, src_image_stride, n)) return rc;
    if (p->inflight >= 2) return fail(IK_ERR_INVALID, "two batches already in flight: collect one first");
    ik_pipeline::Slot& s = p->slot[p->head & 1];
    if (int rc = enqueue(p, s, dev_src, src_pitch, src_image_stride, n, true)) return rc;
    ++p->head;
    ++p->inflight;
    return IK_OK;
}

int ik_pipeline_collect(ik_pipeline* p, uint8_t* out, size_t out_cap, size_t* out_sizes, uint32_t* n_out) {
    IK_API_ENTER();
    if (!p) return fail(IK_ERR_INVALID, "null pipeline");
    if (!p->inflight) return fail(IK_ERR_INVALID, "no batch in flight");
    ik_pipeline::Slot& s = p->slot[(p->head - p->inflight) & 1];
    --p->inflight;  // the slot is free again whatever happens below
    if (n_out) *n_out = s.n;
    if (int rc = finish_device(p, s)) return rc;
    return host_stage(p, s, out, out_cap, out_sizes);
}

int ik_pipeline_run(ik_pipeline* p, const uint8_t* dev_src, size_t src_pitch, size_t src_image_stride,
                    uint32_t n, uint8_t* out, size_t out_cap, size_t* out_sizes) {
    IK_API_ENTER();
    if (p && p->inflight) return fail(IK_ERR_INVALID, "batches in flight: collect them first");
    if (int rc = ik_pipeline_submit(p, dev_src, src_pitch, src_image_stride, n)) return rc;
    return ik_pipeline_collect(p, out, out_cap, out_sizes, nullptr);
}

double ik_pipeline_kernel_ms(const ik_pipeline* p, int which) {
    if (!p || which < 0 || which > 3) return -1.0;
    return p->ms[which];
}

int ik_pipeline_fetch_resized(ik_pipeline* p, uint32_t i, uint8_t* dst, size_t cap) {
    IK_API_ENTER();
    if (!p || !dst || i >= p->last_n) return fail(IK_ERR_INVALID, "bad image index");
    const size_t row = (size_t)p->nw * p->C;
    if (cap < row * p->nh) return fail(IK_ERR_INVALID, "destination too small");
    return copy_d2h_2d(dst, row, p->d_resized + p->r_img_stride * i, p->r_pitch, row, p->nh, p->stream);
}

void ik_pipeline_destroy(ik_pipeline* p) {
    IK_API_ENTER_VOID();
    if (!p) return;
    (void)hipSetDevice(p->device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    if (p->stream2) (void)hipStreamSynchronize(p->stream2);
    delete p->pool;
    if (p->d_resized) (void)hipFree(p->d_resized);
    if (p->d_stage) (void)hipFree(p->d_stage);
    if (p->d_qt) (void)hipFree(p->d_qt);
    if (p->d_tmp) (void)hipFree(p->d_tmp);
    if (p->d_jwork) (void)hipFree(p->d_jwork);
    for (auto& sl : p->slot) {
        if (sl.h_stage) (void)hipHostFree(sl.h_stage);
        if (sl.h_jpeg) (void)hipHostFree(sl.h_jpeg);
        if (sl.h_jlen) (void)hipHostFree(sl.h_jlen);
        if (sl.d_aflag) (void)hipFree(sl.d_aflag);
        if (sl.h_aflag) (void)hipHostFree(sl.h_aflag);
        for (auto& e : sl.ev)
            if (e) (void)hipEventDestroy(e);
    }
    if (p->stream) (void)hipStreamDestroy(p->stream);
    if (p->stream2) (void)hipStreamDestroy(p->stream2);
    delete p;
}

}  // extern "C"
