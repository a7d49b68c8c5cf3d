/*
 * imagekit_hip.h -- C ABI of libimagekit_hip.so, the MI355X-native drop-in for
 * the reference's transform hot path (Shreyas2409/Rust-Image-Transform,
 * crate `imagekit`, module `imagekit::transform`).
 *
 * The reference has no plugin registry: its "operator API" is three free Rust
 * functions (src/transform.rs) called by the /img and /upload handlers
 * (src/lib.rs:175,180,188 and :281,286,294).  Each entry point below names the
 * reference item it replaces.  Plain pointers and sizes only; images are
 * device-resident handles (ik_image) so a decode -> resize -> encode chain
 * keeps pixels in HBM.  All functions are thread-safe; errors are reported as
 * an ik_status plus a thread-local message (ik_last_error), never a panic or
 * abort across the ABI (reference: every failure maps to
 * ImageKitError::TransformError, src/lib.rs:34-52).
 */
#ifndef IMAGEKIT_HIP_H
#define IMAGEKIT_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ImageFormat (reference src/config.rs:11-17): jpeg, webp, avif */
typedef enum { IK_FORMAT_JPEG = 0, IK_FORMAT_WEBP = 1, IK_FORMAT_AVIF = 2 } ik_format;

/* image::imageops::FilterType (image 0.25.8).  The reference always uses
 * Lanczos3 (src/transform.rs:88); the others are extensions. */
typedef enum {
    IK_FILTER_NEAREST = 0,
    IK_FILTER_TRIANGLE = 1,
    IK_FILTER_CATMULLROM = 2,
    IK_FILTER_GAUSSIAN = 3,
    IK_FILTER_LANCZOS3 = 4
} ik_filter;

typedef enum {
    IK_OK = 0,
    IK_ERR_TRANSFORM = 1,   /* ImageKitError::TransformError (decode/encode failure) */
    IK_ERR_INVALID = 2,     /* bad argument (null pointer, zero size, bad enum)    */
    IK_ERR_DEVICE = 3,      /* HIP runtime failure                                  */
    IK_ERR_UNSUPPORTED = 4, /* recognised but not compiled in (e.g. AVIF decode)    */
    IK_ERR_NOMEM = 5
} ik_status;

/* DynamicImage (image 0.25.8): 8-bit, 1..4 interleaved channels
 * (Luma8, LumaA8, Rgb8, Rgba8), pixels resident in device memory. */
typedef struct ik_image ik_image;

/* ---- runtime ---------------------------------------------------------- */
/* ik_init(d >= 0): select HIP device d for the calling thread.
 * ik_init(-1): one process drives every visible GPU (or the list in IK_DEVICES,
 *   e.g. "0,1,2,3"; a device may repeat, "0,0" = two logical devices on GPU 0).
 *   From then on ik_transform / ik_transform_batch / ik_decode called from any
 *   number of threads feed a host work queue: each request goes to the logical
 *   device with the least outstanding cost (ik_request_cost), and runs there on
 *   that device's persistent workers.  The reference's analogue is tokio's
 *   multi-thread runtime calling the transform from every worker
 *   (src/main.rs:20, src/lib.rs:175-191). */
int ik_init(int device);
int ik_init_devices(const int *devices, int n); /* ik_init(-1) with an explicit list */
int ik_device_count(void);
int ik_logical_device_count(void);  /* 0 unless multi-device dispatch is on */
/* per logical device: requests taken, cost completed, cost still outstanding */
int ik_logical_device_stats(uint32_t logical, uint64_t *jobs, uint64_t *cost_done, uint64_t *outstanding);
/* the scheduler's cost of one request, in bytes-equivalent: encoded input +
 * decoded pixels (from the header) + an encoder weight per output pixel */
uint64_t ik_request_cost(const uint8_t *bytes, size_t len, int64_t w, int64_t h, int fmt);
/* the batch placement policy on its own (no device work): n requests with
 * costs[i] over ndev devices already carrying outstanding[d] (may be NULL) ->
 * assign[i]; largest request first to the least-loaded device */
void ik_schedule_plan(const uint64_t *costs, uint32_t n, uint32_t ndev, const uint64_t *outstanding,
                      uint32_t *assign);
/* a batch submit's split over ndev logical devices on its own (no device work):
 * min(ndev, n / min_batch) contiguous parts (at least one) -- part q is requests
 * [part_lo[q], part_lo[q+1]) (part_lo: ndev + 1 entries) -- each placed in turn on
 * the least-loaded device (part_dev[q]); returns the part count.  submit uses it
 * with min_batch = IK_MIN_DEVICE_BATCH (64). */
uint32_t ik_schedule_split(const uint64_t *costs, uint32_t n, uint32_t ndev, const uint64_t *outstanding,
                           uint32_t min_batch, uint32_t *part_lo, uint32_t *part_dev);
/* Orderly teardown: waits for every submitted batch, ends
 * the library's stage threads and worker pools (each releases its HIP streams
 * and arenas), then frees the pooled images, upload areas, resize plans and
 * pinned blocks -- while the HIP runtime is still alive, so that nothing is left
 * to destructors running at process exit.  Call it once before exit (the Python
 * package registers it with atexit; the Rust shim calls it from Drop of its
 * runtime guard).  Images, pipelines and buffers the caller still holds must be
 * freed first; the library may be used again afterwards (ik_init).  Callers
 * still inside the library on other threads return first: every entry point
 * holds the library's lifetime lock shared, teardown takes it exclusively. */
int ik_shutdown(void);
/* ik_shutdown for process exit, when threads of the caller (a server's daemon
 * request threads) may still call in: afterwards every entry point that does
 * device work returns IK_ERR_INVALID ("closed") instead of bringing the library
 * back up.  The Python package registers this one with atexit. */
int ik_close(void);
/* bytes the library holds, by pool (n <= 7 values): [0] device image blocks in
 * use, [1] image blocks kept free for reuse, [2] per-thread device arenas, [3]
 * per-thread pinned arenas, [4] upload areas (device), [5] upload areas (pinned),
 * [6] cached resize plans' device tables */
int ik_memory_stats(uint64_t *out, int n);
size_t ik_last_error(char *buf, size_t cap); /* thread-local message of the last failure */
const char *ik_version(void);

/* ---- image handles ---------------------------------------------------- */
/* ImageBuffer::from_raw: copy a tightly packed host buffer to the device */
int ik_image_from_host(const uint8_t *pixels, uint32_t width, uint32_t height, uint32_t channels,
                       ik_image **out);
/* wrap an existing device buffer (not owned; must outlive the handle) */
int ik_image_wrap_device(uint8_t *dev_pixels, uint32_t width, uint32_t height, uint32_t channels,
                         size_t pitch, ik_image **out);
int ik_image_info(const ik_image *img, uint32_t *width, uint32_t *height, uint32_t *channels);
/* 16-bit images (Rgb16 / Rgba16 / L16 / La16 of DynamicImage; 16-bit PNG decodes to
 * them): bytes per sample, 1 or 2; ik_image_to_host writes native-endian u16 for 2.
 * resize_image keeps the depth; encode_image rescales to 8 bits first (to_rgb8). */
int ik_image_depth(const ik_image *img);
int ik_image_from_host16(const uint16_t *pixels, uint32_t width, uint32_t height, uint32_t channels,
                         ik_image **out);
int ik_image_to_host(const ik_image *img, uint8_t *dst, size_t cap); /* tightly packed */
void ik_image_free(ik_image *img);
void ik_buf_free(uint8_t *buf);

/* ---- caller-pinned input memory ------------------------------------------ */
/* Encoded inputs in page-locked host memory are DMAed to the GPU in place (no
 * staging copy): a server reads request bodies into buffers from ik_host_alloc
 * (or registers its own buffer arena once with ik_host_register).  Inputs in
 * ordinary memory work too; they are copied through pinned staging first. */
int ik_host_alloc(size_t bytes, void **out);  /* page-locked, usable by every device */
int ik_host_free(void *p);                     /* only for ik_host_alloc memory */
int ik_host_register(void *p, size_t bytes);   /* page-lock an existing range */
int ik_host_unregister(void *p);               /* the start of a registered range */

/* ---- the three reference functions ------------------------------------ */
/* decode_image (src/transform.rs:27-43): guess_format + load_from_memory_with_format.
 * *fmt_out = IK_FORMAT_* for webp/jpeg/avif, -1 (None) for other formats. */
int ik_decode(const uint8_t *bytes, size_t len, ik_image **out, int *fmt_out);

/* decode_image over n inputs at once (the /img handler under load).  Baseline
 * JPEG scans (with or without restart markers) are entropy-decoded together by
 * the self-synchronising GPU decoder (a few launches for the whole batch) and
 * reconstructed on the GPU; PNG streams go through the batched GPU inflate; other
 * inputs through ik_decode.  outs[i] / fmts[i] / status[i] per input (outs[i]
 * NULL on failure; fmts and status may be NULL); returns the first failure or
 * IK_OK. */
int ik_decode_batch(const uint8_t *const *bytes, const size_t *lens, uint32_t n, ik_image **outs,
                    int *fmts, int *status);

/* PNG decoding on the GPU (ik_decode / ik_decode_batch / ik_transform*): streams
 * whose filtered image data is at least min_raw_bytes are inflated and unfiltered
 * on the GPU (parallel DEFLATE over block-start candidates, row-wavefront
 * unfilter), every non-interlaced colour type included (palette, low bit depths,
 * tRNS, 16-bit); smaller ones, interlaced (Adam7) streams and any the GPU finds
 * inconsistent use the host decoder.  -1 = host decoder only.  Default 256 KiB
 * (IK_PNG_GPU_MIN; IK_PNG_GPU=0 = off). */
int ik_set_png_gpu_min(long long min_raw_bytes);
/* the last GPU PNG batch finished on the calling thread's device (n <= 17 values):
 * [0] upload stage host ms (parse, staging copies of unpinned inputs, DMA issue),
 * device ms of [1] the upload (first DMA .. gather + CRC done) [2] decode rounds
 * [3] expand [4] resolve [5] unfilter, [6] kernel stage wall ms, [7] decode rounds,
 * [8] decoder lanes, [9] streams sent to the GPU, [10] PNG streams of the batch the
 * GPU decoded, [11] streams the host decoder took (outside the GPU path, or
 * rejected by it), [12] tokens written by the verified decoder lanes (u16 each),
 * device ms of [13] the block search [14] the gather + CRC pass, [15] kernel stage
 * ms until the block search's candidates were back (waiting for the upload
 * included), [16] 1 if the block search ran beside the previous batch's kernels */
int ik_png_last_timing(double *out, int n);
/* the last batch the calling thread's device ran through its kernel stage
 * (ik_transform_batch*): device ms from HIP events on the kernel stream and the
 * algorithmic bytes of the same launches (n <= 13 values): [0] JPEG entropy
 * decoding ms, [1] entropy-coded bytes read, [2] int16 coefficient bytes written,
 * [3] images, [4] decoder lanes; [5] grouped resize ms, [6] resize bytes (C*W*H
 * in + C*w*h out per image), [7] images resized in groups; [8] batched JPEG
 * encoder ms (coefficients + Huffman), [9] images it coded; the host coder stage
 * (libwebp / libavif on the worker pool): [10] wall ms of the batch, [11] thread
 * CPU ms summed over its requests (core-ms), [12] requests it coded */
int ik_batch_last_timing(double *out, int n);
/* process-wide counts of PNG streams decoded since load: out[0] by the GPU path,
 * out[1] by the host decoder (outside the GPU path, or rejected by it) */
int ik_png_counters(unsigned long long *out);
/* process-wide JPEG counters: out[0] = streams whose entropy decoding ran on the
 * GPU (restart intervals or self-synchronising scans), out[1] = on the host */
int ik_jpeg_counters(unsigned long long *out);

/* resize_image (src/transform.rs:62-90).  w/h < 0 mean None.  Both None returns
 * the input unchanged (*out == img); otherwise a new image (img is not freed:
 * the Rust shim drops its by-value argument).  filter: IK_FILTER_* (Lanczos3 in
 * the reference). */
int ik_resize(ik_image *img, int64_t w, int64_t h, int filter, ik_image **out);

/* Resampler arithmetic.  IK_RESIZE_EXACT (default): image 0.25.8's f32 sequence,
 * separately rounded multiply and add per tap -- bit-exact.  IK_RESIZE_FMA: one
 * fused multiply-add per tap -- within +-1 LSB per channel (the north star's
 * tolerance for bilinear/Lanczos), fewer vector instructions.  Process-wide; the
 * default also comes from IK_RESIZE_MODE=exact|fma when first used. */
typedef enum { IK_RESIZE_EXACT = 0, IK_RESIZE_FMA = 1 } ik_resize_mode;
int ik_set_resize_mode(int mode);
int ik_get_resize_mode(void);
/* The resampler kernel a launch of this geometry takes under the current modes
 * (for profiles and benchmarks): "k_resize_periodic" (integer vertical ratios),
 * "k_resize_fused", or "k_vert_naive" (the two-pass fallback); NULL on bad
 * arguments or without a device. */
const char *ik_resize_kernel_name(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter);

/* JPEG reconstruction behind decode_image (src/transform.rs:31 -> image 0.25.8
 * -> zune-jpeg 0.4.21, Cargo.lock:3106).  IK_JPEG_RECON_ZUNE (default): zune-jpeg's
 * integer IDCT (stb_image-derived, DC-only shortcut), upsampler and i16 YCbCr->RGB,
 * restated (parity unpinned: no zune-jpeg in this environment).
 * IK_JPEG_RECON_LIBJPEG: libjpeg-turbo's islow IDCT, fancy upsampling and
 * jdcolor.c -- bit-exact with Pillow's decoder.  Entropy decoding is the same in
 * both.  Process-wide; the default also comes from IK_JPEG_RECON=zune|libjpeg. */
typedef enum { IK_JPEG_RECON_LIBJPEG = 0, IK_JPEG_RECON_ZUNE = 1 } ik_jpeg_recon;
int ik_set_jpeg_reconstruction(int mode);
int ik_get_jpeg_reconstruction(void);

/* imageops::resize to exact dimensions (the resampler under resize_image) */
int ik_resize_exact(const ik_image *img, uint32_t nw, uint32_t nh, int filter, ik_image **out);

/* encode_image (src/transform.rs:113-150): quality clamped to [1,100].
 * *out is allocated by the library; release with ik_buf_free. */
int ik_encode(const ik_image *img, int fmt, int quality, uint8_t **out, size_t *out_len);

/* WebP coder behind encode_image (src/transform.rs:129-137); every choice writes the
 * bytes of the reference's webp 0.3.1 -> libwebp WebPEncodeRGB.
 * IK_WEBP_LIBWEBP: libwebp's VP8 coder on host threads over device-made YUV420 planes.
 * IK_WEBP_EXACT: libwebp's own method-4 decisions on the GPU (segment analysis, RD mode
 *   search, token statistics: ik_webp_encode_exact_device) and its bitstream on the
 *   host -- the same files, with the coding off the host cores.
 * IK_WEBP_AUTO (the default): the exact GPU coder for a batch's same-geometry groups
 *   of 32 or more images and pipelines of max_batch >= 32 (its chain of macroblock steps costs
 *   about as much for 64 images as for one), libwebp for smaller groups and lone
 *   images (one host core codes a 512^2 image in ~8 ms, the GPU chain takes ~18).
 * The process default comes from IK_WEBP_ENCODER=auto|exact|libwebp when first used.
 * (Value 1, a non-exact GPU VP8 encoder of earlier rounds, is retired: refused.) */
typedef enum { IK_WEBP_LIBWEBP = 0, IK_WEBP_EXACT = 2, IK_WEBP_AUTO = 3 } ik_webp_encoder;
int ik_set_webp_encoder(int encoder); /* process-wide, for ik_encode / ik_transform */
/* version of the libwebp that codes WebP (WebPGetEncoderVersion, e.g. 0x010600),
 * -1 when none could be loaded.  The codec libraries are explicit dependencies:
 * IK_LIBWEBP=<path> / IK_LIBAVIF=<path> when set, else the system sonames
 * libwebp.so.7 / libavif.so.16 through the dynamic loader (no other search). */
int ik_libwebp_version(void);
/* path of the library that codes fmt (IK_FORMAT_WEBP / IK_FORMAT_AVIF) into buf
 * (NUL-terminated, truncated to cap); returns its length, 0 when none loaded */
size_t ik_codec_library(int fmt, char *buf, size_t cap);
int ik_get_webp_encoder(void);

/* ---- fused / batched entry points (pixels stay in HBM) ----------------- */
/* decode -> resize_image -> encode_image in one call (handler src/lib.rs:175-191) */
int ik_transform(const uint8_t *bytes, size_t len, int64_t w, int64_t h, int fmt, int quality,
                 int filter, uint8_t **out, size_t *out_len);

/* ik_transform over n requests at once (the /img handler under load, loadtest C4
 * mix): decode_image (one set of GPU launches for the batch's PNG streams, one set
 * of self-synchronising entropy launches for its baseline JPEGs), one resize launch
 * per group of
 * same-geometry requests, encode_image (device front ends; libwebp / libavif on
 * `threads` host threads, 0 = default).  w/h (-1 = None), fmt and quality per
 * request; outs[i] (ik_buf_free) / out_lens[i] / status[i] per request (status
 * may be NULL); returns the first failure or IK_OK.  Equivalent to
 * ik_transform_batch_submit + ik_transform_batch_wait. */
int ik_transform_batch(const uint8_t *const *bytes, const size_t *lens, uint32_t n, const int64_t *w,
                       const int64_t *h, const int *fmt, const int *quality, int filter, int threads,
                       uint8_t **outs, size_t *out_lens, int *status);

/* ik_transform_batch as two calls.  Each device runs batches through four
 * stages on their own threads -- upload (the PNG / JPEG files' DMA, in place when
 * the caller pinned them, then a GPU pass that assembles the zlib streams and
 * checks the IDAT CRCs), decode kernels, post (resize and the encoders' device
 * front ends) and host coders (the device's worker pool) -- so consecutive
 * batches overlap: batch k+1's upload runs under batch k's kernels, batch k's
 * resize beside batch k+1's decode, batch k's libwebp beside both.
 * submit queues the batch and returns at once; wait blocks until its bytes are
 * ready, fills status[] (may be NULL) and returns the first failure, as
 * ik_transform_batch does.  Every array passed to submit -- the inputs included
 * -- must stay valid until wait returns; each ticket is waited for exactly once.
 * With several logical devices (ik_init(-1) / IK_DEVICES) a batch goes whole to
 * the least-loaded device, or in parts of at least IK_MIN_DEVICE_BATCH (64)
 * requests to several.  (The reference's handlers, src/lib.rs:175-191, serving
 * many requests at once.) */
int ik_transform_batch_submit(const uint8_t *const *bytes, const size_t *lens, uint32_t n, const int64_t *w,
                              const int64_t *h, const int *fmt, const int *quality, int filter, int threads,
                              uint8_t **outs, size_t *out_lens, int *status, uint64_t *ticket);
int ik_transform_batch_wait(uint64_t ticket);

/* ik_transform_batch_submit over request bodies already in device memory (HBM)
 * of one device: dev_bytes[i] are device addresses (hipMalloc / ik_dev_alloc),
 * valid until the wait returns.  The batch runs on the device that holds them.
 * PNG files are walked, gathered, CRC-checked and decoded on the GPU where they
 * lie (no PCIe transfer of the compressed bytes); any other item, and a PNG the
 * GPU path does not take, is copied back to host memory first.  Outputs, status
 * and errors as ik_transform_batch_submit; wait with ik_transform_batch_wait.
 * (The reference's handlers receive bodies in host memory, src/lib.rs:175-191;
 * this entry serves callers that already hold them on the device.) */
int ik_transform_batch_submit_device(const uint8_t *const *dev_bytes, const size_t *lens, uint32_t n,
                                     const int64_t *w, const int64_t *h, const int *fmt, const int *quality,
                                     int filter, int threads, uint8_t **outs, size_t *out_lens, int *status,
                                     uint64_t *ticket);

/* A batch of n same-geometry 8-bit images already resident in device memory
 * (image i at dev_src + i*src_image_stride, rows src_pitch bytes apart) ->
 * resize to nw x nh -> encode.  Encoded bytes are written into the caller's
 * host buffer `out` (capacity out_cap) back to back; out_sizes[i] receives each
 * size.  threads = host entropy-coder threads (0 = default).  fmt: any
 * IK_FORMAT_*; JPEG is coded on the GPU, WebP by libwebp (or the GPU VP8
 * encoder) and AVIF by libavif/aom on the host threads, from planes the GPU
 * converted (the encode_image branches, src/transform.rs:121-146). */
typedef struct ik_pipeline ik_pipeline;
int ik_pipeline_create(uint32_t W, uint32_t H, uint32_t C, uint32_t nw, uint32_t nh, int filter,
                       int fmt, int quality, uint32_t max_batch, int threads, ik_pipeline **out);
int ik_pipeline_run(ik_pipeline *p, const uint8_t *dev_src, size_t src_pitch,
                    size_t src_image_stride, uint32_t n, uint8_t *out, size_t out_cap,
                    size_t *out_sizes);
/* Streaming form of ik_pipeline_run: submit enqueues the device stage of a batch
 * (and the copy of what the host stage needs) and returns; collect finishes the
 * oldest submitted batch -- its host entropy stage -- and writes its bytes like
 * ik_pipeline_run (*n_out = its image count).  At most two batches are in flight,
 * so the host stage of batch k overlaps the device stage of batch k+1.  The
 * source frames of a submitted batch must stay valid until it is collected. */
int ik_pipeline_submit(ik_pipeline *p, const uint8_t *dev_src, size_t src_pitch,
                       size_t src_image_stride, uint32_t n);
int ik_pipeline_collect(ik_pipeline *p, uint8_t *out, size_t out_cap, size_t *out_sizes,
                        uint32_t *n_out);
/* WebP encoder of this pipeline (IK_WEBP_*; default: the process default) */
int ik_pipeline_set_webp_encoder(ik_pipeline *p, int encoder);
/* device-only part (resize + colour convert/FDCT [+ GPU VP8]) for n images, no host stage */
int ik_pipeline_run_device(ik_pipeline *p, const uint8_t *dev_src, size_t src_pitch,
                           size_t src_image_stride, uint32_t n);
/* device time (ms) of stage `which` (0 = resize, 1 = colour convert, 2 = GPU VP8
 * wavefront) in the last run, from HIP events on the pipeline's stream;
 * 3 = wall time (ms) of the last collected batch's host entropy stage */
double ik_pipeline_kernel_ms(const ik_pipeline *p, int which);
/* resized pixels of image i of the last run (tightly packed nw*nh*C) */
int ik_pipeline_fetch_resized(ik_pipeline *p, uint32_t i, uint8_t *dst, size_t cap);
void ik_pipeline_destroy(ik_pipeline *p);

/* raw device kernels, for parity tests and the bench (dev_* = device pointers) */
int ik_resize_batch_device(const uint8_t *dev_src, uint32_t W, uint32_t H, uint32_t C,
                           size_t src_pitch, size_t src_image_stride, uint32_t n, uint32_t nw,
                           uint32_t nh, int filter, uint8_t *dev_dst, size_t dst_pitch,
                           size_t dst_image_stride, void *hip_stream);
/* the WebP colour conversion (to_rgb8 + libwebp RGB->YUV420) on the device;
 * dev_yuv receives the Y (w*h), U and V ((w+1)/2 * (h+1)/2) planes back to back */
int ik_webp_yuv420_device(const uint8_t *dev_src, uint32_t w, uint32_t h, uint32_t C,
                          size_t pitch, uint8_t *dev_yuv, void *hip_stream);
/* libwebp's method-4 segment analysis on the GPU -- the first stage of
 * encode_image's WebP coder (src/transform.rs:129-137 -> libwebp VP8EncAnalyze +
 * VP8SetSegmentParams), exact: the same segment map and segment header libwebp
 * writes for these planes at this quality.  n images of w x h YUV420 planes in
 * device memory (the ik_webp_yuv420_device layout), image i at dev_yuv +
 * i*yuv_stride.  seg (host) receives n * mb_w * mb_h segment ids, raster order per
 * image; hdr (host) n headers.  Runs on the calling thread's stream and waits. */
typedef struct {
    int32_t num_segments;  /* after libwebp's SimplifySegments (1..4) */
    int32_t update_map;    /* the frame codes a segment map */
    int32_t quant[4];      /* segment quantiser indices (the header's absolute values) */
    int32_t fstrength[4];  /* initial filter levels (libwebp raises them after coding) */
    int32_t base_quant;    /* y_ac_qi */
    int32_t dq_uv_dc, dq_uv_ac;
    int32_t probs[3];      /* segment-tree probabilities */
    int32_t alpha, uv_alpha; /* frame susceptibilities (enc->alpha_, enc->uv_alpha_) */
} ik_vp8_segment_header;
int ik_vp8_analyze_device(const uint8_t *dev_yuv, size_t yuv_stride, uint32_t n, uint32_t w, uint32_t h,
                          float quality, uint8_t *seg, ik_vp8_segment_header *hdr);
/* the exact WebP coder on the GPU: libwebp method 4's segment analysis and macroblock
 * decisions on the device (a wavefront per probability-refresh epoch), the bitstream on
 * the host -- the file WebPEncodeRGB writes for these planes at this quality.  n images
 * of w x h device YUV420 planes (the ik_webp_yuv420_device layout) yuv_stride apart;
 * outs[i] / out_lens[i] receive each file (library-allocated, ik_buf_free). */
int ik_webp_encode_exact_device(const uint8_t *dev_yuv, size_t yuv_stride, uint32_t n, uint32_t w, uint32_t h,
                                int quality, uint8_t **outs, size_t *out_lens);
/* the JPEG front end (to_rgb8 + RGB->YCbCr + FDCT + quantise) on the device:
 * int16 coefficients, MCU-major, Y/Cb/Cr, natural order */
int ik_jpeg_coeffs_device(const uint8_t *dev_src, uint32_t w, uint32_t h, uint32_t C,
                          size_t pitch, int quality, int16_t *dev_coef, void *hip_stream);

/* device memory helpers (so callers need no HIP headers) */
int ik_dev_alloc(size_t bytes, void **dev_ptr);
int ik_dev_free(void *dev_ptr);
int ik_memcpy_h2d(void *dev_dst, const void *host_src, size_t bytes);
int ik_memcpy_d2h(void *host_dst, const void *dev_src, size_t bytes);
int ik_dev_synchronize(void);

#ifdef __cplusplus
}
#endif
#endif
