// ik_internal.h -- shared declarations between the HIP kernels (ik_kernels.hip)
// and the host runtime (ik_*.cpp) of libimagekit_hip.so.  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/imagekit_hip.h"
#include "ik_jpeg_sync.h"

namespace ik {

// resize arithmetic (ik_set_resize_mode): IK_RESIZE_EXACT (the reference's f32
// sequence, bit-exact) or IK_RESIZE_FMA (fused multiply-add, within 1 LSB)
int resize_mode();

constexpr int kThreads = 256;            // workgroup size (4 wave64s)
constexpr int kBytesPerLane = 8;         // vertical pass: bytes of a source row per lane
constexpr int kStripBytes = kBytesPerLane * kThreads;  // 2048 source bytes per strip
constexpr int kRowWords = kStripBytes + kStripBytes / 8;  // LDS f32 row, +4 words per 32
constexpr int kMaxFlushRows = 4;         // vertical rows staged in LDS per horizontal pass (plan: 2..4)
constexpr int kMaxStripCols = 512;       // output columns per strip (LDS offset/count tables)
constexpr int kMaxStripWeights = 4096;   // horizontal weights per strip kept in LDS (16 KB: an RGB Lanczos3 8x strip's 85 x 48)

// Everything the resize kernels read.  Weight tables follow image 0.25.8
// sample.rs (see ik_plan.cpp); tables live in one device allocation per plan.
struct ResizeArgs {
    const uint8_t* src;
    size_t src_pitch, src_img_stride;
    uint8_t* dst;
    size_t dst_pitch, dst_img_stride;
    int W, H, C, nw, nh, row_bytes;
    const int* ly;     // [nh]   first source row of each output row
    const int* ny;     // [nh]   tap count
    const float* wy;   // [nh*Ty] normalised weights, zero padded
    int Ty;
    const int* lx;     // [nw]
    const int* nx;     // [nw]
    const float* wx;   // [nw*Tx]
    int Tx;
    const int* strips; // [NS*3] (ox0, ox1, first source byte)
    int NS;
    const int* bands;  // [NB*2] (oy0, oy1)
    int NB;
    // fused-kernel step tables.  A band is a sequence of steps; a step brings in
    // up to R new source rows [start, start+count) and scatters them into the A
    // rolling accumulators (acc[d] = output row next+d); `emit` completes row next.
    const int* step_hdr;        // [nsteps][4] (start, count, emit, 0)
    const unsigned long long* step_mask;  // [nsteps] bit j*A+d: row start+j feeds acc[d]
    const float* step_w;        // [nsteps][R][A] the matching weights (0 elsewhere)
    const int* band_step;       // [NB+1] first step of each band
    // periodic sweep (k_resize_periodic): step t brings in source rows
    // R*t + per_base .. +R-1, and output row y takes its taps from steps y .. y+A-1
    const float* per_w;      // [steps][A*R]: per_w[t][e*R + j] = weight of row j of step t in output t-e
    const int* per_bands;    // [NBp*2] (oy0, oy1)
    int per_base, NBp;
    int max_strip_cols;      // max output columns of a strip (LDS table size)
    int max_strip_weights;   // max nox*Tx of a strip (LDS weights size when in LDS)
    float* tmp;        // naive path only: f32 vertical intermediate [n][nh][row_bytes]
    // fused path, images anywhere in memory: per-image base pointers (device
    // arrays, [n]); null = src + img * src_img_stride / dst + img * dst_img_stride
    const uint64_t* src_tab;
    const uint64_t* dst_tab;
};

// Host-side plan for one (W,H,C,nw,nh,filter,band height) geometry.
struct ResizePlan {
    int W = 0, H = 0, C = 0, nw = 0, nh = 0, filter = 0;
    int slots = 0;        // accumulator slots the fused kernel needs (0 = naive path)
    int rows = 0;         // prefetch depth: max source rows consumed per output row
    bool weights_in_lds = false;
    int flush = 3;        // completed vertical rows staged in LDS per horizontal pass
    int NS = 0, NB = 0;
    int per_A = 0, per_R = 0;  // periodic geometry (k_resize_periodic); 0 = not periodic
    size_t table_bytes = 0;
    void* dev_tables = nullptr;
    ResizeArgs args{};    // pointers into dev_tables; src/dst/tmp filled per launch
};

// ---- launchers (ik_kernels.hip) ----
// The fused kernel addresses one source image through a buffer descriptor with
// 32-bit num_records and row offsets: images over INT32_MAX bytes take the naive
// two-pass path (whose caller must then pass naive_tmp).
inline bool resize_fused_fits(size_t src_pitch, size_t H) { return src_pitch * H <= 0x7FFFFFFFull; }
// 16-bit images: the two-pass path over u16 samples (tmp: nh * W * C floats), and
// the u16 -> u8 rescale of to_rgb8 / to_rgba8
hipError_t launch_resize16(const ResizePlan& plan, const uint8_t* src, size_t src_pitch, uint8_t* dst,
                           size_t dst_pitch, float* tmp, hipStream_t s);
hipError_t launch_u16_to_u8(const uint8_t* src, size_t sp, uint8_t* dst, size_t dp, int row_samples, int rows,
                            hipStream_t s);
hipError_t launch_resize(const ResizePlan& plan, const uint8_t* src, size_t src_pitch,
                         size_t src_img_stride, uint8_t* dst, size_t dst_pitch,
                         size_t dst_img_stride, int n, float* naive_tmp, hipStream_t s,
                         const uint64_t* src_tab = nullptr, const uint64_t* dst_tab = nullptr);
// dynamic LDS bytes of the fused kernel
size_t resize_lds_bytes(const ResizeArgs& a, bool wl, int flush);
// k_resize_periodic (ik_kernels.hip): whether (A accumulators, R rows per step) has
// an instance; its band plan aims at kPerTargetWG workgroups, bands >= kPerMinBand rows
bool periodic_instance(int A, int R);
// the kernel launch_resize picks for this plan (ik_resize_kernel_name)
const char* resize_kernel_name(const ResizePlan& plan, size_t src_pitch);
constexpr int kPerTargetWG = 4096, kPerMinBand = 32;
hipError_t launch_webp_yuv420(const uint8_t* src, int w, int h, int C, size_t pitch,
                              size_t img_stride, uint8_t* yuv /* Y, U, V planes per image */,
                              size_t yuv_img_stride, int n, const uint16_t* gamma_to_lin,
                              const int* lin_to_gamma, hipStream_t s,
                              const uint64_t* src_tab = nullptr /* per-image bases instead of img_stride */);
// n images; planes (Y, U, V, A: w*h each) plane_img_stride apart; transparent[n]
// zeroed here, then set to 1 for every image with an alpha < 255
hipError_t launch_avif_yuv444(const uint8_t* src, int w, int h, int C, size_t pitch, size_t img_stride,
                              uint8_t* planes, size_t plane_img_stride, int* transparent, int n, hipStream_t s);
hipError_t launch_jpeg_coeffs(const uint8_t* src, int w, int h, int C, size_t pitch,
                              size_t img_stride, const uint8_t* qtables /*dev, 128 B*/,
                              int16_t* coef, size_t coef_img_stride, int n, hipStream_t s,
                              const uint64_t* src_tab = nullptr /* per-image bases (device), or src + i * img_stride */);

// JPEG reconstruction (ik_jpeg.hip): dequantise + islow IDCT every 8x8 block of
// the coefficient image into per-component sample planes, then fancy-upsample +
// colour-convert into the device image.
struct JpegGeom {
    int ncomp, W, H, hmax, vmax;
    int colorspace;                 // 0 gray, 1 YCbCr, 2 RGB, 3 CMYK, 4 YCCK (4 components -> RGB8)
    int adobe;                      // APP14 Adobe present: CMYK / YCCK samples are stored inverted
    int recon;                      // IK_JPEG_RECON_LIBJPEG / IK_JPEG_RECON_ZUNE (ik_jpeg.hip)
    int h[4], v[4], bw[4], bh[4], dw[4], dh[4];
    long long blk0[4];              // first block of each component in coef
    long long plane0[4];            // byte offset of each component plane (bw*8 x bh*8)
    long long nblocks;
    const uint16_t* qt;             // [component][64] natural order
    const int16_t* coef;            // [block][64] natural order, quantised
    uint8_t* planes;
};
hipError_t launch_jpeg_reconstruct(const JpegGeom& g, uint8_t* dst, size_t dst_pitch, hipStream_t s);
// a batch's reconstructions in three launches (items in device memory)
struct JpegReconItem {
    JpegGeom g;
    uint8_t* dst;
    size_t pitch;
    int fast;  // jpeg_zune_fast(g)
    int pad;
};
hipError_t launch_jpeg_reconstruct_batch(const JpegReconItem* items, int m, long long max_blocks, int max_w, int max_h,
                                         bool any_fast, bool any_slow, bool idct, hipStream_t s);
bool jpeg_zune_fast(const JpegGeom& g);

// Baseline Huffman tables (JpegHuffTables) and the self-synchronising decoder's
// per-lane code are in ik_jpeg_sync.h (shared with its CPU model).
//
// The self-synchronising baseline decoder (ik_jsync.hip), one batch of scans:
// one image's scan as the unstuffing kernels see it
struct JsImageDev {
    const uint8_t* scan;   // the entropy-coded bytes (stuffed, with RSTn markers), device
    long long scan_len;
    uint8_t* out;          // unstuffed bytes as big-endian words (scan_len + 4 kPadWords + 8 bytes)
    long long* ivl;        // interval start bits: ivl_cap entries (intervals + 1)
    int ivl_cap;
    int chunk0, nchunks;   // the image's 4 KiB chunks in the batch's chunk table
    int pad;
    uint32_t* totals;      // [0] bytes kept, [1] restart markers
    int* status;           // bit 0 a stray marker, 1 too many restart markers, 4 inconsistent / missing
                           // blocks, 8 a bad code in the decode pass: the host decoder decides
};
hipError_t launch_jsync_unstuff(JsImageDev* imgs, int nimg, const int2* chunks, int nchunks, uint2* counts,
                                hipStream_t s);
// wgs: (image, first lane of the image) per 256-lane workgroup; every image's lanes
// start on a multiple of 256 (jsync::Scan::lane0)
hipError_t launch_jsync_sync(const jsync::Scan* scans, const int2* wgs, int nwg, jsync::LaneRec* recs, hipStream_t s);
hipError_t launch_jsync_fix(const jsync::Scan* scans, int nimg, const int2* wgs, int nwg, jsync::LaneRec* recs,
                            int* rounds, hipStream_t s);
// bases (segmented prefix sums over each interval's lanes) then the decode pass;
// chunk_scratch: jsync_chunk_scratch_bytes(lanes); status[image]
hipError_t launch_jsync_bases_decode(const jsync::Scan* scans, int nimg, const int2* wgs, int nwg,
                                     const jsync::LaneRec* recs, jsync::LaneBase* bases, void* chunk_scratch,
                                     int* status, hipStream_t s);
size_t jsync_chunk_scratch_bytes(long long lanes);
struct JpegScanArgs {
    const uint8_t* data;          // the scan's entropy-coded bytes (stuffed, with RST markers)
    long long size;
    const unsigned* seg;          // first byte of each restart interval (n_seg entries)
    int n_seg, restart;           // intervals, MCUs per interval
    long long total_mcu;
    int mcux;                     // MCUs per row (interleaved scans)
    int single, single_bw;        // one-component scan: an MCU is one block, single_bw per row
    int ns;                       // components in the scan, in scan order:
    int h[4], v[4], bw[4], td[4], ta[4];
    long long blk0[4];
    const JpegHuffTables* tabs;
    int16_t* coef;                // [block][64] natural order, pre-zeroed
    int* err;                     // set non-zero on a bad code (the host then redoes the scan)
    int lanes;                    // intervals per 64-lane workgroup (64, or fewer to cut divergence)
    // progressive scans (k_jpeg_prog): 1 DC first, 2 DC refine, 3 AC first, 4 AC refine
    int kind, Ss, Se, Al;
};
// One progressive scan with restart intervals (ik_jpeg.hip k_jpeg_prog): a lane per
// interval, the EOB run and DC predictions reset at each RSTn; the scans of an
// image run in stream order, each refining the coefficients of the ones before.
hipError_t launch_jpeg_prog(const JpegScanArgs& a, hipStream_t s);
int jpeg_lanes_for(long long total_lanes);  // lanes per wave for that many independent decoders

// Baseline Huffman coding of k_jpeg_coeffs' output on the GPU (ik_jpeg_enc.hip),
// the same bytes as ik_codec.cpp's host coder.  Per image: entropy-coded segment
// (stuffed, with pad_byte) in out + i*out_img_stride, its length in out_len[i]
// (0xffffffff: does not fit out_cap -> code it on the host).
struct JpegEncArgs {
    const int16_t* coef;       // [mcu][Y,Cb,Cr][64] natural order per image
    size_t coef_img_stride;    // int16 elements between images
    int nmcu;
    const uint32_t* huff;      // [ldc, lac, cdc, cac][256]: code << 8 | size
    uint8_t* work;             // per image: words_bytes of bit words, then out_cap staging bytes
    size_t work_img_bytes, words_bytes;
    uint8_t* out;              // device or pinned host memory
    size_t out_img_stride, out_cap;
    uint32_t* out_len;
};
hipError_t launch_jpeg_huff_enc(const JpegEncArgs& a, int n, hipStream_t s);
inline size_t jpeg_enc_cap(int w, int h) {  // stuffed-stream capacity per image
    return ((size_t)3 * w * h + 4096 + 15) & ~(size_t)15;
}

// ---- plans (ik_plan.cpp) ----
// sample.rs weights for one axis; returns the tap count T (row stride of w).
int axis_weights(int in, int out, int filter, std::vector<int>& left, std::vector<int>& cnt,
                 std::vector<float>& w);
int required_slots(const std::vector<int>& left, const std::vector<int>& cnt);
ResizePlan* get_resize_plan(int device, int W, int H, int C, int nw, int nh, int filter, int n);

}  // namespace ik
