// ik_vp8d.hip -- device half of the GPU WebP (VP8 lossy) decoder (host half:
// ik_vp8d_host.cpp, which also decodes the token partitions: an arithmetic-coded
// stream, serial symbol by symbol -- one wave decoding it on the scalar unit ran at
// 1/12 of a CPU core).  Two launches per batch of images:
//   k_vp8d_recon   prediction + inverse transforms + loop filter (frame_dec.c
//                  ReconstructRow / DoFilter): one workgroup per image, one wave per MB
//                  row, kReconWaves rows in flight, each two MBs behind the row above
//                  (the unfiltered top row, the top-right samples and the filtered
//                  pixels its edges touch are final by then); per wave an LDS work area
//                  holds the MB being predicted and its filter window, so each pixel is
//                  written to HBM once per MB.  Intra-4 MBs go by sub-block diagonals
//                  (x + 2y: ten steps, a lane per pixel), the other blocks a lane each.
//   k_vp8d_rgb     fancy chroma upsampling + YUV -> RGB (io_dec.c EmitFancyRGB,
//                  upsampling.c UPSAMPLE_FUNC, yuv.h VP8YuvToRgb) into the ik_image
#include <hip/hip_runtime.h>

#include "ik_vp8d_gpu.h"

namespace ik {
namespace vp8d {

namespace {

template <typename T>
using cptr = const __attribute__((address_space(4))) T*;  // read-only for the launch: scalar loads

#define WSYNC()                                                \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                       \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)

__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace

namespace {

// per wave: R, the MB being predicted (rows -1..15, cols -4..27, BPS-pitched: the
// unfiltered top row, the left column and the corner rotate in as libwebp's
// ReconstructRow does), F, its filter window (rows -4..15; cols -16..15: the MB to
// the left whole, written out once the left edge has been filtered, and the filtered
// bottom rows of the MB above), and its coefficients
struct alignas(16) WaveLds {
    uint8_t ry[17 * 32], ru[9 * 32], rv[9 * 32];
    uint8_t fy[20 * 32], fu[12 * 16], fv[12 * 16];
    int16_t coef[384];
};

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr int kCpolSc1 = 16;  // buffer cache policy sc1: write-through stores, L1-bypassing loads

// A plane as a buffer resource: the MB rows hand their pixels to the row below (often
// on another CU or XCD) with sc1 stores, sc1 loads and an sc1 progress flag
// (MI355X_MICROARCH.md "inter-workgroup visibility", the first row of its table)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* base, uint32_t bytes) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)base);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uintptr_t)base >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}

// libwebp's ten intra-4 predictors (pred4, ik_vp8x.h) as per-pixel taps: per (mode,
// pixel y*4+x) the samples e[i0], e[i1], e[i2] of e[] = L K J I X A B C D E F G H
// (bits 0-3, 4-7, 8-11) and the op (bits 12-14): 0 avg3, 1 avg2, 2 e[i0], 3 TM, 4 DC
// (the exact coder's table, ik_vp8x.hip, tools/gen_i4_taps.py)
__constant__ uint16_t kTap[10][16] = {
    {0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000},
    {0x3453, 0x3463, 0x3473, 0x3483, 0x3452, 0x3462, 0x3472, 0x3482, 0x3451, 0x3461, 0x3471, 0x3481, 0x3450, 0x3460, 0x3470, 0x3480},
    {0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987},
    {0x0234, 0x0234, 0x0234, 0x0234, 0x0123, 0x0123, 0x0123, 0x0123, 0x0012, 0x0012, 0x0012, 0x0012, 0x0001, 0x0001, 0x0001, 0x0001},
    {0x0345, 0x0456, 0x0567, 0x0678, 0x0234, 0x0345, 0x0456, 0x0567, 0x0123, 0x0234, 0x0345, 0x0456, 0x0012, 0x0123, 0x0234, 0x0345},
    {0x1054, 0x1065, 0x1076, 0x1087, 0x0543, 0x0654, 0x0765, 0x0876, 0x0432, 0x1054, 0x1065, 0x1076, 0x0321, 0x0543, 0x0654, 0x0765},
    {0x0765, 0x0876, 0x0987, 0x0a98, 0x0876, 0x0987, 0x0a98, 0x0ba9, 0x0987, 0x0a98, 0x0ba9, 0x0cba, 0x0a98, 0x0ba9, 0x0cba, 0x0ccb},
    {0x1065, 0x1076, 0x1087, 0x1098, 0x0765, 0x0876, 0x0987, 0x0a98, 0x1076, 0x1087, 0x1098, 0x0ba9, 0x0876, 0x0987, 0x0a98, 0x0cba},
    {0x1043, 0x0543, 0x0654, 0x0765, 0x1032, 0x0432, 0x1043, 0x0543, 0x1021, 0x0321, 0x1032, 0x0432, 0x1010, 0x0210, 0x1021, 0x0321},
    {0x1023, 0x0123, 0x1012, 0x0012, 0x1012, 0x0012, 0x1001, 0x0001, 0x1001, 0x0001, 0x2000, 0x2000, 0x2000, 0x2000, 0x2000, 0x2000},
};

// sample e[k] around the 4x4 block at blk (BPS-pitched)
__device__ __forceinline__ int tap_sample(const uint8_t* blk, int k) {
    return k < 4 ? blk[(3 - k) * 32 - 1] : k == 4 ? blk[-33] : blk[k - 5 - 32];
}

__device__ __forceinline__ int mul1(int a) { return ((a * 20091) >> 16) + a; }
__device__ __forceinline__ int mul2(int a) { return (a * 35468) >> 16; }

// pixel (r, c) of libwebp's TransformOne of the block's coefficients q (raster):
// the vertical pass's row r for the four columns, then the horizontal pass's column c
__device__ __forceinline__ int idct_pixel(const int16_t* q, int r, int c) {
    int v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int a = q[k] + q[8 + k], b = q[k] - q[8 + k];
        const int cc = mul2(q[4 + k]) - mul1(q[12 + k]), d = mul1(q[4 + k]) + mul2(q[12 + k]);
        v[k] = r == 0 ? a + d : r == 1 ? b + cc : r == 2 ? b - cc : a - d;
    }
    const int dc = v[0] + 4;
    const int a = dc + v[2], b = dc - v[2];
    const int cc = mul2(v[1]) - mul1(v[3]), d = mul1(v[1]) + mul2(v[3]);
    return (c == 0 ? a + d : c == 1 ? b + cc : c == 2 ? b - cc : a - d) >> 3;
}

}  // namespace

// One wave per workgroup; waves take (image, MB row) tickets in order, so a row only
// ever waits for the row ticketed just before it, which a running wave holds: the
// grid drains whatever the residency.  A row publishes its progress (MBs done) after
// its stores of each MB; the row below starts MB x once the row above has done x + 2.
__global__ __launch_bounds__(64) void k_vp8d_recon(const DImg* __restrict__ imgs, int n, uint32_t* __restrict__ ticket) {
    __shared__ WaveLds L;
    __shared__ uint16_t s_tap[10 * 16];  // the predictor taps (a divergent index into them: LDS, not memory)
    const int lane = threadIdx.x;
    for (int i = lane; i < 10 * 16; i += 64) s_tap[i] = kTap[i >> 4][i & 15];
    uint8_t* const Ry = L.ry + 36;
    uint8_t* const Ru = L.ru + 36;
    uint8_t* const Rv = L.rv + 36;
    uint8_t* const Fy = L.fy + 4 * 32 + 16;  // F origin: row 0, col 0 (pitch 32; cols -16..15)
    uint8_t* const Fu = L.fu + 4 * 16 + 8;   // (pitch 16; cols -8..7)
    uint8_t* const Fv = L.fv + 4 * 16 + 8;
    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = (uint32_t)ufl((int)t);
        int ii = 0;
        uint32_t r0 = 0;
        for (; ii < n; ++ii) {
            r0 = ((cptr<DImg>)imgs)[ii].row0;
            if (t < r0 + ((cptr<DImg>)imgs)[ii].rows) break;
        }
        if (ii == n) return;
        const cptr<DImg> di = (cptr<DImg>)imgs + ii;
        const int mb_y = (int)(t - r0);
        const cptr<DFrame> fr = (cptr<DFrame>)di->fr;
        // per-MB records as dwords (a byte through a scalar pointer becomes a vector
        // load and a wait per field)
        const cptr<uint32_t> mbw = (cptr<uint32_t>)di->mbs;  // 6 words per DMB
        const cptr<uint32_t> flagw = (cptr<uint32_t>)di->flags;
        const cptr<uint32_t> segw = (cptr<uint32_t>)di->fr->seg;  // 5 words per DSeg
        const uint32_t* const coef = di->coef;
        const cptr<uint32_t> coef_at = (cptr<uint32_t>)di->coef_at;
        uint32_t* const prog = di->prog;
        uint32_t* const err = di->err;
        const int ys = (int)di->ys, uvs = (int)di->uvs;
        const int mb_w = fr->mb_w, mb_h = fr->mb_h, ftype = fr->filter_type;
        const __amdgpu_buffer_rsrc_t rY = rsrc(di->y, (uint32_t)ys * mb_h * 16);
        const __amdgpu_buffer_rsrc_t rU = rsrc(di->u, (uint32_t)uvs * mb_h * 8);
        const __amdgpu_buffer_rsrc_t rV = rsrc(di->v, (uint32_t)uvs * mb_h * 8);
        const __amdgpu_buffer_rsrc_t rT = rsrc(di->top, (uint32_t)mb_w * 64);
        const int has_top = mb_y > 0;
        const uint32_t tbase_in = (uint32_t)((mb_y - 1) & 1) * mb_w * 32, tbase_out = (uint32_t)(mb_y & 1) * mb_w * 32;
        uint32_t seen = 0;  // the row above's progress last read
        // the next MB's first 64 coefficient words, loaded a step ahead (after this
        // step's publish, so the drain before the flag does not wait for them)
        uint32_t c0 = coef_at[mb_y * mb_w], c1 = coef_at[mb_y * mb_w + 1];
        uint32_t e0 = c0 + lane < c1 ? coef[c0 + lane] : ~0u;
        for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
            const int mb = mb_y * mb_w + mb_x;
            const int has_left = mb_x > 0;
            // the MB's coefficients: the first 64 entries load now, under the wait
            if (lane < 48) reinterpret_cast<uint4*>(L.coef)[lane] = make_uint4(0, 0, 0, 0);
            const cptr<uint32_t> m = mbw + 6 * mb;
            const uint32_t m0 = m[0], bm0 = m[2], bm1 = m[3], bm2 = m[4], bm3 = m[5];
            const int is_i4 = m0 & 255, ymode = (m0 >> 8) & 255, uvmode = (m0 >> 16) & 255, seg = m0 >> 24;
            const uint32_t sgf = segw[5 * seg + 3], sgh = segw[5 * seg + 4];  // limit[2] ilevel[2], hev[2]
            const int nonzero = (flagw[mb >> 2] >> (8 * (mb & 3))) & 255;
            if (has_top) {  // the row above has done MBs mb_x and mb_x + 1
                const uint32_t need = (uint32_t)min(mb_x + 2, mb_w);
                if (seen < need) {
                    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;  // 4 s
                    for (;;) {
                        seen = (uint32_t)ufl((int)__hip_atomic_load(prog + mb_y - 1, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT));
                        if (seen >= need) break;
                        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                            __builtin_amdgcn_s_memrealtime() > t_end) {
                            if (lane == 0) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            return;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                // the unfiltered row above (+ top-right) and the filter's top strip (rows
                // 12..15 of the MB above, filtered), all sc1 loads
                const uint32_t tp = tbase_in + (uint32_t)mb_x * 32;
                if (lane < 2) {
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rT, tp + 16 * lane, 0, kCpolSc1);
                    if (lane == 0) {  // (R rows are 4-byte aligned only)
                        st32(Ry - 32, v.x);
                        st32(Ry - 28, v.y);
                        st32(Ry - 24, v.z);
                        st32(Ry - 20, v.w);
                    } else {
                        st32(Ru - 32, v.x);
                        st32(Ru - 28, v.y);
                        st32(Rv - 32, v.z);
                        st32(Rv - 28, v.w);
                    }
                } else if (lane == 2) {
                    uint32_t tr;
                    if (mb_x < mb_w - 1) {
                        tr = __builtin_amdgcn_raw_buffer_load_b32(rT, tp + 32, 0, kCpolSc1);
                    } else {
                        tr = 0x01010101u * (__builtin_amdgcn_raw_buffer_load_b32(rT, tp + 12, 0, kCpolSc1) >> 24);
                    }
                    st32(Ry - 32 + 16, tr);
                } else if (lane >= 16 && lane < 20) {
                    const int r = lane - 16;
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                        rY, (uint32_t)(16 * mb_y - 4 + r) * ys + 16 * mb_x, 0, kCpolSc1);
                    reinterpret_cast<u32x4*>(Fy + (r - 4) * 32)[0] = v;
                } else if (lane >= 32 && lane < 40) {
                    const int k = lane - 32, c = k >> 2, r = k & 3;
                    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(
                        c ? rV : rU, (uint32_t)(8 * mb_y - 4 + r) * uvs + 8 * mb_x, 0, kCpolSc1);
                    reinterpret_cast<u32x2*>((c ? Fv : Fu) + (r - 4) * 16)[0] = v;
                }
                if (!has_left && lane == 63) Ry[-33] = Ru[-33] = Rv[-33] = 129;
            } else {  // frame top: 127 above (corner and top-right included)
                if (lane < 6) st32(Ry - 36 + 4 * lane, 0x7f7f7f7fu);
                else if (lane < 9) st32(Ru - 36 + 4 * (lane - 6), 0x7f7f7f7fu);
                else if (lane < 12) st32(Rv - 36 + 4 * (lane - 9), 0x7f7f7f7fu);
            }
            if (!has_left) {  // frame left: 129
                if (lane < 16) Ry[lane * 32 - 1] = 129;
                else if (lane < 24) Ru[(lane - 16) * 32 - 1] = 129;
                else if (lane < 32) Rv[(lane - 24) * 32 - 1] = 129;
            }
            WSYNC();
            if (is_i4 && lane < 3) st32(Ry + (4 * lane + 3) * 32 + 16, ld32(Ry - 32 + 16));  // top-right, replicated
            if (e0 != ~0u) L.coef[e0 & 511] = (int16_t)(e0 >> 16);
            for (uint32_t k = c0 + 64 + lane; k < c1; k += 64) {
                const uint32_t e = coef[k];
                L.coef[e & 511] = (int16_t)(e >> 16);
            }
            WSYNC();
            // ---- prediction + residuals ----
            if (!is_i4) {
                if (lane < 16) {
                    const int bx = lane & 3, by = lane >> 2;
                    uint8_t* blk = Ry + by * 4 * 32 + bx * 4;
                    pred_block(blk, ymode, Ry - 1, 32, Ry - 32, Ry[-33], 16, has_top, has_left, bx, by);
                    vp8x::itransform(blk, L.coef + 16 * lane, blk);
                }
            } else {
                // intra-4: sub-block (x, y) needs (x - 1, y), (x, y - 1), (x + 1, y - 1) and
                // the corner, so the blocks of one diagonal t = x + 2y (at most two) go
                // together, a lane per pixel
                const int px = lane & 15, pr = px >> 2, pc = px & 3;
                for (int d = 0; d < 10; ++d) {
                    const int by = (d < 3 ? 0 : (d - 2) >> 1) + (lane >> 4), bx = d - 2 * by;
                    if (lane < 32 && by <= 3 && bx >= 0 && bx <= 3) {
                        const int nb = 4 * by + bx;
                        const uint8_t* blk = Ry + by * 4 * 32 + bx * 4;
                        const uint32_t bw = (nb >> 2) == 0 ? bm0 : (nb >> 2) == 1 ? bm1 : (nb >> 2) == 2 ? bm2 : bm3;
                        const uint32_t tap = s_tap[((bw >> (8 * (nb & 3))) & 255) * 16 + px];
                        const int op = tap >> 12;
                        int p;
                        if (op == 4) {
                            p = 4;
#pragma unroll
                            for (int k = 0; k < 4; ++k) p += blk[k - 32] + blk[k * 32 - 1];
                            p >>= 3;
                        } else {
                            const int a = tap_sample(blk, tap & 15), b = tap_sample(blk, (tap >> 4) & 15);
                            const int c = tap_sample(blk, (tap >> 8) & 15);
                            p = op == 0 ? (a + 2 * b + c + 2) >> 2 : op == 1 ? (a + b + 1) >> 1 : op == 2 ? a
                                                                                                 : xclip8(a + b - c);
                        }
                        Ry[(4 * by + pr) * 32 + 4 * bx + pc] = xclip8(p + idct_pixel(L.coef + 16 * nb, pr, pc));
                    }
                    WSYNC();
                }
            }
            if (lane >= 32 && lane < 40) {
                const int k = lane - 32, c = k >> 2, b = k & 3;
                uint8_t* R = c ? Rv : Ru;
                uint8_t* blk = R + (b >> 1) * 4 * 32 + (b & 1) * 4;
                pred_block(blk, uvmode, R - 1, 32, R - 32, R[-33], 8, has_top, has_left, b & 1, b >> 1);
                vp8x::itransform(blk, L.coef + (16 + k) * 16, blk);
            }
            WSYNC();
            // ---- the unfiltered bottom row for the row below; the MB into F ----
            if (mb_y < mb_h - 1 && lane < 2) {
                u32x4 v;
                if (lane == 0) {
                    v.x = ld32(Ry + 15 * 32);
                    v.y = ld32(Ry + 15 * 32 + 4);
                    v.z = ld32(Ry + 15 * 32 + 8);
                    v.w = ld32(Ry + 15 * 32 + 12);
                } else {
                    v.x = ld32(Ru + 7 * 32);
                    v.y = ld32(Ru + 7 * 32 + 4);
                    v.z = ld32(Rv + 7 * 32);
                    v.w = ld32(Rv + 7 * 32 + 4);
                }
                __builtin_amdgcn_raw_buffer_store_b128(v, rT, tbase_out + (uint32_t)mb_x * 32 + 16 * lane, 0, kCpolSc1);
            }
            st32(Fy + (lane >> 2) * 32 + 4 * (lane & 3), ld32(Ry + (lane >> 2) * 32 + 4 * (lane & 3)));
            if (lane < 32) {
                const int c = lane >> 4, r = (lane & 15) >> 1, g = lane & 1;
                st32((c ? Fv : Fu) + r * 16 + 4 * g, ld32((c ? Rv : Ru) + r * 32 + 4 * g));
            }
            WSYNC();
            // rotate the left samples (and the corner) in for the next MB
            if (lane < 17) st32(Ry + (lane - 1) * 32 - 4, ld32(Ry + (lane - 1) * 32 + 12));
            else if (lane < 26) st32(Ru + (lane - 18) * 32 - 4, ld32(Ru + (lane - 18) * 32 + 4));
            else if (lane < 35) st32(Rv + (lane - 27) * 32 - 4, ld32(Rv + (lane - 27) * 32 + 4));
            // ---- loop filter (DoFilter) ----
            const int i4 = is_i4 ? 1 : 0;
            const int limit = ftype ? (int)((sgf >> (8 * i4)) & 255) : 0;
            if (limit) {
                const int ilevel = (sgf >> (16 + 8 * i4)) & 255, hev_t = (sgh >> (8 * i4)) & 255;
                const int inner = is_i4 || nonzero;
                const int t_mb = 2 * (limit + 4) + 1, t_in = 2 * limit + 1;
                if (ftype == 1) {  // simple: luma only
                    if (has_left && lane < 16) simple_line(Fy + lane * 32, 1, t_mb);
                    WSYNC();
                    if (inner && lane < 16)
                        for (int k = 1; k < 4; ++k) simple_line(Fy + lane * 32 + 4 * k, 1, t_in);
                    WSYNC();
                    if (has_top && lane < 16) simple_line(Fy + lane, 32, t_mb);
                    WSYNC();
                    if (inner && lane < 16)
                        for (int k = 1; k < 4; ++k) simple_line(Fy + 4 * k * 32 + lane, 32, t_in);
                } else {
                    uint8_t* const fc = lane < 24 ? Fu : Fv;
                    const int cl = lane < 24 ? lane - 16 : lane - 24;
                    if (has_left && lane < 32) {
                        uint8_t* p = lane < 16 ? Fy + lane * 32 : fc + cl * 16;
                        filter_line(p, 1, t_mb, ilevel, hev_t, true);
                    }
                    // (luma lanes 0-15 and chroma lanes 16-31 on one code path: pointer, pitch and
                    // edge count per lane, so a phase is not run twice under two masks)
                    const bool lu = lane < 16;
                    uint8_t* const rowp = lu ? Fy + lane * 32 : fc + cl * 16;  // this lane's row
                    uint8_t* const colp = lu ? Fy + lane : fc + cl;             // this lane's column
                    const int pitch = lu ? 32 : 16, nin = lu ? 4 : 2;           // inner edges: 3 luma, 1 chroma
                    WSYNC();
                    if (inner && lane < 32)
                        for (int k = 1; k < 4; ++k)
                            if (k < nin) filter_line(rowp + 4 * k, 1, t_in, ilevel, hev_t, false);
                    WSYNC();
                    if (has_top && lane < 32) filter_line(colp, pitch, t_mb, ilevel, hev_t, true);
                    WSYNC();
                    if (inner && lane < 32)
                        for (int k = 1; k < 4; ++k)
                            if (k < nin) filter_line(colp + 4 * k * pitch, pitch, t_in, ilevel, hev_t, false);
                }
                WSYNC();
                if (has_top) {  // the MB above's filtered bottom rows
                    if (lane < 4) {
                        __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4*>(Fy + (lane - 4) * 32)[0], rY,
                                                               (uint32_t)(16 * mb_y - 4 + lane) * ys + 16 * mb_x, 0, kCpolSc1);
                    } else if (lane >= 8 && lane < 16) {
                        const int k = lane - 8, c = k >> 2, r = k & 3;
                        __builtin_amdgcn_raw_buffer_store_b64(reinterpret_cast<const u32x2*>((c ? Fv : Fu) + (r - 4) * 16)[0],
                                                              c ? rV : rU, (uint32_t)(8 * mb_y - 4 + r) * uvs + 8 * mb_x,
                                                              0, kCpolSc1);
                    }
                }
            }
            // ---- out: the MB to the left, final now; at the row's end this one too ----
            if (has_left) {
                if (lane < 16) {
                    __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4*>(Fy + lane * 32 - 16)[0], rY,
                                                           (uint32_t)(16 * mb_y + lane) * ys + 16 * (mb_x - 1), 0, kCpolSc1);
                } else if (lane < 32) {
                    const int k = lane - 16, c = k >> 3, r = k & 7;
                    __builtin_amdgcn_raw_buffer_store_b64(reinterpret_cast<const u32x2*>((c ? Fv : Fu) + r * 16 - 8)[0],
                                                          c ? rV : rU, (uint32_t)(8 * mb_y + r) * uvs + 8 * (mb_x - 1), 0,
                                                          kCpolSc1);
                }
            }
            if (mb_x == mb_w - 1) {
                if (lane >= 32 && lane < 48) {
                    const int r = lane - 32;
                    __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4*>(Fy + r * 32)[0], rY,
                                                           (uint32_t)(16 * mb_y + r) * ys + 16 * mb_x, 0, kCpolSc1);
                } else if (lane >= 48) {
                    const int k = lane - 48, c = k >> 3, r = k & 7;
                    __builtin_amdgcn_raw_buffer_store_b64(reinterpret_cast<const u32x2*>((c ? Fv : Fu) + r * 16)[0],
                                                          c ? rV : rU, (uint32_t)(8 * mb_y + r) * uvs + 8 * mb_x, 0, kCpolSc1);
                }
            }
            WSYNC();
            // this MB becomes the one to the left
            if (lane < 16) {
                reinterpret_cast<u32x4*>(Fy + lane * 32 - 16)[0] = reinterpret_cast<const u32x4*>(Fy + lane * 32)[0];
            } else if (lane < 32) {
                const int k = lane - 16, c = k >> 3, r = k & 7;
                uint8_t* F = c ? Fv : Fu;
                reinterpret_cast<u32x2*>(F + r * 16 - 8)[0] = reinterpret_cast<const u32x2*>(F + r * 16)[0];
            }
            // publish: every store of this MB step has left (sc1), then the flag
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(prog + mb_y, (uint32_t)mb_x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (mb_x + 1 < mb_w) {
                c0 = c1;
                c1 = coef_at[mb + 2];
                e0 = c0 + lane < c1 ? coef[c0 + lane] : ~0u;
            }
            WSYNC();
        }
    }
}

// fancy upsampling + colour: one workgroup per output row of one image
__global__ __launch_bounds__(256) void k_vp8d_rgb(const DImg* __restrict__ imgs) {
    const cptr<DImg> di = (cptr<DImg>)imgs + blockIdx.y;
    const cptr<DFrame> fr = (cptr<DFrame>)di->fr;
    const int w = fr->w, h = fr->h, r = blockIdx.x;
    if (r >= h) return;
    const int uvh = (h + 1) >> 1;
    int nr, fr_;
    if (r == 0) {
        nr = fr_ = 0;
    } else if (r & 1) {
        nr = (r - 1) >> 1;
        fr_ = min((r + 1) >> 1, uvh - 1);
    } else {
        nr = r >> 1;
        fr_ = nr - 1;
    }
    const uint8_t* yrow = di->y + (size_t)r * di->ys;
    const uint8_t *nu = di->u + (size_t)nr * di->uvs, *fu = di->u + (size_t)fr_ * di->uvs;
    const uint8_t *nv = di->v + (size_t)nr * di->uvs, *fv = di->v + (size_t)fr_ * di->uvs;
    uint8_t* out = di->out + (size_t)r * di->out_pitch;
    for (int c = threadIdx.x; c < w; c += 256) {
        const int yy = yrow[c], u = fancy_chroma(nu, fu, c, w), v = fancy_chroma(nv, fv, c, w);
        out[3 * c + 0] = (uint8_t)yuv_r(yy, v);
        out[3 * c + 1] = (uint8_t)yuv_g(yy, u, v);
        out[3 * c + 2] = (uint8_t)yuv_b(yy, u);
    }
}

hipError_t launch_vp8d_recon(const DImg* imgs, int n, uint32_t total_rows, uint32_t* ticket, hipStream_t s) {
    // about one wave per CU: the rows in flight are bounded by the wavefront anyway
    const uint32_t grid = total_rows < 256 ? total_rows : 256;
    hipLaunchKernelGGL(k_vp8d_recon, dim3(grid), dim3(64), 0, s, imgs, n, ticket);
    return hipGetLastError();
}
hipError_t launch_vp8d_rgb(const DImg* imgs, int n, int max_h, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8d_rgb, dim3(max_h, n), dim3(256), 0, s, imgs);
    return hipGetLastError();
}

}  // namespace vp8d
}  // namespace ik
