// ik_kernels.hip -- hand-written gfx950 (CDNA4, wave64) kernels of the transform
// hot path (reference src/transform.rs:62-150):
//
//   k_resize_fused<A>  resize_image's resampler (image 0.25.8 imageops::resize:
//                      vertical_sample then horizontal_sample) fused in one pass:
//                      source rows stream HBM -> VGPRs once per column strip, the
//                      f32 vertical intermediate lives only in LDS.
//   k_vert_naive / k_horz_naive   general fallback (huge ratios, extreme upscales)
//   k_webp_yuv420      encode_image webp branch front end: to_rgb8 + libwebp's
//                      RGB -> YUV420 (gamma-corrected chroma averaging)
//   k_jpeg_coeffs      encode_image jpeg branch front end: to_rgb8 + f32 RGB->YCbCr
//                      + libjpeg-islow FDCT + quantise (image JpegEncoder)
//
// Bit-exactness with the reference's f32 arithmetic: no FMA contraction in this
// file (rustc never contracts), sequential tap order, host-computed weights,
// correctly rounded division, Rust round-half-away-from-zero.
#include "ik_internal.h"

#include <utility>

#pragma clang fp contract(off)

namespace ik {

__device__ __forceinline__ int lds_idx(int i) { return i + ((i >> 5) << 2); }

// Read-only plan tables through the constant address space: wave-uniform
// addresses then compile to scalar (SMEM) loads instead of vector loads +
// v_readfirstlane (the tables are never written by a kernel).
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
// output rows in the global address space: global_store (vmcnt only).  A generic
// pointer makes them flat_store, which count in vmcnt and lgkmcnt; with one
// pending, LLVM's wait-count pass cannot order vmcnt and falls back to vmcnt(0)
// at every row of the fused kernel's prefetch ring (measured 1.44 vs 1.03 ms per
// 64 x 4096^2 -> 512^2 Triangle launch when dst became a loaded generic pointer)
typedef __attribute__((address_space(1))) uint8_t g_u8;
template <typename T>
__device__ __forceinline__ cptr<T> as_const(const T* p) { return (cptr<T>)p; }

// clamp(t, 0, 255) then f32::round (half away from zero) -> u8   (sample.rs FloatNearest)
__device__ __forceinline__ uint8_t float_nearest_u8(float t) {
    t = t < 0.0f ? 0.0f : (t > 255.0f ? 255.0f : t);
    return (uint8_t)roundf(t);
}

// LDS row layout of the vertical results.  C != 3: strip byte b at word lds_idx(b)
// (4 pad words per 32).  C == 3: x = b + phi (phi = sb % 3, so x = 0 starts a pixel)
// at word x + x / 24 -- one pad word per 8 pixels, never inside a pixel, so the
// horizontal pass reads a pixel's three channels at one address with immediate
// offsets, and 8-pixel lanes (25 words apart) hit distinct banks.
struct RowPut {
    int lo, hi;  // C == 3: word of the lane's first byte; +1 from the pad crossing on
    int phi;     // C == 3: sb % 3 (wave-uniform); -1: the 4-per-32 layout (lo = lds_idx)
};

__device__ __forceinline__ RowPut row_put_init(int C, int sb) {
    RowPut r;
    const int b0 = kBytesPerLane * (int)threadIdx.x;
    if (C == 3) {
        r.phi = sb % 3;
        const int x0 = b0 + r.phi;
        r.lo = x0 + ((x0 * 2731) >> 16);  // x0 / 24 for x0 < 2200
        // only a lane whose bytes start at 16 + phi (mod 24) crosses a pad, at byte 8 - phi
        r.hi = r.lo + (((b0 % 24) == 16 && r.phi > 0) ? 1 : 0);
    } else {
        r.phi = -1;
        r.lo = r.hi = lds_idx(b0);
    }
    return r;
}

__device__ __forceinline__ void row_put(float* __restrict__ row, const RowPut& r, const float (&v)[kBytesPerLane]) {
    if (r.phi < 0) {
        *reinterpret_cast<float4*>(row + r.lo) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(row + r.lo + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else if (r.phi == 0) {
#pragma unroll
        for (int i = 0; i < kBytesPerLane; ++i) row[r.lo + i] = v[i];
    } else if (r.phi == 1) {
#pragma unroll
        for (int i = 0; i < kBytesPerLane; ++i) row[(i < 7 ? r.lo : r.hi) + i] = v[i];
    } else {
#pragma unroll
        for (int i = 0; i < kBytesPerLane; ++i) row[(i < 6 ? r.lo : r.hi) + i] = v[i];
    }
}

// Horizontal pass over `nrows` (<= F) completed vertical rows staged
// in LDS.  Lane = (row, output column) of the strip, all C channels per lane:
// one LDS read of C consecutive f32 per tap (ds_read_b128 for RGBA; the 4-per-32
// word padding makes the 36-word column stride bank-conflict free), C separate
// sequential sums, one C-byte store.  Taps run over the plan's Tx (a multiple of
// 4; zero weights past the column's own count), kHTaps at a time so their LDS
// reads are in flight together.  A zero-weight tap past the strip reads finite
// data (the next LDS row or the tables after the rows; the rows are zeroed at the
// start) and adds +-0, which leaves the sum bit-identical.
// out(r, ox, c) = round(sum_k tmp[r][(lx[ox]+k)*C + c] * wx[ox][k]), sequential k.
template <int C, bool FMA, int kHTaps = 2>
__device__ __forceinline__ void horizontal_rows_c(const ResizeArgs& a, const float* __restrict__ lds,
                                                  const float* __restrict__ sw, const int* __restrict__ soff,
                                                  int r0, int nrows, int ox0, int nox, int hq, int hox,
                                                  g_u8* __restrict__ dst) {
    const int total = nox * nrows;
    const int Tx = a.Tx;
    for (int v = threadIdx.x; v < total; v += kThreads) {
        int q = hq, oxl = hox;  // (v / nox, v % nox) for v = threadIdx.x, precomputed
        if (v != (int)threadIdx.x) { q = v / nox; oxl = v - q * nox; }
        const float* __restrict__ w = sw + oxl * Tx;
        const float* __restrict__ row = lds + q * kRowWords;
        const int base = soff[oxl];
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.0f;
#pragma unroll 1
        for (int k = 0; k < Tx; k += kHTaps) {
            float wk[kHTaps];
            if constexpr (kHTaps == 4) {
                const float4 w4 = *reinterpret_cast<const float4*>(w + k);
                wk[0] = w4.x; wk[1] = w4.y; wk[2] = w4.z; wk[3] = w4.w;
            } else {
                const float2 w2 = *reinterpret_cast<const float2*>(w + k);
                wk[0] = w2.x; wk[1] = w2.y;
            }
            float t[kHTaps][C];
#pragma unroll
            for (int u = 0; u < kHTaps; ++u) {
                const int idx = base + (k + u) * C;
                if constexpr (C == 4) {
                    const float4 t4 = *reinterpret_cast<const float4*>(row + lds_idx(idx));
                    t[u][0] = t4.x; t[u][1] = t4.y; t[u][2] = t4.z; t[u][3] = t4.w;
                } else if constexpr (C == 2) {
                    const float2 t2 = *reinterpret_cast<const float2*>(row + lds_idx(idx));
                    t[u][0] = t2.x; t[u][1] = t2.y;
                } else if constexpr (C == 3) {
                    // base counts pixels here (row_put's RGB layout: pixel p at 3p + p/8)
                    const int px = base + k + u;
                    const float* __restrict__ pp = row + 3 * px + (px >> 3);
                    t[u][0] = pp[0]; t[u][1] = pp[1]; t[u][2] = pp[2];
                } else {
                    t[u][0] = row[lds_idx(idx)];
                }
            }
#pragma unroll
            for (int u = 0; u < kHTaps; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if constexpr (FMA) {
                        acc[c] = __builtin_fmaf(t[u][c], wk[u], acc[c]);
                    } else {
                        const float prod = t[u][c] * wk[u];
                        acc[c] = acc[c] + prod;
                    }
                }
        }
        g_u8* o = dst + (size_t)(r0 + q) * a.dst_pitch + (size_t)(ox0 + oxl) * C;
        if constexpr (C == 4) {
            const unsigned u = (unsigned)float_nearest_u8(acc[0]) | ((unsigned)float_nearest_u8(acc[1]) << 8) |
                               ((unsigned)float_nearest_u8(acc[2]) << 16) | ((unsigned)float_nearest_u8(acc[3]) << 24);
            *reinterpret_cast<__attribute__((address_space(1))) unsigned*>(o) = u;  // dst rows are 256-B pitched, columns 4-B aligned
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) o[c] = float_nearest_u8(acc[c]);
        }
    }
}

template <bool FMA>
__device__ __forceinline__ void horizontal_rows(const ResizeArgs& a, const float* __restrict__ lds,
                                                const float* __restrict__ sw, const int* __restrict__ soff,
                                                int r0, int nrows, int ox0, int nox, int hq, int hox,
                                                g_u8* __restrict__ dst) {
    switch (a.C) {
    case 4:
        horizontal_rows_c<4, FMA>(a, lds, sw, soff, r0, nrows, ox0, nox, hq, hox, dst);
        break;
    case 3:  // four taps per iteration: twelve LDS reads in flight (6.48 -> 6.14 ms per 256 RGB 4096^2 -> 512^2
             // Lanczos3 launches, profiles/r04u_resize_horizontal_variants.txt; RGBA measured better at two)
        horizontal_rows_c<3, FMA, 4>(a, lds, sw, soff, r0, nrows, ox0, nox, hq, hox, dst);
        break;
    case 2: horizontal_rows_c<2, FMA>(a, lds, sw, soff, r0, nrows, ox0, nox, hq, hox, dst); break;
    default: horizontal_rows_c<1, FMA>(a, lds, sw, soff, r0, nrows, ox0, nox, hq, hox, dst); break;
    }
}

// waves per SIMD to ask the register allocator for (A=8 fits 168 VGPRs at 3)
template <int A>
struct FusedOcc { static constexpr int value = A <= 4 ? 4 : (A <= 8 ? 3 : 1); };

// Fused resampler.  Workgroup = (column strip, band of output rows, image).
// Each lane owns kBytesPerLane consecutive bytes of the strip (the vertical pass
// is channel-agnostic) and sweeps the band's source rows top to bottom once, as
// a host-built sequence of steps: step k brings in up to R new source rows and
// scatters each converted row into the A rolling accumulators acc[d] = output
// row next+d (host-computed activity mask + weights, wave-uniform scalar loads);
// an `emit` step completes row `next`: acc[0] goes to LDS and the accumulators
// shift down.  Prefetch is a rolling two-step register ring: step k sits in
// buf[k&1]; as soon as row j of step k is converted its registers are refilled
// (unconditionally, so the compiler's vmcnt bookkeeping stays exact) with row j
// of step k+2, keeping ~2R loads per lane in flight.  Every F
// completed rows the workgroup runs the horizontal pass from LDS.  LDS is
// dynamic: [F rows of f32 tmp][strip weights if WL][column offsets].
template <int A, int R, int F, bool WL, bool FMA>
__global__ __launch_bounds__(kThreads, FusedOcc<A>::value) void k_resize_fused(ResizeArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];

    // XCD-aware order: hardware deals workgroup h to XCD h % 8, so logical tile L
    // = (h % 8)-th eighth of the grid + h / 8 gives each XCD a contiguous run of
    // (strip, band, image) tiles; neighbouring strips (which share the 128-B lines
    // at their edges) and neighbouring bands then meet in the same L2.
    const int G = (int)gridDim.x;
    const int h = (int)blockIdx.x;
    const int per = G >> 3, rem = G & 7, x = h & 7;
    const int L = x * per + (x < rem ? x : rem) + (h >> 3);
    const int tiles = a.NS * a.NB;
    const int img = L / tiles;
    const int tile = L - img * tiles;
    const int strip = tile % a.NS;
    const int band = tile / a.NS;
    const cptr<int> strips = as_const(a.strips);
    const cptr<int> bands = as_const(a.bands);
    const cptr<int> shdr = as_const(a.step_hdr);
    const cptr<unsigned long long> smask = as_const(a.step_mask);
    const cptr<float> sw = as_const(a.step_w);
    const cptr<int> bstep = as_const(a.band_step);
    const int ox0 = strips[3 * strip], ox1 = strips[3 * strip + 1], sb = strips[3 * strip + 2];
    const int nox = ox1 - ox0;
    const int oy0 = bands[2 * band], oy1 = bands[2 * band + 1];
    const int kb = bstep[band], ke = bstep[band + 1];
    // per-image bases through the constant address space (img is wave-uniform:
    // scalar loads); dst in the global address space (g_u8, see above)
    const uint8_t* __restrict__ src =
        a.src_tab ? reinterpret_cast<const uint8_t*>(as_const(a.src_tab)[img]) : a.src + (size_t)img * a.src_img_stride;
    g_u8* __restrict__ dst = (g_u8*)(a.dst_tab ? reinterpret_cast<uint8_t*>(as_const(a.dst_tab)[img])
                                               : a.dst + (size_t)img * a.dst_img_stride);

    float* __restrict__ s_w = lds + F * kRowWords;
    int* __restrict__ s_off = reinterpret_cast<int*>(s_w + (WL ? a.max_strip_weights : 0));
    for (int t = threadIdx.x; t < nox; t += kThreads)  // byte in the strip (C == 3: pixel, see row_put)
        s_off[t] = a.C == 3 ? a.lx[ox0 + t] - sb / 3 : a.lx[ox0 + t] * a.C - sb;
    for (int t = threadIdx.x; t < F * kRowWords / 4; t += kThreads)
        reinterpret_cast<float4*>(lds)[t] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int hq = (int)threadIdx.x / nox, hox = (int)threadIdx.x - hq * nox;
    if (WL) {
        const float* __restrict__ gw = a.wx + (size_t)ox0 * a.Tx;
        for (int t = threadIdx.x; t < nox * a.Tx; t += kThreads) s_w[t] = gw[t];
    }
    const float* __restrict__ hw = WL ? s_w : a.wx + (size_t)ox0 * a.Tx;

    // Source rows through a buffer descriptor over this image: per-lane byte
    // offset in voffset (constant), row * pitch in soffset (scalar).
    const int mybyte = sb + kBytesPerLane * (int)threadIdx.x;
    const int voff = mybyte < a.row_bytes ? mybyte : 0;
    const unsigned long long base = (unsigned long long)src;
    const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)base);
    const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(base >> 32));
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)bhi << 32) | blo), (short)0, (int)(a.src_pitch * a.H), 0x00020000);
    const RowPut rput = row_put_init(a.C, sb);
    const int Hm1 = a.H - 1;
    const int pitch = (int)a.src_pitch;
    auto ld = [&](int row) -> uint2 {
        row = row < Hm1 ? row : Hm1;
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, row * pitch, 0);
        return make_uint2(v[0], v[1]);
    };

    float acc[A][kBytesPerLane];
#pragma unroll
    for (int d = 0; d < A; ++d)
#pragma unroll
        for (int j = 0; j < kBytesPerLane; ++j) acc[d][j] = 0.0f;

    uint2 buf0[R], buf1[R];
    {
        const int s0 = shdr[4 * kb];
        const int s1 = kb + 1 < ke ? shdr[4 * (kb + 1)] : s0;
#pragma unroll
        for (int j = 0; j < R; ++j) buf0[j] = ld(s0 + j);
#pragma unroll
        for (int j = 0; j < R; ++j) buf1[j] = ld(s1 + j);
    }
    __syncthreads();  // s_w / s_off / s_n ready

    int next = oy0;  // next output row to complete
    auto body = [&](int k, uint2 (&cur)[R]) {
        const int hstart = shdr[4 * k], hemit = shdr[4 * k + 2];
        const unsigned long long m = smask[k];
        const cptr<float> w = sw + (size_t)k * (R * A);
        const int s2 = k + 2 < ke ? shdr[4 * (k + 2)] : hstart;
        // all of the step's weights in SGPRs up front (a few wide scalar loads and
        // one wait, instead of one dependent load per active tap)
        constexpr int kWregs = R * A <= 64 ? R * A : 1;
        float wv[kWregs];
        if constexpr (R * A <= 64) {
#pragma unroll
            for (int i = 0; i < kWregs; ++i) wv[i] = w[i];
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if ((m >> (j * A)) & ((1ull << A) - 1ull)) {
                const uint2 raw = cur[j];
                float p[kBytesPerLane];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p[q] = (float)((raw.x >> (8 * q)) & 0xffu);
                    p[4 + q] = (float)((raw.y >> (8 * q)) & 0xffu);
                }
#pragma unroll
                for (int d = 0; d < A; ++d) {
                    if ((m >> (j * A + d)) & 1ull) {
                        float wt;
                        if constexpr (R * A <= 64) wt = wv[j * A + d];
                        else wt = w[j * A + d];
#pragma unroll
                        for (int q = 0; q < kBytesPerLane; ++q) {
                            if constexpr (FMA) {
                                acc[d][q] = __builtin_fmaf(p[q], wt, acc[d][q]);
                            } else {
#ifdef IK_ABL_NOVMATH  // dev ablation: the loads and conversions only
                                if (d == 0) acc[0][q] = acc[0][q] + p[q];
                                (void)wt;
#else
                                const float prod = p[q] * wt;
                                acc[d][q] = acc[d][q] + prod;
#endif
                            }
                        }
                    }
                }
            }
            cur[j] = ld(s2 + j);  // refill: row j of step k+2 (a valid re-read at the end)
        }
        if (hemit) {
            // row `next` complete -> LDS slot, shift the accumulators down
            row_put(lds + ((next - oy0) % F) * kRowWords, rput, acc[0]);
#pragma unroll
            for (int d = 0; d + 1 < A; ++d)
#pragma unroll
                for (int q = 0; q < kBytesPerLane; ++q) acc[d][q] = acc[d + 1][q];
#pragma unroll
            for (int q = 0; q < kBytesPerLane; ++q) acc[A - 1][q] = 0.0f;
            const int nrows = (next - oy0) % F + 1;
            if (nrows == F || next == oy1 - 1) {
#ifndef IK_ABL_NOBAR  // dev ablations: without the barriers / the horizontal pass (wrong pixels)
                __syncthreads();
#endif
#ifndef IK_ABL_NOHORZ
                horizontal_rows<FMA>(a, lds, hw, s_off, next - nrows + 1, nrows, ox0, nox, hq, hox, dst);
#endif
#ifndef IK_ABL_NOBAR
                __syncthreads();
#endif
            }
            ++next;
        }
    };

    // bands hold an even number of steps (ik_plan.cpp pads with a no-op step), so
    // both halves run unconditionally and the vmcnt accounting stays at 2R
    for (int k = kb; k < ke; k += 2) {
        body(k, buf0);
        body(k + 1, buf1);
    }
}

// Periodic resampler (integer ratio R, every output window inside A steps of R
// rows; ik_plan.cpp): the vertical pass of k_resize_fused without its step tables.
// Step t brings in rows R*t + per_base .. +R-1; output row y takes tap e*R + j from
// row j of step y + e, so each step feeds A open output rows and completes one.
// The loop is unrolled over G steps (G = A, or 2A for odd A, so that the two-step
// prefetch ring keeps its parity), which fixes every accumulator's role at compile
// time: the output that starts at phase u sits in acc[u], and the one that
// completes at phase u is acc[(u + 1) % A].  No masks, no shifts, no branches in the
// tap loop; a step's A*R weights come in with a few wide scalar loads.  Bands sweep
// a whole number of groups (ik_plan.cpp); steps past the band's last row and the
// first A-1 steps' rows of the band above accumulate rows that are never emitted.
// The horizontal pass, LDS layout and tile mapping are k_resize_fused's.
template <typename Fn, int... U>
__device__ __forceinline__ void unroll_seq(Fn&& f, std::integer_sequence<int, U...>) {
    (f(std::integral_constant<int, U>()), ...);
}

template <int A, int R, int F, bool WL>
__global__ __launch_bounds__(kThreads) void k_resize_periodic(ResizeArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int G = A % 2 ? 2 * A : A;
    const int Gd = (int)gridDim.x;
    const int h = (int)blockIdx.x;
    const int per = Gd >> 3, rem = Gd & 7, x = h & 7;
    const int L = x * per + (x < rem ? x : rem) + (h >> 3);
    const int tiles = a.NS * a.NBp;
    const int img = L / tiles;
    const int tile = L - img * tiles;
    const int strip = tile % a.NS;
    const int band = tile / a.NS;
    const cptr<int> strips = as_const(a.strips);
    const cptr<int> bands = as_const(a.per_bands);
    const cptr<float> pw = as_const(a.per_w);
    const int ox0 = strips[3 * strip], ox1 = strips[3 * strip + 1], sb = strips[3 * strip + 2];
    const int nox = ox1 - ox0;
    const int oy0 = bands[2 * band], oy1 = bands[2 * band + 1];
    const uint8_t* __restrict__ src =
        a.src_tab ? reinterpret_cast<const uint8_t*>(as_const(a.src_tab)[img]) : a.src + (size_t)img * a.src_img_stride;
    g_u8* __restrict__ dst = (g_u8*)(a.dst_tab ? reinterpret_cast<uint8_t*>(as_const(a.dst_tab)[img])
                                               : a.dst + (size_t)img * a.dst_img_stride);

    float* __restrict__ s_w = lds + F * kRowWords;
    int* __restrict__ s_off = reinterpret_cast<int*>(s_w + (WL ? a.max_strip_weights : 0));
    for (int t = threadIdx.x; t < nox; t += kThreads)  // byte in the strip (C == 3: pixel, see row_put)
        s_off[t] = a.C == 3 ? a.lx[ox0 + t] - sb / 3 : a.lx[ox0 + t] * a.C - sb;
    for (int t = threadIdx.x; t < F * kRowWords / 4; t += kThreads)
        reinterpret_cast<float4*>(lds)[t] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int hq = (int)threadIdx.x / nox, hox = (int)threadIdx.x - hq * nox;
    if (WL) {
        const float* __restrict__ gw = a.wx + (size_t)ox0 * a.Tx;
        for (int t = threadIdx.x; t < nox * a.Tx; t += kThreads) s_w[t] = gw[t];
    }
    const float* __restrict__ hw = WL ? s_w : a.wx + (size_t)ox0 * a.Tx;

    const int mybyte = sb + kBytesPerLane * (int)threadIdx.x;
    const int voff = mybyte < a.row_bytes ? mybyte : 0;
    const unsigned long long base = (unsigned long long)src;
    const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)base);
    const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(base >> 32));
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)bhi << 32) | blo), (short)0, (int)(a.src_pitch * a.H), 0x00020000);
    const RowPut rput = row_put_init(a.C, sb);
    const int Hm1 = a.H - 1;
    const int pitch = (int)a.src_pitch;
    const int rb = a.per_base;
    auto ld = [&](int row) -> uint2 {
        row = row < 0 ? 0 : (row < Hm1 ? row : Hm1);
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, row * pitch, 0);
        return make_uint2(v[0], v[1]);
    };

    float acc[A][kBytesPerLane];
#pragma unroll
    for (int d = 0; d < A; ++d)
#pragma unroll
        for (int j = 0; j < kBytesPerLane; ++j) acc[d][j] = 0.0f;
    const int t0 = oy0;
    const int t1 = t0 + ((oy1 - oy0 + A - 1 + G - 1) / G) * G;
    uint2 buf0[R], buf1[R];
#pragma unroll
    for (int j = 0; j < R; ++j) buf0[j] = ld(R * t0 + rb + j);
#pragma unroll
    for (int j = 0; j < R; ++j) buf1[j] = ld(R * (t0 + 1) + rb + j);
    __syncthreads();  // s_w / s_off ready

    auto step = [&](auto UC, int t, uint2 (&cur)[R]) {
        constexpr int U = decltype(UC)::value % A;
        // the scheduler keeps each step's work within the step (A=6, R=8: 117 VGPRs
        // instead of 124; the same speed either way)
        __builtin_amdgcn_sched_barrier(0);
        const cptr<float> w = pw + (size_t)t * (A * R);
        float wv[A * R];
#pragma unroll
        for (int i = 0; i < A * R; ++i) wv[i] = w[i];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint2 raw = cur[j];
            float p[kBytesPerLane];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[q] = (float)((raw.x >> (8 * q)) & 0xffu);
                p[4 + q] = (float)((raw.y >> (8 * q)) & 0xffu);
            }
#pragma unroll
            for (int e = 0; e < A; ++e) {
                const int slot = (U - e + A) % A;  // the output that started e steps ago
                const float wt = wv[e * R + j];
#pragma unroll
                for (int q = 0; q < kBytesPerLane; ++q) {
                    const float prod = p[q] * wt;
                    if (e == 0 && j == 0) acc[slot][q] = prod;  // its first tap
                    else acc[slot][q] = acc[slot][q] + prod;
                }
            }
            cur[j] = ld(R * (t + 2) + rb + j);  // refill: row j of step t+2
        }
        // the step's taps all land before the emit test: otherwise the compiler sinks
        // part of them into both sides of it and keeps the converted rows live across
        // (A=2, R=8: 167 VGPRs instead of ~70)
#pragma unroll
        for (int d = 0; d < A; ++d)
            asm volatile("" : "+v"(acc[d][0]), "+v"(acc[d][1]), "+v"(acc[d][2]), "+v"(acc[d][3]), "+v"(acc[d][4]),
                              "+v"(acc[d][5]), "+v"(acc[d][6]), "+v"(acc[d][7]));
        const int y = t - (A - 1);  // completed by this step
        if (y >= oy0 && y < oy1) {
            constexpr int done = (U + 1) % A;
            row_put(lds + ((y - oy0) % F) * kRowWords, rput, acc[done]);
            const int nrows = (y - oy0) % F + 1;
            if (nrows == F || y == oy1 - 1) {
#ifndef IK_ABL_NOBAR  // dev ablations, as in k_resize_fused
                __syncthreads();
#endif
#ifndef IK_ABL_NOHORZ
                horizontal_rows<false>(a, lds, hw, s_off, y - nrows + 1, nrows, ox0, nox, hq, hox, dst);
#endif
#ifndef IK_ABL_NOBAR
                __syncthreads();
#endif
            }
        }
    };
    for (int t = t0; t < t1; t += G)
        unroll_seq([&](auto UC) {
            constexpr int u = decltype(UC)::value;
            if constexpr (u & 1) step(UC, t + u, buf1);
            else step(UC, t + u, buf0);
        }, std::make_integer_sequence<int, G>());
}

// Fallback vertical pass: one thread per (byte column, output row, image).
__global__ __launch_bounds__(kThreads) void k_vert_naive(ResizeArgs a) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    const int r = blockIdx.y;
    const int img = blockIdx.z;
    if (b >= a.row_bytes) return;
    const uint8_t* __restrict__ src = a.src + (size_t)img * a.src_img_stride + b;
    const int l = a.ly[r], n = a.ny[r];
    const float* __restrict__ w = a.wy + (size_t)r * a.Ty;
    float t = 0.0f;
    for (int k = 0; k < n; ++k) {
        const float prod = (float)src[(size_t)(l + k) * a.src_pitch] * w[k];
        t = t + prod;
    }
    a.tmp[((size_t)img * a.nh + r) * a.row_bytes + b] = t;
}

// Fallback horizontal pass: one thread per (output byte, output row, image).
__global__ __launch_bounds__(kThreads) void k_horz_naive(ResizeArgs a) {
    const int v = blockIdx.x * kThreads + threadIdx.x;
    const int r = blockIdx.y;
    const int img = blockIdx.z;
    if (v >= a.nw * a.C) return;
    const int ox = v / a.C, c = v - ox * a.C;
    const float* __restrict__ t = a.tmp + ((size_t)img * a.nh + r) * a.row_bytes;
    const int n = a.nx[ox];
    const float* __restrict__ w = a.wx + (size_t)ox * a.Tx;
    int idx = a.lx[ox] * a.C + c;
    float acc = 0.0f;
    for (int k = 0; k < n; ++k, idx += a.C) {
        const float prod = t[idx] * w[k];
        acc = acc + prod;
    }
    a.dst[(size_t)img * a.dst_img_stride + (size_t)r * a.dst_pitch + v] = float_nearest_u8(acc);
}

// ---- 16-bit images (Rgb16 / Rgba16 / L16 / La16 from 16-bit PNG) ----------------
// image 0.25.8 resamples u16 samples with the same f32 sequence as u8 ones and
// clamps to u16::MAX before FloatNearest; the two passes of the fallback path,
// over samples instead of bytes (a.row_bytes counts samples here).
__global__ __launch_bounds__(kThreads) void k_vert_naive16(ResizeArgs a) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    const int r = blockIdx.y;
    if (b >= a.row_bytes) return;
    const int l = a.ly[r], n = a.ny[r];
    const float* __restrict__ w = a.wy + (size_t)r * a.Ty;
    float t = 0.0f;
    for (int k = 0; k < n; ++k) {
        const uint16_t v = *reinterpret_cast<const uint16_t*>(a.src + (size_t)(l + k) * a.src_pitch + 2 * (size_t)b);
        const float prod = (float)v * w[k];
        t = t + prod;
    }
    a.tmp[(size_t)r * a.row_bytes + b] = t;
}

__global__ __launch_bounds__(kThreads) void k_horz_naive16(ResizeArgs a) {
    const int v = blockIdx.x * kThreads + threadIdx.x;
    const int r = blockIdx.y;
    if (v >= a.nw * a.C) return;
    const int ox = v / a.C, c = v - ox * a.C;
    const float* __restrict__ t = a.tmp + (size_t)r * a.row_bytes;
    const int n = a.nx[ox];
    const float* __restrict__ w = a.wx + (size_t)ox * a.Tx;
    int idx = a.lx[ox] * a.C + c;
    float acc = 0.0f;
    for (int k = 0; k < n; ++k, idx += a.C) {
        const float prod = t[idx] * w[k];
        acc = acc + prod;
    }
    acc = acc < 0.0f ? 0.0f : (acc > 65535.0f ? 65535.0f : acc);
    *reinterpret_cast<uint16_t*>(a.dst + (size_t)r * a.dst_pitch + 2 * (size_t)v) = (uint16_t)roundf(acc);
}

hipError_t launch_resize16(const ResizePlan& plan, const uint8_t* src, size_t src_pitch, uint8_t* dst,
                           size_t dst_pitch, float* tmp, hipStream_t s) {
    ResizeArgs a = plan.args;
    a.src = src; a.src_pitch = src_pitch; a.src_img_stride = 0;
    a.dst = dst; a.dst_pitch = dst_pitch; a.dst_img_stride = 0;
    a.src_tab = nullptr; a.dst_tab = nullptr;
    a.tmp = tmp;
    dim3 g1((a.row_bytes + kThreads - 1) / kThreads, a.nh);
    hipLaunchKernelGGL(k_vert_naive16, g1, dim3(kThreads), 0, s, a);
    dim3 g2((a.nw * a.C + kThreads - 1) / kThreads, a.nh);
    hipLaunchKernelGGL(k_horz_naive16, g2, dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// to_rgb8 / to_rgba8 of a 16-bit image, per sample: u8 = (v + 128) / 257
// (image's u16 -> u8 rescale, rounding; parity unpinned)
__global__ __launch_bounds__(kThreads) void k_u16_to_u8(const uint8_t* src, size_t sp, uint8_t* dst, size_t dp,
                                                        int row_samples) {
    const int x = blockIdx.x * kThreads + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= row_samples) return;
    const uint32_t v = *reinterpret_cast<const uint16_t*>(src + (size_t)y * sp + 2 * (size_t)x);
    dst[(size_t)y * dp + x] = (uint8_t)((v + 128u) / 257u);
}

hipError_t launch_u16_to_u8(const uint8_t* src, size_t sp, uint8_t* dst, size_t dp, int row_samples, int rows,
                            hipStream_t s) {
    if (row_samples <= 0 || rows <= 0) return hipSuccess;
    dim3 g((row_samples + kThreads - 1) / kThreads, rows);
    hipLaunchKernelGGL(k_u16_to_u8, g, dim3(kThreads), 0, s, src, sp, dst, dp, row_samples);
    return hipGetLastError();
}

#define IK_PERIODIC_INSTANCES(X) X(2, 2) X(2, 4) X(2, 8) X(4, 2) X(4, 4) X(4, 8) X(6, 2) X(6, 4) X(6, 8)

bool periodic_instance(int A, int R) {
#define IK_PER_HAS(A_, R_) if (A == A_ && R == R_) return true;
    IK_PERIODIC_INSTANCES(IK_PER_HAS)
#undef IK_PER_HAS
    return false;
}

// IK_RESIZE_PERIODIC=0: periodic geometries on k_resize_fused too (A/B, tests)
static bool periodic_enabled() {
    const char* e = getenv("IK_RESIZE_PERIODIC");
    return !(e && e[0] == '0');
}

const char* resize_kernel_name(const ResizePlan& plan, size_t src_pitch) {
    if (!(plan.slots > 0 && resize_fused_fits(src_pitch, (size_t)plan.H))) return "k_vert_naive";
    if (plan.per_A && resize_mode() != IK_RESIZE_FMA && plan.flush == 3 && periodic_enabled() &&
        periodic_instance(plan.per_A, plan.per_R))
        return "k_resize_periodic";
    return "k_resize_fused";
}

size_t resize_lds_bytes(const ResizeArgs& a, bool wl, int flush) {
    return sizeof(float) * ((size_t)flush * kRowWords + (wl ? (size_t)a.max_strip_weights : 0) +
                            (size_t)a.max_strip_cols);
}

// Instances that fit the register file without spilling (ik_plan.cpp picks A, R);
// X(A, R, F) for every flush depth F the plan may choose.
#define IK_FUSED_INSTANCES(X)                                               \
    X(2, 4, 2) X(2, 4, 3) X(2, 4, 4) X(2, 8, 2) X(2, 8, 3) X(2, 8, 4)       \
    X(4, 4, 2) X(4, 4, 3) X(4, 4, 4) X(4, 8, 2) X(4, 8, 3) X(4, 8, 4)       \
    X(8, 4, 2) X(8, 4, 3) X(8, 4, 4) X(8, 8, 2) X(8, 8, 3) X(8, 8, 4)       \
    X(16, 4, 2) X(16, 4, 3) X(16, 4, 4)

hipError_t launch_resize(const ResizePlan& plan, const uint8_t* src, size_t src_pitch,
                         size_t src_img_stride, uint8_t* dst, size_t dst_pitch,
                         size_t dst_img_stride, int n, float* naive_tmp, hipStream_t s,
                         const uint64_t* src_tab, const uint64_t* dst_tab) {
    ResizeArgs a = plan.args;
    a.src = src; a.src_pitch = src_pitch; a.src_img_stride = src_img_stride;
    a.dst = dst; a.dst_pitch = dst_pitch; a.dst_img_stride = dst_img_stride;
    a.src_tab = src_tab; a.dst_tab = dst_tab;
    a.tmp = naive_tmp;
    if (src_tab && !(plan.slots > 0 && resize_fused_fits(src_pitch, (size_t)a.H))) return hipErrorInvalidValue;
    if (plan.slots > 0 && resize_fused_fits(src_pitch, (size_t)a.H)) {
        dim3 grid(plan.NS * plan.NB * n);  // 1-D: the kernel maps it XCD-aware
        const bool wl = plan.weights_in_lds;
        const size_t lds = resize_lds_bytes(a, wl, plan.flush);
        const bool fma = resize_mode() == IK_RESIZE_FMA;
        if (plan.per_A && !fma && plan.flush == 3 && periodic_enabled()) {
            dim3 pgrid(plan.NS * a.NBp * n);
#define IK_PLAUNCH(A_, R_)                                                                                    \
    if (plan.per_A == A_ && plan.per_R == R_) {                                                               \
        if (wl) hipLaunchKernelGGL((k_resize_periodic<A_, R_, 3, true>), pgrid, dim3(kThreads), lds, s, a);   \
        else hipLaunchKernelGGL((k_resize_periodic<A_, R_, 3, false>), pgrid, dim3(kThreads), lds, s, a);     \
        return hipGetLastError();                                                                             \
    }
            IK_PERIODIC_INSTANCES(IK_PLAUNCH)
#undef IK_PLAUNCH
        }
#define IK_LAUNCH(A_, R_, F_)                                                                                 \
    if (plan.slots == A_ && plan.rows == R_ && plan.flush == F_) {                                            \
        if (fma) {                                                                                            \
            if (wl) hipLaunchKernelGGL((k_resize_fused<A_, R_, F_, true, true>), grid, dim3(kThreads), lds, s, a); \
            else hipLaunchKernelGGL((k_resize_fused<A_, R_, F_, false, true>), grid, dim3(kThreads), lds, s, a);   \
        } else {                                                                                              \
            if (wl) hipLaunchKernelGGL((k_resize_fused<A_, R_, F_, true, false>), grid, dim3(kThreads), lds, s, a); \
            else hipLaunchKernelGGL((k_resize_fused<A_, R_, F_, false, false>), grid, dim3(kThreads), lds, s, a);   \
        }                                                                                                     \
        return hipGetLastError();                                                                             \
    }
        IK_FUSED_INSTANCES(IK_LAUNCH)
#undef IK_LAUNCH
        return hipErrorInvalidValue;
    }
    if (!naive_tmp) return hipErrorInvalidValue;
    dim3 g1((a.row_bytes + kThreads - 1) / kThreads, a.nh, n);
    hipLaunchKernelGGL(k_vert_naive, g1, dim3(kThreads), 0, s, a);
    dim3 g2((a.nw * a.C + kThreads - 1) / kThreads, a.nh, n);
    hipLaunchKernelGGL(k_horz_naive, g2, dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// WebP front end: to_rgb8 (image 0.25.8: Rgba drops alpha, Luma replicates) then
// libwebp ImportYUVAFromRGBA for opaque input (src/enc/picture_csp_enc.c):
//   Y = (16839 r + 33059 g + 6420 b + 2^15 + (16 << 16)) >> 16
//   U/V from gamma-linearised 2x2 sums (SUM4 / SUM2 on odd edges), rounding 2^17.
// One thread per chroma sample (2x2 luma block).
__device__ __forceinline__ void load_rgb(const uint8_t* __restrict__ row, int x, int C, int& r,
                                         int& g, int& b) {
    const uint8_t* p = row + x * C;
    if (C >= 3) { r = p[0]; g = p[1]; b = p[2]; }
    else { r = g = b = p[0]; }
}

__device__ __forceinline__ int webp_y(int r, int g, int b) {
    return (16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16;
}

__device__ __forceinline__ int webp_clip_uv(int uv) {
    uv = (uv + (1 << 17) + (128 << 18)) >> 18;
    return ((uv & ~0xff) == 0) ? uv : (uv < 0) ? 0 : 255;
}

__device__ __forceinline__ int lin_to_gamma(const int* __restrict__ tab, uint32_t base, int shift) {
    const int v = (int)(base << shift);
    const int pos = v >> 9;
    const int x = v & 511;
    const int y = tab[pos + 1] * x + tab[pos] * (512 - x);
    return (y + 64) >> 7;
}

__global__ __launch_bounds__(kThreads) void k_webp_yuv420(const uint8_t* __restrict__ src, int w,
                                                          int h, int C, size_t pitch,
                                                          size_t img_stride, uint8_t* __restrict__ Y,
                                                          size_t yuv_img_stride,
                                                          const uint16_t* __restrict__ g2l,
                                                          const int* __restrict__ l2g,
                                                          const uint64_t* __restrict__ src_tab) {
    __shared__ uint16_t s_g2l[256];
    __shared__ int s_l2g[33];
    for (int t = threadIdx.x; t < 256; t += kThreads) s_g2l[t] = g2l[t];
    if (threadIdx.x < 33) s_l2g[threadIdx.x] = l2g[threadIdx.x];
    __syncthreads();
    const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
    const int cx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int cy = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int img = blockIdx.z;
    if (cx >= uvw || cy >= uvh) return;
    const uint8_t* __restrict__ base =
        src_tab ? reinterpret_cast<const uint8_t*>(src_tab[img]) : src + (size_t)img * img_stride;
    uint8_t* __restrict__ y_img = Y + (size_t)img * yuv_img_stride;
    uint8_t* __restrict__ u_img = y_img + (size_t)w * h;
    uint8_t* __restrict__ v_img = u_img + (size_t)uvw * uvh;
    const int x0 = 2 * cx, y0 = 2 * cy;
    const bool has_x1 = x0 + 1 < w, has_y1 = y0 + 1 < h;
    int R[4], G[4], B[4];
    const uint8_t* row0 = base + (size_t)y0 * pitch;
    const uint8_t* row1 = base + (size_t)(has_y1 ? y0 + 1 : y0) * pitch;  // rgb_stride = 0 on odd last row
    load_rgb(row0, x0, C, R[0], G[0], B[0]);
    load_rgb(row1, x0, C, R[2], G[2], B[2]);
    if (has_x1) {
        load_rgb(row0, x0 + 1, C, R[1], G[1], B[1]);
        load_rgb(row1, x0 + 1, C, R[3], G[3], B[3]);
    } else {
        R[1] = R[0]; G[1] = G[0]; B[1] = B[0];
        R[3] = R[2]; G[3] = G[2]; B[3] = B[2];
    }
    y_img[(size_t)y0 * w + x0] = (uint8_t)webp_y(R[0], G[0], B[0]);
    if (has_x1) y_img[(size_t)y0 * w + x0 + 1] = (uint8_t)webp_y(R[1], G[1], B[1]);
    if (has_y1) {
        y_img[(size_t)(y0 + 1) * w + x0] = (uint8_t)webp_y(R[2], G[2], B[2]);
        if (has_x1) y_img[(size_t)(y0 + 1) * w + x0 + 1] = (uint8_t)webp_y(R[3], G[3], B[3]);
    }
    int sum[3];
    const int* comp[3] = {R, G, B};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int* q = comp[c];
        if (has_x1) {
            const uint32_t s4 = s_g2l[q[0]] + s_g2l[q[1]] + s_g2l[q[2]] + s_g2l[q[3]];
            sum[c] = lin_to_gamma(s_l2g, s4, 0);
        } else {
            const uint32_t s2 = s_g2l[q[0]] + s_g2l[q[2]];
            sum[c] = lin_to_gamma(s_l2g, s2, 1);
        }
    }
    u_img[(size_t)cy * uvw + cx] = (uint8_t)webp_clip_uv(-9719 * sum[0] - 19081 * sum[1] + 28800 * sum[2]);
    v_img[(size_t)cy * uvw + cx] = (uint8_t)webp_clip_uv(28800 * sum[0] - 24116 * sum[1] - 4684 * sum[2]);
}

hipError_t launch_webp_yuv420(const uint8_t* src, int w, int h, int C, size_t pitch,
                              size_t img_stride, uint8_t* yuv, size_t yuv_img_stride, int n, const uint16_t* gamma_to_lin,
                              const int* lin_to_gamma_tab, hipStream_t s, const uint64_t* src_tab) {
    const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
    dim3 grid((uvw + 63) / 64, (uvh + 3) / 4, n);
    hipLaunchKernelGGL(k_webp_yuv420, grid, dim3(kThreads), 0, s, src, w, h, C, pitch, img_stride,
                       yuv, yuv_img_stride, gamma_to_lin, lin_to_gamma_tab, src_tab);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// AVIF front end (image 0.25.8 AvifEncoder: to_rgba8 -> ravif RGB->YCbCr): BT.601
// full-range 4:4:4 planes plus the alpha plane; transparent[z] becomes 1 when any
// alpha of image z is < 255 (ravif then codes an alpha plane; the caller zeroes
// the flags).  One lane per pixel, grid.z = image of the batch.
__global__ __launch_bounds__(kThreads) void k_avif_yuv444(const uint8_t* __restrict__ src, int w, int h, int C,
                                                          size_t pitch, size_t img_stride,
                                                          uint8_t* __restrict__ planes, size_t plane_img_stride,
                                                          int* __restrict__ transparent) {
    const int x = blockIdx.x * kThreads + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
    if (x >= w) return;
    const uint8_t* p = src + img_stride * z + (size_t)y * pitch + (size_t)x * C;
    planes += plane_img_stride * z;
    int r, g, b, al = 255;
    if (C >= 3) { r = p[0]; g = p[1]; b = p[2]; if (C == 4) al = p[3]; }
    else { r = g = b = p[0]; if (C == 2) al = p[1]; }
    const float Y = 0.299f * r + 0.587f * g + 0.114f * b;
    const float U = (b - Y) * (0.5f / 0.886f) + 128.0f;
    const float V = (r - Y) * (0.5f / 0.701f) + 128.0f;
    auto q8 = [](float v) -> uint8_t { v = floorf(v + 0.5f); return (uint8_t)(v < 0.f ? 0.f : (v > 255.f ? 255.f : v)); };
    const size_t n = (size_t)w * h, i = (size_t)y * w + x;
    planes[i] = q8(Y);
    planes[n + i] = q8(U);
    planes[2 * n + i] = q8(V);
    planes[3 * n + i] = (uint8_t)al;
    // one atomic per wave at most: the first lane that sees a translucent pixel
    const uint64_t m = __ballot(al != 255);
    if (m && (threadIdx.x & 63) == (int)__builtin_ctzll(m)) atomicOr(transparent + z, 1);
}

hipError_t launch_avif_yuv444(const uint8_t* src, int w, int h, int C, size_t pitch, size_t img_stride,
                              uint8_t* planes, size_t plane_img_stride, int* transparent, int n, hipStream_t s) {
    if (hipError_t e = hipMemsetAsync(transparent, 0, sizeof(int) * (size_t)n, s)) return e;
    hipLaunchKernelGGL(k_avif_yuv444, dim3((w + kThreads - 1) / kThreads, h, n), dim3(kThreads), 0, s, src, w, h, C,
                       pitch, img_stride, planes, plane_img_stride, transparent);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// JPEG front end (image 0.25.8 JpegEncoder::encode_rgb, 4:4:4): per 8x8 block
// and component: pixel_at_or_near -> rgb_to_ycbcr (f32, `as u8`) -> fdct (libjpeg
// 9a islow, integer) -> ((c / 8) as f32 / q).round().  Workgroup = 8 MCUs x 3
// components x 8 lines; pass 1 (rows) and pass 2 (columns) meet in LDS.
constexpr int CB = 13, P1 = 2;

__device__ __forceinline__ uint8_t f32_as_u8(float v) {
    if (!(v > 0.0f)) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}

__device__ __forceinline__ void dct8(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7,
                                     int out[8], bool pass1) {
    int t0 = s0 + s7, t1 = s1 + s6, t2 = s2 + s5, t3 = s3 + s4;
    int t10 = t0 + t3, t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
    if (!pass1) t10 += 1 << (P1 - 1);
    t0 = s0 - s7; t1 = s1 - s6; t2 = s2 - s5; t3 = s3 - s4;
    const int sh = pass1 ? CB - P1 : CB + P1;
    if (pass1) {
        out[0] = (t10 + t11 - 8 * 128) << P1;
        out[4] = (t10 - t11) << P1;
    } else {
        out[0] = (t10 + t11) >> P1;
        out[4] = (t10 - t11) >> P1;
    }
    int z1 = (t12 + t13) * 4433;
    z1 += 1 << (sh - 1);
    out[2] = (z1 + t12 * 6270) >> sh;
    out[6] = (z1 - t13 * 15137) >> sh;
    t12 = t0 + t2; t13 = t1 + t3;
    z1 = (t12 + t13) * 9633;
    z1 += 1 << (sh - 1);
    t12 = t12 * (-3196); t13 = t13 * (-16069);
    t12 += z1; t13 += z1;
    z1 = (t0 + t3) * (-7373);
    t0 = t0 * 12299; t3 = t3 * 2446;
    t0 += z1 + t12; t3 += z1 + t13;
    z1 = (t1 + t2) * (-20995);
    t1 = t1 * 25172; t2 = t2 * 16819;
    t1 += z1 + t13; t2 += z1 + t12;
    out[1] = t0 >> sh; out[3] = t1 >> sh; out[5] = t2 >> sh; out[7] = t3 >> sh;
}

__global__ __launch_bounds__(192) void k_jpeg_coeffs(const uint8_t* __restrict__ src, int w, int h,
                                                     int C, size_t pitch, size_t img_stride,
                                                     const uint8_t* __restrict__ qt,
                                                     int16_t* __restrict__ coef,
                                                     size_t coef_img_stride, int nmcu,
                                                     const uint64_t* __restrict__ src_tab) {
    __shared__ int rows[24][8][9];
    const int t = threadIdx.x;
    const int blk = t >> 3, line = t & 7;
    const int m = blockIdx.x * 8 + blk / 3, comp = blk % 3;
    const int img = blockIdx.y;
    const int nbx = (w + 7) >> 3;
    const bool ok = m < nmcu;
    if (ok) {
        const int bx = m % nbx, by = m / nbx;
        int py = by * 8 + line;
        if (py >= h) py = h - 1;
        const uint8_t* base = src_tab ? reinterpret_cast<const uint8_t*>(src_tab[img]) : src + (size_t)img * img_stride;
        const uint8_t* row = base + (size_t)py * pitch;
        int smp[8];
        const float mx = 255.0f;
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            int px = bx * 8 + x;
            if (px >= w) px = w - 1;
            int ri, gi, bi;
            load_rgb(row, px, C, ri, gi, bi);
            const float r = (float)ri, g = (float)gi, b = (float)bi;
            float v;
            if (comp == 0) v = 76.245f / mx * r + 149.685f / mx * g + 29.07f / mx * b;
            else if (comp == 1) v = -43.0185f / mx * r - 84.4815f / mx * g + 127.5f / mx * b + 128.0f;
            else v = 127.5f / mx * r - 106.7685f / mx * g - 20.7315f / mx * b + 128.0f;
            smp[x] = f32_as_u8(v);
        }
        int o[8];
        dct8(smp[0], smp[1], smp[2], smp[3], smp[4], smp[5], smp[6], smp[7], o, true);
#pragma unroll
        for (int k = 0; k < 8; ++k) rows[blk][line][k] = o[k];
    }
    __syncthreads();
    if (!ok) return;
    const int x = line;  // column
    int o[8];
    dct8(rows[blk][0][x], rows[blk][1][x], rows[blk][2][x], rows[blk][3][x], rows[blk][4][x],
         rows[blk][5][x], rows[blk][6][x], rows[blk][7][x], o, false);
    const uint8_t* q = qt + (comp ? 64 : 0);
    int16_t* out = coef + (size_t)img * coef_img_stride + ((size_t)m * 3 + comp) * 64;
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        const int d = o[y];
        out[y * 8 + x] = (int16_t)(int)roundf((float)(d / 8) / (float)q[y * 8 + x]);
    }
}

hipError_t launch_jpeg_coeffs(const uint8_t* src, int w, int h, int C, size_t pitch,
                              size_t img_stride, const uint8_t* qtables, int16_t* coef,
                              size_t coef_img_stride, int n, hipStream_t s, const uint64_t* src_tab) {
    const int nmcu = ((w + 7) >> 3) * ((h + 7) >> 3);
    dim3 grid((nmcu + 7) / 8, n);
    hipLaunchKernelGGL(k_jpeg_coeffs, grid, dim3(192), 0, s, src, w, h, C, pitch, img_stride,
                       qtables, coef, coef_img_stride, nmcu, src_tab);
    return hipGetLastError();
}

}  // namespace ik
