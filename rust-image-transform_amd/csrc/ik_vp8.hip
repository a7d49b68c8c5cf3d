// ik_vp8.hip -- GPU VP8 key-frame macroblock encoder: the encode_image WebP
// branch (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp), with the
// macroblock analysis, rate-distortion mode search, transforms and quantisation
// on the MI355X instead of libwebp on host threads.
//
// VP8 intra coding is a dependency chain: a macroblock predicts from the
// reconstruction of its left, top-left, top and top-right neighbours.  All MBs
// with mb_x + 2*mb_y == t are independent, so a frame is coded as a wavefront of
// (mb_w - 1) + 2*(mb_h - 1) + 1 diagonals: one launch per diagonal, every image of
// the batch in the same launch (grid.y = image).  One wave64 owns one MB and runs
// the decision of ik_vp8.h's scalar encode_mb with its lanes:
//   i16  lane = (mode, 4x4 block): 4 x 16 = 64 lanes
//   i4   lane = mode (10 lanes), the 16 blocks in order (each predicts from the last)
//   uv   lane = (mode, channel, block): 4 x 2 x 4 = 32 lanes
// Rates and distortions are integer sums and ties keep the lowest mode, so the
// decisions -- and the bitstream -- are identical to the scalar encoder's
// (tests/test_gpu_vp8.py).  Per-lane trial levels live in LDS (the token-cost
// scan indexes them at run time).
#include <hip/hip_runtime.h>

#include "ik_vp8_gpu.h"

namespace ik {
namespace vp8 {

namespace {

__device__ __forceinline__ int i16_mode(int m) {  // trial order of encode_mb
    return m == 0 ? DC_PRED : (m == 1 ? V_PRED : (m == 2 ? H_PRED : TM_PRED));
}
__device__ __forceinline__ int sum16(int v) {  // over each aligned group of 16 lanes
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    return v;
}
__device__ __forceinline__ int sum8(int v) {
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    return v;
}
__device__ __forceinline__ int any_nz(const int16_t* lv, int first) {
    int nz = 0;
    for (int n = first; n < 16; ++n) nz |= lv[n] != 0;
    return nz;
}

}  // namespace

__global__ __launch_bounds__(64) void k_vp8_diag(Vp8Args a, int t) {
    const int lane = (int)threadIdx.x;
    const int img = (int)blockIdx.y;
    int y_lo = t - a.mb_w + 1;
    y_lo = y_lo > 0 ? (y_lo + 1) >> 1 : 0;
    const int my = y_lo + (int)blockIdx.x, mx = t - 2 * my;
    if (my >= a.mb_h || mx < 0) return;  // uniform over the wave
    const int mb_w = a.mb_w;
    const int mbi = my * mb_w + mx;
    const QParams& q = a.q;
    const uint8_t* probs = kCoeffProbs0;

    __shared__ uint8_t s_src_y[256], s_src_u[64], s_src_v[64];
    __shared__ uint8_t s_y[17 * kBps], s_u[9 * kBps], s_v[9 * kBps], s_y4[17 * kBps];
    __shared__ uint8_t s_rec16[4][256];
    __shared__ uint8_t s_recuv[4][2][64];
    __shared__ int16_t s_lv[64][16];   // per-lane trial levels (zigzag order)
    __shared__ int16_t s_out[25][16];  // the chosen levels (MBOut.lv layout)
    __shared__ int16_t s_lv4[16][16];  // i4 levels, block by block
    __shared__ int16_t s_y2[4][16], s_dc[4][16], s_dcq[4][16];
    __shared__ long long s_j[64];
    __shared__ int s_last[16], s_rate_y2[4];
    __shared__ uint8_t s_nzb[64], s_bm4[16];
    __shared__ uint8_t s_ctx[26];  // top_nz[9], left_nz[9], top_bmodes[4], left_bmodes[4]

    // ---- source pixels (edge-replicated) and neighbour contexts ----
    const uint8_t* Y = a.yuv + (size_t)img * a.yuv_stride;
    const int uvw = (a.w + 1) >> 1, uvh = (a.h + 1) >> 1;
    const uint8_t* U = Y + (size_t)a.w * a.h;
    const uint8_t* V = U + (size_t)uvw * uvh;
    for (int i = lane; i < 256; i += 64) {
        const int sx = min(mx * 16 + (i & 15), a.w - 1), sy = min(my * 16 + (i >> 4), a.h - 1);
        s_src_y[i] = Y[(size_t)sy * a.w + sx];
    }
    {
        const int sx = min(mx * 8 + (lane & 7), uvw - 1), sy = min(my * 8 + (lane >> 3), uvh - 1);
        s_src_u[lane] = U[(size_t)sy * uvw + sx];
        s_src_v[lane] = V[(size_t)sy * uvw + sx];
    }
    const int rw = mb_w * 16, cw = mb_w * 8;
    uint8_t* RY = a.rec + (size_t)img * a.rec_stride;
    uint8_t* RU = RY + (size_t)rw * a.mb_h * 16;
    uint8_t* RV = RU + (size_t)cw * a.mb_h * 8;
    MBOut* mbs = a.mbs + (size_t)img * mb_w * a.mb_h;
    uint8_t* nzs = a.nz + (size_t)img * mb_w * a.mb_h * 18;
    for (int i = lane; i < 17 * kBps; i += 64) s_y[i] = 0;
    for (int i = lane; i < 9 * kBps; i += 64) { s_u[i] = 0; s_v[i] = 0; }
    __syncthreads();
    // context row / column (libwebp's frame-edge 127 / 129 fills and top-right rule)
    auto fill = [&](uint8_t* buf, const uint8_t* rec, int stride, int n, int extra) {
        const int x0 = mx * n, y0 = my * n;
        for (int x = lane - 1; x < n + extra; x += 64) {
            int v;
            if (my == 0) v = 127;
            else if (x < 0) v = mx == 0 ? 129 : rec[(size_t)(y0 - 1) * stride + x0 - 1];
            else if (x < n) v = rec[(size_t)(y0 - 1) * stride + x0 + x];
            else v = mx == mb_w - 1 ? rec[(size_t)(y0 - 1) * stride + x0 + n - 1]
                                    : rec[(size_t)(y0 - 1) * stride + x0 + x];
            buf[x + 1] = (uint8_t)v;
        }
        for (int y = lane; y < n; y += 64)
            buf[(y + 1) * kBps] = mx == 0 ? 129 : rec[(size_t)(y0 + y) * stride + x0 - 1];
    };
    fill(s_y, RY, rw, 16, 4);
    fill(s_u, RU, cw, 8, 0);
    fill(s_v, RV, cw, 8, 0);
    if (lane < 9) {
        s_ctx[lane] = my ? nzs[(size_t)(mbi - mb_w) * 18 + lane] : 0;       // above MB's outgoing top
        s_ctx[9 + lane] = mx ? nzs[(size_t)(mbi - 1) * 18 + 9 + lane] : 0;  // left MB's outgoing left
    } else if (lane < 13) {
        const int i = lane - 9;
        s_ctx[18 + i] = my ? mbs[mbi - mb_w].bmodes[12 + i] : (uint8_t)B_DC;
        s_ctx[22 + i] = mx ? mbs[mbi - 1].bmodes[i * 4 + 3] : (uint8_t)B_DC;
    }
    __syncthreads();
    if (lane < 12) {  // 4x4 top-right of block rows 1..3 = the MB's own top-right samples
        const int r = 1 + (lane >> 2), i = lane & 3;
        s_y[(4 * r) * kBps + 17 + i] = s_y[17 + i];
    }
    __syncthreads();
    for (int i = lane; i < 17 * kBps; i += 64) s_y4[i] = s_y[i];
    const uint8_t* top_nz = s_ctx;
    const uint8_t* left_nz = s_ctx + 9;
    const uint8_t* top_bm = s_ctx + 18;
    const uint8_t* left_bm = s_ctx + 22;

    // ---- luma 16x16 (try_i16): lane = (mode, block) ----
    int best_mode;
    long long best;
    int bm16;
    {
        const int m = lane >> 4, b = lane & 15, bx = b & 3, by = b >> 2;
        const int mode = i16_mode(m);
        uint8_t pr[16];
        pred_blk(mode, 16, s_y + kBps + 1, mx, my, bx, by, pr);
        int16_t coef[16];
        const uint8_t* src = s_src_y + by * 4 * 16 + bx * 4;
        fdct4(src, 16, pr, 4, coef);
        s_dc[m][b] = coef[0];
        __syncthreads();
        if (b == 0) {
            int16_t y2[16];
            fwht(s_dc[m], y2);
            const int l2 = quantize(y2, s_y2[m], q.y2, 0);
            s_rate_y2[m] = block_cost(s_y2[m], 0, l2, top_nz[8] + left_nz[8], 1, probs);
            iwht(y2, s_dcq[m]);
        }
        int16_t* lv = s_lv[lane];
        const int last = quantize(coef, lv, q.y1, 1);
        s_nzb[lane] = last > 1;
        __syncthreads();
        const int tctx = by ? s_nzb[lane - 4] : top_nz[bx];
        const int lctx = bx ? s_nzb[lane - 1] : left_nz[by];
        int rate = block_cost(lv, 1, last, tctx + lctx, 0, probs);
        coef[0] = s_dcq[m][b];
        uint8_t* rec = s_rec16[m] + by * 4 * 16 + bx * 4;
        idct4_add(coef, pr, 4, rec, 16);
        int dist = sse(src, 16, rec, 16, 4, 4);
        rate = sum16(rate);
        dist = sum16(dist);
        if (b == 0) s_j[m] = 256ll * dist + (long long)q.lambda * (rate + ymode_cost(mode) + s_rate_y2[m]);
        __syncthreads();
        bm16 = 0;
        best = s_j[0];
        for (int k = 1; k < 4; ++k)
            if (s_j[k] < best) { best = s_j[k]; bm16 = k; }
        best_mode = i16_mode(bm16);
        // keep the winner's levels: the i4 search reuses s_lv
        for (int i = lane; i < 256; i += 64) s_out[i >> 4][i & 15] = s_lv[bm16 * 16 + (i >> 4)][i & 15];
        if (lane < 16) s_out[24][lane] = s_y2[bm16][lane];
        __syncthreads();
    }

    // ---- luma 4x4 (B_PRED): the 16 blocks in order, lane = mode ----
    {
        long long total = (long long)q.lambda * ymode_cost(B_PRED);
        int tnz[4] = {top_nz[0], top_nz[1], top_nz[2], top_nz[3]};
        int lnz[4] = {left_nz[0], left_nz[1], left_nz[2], left_nz[3]};
        bool ok = true;
        for (int b = 0; b < 16; ++b) {
            const int bx = b & 3, by = b >> 2;
            uint8_t* d = s_y4 + (by * 4 + 1) * kBps + bx * 4 + 1;
            const uint8_t* src = s_src_y + by * 4 * 16 + bx * 4;
            const int top = by ? s_bm4[b - 4] : top_bm[bx];
            const int left = bx ? s_bm4[b - 1] : left_bm[by];
            uint8_t r4[16];
            if (lane < NUM_BMODES) {
                uint8_t pr[16];
                int16_t coef[16];
                pred4(lane, d, pr);
                fdct4(src, 16, pr, 4, coef);
                const int last = quantize(coef, s_lv[lane], q.y1, 0);
                idct4_add(coef, pr, 4, r4, 4);
                const int rate = bmode_cost(lane, top, left) +
                                 block_cost(s_lv[lane], 0, last, tnz[bx] + lnz[by], 3, probs);
                s_j[lane] = 256ll * sse(src, 16, r4, 4, 4, 4) + (long long)q.lambda * rate;
                s_last[lane] = last;
            }
            __syncthreads();
            int bmode = 0;
            long long bj = s_j[0];
            for (int k = 1; k < NUM_BMODES; ++k)
                if (s_j[k] < bj) { bj = s_j[k]; bmode = k; }
            if (lane == bmode)
                for (int y = 0; y < 4; ++y)
                    for (int x = 0; x < 4; ++x) d[y * kBps + x] = r4[y * 4 + x];
            if (lane < 16) s_lv4[b][lane] = s_lv[bmode][lane];
            if (lane == 0) s_bm4[b] = (uint8_t)bmode;
            total += bj;
            tnz[bx] = lnz[by] = s_last[bmode] > 0;
            __syncthreads();
            if (total >= best) { ok = false; break; }  // 16x16 already better (uniform)
        }
        if (ok && total < best) {
            best_mode = B_PRED;
            for (int i = lane; i < 256; i += 64) s_out[i >> 4][i & 15] = s_lv4[i >> 4][i & 15];
            if (lane < 16) s_out[24][lane] = 0;
        }
    }
    __syncthreads();

    // ---- chroma (try_uv): lane = (mode, channel, block) ----
    int bmuv;
    {
        const bool act = lane < 32;
        const int m = (lane >> 3) & 3, ch = (lane >> 2) & 1, b = lane & 3, bx = b & 1, by = b >> 1;
        const int mode = i16_mode(m);
        const uint8_t* src = (ch ? s_src_v : s_src_u) + by * 4 * 8 + bx * 4;
        uint8_t pr[16];
        int16_t coef[16];
        int last = 0;
        if (act) {
            pred_blk(mode, 8, (ch ? s_v : s_u) + kBps + 1, mx, my, bx, by, pr);
            fdct4(src, 8, pr, 4, coef);
            last = quantize(coef, s_lv[lane], q.uv, 0);
            s_nzb[lane] = last > 0;
        }
        __syncthreads();
        int rate = 0, dist = 0;
        if (act) {
            const int tctx = by ? s_nzb[lane - 2] : top_nz[4 + 2 * ch + bx];
            const int lctx = bx ? s_nzb[lane - 1] : left_nz[4 + 2 * ch + by];
            rate = block_cost(s_lv[lane], 0, last, tctx + lctx, 2, probs);
            uint8_t* rec = s_recuv[m][ch] + by * 4 * 8 + bx * 4;
            idct4_add(coef, pr, 4, rec, 8);
            dist = sse(src, 8, rec, 8, 4, 4);
        }
        rate = sum8(rate);
        dist = sum8(dist);
        if (act && (lane & 7) == 0) s_j[m] = 256ll * dist + (long long)q.lambda * (rate + uvmode_cost(mode));
        __syncthreads();
        bmuv = 0;
        long long bj = s_j[0];
        for (int k = 1; k < 4; ++k)
            if (s_j[k] < bj) { bj = s_j[k]; bmuv = k; }
        for (int i = lane; i < 128; i += 64) s_out[16 + (i >> 4)][i & 15] = s_lv[bmuv * 8 + (i >> 4)][i & 15];
    }
    __syncthreads();

    // ---- outputs: MBOut, reconstruction, outgoing non-zero contexts ----
    int nzv = 0;
    for (int i = lane; i < 25 * 16; i += 64) nzv |= (&s_out[0][0])[i] != 0;
    const bool skip = __ballot(nzv) == 0ull;
    MBOut& o = mbs[mbi];
    if (lane == 0) {
        o.ymode = (uint8_t)best_mode;
        o.uvmode = (uint8_t)i16_mode(bmuv);
        o.skip = skip ? 1 : 0;
        o.pad = 0;
    }
    if (lane < 16) o.bmodes[lane] = best_mode == B_PRED ? s_bm4[lane] : (uint8_t)best_mode;
    {
        uint32_t* dst = reinterpret_cast<uint32_t*>(&o.lv[0][0]);
        const uint32_t* sv = reinterpret_cast<const uint32_t*>(&s_out[0][0]);
        for (int i = lane; i < 200; i += 64) dst[i] = sv[i];
    }
    const uint8_t* ybest = best_mode == B_PRED ? nullptr : s_rec16[bm16];
    for (int i = lane; i < 256; i += 64) {
        const int y = i >> 4, x = i & 15;
        RY[(size_t)(my * 16 + y) * rw + mx * 16 + x] = ybest ? ybest[i] : s_y4[(y + 1) * kBps + x + 1];
    }
    RU[(size_t)(my * 8 + (lane >> 3)) * cw + mx * 8 + (lane & 7)] = s_recuv[bmuv][0][lane];
    RV[(size_t)(my * 8 + (lane >> 3)) * cw + mx * 8 + (lane & 7)] = s_recuv[bmuv][1][lane];
    if (lane < 18) {
        const int first = best_mode == B_PRED ? 0 : 1;
        const int k = lane < 9 ? lane : lane - 9;
        const bool top = lane < 9;
        int v;
        if (k < 4) v = any_nz(s_out[top ? 12 + k : k * 4 + 3], first);
        else if (k < 8) {
            const int ch = (k - 4) >> 1, i = (k - 4) & 1;
            v = any_nz(s_out[16 + 4 * ch + (top ? 2 + i : i * 2 + 1)], 0);
        } else {
            v = best_mode == B_PRED ? (top ? top_nz[8] : left_nz[8]) : any_nz(s_out[24], 0);
        }
        nzs[(size_t)mbi * 18 + lane] = (uint8_t)v;
    }
}

hipError_t launch_vp8_encode(const Vp8Args& a, int n, hipStream_t s) {
    const int per_diag = a.mb_h < (a.mb_w + 1) / 2 ? a.mb_h : (a.mb_w + 1) / 2;
    const int T = (a.mb_w - 1) + 2 * (a.mb_h - 1) + 1;
    for (int t = 0; t < T; ++t) hipLaunchKernelGGL(k_vp8_diag, dim3(per_diag, n), dim3(64), 0, s, a, t);
    return hipGetLastError();
}

}  // namespace vp8
}  // namespace ik
