// ik_vp8.hip -- GPU VP8 key-frame macroblock encoder: the encode_image WebP
// branch (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp), with the
// rate-distortion mode search, transforms and quantisation on the MI355X
// instead of libwebp on host threads.
//
// VP8 intra coding is a dependency chain: a macroblock predicts from the
// reconstruction of its left, top-left, top and top-right neighbours.  All MBs
// with mb_x + 2*mb_y == t are independent, so a frame is coded as a wavefront of
// (mb_w - 1) + 2*(mb_h - 1) + 1 diagonals: one launch per diagonal, every image of
// the batch in the same launch (grid.y = image).  A workgroup of two wave64s owns
// one MB and runs the decision of ik_vp8.h's scalar encode_mb:
//   phase A  wave 0: i16, lane = (mode, 4x4 block), 4 x 16 lanes
//            wave 1: chroma, lane = (mode, channel, block), 4 x 2 x 4 lanes
//   phase B  i4 (B_PRED): the 16 blocks in 10 wavefront steps (bx + 2*by), a step's
//            one or two blocks on the two waves; per block lane = (mode, row),
//            10 x 4 lanes: row r of mode m is predicted through a tap table (no
//            divergence across modes), transformed, its column quantised and
//            inverse-transformed, the transposes going through LDS
// Rates and distortions are integer sums and ties keep the lowest mode, so the
// decisions -- and the bitstream -- are identical to the scalar encoder's
// (tests/test_gpu_vp8.py).  Levels stay in registers; token rates come from
// compile-time probabilities (block_cost_fixed) or LDS cost rows (i4).
#include <hip/hip_runtime.h>

#include "ik_vp8_gpu.h"

namespace ik {
namespace vp8 {

namespace {

constexpr int kThreadsMB = 128;

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
// i4 wavefront: step t holds the blocks with bx + 2*by == t (their left, top,
// top-left and top-right neighbours are all in earlier steps); -1 = empty slot.
// Slot 0: bx in {2, 3} (or the first / last two blocks), slot 1: bx in {0, 1}.
__device__ __forceinline__ int i4_block(int t, int slot) {
    if (slot == 0) {
        if (t < 2) return t;
        if (t > 7) return t + 6;  // 14, 15
        const int bx = 2 + (t & 1);
        return ((t - bx) >> 1) * 4 + bx;
    }
    if (t < 2 || t > 7) return -1;
    const int bx = t & 1;
    return ((t - bx) >> 1) * 4 + bx;
}

}  // namespace

__global__ __launch_bounds__(kThreadsMB) void k_vp8_diag(Vp8Args a, int t) {
    const int tid = (int)threadIdx.x;
    // wave index in an SGPR: the phase-A branch (which holds barriers) and the i4
    // slot selection compile to scalar branches, so each wave runs exactly one side
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int img = (int)blockIdx.y;
    int y_lo = t - a.mb_w + 1;
    y_lo = y_lo > 0 ? (y_lo + 1) >> 1 : 0;
    const int my = y_lo + (int)blockIdx.x, mx = t - 2 * my;
    if (my >= a.mb_h || mx < 0) return;  // uniform over the workgroup
    const int mb_w = a.mb_w;
    const int mbi = my * mb_w + mx;
    const QParams& q = a.q;
    unsigned long long* stamp = (a.stamps && img == 0 && blockIdx.x == 0 && tid == 0) ? a.stamps + 8 * t : nullptr;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();

    __shared__ __attribute__((aligned(16))) uint8_t s_src_y[256];
    __shared__ __attribute__((aligned(16))) uint8_t s_src_u[64], s_src_v[64];
    __shared__ __attribute__((aligned(16))) uint8_t s_y[17 * kBps], s_y4[17 * kBps], s_u[9 * kBps], s_v[9 * kBps];
    __shared__ __attribute__((aligned(16))) uint8_t s_rec16[4][256];
    __shared__ __attribute__((aligned(16))) uint8_t s_recuv[4][2][64];
    __shared__ __attribute__((aligned(16))) int16_t s_lv16[64][16];  // i16 trial levels, lane = (mode, block)
    __shared__ __attribute__((aligned(16))) int16_t s_lvuv[32][16];  // chroma trial levels
    __shared__ __attribute__((aligned(16))) int16_t s_lvt[2][NUM_BMODES][16];  // i4 trial levels, per wave
    __shared__ __attribute__((aligned(16))) int16_t s_out[25][16];   // the chosen levels (MBOut.lv layout)
    __shared__ __attribute__((aligned(16))) int16_t s_lv4[16][16];   // i4 levels as chosen, per block
    __shared__ int16_t s_y2[4][16], s_dc[4][16], s_dcq[4][16];
    __shared__ long long s_j16[4], s_juv[4], s_jt[2][NUM_BMODES], s_bj[16];
    __shared__ int s_lastt[2][NUM_BMODES], s_rate_y2[4];
    __shared__ int s_tr[2][64][4];  // i4 transposes, per wave
    __shared__ __attribute__((aligned(16))) uint16_t s_tok[8][3][24];                          // kTokCostI4
    __shared__ __attribute__((aligned(16))) uint16_t s_bmc[NUM_BMODES][NUM_BMODES][NUM_BMODES];  // kBModeCost
    __shared__ uint8_t s_nzb16[64], s_nzbuv[32], s_bm4[16], s_bnz[16];
    __shared__ uint8_t s_ctx[26];  // top_nz[9], left_nz[9], top_bmodes[4], left_bmodes[4]

    // ---- load: every global read of the MB formed first and issued at once ----
    const uint8_t* Y = a.yuv + (size_t)img * a.yuv_stride;
    const int uvw = (a.w + 1) >> 1, uvh = (a.h + 1) >> 1;
    const uint8_t* U = Y + (size_t)a.w * a.h;
    const uint8_t* V = U + (size_t)uvw * uvh;
    const int rw = mb_w * 16, cw = mb_w * 8;
    uint8_t* RY = a.rec + (size_t)img * a.rec_stride;
    uint8_t* RU = RY + (size_t)rw * a.mb_h * 16;
    uint8_t* RV = RU + (size_t)cw * a.mb_h * 8;
    MBOut* mbs = a.mbs + (size_t)img * mb_w * a.mb_h;
    uint8_t* nzs = a.nz + (size_t)img * mb_w * a.mb_h * 18;
    {
        const uint32_t* g = reinterpret_cast<const uint32_t*>(&kTokCostI4);
        uint32_t* l = reinterpret_cast<uint32_t*>(&s_tok[0][0][0]);
        for (int i = tid; i < (int)(sizeof(s_tok) / 4); i += kThreadsMB) l[i] = g[i];
        const uint32_t* g2 = reinterpret_cast<const uint32_t*>(&kBModeCost);
        uint32_t* l2 = reinterpret_cast<uint32_t*>(&s_bmc[0][0][0]);
        for (int i = tid; i < (int)(sizeof(s_bmc) / 4); i += kThreadsMB) l2[i] = g2[i];
    }
    for (int i = tid; i < 256; i += kThreadsMB) {
        const int sx = min(mx * 16 + (i & 15), a.w - 1), sy = min(my * 16 + (i >> 4), a.h - 1);
        s_src_y[i] = Y[(size_t)sy * a.w + sx];
    }
    {
        const int cx = min(mx * 8 + (lane & 7), uvw - 1), cy = min(my * 8 + (lane >> 3), uvh - 1);
        (wv == 0 ? s_src_u : s_src_v)[lane] = (wv == 0 ? U : V)[(size_t)cy * uvw + cx];
    }
    // Work buffers: context row 0 (top-left, top, top-right) and column 0 (left)
    // with libwebp's frame-edge 127 / 129 fills, the 4x4 top-right copies of the
    // MB's top-right samples in block rows 1..3, zero elsewhere.  Each byte is a
    // constant or one reconstructed sample: addresses first, then every load
    // unconditionally (one memory round trip), then the selects.
    auto ctx_src = [&](const uint8_t* rec, int stride, int n, int extra, int row, int col, int& cval) -> const uint8_t* {
        const int x0 = mx * n, y0 = my * n;
        cval = 0;
        if (row == 0 || (n == 16 && (row == 4 || row == 8 || row == 12) && col >= 17 && col <= 20)) {
            const int x = col - 1;
            if (x >= n + extra) return nullptr;
            if (my == 0) { cval = 127; return nullptr; }
            if (x < 0) {
                if (mx == 0) { cval = 129; return nullptr; }
                return rec + (size_t)(y0 - 1) * stride + x0 - 1;
            }
            return rec + (size_t)(y0 - 1) * stride + x0 + (x >= n && mx == mb_w - 1 ? n - 1 : x);
        }
        if (col == 0 && row >= 1 && row <= n) {
            if (mx == 0) { cval = 129; return nullptr; }
            return rec + (size_t)(y0 + row - 1) * stride + x0 - 1;
        }
        return nullptr;
    };
    auto ctx_word = [&](const uint8_t* rec, int stride, int n, int extra, int row, int col) -> uint32_t {
        const uint8_t* p[4];
        int cv[4], v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = ctx_src(rec, stride, n, extra, row, col + k, cv[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *(p[k] ? p[k] : rec);  // rec: a valid dummy address
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) w |= (uint32_t)(p[k] ? v[k] : cv[k]) << (8 * k);
        return w;
    };
    // 136 luma words + 144 chroma words over the 128 threads, loads of all rounds
    // issued before any select (the loop is unrolled)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int wd = tid + k * kThreadsMB;
        if (wd < 17 * kBps / 4) {
            const int row = (wd * 4) / kBps, col = (wd * 4) % kBps;
            const uint32_t w = ctx_word(RY, rw, 16, 4, row, col);
            reinterpret_cast<uint32_t*>(s_y)[wd] = w;
            reinterpret_cast<uint32_t*>(s_y4)[wd] = w;
        } else if (wd < 17 * kBps / 4 + 2 * 9 * kBps / 4) {
            const int w1 = wd - 17 * kBps / 4;
            const int ch = w1 >= 9 * kBps / 4, w2 = w1 - ch * (9 * kBps / 4);
            const int row = (w2 * 4) / kBps, col = (w2 * 4) % kBps;
            reinterpret_cast<uint32_t*>(ch ? s_v : s_u)[w2] = ctx_word(ch ? RV : RU, cw, 8, 0, row, col);
        }
    }
    if (tid < 9) {
        s_ctx[tid] = my ? nzs[(size_t)(mbi - mb_w) * 18 + tid] : 0;       // above MB's outgoing top
        s_ctx[9 + tid] = mx ? nzs[(size_t)(mbi - 1) * 18 + 9 + tid] : 0;  // left MB's outgoing left
    } else if (tid < 13) {
        const int i = tid - 9;
        s_ctx[18 + i] = my ? mbs[mbi - mb_w].bmodes[12 + i] : (uint8_t)B_DC;
        s_ctx[22 + i] = mx ? mbs[mbi - 1].bmodes[i * 4 + 3] : (uint8_t)B_DC;
    }
    __syncthreads();
    const uint8_t* top_nz = s_ctx;
    const uint8_t* left_nz = s_ctx + 9;
    const uint8_t* top_bm = s_ctx + 18;
    const uint8_t* left_bm = s_ctx + 22;
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();

    // ---- phase A: wave 0 = luma 16x16 (try_i16), wave 1 = chroma (try_uv) ----
    {
        const bool luma = wv == 0;  // wave 0: (mode, block); wave 1 lanes < 32: (mode, channel, block)
        const bool act = luma || lane < 32;
        const int m = luma ? lane >> 4 : (lane >> 3) & 3;
        const int ch = (lane >> 2) & 1;
        const int b = luma ? lane & 15 : lane & 3;
        const int bx = luma ? b & 3 : b & 1, by = luma ? b >> 2 : b >> 1;
        const int mode = i16_mode(m);
        const uint8_t* src = luma ? s_src_y + by * 4 * 16 + bx * 4 : (ch ? s_src_v : s_src_u) + by * 4 * 8 + bx * 4;
        uint8_t pr[16];
        int16_t coef[16], lv[16];
        int last = 0;
        if (luma) {
            pred_blk(mode, 16, s_y + kBps + 1, mx, my, bx, by, pr);
            fdct4(src, 16, pr, 4, coef);
            s_dc[m][b] = coef[0];
        } else if (act) {
            pred_blk(mode, 8, (ch ? s_v : s_u) + kBps + 1, mx, my, bx, by, pr);
            fdct4(src, 8, pr, 4, coef);
            last = quantize(coef, lv, q.uv, 0);
            for (int i = 0; i < 16; ++i) s_lvuv[lane][i] = lv[i];
            s_nzbuv[lane] = last > 0;
        }
        __syncthreads();  // A1
        if (luma) {
            if (b == 0) {
                int16_t y2[16], l2v[16];
                fwht(s_dc[m], y2);
                const int l2 = quantize(y2, l2v, q.y2, 0);
                for (int i = 0; i < 16; ++i) s_y2[m][i] = l2v[i];
                s_rate_y2[m] = block_cost_fixed<1, 0>(l2v, l2, top_nz[8] + left_nz[8]);
                iwht(y2, s_dcq[m]);
            }
            last = quantize(coef, lv, q.y1, 1);
            for (int i = 0; i < 16; ++i) s_lv16[lane][i] = lv[i];
            s_nzb16[lane] = last > 1;
        } else {
            int rate = 0, dist = 0;
            if (act) {
                const int tctx = by ? s_nzbuv[lane - 2] : top_nz[4 + 2 * ch + bx];
                const int lctx = bx ? s_nzbuv[lane - 1] : left_nz[4 + 2 * ch + by];
                rate = block_cost_fixed<2, 0>(lv, last, tctx + lctx);
                uint8_t* rec = s_recuv[m][ch] + by * 4 * 8 + bx * 4;
                idct4_add(coef, pr, 4, rec, 8);
                dist = sse(src, 8, rec, 8, 4, 4);
            }
            rate = sum8(rate);
            dist = sum8(dist);
            if (act && (lane & 7) == 0) s_juv[m] = 256ll * dist + (long long)q.lambda * (rate + uvmode_cost(mode));
        }
        __syncthreads();  // A2
        if (luma) {
            const int tctx = by ? s_nzb16[lane - 4] : top_nz[bx];
            const int lctx = bx ? s_nzb16[lane - 1] : left_nz[by];
            int rate = block_cost_fixed<0, 1>(lv, last, tctx + lctx);
            coef[0] = s_dcq[m][b];
            uint8_t* rec = s_rec16[m] + by * 4 * 16 + bx * 4;
            idct4_add(coef, pr, 4, rec, 16);
            int dist = sse(src, 16, rec, 16, 4, 4);
            rate = sum16(rate);
            dist = sum16(dist);
            if (b == 0) s_j16[m] = 256ll * dist + (long long)q.lambda * (rate + ymode_cost(mode) + s_rate_y2[m]);
        }
        __syncthreads();  // A3
    }
    int bm16 = 0, bmuv = 0;
    long long best = s_j16[0];
    for (int k = 1; k < 4; ++k)
        if (s_j16[k] < best) { best = s_j16[k]; bm16 = k; }
    {
        long long bj = s_juv[0];
        for (int k = 1; k < 4; ++k)
            if (s_juv[k] < bj) { bj = s_juv[k]; bmuv = k; }
    }
    int best_mode = i16_mode(bm16);
    if (wv == 0) {
        for (int i = lane; i < 256; i += 64) s_out[i >> 4][i & 15] = s_lv16[bm16 * 16 + (i >> 4)][i & 15];
        if (lane < 16) s_out[24][lane] = s_y2[bm16][lane];
    } else {
        for (int i = lane; i < 128; i += 64) s_out[16 + (i >> 4)][i & 15] = s_lvuv[bmuv * 8 + (i >> 4)][i & 15];
    }
    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();

    // ---- phase B: luma 4x4 (B_PRED), 10 wavefront steps, one block per wave ----
    {
        const int m = lane < 4 * NUM_BMODES ? lane >> 2 : 0, r = lane & 3, quad = lane & ~3;
        long long total = (long long)q.lambda * ymode_cost(B_PRED);
        bool ok = true;
        // per-lane constants: zigzag index + quantiser of column r's coefficients,
        // bands of zigzag positions 4r..4r+3, tap descriptors of row r of mode m
        int desc[4], zn[4], qiq[4], qbias[4], qq[4], bnd[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            desc[x] = kPred4Tab[m][r * 4 + x];
            zn[x] = izigzag(r + 4 * x);
            const int k = zn[x] > 0;
            qiq[x] = q.y1.iq[k];
            qbias[x] = q.y1.bias[k];
            qq[x] = q.y1.q[k];
            bnd[x] = band(4 * r + x);
        }
        int (*tr)[4] = s_tr[wv];
        for (int st = 0; st < 10; ++st) {
            const int b = i4_block(st, wv);
            const bool blk = b >= 0;  // uniform over the wave
            const bool act = blk && lane < 4 * NUM_BMODES;
            const int bx = b & 3, by = b >> 2;
            uint8_t* d = s_y4 + (by * 4 + 1) * kBps + bx * 4 + 1;
            int pr[4], sv[4], cf[4], last = 0;
            int top = 0, left = 0, ctx0 = 0;
            if (blk) {
                const uint8_t* src = s_src_y + (by * 4 + r) * 16 + bx * 4;  // row r of the block
                top = by ? s_bm4[b - 4] : top_bm[bx];
                left = bx ? s_bm4[b - 1] : left_bm[by];
                ctx0 = (by ? s_bnz[b - 4] : top_nz[bx]) + (bx ? s_bnz[b - 1] : left_nz[by]);
                const int dcv = pred4_dc(d);
#pragma unroll
                for (int x = 0; x < 4; ++x) {  // pred4_px without the switch
                    const int tt = desc[x];
                    const int pa = d[p4_off((tt >> 8) & 15)], pb = d[p4_off((tt >> 4) & 15)], pc = d[p4_off(tt & 15)];
                    const int kind = tt >> 12;
                    pr[x] = kind == P4_CP ? pa : kind == P4_A2 ? avg2(pa, pb) : kind == P4_A3 ? avg3(pa, pb, pc)
                          : kind == P4_TM ? clip8(pa + pb - pc) : dcv;
                    sv[x] = src[x];
                }
                // fdct4 row pass (row r)
                const int d0 = sv[0] - pr[0], d1 = sv[1] - pr[1], d2 = sv[2] - pr[2], d3 = sv[3] - pr[3];
                const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
                tr[lane][0] = (a0 + a1) * 8;
                tr[lane][1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
                tr[lane][2] = (a0 - a1) * 8;
                tr[lane][3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
            }
            __syncthreads();  // B1
            if (blk) {
                // fdct4 column pass (column r: raster r, 4+r, 8+r, 12+r), quantise
                const int T0 = tr[quad][r], T1 = tr[quad + 1][r], T2 = tr[quad + 2][r], T3 = tr[quad + 3][r];
                const int a0 = T0 + T3, a1 = T1 + T2, a2 = T1 - T2, a3 = T0 - T3;
                cf[0] = (int16_t)((a0 + a1 + 7) >> 4);
                cf[1] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
                cf[2] = (int16_t)((a0 - a1 + 7) >> 4);
                cf[3] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int n = zn[i];
                    const int c = cf[i], sgn = c < 0, av = sgn ? -c : c;
                    int l = (int)(((unsigned)av * (unsigned)qiq[i] + (unsigned)qbias[i]) >> 17);
                    if (l > 2047) l = 2047;
                    if (act) s_lvt[wv][m][n] = (int16_t)(sgn ? -l : l);
                    cf[i] = (int16_t)((sgn ? -l : l) * qq[i]);  // dequantised
                    if (l && n + 1 > last) last = n + 1;
                }
                last = max(last, __shfl_xor(last, 1));
                last = max(last, __shfl_xor(last, 2));
            }
            __syncthreads();  // B2
            int rate = 0;
            if (blk) {
                int16_t lv[16];
                {
                    const uint4 w0 = *reinterpret_cast<const uint4*>(&s_lvt[wv][m][0]);
                    const uint4 w1 = *reinterpret_cast<const uint4*>(&s_lvt[wv][m][8]);
                    const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                    for (int i = 0; i < 8; ++i) { lv[2 * i] = (int16_t)(w[i] & 0xffff); lv[2 * i + 1] = (int16_t)(w[i] >> 16); }
                }
                // token rate (== block_cost(lv, 0, last, ctx0, 3)): lane r prices zigzag
                // positions 4r..4r+3 from the LDS cost rows, the quad sums
                int prev = r == 0 ? 0 : (r == 1 ? lv[3] : (r == 2 ? lv[7] : lv[11]));
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int n = 4 * r + k;
                    const int cur = r == 0 ? lv[k] : (r == 1 ? lv[4 + k] : (r == 2 ? lv[8 + k] : lv[12 + k]));
                    const int pv = prev < 0 ? -prev : prev, v = cur < 0 ? -cur : cur;
                    const int ctx = n == 0 ? ctx0 : (pv == 0 ? 0 : (pv == 1 ? 1 : 2));
                    const bool chk = n == 0 || pv != 0;
                    const uint16_t* row = s_tok[bnd[k]][ctx];
                    const uint4 rr = *reinterpret_cast<const uint4*>(row);
                    const int c1p0 = rr.x & 0xffff, c0p0 = rr.x >> 16, c0p1 = rr.y & 0xffff, c1p1 = rr.y >> 16;
                    const int c0p2 = rr.z & 0xffff, c1p2 = rr.z >> 16;
                    int c = 0;
                    if (n < last) {
                        c = chk ? c1p0 : 0;
                        if (v == 0) c += c0p1;
                        else if (v == 1) c += c1p1 + c0p2;
                        else c += c1p1 + c1p2 + large_cost_row(v, row + 8);
                    } else if (n == last) {
                        c = c0p0;
                    }
                    rate += c;
                    prev = cur;
                }
                rate += __shfl_xor(rate, 1);
                rate += __shfl_xor(rate, 2);
                rate += s_bmc[top][left][m];
                // inverse transform, vertical pass on column r
                const int aa = cf[0] + cf[2], bb = cf[0] - cf[2];
                const int c = mul2(cf[1]) - mul1(cf[3]), dd = mul1(cf[1]) + mul2(cf[3]);
                tr[lane][0] = aa + dd;
                tr[lane][1] = bb + c;
                tr[lane][2] = bb - c;
                tr[lane][3] = aa - dd;
            }
            __syncthreads();  // B3
            int rec[4] = {0, 0, 0, 0};
            if (blk) {
                // horizontal pass for row r, reconstruction, distortion
                const int T0 = tr[quad][r], T1 = tr[quad + 1][r], T2 = tr[quad + 2][r], T3 = tr[quad + 3][r];
                const int dc = T0 + 4;
                const int aa = dc + T2, bb = dc - T2;
                const int c = mul2(T1) - mul1(T3), dd = mul1(T1) + mul2(T3);
                rec[0] = clip8(pr[0] + ((aa + dd) >> 3));
                rec[1] = clip8(pr[1] + ((bb + c) >> 3));
                rec[2] = clip8(pr[2] + ((bb - c) >> 3));
                rec[3] = clip8(pr[3] + ((aa - dd) >> 3));
                int e = 0;
#pragma unroll
                for (int x = 0; x < 4; ++x) e += (sv[x] - rec[x]) * (sv[x] - rec[x]);
                e += __shfl_xor(e, 1);
                e += __shfl_xor(e, 2);
                if (act && r == 0) {
                    s_jt[wv][m] = 256ll * e + (long long)q.lambda * rate;
                    s_lastt[wv][m] = last;
                }
            }
            __syncthreads();  // B4
            if (blk) {
                int bmode = 0;
                long long bj = s_jt[wv][0];
                for (int k = 1; k < NUM_BMODES; ++k)
                    if (s_jt[wv][k] < bj) { bj = s_jt[wv][k]; bmode = k; }
                if (act && m == bmode)
#pragma unroll
                    for (int x = 0; x < 4; ++x) d[r * kBps + x] = (uint8_t)rec[x];
                if (lane < 16) s_lv4[b][lane] = s_lvt[wv][bmode][lane];
                if (lane == 0) {
                    s_bm4[b] = (uint8_t)bmode;
                    s_bnz[b] = s_lastt[wv][bmode] > 0;
                    s_bj[b] = bj;
                }
            }
            __syncthreads();  // B5
            const int b0 = i4_block(st, 0), b1 = i4_block(st, 1);
            total += s_bj[b0] + (b1 >= 0 ? s_bj[b1] : 0ll);
            if (total >= best) { ok = false; break; }  // 16x16 already better (uniform over the workgroup)
        }
        if (ok && total < best) {
            best_mode = B_PRED;
            for (int i = tid; i < 256; i += kThreadsMB) s_out[i >> 4][i & 15] = s_lv4[i >> 4][i & 15];
            if (tid < 16) s_out[24][tid] = 0;
        }
    }
    __syncthreads();
    if (stamp) stamp[3] = __builtin_amdgcn_s_memtime();

    // ---- outputs: MBOut, reconstruction, outgoing non-zero contexts ----
    int nzv = 0;
    for (int i = tid; i < 25 * 16; i += kThreadsMB) nzv |= (&s_out[0][0])[i] != 0;
    const bool skip = __syncthreads_or(nzv) == 0;
    MBOut& o = mbs[mbi];
    if (tid == 0) {
        o.ymode = (uint8_t)best_mode;
        o.uvmode = (uint8_t)i16_mode(bmuv);
        o.skip = skip ? 1 : 0;
        o.pad = 0;
    }
    if (tid < 16) o.bmodes[tid] = best_mode == B_PRED ? s_bm4[tid] : (uint8_t)best_mode;
    {
        uint32_t* dst = reinterpret_cast<uint32_t*>(&o.lv[0][0]);
        const uint32_t* sv = reinterpret_cast<const uint32_t*>(&s_out[0][0]);
        for (int i = tid; i < 200; i += kThreadsMB) dst[i] = sv[i];
    }
    if (tid < 64) {  // luma reconstruction: one 4-byte word per thread
        const int y = tid >> 2, x4 = (tid & 3) * 4;
        uint32_t v;
        if (best_mode == B_PRED) {
            const uint8_t* p = &s_y4[(y + 1) * kBps + 1 + x4];
            v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        } else {
            v = *reinterpret_cast<const uint32_t*>(&s_rec16[bm16][y * 16 + x4]);
        }
        *reinterpret_cast<uint32_t*>(&RY[(size_t)(my * 16 + y) * rw + mx * 16 + x4]) = v;
    } else if (tid < 96) {  // chroma: 2 planes x 8 rows x 2 words
        const int i = tid - 64, ch = i >> 4, y = (i >> 1) & 7, x4 = (i & 1) * 4;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(&s_recuv[bmuv][ch][y * 8 + x4]);
        *reinterpret_cast<uint32_t*>(&(ch ? RV : RU)[(size_t)(my * 8 + y) * cw + mx * 8 + x4]) = v;
    } else if (tid < 96 + 18) {
        const int k0 = tid - 96;
        const int first = best_mode == B_PRED ? 0 : 1;
        const bool top = k0 < 9;
        const int k = top ? k0 : k0 - 9;
        int v;
        if (k < 4) v = any_nz(s_out[top ? 12 + k : k * 4 + 3], first);
        else if (k < 8) {
            const int ch = (k - 4) >> 1, i = (k - 4) & 1;
            v = any_nz(s_out[16 + 4 * ch + (top ? 2 + i : i * 2 + 1)], 0);
        } else {
            v = best_mode == B_PRED ? (top ? top_nz[8] : left_nz[8]) : any_nz(s_out[24], 0);
        }
        nzs[(size_t)mbi * 18 + k0] = (uint8_t)v;
    }
    if (stamp) stamp[4] = __builtin_amdgcn_s_memtime();
}

// ---- compact MB records for the host ------------------------------------------
// One workgroup per image.  The records of k_vp8_diag (820 B per MB, mostly zero
// levels) are rewritten as a byte stream (layout in ik_vp8_gpu.h) in a device
// scratch image, then copied with 16-byte stores straight into the caller's pinned
// host buffer: a small fraction of the bytes of a plain D2H of the records, and no
// copy-engine pass on the stream.
namespace {

constexpr int kPackThreads = 1024;  // 16 waves: MB loads of an image in flight together

__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ int wave_excl_scan(int v) {
    const int lane = threadIdx.x & 63;
    int inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
    }
    return inc - v;
}
// lane = (block b = lane >> 1, half = lane & 1): its 8 levels, their nonzero mask,
// and the whole block's 16-bit mask
struct PackLane {
    int16_t v[8];
    int m8, cm;
};
__device__ __forceinline__ PackLane pack_load(const MBOut& o, int lane) {
    PackLane p;
    uint32_t w[4] = {0, 0, 0, 0};
    if (lane < 50) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&o.lv[0][0]) + lane * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = src[k];
    }
    p.m8 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        p.v[2 * k] = (int16_t)(w[k] & 0xffff);
        p.v[2 * k + 1] = (int16_t)(w[k] >> 16);
        p.m8 |= (p.v[2 * k] != 0 ? 1 : 0) << (2 * k);
        p.m8 |= (p.v[2 * k + 1] != 0 ? 1 : 0) << (2 * k + 1);
    }
    const int other = __shfl_xor(p.m8, 1);
    p.cm = (lane & 1) ? (other | (p.m8 << 8)) : (p.m8 | (other << 8));
    return p;
}

}  // namespace

__global__ __launch_bounds__(kPackThreads) void k_vp8_pack(const MBOut* __restrict__ mbs, int nmb,
                                                          uint8_t* __restrict__ scratch, uint8_t* __restrict__ dst,
                                                          size_t cap_img) {
    __shared__ uint32_t s_off[kMaxPackMBs];
    __shared__ uint32_t s_part[kPackThreads / 64];
    const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const MBOut* m0 = mbs + (size_t)img * nmb;
    uint8_t* sc = scratch + (size_t)img * cap_img;
    // 1. record sizes
    for (int m = wv; m < nmb; m += kPackThreads / 64) {
        const MBOut& o = m0[m];
        const PackLane p = pack_load(o, lane);
        const int bsz = ((lane & 1) == 0 && p.cm) ? 2 + 2 * __popc(p.cm) : 0;
        const int tot = wave_sum(bsz);
        if (lane == 0) s_off[m] = 8 + (o.ymode == B_PRED ? 16 : 0) + tot;
    }
    __syncthreads();
    // 2. exclusive scan of the sizes (each thread: a run of consecutive MBs)
    const int per = (nmb + kPackThreads - 1) / kPackThreads;
    const int lo = min(tid * per, nmb), hi = min(lo + per, nmb);
    uint32_t run = 0;
    for (int m = lo; m < hi; ++m) run += s_off[m];
    const uint32_t wex = (uint32_t)wave_excl_scan((int)run);
    if (lane == 63) s_part[wv] = wex + run;
    __syncthreads();
    uint32_t base = kPackHeaderBytes + wex;
    for (int k = 0; k < wv; ++k) base += s_part[k];
    uint32_t total = kPackHeaderBytes;
    for (int k = 0; k < kPackThreads / 64; ++k) total += s_part[k];
    for (int m = lo; m < hi; ++m) {  // each thread rewrites only its own run
        const uint32_t sz = s_off[m];
        s_off[m] = base;
        base += sz;
    }
    __syncthreads();
    // 3. the records
    for (int m = wv; m < nmb; m += kPackThreads / 64) {
        const MBOut& o = m0[m];
        const PackLane p = pack_load(o, lane);
        const bool i4 = o.ymode == B_PRED;
        const int bsz = ((lane & 1) == 0 && p.cm) ? 2 + 2 * __popc(p.cm) : 0;
        const int boff = wave_excl_scan(bsz);  // block offsets in record order (= lane order)
        const unsigned long long nzl = __ballot((lane & 1) == 0 && p.cm != 0);
        uint8_t* r = sc + s_off[m];
        if (lane == 0) {
            uint32_t nzmask = 0;
            for (int b = 0; b < 25; ++b) nzmask |= (uint32_t)((nzl >> (2 * b)) & 1) << b;
            r[0] = o.ymode;
            r[1] = o.uvmode;
            r[2] = o.skip;
            r[3] = 0;
            *reinterpret_cast<uint32_t*>(r + 4) = nzmask;
        }
        if (i4 && lane < 16) r[8 + lane] = o.bmodes[lane];
        const int blk = __shfl(boff, lane & ~1) + 8 + (i4 ? 16 : 0);  // the block's start (even lane)
        if (lane < 50 && p.cm) {
            int16_t* vals = reinterpret_cast<int16_t*>(r + blk + 2);
            if ((lane & 1) == 0) *reinterpret_cast<uint16_t*>(r + blk) = (uint16_t)p.cm;
            int rank = (lane & 1) ? __popc(p.cm & 0xff) : 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if ((p.m8 >> j) & 1) vals[rank++] = p.v[j];
        }
    }
    if (tid == 0) {
        uint32_t* h = reinterpret_cast<uint32_t*>(sc);
        h[0] = total;
        h[1] = (uint32_t)nmb;
        h[2] = kPackMagic;
        h[3] = 0;
    }
    __syncthreads();
    // 4. to the host, 16 bytes per store
    const uint4* s4 = reinterpret_cast<const uint4*>(sc);
    uint4* d4 = reinterpret_cast<uint4*>(dst + (size_t)img * cap_img);
    for (uint32_t i = tid; i < (total + 15) / 16; i += kPackThreads) d4[i] = s4[i];
}

hipError_t launch_vp8_pack(const MBOut* mbs, int nmb, int n, uint8_t* scratch, uint8_t* host_dst, size_t cap_img,
                           hipStream_t s) {
    if (nmb > kMaxPackMBs || (cap_img & 15)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_vp8_pack, dim3(n), dim3(kPackThreads), 0, s, mbs, nmb, scratch, host_dst, cap_img);
    return hipGetLastError();
}

hipError_t launch_vp8_encode(const Vp8Args& a, int n, hipStream_t s) {
    const int per_diag = a.mb_h < (a.mb_w + 1) / 2 ? a.mb_h : (a.mb_w + 1) / 2;
    const int T = (a.mb_w - 1) + 2 * (a.mb_h - 1) + 1;
    for (int t = 0; t < T; ++t)
        hipLaunchKernelGGL(k_vp8_diag, dim3(per_diag, n), dim3(kThreadsMB), 0, s, a, t);
    return hipGetLastError();
}

}  // namespace vp8
}  // namespace ik
