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
//   i4   lane = (mode, row): 10 x 4 lanes, the 16 blocks in order (each predicts
//        from the last)
//   uv   lane = (mode, channel, block): 4 x 2 x 4 = 32 lanes
// Rates and distortions are integer sums and ties keep the lowest mode, so the
// decisions -- and the bitstream -- are identical to the scalar encoder's
// (tests/test_gpu_vp8.py).  Levels stay in registers: the token rate is
// block_cost_fixed (compile-time probabilities, no table loads); LDS holds only
// what crosses lanes (contexts, the winners' levels, reconstructions).
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
    unsigned long long* stamp = (a.stamps && img == 0 && blockIdx.x == 0 && lane == 0) ? a.stamps + 8 * t : nullptr;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();

    __shared__ uint8_t s_src_y[256], s_src_u[64], s_src_v[64];
    __shared__ uint8_t s_y[17 * kBps], s_u[9 * kBps], s_v[9 * kBps], s_y4[17 * kBps];
    __shared__ uint8_t s_rec16[4][256];
    __shared__ uint8_t s_recuv[4][2][64];
    __shared__ __attribute__((aligned(16))) int16_t s_lv[64][16];  // per-lane trial levels (zigzag order)
    __shared__ int16_t s_out[25][16];  // the chosen levels (MBOut.lv layout)
    __shared__ int16_t s_lv4[16][16];  // i4 levels, block by block
    __shared__ int16_t s_y2[4][16], s_dc[4][16], s_dcq[4][16];
    __shared__ long long s_j[64];
    __shared__ int s_last[16], s_rate_y2[4];
    __shared__ int s_tr[64][4];        // i4 transposes
    __shared__ __attribute__((aligned(16))) uint16_t s_tok[8][3][24];  // kTokCostI4 (i4 token-cost rows)
    __shared__ __attribute__((aligned(16))) uint16_t s_bmc[NUM_BMODES][NUM_BMODES][NUM_BMODES];  // kBModeCost
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
    {
        const uint32_t* g = reinterpret_cast<const uint32_t*>(&kTokCostI4);
        uint32_t* l = reinterpret_cast<uint32_t*>(&s_tok[0][0][0]);
        for (int i = lane; i < (int)(sizeof(s_tok) / 4); i += 64) l[i] = g[i];
        const uint32_t* g2 = reinterpret_cast<const uint32_t*>(&kBModeCost);
        uint32_t* l2 = reinterpret_cast<uint32_t*>(&s_bmc[0][0][0]);
        for (int i = lane; i < (int)(sizeof(s_bmc) / 4); i += 64) l2[i] = g2[i];
    }
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

    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();
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
            int16_t l2v[16];
            const int l2 = quantize(y2, l2v, q.y2, 0);
            for (int i = 0; i < 16; ++i) s_y2[m][i] = l2v[i];
            s_rate_y2[m] = block_cost_fixed<1, 0>(l2v, l2, top_nz[8] + left_nz[8]);
            iwht(y2, s_dcq[m]);
        }
        int16_t lv[16];
        const int last = quantize(coef, lv, q.y1, 1);
        for (int i = 0; i < 16; ++i) s_lv[lane][i] = lv[i];
        s_nzb[lane] = last > 1;
        __syncthreads();
        const int tctx = by ? s_nzb[lane - 4] : top_nz[bx];
        const int lctx = bx ? s_nzb[lane - 1] : left_nz[by];
        int rate = block_cost_fixed<0, 1>(lv, last, tctx + lctx);
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

    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();
    // ---- luma 4x4 (B_PRED): the 16 blocks in order, lane = (mode, row) ----
    // Lane (m, r) predicts row r of mode m (tap table: no divergence across modes),
    // transforms it, owns column r of the coefficients (quantise, inverse
    // vertical pass) and row r of the reconstruction; the two transposes go
    // through LDS.  40 of 64 lanes.
    {
        const bool act = lane < 4 * NUM_BMODES;
        const int m = act ? lane >> 2 : 0, r = lane & 3, quad = lane & ~3;
        long long total = (long long)q.lambda * ymode_cost(B_PRED);
        int tnz[4] = {top_nz[0], top_nz[1], top_nz[2], top_nz[3]};
        int lnz[4] = {left_nz[0], left_nz[1], left_nz[2], left_nz[3]};
        bool ok = true;
        // per-lane constants of the block loop: tap descriptors of row r of mode m,
        // zigzag index + quantiser of column r's coefficients, bands of positions 4r..4r+3
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
        for (int b = 0; b < 16; ++b) {
            const int bx = b & 3, by = b >> 2;
            uint8_t* d = s_y4 + (by * 4 + 1) * kBps + bx * 4 + 1;
            const uint8_t* src = s_src_y + (by * 4 + r) * 16 + bx * 4;  // row r of the block
            const int top = by ? s_bm4[b - 4] : top_bm[bx];
            const int left = bx ? s_bm4[b - 1] : left_bm[by];
            const int dcv = pred4_dc(d);
            int pr[4], sv[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) {  // pred4_px without the switch
                const int t = desc[x];
                const int pa = d[p4_off((t >> 8) & 15)], pb = d[p4_off((t >> 4) & 15)], pc = d[p4_off(t & 15)];
                const int kind = t >> 12;
                const int v = kind == P4_CP ? pa : kind == P4_A2 ? avg2(pa, pb) : kind == P4_A3 ? avg3(pa, pb, pc)
                            : kind == P4_TM ? clip8(pa + pb - pc) : dcv;
                pr[x] = v;
                sv[x] = src[x];
            }
            // fdct4 row pass (row r) -> transpose -> column pass (column r)
            {
                const int d0 = sv[0] - pr[0], d1 = sv[1] - pr[1], d2 = sv[2] - pr[2], d3 = sv[3] - pr[3];
                const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
                s_tr[lane][0] = (a0 + a1) * 8;
                s_tr[lane][1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
                s_tr[lane][2] = (a0 - a1) * 8;
                s_tr[lane][3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
            }
            __syncthreads();
            int cf[4];  // raster r, 4+r, 8+r, 12+r
            {
                const int T0 = s_tr[quad][r], T1 = s_tr[quad + 1][r], T2 = s_tr[quad + 2][r], T3 = s_tr[quad + 3][r];
                const int a0 = T0 + T3, a1 = T1 + T2, a2 = T1 - T2, a3 = T0 - T3;
                cf[0] = (int16_t)((a0 + a1 + 7) >> 4);
                cf[1] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
                cf[2] = (int16_t)((a0 - a1 + 7) >> 4);
                cf[3] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
            }
            // quantise (quantize(), first = 0) the column's 4 coefficients
            int last = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = zn[i];
                const int c = cf[i], sgn = c < 0, av = sgn ? -c : c;
                int l = (int)(((unsigned)av * (unsigned)qiq[i] + (unsigned)qbias[i]) >> 17);
                if (l > 2047) l = 2047;
                if (act) s_lv[m][n] = (int16_t)(sgn ? -l : l);
                cf[i] = (int16_t)((sgn ? -l : l) * qq[i]);  // dequantised
                if (l && n + 1 > last) last = n + 1;
            }
            last = max(last, __shfl_xor(last, 1));
            last = max(last, __shfl_xor(last, 2));
            __syncthreads();
            int16_t lv[16];
            {
                const uint4 w0 = *reinterpret_cast<const uint4*>(&s_lv[m][0]);
                const uint4 w1 = *reinterpret_cast<const uint4*>(&s_lv[m][8]);
                const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                for (int i = 0; i < 8; ++i) { lv[2 * i] = (int16_t)(w[i] & 0xffff); lv[2 * i + 1] = (int16_t)(w[i] >> 16); }
            }
            // token rate (== block_cost(lv, 0, last, ctx, 3)): lane r prices zigzag
            // positions 4r..4r+3 from the LDS cost rows, the quad sums
            int rate = 0;
            {
                const int ctx0 = tnz[bx] + lnz[by];
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
            }
            // inverse transform: vertical pass on column r -> transpose -> row r
            {
                const int a = cf[0] + cf[2], bb = cf[0] - cf[2];
                const int c = mul2(cf[1]) - mul1(cf[3]), dd = mul1(cf[1]) + mul2(cf[3]);
                s_tr[lane][0] = a + dd;
                s_tr[lane][1] = bb + c;
                s_tr[lane][2] = bb - c;
                s_tr[lane][3] = a - dd;
            }
            __syncthreads();
            int rec[4], e = 0;
            {
                const int T0 = s_tr[quad][r], T1 = s_tr[quad + 1][r], T2 = s_tr[quad + 2][r], T3 = s_tr[quad + 3][r];
                const int dc = T0 + 4;
                const int a = dc + T2, bb = dc - T2;
                const int c = mul2(T1) - mul1(T3), dd = mul1(T1) + mul2(T3);
                rec[0] = clip8(pr[0] + ((a + dd) >> 3));
                rec[1] = clip8(pr[1] + ((bb + c) >> 3));
                rec[2] = clip8(pr[2] + ((bb - c) >> 3));
                rec[3] = clip8(pr[3] + ((a - dd) >> 3));
#pragma unroll
                for (int x = 0; x < 4; ++x) e += (sv[x] - rec[x]) * (sv[x] - rec[x]);
            }
            e += __shfl_xor(e, 1);
            e += __shfl_xor(e, 2);
            if (act && r == 0) {
                s_j[m] = 256ll * e + (long long)q.lambda * rate;
                s_last[m] = last;
            }
            __syncthreads();
            int bmode = 0;
            long long bj = s_j[0];
            for (int k = 1; k < NUM_BMODES; ++k)
                if (s_j[k] < bj) { bj = s_j[k]; bmode = k; }
            if (act && m == bmode)
#pragma unroll
                for (int x = 0; x < 4; ++x) d[r * kBps + x] = (uint8_t)rec[x];
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

    if (stamp) stamp[3] = __builtin_amdgcn_s_memtime();
    // ---- chroma (try_uv): lane = (mode, channel, block) ----
    int bmuv;
    {
        const bool act = lane < 32;
        const int m = (lane >> 3) & 3, ch = (lane >> 2) & 1, b = lane & 3, bx = b & 1, by = b >> 1;
        const int mode = i16_mode(m);
        const uint8_t* src = (ch ? s_src_v : s_src_u) + by * 4 * 8 + bx * 4;
        uint8_t pr[16];
        int16_t coef[16], lv[16];
        int last = 0;
        if (act) {
            pred_blk(mode, 8, (ch ? s_v : s_u) + kBps + 1, mx, my, bx, by, pr);
            fdct4(src, 8, pr, 4, coef);
            last = quantize(coef, lv, q.uv, 0);
            for (int i = 0; i < 16; ++i) s_lv[lane][i] = lv[i];
            s_nzb[lane] = last > 0;
        }
        __syncthreads();
        int rate = 0, dist = 0;
        if (act) {
            const int tctx = by ? s_nzb[lane - 2] : top_nz[4 + 2 * ch + bx];
            const int lctx = bx ? s_nzb[lane - 1] : left_nz[4 + 2 * ch + by];
            rate = block_cost_fixed<2, 0>(lv, last, tctx + lctx);
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

    if (stamp) stamp[4] = __builtin_amdgcn_s_memtime();
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
    if (stamp) stamp[5] = __builtin_amdgcn_s_memtime();
}

hipError_t launch_vp8_encode(const Vp8Args& a, int n, hipStream_t s) {
    const int per_diag = a.mb_h < (a.mb_w + 1) / 2 ? a.mb_h : (a.mb_w + 1) / 2;
    const int T = (a.mb_w - 1) + 2 * (a.mb_h - 1) + 1;
    for (int t = 0; t < T; ++t) hipLaunchKernelGGL(k_vp8_diag, dim3(per_diag, n), dim3(64), 0, s, a, t);
    return hipGetLastError();
}

}  // namespace vp8
}  // namespace ik
