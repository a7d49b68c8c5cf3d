// ik_vp8x.hip -- the exact WebP coder's device half: libwebp method 4's macroblock
// decisions (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp; the arithmetic
// is ik_vp8x.h, the same as oracle/vp8_modes.c, whose files equal WebPEncodeRGB's).
//
// Dependencies and how they are scheduled:
//  - a macroblock predicts from the reconstruction of its left, top-left, top and
//    top-right neighbours, and reads their non-zero contexts and chroma DC errors: all
//    MBs with the same mb_x + 2 mb_y are independent (a diagonal);
//  - libwebp's token loop refreshes the coefficient probabilities -- hence the level
//    costs every decision uses -- from the statistics of all MBs before it, at MB
//    indices M, 2M+1, 3M+2, ... (M = max(mb_count / 8, 96)): an epoch's MBs may only
//    start when every earlier MB is decided and the statistics folded.
// So per epoch: one k_vp8x_mb launch per diagonal (every image of the batch in the
// launch, grid.y = image), then k_vp8x_stats (one wave per image) folds the epoch's
// token statistics in raster order (libwebp halves a counter pair at 65534, so the
// order matters) and refreshes probabilities and level costs.
//
// k_vp8x_mb: one wave64 per MB; the modes of each stage run on their own lanes --
// i16: 4 lanes, intra-4: 10 lanes per sub-block (16 sub-blocks in order), chroma: 4
// lanes -- and the winner is the lowest score, ties to the lowest mode (libwebp's
// early-out in the intra-4 loop never changes that argmin: a skipped mode's partial
// score already reaches the best full score).
#include <hip/hip_runtime.h>

#include "ik_vp8x.h"
#include "ik_vp8x_gpu.h"

namespace ik {
namespace vp8x {

namespace {

constexpr int kTopLeftI4[16] = {17, 21, 25, 29, 13, 17, 21, 25, 9, 13, 17, 21, 5, 9, 13, 17};

// GetResidualCost with libwebp's fixed level costs and entropy costs staged in LDS
// (the constant tables would be per-lane divergent global loads inside the serial
// coefficient loop).  Every coefficient's context is known from its predecessor's
// level, so the 16 terms are independent: the block comes in with two 16-byte LDS
// reads, and all 32 table reads are issued together (unrolled; a position outside
// [first, last] reads a valid entry and adds 0) instead of a chain of dependent
// reads per coefficient.  Same integer sum as residual_cost (ik_vp8x.h): the last
// position is max(last non-zero, first), as in libwebp's loop.
__device__ __forceinline__ int rcost(const uint16_t* lc, const uint8_t* pr, const uint16_t* fixed, const uint16_t* ent,
                                     const uint8_t* bands, int type, int first, int ctx0, const int16_t* c) {
    int v[16];
    {
        const uint4 q0 = reinterpret_cast<const uint4*>(c)[0], q1 = reinterpret_cast<const uint4*>(c)[1];
        const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int lo = (int16_t)(w[i] & 0xffffu), hi = (int16_t)(w[i] >> 16);
            v[2 * i] = lo < 0 ? -lo : lo;
            v[2 * i + 1] = hi < 0 ? -hi : hi;
        }
    }
    int last = -1;
#pragma unroll
    for (int n = 0; n < 16; ++n)
        if (v[n]) last = n;
    const int p0 = pr[((type * 8 + kEncBands[first]) * 3 + ctx0) * 11];
    if (last < 0) return ent[p0];
    if (last < first) last = first;
    int cost = ctx0 == 0 ? ent[255 - p0] : 0;
    const int rowbase = type * 8 * 3;
#pragma unroll
    for (int n = 0; n < 16; ++n) {
        const int ctx = n == 0 ? ctx0 : (n == first ? ctx0 : (v[n - 1] >= 2 ? 2 : v[n - 1]));
        const int vv = v[n];
        const int term = fixed[vv] + lc[(rowbase + kEncBands[n] * 3 + ctx) * kLevelTab + (vv > kMaxVarLevel ? kMaxVarLevel : vv)];
        cost += (n >= first && n <= last) ? term : 0;
    }
    int vl = 0;
#pragma unroll
    for (int n = 0; n < 16; ++n)
        if (n == last) vl = v[n];
    if (last < 15) {
        int bl = 0;
#pragma unroll
        for (int n = 0; n < 15; ++n)
            if (n == last) bl = kEncBands[n + 1];
        cost += ent[pr[((type * 8 + bl) * 3 + (vl == 1 ? 1 : 2)) * 11]];
    }
    return cost;
}

// row y of pred_nxn(dst, m, left, top, 8) (ik_vp8x.h), built in registers and stored as
// two words: the chroma predictors on 8 lanes per mode instead of one
__device__ __forceinline__ void pred8_row(uint8_t* dst, int m, const uint8_t* left, const uint8_t* top, int y) {
    uint8_t o[8];
    if (m == 0) {
        int DC = 0;
        if (top) {
            for (int j = 0; j < 8; ++j) DC += top[j];
            if (left) for (int j = 0; j < 8; ++j) DC += left[j];
            else DC += DC;
            DC = (DC + 8) >> 4;
        } else if (left) {
            for (int j = 0; j < 8; ++j) DC += left[j];
            DC += DC;
            DC = (DC + 8) >> 4;
        } else {
            DC = 0x80;
        }
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = (uint8_t)DC;
    } else if (m == 1 && left && top) {
        const int ly = left[y], c = left[-1];
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = xclip8(ly + top[x] - c);
    } else if ((m == 1 && top) || m == 2) {  // TM without left, V: the row above (127 at the top edge)
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = top ? top[x] : (m == 1 ? 129 : 127);
    } else {  // TM without top, H: the left sample (129 at the left edge; TM with neither: 129)
        const uint8_t v = left ? left[y] : 129;
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = v;
    }
    uint32_t w0 = 0, w1 = 0;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        w0 |= (uint32_t)o[x] << (8 * x);
        w1 |= (uint32_t)o[4 + x] << (8 * x);
    }
    *reinterpret_cast<uint2*>(dst + y * BPS) = make_uint2(w0, w1);
}

__device__ __forceinline__ int64_t rdlane64(int64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t rd_score(int64_t R, int64_t H, int64_t D, int64_t SD, int lambda) {
    return (R + H) * lambda + 256 * (D + SD);
}

}  // namespace

// dev switch IK_VP8X_STAMPS: per-phase shader-clock sums over image 0's MBs
// (tools/vp8x_timing.py --stamps reads them through ik_vp8x_stamps)
#ifdef IK_VP8X_STAMPS
__device__ unsigned long long g_vp8x_stamps[32];
#define IK_STAMP(i)                                                         \
    do {                                                                    \
        if (l == 0 && img == 0) {                                           \
            const unsigned long long t_ = clock64();                        \
            atomicAdd(&g_vp8x_stamps[i], t_ - t_prev);                      \
            t_prev = t_;                                                    \
        }                                                                   \
    } while (0)
#else
#define IK_STAMP(i) do {} while (0)
#endif

__global__ __launch_bounds__(64) void k_vp8x_mb(XArgs a, const int* __restrict__ list) {
    const int l = threadIdx.x;
    const int img = blockIdx.y;
    const int mb = list[blockIdx.x];
#ifdef IK_VP8X_STAMPS
    unsigned long long t_prev = clock64();
#endif
    const int mx = mb % a.mb_w, my = mb / a.mb_w;
    const int nmb = a.mb_w * a.mb_h;
    const int W = a.mb_w * 16, H = a.mb_h * 16;
    const int uw = (a.w + 1) >> 1, uh = (a.h + 1) >> 1;
    const uint8_t* Y = a.yuv + (size_t)img * a.yuv_stride;
    const uint8_t* U = Y + (size_t)a.w * a.h;
    const uint8_t* V = U + (size_t)uw * uh;
    uint8_t* RY = a.rec + (size_t)img * a.rec_stride;
    uint8_t* RU = RY + (size_t)W * H;
    uint8_t* RV = RU + (size_t)(W / 2) * (H / 2);
    XMB* mbs = a.mbs + (size_t)img * nmb;
    uint32_t* nzs = a.nz + (size_t)img * nmb;
    int8_t* derrs = a.derr + (size_t)img * nmb * 8;
    const int sg = a.seg[(size_t)img * nmb + mb];
    // the image's level costs and probabilities, read at every coefficient of every
    // candidate: staged in LDS (13.4 KB)
#ifdef IK_VP8X_LC_GLOBAL
    const uint16_t* lc = a.lc + (size_t)img * kCostRows * kLevelTab;
#else
    __shared__ __attribute__((aligned(16))) uint16_t lc[kCostRows * kLevelTab];
#endif
    __shared__ __attribute__((aligned(16))) uint8_t pr[1056];
    __shared__ __attribute__((aligned(16))) uint16_t s_fixed[2048];
    __shared__ uint16_t s_ent[256];
    __shared__ uint8_t s_bands[17];
    __shared__ uint16_t s_fi4[1000];
    // staging: every lane issues all of its global reads first (one memory latency for
    // the whole prologue), then writes them to LDS
    {
        constexpr int kFi4 = (1000 + 63) / 64, kFix = 2048 / 64, kEnt = 256 / 64;
        constexpr int kPr = (1056 / 16 + 63) / 64;
        uint16_t rf4[kFi4], rfx[kFix], ren[kEnt];
#pragma unroll
        for (int j = 0; j < kFi4; ++j) rf4[j] = kFixedCostsI4[min(l + 64 * j, 999)];
#pragma unroll
        for (int j = 0; j < kFix; ++j) rfx[j] = kLevelFixedCosts[l + 64 * j];
#pragma unroll
        for (int j = 0; j < kEnt; ++j) ren[j] = kEntropyCost[l + 64 * j];
        const uint4* gp = (const uint4*)(a.pr + (size_t)img * 1056);
        uint4 rpr[kPr];
#pragma unroll
        for (int j = 0; j < kPr; ++j) rpr[j] = gp[min(l + 64 * j, 1056 / 16 - 1)];
#pragma unroll
        for (int j = 0; j < kFi4; ++j)
            if (l + 64 * j < 1000) s_fi4[l + 64 * j] = rf4[j];
#pragma unroll
        for (int j = 0; j < kFix; ++j) s_fixed[l + 64 * j] = rfx[j];
#pragma unroll
        for (int j = 0; j < kEnt; ++j) s_ent[l + 64 * j] = ren[j];
#ifndef IK_VP8X_LC_GLOBAL
        {  // 13 x 16 B per lane (a register array this size would go to scratch)
            const uint4* g = (const uint4*)(a.lc + (size_t)img * kCostRows * kLevelTab);
            for (int i = l; i < kCostRows * kLevelTab / 8; i += 64) ((uint4*)lc)[i] = g[i];
        }
#endif
#pragma unroll
        for (int j = 0; j < kPr; ++j)
            if (l + 64 * j < 1056 / 16) ((uint4*)pr)[l + 64 * j] = rpr[j];
    }
    if (l < 17) s_bands[l] = kEncBands[l];
    // the segment's matrices and lambdas, read per lane in every quantisation: LDS
    __shared__ __attribute__((aligned(16))) XSeg s_Q;
    {
        static_assert(sizeof(XSeg) % 4 == 0, "XSeg copied as words");
        const uint32_t* gq = reinterpret_cast<const uint32_t*>(a.segs + img * 4 + sg);
        for (int i = l; i < (int)(sizeof(XSeg) / 4); i += 64) reinterpret_cast<uint32_t*>(&s_Q)[i] = gq[i];
    }
    const XSeg& Q = s_Q;

    __shared__ __attribute__((aligned(16))) uint8_t s_in[BPS * 16];      // Y 0..15, U 16..23, V 24..31
    __shared__ uint8_t s_yl[17], s_yt[20], s_ul[9], s_ut[8], s_vl[9], s_vt[8];
    __shared__ int s_tnz[9], s_lnz[9];
    __shared__ int8_t s_derr_t[2][2], s_derr_l[2][2];
    __shared__ __attribute__((aligned(16))) uint8_t s_rec16[4][BPS * 16];
    __shared__ __attribute__((aligned(16))) int16_t s_lv16[4][17][16];
    __shared__ int64_t s_sc[16], s_part[16][4];
    __shared__ int s_flat[4], s_nz16[4];
    __shared__ __attribute__((aligned(16))) uint8_t s_best4[BPS * 16];
    __shared__ uint8_t s_bound[37];
    __shared__ int16_t s_lv4[16][16];
    __shared__ uint8_t s_modes4[16];
    __shared__ uint8_t s_nbm[8];  // the left MB's right column of sub-block modes, the top MB's bottom row
    __shared__ __attribute__((aligned(16))) uint8_t s_blk[10][4 * BPS];
    __shared__ __attribute__((aligned(16))) int16_t s_blv[10][16];
    __shared__ __attribute__((aligned(16))) uint8_t s_recuv[4][BPS * 8];
    __shared__ __attribute__((aligned(16))) int16_t s_lvuv[4][8][16];
    __shared__ int8_t s_duv[4][2][3];
    __shared__ int s_b16, s_buv, s_i4ok;
    __shared__ int64_t s_s16;  // the i16 best's score at lambda_mode (the intra-4 bar)
    // per-lane work buffers in LDS (private arrays would live in scratch memory)
    __shared__ __attribute__((aligned(16))) uint8_t s_pred16[4][BPS * 16];
    __shared__ __attribute__((aligned(16))) int16_t s_tmp16[4][16][16];
    __shared__ __attribute__((aligned(16))) uint8_t s_pred4[10][4 * BPS];
    __shared__ __attribute__((aligned(16))) uint8_t s_predc[4][BPS * 8];
    __shared__ __attribute__((aligned(16))) int16_t s_tmpc[4][8][16];
    __shared__ int16_t s_dc16[4][16];
    __shared__ int s_bnz[4][16], s_cnz[4][8];
    __shared__ int s_ft4[10][16], s_C4[10][16], s_tt4[10][2][16];
    __shared__ int16_t s_cf4[10][16];

    // ---- load the source MB (ImportBlock: clamped coordinates) and the boundaries ----
    for (int i = l; i < 256; i += 64) {
        const int y = i >> 4, x = i & 15;
        s_in[y * BPS + x] = Y[(size_t)min(16 * my + y, a.h - 1) * a.w + min(16 * mx + x, a.w - 1)];
    }
    for (int i = l; i < 128; i += 64) {
        const int c = i >> 6, k = i & 63, y = k >> 3, x = k & 7;
        const uint8_t* P = c ? V : U;
        s_in[y * BPS + 16 + 8 * c + x] = P[(size_t)min(8 * my + y, uh - 1) * uw + min(8 * mx + x, uw - 1)];
    }
    if (l < 16) {
        s_yl[1 + l] = mx ? RY[(size_t)(16 * my + l) * W + 16 * mx - 1] : 129;
        s_yt[l] = my ? RY[(size_t)(16 * my - 1) * W + 16 * mx + l] : 127;
    } else if (l < 20) {
        const int k = l - 16;
        s_yt[16 + k] = !my ? 127 : (mx < a.mb_w - 1 ? RY[(size_t)(16 * my - 1) * W + 16 * mx + 16 + k]
                                                       : RY[(size_t)(16 * my - 1) * W + 16 * mx + 15]);
    } else if (l < 28) {
        const int k = l - 20;
        s_ul[1 + k] = mx ? RU[(size_t)(8 * my + k) * (W / 2) + 8 * mx - 1] : 129;
        s_vl[1 + k] = mx ? RV[(size_t)(8 * my + k) * (W / 2) + 8 * mx - 1] : 129;
        s_ut[k] = my ? RU[(size_t)(8 * my - 1) * (W / 2) + 8 * mx + k] : 127;
        s_vt[k] = my ? RV[(size_t)(8 * my - 1) * (W / 2) + 8 * mx + k] : 127;
    } else if (l == 28) {
        s_yl[0] = !mx ? (my ? 129 : 127) : (my ? RY[(size_t)(16 * my - 1) * W + 16 * mx - 1] : 127);
        s_ul[0] = !mx ? (my ? 129 : 127) : (my ? RU[(size_t)(8 * my - 1) * (W / 2) + 8 * mx - 1] : 127);
        s_vl[0] = !mx ? (my ? 129 : 127) : (my ? RV[(size_t)(8 * my - 1) * (W / 2) + 8 * mx - 1] : 127);
    } else if (l == 29) {  // NzToBytes (+ the row's running left DC bit in bit 25)
        const uint32_t tnz = my ? nzs[mb - a.mb_w] : 0u, lnz = mx ? nzs[mb - 1] : 0u;
        const int tb[9] = {12, 13, 14, 15, 18, 19, 22, 23, 24}, lb[8] = {3, 7, 11, 15, 17, 19, 21, 23};
        for (int i = 0; i < 9; ++i) s_tnz[i] = (int)((tnz >> tb[i]) & 1u);
        for (int i = 0; i < 8; ++i) s_lnz[i] = (int)((lnz >> lb[i]) & 1u);
        s_lnz[8] = (int)((lnz >> 25) & 1u);
    } else if (l >= 32 && l < 40) {
        const int k = l - 32;
        s_nbm[k] = k < 4 ? (mx ? mbs[mb - 1].bmodes[k * 4 + 3] : 0) : (my ? mbs[mb - a.mb_w].bmodes[12 + k - 4] : 0);
    } else if (l == 30) {
        for (int c = 0; c < 2; ++c)
            for (int k = 0; k < 2; ++k) {
                s_derr_t[c][k] = (a.use_derr && my) ? derrs[(size_t)(mb - a.mb_w) * 8 + c * 2 + k] : 0;
                s_derr_l[c][k] = (a.use_derr && mx) ? derrs[(size_t)(mb - 1) * 8 + 4 + c * 2 + k] : 0;
            }
    }
    __syncthreads();
    IK_STAMP(0);

    // ---- intra-16: lane = (mode, 4x4 block), 4 x 16 lanes ----
    {
        const int m = l >> 4, n = l & 15, bx = n & 3, by = n >> 2;
        const int off = bx * 4 + by * 4 * BPS;
        uint8_t* pred = s_pred16[m];
        pred16_block(pred, m, mx ? s_yl + 1 : nullptr, my ? s_yt : nullptr, bx, by);
        ftransform(s_in + off, pred + off, s_tmp16[m][n]);
        __syncthreads();
        if (n == 0) {  // the mode's Y2: WHT of the 16 DCs, quantised
            ftransform_wht(s_tmp16[m][0], s_dc16[m]);
            s_nz16[m] = quantize_block(s_dc16[m], s_lv16[m][0], Q.y2) << 24;
        }
        __syncthreads();
        s_tmp16[m][n][0] = 0;
        const int bnz = quantize_block(s_tmp16[m][n], s_lv16[m][1 + n], Q.y1);
        s_bnz[m][n] = bnz;
        __syncthreads();
        if (n == 0) itransform_wht(s_dc16[m], s_tmp16[m][0]);  // the DCs back into the blocks
        __syncthreads();
        itransform(pred + off, s_tmp16[m][n], s_rec16[m] + off);
        // this block's distortion, rate (VP8GetCostLuma16's contexts: the block above and
        // to the left in this mode, or the MB's incoming ones) and AC count
        int D = 0;
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) {
                const int d = s_in[off + x + y * BPS] - s_rec16[m][off + x + y * BPS];
                D += d * d;
            }
        int dis = Q.tlambda ? disto4x4(s_in + off, s_rec16[m] + off) : 0;
        const int ctx = (by ? s_bnz[m][n - 4] : s_tnz[bx]) + (bx ? s_bnz[m][n - 1] : s_lnz[by]);
        int R = rcost(lc, pr, s_fixed, s_ent, s_bands, 0, 1, ctx, s_lv16[m][1 + n]);
        if (n == 0) R += rcost(lc, pr, s_fixed, s_ent, s_bands, 1, 0, s_tnz[8] + s_lnz[8], s_lv16[m][0]);
        int cnt = 0;
        for (int k = 1; k < 16; ++k) cnt += s_lv16[m][1 + n][k] != 0;
        int nzm = bnz << n;
        for (int o = 8; o; o >>= 1) {  // sums over the mode's 16 lanes
            D += __shfl_xor(D, o, 64);
            dis += __shfl_xor(dis, o, 64);
            R += __shfl_xor(R, o, 64);
            cnt += __shfl_xor(cnt, o, 64);
            nzm |= __shfl_xor(nzm, o, 64);
        }
        if (n == 0) {
            s_flat[m] = cnt <= 10;  // IsFlat(levels, 16 blocks, FLATNESS_LIMIT_I16)
            s_nz16[m] |= nzm;
            s_part[m][0] = D;
            s_part[m][1] = Q.tlambda ? ((Q.tlambda * dis + 128) >> 8) : 0;
            s_part[m][2] = R;
            s_part[m][3] = kFixedCostsI16[m];
        }
    }
    __syncthreads();
    IK_STAMP(1);
    if (l == 0) {
        // IsFlatSource16; the doubling chain of PickBestIntra16 (flat so far in mode order)
        int flat = 1;
        for (int i = 1; i < 256 && flat; ++i) flat = s_in[(i >> 4) * BPS + (i & 15)] == s_in[0];
        int best = 0;
        int64_t bs = 0, bD = 0, bSD = 0, bR = 0, bH = 0;
        for (int m = 0; m < 4; ++m) {
            int64_t D = s_part[m][0], SD = s_part[m][1];
            if (flat) {
                flat = s_flat[m];
                if (flat) { D *= 2; SD *= 2; }
            }
            const int64_t sc = rd_score(s_part[m][2], s_part[m][3], D, SD, Q.lambda_i16);
            if (m == 0 || sc < bs) { bs = sc; best = m; bD = D; bSD = SD; bR = s_part[m][2]; bH = s_part[m][3]; }
        }
        s_b16 = best;
        s_s16 = rd_score(bR, bH, bD, bSD, Q.lambda_mode);  // the i16 score for the mode decision
        // StoreMaxDelta: a DC-only MB of fairly high distortion
        if (((uint32_t)s_nz16[best] & 0x100ffffu) == 0x1000000u && bD > Q.min_disto) {
            const int16_t* d = s_lv16[best][0];
            int mv = xabs(d[1]) > xabs(d[2]) ? xabs(d[1]) : xabs(d[2]);
            mv = xabs(d[4]) > mv ? xabs(d[4]) : mv;
            atomicMax(a.max_edge + img * 4 + sg, mv);
        }
        // VP8IteratorStartI4: the intra-4 boundary, contexts re-imported
        for (int i = 0; i < 17; ++i) s_bound[i] = s_yl[16 - i];
        for (int i = 0; i < 20; ++i) s_bound[17 + i] = s_yt[i];
        s_i4ok = 1;
    }
    __syncthreads();
    IK_STAMP(2);

    // ---- intra-4: 16 sub-blocks in order, lane = mode ----
    {
        int tnz4[4], lnz4[4];
        for (int i = 0; i < 4; ++i) { tnz4[i] = s_tnz[i]; lnz4[i] = s_lnz[i]; }
        int64_t aS = 211ll * Q.lambda_mode;  // rd_best: H = 211 = VP8BitCost(0, 145)
        int header_bits = 0;
#ifdef IK_VP8X_NO_I4
        if (l == 0) s_i4ok = 0;
        for (int i4 = 0; i4 < 0; ++i4) {
#else
        for (int i4 = 0; i4 < 16; ++i4) {
#endif
            const int bx = i4 & 3, by = i4 >> 2;
            const int off = bx * 4 + by * 4 * BPS;
            // lanes = (mode, row): 10 x 4; each transform split into its row and column passes
            const int m = l >> 2, r = l & 3;
            const bool act = l < 40;
            if (act) {  // the mode's block in registers, row r stored by lane r
                // the 13 boundary samples are the same for every lane: read them once and
                // make them wave-uniform (SGPRs), so the ten divergent mode paths below are
                // pure ALU instead of ten rounds of LDS reads
                const uint8_t* tp = s_bound + kTopLeftI4[i4];
                uint8_t e[13];
#pragma unroll
                for (int k = 0; k < 13; ++k) e[k] = (uint8_t)__builtin_amdgcn_readfirstlane((int)tp[k - 5]);
                // every mode's block from the uniform samples (scalar ALU, no divergent
                // paths); lane (m, r) keeps its mode's row r by selects
                uint32_t mine = 0;
#pragma unroll
                for (int mm = 0; mm < 10; ++mm) {
                    uint8_t d[16];
                    pred4<4>(d, mm, e + 5);
                    uint32_t rw[4];
#pragma unroll
                    for (int y = 0; y < 4; ++y)
                        rw[y] = (uint32_t)d[4 * y] | ((uint32_t)d[4 * y + 1] << 8) | ((uint32_t)d[4 * y + 2] << 16) |
                                ((uint32_t)d[4 * y + 3] << 24);
                    const uint32_t row = r == 0 ? rw[0] : r == 1 ? rw[1] : r == 2 ? rw[2] : rw[3];
                    mine = m == mm ? row : mine;
                }
                *reinterpret_cast<uint32_t*>(s_pred4[m] + r * BPS) = mine;
            }
            __syncthreads();
            IK_STAMP(10);
            if (act) {  // FTransform, row r
                const uint8_t* sr = s_in + off + r * BPS;
                const uint8_t* pp = s_pred4[m] + r * BPS;
                const int d0 = sr[0] - pp[0], d1 = sr[1] - pp[1], d2 = sr[2] - pp[2], d3 = sr[3] - pp[3];
                const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
                s_ft4[m][0 + 4 * r] = (a0 + a1) * 8;
                s_ft4[m][1 + 4 * r] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
                s_ft4[m][2 + 4 * r] = (a0 - a1) * 8;
                s_ft4[m][3 + 4 * r] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
            }
            __syncthreads();
            IK_STAMP(11);
            if (act) {  // column r
                const int* t = s_ft4[m];
                const int i = r;
                const int a0 = t[0 + i] + t[12 + i], a1 = t[4 + i] + t[8 + i];
                const int a2 = t[4 + i] - t[8 + i], a3 = t[0 + i] - t[12 + i];
                s_cf4[m][0 + i] = (int16_t)((a0 + a1 + 7) >> 4);
                s_cf4[m][4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
                s_cf4[m][8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
                s_cf4[m][12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
            }
            __syncthreads();
            IK_STAMP(12);
            int nzl = 0, cnt = 0;
            if (act) {  // QuantizeBlock: zigzag positions 4r .. 4r+3 (all reads first, then the
                        // stores: the reads of one position no longer wait for the last one's store)
                int jj[4], vv[4], lv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    jj[k] = zigzag(4 * r + k);
                    vv[k] = s_cf4[m][jj[k]];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int j = jj[k], v = vv[k];
                    const int sign = v < 0;
                    const uint32_t coeff = (uint32_t)((sign ? -v : v) + Q.y1.sharpen[j]);
                    int level = 0;
                    if (coeff > Q.y1.zthresh[j]) {
                        level = (int)((coeff * Q.y1.iq[j] + Q.y1.bias[j]) >> QFIX);
                        if (level > 2047) level = 2047;
                        if (sign) level = -level;
                    }
                    lv[k] = level;
                    nzl |= level != 0;
                    cnt += (4 * r + k) > 0 && level != 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    s_cf4[m][jj[k]] = (int16_t)(lv[k] * (int)Q.y1.q[jj[k]]);
                    s_blv[m][4 * r + k] = (int16_t)lv[k];
                }
            }
            __syncthreads();
            IK_STAMP(13);
            if (act) {  // ITransform, column r
                const int16_t* in = s_cf4[m];
                const int i = r;
                const int a = in[i] + in[8 + i], b = in[i] - in[8 + i];
                const int c = ((in[4 + i] * 35468) >> 16) - (((in[12 + i] * 20091) >> 16) + in[12 + i]);
                const int d = (((in[4 + i] * 20091) >> 16) + in[4 + i]) + ((in[12 + i] * 35468) >> 16);
                s_C4[m][4 * i + 0] = a + d;
                s_C4[m][4 * i + 1] = b + c;
                s_C4[m][4 * i + 2] = b - c;
                s_C4[m][4 * i + 3] = a - d;
            }
            __syncthreads();
            IK_STAMP(14);
            int sse = 0;
            if (act) {  // row r: the reconstruction, its SSE and the spectral rows of source and reconstruction
                const int* C = s_C4[m];
                const int i = r;
                const int dc = C[i] + 4;
                const int a = dc + C[8 + i], b = dc - C[8 + i];
                const int c = ((C[4 + i] * 35468) >> 16) - (((C[12 + i] * 20091) >> 16) + C[12 + i]);
                const int d = (((C[4 + i] * 20091) >> 16) + C[4 + i]) + ((C[12 + i] * 35468) >> 16);
                const uint8_t* pp = s_pred4[m] + i * BPS;
                uint8_t* o = s_blk[m] + i * BPS;
                o[0] = xclip8(pp[0] + ((a + d) >> 3));
                o[1] = xclip8(pp[1] + ((b + c) >> 3));
                o[2] = xclip8(pp[2] + ((b - c) >> 3));
                o[3] = xclip8(pp[3] + ((a - d) >> 3));
                const uint8_t* sr = s_in + off + i * BPS;
                for (int x = 0; x < 4; ++x) {
                    const int e = sr[x] - o[x];
                    sse += e * e;
                }
                for (int q = 0; q < 2; ++q) {
                    const uint8_t* in = q ? o : sr;
                    const int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[1] - in[3], a3 = in[0] - in[2];
                    s_tt4[m][q][0 + 4 * i] = a0 + a1;
                    s_tt4[m][q][1 + 4 * i] = a3 + a2;
                    s_tt4[m][q][2 + 4 * i] = a3 - a2;
                    s_tt4[m][q][3 + 4 * i] = a0 - a1;
                }
            }
            __syncthreads();
            IK_STAMP(15);
            int tA = 0, tB = 0;
            if (act) {  // the spectral columns, weighted
                const int i = r;
                for (int q = 0; q < 2; ++q) {
                    const int* t = s_tt4[m][q];
                    const int a0 = t[0 + i] + t[8 + i], a1 = t[4 + i] + t[12 + i];
                    const int a2 = t[4 + i] - t[12 + i], a3 = t[0 + i] - t[8 + i];
                    const int v = kWeightY[i] * xabs(a0 + a1) + kWeightY[4 + i] * xabs(a3 + a2) +
                                  kWeightY[8 + i] * xabs(a3 - a2) + kWeightY[12 + i] * xabs(a0 - a1);
                    if (q) tB = v;
                    else tA = v;
                }
            }
            for (int o = 1; o <= 2; o <<= 1) {  // over the mode's 4 lanes
                sse += __shfl_xor(sse, o, 64);
                tA += __shfl_xor(tA, o, 64);
                tB += __shfl_xor(tB, o, 64);
                cnt += __shfl_xor(cnt, o, 64);
                nzl |= __shfl_xor(nzl, o, 64);
            }
            // the mode's score and terms on its lane r == 0 (4m)
            int64_t myS = INT64_MAX, myD = 0, mySD = 0, myR = 0, myH = 0;
            if (act && r == 0) {
                // mode costs from the neighbouring sub-blocks' modes (frame edge: B_DC)
                const int left = bx ? s_modes4[i4 - 1] : s_nbm[by];
                const int topm = by ? s_modes4[i4 - 4] : s_nbm[4 + bx];
                myD = sse;
                mySD = Q.tlambda ? ((Q.tlambda * (xabs(tB - tA) >> 5) + 128) >> 8) : 0;
                myH = s_fi4[(topm * 10 + left) * 10 + m];
                myR = (m > 0 && cnt <= 3) ? 140 : 0;  // IsFlat(levels, 1, FLATNESS_LIMIT_I4)
                myR += rcost(lc, pr, s_fixed, s_ent, s_bands, 3, 0, tnz4[bx] + lnz4[by], s_blv[m]);
                myS = rd_score(myR, myH, myD, mySD, Q.lambda_i4);
            }
            // lane 4m holds mode m's score: read the ten with v_readlane (wave-uniform
            // results, no LDS), strict "<" in mode order = ties to the lowest mode
            int64_t bsc = INT64_MAX;
            int best = 0;
#pragma unroll
            for (int mm = 0; mm < 10; ++mm) {
                const int64_t sc = rdlane64(myS, 4 * mm);
                if (sc < bsc) { bsc = sc; best = mm; }
            }
            const int64_t sD = rdlane64(myD, 4 * best), sSD = rdlane64(mySD, 4 * best), sR = rdlane64(myR, 4 * best),
                          sH = rdlane64(myH, 4 * best);
            const int nzb = __builtin_amdgcn_readlane(nzl, 4 * best);
            aS += rd_score(sR, sH, sD, sSD, Q.lambda_mode);
            header_bits += (int)sH;
            const bool stop = aS >= s_s16 || header_bits > 256 * 16 * 16;
            if (l < 16) s_lv4[i4][l] = s_blv[best][l];
            if (l < 16) s_best4[off + (l & 3) + (l >> 2) * BPS] = s_blk[best][(l & 3) + (l >> 2) * BPS];
            __syncthreads();
            IK_STAMP(16);
            if (stop) {
                if (l == 0) s_i4ok = 0;
                break;
            }
            tnz4[bx] = lnz4[by] = nzb;
            if (l == 0) s_modes4[i4] = (uint8_t)best;
            if (l < 4) {
                // VP8IteratorRotateI4, one position per lane (the writes [-4, 4) never
                // overlap another lane's reads: [4, 8) or the block)
                uint8_t* top = s_bound + kTopLeftI4[i4];
                const uint8_t* blk = s_best4 + off;
                const uint8_t b0 = blk[l + 3 * BPS];
                const uint8_t b1 = (i4 & 3) != 3 ? (l < 3 ? blk[3 + (2 - l) * BPS] : top[3]) : top[l + 4];
                top[-4 + l] = b0;
                top[l] = b1;
            }
            __syncthreads();
            IK_STAMP(17);
        }
    }
    __syncthreads();
    IK_STAMP(3);

    // ---- chroma: lane = (mode, 4x4 block), 4 x 8 lanes ----
    {
        const int m = (l >> 3) & 3, n = l & 7, ch = n >> 2, b = n & 3, bx = b & 1, by = b >> 1;
        const int off = bx * 4 + by * 4 * BPS + ch * 8;  // VP8ScanUV
        const bool act = l < 32;
        uint8_t* pred = s_predc[m];
        if (act) {  // lane (m, n): row n of both channels
            pred8_row(pred, m, mx ? s_ul + 1 : nullptr, my ? s_ut : nullptr, n);
            pred8_row(pred + 8, m, mx ? s_vl + 1 : nullptr, my ? s_vt : nullptr, n);
        }
        __syncthreads();
        if (act) ftransform(s_in + 16 + off, pred + off, s_tmpc[m][n]);
        __syncthreads();
        if (act && a.use_derr && b == 0) {  // CorrectDCValues, one channel: its 4 DCs in order
            const int8_t* top = s_derr_t[ch];
            const int8_t* left = s_derr_l[ch];
            int16_t(*c)[16] = &s_tmpc[m][ch * 4];
            auto qs = [&](int16_t* v) {
                int Vv = *v;
                const int sign = Vv < 0;
                if (sign) Vv = -Vv;
                if (Vv > (int)Q.uv.zthresh[0]) {
                    const int qV = (int)(((uint32_t)Vv * Q.uv.iq[0] + Q.uv.bias[0]) >> QFIX) * Q.uv.q[0];
                    const int err = Vv - qV;
                    *v = (int16_t)(sign ? -qV : qV);
                    return (sign ? -err : err) >> 1;
                }
                *v = 0;
                return (sign ? -Vv : Vv) >> 1;
            };
            c[0][0] = (int16_t)(c[0][0] + ((7 * top[0] + 8 * left[0]) >> 3));
            const int e0 = qs(&c[0][0]);
            c[1][0] = (int16_t)(c[1][0] + ((7 * top[1] + 8 * e0) >> 3));
            const int e1 = qs(&c[1][0]);
            c[2][0] = (int16_t)(c[2][0] + ((7 * e0 + 8 * left[1]) >> 3));
            const int e2 = qs(&c[2][0]);
            c[3][0] = (int16_t)(c[3][0] + ((7 * e1 + 8 * e2) >> 3));
            const int e3 = qs(&c[3][0]);
            s_duv[m][ch][0] = (int8_t)e1;
            s_duv[m][ch][1] = (int8_t)e2;
            s_duv[m][ch][2] = (int8_t)e3;
        }
        __syncthreads();
        int D = 0, R = 0, cnt = 0;
        if (act) {
            s_cnz[m][n] = quantize_block(s_tmpc[m][n], s_lvuv[m][n], Q.uv);
            itransform(pred + off, s_tmpc[m][n], s_recuv[m] + off);
            for (int y = 0; y < 4; ++y)
                for (int x = 0; x < 4; ++x) {
                    const int d = s_in[16 + off + x + y * BPS] - s_recuv[m][off + x + y * BPS];
                    D += d * d;
                }
            for (int k = 1; k < 16; ++k) cnt += s_lvuv[m][n][k] != 0;
        }
        __syncthreads();
        if (act) {
            const int ctx = (by ? s_cnz[m][n - 2] : s_tnz[4 + 2 * ch + bx]) + (bx ? s_cnz[m][n - 1] : s_lnz[4 + 2 * ch + by]);
            R = rcost(lc, pr, s_fixed, s_ent, s_bands, 2, 0, ctx, s_lvuv[m][n]);
        }
        for (int o = 4; o; o >>= 1) {  // sums over the mode's 8 lanes
            D += __shfl_xor(D, o, 64);
            R += __shfl_xor(R, o, 64);
            cnt += __shfl_xor(cnt, o, 64);
        }
        if (act && n == 0) {
            if (m > 0 && cnt <= 2) R += 140 * 8;  // IsFlat(uv levels, 8, FLATNESS_LIMIT_UV)
            s_sc[m] = rd_score(R, kFixedCostsUV[m], D, 0, Q.lambda_uv);
        }
    }
    __syncthreads();
    if (l == 0) {
        int best = 0;
        for (int m = 1; m < 4; ++m)
            if (s_sc[m] < s_sc[best]) best = m;
        s_buv = best;
    }
    __syncthreads();
    IK_STAMP(4);

    // ---- outputs: reconstruction, the MB record, contexts, chroma errors ----
    const bool i4 = s_i4ok != 0;
    const int b16 = s_b16, buv = s_buv;
    for (int i = l; i < 256; i += 64) {
        const int y = i >> 4, x = i & 15;
        RY[(size_t)(16 * my + y) * W + 16 * mx + x] = i4 ? s_best4[y * BPS + x] : s_rec16[b16][y * BPS + x];
    }
    for (int i = l; i < 128; i += 64) {
        const int c = i >> 6, k = i & 63, y = k >> 3, x = k & 7;
        (c ? RV : RU)[(size_t)(8 * my + y) * (W / 2) + 8 * mx + x] = s_recuv[buv][y * BPS + 8 * c + x];
    }
    XMB& o = mbs[mb];
    for (int i = l; i < 16 * 16; i += 64) o.ac[i >> 4][i & 15] = i4 ? s_lv4[i >> 4][i & 15] : s_lv16[b16][1 + (i >> 4)][i & 15];
    for (int i = l; i < 8 * 16; i += 64) o.uv[i >> 4][i & 15] = s_lvuv[buv][i >> 4][i & 15];
    if (l < 16) {
        o.dc[l] = i4 ? 0 : s_lv16[b16][0][l];
        o.bmodes[l] = i4 ? s_modes4[l] : (uint8_t)b16;
    }
    if (l == 0) {
        o.ymode = i4 ? 4 : (uint8_t)b16;
        o.uvmode = (uint8_t)buv;
        o.seg = (uint8_t)sg;
        o.pad = 0;
        // the contexts after this MB (RecordTokens' nz, packed as BytesToNz + bit 25 = left DC)
        int tnz[9], lnz[9];
        for (int i = 0; i < 9; ++i) { tnz[i] = s_tnz[i]; lnz[i] = s_lnz[i]; }
        auto anynz = [](const int16_t* c) { int r = 0; for (int k = 0; k < 16; ++k) r |= c[k] != 0; return r; };
        if (!i4) tnz[8] = lnz[8] = anynz(s_lv16[b16][0]);
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) tnz[x] = lnz[y] = anynz(i4 ? s_lv4[x + 4 * y] : s_lv16[b16][1 + x + 4 * y]);
        for (int ch = 0; ch <= 2; ch += 2)
            for (int y = 0; y < 2; ++y)
                for (int x = 0; x < 2; ++x) tnz[4 + ch + x] = lnz[4 + ch + y] = anynz(s_lvuv[buv][ch * 2 + x + y * 2]);
        uint32_t nz = 0;
        nz |= (uint32_t)((tnz[0] << 12) | (tnz[1] << 13) | (tnz[2] << 14) | (tnz[3] << 15));
        nz |= (uint32_t)((tnz[4] << 18) | (tnz[5] << 19) | (tnz[6] << 22) | (tnz[7] << 23));
        nz |= (uint32_t)(tnz[8] << 24);
        nz |= (uint32_t)((lnz[0] << 3) | (lnz[1] << 7) | (lnz[2] << 11));
        nz |= (uint32_t)((lnz[4] << 17) | (lnz[6] << 21));
        nz |= (uint32_t)(lnz[8] << 25);
        nzs[mb] = nz;
        // StoreDiffusionErrors: [0..3] the top pair per channel (for the MB below), [4..7] the left pair
        int8_t* d = derrs + (size_t)mb * 8;
        for (int ch = 0; ch < 2; ++ch) {
            const int8_t* e = s_duv[buv][ch];
            const int8_t l1 = a.use_derr ? (int8_t)((3 * e[2]) >> 2) : 0;
            d[4 + ch * 2 + 0] = a.use_derr ? e[0] : 0;
            d[4 + ch * 2 + 1] = l1;
            d[ch * 2 + 0] = a.use_derr ? e[1] : 0;
            d[ch * 2 + 1] = a.use_derr ? (int8_t)(e[2] - l1) : 0;
        }
    }
    IK_STAMP(5);
}

// One wave per image: fold the epoch's token statistics in raster order, then refresh
// the probabilities and the level costs the next epoch's decisions use.
__global__ __launch_bounds__(64) void k_vp8x_stats(XArgs a, int k0, int k1) {
    const int img = blockIdx.x, l = threadIdx.x;
    const int nmb = a.mb_w * a.mb_h;
    const XMB* mbs = a.mbs + (size_t)img * nmb;
    const uint32_t* nzs = a.nz + (size_t)img * nmb;
    uint32_t* stats = a.stats + (size_t)img * 1056;
    uint8_t* pr = a.pr + (size_t)img * 1056;
    uint16_t* lc = a.lc + (size_t)img * kCostRows * kLevelTab;
    // the counters in LDS.  libwebp halves a counter pair when its total reaches 65534,
    // which makes the fold order-dependent; an epoch adds at most 25 blocks x 16
    // records per slot per MB, so when every total is below 65534 minus that bound no
    // counter can reach the halving point and the MBs fold in parallel (LDS atomics);
    // otherwise lane 0 walks them in raster order, staged in LDS.
    __shared__ uint32_t s_st[1056];
    __shared__ __attribute__((aligned(16))) XMB s_mb;
    __shared__ int s_serial;
    static_assert(sizeof(XMB) % 4 == 0, "XMB words");
    if (l == 0) s_serial = 0;
    __syncthreads();
    const uint32_t bound = (uint32_t)(k1 - k0) * 25u * 16u;
    for (int i = l; i < 1056; i += 64) {
        s_st[i] = stats[i];
        if ((s_st[i] >> 16) + bound >= 0xfffeu) s_serial = 1;
    }
    __syncthreads();
    auto ctx_of = [&](int k, int* t, int* lf) {
        const int mx = k % a.mb_w, my = k / a.mb_w;
        const uint32_t tnz = my ? nzs[k - a.mb_w] : 0u, lnz = mx ? nzs[k - 1] : 0u;
        const int tb[9] = {12, 13, 14, 15, 18, 19, 22, 23, 24}, lb[8] = {3, 7, 11, 15, 17, 19, 21, 23};
        for (int i = 0; i < 9; ++i) t[i] = (int)((tnz >> tb[i]) & 1u);
        for (int i = 0; i < 8; ++i) lf[i] = (int)((lnz >> lb[i]) & 1u);
        lf[8] = (int)((lnz >> 25) & 1u);
    };
    if (!s_serial) {
        uint32_t* st = s_st;
        for (int k = k0 + l; k < k1; k += 64) {
            int t[9], lf[9];
            ctx_of(k, t, lf);
            record_mb([st](uint32_t slot, int bit) { atomicAdd(st + slot, 0x00010000u + (uint32_t)bit); return bit; },
                      mbs[k], t, lf, [](int, uint32_t) {});
        }
        __syncthreads();
    } else {
        for (int k = k0; k < k1; ++k) {
            const uint32_t* src = (const uint32_t*)(mbs + k);
            for (int i = l; i < (int)(sizeof(XMB) / 4); i += 64) ((uint32_t*)&s_mb)[i] = src[i];
            __syncthreads();
            if (l == 0) {
                int t[9], lf[9];
                ctx_of(k, t, lf);
                record_mb([&](uint32_t slot, int bit) { return record_stats(bit, s_st + slot); }, s_mb, t, lf,
                          [](int, uint32_t) {});
            }
            __syncthreads();
        }
    }
    for (int i = l; i < 1056; i += 64) {
        stats[i] = s_st[i];
        pr[i] = (uint8_t)finalize_proba(s_st[i], i);
    }
    __syncthreads();
    for (int r = l; r < kCostRows; r += 64) level_cost_row(pr + r * 11, r % 3, lc + r * kLevelTab);
}

hipError_t launch_vp8x_mb(const XArgs& a, const int* list, int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_vp8x_mb, dim3(count, n), dim3(64), 0, s, a, list);
    return hipGetLastError();
}

hipError_t launch_vp8x_stats(const XArgs& a, int k0, int k1, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8x_stats, dim3(n), dim3(64), 0, s, a, k0, k1);
    return hipGetLastError();
}

}  // namespace vp8x
}  // namespace ik

#ifdef IK_VP8X_STAMPS
extern "C" int ik_vp8x_stamps(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ik::vp8x::g_vp8x_stamps), sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    unsigned long long z[32] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(ik::vp8x::g_vp8x_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
