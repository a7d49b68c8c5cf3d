// ik_vp8_analysis.hip -- libwebp's method-4 segment analysis on the GPU: the first
// stage of the reference's WebP coder (reference src/transform.rs:129-137 -> webp
// 0.3.1 -> libwebp WebPEncode; libwebp analysis_enc.c VP8EncAnalyze / MBAnalyze /
// AssignSegments), exact.  The rest of the segment set-up (quantisers by pow(),
// SimplifySegments, tree probabilities) is host arithmetic in ik_webp_gpu.cpp.
//
// k_vp8_analyze: one wave64 per macroblock, every image of the batch in one launch
// (grid.y = image).  The MB's source samples and its source neighbours (libwebp
// analyses against the source, never a reconstruction: VP8IteratorImport with a
// boundary buffer) are staged in LDS with the ImportBlock edge replication
// (clamped coordinates).  Lane = (mode, 4x4 block): 2 luma modes x 16 blocks +
// 2 chroma modes x 8 blocks = 48 lanes -- the analysis tries DC and TM only
// (MAX_INTRA16_MODE = MAX_UV_MODE = 2).  Each lane runs FTransform on its block's
// residual and bins the 16 coefficients as min(|c| >> 3, 31) into the mode's LDS
// histogram; a mode's alpha is 510 * last_non_zero / max_count (0 when the
// largest bin holds <= 1).  The MB keeps the largest luma and chroma alphas,
// mixes them 3:1 and inverts: alpha = clip(255 - ((3 a + uv + 2) >> 2)).
//
// k_vp8_kmeans: one workgroup per image: the 256-bin alpha histogram, libwebp's
// k-means (<= 6 iterations, 4 centres spread over the used range, ties to the
// lower centre), the per-MB segment (map[alpha]) and a per-image record (centres,
// weighted average, alpha sums) for the host.  Bytes: w*h*1.5 read per image
// (L2-resident neighbours), 3 B written per MB -- a few microseconds per batch.
#include <hip/hip_runtime.h>

#include "ik_vp8_gpu.h"

namespace ik {
namespace vp8 {

namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// libwebp FTransform_C (dsp/enc.c) of src - pred, 4x4, row pitch 4 in both
__device__ __forceinline__ void ftransform4(const int* d, int* out) {
    int tmp[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d0 = d[4 * i], d1 = d[4 * i + 1], d2 = d[4 * i + 2], d3 = d[4 * i + 3];
        const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
        tmp[0 + 4 * i] = (a0 + a1) * 8;
        tmp[1 + 4 * i] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
        tmp[2 + 4 * i] = (a0 - a1) * 8;
        tmp[3 + 4 * i] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a0 = tmp[0 + i] + tmp[12 + i], a1 = tmp[4 + i] + tmp[8 + i];
        const int a2 = tmp[4 + i] - tmp[8 + i], a3 = tmp[0 + i] - tmp[12 + i];
        out[0 + i] = (a0 + a1 + 7) >> 4;
        out[4 + i] = ((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0);
        out[8 + i] = (a0 - a1 + 7) >> 4;
        out[12 + i] = (a3 * 2217 - a2 * 5352 + 51000) >> 16;
    }
}

}  // namespace

// Per MB: alpha[] (final mixed susceptibility, 0..255) and uva[] (best chroma
// alpha, unclipped, as MBAnalyze accumulates it).
__global__ __launch_bounds__(64) void k_vp8_analyze(const uint8_t* __restrict__ yuv, size_t yuv_stride, int w,
                                                    int h, int mb_w, int mb_h, uint8_t* __restrict__ alpha,
                                                    uint16_t* __restrict__ uva) {
    __shared__ uint8_t s_src[3][16][16];  // Y 16x16; U, V 8x8 (in the first 8 rows / columns)
    __shared__ int s_left[3][16], s_top[3][16], s_tl[3];
    __shared__ int s_hist[4][32];  // luma DC, luma TM, chroma DC, chroma TM
    const int mb = blockIdx.x, img = blockIdx.y, l = threadIdx.x;
    const int mx = mb % mb_w, my = mb / mb_w;
    const int uw = (w + 1) >> 1, uh = (h + 1) >> 1;
    const uint8_t* Y = yuv + (size_t)img * yuv_stride;
    const uint8_t* U = Y + (size_t)w * h;
    const uint8_t* V = U + (size_t)uw * uh;
    // stage: 256 + 2 x 64 source samples (6 per lane), the neighbours (clamped
    // coordinates = ImportBlock / ImportLine's replication of the last sample)
    for (int i = l; i < 384; i += 64) {
        if (i < 256) {
            const int y = i >> 4, x = i & 15;
            s_src[0][y][x] = Y[(size_t)clampi(16 * my + y, 0, h - 1) * w + clampi(16 * mx + x, 0, w - 1)];
        } else {
            const int c = (i - 256) >> 6, k = (i - 256) & 63, y = k >> 3, x = k & 7;
            const uint8_t* P = c ? V : U;
            s_src[1 + c][y][x] = P[(size_t)clampi(8 * my + y, 0, uh - 1) * uw + clampi(8 * mx + x, 0, uw - 1)];
        }
    }
    if (l < 16) {
        if (mx) s_left[0][l] = Y[(size_t)clampi(16 * my + l, 0, h - 1) * w + 16 * mx - 1];
        if (my) s_top[0][l] = Y[(size_t)(16 * my - 1) * w + clampi(16 * mx + l, 0, w - 1)];
    } else if (l < 32) {
        const int c = (l - 16) >> 3, k = (l - 16) & 7;
        const uint8_t* P = c ? V : U;
        if (mx) s_left[1 + c][k] = P[(size_t)clampi(8 * my + k, 0, uh - 1) * uw + 8 * mx - 1];
        if (my) s_top[1 + c][k] = P[(size_t)(8 * my - 1) * uw + clampi(8 * mx + k, 0, uw - 1)];
    } else if (l < 35) {
        const int c = l - 32;
        if (mx && my) {
            s_tl[c] = c == 0 ? Y[(size_t)(16 * my - 1) * w + 16 * mx - 1]
                             : (c == 1 ? U : V)[(size_t)(8 * my - 1) * uw + 8 * mx - 1];
        }
    }
    for (int i = l; i < 128; i += 64) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    if (l < 48) {
        const bool luma = l < 32;
        const int m = luma ? l >> 4 : (l - 32) >> 3;           // 0 = DC, 1 = TM
        const int b = luma ? l & 15 : (l - 32) & 7;
        const int c = luma ? 0 : 1 + (b >> 2);                  // plane
        const int bx = luma ? 4 * (b & 3) : 4 * (b & 1), by = luma ? 4 * (b >> 2) : 4 * ((b >> 1) & 1);
        const int size = luma ? 16 : 8, shift = luma ? 5 : 4;
        const bool hl = mx > 0, ht = my > 0;
        // DC (DCMode: both / top only / left only: doubled / none: 128)
        int dc = 0x80;
        if (hl || ht) {
            int s = 0;
            for (int k = 0; k < size; ++k) s += (ht ? s_top[c][k] : 0) + (hl ? s_left[c][k] : 0);
            if (!(hl && ht)) s += s;
            dc = (s + (1 << (shift - 1))) >> shift;
        }
        int d[16], out[16];
#pragma unroll
        for (int y = 0; y < 4; ++y) {
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                int p;
                if (m == 0) {
                    p = dc;
                } else if (hl && ht) {  // TrueMotion
                    p = clampi(s_left[c][by + y] + s_top[c][bx + x] - s_tl[c], 0, 255);
                } else if (hl) {        // no top: HorizontalPred
                    p = s_left[c][by + y];
                } else if (ht) {        // no left: VerticalPred
                    p = s_top[c][bx + x];
                } else {
                    p = 129;
                }
                d[4 * y + x] = (int)s_src[c][by + y][bx + x] - p;
            }
        }
        ftransform4(d, out);
        const int hh = (luma ? 0 : 2) + m;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int a = out[k] < 0 ? -out[k] : out[k];
            atomicAdd(&s_hist[hh][min(a >> 3, 31)], 1);
        }
    }
    __syncthreads();
    if (l < 4) {  // GetAlpha of histogram l
        int maxv = 0, last = 1;
        for (int k = 0; k < 32; ++k) {
            const int v = s_hist[l][k];
            if (v > 0) {
                maxv = v > maxv ? v : maxv;
                last = k;
            }
        }
        s_hist[l][0] = maxv > 1 ? 510 * last / maxv : 0;  // (each lane reads only its own row)
    }
    __syncthreads();
    if (l == 0) {
        const int a16 = max(s_hist[0][0], s_hist[1][0]), auv = max(s_hist[2][0], s_hist[3][0]);
        const int mixed = (3 * a16 + auv + 2) >> 2;
        const size_t o = (size_t)img * mb_w * mb_h + mb;
        alpha[o] = (uint8_t)clampi(255 - mixed, 0, 255);
        uva[o] = (uint16_t)auv;
    }
}

// One workgroup per image: AssignSegments' k-means (analysis_enc.c).
__global__ __launch_bounds__(256) void k_vp8_kmeans(const uint8_t* __restrict__ alpha, const uint16_t* __restrict__ uva,
                                                    int nmb, uint8_t* __restrict__ seg, SegRecord* __restrict__ rec) {
    __shared__ int s_h[256];
    __shared__ int s_map[256];
    __shared__ unsigned long long s_sum[2][256];
    const int img = blockIdx.x, t = threadIdx.x;
    const uint8_t* A = alpha + (size_t)img * nmb;
    const uint16_t* UV = uva + (size_t)img * nmb;
    s_h[t] = 0;
    s_map[t] = 0;
    __syncthreads();
    unsigned long long sa = 0, su = 0;
    for (int i = t; i < nmb; i += 256) {
        const int a = A[i];
        atomicAdd(&s_h[a], 1);
        sa += (unsigned)a;
        su += UV[i];
    }
    s_sum[0][t] = sa;
    s_sum[1][t] = su;
    __syncthreads();
    if (t == 0) {
        unsigned long long ta = 0, tu = 0;
        for (int k = 0; k < 256; ++k) {
            ta += s_sum[0][k];
            tu += s_sum[1][k];
        }
        constexpr int nb = 4;
        int min_a = 0, max_a = 255;
        while (min_a <= 255 && s_h[min_a] == 0) ++min_a;
        while (max_a > min_a && s_h[max_a] == 0) --max_a;
        const int range_a = max_a - min_a;
        int centers[nb];
        for (int k = 0, n = 1; k < nb; ++k, n += 2) centers[k] = min_a + (n * range_a) / (2 * nb);
        int weighted_average = 0;
        for (int it = 0; it < 6; ++it) {
            int accum[nb] = {0, 0, 0, 0}, dist[nb] = {0, 0, 0, 0};
            int n = 0;
            for (int a = min_a; a <= max_a; ++a) {
                if (s_h[a]) {
                    while (n + 1 < nb && abs(a - centers[n + 1]) < abs(a - centers[n])) ++n;
                    s_map[a] = n;
                    dist[n] += a * s_h[a];
                    accum[n] += s_h[a];
                }
            }
            int displaced = 0, total = 0;
            weighted_average = 0;
            for (int k = 0; k < nb; ++k) {
                if (accum[k]) {
                    const int nc = (dist[k] + accum[k] / 2) / accum[k];
                    displaced += abs(centers[k] - nc);
                    centers[k] = nc;
                    weighted_average += nc * accum[k];
                    total += accum[k];
                }
            }
            weighted_average = (weighted_average + total / 2) / total;
            if (displaced < 5) break;
        }
        SegRecord r;
        for (int k = 0; k < nb; ++k) r.centers[k] = centers[k];
        r.mid = weighted_average;
        r.nmb = nmb;
        r.alpha_sum = ta;
        r.uv_alpha_sum = tu;
        rec[img] = r;
    }
    __syncthreads();
    for (int i = t; i < nmb; i += 256) seg[(size_t)img * nmb + i] = (uint8_t)s_map[A[i]];
}

hipError_t launch_vp8_analysis(const uint8_t* yuv, size_t yuv_stride, int n, int w, int h, uint8_t* alpha,
                               uint16_t* uva, uint8_t* seg, SegRecord* rec, hipStream_t s) {
    const int mb_w = (w + 15) >> 4, mb_h = (h + 15) >> 4, nmb = mb_w * mb_h;
    if (n < 1 || nmb < 1 || n > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_vp8_analyze, dim3(nmb, n), dim3(64), 0, s, yuv, yuv_stride, w, h, mb_w, mb_h, alpha, uva);
    hipLaunchKernelGGL(k_vp8_kmeans, dim3(n), dim3(256), 0, s, alpha, uva, nmb, seg, rec);
    return hipGetLastError();
}

}  // namespace vp8
}  // namespace ik
