// Dev probe (not product code): how fast can the exact vertical Lanczos3 8x pass run
// when it is written as a periodic sweep -- 6 rotating accumulators fixed at compile
// time, 8 source rows per step, every row into all six open output rows, no mask
// tests, no accumulator shifts -- against the fused kernel's vertical pass
// (lib_ab/nohorz.so, tools/resize_ab.py).  Same strips (2048 B per 256 lanes, 8 B per
// lane), same bands, same prefetch ring; the completed rows go to LDS and a checksum
// keeps the work alive.  64 x 4096^2 RGBA8 -> 512 rows.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize tools/vprobe.hip -o tools/vprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang fp contract(off)

constexpr int S = 4096, RB = S * 4, OH = 512, NSTRIP = 9, STRIPB = 2048;

__device__ __forceinline__ int lds_idx(int i) { return i + ((i >> 5) << 2); }

template <int BAND>
__global__ __launch_bounds__(256) void k_vprobe(const uint8_t* __restrict__ src, const float* __restrict__ wtab,
                                                float* __restrict__ out, int nimg) {
    __shared__ __attribute__((aligned(16))) float lds[2 * 2304];
    const int nb = OH / BAND;
    const int L = blockIdx.x;
    const int img = L / (NSTRIP * nb);
    const int rem = L - img * NSTRIP * nb;
    const int band = rem / NSTRIP, strip = rem - band * NSTRIP;
    const int sb = strip * 1792;  // strips overlap like the fused kernel's (9 x 2048 B over 16384 B)
    const int mybyte = sb + 8 * (int)threadIdx.x;
    const int voff = mybyte < RB ? mybyte : 0;
    const unsigned long long base = (unsigned long long)(src + (size_t)img * S * RB);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(RB * S), 0x00020000);
    auto ld = [&](int row) -> uint2 {
        row = row < 0 ? 0 : (row > S - 1 ? S - 1 : row);
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, row * RB, 0);
        return make_uint2(v[0], v[1]);
    };
    // 48 taps: uniform interior weights (scalar loads)
    float w[48];
#pragma unroll
    for (int i = 0; i < 48; ++i) w[i] = wtab[i];

    const int oy0 = band * BAND;
    const int t0 = oy0, t1 = oy0 + BAND + 5;  // step t covers rows 8t-20 .. 8t-13
    float acc[6][8];
#pragma unroll
    for (int d = 0; d < 6; ++d)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[d][q] = 0.0f;
    uint2 b0[8], b1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = ld(8 * t0 - 20 + j);
#pragma unroll
    for (int j = 0; j < 8; ++j) b1[j] = ld(8 * (t0 + 1) - 20 + j);
    float* my = lds + lds_idx(8 * (int)threadIdx.x);
    float chk = 0.0f;

    // step with phase U (slot of the output that starts at this step = U)
    auto step = [&](auto UC, int t, uint2 (&cur)[8]) {
        constexpr int U = decltype(UC)::value;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint2 raw = cur[j];
            float p[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                p[q] = (float)((raw.x >> (8 * q)) & 0xffu);
                p[4 + q] = (float)((raw.y >> (8 * q)) & 0xffu);
            }
            // output started e steps ago sits in slot (U - e) mod 6 and takes tap 8e + j
#pragma unroll
            for (int e = 5; e >= 0; --e) {
                constexpr int dummy = 0;
                (void)dummy;
                const int slot = ((U - e) % 6 + 6) % 6;
                const float wt = w[8 * e + j];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float prod = p[q] * wt;
                    if (e == 0 && j == 0) acc[slot][q] = prod;
                    else acc[slot][q] = acc[slot][q] + prod;
                }
            }
            cur[j] = ld(8 * (t + 2) - 20 + j);
        }
        // the output started 5 steps ago is complete
        constexpr int done = ((U - 5) % 6 + 6) % 6;
        float* o = my + ((t & 1) ? 2304 : 0);
        *reinterpret_cast<float4*>(o) = make_float4(acc[done][0], acc[done][1], acc[done][2], acc[done][3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(acc[done][4], acc[done][5], acc[done][6], acc[done][7]);
        chk += acc[done][0];
    };
    for (int t = t0; t < t1; t += 6) {
        step(std::integral_constant<int, 0>(), t, b0);
        if (t + 1 < t1) step(std::integral_constant<int, 1>(), t + 1, b1);
        if (t + 2 < t1) step(std::integral_constant<int, 2>(), t + 2, b0);
        if (t + 3 < t1) step(std::integral_constant<int, 3>(), t + 3, b1);
        if (t + 4 < t1) step(std::integral_constant<int, 4>(), t + 4, b0);
        if (t + 5 < t1) step(std::integral_constant<int, 5>(), t + 5, b1);
    }
    __syncthreads();
    chk += lds[(threadIdx.x * 37) % 4608];
    if (chk == 1234.5f) out[L * 256 + threadIdx.x] = chk;
}

int main(int argc, char** argv) {
    const int nimg = 64;
    uint8_t* src;
    float *wt, *out;
    if (hipMalloc(&src, (size_t)nimg * S * RB) != hipSuccess) return 1;
    if (argc > 1) {  // random bytes (one frame's worth, copied to every frame)
        std::vector<uint8_t> h((size_t)S * RB);
        unsigned x = 12345;
        for (auto& b : h) { x = x * 1664525u + 1013904223u; b = (uint8_t)(x >> 24); }
        for (int i = 0; i < nimg; ++i) (void)hipMemcpy(src + (size_t)i * S * RB, h.data(), h.size(), hipMemcpyHostToDevice);
    } else {
        (void)hipMemset(src, 0x5a, (size_t)nimg * S * RB);
    }
    float hw[48];
    for (int i = 0; i < 48; ++i) hw[i] = 0.01f * (i % 7) - 0.013f;
    (void)hipMalloc(&wt, sizeof(hw));
    (void)hipMemcpy(wt, hw, sizeof(hw), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, (size_t)nimg * NSTRIP * 64 * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int band : {32, 64}) {
        const int grid = nimg * NSTRIP * (OH / band);
        float best = 1e9f;
        for (int r = 0; r < 6; ++r) {
            (void)hipEventRecord(e0);
            if (band == 32) hipLaunchKernelGGL(k_vprobe<32>, dim3(grid), dim3(256), 0, 0, src, wt, out, nimg);
            else hipLaunchKernelGGL(k_vprobe<64>, dim3(grid), dim3(256), 0, 0, src, wt, out, nimg);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r && ms < best) best = ms;
        }
        printf("vprobe band=%d: %.4f ms per %d frames (%.0f GB/s of 4*W*H)\n", band, best, nimg,
               (double)nimg * S * RB / (best * 1e-3) / 1e9);
    }
    return 0;
}
