// Dev probe: sustained f32 VALU rate on gfx950 for the resize kernel's tap pattern
// (separately rounded mul then add, many independent accumulators), unpacked and
// packed (float2 -> v_pk_mul_f32 / v_pk_add_f32), at 1..8 waves per SIMD.
// Prints wave-instructions per SIMD per ns (= shader GHz / cycles per instruction).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
typedef float f2 __attribute__((ext_vector_type(2)));

template <int ACC>
__global__ __launch_bounds__(256) void k_scalar(float* out, int iters, float w0) {
    const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    float acc[ACC], p[8];
    for (int i = 0; i < ACC; ++i) acc[i] = 0.f;
    for (int i = 0; i < 8; ++i) p[i] = (float)((threadIdx.x + i) & 255);
    float w = w0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < ACC / 8; ++d)
            { const float wd = w + 0.01f * d;
#pragma unroll
            for (int q = 0; q < 8; ++q) { float pr = p[q] * wd; acc[d * 8 + q] = acc[d * 8 + q] + pr; } }
        w = w * 0.999f;
    }
    float s = 0.f;
    for (int i = 0; i < ACC; ++i) s += acc[i];
    if (s == 12345.f) out[threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // shader clock: s_memtime ticks per 100 MHz s_memrealtime tick
        const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
        reinterpret_cast<double*>(out)[64] = (double)(t1 - t0) / (double)(r1 - r0) * 0.1;
    }
}

template <int ACC>
__global__ __launch_bounds__(256) void k_packed(float* out, int iters, float w0) {
    f2 acc[ACC / 2], p[4];
    for (int i = 0; i < ACC / 2; ++i) acc[i] = (f2){0.f, 0.f};
    for (int i = 0; i < 4; ++i) p[i] = (f2){(float)((threadIdx.x + 2 * i) & 255), (float)((threadIdx.x + 2 * i + 1) & 255)};
    float w = w0;
    for (int it = 0; it < iters; ++it) {
        f2 ww = (f2){w, w};
#pragma unroll
        for (int d = 0; d < ACC / 8; ++d)
            { const f2 wd = ww + 0.01f * d;
#pragma unroll
            for (int q = 0; q < 4; ++q) { f2 pr = p[q] * wd; acc[d * 4 + q] = acc[d * 4 + q] + pr; } }
        w = w * 0.999f;
    }
    float s = 0.f;
    for (int i = 0; i < ACC / 2; ++i) s += acc[i].x + acc[i].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 4096);
    hipMemset(out, 0, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = 256 * wps;  // 256 CUs x wps workgroups of 4 waves = wps waves per SIMD
        for (int pk = 0; pk < 2; ++pk) {
            float best = 1e30f;
            for (int r = 0; r < 4; ++r) {
                hipEventRecord(e0);
                if (pk) hipLaunchKernelGGL(k_packed<48>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f);
                else hipLaunchKernelGGL(k_scalar<48>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            // tap instructions per wave: iters * 48 * 2 (unpacked) or iters * 24 * 2 (packed)
            const double winstr = (double)blocks * 4 * iters * (pk ? 48.0 : 96.0);
            const double per_simd_ns = winstr / 1024.0 / (best * 1e6);
            double ghz = 0;
            hipMemcpy(&ghz, reinterpret_cast<double*>(out) + 64, 8, hipMemcpyDeviceToHost);
            printf("[clock %.3f GHz] ", pk ? 0.0 : ghz);
            printf("waves/SIMD=%d %s: %.3f ms, %.3f wave-instr/SIMD/ns, lane-flop %.1f TF\n", wps,
                   pk ? "packed  " : "unpacked", best, per_simd_ns, (double)blocks * 256 * iters * 96.0 / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
