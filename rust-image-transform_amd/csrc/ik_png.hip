// ik_png.hip -- gfx950 kernels of the GPU PNG decoder (decode_image on a PNG:
// reference src/transform.rs:31 -> image 0.25.8 -> png 0.18: zlib inflate of the
// IDAT stream, then per-row unfiltering).  Host side: ik_png_decode.cpp; the
// DEFLATE core and the algorithm are in ik_inflate.h.
//
//   k_png_find      one wave per (chunk, image): the first plausible dynamic
//                   block header in the chunk (64 bit offsets per wave step)
//   k_png_inflate   one thread per decoder lane: whole blocks from its start to
//                   the next lane's start; count pass (lengths) or emit pass
//                   (u16 symbols with window markers).  Root Huffman tables live
//                   in LDS per thread, subtables in a per-lane global area.
//   k_png_resolve   u16 symbols -> the filtered bytes of every row, 16 per thread,
//                   markers followed to their source; rows land 16-B aligned in
//                   the destination image (pitched) and filter types in ft[]
//   k_png_unfilter  PNG row filters (None/Sub/Up/Average/Paeth) in place.  A row
//                   depends on the row above and on its own left bytes, so it is a
//                   skewed wavefront: lane = row (64 rows per wave, one band),
//                   16-byte chunks, lane l works on chunk s - l at step s and hands
//                   its unfiltered chunk to lane l+1 by a DPP wave shift.  The
//                   workgroup's waves take consecutive bands; a band's first row
//                   reads the previous band's last row from memory once the
//                   previous wave has published it (LDS progress counter,
//                   workgroup-scope release/acquire).
#include "ik_inflate.h"
#include "ik_internal.h"
#include "ik_png.h"

namespace ik {

// ---- find ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx,
                                                 int nchunks_total, uint64_t chunk_bits, int64_t* cand) {
    __shared__ uint8_t s_tab[64 * 128];  // per lane: code-length code lookup (symbol | length << 5)
    const int g = blockIdx.x;
    if (g >= nchunks_total) return;
    const int im = chunk_img[g];
    const int c = chunk_idx[g];
    const PngImgDev I = imgs[im];
    const uint64_t b0 = I.bit0 + (uint64_t)c * chunk_bits;
    const uint64_t b1 = b0 + chunk_bits < I.nbits ? b0 + chunk_bits : I.nbits;
    if (c == 0) {
        if (threadIdx.x == 0) cand[g] = (int64_t)I.bit0;
        return;
    }
    const int lane = threadIdx.x;
    int64_t found = -1;
    for (uint64_t base = b0; base < b1; base += 64) {
        const uint64_t p = base + lane;
        bool ok = false;
        if (p < b1) {
            // quick filters on 17 header bits, then the precode's completeness,
            // then the full header parse (rare)
            const uint64_t wi = p >> 5;
            const uint64_t v = ((uint64_t)I.words[wi] | ((uint64_t)I.words[wi + 1] << 32)) >> (p & 31);
            const uint32_t h = (uint32_t)v;
            if (((h >> 1) & 3u) == 2u && ((h >> 3) & 31u) <= 29u && ((h >> 8) & 31u) <= 29u) {
                const int ncode = (int)((h >> 13) & 15u) + 4;
                // precode lengths: up to 57 bits from bit 17
                const uint64_t q = p + 17;
                const uint64_t qi = q >> 5;
                const uint32_t sh = (uint32_t)(q & 31);
                const uint64_t lo = (uint64_t)I.words[qi] | ((uint64_t)I.words[qi + 1] << 32);
                const uint64_t hi = (uint64_t)I.words[qi + 2];
                const uint64_t bits = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
                int kraft = 0, nz = 0;
                for (int i = 0; i < ncode; ++i) {
                    const int l = (int)((bits >> (3 * i)) & 7u);
                    if (l) { kraft += 128 >> l; ++nz; }
                }
                if (kraft == 128 && nz)
                    ok = infl::dynamic_header_ok(I.words, I.nbits, p, h, bits, s_tab + 128 * lane);
            }
        }
        const unsigned long long m = __ballot(ok);
        if (m) {
            found = (int64_t)(base + (uint64_t)__ffsll((long long)m) - 1);
            break;
        }
    }
    if (lane == 0) cand[g] = found;
}

// ---- inflate ------------------------------------------------------------------------
template <bool EMIT>
__global__ __launch_bounds__(kPngInflateThreads) void k_png_inflate(const PngImgDev* imgs, const PngLaneDev* lanes,
                                                                     int nlanes, uint16_t* sub_ws,
                                                                     infl::LaneResult* res) {
    __shared__ uint16_t s_root[kPngInflateThreads * (infl::kLitRootN + infl::kDistRootN)];
    const int t = blockIdx.x * kPngInflateThreads + threadIdx.x;
    if (t >= nlanes) return;
    const PngLaneDev L = lanes[t];
    const PngImgDev I = imgs[L.img];
    uint16_t* lroot = s_root + threadIdx.x * (infl::kLitRootN + infl::kDistRootN);
    uint16_t* droot = lroot + infl::kLitRootN;
    uint16_t* lsub = sub_ws + (size_t)L.slot * (infl::kLitSub + infl::kDistSub);
    uint16_t* dsub = lsub + infl::kLitSub;
    infl::LaneResult r;
    const uint64_t cap = EMIT ? I.raw_total - (uint64_t)L.obase : I.raw_total;
    infl::decode_lane<EMIT>(I.words, I.nbits, L.start, L.stop, lroot, lsub, droot, dsub, I.u16,
                            EMIT ? L.obase : (L.first ? 0 : -1), cap, r);
    res[t] = r;
}

// ---- resolve ------------------------------------------------------------------------
// thread = (16-byte chunk of a row, row, image); grid.y over rows of all images via
// a row table (image, row)
__global__ __launch_bounds__(256) void k_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows,
                                                     int* err) {
    const int rr = blockIdx.y * 65535 + blockIdx.x;  // row of the batch
    if (rr >= nrows) return;
    const int2 ir = rows[rr];
    const PngImgDev I = imgs[ir.x];
    const int y = ir.y;
    const int64_t rs = (int64_t)y * (I.rowbytes + 1);  // filter byte of row y
    if (threadIdx.x == 0) {
        const int v = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, rs);
        I.ft[y] = (uint8_t)(v < 0 ? 255 : v);
        if (v < 0 || v > 4) atomicOr(err + ir.x, 1);
    }
    for (int x0 = threadIdx.x * 16; x0 < I.rowbytes; x0 += 256 * 16) {
        const int64_t e0 = rs + 1 + x0;
        // 16 u16 symbols from 9 aligned dwords (the u16 buffer is padded)
        const uint32_t* w = reinterpret_cast<const uint32_t*>(I.u16) + (e0 >> 1);
        uint32_t d[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = w[k];
        const int odd = (int)(e0 & 1);
        uint32_t o[4] = {0, 0, 0, 0};
        bool any_marker = false;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t v = odd ? (d[(i + 1) >> 1] >> (16 * ((i + 1) & 1))) & 0xFFFFu
                                   : (d[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            any_marker |= v >= 256u;
            o[i >> 2] |= (v & 255u) << (8 * (i & 3));
        }
        if (any_marker) {  // window markers: follow them to the byte they name
            const int n = I.rowbytes - x0 < 16 ? I.rowbytes - x0 : 16;
#pragma unroll 1
            for (int i = 0; i < n; ++i) {
                const uint32_t v = I.u16[e0 + i];
                if (v < 256u) continue;
                const int rv = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, e0 + i);
                if (rv < 0) atomicOr(err + ir.x, 2);
                o[i >> 2] = (o[i >> 2] & ~(255u << (8 * (i & 3)))) | (((uint32_t)rv & 255u) << (8 * (i & 3)));
            }
        }
        uint8_t* dp = I.dst + (size_t)y * I.pitch + x0;
        *reinterpret_cast<uint4*>(dp) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// ---- unfilter -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t lane0) {
    // lane l gets lane l-1's v; lane 0 gets lane0 (DPP wave_shr:1, bound_ctrl off)
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 255u; }

template <int BPP>
__global__ __launch_bounds__(kPngUnfilterThreads) void k_png_unfilter(const PngImgDev* imgs) {
    constexpr int NW = kPngUnfilterThreads / 64;
    __shared__ unsigned s_prog[NW];
    const PngImgDev I = imgs[blockIdx.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < NW) s_prog[threadIdx.x] = 0;
    __syncthreads();
    const int nch = (I.rowbytes + 15) >> 4;
    const int nbands = (I.H + 63) >> 6;
    const int pw = (wave + NW - 1) % NW;  // the wave that owns the previous band
    int m = 0;                            // this wave's band sequence number
    for (int band = wave; band < nbands; band += NW, ++m) {
        const int y = band * 64 + lane;
        const bool live = y < I.H;
        uint8_t* row = I.dst + (size_t)(live ? y : 0) * I.pitch;
        const uint32_t ft = live ? I.ft[y] : 0u;
        const uint8_t* above = band > 0 ? I.dst + (size_t)(band * 64 - 1) * I.pitch : nullptr;
        // the previous band's sequence number in its wave
        const int pm = band > 0 ? (band - 1) / NW : 0;
        uint32_t cur[4] = {0, 0, 0, 0}, up[4] = {0, 0, 0, 0};
        uint32_t prevcur[4] = {0, 0, 0, 0}, prevup[4] = {0, 0, 0, 0};  // last chunk (left context)
        uint32_t raw[4] = {0, 0, 0, 0};
        const int steps = nch + 63;
        for (int s = 0; s < steps; ++s) {
            const int j = s - lane;
            // up chunk: lane l-1's result of the previous step; lane 0: previous band
            uint32_t from_above[4] = {0, 0, 0, 0};
            if (lane == 0 && above && j < nch) {
                const unsigned need = (unsigned)(pm * nch + j + 1);
                while (__hip_atomic_load(&s_prog[pw], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
                    __builtin_amdgcn_s_sleep(1);
                // the other wave's stores: read through to L2 (sc1), not a stale L1 line
                const unsigned* ap = reinterpret_cast<const unsigned*>(above + 16 * j);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    from_above[k] = __hip_atomic_load(ap + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            uint32_t nup[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) nup[k] = wave_shr1(cur[k], from_above[k]);
            const bool act = live && j >= 0 && j < nch;
            if (act) {
                const uint4 u = *reinterpret_cast<const uint4*>(row + 16 * j);
                raw[0] = u.x; raw[1] = u.y; raw[2] = u.z; raw[3] = u.w;
#pragma unroll
                for (int k = 0; k < 4; ++k) { prevup[k] = up[k]; up[k] = nup[k]; prevcur[k] = cur[k]; }
                if (j == 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) { prevup[k] = 0; prevcur[k] = 0; }
                }
                uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    // a = left, b = up, c = up-left (bytes BPP back; from the previous chunk at its start)
                    const uint32_t a = i >= BPP ? ((o[(i - BPP) >> 2] >> (8 * ((i - BPP) & 3))) & 255u)
                                                : byte_of(prevcur, 16 + i - BPP);
                    const uint32_t b = byte_of(up, i);
                    const uint32_t c = i >= BPP ? byte_of(up, i - BPP) : byte_of(prevup, 16 + i - BPP);
                    const int d1 = (int)b - (int)c, d2 = (int)a - (int)c;
                    const int pa = d1 < 0 ? -d1 : d1, pb = d2 < 0 ? -d2 : d2, pc = (d1 + d2) < 0 ? -(d1 + d2) : (d1 + d2);
                    const uint32_t paeth = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    const uint32_t pred = ft == 1 ? a : ft == 2 ? b : ft == 3 ? ((a + b) >> 1) : ft == 4 ? paeth : 0u;
                    const uint32_t v = (byte_of(raw, i) + pred) & 255u;
                    o[i >> 2] |= v << (8 * (i & 3));
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = o[k];
                *reinterpret_cast<uint4*>(row + 16 * j) = make_uint4(o[0], o[1], o[2], o[3]);
            }
            // the band's last row publishes its chunks for the next band's first row
            if (lane == 63 && act) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the chunk's store has reached L2
                __hip_atomic_store(&s_prog[wave], (unsigned)(m * nch + j + 1), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        // rows past the image (last band): publish completion so no waiter stalls
        if (lane == 63 && !live)
            __hip_atomic_store(&s_prog[wave], (unsigned)((m + 1) * nch), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// ---- launchers --------------------------------------------------------------------
hipError_t launch_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx, int n,
                           uint64_t chunk_bits, int64_t* cand, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_find, dim3(n), dim3(64), 0, s, imgs, chunk_img, chunk_idx, n, chunk_bits, cand);
    return hipGetLastError();
}

hipError_t launch_png_inflate(bool emit, const PngImgDev* imgs, const PngLaneDev* lanes, int n, uint16_t* sub_ws,
                              infl::LaneResult* res, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((n + kPngInflateThreads - 1) / kPngInflateThreads);
    if (emit)
        hipLaunchKernelGGL(k_png_inflate<true>, grid, dim3(kPngInflateThreads), 0, s, imgs, lanes, n, sub_ws, res);
    else
        hipLaunchKernelGGL(k_png_inflate<false>, grid, dim3(kPngInflateThreads), 0, s, imgs, lanes, n, sub_ws, res);
    return hipGetLastError();
}

hipError_t launch_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows, int* err, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    const dim3 grid(nrows < 65535 ? nrows : 65535, (nrows + 65534) / 65535);
    hipLaunchKernelGGL(k_png_resolve, grid, dim3(256), 0, s, imgs, rows, nrows, err);
    return hipGetLastError();
}

hipError_t launch_png_unfilter(const PngImgDev* imgs, int n, int bpp, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid(n), block(kPngUnfilterThreads);
    switch (bpp) {
    case 1: hipLaunchKernelGGL(k_png_unfilter<1>, grid, block, 0, s, imgs); break;
    case 2: hipLaunchKernelGGL(k_png_unfilter<2>, grid, block, 0, s, imgs); break;
    case 3: hipLaunchKernelGGL(k_png_unfilter<3>, grid, block, 0, s, imgs); break;
    case 4: hipLaunchKernelGGL(k_png_unfilter<4>, grid, block, 0, s, imgs); break;
    case 6: hipLaunchKernelGGL(k_png_unfilter<6>, grid, block, 0, s, imgs); break;
    case 8: hipLaunchKernelGGL(k_png_unfilter<8>, grid, block, 0, s, imgs); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace ik
