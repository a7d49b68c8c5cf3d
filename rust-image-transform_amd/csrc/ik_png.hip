// ik_png.hip -- gfx950 kernels of the GPU PNG decoder (decode_image on a PNG:
// reference src/transform.rs:31 -> image 0.25.8 -> png 0.18: zlib inflate of the
// IDAT stream, then per-row unfiltering).  Host side: ik_png_decode.cpp; the
// DEFLATE core and the algorithm are in ik_inflate.h.
//
//   k_png_find      one wave per (chunk, image): the first plausible dynamic
//                   block header in the chunk (2,048 bit offsets per wave step)
//   k_png_decode    one thread per decoder lane: whole blocks from its start to
//                   the next lane's start -> the lane's token stream and output
//                   length.  Code tables in LDS per thread (192 B), input through
//                   an LDS ring filled by LDS-DMA (128 B per thread)
//   k_png_wave      one wave per decoder lane of the wave decoder (ik_png_wave.h):
//                   64 self-synchronising sub-lanes per block window -> token
//                   pieces, their piece table and the lane's expand-unit records
//   k_png_units     the expand units' offset, unit -> lane and page tables
//   k_png_expand8   one wave per expand unit (or per lane of the lane decoder):
//                   tokens -> u16 symbols (bytes, window markers) at the unit's
//                   output offset, 512 tokens per step, literals by a wave prefix
//                   sum, copies in token order; status and clock ticks / 1024 per
//                   unit (status[2 t], [2 t + 1])
//   k_png_resolve   u16 symbols -> the filtered bytes of every row, 16 per thread,
//                   markers followed to their source; rows land 16-B aligned in
//                   the destination image (pitched) and filter types in ft[]
//   k_png_unfilter  PNG row filters (None/Sub/Up/Average/Paeth) in place.  A row
//                   depends on the row above and on its own left bytes, so it is a
//                   skewed wavefront: lane = row (64 rows per wave, one band),
//                   16-byte chunks, lane l works on chunk s - l at step s and hands
//                   its unfiltered chunk to lane l+1 by a DPP wave shift.  One wave
//                   per band, an image's bands over several workgroups; a band's
//                   first row reads the previous band's last row from memory once
//                   it is published (global progress counters, agent-scope
//                   release/acquire; workgroups ordered by a start ticket).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "ik_crc.h"
#include "ik_inflate.h"
#include "ik_internal.h"
#include "ik_png.h"
#include "ik_png_wave.h"
#include "ik_unfilter.h"

namespace ik {

// The next batch's block search runs beside this batch's later kernels (ik_host.cpp
// StageExec): those raise their waves' issue priority so that the search's
// VALU-heavy waves take the SIMD cycles they leave idle, not the ones their
// latency-bound chains wait for.
__device__ __forceinline__ void raise_priority() { __builtin_amdgcn_s_setprio(3); }

// ---- find ------------------------------------------------------------------------
// One wave per (chunk, image).  A lane owns one 32-bit stream word, i.e. 32
// consecutive bit offsets, so a wave step covers 2,048 offsets from 64
// coalesced word loads (prefetched one step ahead).  The cheap header tests run
// bit-parallel over the lane's 32 offsets on shifted copies of its 128-bit
// window -- BTYPE = 2 (bit 1 clear, bit 2 set), HLIT <= 29 and HDIST <= 29 (not
// all of their top four bits set) -- and only the survivors (about a fifth)
// take the scalar Kraft test of the code-length code (complete: sum 2^-len == 1).
// Offsets passing it (~0.1 %: under two per wave step) go into a per-wave LDS
// queue, and the streaming header check (find_check_win: infl::dynamic_header_win,
// dynamic_header_ok's test over an LDS window of the stream) runs on 64 queued
// offsets at a time, one per lane -- run one by one as they turn up, it would
// take the whole wave for one or two active lanes.  The queue is checked whenever
// it holds 64 offsets (its first 64; the rest wait for the next check) and at the
// end of the chunk; the search stops at the first check that passes an offset,
// with the smallest passing one of that check.  It need not be the chunk's first
// header: any block start serves as a lane start, and an offset that passes the
// check but starts no block is dropped by the decode's chain check.
// win: this lane's window, word k at win[64 k].
typedef __attribute__((address_space(3))) uint32_t lds_word;
// The lane's stream window for infl::dynamic_header_win: 32 words by LDS-DMA
// (global_load_lds_dword: lane l's word lands at M0 + 4 l, so row k of the
// lane-minor window takes one instruction for the whole wave), all in flight at
// once, no VGPRs; near the end of the stream (past the zero padding the window
// could reach) word by word with the bounds check.
struct FindWin {
    const IK_GLOBAL uint32_t* W;
    uint64_t wend;  // words past it read as zero (as infl::Bits)
    lds_word* win;  // this lane's word 0; word k at win[64 k]
    uint32_t r0;    // LDS address of row 0, lane 0 (wave-uniform)
    __device__ void fetch(uint64_t base) {
        if (base + 32 > wend + 64) {
            for (int k = 0; k < 32; ++k) win[64 * k] = base + k < wend ? W[base + k] : 0u;
            return;
        }
        const IK_GLOBAL uint32_t* src = W + base;
        uint32_t keep;
#define IK_FWIN(K)                                                                                     \
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t" \
                 "s_mov_b32 m0, %0 ; fwin " #K                                                         \
                 : "=&s"(keep)                                                                         \
                 : "v"(src + K), "s"(__builtin_amdgcn_readfirstlane(r0 + 256u * K))                   \
                 : "memory")
        IK_FWIN(0); IK_FWIN(1); IK_FWIN(2); IK_FWIN(3); IK_FWIN(4); IK_FWIN(5); IK_FWIN(6); IK_FWIN(7);
        IK_FWIN(8); IK_FWIN(9); IK_FWIN(10); IK_FWIN(11); IK_FWIN(12); IK_FWIN(13); IK_FWIN(14); IK_FWIN(15);
        IK_FWIN(16); IK_FWIN(17); IK_FWIN(18); IK_FWIN(19); IK_FWIN(20); IK_FWIN(21); IK_FWIN(22); IK_FWIN(23);
        IK_FWIN(24); IK_FWIN(25); IK_FWIN(26); IK_FWIN(27); IK_FWIN(28); IK_FWIN(29); IK_FWIN(30); IK_FWIN(31);
#undef IK_FWIN
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __device__ uint32_t word(uint32_t k) const { return win[64 * k]; }
};

__device__ __attribute__((noinline)) bool find_check_win(const IK_GLOBAL uint32_t* W, uint64_t nbits, uint64_t p,
                                                         uint32_t h, uint64_t bits, lds_word* win) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    FindWin fw{W, (nbits >> 5) + 4, win, (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(size_t)win - 4u * lane)};
    return infl::dynamic_header_win(p, h, bits, fw);
}

__device__ __forceinline__ uint32_t fsh(uint32_t lo, uint32_t hi, int k) {  // bits k .. k+31 of hi:lo, 0 < k < 32
    return (lo >> k) | (hi << (32 - k));
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
        v = u < v ? u : v;
    }
    return v;
}

// inclusive wave prefix sum: row_shr steps within rows of 16, then row totals
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const int row = threadIdx.x >> 4;
    return v + (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
}

constexpr uint32_t kFindQueue = 128;

#ifdef IK_FIND_PROF  // dev build: per-phase clock sums of k_png_find (tools/gpu_*.sh experiments)
__device__ unsigned long long g_find_prof[8];
hipError_t png_find_prof_read(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_find_prof), sizeof(g_find_prof));
    unsigned long long z[8] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_find_prof), z, sizeof(z));
    return e;
}
#endif

__global__ __launch_bounds__(64) void k_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx,
                                                 int nchunks_total, uint64_t chunk_bits, int64_t* cand) {
    __shared__ uint32_t s_win[64 * 32];     // per lane: 32 stream words of the candidate being checked (lane-minor)
    __shared__ uint32_t s_q[kFindQueue];    // Kraft-passing offsets (relative to the chunk) awaiting the full check
    __shared__ uint8_t s_kraft[512];        // 3 code-length-code lengths (9 bits) -> sum of 2^(7 - len), len > 0
    const int g = blockIdx.x;
    if (g >= nchunks_total) return;
    for (int v = threadIdx.x; v < 512; v += 64) {
        uint32_t k = 0;
        for (int f = 0; f < 3; ++f) {
            const uint32_t l = ((uint32_t)v >> (3 * f)) & 7u;
            k += l ? (128u >> l) : 0u;
        }
        s_kraft[v] = (uint8_t)k;
    }
    __syncthreads();
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
    const IK_GLOBAL uint32_t* W = (const IK_GLOBAL uint32_t*)I.words;
    uint32_t qlen = 0;           // wave-uniform
    uint32_t best = 0xFFFFFFFFu; // smallest passing offset checked so far (relative to b0)
#ifdef IK_FIND_PROF
    const unsigned long long t_begin = __builtin_readcyclecounter();
    unsigned long long t_flush = 0, n_flush = 0, n_steps = 0, n_cand = 0;
#endif
    // check the queue: all of it at the end of the chunk (all), else its first 64
    // entries, the rest moving to the front for the next check -- one candidate
    // past 64 would otherwise take a check round of its own, the wave waiting on
    // its one lane for up to a true header's ~300 code lengths
    auto flush = [&](bool all) {
        const uint32_t take = all || qlen < 64 ? qlen : 64u;
#ifdef IK_FIND_PROF
        const unsigned long long tf0 = __builtin_readcyclecounter();
        n_flush += take ? 1 : 0;
        n_cand += take;
#endif
        for (uint32_t q0 = 0; q0 < take; q0 += 64) {
            uint32_t v = 0xFFFFFFFFu;
            if (q0 + (uint32_t)lane < take) {
                const uint32_t off = s_q[q0 + lane];
                const uint64_t p = b0 + off;
                const uint64_t wi = p >> 5;
                const uint32_t sh = (uint32_t)(p & 31);
                const uint64_t lo = (uint64_t)W[wi] | ((uint64_t)W[wi + 1] << 32);
                const uint64_t hi = (uint64_t)W[wi + 2] | ((uint64_t)W[wi + 3] << 32);
                const uint64_t x = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;   // bits p .. p+63
                const uint64_t x2 = sh ? (hi >> sh) : hi;                        // bits p+64 ..
                const uint64_t cl = (x >> 17) | (x2 << 47);
                if (find_check_win(W, I.nbits, p, (uint32_t)x, cl, (lds_word*)(s_win + lane)))
                    v = off;
            }
            v = wave_min(v);
            best = v < best ? v : best;
        }
        const uint32_t rest = qlen - take;  // < 64 (the queue holds < 128)
        const uint32_t moved = (uint32_t)lane < rest ? s_q[take + lane] : 0u;
        if ((uint32_t)lane < rest) s_q[lane] = moved;
        qlen = rest;
#ifdef IK_FIND_PROF
        t_flush += __builtin_readcyclecounter() - tf0;
#endif
    };
    const uint64_t wlast = (b1 + 31) >> 5;  // words holding offsets < b1 (the stream is zero padded past them)
    uint64_t wi = (b0 >> 5) + (uint64_t)lane;
    uint32_t n0 = W[wi], n1 = W[wi + 1], n2 = W[wi + 2], n3 = W[wi + 3];
    for (;;) {
#ifdef IK_FIND_PROF
        ++n_steps;
#endif
        const uint32_t w0 = n0, w1 = n1, w2 = n2, w3 = n3;
        const uint64_t wn = wi + 64;
        if (wn - (uint64_t)lane < wlast) {  // wave-uniform: prefetch the next step's words
            n0 = W[wn]; n1 = W[wn + 1]; n2 = W[wn + 2]; n3 = W[wn + 3];
        }
        // bit-parallel filters over offsets p = 32 wi + j, j = 0..31
        uint32_t m = ~fsh(w0, w1, 1) & fsh(w0, w1, 2);                                          // BTYPE == 2
        m &= ~(fsh(w0, w1, 4) & fsh(w0, w1, 5) & fsh(w0, w1, 6) & fsh(w0, w1, 7));             // HLIT <= 29
        m &= ~(fsh(w0, w1, 9) & fsh(w0, w1, 10) & fsh(w0, w1, 11) & fsh(w0, w1, 12));           // HDIST <= 29
        const uint64_t pw = wi << 5;
        if (pw < b0) m &= b0 - pw >= 32 ? 0u : ~0u << (uint32_t)(b0 - pw);
        if (pw + 32 > b1) m &= pw >= b1 ? 0u : (1u << (uint32_t)(b1 - pw)) - 1u;
        const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32), hi = (uint64_t)w2 | ((uint64_t)w3 << 32);
        uint32_t km = 0;  // offsets passing the Kraft test
        while (m) {
            const uint32_t j = (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            const uint32_t sh = j + 17;  // 17 .. 48
            const uint64_t cl = (lo >> sh) | (hi << (64 - sh));  // code-length code lengths (57 bits)
            const int ncode = (int)((uint32_t)(lo >> (j + 13)) & 15u) + 4;
            // Kraft sum over the ncode lengths, three at a time from the LDS table
            if (infl::cl_kraft_top(cl, ncode, s_kraft) == 128u) km |= 1u << j;
        }
        // queue them: one per lane per round, compacted by lane rank
        for (;;) {
            const unsigned long long bal = __ballot(km != 0);
            if (!bal) break;
            if (qlen + 64 > kFindQueue) flush(false);
            if (km) {
                const uint32_t j = (uint32_t)__builtin_ctz(km);
                km &= km - 1u;
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                s_q[qlen + r] = (uint32_t)(pw + j - b0);
            }
            qlen += (uint32_t)__popcll(bal);
        }
        if (qlen >= 64) flush(false);
        if (best != 0xFFFFFFFFu) break;  // any header that passes will do (the decode chain checks it)
        wi = wn;
        if (wi - (uint64_t)lane >= wlast) break;
    }
    if (best == 0xFFFFFFFFu) flush(true);
    if (lane == 0) cand[g] = best == 0xFFFFFFFFu ? -1 : (int64_t)(b0 + best);
#ifdef IK_FIND_PROF
    if (lane == 0) {
        atomicAdd(&g_find_prof[0], __builtin_readcyclecounter() - t_begin);
        atomicAdd(&g_find_prof[1], t_flush);
        atomicAdd(&g_find_prof[2], n_flush);
        atomicAdd(&g_find_prof[3], n_steps);
        atomicAdd(&g_find_prof[4], n_cand);
        atomicAdd(&g_find_prof[5], 1ull);
    }
#endif
}

// ---- inflate ------------------------------------------------------------------------
// One thread per decoder lane, canonical decoding (ik_inflate.h decode_lane_canon):
// the code-length limits sit in registers and the small per-length tables in
// LDS.  The lane's compressed stream reaches the hot loop through a ring of
// four 32-byte blocks per lane in LDS, filled by LDS-DMA (global_load_lds_dwordx4)
// on a fixed schedule: every kRingTick symbols the lane waits for the DMAs it
// issued last time (vmcnt(0): they are a full interval old) and issues the
// block three ahead of the one it reads.  The loop itself then reads only LDS,
// so no lane's memory latency stalls its wave (a wave's vmcnt is shared by its
// 64 lanes).
constexpr int kRingBW = 8;    // words per block (32 B)
constexpr int kRingTick = 4;  // symbols between refills (< 256 bits: at most one block per interval)

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// a lane's u32 table in LDS, lane-minor (word w at 64 w + lane): conflict-free
// whatever word each lane reads
struct LaneLds {
    lds_u32* p;  // s_tab + lane
    __device__ lds_u32& operator[](int w) const { return p[w * 64]; }
};

struct WinLds {
    const IK_GLOBAL uint32_t* w;
    uint32_t nwords, pos, nextb, it;
    lds_u32* ring;   // this wave's ring, lane-minor: ring word r (0..31) of lane l at 64 r + l
    uint32_t lane;
    __device__ uint32_t word(uint32_t wi) const { return ring[(wi & 31u) * 64u]; }
    // Word k of block B of the calling lanes -> ring word 8 (B % 4) + k: one 4-byte
    // LDS-DMA per word (the destination is M0 + 4 lane, i.e. lane-minor).  M0 is
    // written in the same asm statement (the compiler does not preserve it), and
    // each ring position has its own asm text: identical statements in the four
    // branches would be merged into one with a per-lane base, which M0 cannot hold.
#define IK_GLDS4(TAG)                                                                                  \
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"    \
                 "s_mov_b32 m0, %0 ; ring " TAG                                                        \
                 : "=&s"(keep)                                                                         \
                 : "v"(src), "s"(base)                                                                 \
                 : "memory")
#define IK_GLDS_BLOCK(P)                                                                               \
    src = g + 0; base = r0 + ((P)*8 + 0) * 256; IK_GLDS4(#P "0");                                      \
    src = g + 1; base = r0 + ((P)*8 + 1) * 256; IK_GLDS4(#P "1");                                      \
    src = g + 2; base = r0 + ((P)*8 + 2) * 256; IK_GLDS4(#P "2");                                      \
    src = g + 3; base = r0 + ((P)*8 + 3) * 256; IK_GLDS4(#P "3");                                      \
    src = g + 4; base = r0 + ((P)*8 + 4) * 256; IK_GLDS4(#P "4");                                      \
    src = g + 5; base = r0 + ((P)*8 + 5) * 256; IK_GLDS4(#P "5");                                      \
    src = g + 6; base = r0 + ((P)*8 + 6) * 256; IK_GLDS4(#P "6");                                      \
    src = g + 7; base = r0 + ((P)*8 + 7) * 256; IK_GLDS4(#P "7")
    __device__ void dma(uint32_t B) {
        static_assert(kRingBW == 8, "eight words per block");
        const IK_GLOBAL uint32_t* g = w + (size_t)B * kRingBW;
        const uint32_t r0 = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)ring - 4u * lane);  // ring base (lane 0)
        uint32_t keep;
        const IK_GLOBAL uint32_t* src;
        uint32_t base;
        switch (B & 3u) {
        case 0: IK_GLDS_BLOCK(0); break;
        case 1: IK_GLDS_BLOCK(1); break;
        case 2: IK_GLDS_BLOCK(2); break;
        default: IK_GLDS_BLOCK(3); break;
        }
    }
#undef IK_GLDS_BLOCK
#undef IK_GLDS4
    __device__ void init(const IK_GLOBAL uint32_t* words, uint32_t nw, uint32_t bit) {
        w = words;
        nwords = nw;
        pos = bit;
        it = 0;
        const uint32_t B0 = (bit >> 5) / kRingBW;
        for (uint32_t k = 0; k < 4; ++k) dma(B0 + k);
        nextb = B0 + 4;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // Every kRingTick symbols: store the lane's pending token group (if any lane
    // has one: one 16-byte store instruction for the wave), wait until all but
    // that store are done -- the ring's DMA from the last tick among them -- and
    // issue the block three ahead.  Between ticks the loop issues no memory
    // instruction, so the count in the wait is exact.
    // Why these hand-counted waits are safe (round 3's unfilter bug was
    // asm loads whose destination VGPRs the register allocator copied before the
    // asm wait): a global_load_lds_dword has no destination VGPR -- the data goes
    // to LDS at M0 -- so there is no register for the allocator to copy early, and
    // the ring words are read only by ds_read after the wait.  The only vector-
    // memory instructions between two ticks are this tick's st stores (issued
    // after the DMAs, gfx9 counts stores in vmcnt and retires the counter in
    // issue order), so vmcnt(st) leaves exactly them outstanding and every DMA of
    // the previous tick complete.  The wave decoder (the default, k_png_wave)
    // stages its windows with plain loads and LDS stores the compiler waits for.
    __device__ void tick(infl::TokOut& o) {
        if (++it % kRingTick) return;
        const int st = o.flush();  // 0, 1 or 2 stores for this lane; the wave issued as many as its max
        if (__ballot(st >= 2))
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if (__ballot(st >= 1))
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (nextb <= ((pos >> 5) / kRingBW) + 3u) {
            dma(nextb);
            ++nextb;
        }
    }
    // The next 64+ bits: three words read from the ring.  (A register window
    // sliding by selects, with the next words read one symbol ahead, measured
    // slower: 2,382 vs 2,187 cycles per symbol -- these reads are not what the
    // symbol-to-symbol chain waits for.)
    __device__ uint64_t bits64() const {
        const uint32_t wi = pos >> 5, sh = pos & 31u;
        const uint32_t a = word(wi), b = word(wi + 1), c = word(wi + 2);
        const uint64_t lo = (uint64_t)a | ((uint64_t)b << 32);
        return sh ? (lo >> sh) | ((uint64_t)c << (64 - sh)) : lo;
    }
    __device__ void advance(uint32_t k) { pos += k; }
};

__global__ __launch_bounds__(kPngInflateThreads) void k_png_decode(const PngImgDev* imgs, const PngLaneDev* lanes,
                                                                   const uint32_t* order, int nlanes, uint16_t* tok,
                                                                   infl::LaneResult* res) {
    __shared__ uint32_t s_tab[kPngInflateThreads * infl::kCanonWords];  // lane-minor (LaneLds)
    __shared__ uint32_t s_ring[4 * kRingBW * 64];                        // 4 blocks x 32 B per lane, lane-minor
    const int slot = blockIdx.x * kPngInflateThreads + threadIdx.x;
    if (slot >= nlanes) return;
    const int t = order ? (int)order[slot] : slot;  // launch order (ik_png_decode.cpp order_lanes)
    const PngLaneDev L = lanes[t];
    const PngImgDev I = imgs[L.img];
    const LaneLds m{(lds_u32*)s_tab + threadIdx.x};
    WinLds win;
    win.ring = (lds_u32*)s_ring + threadIdx.x;
    win.lane = threadIdx.x;
    infl::TokOut out;
    out.p = (IK_GLOBAL uint16_t*)(tok + L.tbase);
    infl::LaneResult r;
    const uint64_t c0 = clock64();
    infl::decode_lane_tok(I.words, I.nbits, L.start, L.stop, m, out, L.ntok, L.first != 0, I.raw_total, r, win);
    r.kcycles = (uint32_t)((clock64() - c0) >> 10);
    res[t] = r;
}

// ---- the wave decoder (ik_png_wave.h) ------------------------------------------------
// One wave per decoder lane: the lane's blocks one after another; per block the
// header (lane 0), the shared lookup tables (all lanes), then the body window by
// window: the window's stream words staged in LDS with coalesced 16-byte loads,
// 64 sub-lanes decoding sub-ranges at once (wave::sub_decode), fix rounds until
// the sub-lanes' starts and exits chain, the chained sub-lanes' token pieces
// recorded.  Every branch around the sub-lane passes is wave-uniform.
constexpr uint32_t kWaveWinWords = (uint32_t)(wave::kWindowBits / 32) + 16;  // + the last sub-lane's overshoot

typedef __attribute__((address_space(3))) uint16_t lds_u16;

// The 64 stream bits at a sub-lane's position in the staged window (relative
// positions: w[0]'s bit 0 = 0), as a cursor: words wi .. wi+3 in registers, and
// wi+4, wi+5 read from LDS one step ahead -- a step consumes at most 48 bits (two
// words), so the step's bits never wait on an LDS read; only its table lookups do.
struct WaveLdsCursor {
    const lds_u32* w;
    uint32_t wi = 0, b0 = 0, b1 = 0, b2 = 0, b3 = 0, p0 = 0, p1 = 0;
    __device__ void init(uint32_t pos) {
        wi = pos >> 5;
        b0 = w[wi];
        b1 = w[wi + 1];
        b2 = w[wi + 2];
        b3 = w[wi + 3];
        p0 = w[wi + 4];
        p1 = w[wi + 5];
    }
    __device__ uint64_t operator()(uint32_t pos) {
        const uint32_t d = (pos >> 5) - wi;  // 0, 1 or 2
        // (opaque to the optimizer: a select between two of these loaded fields would
        // otherwise become a load through a selected address, and the cursor scratch memory)
        asm("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(p0), "+v"(p1));
        const uint32_t n0 = d == 0 ? b0 : d == 1 ? b1 : b2;
        const uint32_t n1 = d == 0 ? b1 : d == 1 ? b2 : b3;
        const uint32_t n2 = d == 0 ? b2 : d == 1 ? b3 : p0;
        const uint32_t n3 = d == 0 ? b3 : d == 1 ? p0 : p1;
        b0 = n0;
        b1 = n1;
        b2 = n2;
        b3 = n3;
        wi += d;
        p0 = w[wi + 4];  // the next step's (in flight during this one)
        p1 = w[wi + 5];
        const uint32_t sh = pos & 31u;
        return ((uint64_t)__builtin_amdgcn_alignbit(b2, b1, sh) << 32) | __builtin_amdgcn_alignbit(b1, b0, sh);
    }
};
// the same straight from the stream in memory (block headers, stored blocks)
struct WaveGlobalWin {
    const IK_GLOBAL uint32_t* w;
    __device__ uint64_t operator()(uint64_t pos) const {
        const uint64_t wi = pos >> 5;
        const uint32_t sh = (uint32_t)(pos & 31u);
        const uint32_t a = w[wi], b = w[wi + 1], c = w[wi + 2];
        const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(c, b, sh);
        return ((uint64_t)hi << 32) | lo;
    }
};

// A sub-lane's token output on the GPU: the open group of 8 tokens sits in two
// 64-bit registers (token slot i at bits 16 i of g0:g1), each completed group goes
// to the sub-lane's piece with one 16-byte store -- no LDS traffic per token.
struct WaveOut {
    IK_GLOBAL uint16_t* p;
    uint32_t cap;        // tokens (a multiple of 8)
    uint32_t n = 0;      // tokens put
    uint64_t g0 = 0, g1 = 0;
    __device__ void reset() { n = 0; g0 = 0; g1 = 0; }
    __device__ void mark(uint32_t, uint32_t) const {}  // (the CPU model's step profile)
    __device__ void store(uint32_t g) const {  // the group of tokens [g, g + 8) (g a multiple of 8)
        if (g + 8u > cap) return;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 q = {(uint32_t)g0, (uint32_t)(g0 >> 32), (uint32_t)g1, (uint32_t)(g1 >> 32)};
        *reinterpret_cast<IK_GLOBAL u4*>(p + g) = q;
    }
    // the first k of the four tokens at slot n & 7 (the part past slot 7 opens the next group)
    __device__ void put4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        uint64_t T = (uint64_t)(a & 0xFFFFu) | ((uint64_t)(b & 0xFFFFu) << 16) | ((uint64_t)(c & 0xFFFFu) << 32) |
                     ((uint64_t)d << 48);
        T &= k >= 4u ? ~0ull : (1ull << (16u * k)) - 1ull;
        // (selects of shifts, no branches: the 128-bit group g0:g1 |= T << off, the part
        // past bit 128 is the next group's start)
        const uint32_t off = 16u * (n & 7u);  // 0 .. 112
        const uint64_t lo_part = T << (off & 63u), hi_part = (T >> 1) >> (63u - (off & 63u));
        g0 |= off < 64u ? lo_part : 0ull;
        g1 |= off < 64u ? hi_part : lo_part;  // (off 0: hi_part is 0)
        const uint64_t carry = off > 64u ? hi_part : 0ull;
        const uint32_t n2 = n + k;
        const bool done = ((n2 ^ n) & ~7u) != 0u;  // a group completed
        if (done) store(n & ~7u);
        g0 = done ? carry : g0;
        g1 = done ? 0ull : g1;
        n = n2;
    }
    __device__ void finish() {  // pad the open group and store it
        if (n & 7u) {
            constexpr uint64_t P = 0xFFFEFFFEFFFEFFFEull;
            const uint32_t off = 16u * (n & 7u);  // 16 .. 112
            if (off < 64u) {
                g0 |= P << off;
                g1 |= P;
            } else {
                g1 |= P << (off - 64u);
            }
            store(n & ~7u);
        }
    }
};

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// rank of this lane among the lanes of mask m below it
__device__ __forceinline__ uint32_t lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One canonical code built by the wave (wave::code_build's result, without its
// serial loops): lens[0..n) in LDS; per-length counts by ballots, the validity
// rule of zlib, the left-justified limits and per-length info (C, lane 0 writes
// it) and the symbols in canonical order (syms), each lane placing its symbols.
__device__ bool wave_code_build(const uint8_t* lens, int n, bool is_dist, bool fixed, wave::Code& C, uint16_t* syms) {
    const int lane = threadIdx.x;
    uint32_t cnt[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int sy = c0 + lane;
        const uint32_t l = sy < n ? lens[sy] & 15u : 0u;
#pragma unroll
        for (int L = 1; L <= 15; ++L) cnt[L] += (uint32_t)__popcll(__ballot(l == (uint32_t)L));
    }
    int maxl = 0, left = 1;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        if (cnt[L]) maxl = L;
        left = (left << 1) - (int)cnt[L];
    }
    bool ok = left >= 0;
    if (!fixed) {
        if (maxl == 0) ok = ok && is_dist;
        else if (left > 0 && maxl != 1) ok = false;
    }
    if (!ok) return false;
    uint32_t lim[15], off[16], code = 0, rank = 0;
    off[0] = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        code = (code + (L > 1 ? cnt[L - 1] : 0u)) << 1;
        if (lane == 0) C.info[L] = (code & 0x7FFFu) | (rank << 16);
        lim[L - 1] = (code + cnt[L]) << (15 - L);
        off[L] = rank;
        rank += cnt[L];
    }
    if (lane == 0) {
        C.info[0] = 0;
        uint32_t pk[8];
        infl::pack_limits(lim, pk);
#pragma unroll
        for (int k = 0; k < 8; ++k) C.pk[k] = pk[k];
    }
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int sy = c0 + lane;
        const uint32_t l = sy < n ? lens[sy] & 15u : 0u;
#pragma unroll
        for (int L = 1; L <= 15; ++L) {
            const unsigned long long m = __ballot(l == (uint32_t)L);
            if (l == (uint32_t)L) syms[off[L] + lane_rank(m)] = (uint16_t)sy;
            off[L] += (uint32_t)__popcll(m);
        }
    }
    return true;
}

#ifdef IK_WAVE_PROF  // dev build: k_png_wave's phase clock sums (tools/dev_png experiments)
__device__ unsigned long long g_wave_prof[8];
hipError_t png_wave_prof_read(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_prof), sizeof(g_wave_prof));
    unsigned long long z[8] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_prof), z, sizeof(z));
    return e;
}
#define IK_WP(k, t0) (wprof[k] += clock64() - (t0))
#else
#define IK_WP(k, t0) ((void)0)
#endif

// The block's codes by the wave: a dynamic header's code-length code (lanes 0..18
// take one length each) and its 7-bit decode table, then the literal/length and
// distance code lengths, then both codes (wave_code_build).  Checks as
// infl::parse_dynamic (zlib).  *body = the first bit of the block's data.
// The header's 160 words (17 + 57 + 316 * 14 bits at most) stay in registers, lane
// l holding words l, 64 + l, 128 + l, and so does the 128-entry decode table (lane l:
// entries l and 64 + l): the code-length symbols -- a serial chain, each one's
// length places the next -- are decoded by the whole wave in step, every value
// wave-uniform (scalar ALU, v_readlane lookups), with no memory latency in the
// chain; a repeat run is written by as many lanes at once.
__device__ bool wave_block_codes(const IK_GLOBAL uint32_t* W, uint64_t nbits, uint64_t p, int btype,
                                 uint8_t* lens, wave::Code* code, uint16_t* lsym, uint16_t* dsym, uint64_t* body) {
    const int lane = threadIdx.x;
    __syncthreads();  // the previous block's readers of the tables are done
    if (btype == 1) {
        for (int i = lane; i < 288 + 32; i += 64) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
        __syncthreads();
        *body = p + 3;
        const bool a = wave_code_build(lens, 288, false, true, code[0], lsym);
        const bool b = wave_code_build(lens + 288, 30, true, true, code[1], dsym);
        __syncthreads();
        return a && b;
    }
    const uint64_t hb0 = (p >> 5) << 5;
    const uint64_t wmax = (nbits >> 5) + 64;  // (the stream's zero padding: 128 words)
    auto hload = [&](int k) -> uint32_t { return k < 160 && (p >> 5) + (uint64_t)k < wmax ? W[(p >> 5) + (uint64_t)k] : 0u; };
    const uint32_t hv0 = hload(lane), hv1 = hload(lane + 64), hv2 = hload(lane + 128);
    auto word = [&](uint32_t k) -> uint32_t {  // header word k (wave-uniform k < 192)
        const uint32_t src = k < 64u ? hv0 : k < 128u ? hv1 : hv2;
        return (uint32_t)__builtin_amdgcn_readlane((int)src, (int)(k & 63u));
    };
    auto bits32 = [&](uint32_t o) -> uint32_t {  // 32 bits from relative bit o
        return __builtin_amdgcn_alignbit(word((o >> 5) + 1u), word(o >> 5), o & 31u);
    };
    const uint32_t o0 = (uint32_t)(p - hb0) + 3;
    const uint32_t h = bits32(o0);
    const int nlen = (int)(h & 31u) + 257, ndist = (int)((h >> 5) & 31u) + 1, ncode = (int)((h >> 10) & 15u) + 4;
    if (nlen > 286 || ndist > 30) return false;
    // the code-length code: lane s holds symbol s's length (57 bits from o0 + 14)
    constexpr uint8_t inv_order[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};
    const uint64_t clb = (uint64_t)bits32(o0 + 14) | ((uint64_t)bits32(o0 + 46) << 32);
    uint32_t myl = 0;
    if (lane < 19) {
        const int i = inv_order[lane];
        myl = i < ncode ? (uint32_t)(clb >> (3 * i)) & 7u : 0u;
    }
    uint32_t cnt[8];
#pragma unroll
    for (int L = 1; L <= 7; ++L) cnt[L] = (uint32_t)__popcll(__ballot(myl == (uint32_t)L));
    uint32_t kraft = 0;
#pragma unroll
    for (int L = 1; L <= 7; ++L) kraft += cnt[L] << (7 - L);
    if (kraft != 128u) return false;  // the code-length code must be complete
    // the decode table: entry e (the next 7 bits, first bit lowest) = symbol | length << 5
    uint32_t tab = 0;  // this lane's entries lane (byte 0) and 64 + lane (byte 1)
    {
        uint32_t code_l = 0, first[8];
#pragma unroll
        for (int L = 1; L <= 7; ++L) {
            code_l = (code_l + (L > 1 ? cnt[L - 1] : 0u)) << 1;
            first[L] = code_l;
        }
        uint32_t mine = 0;  // (bit-reversed code | length << 8) of this lane's symbol
#pragma unroll
        for (int L = 1; L <= 7; ++L) {
            const unsigned long long m = __ballot(myl == (uint32_t)L);
            if (myl == (uint32_t)L) mine = (__builtin_bitreverse32(first[L] + lane_rank(m)) >> (32 - L)) | ((uint32_t)L << 8);
        }
        for (int sy = 0; sy < 19; ++sy) {
            const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)mine, sy);
            const uint32_t Ls = q >> 8;
            if (!Ls) continue;
            const uint32_t r = q & 127u, msk = (1u << Ls) - 1u, ent = (uint32_t)sy | (Ls << 5);
            if (((uint32_t)lane & msk) == r) tab |= ent;
            if (((uint32_t)(lane + 64) & msk) == r) tab |= ent << 8;
        }
    }
    // the literal/length and distance code lengths (the distance lengths to lens[288 ..])
#ifdef IK_WAVE_PROF
    const uint64_t tl0 = clock64();
#endif
    uint32_t o = o0 + 14 + 3 * (uint32_t)ncode;
    const int total = nlen + ndist;
    int i = 0, prev = -1;
    bool ok = true;
    // a wave-uniform 64-bit bit buffer (scalar registers): refilled a word at a time
    // when under 32 bits remain (a symbol takes at most 7 + 7), so a symbol costs one
    // table v_readlane and scalar arithmetic
    uint32_t wn = (o >> 5) + 2u;
    uint64_t buf = (((uint64_t)word((o >> 5) + 1u) << 32) | word(o >> 5)) >> (o & 31u);
    uint32_t nb = 64u - (o & 31u);
    while (i < total) {
        if (nb < 32u) {
            buf |= (uint64_t)word(wn) << nb;
            nb += 32u;
            ++wn;
        }
        const uint32_t v = (uint32_t)buf;
        const uint32_t e7 = v & 127u;
        const uint32_t ent = ((uint32_t)__builtin_amdgcn_readlane((int)tab, (int)(e7 & 63u)) >> (8u * (e7 >> 6))) & 255u;
        const uint32_t L = ent >> 5, sym = ent & 31u;
        int rep = 1, val = (int)sym;
        uint32_t xb = 0;
        if (sym == 16) {
            if (prev < 0) { ok = false; break; }
            val = prev;  // (the previous length: the literal/length code's last one for the first distance)
            xb = 2;
            rep = 3 + (int)((v >> L) & 3u);
        } else if (sym == 17) {
            val = 0;
            xb = 3;
            rep = 3 + (int)((v >> L) & 7u);
        } else if (sym == 18) {
            val = 0;
            xb = 7;
            rep = 11 + (int)((v >> L) & 127u);
        }
        if (i + rep > total) { ok = false; break; }
        for (int k0 = 0; k0 < rep; k0 += 64) {
            const int d = i + k0 + lane;
            if (k0 + lane < rep) lens[d < nlen ? d : 288 + (d - nlen)] = (uint8_t)val;
        }
        i += rep;
        prev = val;
        buf >>= L + xb;
        nb -= L + xb;
        o += L + xb;
        if (o > 160 * 32 - 96) { ok = false; break; }  // past any valid header
    }
    __syncthreads();  // the lengths are in LDS
#ifdef IK_WAVE_PROF
    if (lane == 0) atomicAdd(&g_wave_prof[6], (unsigned long long)(clock64() - tl0));
#endif
    if (!ok || lens[256] == 0) return false;  // (no end-of-block code: invalid)
    *body = hb0 + o;
    if (*body > nbits) return false;
    const bool a = wave_code_build(lens, nlen, false, false, code[0], lsym);
    const bool b = wave_code_build(lens + 288, ndist, true, false, code[1], dsym);
    __syncthreads();
    return a && b;
}


__global__ __launch_bounds__(64) void k_png_wave(const PngImgDev* imgs, const PngLaneDev* lanes, const uint32_t* order,
                                                 int nlanes, uint16_t* tok, uint2* pieces, uint2* units,
                                                 infl::LaneResult* res) {
    __shared__ __attribute__((aligned(16))) uint32_t s_win[kWaveWinWords];
    __shared__ uint32_t s_lit[1u << wave::kLB];
    __shared__ uint32_t s_dist[1u << wave::kDB];
    __shared__ uint16_t s_lsym[288];
    __shared__ uint16_t s_dsym[32];
    __shared__ uint8_t s_lens[288 + 32];
    __shared__ wave::Code s_code[2];
    const int slot = blockIdx.x;
    if (slot >= nlanes) return;
    const int t = order ? (int)order[slot] : slot;
    const int lane = threadIdx.x;
    const PngLaneDev L = lanes[t];
    const PngImgDev I = imgs[L.img];
    const uint64_t nbits = I.nbits, start = L.start, stop = L.stop;
    const uint64_t stop_eff = stop == ~0ull ? nbits : (stop < nbits ? stop : nbits);
    const IK_GLOBAL uint32_t* W = (const IK_GLOBAL uint32_t*)I.words;
    const WaveGlobalWin gwin{W};
    IK_GLOBAL uint16_t* const region = (IK_GLOBAL uint16_t*)(tok + L.tbase);
    IK_GLOBAL uint2* const ptab = (IK_GLOBAL uint2*)(pieces + L.pbase);
    IK_GLOBAL uint2* const utab = (IK_GLOBAL uint2*)(units + L.pbase);  // expand-unit records (wave::unit_starts)
    const uint64_t cap = L.ntok;
    const uint32_t pcap = L.npieces;  // piece-table entries of this lane (wave::pieces_capacity)
    const bool big = L.big != 0;
    const uint64_t c0 = clock64();
#ifdef IK_WAVE_PROF
    uint64_t wprof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    uint64_t p = start, used = 0, total = 0;
    uint32_t npieces = 0, nblocks = 0, steps = 0, nunits = 0;
    uint64_t written = 0;  // tokens in the pieces (padding included)
    uint64_t unit_v0 = 0;  // the current expand unit's first token
    uint64_t prev_bits = 0;  // the last block's body length (wave::window_end)
    uint64_t ck_setup = 0;   // profile: clock in codes, tables, staging
    int status = infl::kLaneCorrupt, final_block = 0;
    const lds_u32* lit = (const lds_u32*)s_lit;
    const lds_u32* dist = (const lds_u32*)s_dist;
    const lds_u16* lsym = (const lds_u16*)s_lsym;
    const lds_u16* dsym = (const lds_u16*)s_dsym;
    for (;;) {
        if (p >= stop) {
            status = p == stop ? infl::kLaneOk : infl::kLaneMismatch;
            break;
        }
        if (p + 3 > nbits) break;
        const uint64_t blk_start = p, blk_total = total, blk_used = used, blk_written = written;
        const uint32_t blk_pieces = npieces, blk_units = nunits;
        const uint64_t blk_v0 = unit_v0;
        if (wave::unit_starts(nunits, written, unit_v0)) {  // (undone with the block on a split)
            // (nunits <= npieces <= pcap; at pcap the block splits and the record is dropped)
            if (lane == 0 && nunits < pcap) utab[nunits] = make_uint2(npieces, (uint32_t)total);
            ++nunits;
            unit_v0 = written;
        }
        const uint64_t h = gwin(p);
        const int bfinal = (int)(h & 1u), btype = (int)((h >> 1) & 3u);
        ++nblocks;
        if (btype == 3) break;
        if (btype == 0) {  // stored: one piece of raw tokens, all lanes
            uint64_t q = (p + 3 + 7) & ~7ull;
            const uint64_t lh = gwin(q);
            const uint32_t len = (uint32_t)lh & 0xFFFFu, nlen = (uint32_t)(lh >> 16) & 0xFFFFu;
            if ((len ^ 0xFFFFu) != nlen) break;
            q += 32;
            if (q + 8ull * len > nbits) break;
            if (stop != ~0ull && q + 8ull * len > stop) {  // the block passes the lane's stop: no tokens needed
                p = q + 8ull * len;
                status = infl::kLaneMismatch;
                break;
            }
            const uint32_t n8 = (len + 7u) & ~7u;
            if (used + n8 > cap) { status = infl::kLaneOverflow; break; }
            if (npieces >= pcap) {
                nunits = blk_units;  // (the split lane ends before this block)
                status = p > start ? (int)infl::kLaneSplit : (int)infl::kLaneOverflow;
                break;
            }
            const IK_GLOBAL uint8_t* B = (const IK_GLOBAL uint8_t*)W + (q >> 3);
            for (uint32_t i = (uint32_t)lane; i < n8; i += 64)
                region[used + i] = i < len ? (uint16_t)(infl::kTokRaw | B[i]) : (uint16_t)infl::kTokPad;
            if (lane == 0) ptab[npieces] = make_uint2((uint32_t)used, (uint32_t)written);
            ++npieces;
            used += n8;
            written += n8;
            total += len;
            p = q + 8ull * len;
        } else {
            // ---- the block's codes, by the wave ----
            uint64_t body = 0;
            const uint64_t ck0 = clock64();
            if (!wave_block_codes(W, nbits, p, btype, s_lens, s_code, s_lsym, s_dsym, &body)) break;
            IK_WP(1, ck0);
            // ---- the lookup tables, all lanes ----
            [[maybe_unused]] const uint64_t ckt = clock64();
            {
                // the codes' limits in registers (wave-uniform), their per-length info read from LDS
                struct CodeRegs {
                    uint32_t pk[8];
                    const lds_u32* info;
                };
                CodeRegs lc, dc;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    lc.pk[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_code[0].pk[k]);
                    dc.pk[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_code[1].pk[k]);
                }
                lc.info = (const lds_u32*)s_code[0].info;
                dc.info = (const lds_u32*)s_code[1].info;
                // (unrolled: the entries' dependent LDS reads -- per-length info, then the
                // symbol -- of several entries in flight at once)
#pragma unroll 4
                for (uint32_t e = (uint32_t)lane; e < (1u << wave::kLB); e += 64) s_lit[e] = wave::lit_table_entry(e, lc, lsym);
#pragma unroll
                for (uint32_t e = (uint32_t)lane; e < (1u << wave::kDB); e += 64) s_dist[e] = wave::dist_table_entry(e, dc, dsym);
            }
            __syncthreads();
            IK_WP(2, ckt);
            ck_setup += clock64() - ck0;
            // ---- the body, window by window ----
            uint64_t bp = body;
            const uint64_t est_end = wave::block_end_estimate(body, prev_bits);
            int done = 0;  // 1 block ended, 2 lane ends (status set), 3 corrupt / overflow, 4 split
            while (!done) {
                if (bp >= stop_eff) {
                    status = stop == ~0ull ? infl::kLaneCorrupt : infl::kLaneMismatch;
                    done = 2;
                    break;
                }
                const uint64_t re = wave::window_end(bp, stop_eff, est_end);
                const wave::Split sp = wave::split_range(bp, re, big);
                if (used + (uint64_t)sp.nsub * sp.cap > cap) { status = infl::kLaneOverflow; done = 3; break; }
                // stage the window: words from bp's 16-byte group to past the last sub-lane's overshoot
                const uint64_t w0 = (bp >> 5) & ~3ull;
                // (the last sub-lane reads up to 48 + 64 bits past re)
                uint32_t nq = (uint32_t)((((re + 160) >> 5) + 1 - w0 + 3) >> 2);  // 16-byte groups
                nq = nq < kWaveWinWords / 4 ? nq : kWaveWinWords / 4;
                {
                    const uint64_t ck1 = clock64();
                    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                    const IK_GLOBAL u4* src = (const IK_GLOBAL u4*)(W + w0);
                    __syncthreads();  // the previous window's readers are done
                    // 7 loads in flight per lane (a 12 KiB window is 13 per lane): two memory
                    // latencies per window, not one per load
                    for (uint32_t k0 = (uint32_t)lane; k0 < nq; k0 += 7 * 64) {
                        u4 v[7];
#pragma unroll
                        for (int i = 0; i < 7; ++i)
                            if (k0 + 64u * i < nq) v[i] = src[k0 + 64u * i];
#pragma unroll
                        for (int i = 0; i < 7; ++i)
                            if (k0 + 64u * i < nq) *(u4*)(s_win + 4 * (k0 + 64u * i)) = v[i];
                    }
                    __syncthreads();
                    IK_WP(3, ck1);
                    ck_setup += clock64() - ck1;
                }
                WaveLdsCursor win{(const lds_u32*)s_win};
                const int j = lane;
                const bool act = j < sp.nsub;
                // positions relative to the staged window's first bit (w0 << 5)
                const uint32_t rb = (uint32_t)(bp - (w0 << 5));
                const uint32_t lo = rb + 32u * sp.lw * (uint32_t)j;
                const uint32_t hi = j + 1 < sp.nsub ? lo + 32u * sp.lw : (uint32_t)(re - (w0 << 5));
                WaveOut o{region + used + (uint64_t)j * sp.cap, sp.cap};
                wave::SubRes r{};
                r.start = r.exit = ~0u;
#ifdef IK_WAVE_PROF
                const uint64_t ckp = clock64();
#endif
                if (act) {
                    const uint32_t p0 = j == 0 ? rb : (lo >= rb + wave::kWarmBits ? lo - (uint32_t)wave::kWarmBits : rb);
                    wave::sub_decode(win, p0, lo, hi, lit, dist, s_code[0], lsym, s_code[1], dsym, o, r);
                    o.finish();
                    steps += r.steps;
                }
                IK_WP(4, ckp);
#ifdef IK_WAVE_PROF
                const uint64_t ckf = clock64();
#endif
                // fix rounds (all lanes in the shuffles; the redone sub-lanes diverge)
                int v = 0;
                for (;;) {
                    const uint32_t exp = (uint32_t)__shfl_up((int)r.exit, 1, 64);
                    const int eobp = __shfl_up(r.eob, 1, 64), badp = __shfl_up(r.bad, 1, 64);
                    const bool chain = j == 0 || (r.start == exp && !eobp && !badp);
                    const unsigned long long broken = __ballot(act && j >= 1 && !chain);
                    v = broken ? __builtin_ctzll(broken) - 1 : sp.nsub - 1;
                    if (!broken) break;
                    if (__builtin_amdgcn_readlane(r.eob, v) || __builtin_amdgcn_readlane(r.bad, v)) break;
                    if (act && j > v && !chain && !eobp && !badp) {
                        wave::sub_decode(win, exp, lo, hi, lit, dist, s_code[0], lsym, s_code[1], dsym, o, r);
                        o.finish();
                        steps += r.steps;
                    }
                }
                IK_WP(5, ckf);
                const bool in = j <= v;
                if (__ballot(in && r.over)) { status = infl::kLaneOverflow; done = 3; break; }
                if (npieces + (uint32_t)(v + 1) > pcap) {
                    status = blk_start > start ? (int)infl::kLaneSplit : (int)infl::kLaneOverflow;
                    done = 4;
                    break;
                }
                {
                    // (base, virtual start) of each chained sub-lane's piece: the exclusive scan of the padded counts
                    const uint32_t n8 = in ? (r.ntok + 7u) & ~7u : 0u;
                    const uint32_t incl = wave_incl_scan_dpp(n8);
                    if (in)
                        ptab[npieces + (uint32_t)j] =
                            make_uint2((uint32_t)(used + (uint64_t)j * sp.cap), (uint32_t)written + incl - n8);
                    written += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                }
                npieces += (uint32_t)(v + 1);
                total += wave_sum_u64(in ? r.out : 0ull);
                // the next window's sub-lanes start past the last piece (its region's rest is free)
                used += (uint64_t)v * sp.cap + (uint64_t)((__builtin_amdgcn_readlane((int)r.ntok, v) + 7u) & ~7u);
                const uint64_t exv = (w0 << 5) + (uint32_t)__builtin_amdgcn_readlane((int)r.exit, v);
                if (__builtin_amdgcn_readlane(r.bad, v)) { done = 3; break; }
                if (__builtin_amdgcn_readlane(r.eob, v)) {
                    p = exv;
                    prev_bits = p - body;
                    done = 1;
                    break;
                }
                bp = exv;
            }
            if (done == 4) {
                nunits = blk_units;
                unit_v0 = blk_v0;
                npieces = blk_pieces;
                total = blk_total;
                used = blk_used;
                written = blk_written;
                p = blk_start;
                break;
            }
            if (done != 1) break;
        }
        if (bfinal) {
            final_block = 1;
            status = stop == ~0ull ? infl::kLaneOk : infl::kLaneMismatch;
            break;
        }
    }
    const uint32_t tsteps = (uint32_t)wave_sum_u64(steps);
    if (lane == 0) {
        infl::LaneResult r{};
        r.end_bit = p;
        r.out_len = total;
        r.ntok = (uint32_t)written;
        r.status = status;
        r.final_block = final_block;
        r.iters = tsteps;
        r.kcycles = (uint32_t)((clock64() - c0) >> 10);
        r.blocks = nblocks;
        r.pieces = npieces;
        r.kc_setup = (uint32_t)(ck_setup >> 10);
        r.units = nunits;
        res[t] = r;
#ifdef IK_WAVE_PROF
        wprof[0] = clock64() - c0;
        wprof[7] = 1;
        for (int k = 0; k < 8; ++k) atomicAdd(&g_wave_prof[k], (unsigned long long)wprof[k]);
#endif
    }
}

// ---- expand -----------------------------------------------------------------------
// One WAVE per verified lane (one DEFLATE block, ~32K symbols): the lane's tokens
// -> u16 symbols at its output offset: literal bytes, or window markers (0x8000 |
// index into the 32 KiB before the lane, as the resolve pass expects) for copies
// that reach before the lane's first symbol.
constexpr int kXRing = 2048;            // recent output symbols per wave (LDS, power of two)
constexpr int kXCap = 1024;             // output symbols per batch at most
constexpr int kXNear = kXRing - kXCap;  // sources at most this far back come from the ring
using infl::kTokMatch;
using infl::kTokPad;
using infl::kTokRaw;
using infl::kTokTable;
using infl::kTokTableLen;

// Eight tokens per thread (512 per batch: the batch's fixed costs -- ballots, the
// prefix sum, the ring copy, the barrier -- over twice the tokens of four) and the
// copies done in token order: on the bench frames 98.7 % of the tokens are
// literals and a match (~6 bytes, 97 % of them more than kXNear back) is ~1 in
// 75 tokens, so the batch costs a 16-byte load per thread, a prefix sum (DPP), a
// branch-free classification and one LDS write per literal, ~20 instructions and
// one load per match, and a coalesced ring -> memory copy.
//   1. the literals of the batch go to the LDS ring (indexed by absolute symbol
//      position) at their offsets;
//   2. the matches, in token order, each by the whole wave: a position of the
//      copy reads its source from the ring (this batch's earlier positions --
//      literals and earlier copies are in place -- or <= kXNear back), from
//      memory (farther back, written by an earlier batch), or becomes a window
//      marker (before the lane's first symbol);
//   3. the batch's positions go from the ring to memory in aligned groups of 4
//      (8-byte stores; a group's 1-3 positions before the batch are rewritten
//      with the same values, its positions after the batch -- stale ring data --
//      are rewritten by the next batch; groups are clipped to the lane's output).
constexpr uint32_t kX8Tok = 512;  // tokens per batch: 8 per thread
constexpr int kXFar = 64;          // far matches a batch copies flattened (more: one by one)
constexpr int kXPieces = 192;  // piece-table entries staged in LDS (a unit of one 18 KiB block has ~130)

#ifdef IK_EXP_PROF  // dev build: k_png_expand8's phase clock sums (tools/dev_png experiments)
__device__ unsigned long long g_exp_prof[8];
hipError_t png_exp_prof_read(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp_prof), sizeof(g_exp_prof));
    unsigned long long z[8] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_exp_prof), z, sizeof(z));
    return e;
}
#define IK_XP(k) do { const uint64_t _t = clock64(); xprof[k] += _t - xt; xt = _t; } while (0)
#else
#define IK_XP(k) ((void)0)
#endif

template <bool TAB>
__global__ __launch_bounds__(64) void k_png_expand8(const PngImgDev* imgs, const PngLaneDev* lanes, int nlanes,
                                                    const uint16_t* tok, int* status, const uint2* pieces,
                                                    const uint2* units, const uint32_t* ulane, PngMarks mk_out) {
    raise_priority();
    __shared__ __attribute__((aligned(16))) uint16_t s_ring[kXRing];  // recent output, by absolute position
    __shared__ uint32_t s_tab[TAB ? 64 : 1];                            // the block's literal table (TAB)
    __shared__ uint32_t s_pb[kXPieces], s_ps[kXPieces];                 // wave decoder lanes: piece table
    __shared__ uint32_t s_fo[kXFar], s_fd[kXFar], s_fc[kXFar];          // the batch's far matches (offset, distance, start)
    constexpr uint32_t M = kXRing - 1;
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int li = blockIdx.x;  // lane, or expand unit
    if (li >= nlanes) return;
    const int x = threadIdx.x;
    const uint64_t c0 = clock64();
    const PngLaneDev L = lanes[units ? (int)ulane[li] : li];
    const PngImgDev I = imgs[L.img];
    const IK_GLOBAL uint16_t* T = (const IK_GLOBAL uint16_t*)(tok + L.tbase);
    IK_GLOBAL uint16_t* const U = (IK_GLOBAL uint16_t*)I.u16;
    int64_t ob = L.obase, oe = L.obase + (int64_t)L.out_len;
    uint32_t ntok = L.ntok;
    // the wave decoder's lanes: their tokens are pieces of the region (ik_png_wave.h),
    // read in order as one virtual stream of ntok tokens (each piece a multiple of 8);
    // a thread keeps its current piece (base, virtual start) and the next one's start
    const uint32_t np = pieces ? L.npieces : 0u;
    const IK_GLOBAL uint2* P = (const IK_GLOBAL uint2*)(pieces + (pieces ? L.pbase : 0));
    // an expand unit (ik_png_wave.h unit_starts): pieces [pf, pe) of its lane, virtual
    // tokens [t0, ntok), output [ob, oe) -- markers for copies before ob, as for a lane
    uint32_t pf = 0, t0 = 0;
    if (units) {
        const IK_GLOBAL uint2* R = (const IK_GLOBAL uint2*)(units + L.pbase);
        const uint32_t b = (uint32_t)li - L.ubase;
        const uint2 r0 = make_uint2(R[b].x, R[b].y);
        const bool last = b + 1 >= L.nunits;
        uint2 r1 = make_uint2(np, (uint32_t)L.out_len);
        if (!last) r1 = make_uint2(R[b + 1].x, R[b + 1].y);
        pf = r0.x;
        t0 = P[pf].y;
        ntok = r1.x < np ? P[r1.x].y : L.ntok;
        ob = L.obase + (int64_t)r0.y;
        oe = L.obase + (int64_t)r1.y;
    }
    // the unit's first kXPieces entries staged in LDS; past them, memory.  Each thread
    // keeps the piece of its last token (its index only grows: a window is 512
    // tokens, a piece tens to hundreds), so a load walks a step or two at most
    if (np) {
        for (uint32_t k = (uint32_t)x; pf + k < np && k < (uint32_t)kXPieces; k += 64) {
            s_pb[k] = P[pf + k].x;
            s_ps[k] = P[pf + k].y;
        }
        __syncthreads();
    }
    auto piece_base = [&](uint32_t k) -> uint32_t { return k - pf < (uint32_t)kXPieces ? s_pb[k - pf] : P[k].x; };
    auto piece_start = [&](uint32_t k) -> uint32_t { return k - pf < (uint32_t)kXPieces ? s_ps[k - pf] : P[k].y; };
    uint32_t kc = pf, pc_base = 0, pc_start = t0, pn_start = 0xFFFFFFFFu;
    if (np) {
        pc_base = piece_base(pf);
        pn_start = pf + 1 < np ? piece_start(pf + 1) : 0xFFFFFFFFu;
    }
    uint32_t t = t0;
    int64_t cnt = 0;
    bool have_tab = false, bad = false;
    // this thread's 8 tokens of the batch window at a (a multiple of 8, so one
    // 16-byte load that never straddles two pieces; the region is 16-byte aligned
    // and padded past ntok to a multiple of 8 tokens)
    auto load8 = [&](uint32_t a) -> u4 {
        const uint32_t i = a + 8u * (uint32_t)x;
        if (i >= ntok) return u4{0xFFFEFFFEu, 0xFFFEFFFEu, 0xFFFEFFFEu, 0xFFFEFFFEu};
        if (!np) return *(const IK_GLOBAL u4*)(T + i);
        while (i >= pn_start) {
            ++kc;
            pc_base = piece_base(kc);
            pc_start = pn_start;
            pn_start = kc + 1 < np ? piece_start(kc + 1) : 0xFFFFFFFFu;
        }
        return *(const IK_GLOBAL u4*)(T + pc_base + (i - pc_start));
    };
    u4 w = load8(t0 & ~7u);
#ifdef IK_EXP_PROF
    uint64_t xprof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, xt = clock64();
#endif
    while (t < ntok) {
        IK_XP(5);
        const uint32_t a = t & ~7u, i0 = a + 8u * (uint32_t)x;
        uint32_t u[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u[2 * k] = w[k] & 0xFFFFu;
            u[2 * k + 1] = w[k] >> 16;
        }
        IK_XP(6);
        uint32_t end = a + kX8Tok < ntok ? a + kX8Tok : ntok;
        if constexpr (TAB) {
            // the first table record at or after t in the window
            int ft = 8;
#pragma unroll
            for (int k = 7; k >= 0; --k)
                if (i0 + k >= t && i0 + k < ntok && u[k] == kTokTable) ft = k;
            const unsigned long long tl = __ballot(ft < 8);
            if (tl) {
                const int l = __builtin_ctzll(tl);
                const uint32_t e = a + 8u * (uint32_t)l + (uint32_t)__builtin_amdgcn_readlane(ft, l);
                if (e == t) {  // the table: the literal table -> LDS
                    const uint32_t tt = (t + 8) & ~7u;
                    if (tt + kTokTableLen > ntok) { bad = true; break; }
                    s_tab[x] = ((const IK_GLOBAL uint32_t*)(T + tt))[x];
                    have_tab = true;
                    t = tt + kTokTableLen;
                    w = load8(t & ~7u);
                    __syncthreads();
                    continue;
                }
                end = e;
            }
        }
        // a match's first token last: its distance is in the next window
        {
            const uint32_t q = end - 1u;
            const bool mine = q >= t && (q >> 3) == (i0 >> 3);
            const uint32_t wq = w[(q >> 1) & 3u];
            const uint32_t uq = (q & 1u) ? wq >> 16 : wq & 0xFFFFu;
            if (__ballot(mine && (uq & 0xFF00u) == kTokMatch)) --end;
        }
        if (end <= t) { bad = true; break; }
        // the token after each slot (a match's distance) and before slot 0
        const uint32_t nx = (uint32_t)__shfl_down((int)u[0], 1, 64);
        const uint32_t pv = (uint32_t)__shfl_up((int)u[7], 1, 64);
        // classify (no branches): a literal, a match's length token (its distance is
        // the next token), the distance token itself, padding; bad: anything else
        uint32_t len[8], val[8], lit = 0;  // lit: bit k = slot k is a literal
        uint32_t bd = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t idx = i0 + k;
            const uint32_t prev = k ? u[k - 1] : pv, nxt = k < 7 ? u[k + 1] : nx;
            const uint32_t v = u[k];
            const bool start = (idx >= t) & (idx < end) & !((idx > t) & ((prev & 0xFF00u) == kTokMatch));
            const bool raw = (v & 0xFF00u) == kTokRaw, mt = (v & 0xFF00u) == kTokMatch, pad = v == kTokPad;
            const bool rk = TAB && v < 256u;  // (the lane decoder's Huffman-literal rank)
            const bool isl = raw | rk;
            len[k] = !start ? 0u : isl ? 1u : mt ? (v & 0xFFu) + 3u : 0u;
            uint32_t lv = v & 0xFFu;
            if constexpr (TAB) {
                if (start & rk) lv = (s_tab[v >> 2] >> (8 * (v & 3u))) & 0xFFu;
                bd |= (uint32_t)(start & rk & !have_tab);
            }
            val[k] = isl ? lv : nxt + 1u;  // a literal's byte, or the match's distance
            lit |= (uint32_t)isl << k;
            bd |= (uint32_t)(start & !(isl | mt | pad));
        }
        if (__ballot(bd != 0u)) { bad = true; break; }
        uint32_t off[8], tot;
        for (;;) {
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) sum += len[k];
            const uint32_t incl = wave_incl_scan_dpp(sum);
            tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            off[0] = incl - sum;
#pragma unroll
            for (int k = 1; k < 8; ++k) off[k] = off[k - 1] + len[k - 1];
            if (tot <= (uint32_t)kXCap) break;
            // cut the batch before the first symbol that does not fit (one always does)
            int fk = 8;
#pragma unroll
            for (int k = 7; k >= 0; --k)
                if (len[k] && off[k] + len[k] > (uint32_t)kXCap) fk = k;
            const unsigned long long ov = __ballot(fk < 8);
            const int l = __builtin_ctzll(ov);
            end = a + 8u * (uint32_t)l + (uint32_t)__builtin_amdgcn_readlane(fk, l);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (i0 + k >= end) len[k] = 0;
        }
        IK_XP(1);
        // the next window's tokens, in flight while this batch is written
        const uint32_t t2 = end;
        const u4 wn = t2 < ntok ? load8(t2 & ~7u) : u4{0, 0, 0, 0};
        const uint32_t gb = (uint32_t)(ob + cnt);  // ring index base (absolute position, low bits)
        // 1. literals
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (len[k] && ((lit >> k) & 1u)) s_ring[(gb + off[k]) & M] = (uint16_t)val[k];
        // 2. matches.  A far match (distance > kXNear, so more than the batch's 1,024
        // positions: every source lies before the batch) reads nothing the batch
        // writes: the far matches -- nearly all of them on image data (rows above) --
        // are flattened into one list of positions and copied by all lanes at once, a
        // position per lane (up to 64 of them, listed in LDS by a prefix sum over the
        // lanes); the rest, in token order, each by the whole wave.  (One copy after
        // another, the wave's per-match control -- lane and slot search, readlanes,
        // the loop -- was ~400 scalar instructions per batch, and the CU's one scalar
        // unit bounded the kernel.)
        uint32_t fcnt = 0, flen = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool fk = len[k] != 0u && !((lit >> k) & 1u) && val[k] > (uint32_t)kXNear;
            fcnt += fk ? 1u : 0u;
            flen += fk ? len[k] : 0u;
        }
        const uint32_t fp = fcnt | (flen << 16), fincl = wave_incl_scan_dpp(fp);
        const uint32_t ftot = (uint32_t)__builtin_amdgcn_readlane((int)fincl, 63);
        const uint32_t F = ftot & 0xFFFFu, FT = ftot >> 16;  // far matches, their positions
        const bool flat = F != 0u && F <= (uint32_t)kXFar;
        if (flat) {
            uint32_t ri = (fincl - fp) & 0xFFFFu, rc = (fincl - fp) >> 16;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool fk = len[k] != 0u && !((lit >> k) & 1u) && val[k] > (uint32_t)kXNear;
                if (fk) {
                    s_fo[ri] = off[k];
                    s_fd[ri] = val[k];
                    s_fc[ri] = rc;
                    ++ri;
                    rc += len[k];
                }
            }
            __syncthreads();  // (one wave: orders the list's writes before its reads)
            for (uint32_t j = (uint32_t)x; j < FT; j += 64) {
                uint32_t m = 0;  // the match holding flattened position j: the last with start <= j
                for (uint32_t q = 1; q < F; ++q) m = s_fc[q] <= j ? q : m;
                const uint32_t o = s_fo[m], d = s_fd[m], jj = j - s_fc[m];
                const int32_t sr = (int32_t)(o + jj) - (int32_t)d;  // < -kXNear + ...: before the batch
                const int64_t ab = cnt + sr;
                if (ab < -(int64_t)infl::kWindow) bad = true;
                const uint16_t v = ab < 0 ? (uint16_t)(0x8000u | (uint32_t)(infl::kWindow + ab))
                                          : sr >= -kXNear ? s_ring[(gb + (uint32_t)sr) & M] : U[ob + ab];
                s_ring[(gb + o + jj) & M] = v;
            }
        }
        unsigned long long mk[8], any = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mk[k] = __ballot(len[k] != 0u && !((lit >> k) & 1u) && !(flat && val[k] > (uint32_t)kXNear));
            any |= mk[k];
        }
        IK_XP(2);
#ifdef IK_EXP_PROF
        xprof[7] += 1;
#endif
        auto copy = [&](uint32_t A, uint32_t d) {
            const uint32_t o = A & 0xFFFFu, ln = A >> 16;
            const bool wrap = d < ln;  // overlapping: the source repeats with period d
            const float rd = __builtin_amdgcn_rcpf((float)d);
            for (uint32_t j = (uint32_t)x; j < ln; j += 64) {
                uint32_t jj = j;
                if (wrap) {
                    const uint32_t qq = (uint32_t)((float)j * rd);
                    int32_t r = (int32_t)(j - qq * d);
                    if (r < 0) r += (int32_t)d;
                    else if (r >= (int32_t)d) r -= (int32_t)d;
                    jj = (uint32_t)r;
                }
                const int32_t sr = (int32_t)o - (int32_t)d + (int32_t)jj;  // relative to the batch start
                const int64_t ab = cnt + sr;                                // relative to the lane's first symbol
                uint16_t v;
                if (ab < 0) {
                    if (ab < -(int64_t)infl::kWindow) bad = true;
                    v = (uint16_t)(0x8000u | (uint32_t)(infl::kWindow + ab));
                } else if (sr >= -kXNear) {
                    v = s_ring[(gb + (uint32_t)sr) & M];
                } else {
                    v = U[ob + ab];
                }
                s_ring[(gb + o + j) & M] = v;
            }
        };
        while (any) {
            const int l = __builtin_ctzll(any);
            any &= any - 1ull;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if ((mk[k] >> l) & 1ull)
                    copy((uint32_t)__builtin_amdgcn_readlane((int)(off[k] | (len[k] << 16)), l),
                         (uint32_t)__builtin_amdgcn_readlane((int)val[k], l));
        }
        IK_XP(3);
        // 3. ring -> memory, aligned groups of 4 positions
        {
            const int64_t s0 = ob + cnt, s1 = s0 + tot, cb = s0 & ~3ll;
            const int64_t ng = (s1 - cb + 3) >> 2;
            for (int64_t g = x; g < ng; g += 64) {
                const int64_t ca = cb + 4 * g;
                const uint64_t v4 = *(const uint64_t*)&s_ring[(uint32_t)ca & M];
                if (ca >= ob && ca + 4 <= oe) {
                    *(IK_GLOBAL uint64_t*)(U + ca) = v4;
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (ca + k >= ob && ca + k < oe) U[ca + k] = (uint16_t)(v4 >> (16 * k));
                }
            }
        }
        // 3b. (mk_out.list: the rows directly) the batch's bytes into the image rows
        // (position p of the raw stream is row p / RB, column p % RB: column 0 the
        // filter byte -> ft[], the rest -> dst), its window markers onto the batch's
        // marker list for k_png_marks -- so no pass reads the u16 symbols back whole
        if (mk_out.list) {
            const int64_t RB = (int64_t)I.rowbytes + 1, s0 = ob + cnt;
            const int64_t y0 = s0 / RB;
            int64_t y = y0, c = s0 - y0 * RB + x;
            while (c >= RB) { c -= RB; ++y; }
            uint32_t mm = 0;  // bit i: position s0 + x + 64 i holds a marker (or an invalid symbol)
            for (uint32_t i = 0, q = (uint32_t)x; q < tot; ++i, q += 64) {
                const uint32_t v = s_ring[(uint32_t)(s0 + q) & M];
                if (v >= 256u) mm |= 1u << i;
                else if (c == 0) I.ft[y] = (uint8_t)v;
                else ((IK_GLOBAL uint8_t*)I.dst)[(size_t)y * I.pitch + (size_t)(c - 1)] = (uint8_t)v;
                c += 64;
                while (c >= RB) { c -= RB; ++y; }
            }
            const uint32_t nmk = (uint32_t)__builtin_popcount(mm), incl = wave_incl_scan_dpp(nmk);
            const uint32_t tot_mk = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            if (tot_mk) {
                // one of kMarkLists sub-lists by unit (one counter per list: a single
                // counter for the whole batch serialised ~8 M atomics on one address)
                const uint32_t sl = (uint32_t)li % kMarkLists, scap = mk_out.cap / kMarkLists;
                uint32_t base = 0;
                if (x == 63) base = atomicAdd(mk_out.count + sl, tot_mk);
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, 63) + incl - nmk;
                IK_GLOBAL uint64_t* const out = (IK_GLOBAL uint64_t*)(mk_out.list + (size_t)sl * scap);
                while (mm) {
                    const uint32_t i = (uint32_t)__builtin_ctz(mm);
                    mm &= mm - 1u;
                    if (base < scap) out[base] = ((uint64_t)L.img << 40) | (uint64_t)(s0 + x + 64 * i);
                    ++base;
                }
            }
        }
        __syncthreads();
        IK_XP(4);
        cnt += tot;
        t = t2;
        w = wn;
        if (__ballot(bad)) { bad = true; break; }
    }
    if (x == 0) {
        status[2 * li] = (!bad && cnt == oe - ob) ? 0 : -1;
        status[2 * li + 1] = (int)((clock64() - c0) >> 10);  // profile: clock ticks / 1024
#ifdef IK_EXP_PROF
        xprof[0] = clock64() - c0;
        for (int k = 0; k < 8; ++k) atomicAdd(&g_exp_prof[k], (unsigned long long)xprof[k]);
#endif
    }
}

// ---- expand units ---------------------------------------------------------------
// One thread per verified lane of the wave decoder: its units' output offsets into
// the image's unit offset table (ascending, resolve's lane_obase), unit -> lane,
// and the page table entries of the pages whose first byte lies in each unit.
__global__ __launch_bounds__(256) void k_png_units(const PngImgDev* imgs, const PngLaneDev* lanes, int n,
                                                   const uint2* units, uint32_t* ulane) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const PngLaneDev L = lanes[i];
    const PngImgDev I = imgs[L.img];
    IK_GLOBAL int64_t* const uob = (IK_GLOBAL int64_t*)I.obase;
    IK_GLOBAL int* const pages = (IK_GLOBAL int*)I.page_lane;
    const IK_GLOBAL uint2* R = (const IK_GLOBAL uint2*)(units + L.pbase);
    const uint32_t base = L.ubase - L.uimg;  // the lane's first unit within its image
    constexpr int64_t P = 1ll << kPngPageShift;
    int64_t o = L.obase + (int64_t)R[0].y;
    for (uint32_t b = 0; b < L.nunits; ++b) {
        const int64_t oe = b + 1 < L.nunits ? L.obase + (int64_t)R[b + 1].y : L.obase + (int64_t)L.out_len;
        uob[base + b] = o;
        ulane[L.ubase + b] = (uint32_t)i;
        for (int64_t pg = (o + P - 1) >> kPngPageShift; (pg << kPngPageShift) < oe; ++pg) pages[pg] = (int)(base + b);
        o = oe;
    }
}

// ---- window markers of the direct-rows expand -----------------------------------
// One thread per listed marker (a grid-stride loop: the count is on the device):
// its value followed through the earlier units (infl::resolve_at over the u16
// symbols, which expand still writes), into the row or the filter type.  Then one
// thread per row checks the filter types (png's error for > 4; bit 4: Average /
// Paeth rows, the unfilter's diagonal path).
__global__ __launch_bounds__(256) void k_png_marks(const PngImgDev* imgs, PngMarks mk, int* err) {
    // workgroups in kMarkLists groups, group g taking sub-list g % kMarkLists
    const uint32_t sl = blockIdx.x % kMarkLists, part = blockIdx.x / kMarkLists, parts = gridDim.x / kMarkLists;
    const uint32_t scap = mk.cap / kMarkLists, c = mk.count[sl];
    const uint32_t n = c < scap ? c : scap;
    const uint64_t* list = mk.list + (size_t)sl * scap;
    for (uint32_t i = part * 256 + threadIdx.x; i < n; i += parts * 256) {
        const uint64_t e = list[i];
        const int k = (int)(e >> 40);
        const int64_t pos = (int64_t)(e & ((1ull << 40) - 1));
        const PngImgDev I = imgs[k];
        const int v = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, pos);
        if (v < 0) {
            atomicOr(err + k, 2);
            continue;
        }
        const int64_t RB = (int64_t)I.rowbytes + 1, y = pos / RB, c = pos - y * RB;
        if (c == 0) I.ft[y] = (uint8_t)v;
        else ((IK_GLOBAL uint8_t*)I.dst)[(size_t)y * I.pitch + (size_t)(c - 1)] = (uint8_t)v;
    }
}

__global__ __launch_bounds__(256) void k_png_ftflags(const PngImgDev* imgs, const int2* rows, int nrows, int* err) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrows) return;
    const int2 ir = rows[r];
    const uint32_t v = imgs[ir.x].ft[ir.y];
    if (v > 4) atomicOr(err + ir.x, 1);
    else if (v >= 3) atomicOr(err + ir.x, 4);
}

// ---- resolve ------------------------------------------------------------------------
// thread = (16-byte chunk of a row, row, image); grid.y over rows of all images via
// a row table (image, row).  Window markers (~4 % of the symbols, near each
// decoder lane's start) are collected into an LDS list while the chunks are
// stored, and then followed by all the workgroup's threads at once, one marker
// per thread: a chunk's markers resolved by its own thread one after another
// held the whole row for a chain of dependent loads per marker.
constexpr int kResolveList = 4096;

__global__ __launch_bounds__(256) void k_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows,
                                                     int* err) {
    raise_priority();
    __shared__ uint32_t s_pos[kResolveList];  // marker positions in the row (byte index after the filter byte)
    __shared__ uint32_t s_cnt;
    const int rr = blockIdx.y * 65535 + blockIdx.x;  // row of the batch
    if (rr >= nrows) return;
    const int2 ir = rows[rr];
    const PngImgDev I = imgs[ir.x];
    const int y = ir.y;
    const int64_t rs = (int64_t)y * (I.rowbytes + 1);  // filter byte of row y
    __shared__ int64_t s_hlo, s_hhi;  // the output range of the unit holding the row's first symbol
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        int hl = I.page_lane[rs >> kPngPageShift];
        while (hl + 1 < I.nlanes && I.obase[hl + 1] <= rs) ++hl;
        s_hlo = I.obase[hl];
        s_hhi = hl + 1 < I.nlanes ? I.obase[hl + 1] : INT64_MAX;
        const int v = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, rs);
        I.ft[y] = (uint8_t)(v < 0 ? 255 : v);
        if (v < 0 || v > 4) atomicOr(err + ir.x, 1);
        else if (v >= 3) atomicOr(err + ir.x, 4);  // (Average / Paeth: the unfilter's diagonal path)
    }
    // (global address space: global_* ops, counted in vmcnt only, not flat_*)
    IK_GLOBAL uint8_t* const drow = (IK_GLOBAL uint8_t*)(I.dst + (size_t)y * I.pitch);
    for (int x0 = threadIdx.x * 16; x0 < I.rowbytes; x0 += 256 * 16) {
        const int64_t e0 = rs + 1 + x0;
        // 16 u16 symbols from 9 dwords in three loads (two dwordx4 at a dword-aligned
        // address, the u16 buffer is padded), shifted by one symbol when e0 is odd
        // (uniform over the row), then each output dword packs the low bytes of four
        // symbols with one v_perm
        const IK_GLOBAL uint32_t* w = (const IK_GLOBAL uint32_t*)(reinterpret_cast<const uint32_t*>(I.u16) + (e0 >> 1));
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 va = *reinterpret_cast<const IK_GLOBAL u4*>(w), vb = *reinterpret_cast<const IK_GLOBAL u4*>(w + 4);
        const uint32_t d[9] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w, w[8]};
        uint32_t e[8];
        if (e0 & 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) e[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], 2u);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) e[i] = d[i];
        }
        uint32_t mk = 0;  // bit i: symbol i is a window marker
#pragma unroll
        for (int i = 0; i < 8; ++i)
            mk |= ((e[i] & 0xFF00u) ? 1u : 0u) << (2 * i) | ((e[i] & 0xFF000000u) ? 1u : 0u) << (2 * i + 1);
        const int n = I.rowbytes - x0 < 16 ? I.rowbytes - x0 : 16;
        mk &= (1u << n) - 1u;
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = __builtin_amdgcn_perm(e[2 * k + 1], e[2 * k], 0x06040200u);
        if (mk) {
            // this thread's slots are [at, at + c): those inside the list are filled
            // (so the list never has holes), the rest resolve here
            uint32_t k = atomicAdd(&s_cnt, (uint32_t)__builtin_popcount(mk));
            while (mk) {
                const int i = __builtin_ctz(mk);
                mk &= mk - 1u;
                if (k < (uint32_t)kResolveList) {
                    s_pos[k++] = (uint32_t)(x0 + i);
                    continue;
                }
                const int rv = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, e0 + i);
                if (rv < 0) atomicOr(err + ir.x, 2);
                o[i >> 2] = (o[i >> 2] & ~(255u << (8 * (i & 3)))) | (((uint32_t)rv & 255u) << (8 * (i & 3)));
            }
        }
        *reinterpret_cast<IK_GLOBAL uint4*>(drow + x0) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();  // (also orders the chunk stores before the marker bytes below)
    const uint32_t cnt = s_cnt < (uint32_t)kResolveList ? s_cnt : (uint32_t)kResolveList;
    const int64_t hlo = s_hlo, hhi = s_hhi;
    for (uint32_t m = threadIdx.x; m < cnt; m += 256) {
        const uint32_t x = s_pos[m];
        // the first hop: a marker in the row's first unit resolves against its offset
        // without the page-table walk (then the general walk, from the source)
        const int64_t q = rs + 1 + (int64_t)x;
        int rv;
        if (q >= hlo && q < hhi) {
            const uint32_t mv = I.u16[q];
            const int64_t q2 = hlo - infl::kWindow + (int64_t)(mv & 0x7FFFu);
            rv = (mv & 0x8000u) && q2 >= 0 ? infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, q2) : -1;
        } else {
            rv = infl::resolve_at(I.u16, I.obase, I.nlanes, I.page_lane, kPngPageShift, q);
        }
        if (rv < 0) atomicOr(err + ir.x, 2);
        drow[x] = (uint8_t)rv;
    }
}

// ---- unfilter -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t lane0) {
    // lane l gets lane l-1's v; lane 0 gets lane0 (DPP wave_shr:1, bound_ctrl off)
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 255u; }

// One wave per 64-row band; an image's bands are spread over ceil(bands / 16)
// workgroups (16 waves each), so a batch fills the chip instead of one CU per
// image.  A band's first row needs the previous band's last row: that row's
// lane stores its chunks sc1 (written through) and, once per group of kUnfG
// steps, waits for them and sets the band's progress counter (sc1 store); the
// next band's lane 0 polls it (sc1) and loads the group's kUnfG chunks of the
// row above with sc1 loads -- MI355X_MICROARCH.md's measured cross-CU/XCD
// hand-off, without an agent release (its L2 write-back costs microseconds).
// Each lane's filtered bytes for the next group are prefetched a group ahead, so
// a step waits on memory only at group boundaries.  Workgroups take a ticket from
// a global counter when they start, and the ticket -- not blockIdx -- picks their
// (image, workgroup k of the image's K); wave w takes band w K + k, so the bands
// in flight spread over K CUs.  A band waits on the previous band, held by
// another of the image's workgroups: tickets go out in start order, so at most
// one image is partly started at any time, every other started image has all its
// workgroups running and finishes, and the CUs it frees start the rest -- no
// deadlock whatever the dispatch order (an image needs K <= the resident
// workgroups of the chip, 256 at one per CU; K = bands / 16).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kUnfG = 8;

typedef const __attribute__((address_space(1))) u32x4* gu32x4p;
// buffer intrinsics' cache-policy operand: sc1 (gfx940+ CPol::SC1) -- write-through
// stores, loads served by L2 past the CU's L1
constexpr int kCpolSc1 = 16;

// a wave-uniform 64-bit value in SGPRs (readfirstlane returns int: zero-extend
// each half, or a low word with bit 31 set sign-extends into the high word)
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// per-lane predictor masks (all-ones for the row's filter type): the byte loop
// selects by AND/OR, not by per-lane branches
struct FtMask {
    uint32_t sub, up, avg, paeth;
    __device__ explicit FtMask(uint32_t ft)
        : sub(ft == 1 ? ~0u : 0u), up(ft == 2 ? ~0u : 0u), avg(ft == 3 ? ~0u : 0u), paeth(ft == 4 ? ~0u : 0u) {}
};

template <int BPP, bool SWAR = false>
__device__ __forceinline__ void unfilter_chunk(const u32x4& rawv, const uint32_t (&up)[4], const uint32_t (&prevup)[4],
                                               const uint32_t (&prevcur)[4], const FtMask& fm, uint32_t (&o)[4]) {
    const uint32_t raw[4] = {rawv.x, rawv.y, rawv.z, rawv.w};
    if constexpr (SWAR && (BPP == 4 || BPP == 8)) {
        // a word at a time (ik_unfilter.h): the word BPP bytes back is one word earlier
        // (RGBA8) or two (8-byte pixels), so the chunk's chain is 4 or 2 words long
        constexpr int K = BPP / 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = k >= K ? o[k - K] : prevcur[4 + k - K];
            const uint32_t c = k >= K ? up[k - K] : prevup[4 + k - K];
            o[k] = unfilter_word(raw[k], a, up[k], c, fm.sub, fm.up, fm.avg, fm.paeth);
        }
        return;
    }
    o[0] = o[1] = o[2] = o[3] = 0;
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
        const uint32_t pred = (a & fm.sub) | (b & fm.up) | (((a + b) >> 1) & fm.avg) | (paeth & fm.paeth);
        const uint32_t v = (byte_of(raw, i) + pred) & 255u;
        o[i >> 2] |= v << (8 * (i & 3));
    }
}

#ifdef IK_UNF_PROF  // dev build: per-segment clock sums of k_png_unfilter (s_memtime; costs ~10 %)
__device__ unsigned long long g_unf_prof[8];
hipError_t png_unf_prof_read(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_unf_prof), sizeof(g_unf_prof));
    unsigned long long z[8] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_unf_prof), z, sizeof(z));
    return e;
}
#define IK_UNF_T(k) do { const unsigned long long _t = clock64(); up_[k] += _t - t_; t_ = _t; } while (0)
#else
#define IK_UNF_T(k) do { } while (0)
#endif

template <int BPP, bool SWAR>
__global__ __launch_bounds__(kPngUnfilterThreads) void k_png_unfilter(const PngImgDev* imgs, const int2* groups,
                                                                      const int* prog_base, unsigned* prog,
                                                                      unsigned* ticket) {
    raise_priority();
    constexpr int NW = kPngUnfilterThreads / 64, G = kUnfG;
    __shared__ int s_t;
    if (threadIdx.x == 0) s_t = (int)atomicAdd(ticket, 1u);
    __syncthreads();
    const int2 gk = groups[s_t];  // (image, workgroup of the image)
    const PngImgDev I = imgs[gk.x];
    if (png_unfilter_scan_path(BPP, I.rowbytes, *(const volatile int*)I.flags)) return;  // (k_png_unfilter_su's)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nch = (I.rowbytes + 15) >> 4;
    const int nbands = (I.H + 63) >> 6;
    // bands interleaved over the image's K workgroups: the ~(row chunks / 72)
    // bands in flight at a time sit on K CUs, not all on one; past 16 K bands a
    // wave takes its next band (in order: the lowest unfinished band always has
    // a finished predecessor)
    const int K = png_unfilter_groups(I.H);
    unsigned* pg = prog + prog_base[gk.x];
#ifdef IK_UNF_PROF
    unsigned long long up_[6] = {0, 0, 0, 0, 0, 0}, t_ = clock64();
#endif
    for (int band = wave * K + gk.y; band < nbands; band += NW * K) {
        const int y = band * 64 + lane;
        const bool live = y < I.H;
        const FtMask fm(live ? I.ft[y] : 0u);
        const bool above = band > 0;
        uint32_t cur[4] = {0, 0, 0, 0}, up[4] = {0, 0, 0, 0};
        uint32_t prevcur[4] = {0, 0, 0, 0}, prevup[4] = {0, 0, 0, 0};  // last chunk (left context)
        // The image through a buffer descriptor: the lane's row offset and chunk in
        // voffset.  Every load and store here is an intrinsic the compiler sees, so
        // its own wait counts hold: the prefetch of the next group's chunks is waited
        // for only where those registers are first read.  (Round 3 issued the loads
        // as inline asm and "landed" them with an asm s_waitcnt; the register
        // allocator copied the destination registers before that wait -- v_mov of
        // registers still being loaded -- so a group could read the previous
        // group's bytes when its loads were slow: wrong bands in ~1 of 6 frames at
        // 64-frame batches, none at 8.)
        const uint64_t dbase = uniform_u64((uint64_t)(size_t)I.dst);
        const size_t ibytes = I.pitch * (size_t)I.H;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)dbase, (short)0, (int)(ibytes < 0x7fffffffu ? ibytes : 0x7fffffffu), 0x00020000);
        const uint32_t rowoff = (uint32_t)((size_t)(live ? y : 0) * I.pitch);
        auto fetch = [&](int s0, u32x4 (&r)[G]) {
#pragma unroll
            for (int t = 0; t < G; ++t) {
                const uint32_t off = rowoff + 16u * (uint32_t)min(max(s0 + t - lane, 0), nch - 1);
                r[t] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
            }
        };
        unsigned seen = 0;  // lane 0: the previous band's progress last read
        const int ngrp = (nch + 63 + G - 1) / G;
        // one group of G steps on the chunks in `rc`, the next group's prefetched into `rn`
        auto group = [&](int g, u32x4 (&rc)[G], u32x4 (&rn)[G]) {
            const int s0 = g * G;
            u32x4 ab[G];
#pragma unroll
            for (int t = 0; t < G; ++t) ab[t] = u32x4{0, 0, 0, 0};
            IK_UNF_T(0);
            // Wave-uniform control flow around every load and store (out-of-range
            // buffer offsets are dropped by the hardware instead of branching per lane),
            // so that the compiler's wait counts stay exact across the group loop.
            if (above && s0 < nch) {
                const unsigned need = (unsigned)min(s0 + G, nch);
                while (seen < need) {  // the whole wave polls lane 0's read of the flag
                    const unsigned v = __hip_atomic_load(pg + band - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    seen = (unsigned)__builtin_amdgcn_readfirstlane((int)v);
                    if (seen < need) __builtin_amdgcn_s_sleep(1);
                }
                // the row above, sc1 (L2-served, past this CU's L1): the hand-off's loads,
                // lane 0 only (the other lanes' offsets are out of range: zeros)
                const uint32_t aoff = lane == 0 ? (uint32_t)((size_t)(band * 64 - 1) * I.pitch) : 0x80000000u;
#pragma unroll
                for (int t = 0; t < G; ++t)
                    ab[t] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, (int)(aoff + 16u * (uint32_t)min(s0 + t, nch - 1)), 0, kCpolSc1));
            }
            IK_UNF_T(1);
            if (g + 1 < ngrp) fetch(s0 + G, rn);
#pragma unroll
            for (int t = 0; t < G; ++t) {
                const int j = s0 + t - lane;
                // up chunk: lane l-1's result of the previous step; lane 0: the row above
                uint32_t nup[4];
                nup[0] = wave_shr1(cur[0], ab[t].x);
                nup[1] = wave_shr1(cur[1], ab[t].y);
                nup[2] = wave_shr1(cur[2], ab[t].z);
                nup[3] = wave_shr1(cur[3], ab[t].w);
                const bool act = live && j >= 0 && j < nch;
                if (act) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) { prevup[k] = up[k]; up[k] = nup[k]; prevcur[k] = cur[k]; }
                    if (j == 0) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) { prevup[k] = 0; prevcur[k] = 0; }
                    }
                    uint32_t o[4];
                    unfilter_chunk<BPP, SWAR>(rc[t], up, prevup, prevcur, fm, o);
#pragma unroll
                    for (int k = 0; k < 4; ++k) cur[k] = o[k];
                }
                // every lane issues the store; an inactive lane's offset is out of range (dropped)
                const u32x4 ov = {cur[0], cur[1], cur[2], cur[3]};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, ov),
                                                       rs, (int)(act ? rowoff + 16u * (uint32_t)j : 0x80000000u), 0,
                                                       kCpolSc1);
            }
            IK_UNF_T(2);
            // the band's last row publishes the chunks it finished in this group
            const int jl = s0 + G - 1 - 63;
            if (jl >= 0 && band * 64 + 63 < I.H) {  // (wave-uniform)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // lane 63's sc1 stores have completed
                if (lane == 63)
                    __hip_atomic_store(pg + band, (unsigned)min(jl + 1, nch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            IK_UNF_T(3);
        };
        // ping-pong between two register sets, no copies: the compiler's wait for a
        // group's chunks sits at their first read, a group after their loads went out
        u32x4 ra[G], rb[G];
        fetch(0, ra);
        for (int g = 0; g < ngrp; g += 2) {
            group(g, ra, rb);
            if (g + 1 < ngrp) group(g + 1, rb, ra);
        }
    }
#ifdef IK_UNF_PROF
    if (lane == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_unf_prof[k], up_[k]);
        atomicAdd(&g_unf_prof[7], 1ull);
    }
#endif
}

// ---- unfilter, scan path ----------------------------------------------------------
// RGBA8 images of None / Sub / Up rows only (png_unfilter_scan_path): a segment is a
// None or Sub row (or row 0) and the Up rows under it; segments are independent.
// kSuRanges workgroups per image, workgroup j taking the segments that start in its
// slice of rows (and following each to its end, past the slice if need be).  A
// thread owns 4 consecutive 16-byte chunks (16 pixels) of the row: an Up row adds
// the row above byte-wise (kept in registers), a Sub row is a byte-wise prefix sum
// per channel -- 4-byte pixels, so one SWAR word per pixel: in the thread, across
// the wave (DPP), across the workgroup's 4 waves (LDS).
__device__ __forceinline__ uint32_t add_bytes(uint32_t a, uint32_t b) {  // four independent mod-256 sums
    return ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
}
__device__ __forceinline__ uint32_t wave_scan_bytes(uint32_t v) {  // inclusive, add_bytes
    v = add_bytes(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));  // row_shr:1
    v = add_bytes(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));  // row_shr:2
    v = add_bytes(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));  // row_shr:4
    v = add_bytes(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = add_bytes(r0, (uint32_t)__builtin_amdgcn_readlane((int)v, 31));
    const uint32_t r2 = add_bytes(r1, (uint32_t)__builtin_amdgcn_readlane((int)v, 47));
    const int row = (int)(threadIdx.x & 63) >> 4;
    return add_bytes(v, row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}

// CH chunks per thread: kSuChunks for rows up to 4,096 pixels, kSuChunksWide for
// rows up to 8,192 (each launch takes its own images of the batch).
template <int CH>
__global__ __launch_bounds__(kSuThreads) void k_png_unfilter_su(const PngImgDev* imgs, int nimg) {
    raise_priority();
    constexpr int kSuChunks = CH;
    __shared__ uint32_t s_w[kSuThreads / 64];
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int im = (int)blockIdx.x / kSuRanges, jr = (int)blockIdx.x % kSuRanges;
    if (im >= nimg) return;
    const PngImgDev I = imgs[im];
    if (!png_unfilter_scan_path(4, I.rowbytes, *(const volatile int*)I.flags)) return;
    const int H = I.H, nch = (I.rowbytes + 15) >> 4;
    // (wave-uniform) the narrow kernel takes rows of <= kSuThreads * 4 chunks, the wide one the rest
    if ((nch <= kSuThreads * ::ik::kSuChunks) != (CH == ::ik::kSuChunks)) return;
    const int tid = threadIdx.x, wv = tid >> 6;
    const int c0 = tid * kSuChunks;  // this thread's first chunk
    const int y1 = (int)((int64_t)H * (jr + 1) / kSuRanges);
    int y = (int)((int64_t)H * jr / kSuRanges);
    const IK_GLOBAL uint8_t* ft = (const IK_GLOBAL uint8_t*)I.ft;
    while (y < y1 && y != 0 && ft[y] > 1) ++y;  // (rows of a segment that started above belong to its workgroup)
    while (y < y1) {
        uint32_t prev[4 * kSuChunks];
#pragma unroll
        for (int k = 0; k < 4 * kSuChunks; ++k) prev[k] = 0;
        int r = y;
        do {
            const uint32_t f = ft[r];
            IK_GLOBAL uint8_t* row = (IK_GLOBAL uint8_t*)(I.dst + (size_t)r * I.pitch);
            uint32_t w[4 * kSuChunks];
#pragma unroll
            for (int i = 0; i < kSuChunks; ++i) {
                const u4 v = c0 + i < nch ? *(const IK_GLOBAL u4*)(row + 16 * (c0 + i)) : u4{0, 0, 0, 0};
                w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
            }
            if (f == 2) {
#pragma unroll
                for (int k = 0; k < 4 * kSuChunks; ++k) w[k] = add_bytes(w[k], prev[k]);
            } else if (f == 1) {  // (uniform: the whole workgroup reads the same filter type)
#pragma unroll
                for (int k = 1; k < 4 * kSuChunks; ++k) w[k] = add_bytes(w[k], w[k - 1]);
                const uint32_t incl = wave_scan_bytes(w[4 * kSuChunks - 1]);
                uint32_t carry = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xF, 0xF, true);  // wave_shr:1
                if ((tid & 63) == 63) s_w[wv] = incl;
                __syncthreads();
                for (int q = 0; q < wv; ++q) carry = add_bytes(carry, s_w[q]);
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 4 * kSuChunks; ++k) w[k] = add_bytes(w[k], carry);
            }
#pragma unroll
            for (int i = 0; i < kSuChunks; ++i)
                if (c0 + i < nch) *(IK_GLOBAL u4*)(row + 16 * (c0 + i)) = u4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
#pragma unroll
            for (int k = 0; k < 4 * kSuChunks; ++k) prev[k] = w[k];
            ++r;
        } while (r < H && ft[r] == 2);
        y = r;
    }
}

hipError_t launch_png_unfilter_su(const PngImgDev* imgs, int nimg, hipStream_t s) {
    if (nimg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_unfilter_su<kSuChunks>, dim3(nimg * kSuRanges), dim3(kSuThreads), 0, s, imgs, nimg);
    hipLaunchKernelGGL(k_png_unfilter_su<kSuChunksWide>, dim3(nimg * kSuRanges), dim3(kSuThreads), 0, s, imgs, nimg);
    return hipGetLastError();
}

// ---- small transfers through the compute queue ---------------------------------------
__global__ __launch_bounds__(256) void k_copy_words(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                    size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_copy_words(const uint32_t* src, uint32_t* dst, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const size_t blocks = std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_copy_words, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, n);
    return hipGetLastError();
}

// ---- gather + CRC -----------------------------------------------------------------
// The upload stage DMAs whole PNG files into the raw area; this pass assembles
// each file's zlib stream from its IDAT payloads (and the zero padding after it)
// and computes the CRC-32 png checks on every chunk, so the host neither copies
// nor checksums the compressed bytes.  One 256-thread workgroup per piece of
// <= 64 KiB; thread t copies and checksums bytes [256 t, 256 t + 256) of the
// piece (dword stores once the destination is aligned, the source words
// realigned with v_alignbyte), then the workgroup joins the 256 partial CRCs in
// a tree (ik_crc.h: crc(A || B) = crc(A) x^(8 |B|) + crc(B)).
struct CrcOps {
    uint32_t x2n[32];    // x^(2^k) mod P
    uint32_t level[8];   // x^(8 * 256 * 2^k): the join operator of full subtrees at tree level k
    uint32_t piece;      // x^(8 * kPngGatherPiece): the join operator of a full piece
    uint32_t crc_idat;   // finished CRC of the chunk type "IDAT" (the first 4 bytes a chunk CRC covers)
};

__global__ __launch_bounds__(256) void k_png_gather(uintptr_t raw, uint8_t* __restrict__ stream,
                                                    const PngGatherPiece* __restrict__ pieces,
                                                    uint32_t* __restrict__ piece_crc, CrcOps ops) {
    __shared__ uint32_t t[1024];
    __shared__ uint32_t s_crc[256], s_len[256];
    const int tid = (int)threadIdx.x;
    t[tid] = crc::table_entry((uint32_t)tid);
    __syncthreads();
#pragma unroll
    for (int sl = 1; sl < 4; ++sl) {
        const uint32_t prev = t[256 * (sl - 1) + tid];
        t[256 * sl + tid] = (prev >> 8) ^ t[prev & 255u];
        __syncthreads();
    }
    const PngGatherPiece P = pieces[blockIdx.x];
    const uint32_t b0 = 256u * (uint32_t)tid;
    const uint32_t len = P.len > b0 ? (P.len - b0 < 256u ? P.len - b0 : 256u) : 0u;
    uint32_t c = ~0u;
    IK_GLOBAL uint8_t* dp = (IK_GLOBAL uint8_t*)(stream + P.dst + b0);
    if (len && P.src == kPngNoSrc) {
        for (uint32_t i = 0; i < len; ++i) dp[i] = 0;
    } else if (len) {
        const IK_GLOBAL uint8_t* sp = (const IK_GLOBAL uint8_t*)(raw + (uintptr_t)(P.src + b0));
        uint32_t i = 0;
        const uint32_t mis = (uint32_t)((uintptr_t)dp & 3u);
        const uint32_t pre = mis ? (4u - mis < len ? 4u - mis : len) : 0u;
        for (; i < pre; ++i) {
            const uint32_t b = sp[i];
            dp[i] = (uint8_t)b;
            c = crc::step_byte(c, b, t);
        }
        const uint32_t nw = (len - i) >> 2;
        if (nw) {
            const uintptr_t sa = (uintptr_t)(sp + i);
            const uint32_t sh = (uint32_t)(sa & 3u);
            const IK_GLOBAL uint32_t* ws = reinterpret_cast<const IK_GLOBAL uint32_t*>(sa - sh);
            IK_GLOBAL uint32_t* wd = reinterpret_cast<IK_GLOBAL uint32_t*>(dp + i);
            uint32_t lo = ws[0];
            uint32_t k = 0;
            // eight words at a time: the loads are independent of the CRC chain
            for (; k + 8 <= nw; k += 8) {
                uint32_t in[9];
                in[0] = lo;
#pragma unroll
                for (int u = 1; u <= 8; ++u) in[u] = sh ? ws[k + u] : (u < 8 ? ws[k + u] : 0u);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t v = sh ? __builtin_amdgcn_alignbyte(in[u + 1], in[u], sh) : in[u];
                    wd[k + u] = v;
                    c = crc::step_word(c, v, t);
                }
                lo = sh ? in[8] : (k + 8 < nw ? ws[k + 8] : 0u);
            }
            for (; k < nw; ++k) {
                const uint32_t hi = sh ? ws[k + 1] : 0u;
                const uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
                wd[k] = v;
                c = crc::step_word(c, v, t);
                lo = sh ? hi : (k + 1 < nw ? ws[k + 1] : 0u);
            }
            i += 4u * nw;
        }
        for (; i < len; ++i) {
            const uint32_t b = sp[i];
            dp[i] = (uint8_t)b;
            c = crc::step_byte(c, b, t);
        }
    }
    s_crc[tid] = ~c;  // finished CRC of this thread's bytes (0 for none)
    s_len[tid] = len;
    __syncthreads();
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
        const int stride = 1 << k;
        if ((tid & (2 * stride - 1)) == 0) {
            const uint32_t rl = s_len[tid + stride];
            if (rl) {
                const uint32_t op = rl == (256u << k) ? ops.level[k] : crc::x8n(rl, ops.x2n);
                s_crc[tid] = crc::combine_op(s_crc[tid], s_crc[tid + stride], op);
                s_len[tid] += rl;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        piece_crc[2 * blockIdx.x] = s_crc[0];
        piece_crc[2 * blockIdx.x + 1] = s_len[0];
    }
}

// one thread per IDAT chunk: join "IDAT" and its pieces, compare with the stored CRC
__global__ __launch_bounds__(256) void k_png_crc_check(uintptr_t raw,
                                                       const PngCrcChunk* __restrict__ chunks, int nchunks,
                                                       const uint32_t* __restrict__ piece_crc, int* err, CrcOps ops) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= nchunks) return;
    const PngCrcChunk C = chunks[i];
    uint32_t c = ops.crc_idat;
    for (uint32_t p = C.piece0; p < C.piece0 + C.npieces; ++p) {
        const uint32_t len = piece_crc[2 * p + 1];
        const uint32_t op = len == kPngGatherPiece ? ops.piece : crc::x8n(len, ops.x2n);
        c = crc::combine_op(c, piece_crc[2 * p], op);
    }
    const IK_GLOBAL uint8_t* q = (const IK_GLOBAL uint8_t*)(raw + (uintptr_t)C.crc_at);
    const uint32_t stored = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | (uint32_t)q[3];
    if (c != stored) err[C.stream] = 1;
}

static CrcOps crc_ops() {
    static const CrcOps o = [] {
        CrcOps r{};
        crc::x2n_table(r.x2n);
        for (int k = 0; k < 8; ++k) r.level[k] = crc::x8n((uint64_t)256 << k, r.x2n);
        r.piece = crc::x8n(kPngGatherPiece, r.x2n);
        uint32_t t[1024];
        for (uint32_t i = 0; i < 256; ++i) t[i] = crc::table_entry(i);
        for (int sl = 1; sl < 4; ++sl)
            for (int i = 0; i < 256; ++i) t[256 * sl + i] = (t[256 * (sl - 1) + i] >> 8) ^ t[t[256 * (sl - 1) + i] & 255u];
        uint32_t c = ~0u;
        for (const char ch : {'I', 'D', 'A', 'T'}) c = crc::step_byte(c, (uint8_t)ch, t);
        r.crc_idat = ~c;
        return r;
    }();
    return o;
}

hipError_t launch_png_gather(uintptr_t raw, uint8_t* stream, const PngGatherPiece* pieces, int npieces,
                             uint32_t* piece_crc, hipStream_t s) {
    if (npieces <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_gather, dim3((unsigned)npieces), dim3(256), 0, s, raw, stream, pieces, piece_crc,
                       crc_ops());
    return hipGetLastError();
}

hipError_t launch_png_crc_check(uintptr_t raw, const PngCrcChunk* chunks, int nchunks, const uint32_t* piece_crc,
                                int* err, hipStream_t s) {
    if (nchunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_crc_check, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s, raw, chunks,
                       nchunks, piece_crc, err, crc_ops());
    return hipGetLastError();
}

// ---- chunk walk of device-resident files ------------------------------------------
// One wave per file (PngWalkRec, ik_png.h).  The chunk chain is serial -- each
// length gives the next chunk's position -- so every lane follows it with the
// same (wave-uniform) loads; the lanes then copy a non-IDAT chunk's type, data and
// CRC into the side area together.  Mirrors parse_png's loop (ik_png_decode.cpp):
// chunks while 12 bytes remain, stop after IEND; a length past the file's end, a
// full record table or side area sends the file to the host decoder.
__global__ __launch_bounds__(64) void k_png_walk(const uint64_t* __restrict__ files, const uint64_t* __restrict__ lens,
                                                 PngWalkRec* __restrict__ recs, uint8_t* __restrict__ side,
                                                 int* __restrict__ out_n) {
    const int f = (int)blockIdx.x, lane = (int)threadIdx.x;
    const IK_GLOBAL uint8_t* b = (const IK_GLOBAL uint8_t*)(uintptr_t)files[f];
    const uint64_t n = lens[f];
    PngWalkRec* R = recs + (size_t)f * kPngWalkRecs;
    uint8_t* S = side + (size_t)f * kPngWalkSide;
    uint64_t pos = 8;
    uint32_t used = 0;
    int cnt = 0, st = 0;
    while (pos + 12 <= n) {
        uint8_t h[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) h[k] = b[pos + k];  // length, type, first 4 data (or CRC) bytes
        const uint32_t len = (uint32_t)h[0] << 24 | (uint32_t)h[1] << 16 | (uint32_t)h[2] << 8 | h[3];
        if ((uint64_t)len > n - pos - 12) { st = -3; break; }
        if (cnt == kPngWalkRecs) { st = -1; break; }
        const bool idat = h[4] == 'I' && h[5] == 'D' && h[6] == 'A' && h[7] == 'T';
        uint32_t so = ~0u;
        if (!idat || !len) {
            if (used + len + 8 > kPngWalkSide) { st = -2; break; }
            so = used;
            for (uint32_t i = (uint32_t)lane; i < len + 8; i += 64) S[so + i] = b[pos + 4 + i];
            used += (len + 8 + 3) & ~3u;
        }
        if (lane == 0) {
            PngWalkRec r;
            r.off = pos;
            r.len = len;
            r.side = so;
#pragma unroll
            for (int k = 0; k < 4; ++k) { r.type[k] = h[4 + k]; r.head[k] = h[8 + k]; }
            R[cnt] = r;
        }
        ++cnt;
        pos += 12 + (uint64_t)len;
        if (h[4] == 'I' && h[5] == 'E' && h[6] == 'N' && h[7] == 'D') break;
    }
    if (lane == 0) out_n[f] = st ? st : cnt;
}

// the first 64 bytes of each device-resident file (the host sniffs the format
// and the dimensions from them): one wave per file, a byte per lane
__global__ __launch_bounds__(64) void k_copy_heads(const uint64_t* __restrict__ files, const uint64_t* __restrict__ lens,
                                                   uint8_t* __restrict__ out) {
    const int f = (int)blockIdx.x, t = (int)threadIdx.x;
    const IK_GLOBAL uint8_t* b = (const IK_GLOBAL uint8_t*)(uintptr_t)files[f];
    out[64 * (size_t)f + t] = (uint64_t)t < lens[f] ? b[t] : 0;
}

hipError_t launch_copy_heads(const uint64_t* files, const uint64_t* lens, int n, uint8_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_copy_heads, dim3((unsigned)n), dim3(64), 0, s, files, lens, out);
    return hipGetLastError();
}

hipError_t launch_png_walk(const uint64_t* files, const uint64_t* lens, int n, PngWalkRec* recs, uint8_t* side,
                           int* out_n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_walk, dim3((unsigned)n), dim3(64), 0, s, files, lens, recs, side, out_n);
    return hipGetLastError();
}

// ---- EXPAND -------------------------------------------------------------------------
// png 0.18's EXPAND transformation (image 0.25.8 decodes with it: reference
// src/transform.rs:31): one thread per pixel of the unfiltered rows.  Palette
// index -> PLTE colour (an index past the palette: black) with tRNS alpha (255
// past tRNS); gray of 1/2/4 bits -> v * 255 / (2^d - 1); a gray level or RGB
// triple equal to the tRNS key -> alpha 0, else 255.  16-bit samples (L16 / La16
// / Rgb16 / Rgba16) -> native-endian u16, tRNS alpha 0 / 65535.
__global__ __launch_bounds__(256) void k_png_px(PngPxDev P) {
    __shared__ uint32_t pal[256];
    if (P.ctype == 3) pal[threadIdx.x] = P.pal[threadIdx.x];
    __syncthreads();
    const int x = (int)(blockIdx.x * 256 + threadIdx.x), y = (int)blockIdx.y;
    if (x >= P.w) return;
    const uint8_t* r = P.src + (size_t)y * P.sp;
    if (P.depth == 16) {  // big-endian samples -> native u16; a tRNS key match -> alpha 0, else 65535
        const int spp = P.ctype == 0 ? 1 : P.ctype == 2 ? 3 : P.ctype == 4 ? 2 : 4;
        const uint8_t* s = r + (size_t)2 * spp * x;
        uint16_t* o16 = reinterpret_cast<uint16_t*>(P.dst + (size_t)y * P.dp) + (size_t)x * P.out_c;
        bool key = P.out_c > spp;
#pragma unroll 4
        for (int k = 0; k < spp; ++k) {
            const int v = (int)s[2 * k] << 8 | s[2 * k + 1];
            o16[k] = (uint16_t)v;
            key = key && v == (P.ctype == 0 ? P.key : P.key_rgb[k]);
        }
        if (P.out_c > spp) o16[spp] = key ? 0 : 65535;
        return;
    }
    uint8_t* o = P.dst + (size_t)y * P.dp + (size_t)x * P.out_c;
    if (P.ctype == 2) {  // RGB + tRNS key
        const int R = r[3 * x], G = r[3 * x + 1], B = r[3 * x + 2];
        o[0] = (uint8_t)R; o[1] = (uint8_t)G; o[2] = (uint8_t)B;
        o[3] = (R == P.key_rgb[0] && G == P.key_rgb[1] && B == P.key_rgb[2]) ? 0 : 255;
        return;
    }
    int v;
    if (P.depth == 8) {
        v = r[x];
    } else {
        const int bit = x * P.depth;
        v = (r[bit >> 3] >> (8 - P.depth - (bit & 7))) & ((1 << P.depth) - 1);
    }
    if (P.ctype == 3) {
        const uint32_t c = pal[v];
        o[0] = (uint8_t)c; o[1] = (uint8_t)(c >> 8); o[2] = (uint8_t)(c >> 16);
        if (P.out_c == 4) o[3] = (uint8_t)(c >> 24);
    } else {
        o[0] = (uint8_t)(v * P.scale);
        if (P.out_c == 2) o[1] = v == P.key ? 0 : 255;
    }
}

hipError_t launch_png_px(const PngPxDev& px, hipStream_t s) {
    if (px.w <= 0 || px.h <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_px, dim3((unsigned)((px.w + 255) / 256), (unsigned)px.h), dim3(256), 0, s, px);
    return hipGetLastError();
}

// ---- launchers --------------------------------------------------------------------
hipError_t launch_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx, int n,
                           uint64_t chunk_bits, int64_t* cand, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_find, dim3(n), dim3(64), 0, s, imgs, chunk_img, chunk_idx, n, chunk_bits, cand);
    return hipGetLastError();
}

hipError_t launch_png_decode(const PngImgDev* imgs, const PngLaneDev* lanes, const uint32_t* order, int n,
                             uint16_t* tok, infl::LaneResult* res, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((n + kPngInflateThreads - 1) / kPngInflateThreads);
    hipLaunchKernelGGL(k_png_decode, grid, dim3(kPngInflateThreads), 0, s, imgs, lanes, order, n, tok, res);
    return hipGetLastError();
}

hipError_t launch_png_marks(const PngImgDev* imgs, PngMarks mk, const int2* rows, int nrows, int* err, hipStream_t s) {
    hipLaunchKernelGGL(k_png_marks, dim3(8 * kMarkLists), dim3(256), 0, s, imgs, mk, err);
    if (nrows > 0) hipLaunchKernelGGL(k_png_ftflags, dim3((nrows + 255) / 256), dim3(256), 0, s, imgs, rows, nrows, err);
    return hipGetLastError();
}

hipError_t launch_png_expand(const PngImgDev* imgs, const PngLaneDev* lanes, int n, const uint16_t* tok, int* status,
                             hipStream_t s, const uint2* pieces, const uint2* units, const uint32_t* ulane, PngMarks mk) {
    if (n <= 0) return hipSuccess;
    if ((units != nullptr) != (ulane != nullptr) || (units && !pieces)) return hipErrorInvalidValue;
    if (mk.list && !pieces) return hipErrorInvalidValue;  // (the direct rows: the wave decoder's tokens only)
    // (the lane decoder's tokens may carry literal tables; the wave decoder's never do)
    if (pieces)
        hipLaunchKernelGGL(k_png_expand8<false>, dim3(n), dim3(64), 0, s, imgs, lanes, n, tok, status, pieces, units, ulane, mk);
    else
        hipLaunchKernelGGL(k_png_expand8<true>, dim3(n), dim3(64), 0, s, imgs, lanes, n, tok, status, pieces, units, ulane, mk);
    return hipGetLastError();
}

hipError_t launch_png_wave(const PngImgDev* imgs, const PngLaneDev* lanes, const uint32_t* order, int n,
                           uint16_t* tok, uint2* pieces, uint2* units, infl::LaneResult* res, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_wave, dim3(n), dim3(64), 0, s, imgs, lanes, order, n, tok, pieces, units, res);
    return hipGetLastError();
}

hipError_t launch_png_units(const PngImgDev* imgs, const PngLaneDev* lanes, int n, const uint2* units,
                            uint32_t* ulane, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_png_units, dim3((n + 255) / 256), dim3(256), 0, s, imgs, lanes, n, units, ulane);
    return hipGetLastError();
}

hipError_t launch_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows, int* err, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    const dim3 grid(nrows < 65535 ? nrows : 65535, (nrows + 65534) / 65535);
    hipLaunchKernelGGL(k_png_resolve, grid, dim3(256), 0, s, imgs, rows, nrows, err);
    return hipGetLastError();
}

// 4- and 8-byte pixels (RGBA8, La16, Rgba16) take the word-at-a-time chunk (ik_unfilter.h)
hipError_t launch_png_unfilter(const PngImgDev* imgs, const int2* groups, int ngroups, const int* prog_base,
                               unsigned* prog, unsigned* ticket, int bpp, hipStream_t s) {
    if (ngroups <= 0) return hipSuccess;
    const dim3 grid(ngroups), block(kPngUnfilterThreads);
#define IK_UNF(B, W) hipLaunchKernelGGL((k_png_unfilter<B, W>), grid, block, 0, s, imgs, groups, prog_base, prog, ticket)
    switch (bpp) {
    case 1: IK_UNF(1, false); break;
    case 2: IK_UNF(2, false); break;
    case 3: IK_UNF(3, false); break;
    case 4: IK_UNF(4, true); break;
    case 6: IK_UNF(6, false); break;
    case 8: IK_UNF(8, true); break;
    default: return hipErrorInvalidValue;
    }
#undef IK_UNF
    return hipGetLastError();
}

}  // namespace ik
