// ik_jpeg_enc.hip -- baseline Huffman coding of the JPEG branch of encode_image
// (reference src/transform.rs:121-128 -> image 0.25.8 JpegEncoder) on the GPU,
// byte for byte the host coder of ik_codec.cpp (jpeg_write): standard tables,
// 4:4:4 MCUs of Y, Cb, Cr, DC predicted from the previous MCU, 0xFF stuffing,
// pad_byte's seven one-bits with the leftover bits dropped.
//
// One workgroup per image.  Every block's code length is independent (its DC
// difference reads the previous MCU's DC straight from the coefficients), so:
//   1. each thread sums the bit lengths of a contiguous run of blocks;
//   2. a workgroup scan turns them into bit offsets;
//   3. each thread re-codes its run into a zeroed big-endian word buffer,
//      OR-ing 32-bit words (atomics only at the run's shared edge words);
//   4. a scan of the 0xFF counts places every byte (0xFF -> 0xFF 0x00), and the
//      stuffed stream is written with 16-byte stores into the destination (pinned
//      host memory in the pipeline).
#include <hip/hip_runtime.h>

#include "ik_internal.h"

namespace ik {
namespace {

constexpr int kEncThreads = 1024;

constexpr uint8_t kZigE[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                      12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                      35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                      58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__device__ __forceinline__ void coef_bits_dev(int c, int& nb, uint32_t& val) {
    const uint32_t mag = (uint32_t)(c < 0 ? -c : c);
    nb = mag ? 32 - __clz(mag) : 0;
    const uint32_t mask = (1u << nb) - 1u;
    val = (c < 0 ? (uint32_t)(c - 1) : (uint32_t)c) & mask;
}

// Sink that only counts bits, or writes them MSB-first into `words` starting at
// bit `pos` (the thread's run; edge words are shared with neighbouring runs).
struct BitSink {
    uint32_t* words;
    unsigned long long pos;  // next bit
    unsigned long long acc;  // pending bits, MSB-aligned at bit 63
    int n;                   // pending bit count (< 32 after a flush)
    unsigned long long first_word, last_word;  // shared words of this run: atomics
    bool count_only;
    __device__ __forceinline__ void flush_word() {
        const unsigned long long w = (pos - (unsigned long long)n) >> 5;  // word of the oldest pending bit
        const uint32_t v = (uint32_t)(acc >> 32);
        if (w == first_word || w == last_word) atomicOr(&words[w], v);
        else words[w] = v;
        acc <<= 32;
        n -= 32;
    }
    __device__ __forceinline__ void put(uint32_t bits, int size) {
        if (count_only) {
            pos += (unsigned)size;
            return;
        }
        if (!size) return;
        acc |= (unsigned long long)(bits & ((1u << size) - 1u)) << (64 - n - size);
        n += size;
        pos += (unsigned)size;
        if (n >= 32) flush_word();
    }
    __device__ __forceinline__ void finish() {
        if (count_only || n <= 0) return;
        const unsigned long long w = (pos - (unsigned long long)n) >> 5;
        atomicOr(&words[w], (uint32_t)(acc >> 32));
        if (n > 32) atomicOr(&words[w + 1], (uint32_t)(acc & 0xffffffffu));
        n = 0;
    }
};

// one block of MCU m, component c (coef: [mcu][3][64] natural order, 128-B blocks,
// 16-B aligned).  The block comes in with eight 16-byte loads and the zigzag walk
// is unrolled, so every coefficient is a register with a compile-time index (one
// scattered 2-byte load per coefficient was the kernel's cost).
__device__ __forceinline__ void code_block(BitSink& b, const int16_t* __restrict__ coef, long long blk, const uint32_t* __restrict__ huff) {
    const long long m = blk / 3;
    const int c = (int)(blk - m * 3);
    const int16_t* p = coef + (m * 3 + c) * 64;
    const int prev = m ? coef[((m - 1) * 3 + c) * 64] : 0;
    uint32_t wv[32];
    const uint4* p4 = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint4 t = p4[j];
        wv[4 * j] = t.x; wv[4 * j + 1] = t.y; wv[4 * j + 2] = t.z; wv[4 * j + 3] = t.w;
    }
    auto coefk = [&](int k) -> int { return (int)(int16_t)(wv[k >> 1] >> (16 * (k & 1))); };
    const uint32_t* dc = huff + (c ? 2 : 0) * 256;
    const uint32_t* ac = huff + (c ? 3 : 1) * 256;
    int nb;
    uint32_t v;
    coef_bits_dev(coefk(0) - prev, nb, v);
    b.put(dc[nb] >> 8, dc[nb] & 0xff);
    b.put(v, nb);
    int zr = 0;
#pragma unroll
    for (int i = 1; i < 64; ++i) {
        const int x = coefk(kZigE[i]);
        if (x == 0) { ++zr; continue; }
        while (zr > 15) { b.put(ac[0xF0] >> 8, ac[0xF0] & 0xff); zr -= 16; }
        coef_bits_dev(x, nb, v);
        const int sym = (zr << 4) | nb;
        b.put(ac[sym] >> 8, ac[sym] & 0xff);
        b.put(v, nb);
        zr = 0;
    }
    if (coefk(kZigE[63]) == 0) b.put(ac[0] >> 8, ac[0] & 0xff);
}

__device__ __forceinline__ unsigned long long block_scan_excl(unsigned long long v, unsigned long long* s_tmp, unsigned long long& total) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned long long inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
    }
    if (lane == 63) s_tmp[wv] = inc;
    __syncthreads();
    unsigned long long base = 0;
    total = 0;
    for (int k = 0; k < kEncThreads / 64; ++k) {
        if (k < wv) base += s_tmp[k];
        total += s_tmp[k];
    }
    __syncthreads();
    return base + inc - v;
}

}  // namespace

__global__ __launch_bounds__(kEncThreads) void k_jpeg_huff_enc(JpegEncArgs a) {
    __shared__ uint32_t s_huff[4 * 256];
    __shared__ unsigned long long s_tmp[kEncThreads / 64];
    const int img = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < 4 * 256; i += kEncThreads) s_huff[i] = a.huff[i];
    const int16_t* coef = a.coef + (size_t)img * a.coef_img_stride;
    uint32_t* words = reinterpret_cast<uint32_t*>(a.work + (size_t)img * a.work_img_bytes);
    uint8_t* stage = a.work + (size_t)img * a.work_img_bytes + a.words_bytes;
    __syncthreads();
    const long long nblk = (long long)a.nmcu * 3;
    const long long per = (nblk + kEncThreads - 1) / kEncThreads;
    const long long b0 = min((long long)tid * per, nblk), b1 = min(b0 + per, nblk);
    // 1. bit lengths
    BitSink cnt{words, 0, 0, 0, 0, 0, true};
    for (long long k = b0; k < b1; ++k) code_block(cnt, coef, k, s_huff);
    unsigned long long total_bits;
    const unsigned long long off = block_scan_excl(cnt.pos, s_tmp, total_bits);
    const unsigned long long T = total_bits + 7;  // + pad_byte's 7 one-bits
    const unsigned long long nbytes = T / 8;       // leftover (< 8) bits are dropped
    if (nbytes * 2 > a.out_cap || (T + 31) / 32 * 4 > a.words_bytes) {  // worst case does not fit: host path
        if (tid == 0) a.out_len[img] = 0xffffffffu;
        return;
    }
    // 2. zero the word buffer, then every run codes into it
    const unsigned long long nwords = (T + 31) / 32;
    for (unsigned long long i = tid; i < nwords; i += kEncThreads) words[i] = 0;
    __syncthreads();
    BitSink w{words, off, 0, 0, off >> 5, (off + cnt.pos) >> 5, false};
    w.n = (int)(off & 31);  // align the accumulator to word boundaries: leading zero bits
    w.acc = 0;
    for (long long k = b0; k < b1; ++k) code_block(w, coef, k, s_huff);
    w.finish();
    if (tid == 0) {  // pad_byte: seven one-bits at the end
        BitSink pb{words, total_bits, 0, (int)(total_bits & 31), total_bits >> 5, (total_bits + 7) >> 5, false};
        pb.put(0x7F, 7);
        pb.finish();
    }
    __syncthreads();
    // 3. byte stuffing: thread t owns bytes [t*bp, (t+1)*bp)
    const unsigned long long bp = (nbytes + kEncThreads - 1) / kEncThreads;
    const unsigned long long y0 = min((unsigned long long)tid * bp, nbytes), y1 = min(y0 + bp, nbytes);
    auto byte_at = [&](unsigned long long i) -> uint32_t { return (words[i >> 2] >> (24 - 8 * (i & 3))) & 0xffu; };
    unsigned long long ff = 0;
    for (unsigned long long i = y0; i < y1; ++i) ff += byte_at(i) == 0xFF;
    unsigned long long total_ff;
    const unsigned long long ffo = block_scan_excl(ff, s_tmp, total_ff);
    const unsigned long long out_bytes = nbytes + total_ff;
    unsigned long long o = y0 + ffo;
    for (unsigned long long i = y0; i < y1; ++i) {
        const uint32_t v = byte_at(i);
        stage[o++] = (uint8_t)v;
        if (v == 0xFF) stage[o++] = 0;
    }
    __syncthreads();
    // 4. into the destination, 16 bytes per store
    uint8_t* dst = a.out + (size_t)img * a.out_img_stride;
    const uint4* s4 = reinterpret_cast<const uint4*>(stage);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (unsigned long long i = tid; i < (out_bytes + 15) / 16; i += kEncThreads) d4[i] = s4[i];
    if (tid == 0) a.out_len[img] = (uint32_t)out_bytes;
}

hipError_t launch_jpeg_huff_enc(const JpegEncArgs& a, int n, hipStream_t s) {
    if (n <= 0 || (a.out_img_stride & 15) || (a.work_img_bytes & 15) || (a.words_bytes & 15) ||
        ((uintptr_t)a.coef & 15) || (a.coef_img_stride & 7))  // code_block's 16-byte loads
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_jpeg_huff_enc, dim3(n), dim3(kEncThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace ik
