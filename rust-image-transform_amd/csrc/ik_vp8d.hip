// ik_vp8d.hip -- device half of the GPU WebP (VP8 lossy) decoder (host half:
// ik_vp8d_host.cpp).  Three launches per batch of images, one workgroup per image for the
// first two:
//   k_vp8d_tokens  the token partitions (libwebp vp8_dec.c ParseResiduals / GetCoeffs /
//                  GetLargeValue): an inherently serial arithmetic decode, written
//                  wave-uniform so that it runs on the scalar unit (stream words and
//                  probability rows through scalar loads); the wave stores each MB's
//                  384 dequantised coefficients with 16-byte vector stores
//   k_vp8d_recon   prediction + inverse transforms + loop filter (frame_dec.c
//                  ReconstructRow / DoFilter): one wave per MB row, kReconWaves rows in
//                  flight, each two MBs behind the row above (the unfiltered top row,
//                  top-right samples and the filtered pixels its edges touch are final
//                  by then); per wave an LDS work area holds the MB being predicted and
//                  its filter window, so each pixel is written to HBM once per MB
//   k_vp8d_rgb     fancy chroma upsampling + YUV -> RGB (io_dec.c EmitFancyRGB,
//                  upsampling.c UPSAMPLE_FUNC, yuv.h VP8YuvToRgb) into the ik_image
#include <hip/hip_runtime.h>

#include "ik_vp8d_gpu.h"

namespace ik {
namespace vp8d {

namespace {

template <typename T>
using cptr = const __attribute__((address_space(4))) T*;  // read-only for the launch: scalar loads

#define WSYNC()                                                \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                       \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)

__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// the stream through scalar loads (the file is 16-byte aligned with 16 bytes of slack)
struct ScalarSrc {
    cptr<uint32_t> w;
    __device__ uint32_t be32(uint32_t i) const {
        const uint32_t k = i >> 2, sh = (i & 3) * 8;
        const uint64_t v = ((uint64_t)w[k + 1] << 32) | w[k];
        return __builtin_bswap32((uint32_t)(v >> sh));
    }
    __device__ uint32_t byte(uint32_t i) const { return (w[i >> 2] >> ((i & 3) * 8)) & 255; }
};

constexpr uint64_t nibbles(const uint8_t (&a)[16]) {
    uint64_t v = 0;
    for (int i = 0; i < 16; ++i) v |= (uint64_t)a[i] << (4 * i);
    return v;
}
constexpr uint8_t kZig[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr uint8_t kBand[16] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7};
constexpr uint64_t kZigP = nibbles(kZig);    // zigzag(n) as nibbles
constexpr uint64_t kBandP = nibbles(kBand);  // band(n), n < 16 (band(16) = 0)
static_assert(kZigP == 0xFEB7ADC963258410ull && kBandP == 0x7666666665463210ull, "scan tables");
__device__ __forceinline__ int zig(int n) { return (int)((kZigP >> (4 * n)) & 15); }
__device__ __forceinline__ int bandn(int n) { return n < 16 ? (int)((kBandP >> (4 * n)) & 15) : 0; }

struct alignas(16) PRow {  // one 16-byte probability row (11 used)
    uint32_t x, y, z, w;
};
__device__ __forceinline__ PRow ldrow(cptr<PRow> p) {
    PRow r;
    r.x = p->x;
    r.y = p->y;
    r.z = p->z;
    r.w = p->w;
    return r;
}
// byte i (a constant) of a probability row
template <int I>
__device__ __forceinline__ int pb(const PRow& r) {
    const uint32_t w = I < 4 ? r.x : I < 8 ? r.y : I < 12 ? r.z : r.w;
    return (int)((w >> ((I & 3) * 8)) & 255);
}

__constant__ uint32_t kCat[4][12] = {{173, 148, 140, 0},
                                     {176, 155, 140, 135, 0},
                                     {180, 157, 141, 134, 130, 0},
                                     {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0}};

struct TokCtx {
    BitReader br;
    ScalarSrc src;
    cptr<PRow> rows;  // [type][band][ctx] probability rows
};

__device__ __forceinline__ int bit(TokCtx& t, int p) { return br_bit(t.br, t.src, p); }

__device__ int large_value(TokCtx& t, const PRow& r) {  // GetLargeValue
    int v;
    if (!bit(t, pb<3>(r))) {
        v = !bit(t, pb<4>(r)) ? 2 : 3 + bit(t, pb<5>(r));
    } else if (!bit(t, pb<6>(r))) {
        if (!bit(t, pb<7>(r))) {
            v = 5 + bit(t, 159);
        } else {
            v = 7 + 2 * bit(t, 165);
            v += bit(t, 145);
        }
    } else {
        const int b1 = bit(t, pb<8>(r));
        const int b0 = bit(t, b1 ? pb<10>(r) : pb<9>(r));
        const int cat = 2 * b1 + b0;
        cptr<uint32_t> tab = (cptr<uint32_t>)kCat[cat];
        v = 0;
        for (int k = 0; tab[k]; ++k) v += v + bit(t, (int)tab[k]);
        v += 3 + (8 << cat);
    }
    return v;
}

// GetCoeffs: tokens from position n of one block into out[] (LDS, lane 0 stores);
// returns the position after the last token; *dc: the stored value of position 0
__device__ int get_coeffs(TokCtx& t, int type, int ctx, int dq0, int dq1, int n, int16_t* out, int lane, int* dc) {
    PRow r = ldrow(t.rows + (type * 8 + bandn(n)) * 3 + ctx);
    for (; n < 16; ++n) {
        if (!bit(t, pb<0>(r))) return n;
        while (!bit(t, pb<1>(r))) {
            if (++n == 16) return 16;
            r = ldrow(t.rows + (type * 8 + bandn(n)) * 3);
        }
        int v, nctx;
        if (!bit(t, pb<2>(r))) {
            v = 1;
            nctx = 1;
        } else {
            v = large_value(t, r);
            nctx = 2;
        }
        const int s = bit(t, 0x80);
        const int16_t q = (int16_t)((s ? -v : v) * (n > 0 ? dq1 : dq0));
        if (n == 0) *dc = q;
        if (lane == 0) out[zig(n)] = q;
        r = ldrow(t.rows + (type * 8 + bandn(n + 1)) * 3 + nctx);
    }
    return 16;
}

}  // namespace

// One wave per image, all of it wave-uniform except the LDS traffic.  Contexts
// packed as libwebp's: bits 0-3 luma columns / rows, 4-5 U, 6-7 V, 8 the Y2 block.
__global__ __launch_bounds__(64) void k_vp8d_tokens(const DImg* __restrict__ imgs) {
    __shared__ uint4 cbuf4[48 + 2];  // the MB's 384 coefficients, then the Y2 block
    __shared__ uint16_t tnz[1024];   // top contexts per MB column
    __shared__ BitReader saved[8];   // one per token partition
    int16_t* const cb = reinterpret_cast<int16_t*>(cbuf4);
    int16_t* const dcb = cb + 384;
    const int lane = threadIdx.x;
    const cptr<DImg> di = (cptr<DImg>)imgs + blockIdx.x;
    const DFrame* const frg = di->fr;
    const cptr<DFrame> fr = (cptr<DFrame>)frg;
    const cptr<DMB> mbs = (cptr<DMB>)di->mbs;
    int16_t* const coef = di->coef;
    uint8_t* const flags = di->flags;
    const int mb_w = fr->mb_w, mb_h = fr->mb_h, nparts = fr->num_parts, use_skip = fr->use_skip;
    TokCtx t;
    t.src.w = (cptr<uint32_t>)di->file;
    t.rows = (cptr<PRow>)fr->proba;
    for (int i = lane; i < mb_w; i += 64) tnz[i] = 0;
    for (int p = 0; p < nparts; ++p) {
        br_init(t.br, t.src, fr->part_off[p], fr->part_end[p]);
        if (lane == 0) saved[p] = t.br;
    }
    __syncthreads();
    int err = 0;
    for (int mb_y = 0; mb_y < mb_h && !err; ++mb_y) {
        const int p = mb_y & (nparts - 1);
        {
            const BitReader& s = saved[p];
            t.br.value = ((uint64_t)(uint32_t)ufl((int)(uint32_t)(s.value >> 32)) << 32) |
                         (uint32_t)ufl((int)(uint32_t)s.value);
            t.br.range = (uint32_t)ufl((int)s.range);
            t.br.bits = ufl(s.bits);
            t.br.eof = ufl(s.eof);
            t.br.pos = (uint32_t)ufl((int)s.pos);
            t.br.end = (uint32_t)ufl((int)s.end);
        }
        uint32_t l = 0;
        for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
            const int mb = mb_y * mb_w + mb_x;
            const cptr<DMB> m = mbs + mb;
            const int is_i4 = m->is_i4, skip = use_skip ? m->skip : 0;
            if (lane < 50) cbuf4[lane] = make_uint4(0, 0, 0, 0);
            WSYNC();
            uint32_t tc = (uint32_t)ufl(tnz[mb_x]);
            int any = 0;
            if (!skip) {
                const cptr<DSeg> q = (cptr<DSeg>)&frg->seg[m->seg];
                int first = 0, ytype = 3, dc_any = 0;
                if (!is_i4) {  // the Y2 block, then its inverse WHT into the blocks' DCs
                    int dcv = 0;
                    const int ctx = ((tc >> 8) & 1) + ((l >> 8) & 1);
                    const int nz = get_coeffs(t, 1, ctx, q->y2[0], q->y2[1], 0, dcb, lane, &dcv);
                    const uint32_t b = nz > 0;
                    tc = (tc & ~0x100u) | b << 8;
                    l = (l & ~0x100u) | b << 8;
                    WSYNC();
                    if (lane == 0) vp8x::itransform_wht(dcb, cb);
                    WSYNC();
                    dc_any = __ballot(lane < 16 && cb[16 * lane] != 0) != 0;
                    first = 1;
                    ytype = 0;
                }
                any = dc_any;
                const int dy0 = q->y1[0], dy1 = q->y1[1];
                for (int by = 0; by < 4; ++by) {
                    uint32_t lb = (l >> by) & 1;
                    for (int bx = 0; bx < 4; ++bx) {
                        int dcv = 0;
                        const int ctx = (int)lb + (int)((tc >> bx) & 1);
                        const int nz = get_coeffs(t, ytype, ctx, dy0, dy1, first, cb + (4 * by + bx) * 16, lane, &dcv);
                        lb = nz > first;
                        tc = (tc & ~(1u << bx)) | lb << bx;
                        any |= nz > 1 || (first == 0 && dcv != 0);
                    }
                    l = (l & ~(1u << by)) | lb << by;
                }
                const int du0 = q->uv[0], du1 = q->uv[1];
                for (int c = 0; c < 2; ++c) {
                    const int sh = 4 + 2 * c;
                    for (int by = 0; by < 2; ++by) {
                        uint32_t lb = (l >> (sh + by)) & 1;
                        for (int bx = 0; bx < 2; ++bx) {
                            int dcv = 0;
                            const int ctx = (int)lb + (int)((tc >> (sh + bx)) & 1);
                            const int nz =
                                get_coeffs(t, 2, ctx, du0, du1, 0, cb + (16 + 4 * c + 2 * by + bx) * 16, lane, &dcv);
                            lb = nz > 0;
                            tc = (tc & ~(1u << (sh + bx))) | lb << (sh + bx);
                            any |= nz > 1 || dcv != 0;
                        }
                        l = (l & ~(1u << (sh + by))) | lb << (sh + by);
                    }
                }
            } else {  // (VP8DecodeMB: a skipped MB clears the contexts; Y2's only for i16)
                const uint32_t keep = is_i4 ? 0x100u : 0u;
                tc &= keep;
                l &= keep;
            }
            if (lane == 0) {
                tnz[mb_x] = (uint16_t)tc;
                flags[mb] = (uint8_t)any;
            }
            WSYNC();
            if (lane < 48) reinterpret_cast<uint4*>(coef + (size_t)mb * 384)[lane] = cbuf4[lane];
            if (t.br.eof) err = 1;  // (libwebp: "Premature end-of-file encountered.")
        }
        if (lane == 0) saved[p] = t.br;
        WSYNC();
    }
    if (err && lane == 0) *di->err = 1;
}

namespace {

// per wave: R, the MB being predicted (rows -1..15, cols -4..27, BPS-pitched: the
// unfiltered top row, the left column and the corner rotate in as libwebp's
// ReconstructRow does), F, its filter window (rows -4..15, cols -4..15: the filtered
// bottom of the MB above and right of the MB to the left), and its coefficients
struct alignas(16) WaveLds {
    uint8_t ry[17 * 32], ru[9 * 32], rv[9 * 32];
    uint8_t fy[20 * 20], fu[12 * 12], fv[12 * 12];
    int16_t coef[384];
};

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }

}  // namespace

__global__ __launch_bounds__(64 * kReconWaves) void k_vp8d_recon(const DImg* __restrict__ imgs) {
    __shared__ WaveLds W[kReconWaves];
    __shared__ uint32_t prog[kReconWaves];
    const int wave = ufl(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const cptr<DImg> di = (cptr<DImg>)imgs + blockIdx.x;
    const DFrame* const frg = di->fr;
    const cptr<DFrame> fr = (cptr<DFrame>)frg;
    const cptr<DMB> mbs = (cptr<DMB>)di->mbs;
    const cptr<uint8_t> flags = (cptr<uint8_t>)di->flags;
    const int16_t* const coef = di->coef;
    uint8_t* const Y = di->y;
    uint8_t* const U = di->u;
    uint8_t* const V = di->v;
    uint8_t* const top = di->top;
    const int ys = (int)di->ys, uvs = (int)di->uvs;
    const int mb_w = fr->mb_w, mb_h = fr->mb_h, ftype = fr->filter_type;
    if (lane == 0) prog[wave] = 0;
    __syncthreads();
    WaveLds& L = W[wave];
    uint8_t* const Ry = L.ry + 36;
    uint8_t* const Ru = L.ru + 36;
    uint8_t* const Rv = L.rv + 36;
    uint8_t* const Fy = L.fy + 84;
    uint8_t* const Fu = L.fu + 52;
    uint8_t* const Fv = L.fv + 52;
    const uint32_t rstride = (uint32_t)mb_w + 1;
    const int pw = (wave + kReconWaves - 1) % kReconWaves;
    for (int mb_y = wave; mb_y < mb_h; mb_y += kReconWaves) {
        const int has_top = mb_y > 0;
        for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
            const int mb = mb_y * mb_w + mb_x;
            const int has_left = mb_x > 0;
            if (lane < 48) reinterpret_cast<uint4*>(L.coef)[lane] = reinterpret_cast<const uint4*>(coef + (size_t)mb * 384)[lane];
            const cptr<DMB> m = mbs + mb;
            const int is_i4 = m->is_i4, ymode = m->ymode, uvmode = m->uvmode;
            const cptr<DSeg> sg = (cptr<DSeg>)&frg->seg[m->seg];
            const int nonzero = flags[mb];
            if (has_top) {  // the row above has finished MBs mb_x and mb_x + 1
                const uint32_t need = (uint32_t)(mb_y - 1) * rstride + (uint32_t)min(mb_x + 2, mb_w);
                while ((uint32_t)ufl((int)__hip_atomic_load(&prog[pw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < need)
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint8_t* tp = top + (size_t)((mb_y - 1) & 1) * mb_w * 32 + (size_t)mb_x * 32;
                if (lane < 4) st32(Ry - 32 + 4 * lane, ld32(tp + 4 * lane));
                else if (lane < 6) st32(Ru - 32 + 4 * (lane - 4), ld32(tp + 16 + 4 * (lane - 4)));
                else if (lane < 8) st32(Rv - 32 + 4 * (lane - 6), ld32(tp + 24 + 4 * (lane - 6)));
                else if (lane == 8) st32(Ry - 32 + 16, mb_x < mb_w - 1 ? ld32(tp + 32) : 0x01010101u * tp[15]);
                else if (lane >= 16 && lane < 32) {  // the filter's top strip: rows 12..15 of the MB above
                    const int r = (lane - 16) >> 2, g = (lane - 16) & 3;
                    st32(Fy + (r - 4) * 20 + 4 * g, ld32(Y + (size_t)(16 * mb_y - 4 + r) * ys + 16 * mb_x + 4 * g));
                } else if (lane >= 32 && lane < 48) {
                    const int k = lane - 32, c = k >> 3, r = (k & 7) >> 1, g = k & 1;
                    const uint8_t* P = c ? V : U;
                    st32((c ? Fv : Fu) + (r - 4) * 12 + 4 * g, ld32(P + (size_t)(8 * mb_y - 4 + r) * uvs + 8 * mb_x + 4 * g));
                }
                if (!has_left && lane == 63) Ry[-33] = Ru[-33] = Rv[-33] = 129;
            } else {  // frame top: 127 above (corner and top-right included)
                if (lane < 6) st32(Ry - 36 + 4 * lane, 0x7f7f7f7fu);
                else if (lane < 9) st32(Ru - 36 + 4 * (lane - 6), 0x7f7f7f7fu);
                else if (lane < 12) st32(Rv - 36 + 4 * (lane - 9), 0x7f7f7f7fu);
            }
            if (!has_left) {  // frame left: 129
                if (lane < 16) Ry[lane * 32 - 1] = 129;
                else if (lane < 24) Ru[(lane - 16) * 32 - 1] = 129;
                else if (lane < 32) Rv[(lane - 24) * 32 - 1] = 129;
            }
            WSYNC();
            if (is_i4 && lane < 3) st32(Ry + (4 * lane + 3) * 32 + 16, ld32(Ry - 32 + 16));  // top-right, replicated
            WSYNC();
            // ---- prediction + residuals ----
            if (!is_i4) {
                if (lane < 16) {
                    const int bx = lane & 3, by = lane >> 2;
                    uint8_t* blk = Ry + by * 4 * 32 + bx * 4;
                    pred_block(blk, ymode, Ry - 1, 32, Ry - 32, Ry[-33], 16, has_top, has_left, bx, by);
                    vp8x::itransform(blk, L.coef + 16 * lane, blk);
                }
            } else if (lane == 0) {
                for (int n = 0; n < 16; ++n) {
                    uint8_t* blk = Ry + (n >> 2) * 4 * 32 + (n & 3) * 4;
                    uint8_t ctx[13];
                    ctx[0] = blk[3 * 32 - 1];
                    ctx[1] = blk[2 * 32 - 1];
                    ctx[2] = blk[32 - 1];
                    ctx[3] = blk[-1];
                    ctx[4] = blk[-33];
                    for (int k = 0; k < 8; ++k) ctx[5 + k] = blk[-32 + k];
                    vp8x::pred4<32>(blk, m->bmodes[n], ctx + 5);
                    vp8x::itransform(blk, L.coef + 16 * n, blk);
                }
            }
            if (lane >= 16 && lane < 24) {
                const int k = lane - 16, c = k >> 2, b = k & 3;
                uint8_t* R = c ? Rv : Ru;
                uint8_t* blk = R + (b >> 1) * 4 * 32 + (b & 1) * 4;
                pred_block(blk, uvmode, R - 1, 32, R - 32, R[-33], 8, has_top, has_left, b & 1, b >> 1);
                vp8x::itransform(blk, L.coef + (16 + k) * 16, blk);
            }
            WSYNC();
            // ---- the unfiltered bottom row for the row below; the MB into F ----
            if (mb_y < mb_h - 1 && lane < 8) {
                const uint8_t* src = lane < 4 ? Ry + 15 * 32 + 4 * lane : lane < 6 ? Ru + 7 * 32 + 4 * (lane - 4)
                                                                                    : Rv + 7 * 32 + 4 * (lane - 6);
                st32(top + (size_t)(mb_y & 1) * mb_w * 32 + (size_t)mb_x * 32 + 4 * lane, ld32(src));
            }
            st32(Fy + (lane >> 2) * 20 + 4 * (lane & 3), ld32(Ry + (lane >> 2) * 32 + 4 * (lane & 3)));
            if (lane < 32) {
                const int c = lane >> 4, r = (lane & 15) >> 1, g = lane & 1;
                st32((c ? Fv : Fu) + r * 12 + 4 * g, ld32((c ? Rv : Ru) + r * 32 + 4 * g));
            }
            WSYNC();
            // rotate the left samples (and the corner) in for the next MB
            if (lane < 17) st32(Ry + (lane - 1) * 32 - 4, ld32(Ry + (lane - 1) * 32 + 12));
            else if (lane < 26) st32(Ru + (lane - 18) * 32 - 4, ld32(Ru + (lane - 18) * 32 + 4));
            else if (lane < 35) st32(Rv + (lane - 27) * 32 - 4, ld32(Rv + (lane - 27) * 32 + 4));
            // ---- loop filter (DoFilter) ----
            const int i4 = is_i4 ? 1 : 0;
            const int limit = ftype ? (int)sg->limit[i4] : 0;
            if (limit) {
                const int ilevel = sg->ilevel[i4], hev_t = sg->hev[i4];
                const int inner = is_i4 || nonzero;
                const int t_mb = 2 * (limit + 4) + 1, t_in = 2 * limit + 1;
                if (ftype == 1) {  // simple: luma only
                    if (has_left && lane < 16) simple_line(Fy + lane * 20, 1, t_mb);
                    WSYNC();
                    if (inner && lane < 16)
                        for (int k = 1; k < 4; ++k) simple_line(Fy + lane * 20 + 4 * k, 1, t_in);
                    WSYNC();
                    if (has_top && lane < 16) simple_line(Fy + lane, 20, t_mb);
                    WSYNC();
                    if (inner && lane < 16)
                        for (int k = 1; k < 4; ++k) simple_line(Fy + 4 * k * 20 + lane, 20, t_in);
                } else {
                    uint8_t* const fc = lane < 24 ? Fu : Fv;
                    const int cl = lane < 24 ? lane - 16 : lane - 24;
                    if (has_left && lane < 32) {
                        uint8_t* p = lane < 16 ? Fy + lane * 20 : fc + cl * 12;
                        filter_line(p, 1, t_mb, ilevel, hev_t, true);
                    }
                    WSYNC();
                    if (inner && lane < 32) {
                        if (lane < 16) {
                            for (int k = 1; k < 4; ++k) filter_line(Fy + lane * 20 + 4 * k, 1, t_in, ilevel, hev_t, false);
                        } else {
                            filter_line(fc + cl * 12 + 4, 1, t_in, ilevel, hev_t, false);
                        }
                    }
                    WSYNC();
                    if (has_top && lane < 32) {
                        if (lane < 16) filter_line(Fy + lane, 20, t_mb, ilevel, hev_t, true);
                        else filter_line(fc + cl, 12, t_mb, ilevel, hev_t, true);
                    }
                    WSYNC();
                    if (inner && lane < 32) {
                        if (lane < 16) {
                            for (int k = 1; k < 4; ++k) filter_line(Fy + 4 * k * 20 + lane, 20, t_in, ilevel, hev_t, false);
                        } else {
                            filter_line(fc + 4 * 12 + cl, 12, t_in, ilevel, hev_t, false);
                        }
                    }
                }
                WSYNC();
                if (has_top && lane < 32) {  // the MB above's filtered bottom rows
                    if (lane < 16) {
                        const int r = lane >> 2, g = lane & 3;
                        st32(Y + (size_t)(16 * mb_y - 4 + r) * ys + 16 * mb_x + 4 * g, ld32(Fy + (r - 4) * 20 + 4 * g));
                    } else {
                        const int k = lane - 16, c = k >> 3, r = (k & 7) >> 1, g = k & 1;
                        st32((c ? V : U) + (size_t)(8 * mb_y - 4 + r) * uvs + 8 * mb_x + 4 * g,
                             ld32((c ? Fv : Fu) + (r - 4) * 12 + 4 * g));
                    }
                }
            }
            // ---- out: the MB to the left's last columns (final now) and this MB's
            // first ones; the last MB of the row whole ----
            {
                const int r = lane >> 2, g = lane & 3;
                if (has_left || g) st32(Y + (size_t)(16 * mb_y + r) * ys + 16 * mb_x - 4 + 4 * g, ld32(Fy + r * 20 - 4 + 4 * g));
            }
            if (lane < 32) {
                const int c = lane >> 4, r = (lane & 15) >> 1, g = lane & 1;
                if (has_left || g)
                    st32((c ? V : U) + (size_t)(8 * mb_y + r) * uvs + 8 * mb_x - 4 + 4 * g,
                         ld32((c ? Fv : Fu) + r * 12 - 4 + 4 * g));
            }
            if (mb_x == mb_w - 1 && lane < 32) {
                if (lane < 16) {
                    st32(Y + (size_t)(16 * mb_y + lane) * ys + 16 * mb_x + 12, ld32(Fy + lane * 20 + 12));
                } else {
                    const int k = lane - 16, c = k >> 3, r = k & 7;
                    st32((c ? V : U) + (size_t)(8 * mb_y + r) * uvs + 8 * mb_x + 4, ld32((c ? Fv : Fu) + r * 12 + 4));
                }
            }
            WSYNC();
            if (lane < 16) st32(Fy + lane * 20 - 4, ld32(Fy + lane * 20 + 12));
            else if (lane < 32) {
                const int k = lane - 16, c = k >> 3, r = k & 7;
                uint8_t* F = c ? Fv : Fu;
                st32(F + r * 12 - 4, ld32(F + r * 12 + 4));
            }
            // publish: this MB's top row and the pixels above are in HBM
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0)
                __hip_atomic_store(&prog[wave], (uint32_t)mb_y * rstride + (uint32_t)mb_x + 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            WSYNC();
        }
    }
}

// fancy upsampling + colour: one workgroup per output row of one image
__global__ __launch_bounds__(256) void k_vp8d_rgb(const DImg* __restrict__ imgs) {
    const cptr<DImg> di = (cptr<DImg>)imgs + blockIdx.y;
    const cptr<DFrame> fr = (cptr<DFrame>)di->fr;
    const int w = fr->w, h = fr->h, r = blockIdx.x;
    if (r >= h) return;
    const int uvh = (h + 1) >> 1;
    int nr, fr_;
    if (r == 0) {
        nr = fr_ = 0;
    } else if (r & 1) {
        nr = (r - 1) >> 1;
        fr_ = min((r + 1) >> 1, uvh - 1);
    } else {
        nr = r >> 1;
        fr_ = nr - 1;
    }
    const uint8_t* yrow = di->y + (size_t)r * di->ys;
    const uint8_t *nu = di->u + (size_t)nr * di->uvs, *fu = di->u + (size_t)fr_ * di->uvs;
    const uint8_t *nv = di->v + (size_t)nr * di->uvs, *fv = di->v + (size_t)fr_ * di->uvs;
    uint8_t* out = di->out + (size_t)r * di->out_pitch;
    for (int c = threadIdx.x; c < w; c += 256) {
        const int yy = yrow[c], u = fancy_chroma(nu, fu, c, w), v = fancy_chroma(nv, fv, c, w);
        out[3 * c + 0] = (uint8_t)yuv_r(yy, v);
        out[3 * c + 1] = (uint8_t)yuv_g(yy, u, v);
        out[3 * c + 2] = (uint8_t)yuv_b(yy, u);
    }
}

hipError_t launch_vp8d_tokens(const DImg* imgs, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8d_tokens, dim3(n), dim3(64), 0, s, imgs);
    return hipGetLastError();
}
hipError_t launch_vp8d_recon(const DImg* imgs, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8d_recon, dim3(n), dim3(64 * kReconWaves), 0, s, imgs);
    return hipGetLastError();
}
hipError_t launch_vp8d_rgb(const DImg* imgs, int n, int max_h, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8d_rgb, dim3(max_h, n), dim3(256), 0, s, imgs);
    return hipGetLastError();
}

}  // namespace vp8d
}  // namespace ik
