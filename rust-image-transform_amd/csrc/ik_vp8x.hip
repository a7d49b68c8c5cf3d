// ik_vp8x.hip -- the exact WebP coder's device half: libwebp method 4's macroblock
// decisions (reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp; the arithmetic
// is ik_vp8x.h, the same as oracle/vp8_modes.c, whose files equal WebPEncodeRGB's).
//
// Dependencies:
//  - a macroblock predicts from the reconstruction of its left, top-left, top and
//    top-right neighbours, and reads their non-zero contexts and chroma DC errors;
//  - libwebp's token loop refreshes the coefficient probabilities -- hence the level
//    costs every decision uses -- from the statistics of all MBs before it, at MB
//    indices M, 2M+1, 3M+2, ... (M = max(mb_count / 8, 96)): an epoch's MBs may only
//    start when every earlier MB is decided and the statistics folded.
//
// k_vp8x_run is ONE persistent launch per call.  Its workgroups (one wave each) take
// tasks by ticket from a global counter: the MBs of every image in (epoch, diagonal
// mb_x + 2 mb_y, image) order, each epoch's per-image statistics fold after the
// epoch's MBs.  A task waits only for what it reads -- an MB for its left and
// top-right neighbours (which imply the top-left and top) and its epoch's level
// costs, a fold for its epoch's MB count -- by polling hand-off words, so image 0's
// next diagonal starts as soon as its own MBs are done, not when the slowest MB of
// the whole batch is; no launch per diagonal, no host round trip.  Every dependency
// holds a smaller ticket, so the lowest unfinished ticket can always run and the grid
// drains whatever the residency; every wait is bounded (a timeout sets the error word
// and the grid drains).
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, recipe R1): the payload
// -- an MB's edge record (XEdge) and decision record (XMB), a fold's statistics,
// probabilities and level costs -- is stored write-through (sc1, 16-byte stores),
// drained (s_waitcnt vmcnt(0)), then one lane sets the flag (agent-scope atomic);
// the consumer polls the flag, takes an agent-scope acquire, and loads plainly.
//
// An MB task: one wave64; the modes of each stage run on their own lanes -- i16: 4
// lanes, intra-4: 10 lanes per sub-block (16 sub-blocks in order), chroma: 4 lanes --
// and the winner is the lowest score, ties to the lowest mode (libwebp's early-out in
// the intra-4 loop never changes that argmin: a skipped mode's partial score already
// reaches the best full score).
#include <hip/hip_runtime.h>

#include "ik_vp8x.h"
#include "ik_vp8x_gpu.h"

namespace ik {
namespace vp8x {

namespace {

constexpr int kTopLeftI4[16] = {17, 21, 25, 29, 13, 17, 21, 25, 9, 13, 17, 21, 5, 9, 13, 17};

// libwebp's ten intra-4 predictors (pred4, ik_vp8x.h) as taps: per (mode, pixel y*4+x)
// the samples e[i0], e[i1], e[i2] of e[] = L K J I X A B C D E F G H (bits 0-3, 4-7,
// 8-11) and the op (bits 12-14): 0 avg3(i0, i1, i2) = (i0 + 2 i1 + i2 + 2) >> 2,
// 1 avg2(i0, i1), 2 e[i0], 3 TM clip(e[i0] + e[i1] - e[i2]), 4 DC.  Made by
// transcribing pred4's assignments (tools/gen_i4_taps.py); the byte tests hold it.
constexpr uint16_t kI4Tap[10][16] = {
    {0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000, 0x4000},
    {0x3453, 0x3463, 0x3473, 0x3483, 0x3452, 0x3462, 0x3472, 0x3482, 0x3451, 0x3461, 0x3471, 0x3481, 0x3450, 0x3460, 0x3470, 0x3480},
    {0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987, 0x0654, 0x0765, 0x0876, 0x0987},
    {0x0234, 0x0234, 0x0234, 0x0234, 0x0123, 0x0123, 0x0123, 0x0123, 0x0012, 0x0012, 0x0012, 0x0012, 0x0001, 0x0001, 0x0001, 0x0001},
    {0x0345, 0x0456, 0x0567, 0x0678, 0x0234, 0x0345, 0x0456, 0x0567, 0x0123, 0x0234, 0x0345, 0x0456, 0x0012, 0x0123, 0x0234, 0x0345},
    {0x1054, 0x1065, 0x1076, 0x1087, 0x0543, 0x0654, 0x0765, 0x0876, 0x0432, 0x1054, 0x1065, 0x1076, 0x0321, 0x0543, 0x0654, 0x0765},
    {0x0765, 0x0876, 0x0987, 0x0a98, 0x0876, 0x0987, 0x0a98, 0x0ba9, 0x0987, 0x0a98, 0x0ba9, 0x0cba, 0x0a98, 0x0ba9, 0x0cba, 0x0ccb},
    {0x1065, 0x1076, 0x1087, 0x1098, 0x0765, 0x0876, 0x0987, 0x0a98, 0x1076, 0x1087, 0x1098, 0x0ba9, 0x0876, 0x0987, 0x0a98, 0x0cba},
    {0x1043, 0x0543, 0x0654, 0x0765, 0x1032, 0x0432, 0x1043, 0x0543, 0x1021, 0x0321, 0x1032, 0x0432, 0x1010, 0x0210, 0x1021, 0x0321},
    {0x1023, 0x0123, 0x1012, 0x0012, 0x1012, 0x0012, 0x1001, 0x0001, 0x1001, 0x0001, 0x2000, 0x2000, 0x2000, 0x2000, 0x2000, 0x2000},
};

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


// the other lanes of a quad (DPP quad_perm [1,0,3,2] and [2,3,0,1]): sums over a
// mode's four lanes without LDS
__device__ __forceinline__ int qx1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int qx2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ int qsum(int v) {
    v += qx1(v);
    return v + qx2(v);
}

__device__ __forceinline__ int64_t rd_score(int64_t R, int64_t H, int64_t D, int64_t SD, int lambda) {
    return (R + H) * lambda + 256 * (D + SD);
}

}  // namespace

// dev switch IK_VP8X_STAMPS: per-phase shader-clock sums over image 0's MBs
// (tools/vp8x_timing.py --stamps reads them through ik_vp8x_stamps)
#ifndef IK_VP8X_PRIO
#define IK_VP8X_PRIO 2
#endif

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// buffer intrinsics' cache-policy operand: sc1 (gfx940+ CPol::SC1) -- write-through stores
constexpr int kCpolSc1 = 16;

// a wave-uniform 64-bit value in SGPRs
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// lanes [0, nbytes / 16) store their 16 bytes of `src` (LDS) to `dst` (wave-uniform)
// write-through; the other lanes' offsets are out of range (dropped)
__device__ __forceinline__ void store_wt(void* dst, const void* src, uint32_t nbytes, int l) {
    const uint64_t base = uniform_u64((uint64_t)(uintptr_t)dst);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
    const bool act = (uint32_t)l < nbytes / 16;
    const u32x4 v = act ? reinterpret_cast<const u32x4*>(src)[l] : u32x4{0, 0, 0, 0};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, act ? 16 * l : 0x7ffffff0, 0, kCpolSc1);
}

// threads per task: an MB's intra-4 search runs on wave 0 while wave 1 runs intra-16
// and chroma (the three are independent given the MB's context; libwebp's intra-4
// early-out only ends a search whose result it then rejects, so the search runs to
// the end and the decision compares the final sums)
constexpr int kNT = 128;

// a barrier for one wave's lanes: LDS operations of a wave complete in issue order;
// this keeps the compiler from moving them across
#define WSYNC()                                            \
    do {                                                   \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                   \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)

// the MB task's LDS (the fold's overlays it)
struct MbLds {
    alignas(16) uint8_t pr[1056];
#ifndef IK_VP8X_TABLES_GLOBAL
    alignas(16) uint16_t fixed[2048];
    uint16_t ent[256];
    uint16_t fi4[1000];
#endif
    uint8_t bands[17];
    alignas(16) XSeg Q;  // the segment's matrices and lambdas, read per lane in every quantisation
    alignas(16) uint8_t in[BPS * 16];  // Y 0..15, U 16..23, V 24..31
    uint8_t yl[17], yt[20], ul[9], ut[8], vl[9], vt[8];
    int tnz[9], lnz[9];
    int8_t derr_t[2][2], derr_l[2][2];
    alignas(16) uint8_t rec16[4][BPS * 16];
    alignas(16) int16_t lv16[4][17][16];
    int64_t sc[16], part[16][4];
    int flat[4], nz16[4];
    alignas(16) uint8_t best4[BPS * 16];
    uint8_t bound[37];
    int16_t lv4[16][16];
    uint8_t modes4[16];
    uint8_t nbm[8];  // the left MB's right column of sub-block modes, the top MB's bottom row
    alignas(16) uint8_t blk[10][4 * BPS];
    alignas(16) int16_t blv[10][16];
    alignas(16) uint8_t recuv[4][BPS * 8];
    alignas(16) int16_t lvuv[4][8][16];
    int8_t duv[4][2][3];
    int b16, buv, hb4;
    int64_t s16;  // the i16 best's score at lambda_mode (the intra-4 bar)
    int64_t aS4;  // the intra-4 search's final score and header bits
    // per-lane work buffers (private arrays would live in scratch memory); the
    // neighbours' edge records overlay pred16 (prologue only), the outgoing records
    // tmp16 and pred4 (dead by the outputs)
    alignas(16) uint8_t pred16[4][BPS * 16];
    alignas(16) int16_t tmp16[4][16][16];
    alignas(16) uint8_t pred4[10][4 * BPS];
    alignas(16) uint8_t predc[4][BPS * 8];
    alignas(16) int16_t tmpc[4][8][16];
    int16_t dc16[4][16];
    int bnz[4][16], cnz[4][8];
    int ft4[10][16], C4[10][16], tt4[10][2][16];
    int16_t cf4[10][16];
};
static_assert(sizeof(((MbLds*)0)->pred16) >= 4 * sizeof(XEdge), "neighbour records overlay pred16");
static_assert(sizeof(((MbLds*)0)->tmp16) >= sizeof(XMB), "the MB record overlays tmp16");
static_assert(sizeof(((MbLds*)0)->pred4) >= sizeof(XEdge), "the edge record overlays pred4");

// the statistics fold's LDS
struct FoldLds {
    alignas(16) uint32_t st[1056];
    alignas(16) uint8_t pr[1056];
    alignas(16) uint16_t lc[kCostRows * kLevelTab];
    alignas(16) XMB mb;
    int serial;
};

union XLds {
    MbLds m;
    FoldLds f;
};

#ifdef IK_VP8X_STAMPS
__device__ unsigned long long g_vp8x_stamps[32];
#define IK_STAMP(i)                                                         \
    do {                                                                    \
        if (l == 0 && img == 0) {                                           \
            const unsigned long long t_ = clock64();                        \
            atomicAdd(&stm[i], t_ - t_prev); /* LDS: no vmcnt wait */       \
            t_prev = t_;                                                    \
        }                                                                   \
    } while (0)
#else
#define IK_STAMP(i) do {} while (0)
#endif

// One MB: libwebp's VP8Decimate (i16, intra-4, chroma; RD by the image's current level
// costs), then the MB's decision record and edge record, stored write-through.
__device__ __forceinline__ void mb_body(const XArgs& a, int img, int mb, MbLds& S, int l, unsigned long long* stm) {
#ifdef IK_VP8X_STAMPS
    unsigned long long t_prev = clock64();
#endif
    const int mx = mb % a.mb_w, my = mb / a.mb_w;
    const int nmb = a.mb_w * a.mb_h;
    const int uw = (a.w + 1) >> 1, uh = (a.h + 1) >> 1;
    const uint8_t* Y = a.yuv + (size_t)img * a.yuv_stride;
    const uint8_t* U = Y + (size_t)a.w * a.h;
    const uint8_t* V = U + (size_t)uw * uh;
    const XEdge* edges = a.edges + (size_t)img * nmb;
    const int sg = a.seg[(size_t)img * nmb + mb];
    // the image's level costs (13 KB), read at every coefficient of every candidate:
    // from L1 / L2, not LDS -- as fast alone, and the LDS a resident coder task holds is
    // what another batch's decode kernels beside it lose in occupancy
    const uint16_t* lc = a.lc + (size_t)img * kCostRows * kLevelTab;
    auto& pr = S.pr;
#ifdef IK_VP8X_TABLES_GLOBAL
    const uint16_t* s_fixed = kLevelFixedCosts;
    const uint16_t* s_ent = kEntropyCost;
    const uint16_t* s_fi4 = kFixedCostsI4;
#else
    auto& s_fixed = S.fixed;
    auto& s_ent = S.ent;
    auto& s_fi4 = S.fi4;
#endif
    auto& s_bands = S.bands;
    auto& s_in = S.in;
    auto& s_yl = S.yl;
    auto& s_yt = S.yt;
    auto& s_ul = S.ul;
    auto& s_ut = S.ut;
    auto& s_vl = S.vl;
    auto& s_vt = S.vt;
    auto& s_tnz = S.tnz;
    auto& s_lnz = S.lnz;
    auto& s_derr_t = S.derr_t;
    auto& s_derr_l = S.derr_l;
    auto& s_rec16 = S.rec16;
    auto& s_lv16 = S.lv16;
    auto& s_sc = S.sc;
    auto& s_part = S.part;
    auto& s_flat = S.flat;
    auto& s_nz16 = S.nz16;
    auto& s_best4 = S.best4;
    auto& s_bound = S.bound;
    auto& s_lv4 = S.lv4;
    auto& s_modes4 = S.modes4;
    auto& s_nbm = S.nbm;
    auto& s_blk = S.blk;
    auto& s_blv = S.blv;
    auto& s_recuv = S.recuv;
    auto& s_lvuv = S.lvuv;
    auto& s_duv = S.duv;
    auto& s_b16 = S.b16;
    auto& s_buv = S.buv;
    auto& s_s16 = S.s16;
    auto& s_pred16 = S.pred16;
    auto& s_tmp16 = S.tmp16;
    auto& s_pred4 = S.pred4;
    auto& s_predc = S.predc;
    auto& s_tmpc = S.tmpc;
    auto& s_dc16 = S.dc16;
    auto& s_bnz = S.bnz;
    auto& s_cnz = S.cnz;
    auto& s_ft4 = S.ft4;
    auto& s_C4 = S.C4;
    auto& s_tt4 = S.tt4;

    uint8_t (*s_nb)[sizeof(XEdge)] = reinterpret_cast<uint8_t (*)[sizeof(XEdge)]>(&S.pred16[0][0]);
    // staging: every lane issues all of its global reads first (one memory latency for
    // the whole prologue), then writes them to LDS: libwebp's fixed cost tables, the
    // image's probabilities and level costs, the segment's matrices, the source MB
    // (ImportBlock: clamped coordinates) and the neighbours' edge records (left, top,
    // top-right, top-left; 16 bytes per lane)
    if (l < 64) {
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
#ifndef IK_VP8X_TABLES_GLOBAL
#pragma unroll
        for (int j = 0; j < kFi4; ++j)
            if (l + 64 * j < 1000) S.fi4[l + 64 * j] = rf4[j];
#pragma unroll
        for (int j = 0; j < kFix; ++j) S.fixed[l + 64 * j] = rfx[j];
#pragma unroll
        for (int j = 0; j < kEnt; ++j) S.ent[l + 64 * j] = ren[j];
#else
        (void)rf4;
        (void)rfx;
        (void)ren;
#endif
#pragma unroll
        for (int j = 0; j < kPr; ++j)
            if (l + 64 * j < 1056 / 16) ((uint4*)pr)[l + 64 * j] = rpr[j];
        if (l < 17) s_bands[l] = kEncBands[l];
    } else {
        const int w = l - 64;
        const int q = w >> 3;
        int nb = -1;
        if (w < 32) {
            if (q == 0 && mx) nb = mb - 1;
            else if (q == 1 && my) nb = mb - a.mb_w;
            else if (q == 2 && my && mx < a.mb_w - 1) nb = mb - a.mb_w + 1;
            else if (q == 3 && mx && my) nb = mb - a.mb_w - 1;
        }
        const uint4 rnb = nb >= 0 ? reinterpret_cast<const uint4*>(edges + nb)[w & 7] : uint4{0, 0, 0, 0};
        uint8_t rin[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = w + 64 * k;
            const int y = i >> 4, x = i & 15;
            rin[k] = Y[(size_t)min(16 * my + y, a.h - 1) * a.w + min(16 * mx + x, a.w - 1)];
        }
        uint8_t ruv[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = w + 64 * k;
            const int c = i >> 6, kk = i & 63, y = kk >> 3, x = kk & 7;
            const uint8_t* P = c ? V : U;
            ruv[k] = P[(size_t)min(8 * my + y, uh - 1) * uw + min(8 * mx + x, uw - 1)];
        }
        static_assert(sizeof(XSeg) % 4 == 0, "XSeg copied as words");
        const uint32_t* gq = reinterpret_cast<const uint32_t*>(a.segs + img * 4 + sg);
        for (int i = w; i < (int)(sizeof(XSeg) / 4); i += 64) reinterpret_cast<uint32_t*>(&S.Q)[i] = gq[i];
        if (nb >= 0) reinterpret_cast<uint4*>(s_nb[q])[w & 7] = rnb;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = w + 64 * k;
            s_in[(i >> 4) * BPS + (i & 15)] = rin[k];
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = w + 64 * k;
            const int c = i >> 6, kk = i & 63;
            s_in[(kk >> 3) * BPS + 16 + 8 * c + (kk & 7)] = ruv[k];
        }
    }
    const XSeg& Q = S.Q;
    __syncthreads();
    // ---- the boundaries (libwebp's 127 / 129 edge rules) from the neighbours' records ----
    {
        const XEdge& EL = *reinterpret_cast<const XEdge*>(s_nb[0]);
        const XEdge& ET = *reinterpret_cast<const XEdge*>(s_nb[1]);
        const XEdge& ETR = *reinterpret_cast<const XEdge*>(s_nb[2]);
        const XEdge& ETL = *reinterpret_cast<const XEdge*>(s_nb[3]);
        if (l < 16) {
            s_yl[1 + l] = mx ? EL.yright[l] : 129;
            s_yt[l] = my ? ET.ybot[l] : 127;
        } else if (l < 20) {
            const int k = l - 16;
            s_yt[16 + k] = !my ? 127 : (mx < a.mb_w - 1 ? ETR.ybot[k] : ET.ybot[15]);
        } else if (l < 28) {
            const int k = l - 20;
            s_ul[1 + k] = mx ? EL.uright[k] : 129;
            s_vl[1 + k] = mx ? EL.vright[k] : 129;
            s_ut[k] = my ? ET.ubot[k] : 127;
            s_vt[k] = my ? ET.vbot[k] : 127;
        } else if (l == 28) {
            s_yl[0] = !mx ? (my ? 129 : 127) : (my ? ETL.ybot[15] : 127);
            s_ul[0] = !mx ? (my ? 129 : 127) : (my ? ETL.ubot[7] : 127);
            s_vl[0] = !mx ? (my ? 129 : 127) : (my ? ETL.vbot[7] : 127);
        } else if (l == 29) {  // NzToBytes (+ the row's running left DC bit in bit 25)
            const uint32_t tnz = my ? ET.nz : 0u, lnz = mx ? EL.nz : 0u;
            const int tb[9] = {12, 13, 14, 15, 18, 19, 22, 23, 24}, lb[8] = {3, 7, 11, 15, 17, 19, 21, 23};
            for (int i = 0; i < 9; ++i) s_tnz[i] = (int)((tnz >> tb[i]) & 1u);
            for (int i = 0; i < 8; ++i) s_lnz[i] = (int)((lnz >> lb[i]) & 1u);
            s_lnz[8] = (int)((lnz >> 25) & 1u);
        } else if (l >= 32 && l < 40) {
            const int k = l - 32;
            s_nbm[k] = k < 4 ? (mx ? EL.bmr[k] : 0) : (my ? ET.bmb[k - 4] : 0);
        } else if (l == 30) {
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 2; ++k) {
                    s_derr_t[c][k] = (a.use_derr && my) ? ET.derr[c * 2 + k] : 0;
                    s_derr_l[c][k] = (a.use_derr && mx) ? EL.derr[4 + c * 2 + k] : 0;
                }
        }
    }
    __syncthreads();
    IK_STAMP(0);

    // wave 1: intra-16, then chroma; wave 0: intra-4 (lane numbers per wave)
    auto run_i16_uv = [&](const int l) {
    // ---- intra-16: lane = (mode, 4x4 block), 4 x 16 lanes ----
    {
        const int m = l >> 4, n = l & 15, bx = n & 3, by = n >> 2;
        const int off = bx * 4 + by * 4 * BPS;
        uint8_t* pred = s_pred16[m];
        pred16_block(pred, m, mx ? s_yl + 1 : nullptr, my ? s_yt : nullptr, bx, by);
        ftransform(s_in + off, pred + off, s_tmp16[m][n]);
        WSYNC();
        if (n == 0) {  // the mode's Y2: WHT of the 16 DCs, quantised
            ftransform_wht(s_tmp16[m][0], s_dc16[m]);
            s_nz16[m] = quantize_block(s_dc16[m], s_lv16[m][0], Q.y2) << 24;
        }
        WSYNC();
        s_tmp16[m][n][0] = 0;
        const int bnz = quantize_block(s_tmp16[m][n], s_lv16[m][1 + n], Q.y1);
        s_bnz[m][n] = bnz;
        WSYNC();
        if (n == 0) itransform_wht(s_dc16[m], s_tmp16[m][0]);  // the DCs back into the blocks
        WSYNC();
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
    WSYNC();
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
    }
    WSYNC();
    IK_STAMP(2);

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
        WSYNC();
        if (act) ftransform(s_in + 16 + off, pred + off, s_tmpc[m][n]);
        WSYNC();
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
        WSYNC();
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
        WSYNC();
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
    WSYNC();
    if (l == 0) {
        int best = 0;
        for (int m = 1; m < 4; ++m)
            if (s_sc[m] < s_sc[best]) best = m;
        s_buv = best;
    }
    WSYNC();
    IK_STAMP(4);
    };

    auto run_i4 = [&](const int l) {
    // ---- intra-4: 16 sub-blocks in order; lane = (mode, row), 10 x 4 ----
    // Per sub-block four phases between wave barriers, the rest in registers:
    //  A: the lane's predictor row (mode m's row r, from the tap table) and source row;
    //     FTransform's row pass;
    //  B: column r: FTransform's column pass, QuantizeBlock of its four coefficients
    //     (raster r, 4+r, 8+r, 12+r: quantisation is per coefficient), and
    //     ITransform's column pass on the dequantised four;
    //  C: row r: ITransform's row pass onto the predictor row, the SSE, the spectral
    //     (TTransform) rows of source and reconstruction;
    //  D: the spectral columns, the mode's rate and score, the winner, the rotation.
    if (l == 0) {  // VP8IteratorStartI4: the intra-4 boundary, contexts re-imported
        for (int i = 0; i < 17; ++i) s_bound[i] = s_yl[16 - i];
        for (int i = 0; i < 20; ++i) s_bound[17 + i] = s_yt[i];
    }
    const int m = l >> 2, r = l & 3;
    const bool act = l < 40;
    // the lane's fixed terms: predictor taps, and the quantiser of its column (positions
    // 1..15 share q / iq / bias / zero threshold: expand_matrix; sharpening per position)
    uint32_t tap[4];
    int shq[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        tap[x] = kI4Tap[act ? m : 0][4 * r + x];
        shq[x] = Q.y1.sharpen[r + 4 * x];
    }
    int bandrow[4];  // the level-cost row of zigzag position 4r + k, type 3: (3 * 8 + band) * 3
#pragma unroll
    for (int k = 0; k < 4; ++k) bandrow[k] = (24 + kEncBands[4 * r + k]) * 3;
    const uint32_t zt0 = Q.y1.zthresh[0], zt1 = Q.y1.zthresh[1], iq0 = Q.y1.iq[0], iq1 = Q.y1.iq[1];
    const uint32_t bi0 = Q.y1.bias[0], bi1 = Q.y1.bias[1];
    const int q0 = Q.y1.q[0], q1 = Q.y1.q[1];
    WSYNC();
    {
        int tnz4[4], lnz4[4];
        for (int i = 0; i < 4; ++i) { tnz4[i] = s_tnz[i]; lnz4[i] = s_lnz[i]; }
        int64_t aS = 211ll * Q.lambda_mode;  // rd_best: H = 211 = VP8BitCost(0, 145)
        int header_bits = 0;
#ifdef IK_VP8X_NO_I4
        header_bits = 1 << 30;
        for (int i4 = 0; i4 < 0; ++i4) {
#else
        for (int i4 = 0; i4 < 16; ++i4) {
#endif
            const int bx = i4 & 3, by = i4 >> 2;
            const int off = bx * 4 + by * 4 * BPS;
            const uint8_t* tp = s_bound + kTopLeftI4[i4] - 5;  // e[0..12] = L K J I X A B C D E F G H
            // ---- A ----
            int p[4], sr[4];
            {
                int e0[4], e1[4], e2[4];
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    e0[x] = tp[tap[x] & 15];
                    e1[x] = tp[(tap[x] >> 4) & 15];
                    e2[x] = tp[(tap[x] >> 8) & 15];
                    sr[x] = s_in[off + r * BPS + x];
                }
                const int dc = (4 + tp[0] + tp[1] + tp[2] + tp[3] + tp[5] + tp[6] + tp[7] + tp[8]) >> 3;
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const uint32_t op = tap[x] >> 12;
                    const int v3 = (e0[x] + 2 * e1[x] + e2[x] + 2) >> 2, v2 = (e0[x] + e1[x] + 1) >> 1;
                    const int tm = xclip8(e0[x] + e1[x] - e2[x]);
                    p[x] = op == 0 ? v3 : op == 1 ? v2 : op == 2 ? e0[x] : op == 3 ? tm : dc;
                }
            }
            if (act) {  // FTransform, row r
                const int d0 = sr[0] - p[0], d1 = sr[1] - p[1], d2 = sr[2] - p[2], d3 = sr[3] - p[3];
                const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
                *reinterpret_cast<int4*>(&s_ft4[m][4 * r]) =
                    make_int4((a0 + a1) * 8, (a2 * 2217 + a3 * 5352 + 1812) >> 9, (a0 - a1) * 8,
                              (a3 * 2217 - a2 * 5352 + 937) >> 9);
            }
            WSYNC();
            IK_STAMP(10);
            // ---- B ----
            int nzl = 0, cnt = 0;
            if (act) {
                const int* t = s_ft4[m];
                const int i = r;
                const int a0 = t[0 + i] + t[12 + i], a1 = t[4 + i] + t[8 + i];
                const int a2 = t[4 + i] - t[8 + i], a3 = t[0 + i] - t[12 + i];
                int c[4];
                c[0] = (int16_t)((a0 + a1 + 7) >> 4);
                c[1] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
                c[2] = (int16_t)((a0 - a1 + 7) >> 4);
                c[3] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
                int dq[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // QuantizeBlock of raster position j = r + 4k
                    const int j = r + 4 * k;
                    const int v = c[k];
                    const int sign = v < 0;
                    const uint32_t coeff = (uint32_t)((sign ? -v : v) + shq[k]);
                    const bool z = j == 0;
                    int level = 0;
                    if (coeff > (z ? zt0 : zt1)) {
                        level = (int)((coeff * (z ? iq0 : iq1) + (z ? bi0 : bi1)) >> QFIX);
                        if (level > 2047) level = 2047;
                        if (sign) level = -level;
                    }
                    s_blv[m][izigzag(j)] = (int16_t)level;
                    dq[k] = (int16_t)(level * (z ? q0 : q1));
                    nzl |= level != 0;
                    cnt += j > 0 && level != 0;
                }
                // ITransform, column r
                const int a = dq[0] + dq[2], b = dq[0] - dq[2];
                const int cc = ((dq[1] * 35468) >> 16) - (((dq[3] * 20091) >> 16) + dq[3]);
                const int d = (((dq[1] * 20091) >> 16) + dq[1]) + ((dq[3] * 35468) >> 16);
                *reinterpret_cast<int4*>(&s_C4[m][4 * i]) = make_int4(a + d, b + cc, b - cc, a - d);
            }
            WSYNC();
            IK_STAMP(13);
            // ---- C ----
            int sse = 0;
            if (act) {
                const int* C = s_C4[m];
                const int i = r;
                const int dc = C[i] + 4;
                const int a = dc + C[8 + i], b = dc - C[8 + i];
                const int c = ((C[4 + i] * 35468) >> 16) - (((C[12 + i] * 20091) >> 16) + C[12 + i]);
                const int d = (((C[4 + i] * 20091) >> 16) + C[4 + i]) + ((C[12 + i] * 35468) >> 16);
                int o[4];
                o[0] = xclip8(p[0] + ((a + d) >> 3));
                o[1] = xclip8(p[1] + ((b + c) >> 3));
                o[2] = xclip8(p[2] + ((b - c) >> 3));
                o[3] = xclip8(p[3] + ((a - d) >> 3));
                *reinterpret_cast<uint32_t*>(s_blk[m] + i * BPS) =
                    (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | ((uint32_t)o[3] << 24);
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const int e = sr[x] - o[x];
                    sse += e * e;
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int* in = q ? o : sr;
                    const int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[1] - in[3], a3 = in[0] - in[2];
                    *reinterpret_cast<int4*>(&s_tt4[m][q][4 * i]) = make_int4(a0 + a1, a3 + a2, a3 - a2, a0 - a1);
                }
            }
            WSYNC();
            IK_STAMP(15);
            // ---- D ----
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
            // sums over the mode's 4 lanes
            sse = qsum(sse);
            tA = qsum(tA);
            tB = qsum(tB);
            cnt = qsum(cnt);
            nzl |= qx1(nzl);
            nzl |= qx2(nzl);
            // the mode's rate, GetResidualCost (type 3, first 0) over its four lanes: lane r
            // sums the terms of zigzag positions 4r .. 4r+3 (each position's context is its
            // predecessor's level), the quad's last non-zero position bounds them
            const int ctx0 = tnz4[bx] + lnz4[by];
            int rate_terms = 0, last = -1;
            {
                const int16_t* lvm = s_blv[act ? m : 0];
                const uint2 w2 = *reinterpret_cast<const uint2*>(lvm + 4 * r);
                int v[4] = {(int16_t)(w2.x & 0xffffu), (int16_t)(w2.x >> 16), (int16_t)(w2.y & 0xffffu),
                            (int16_t)(w2.y >> 16)};
                int vp = r ? lvm[4 * r - 1] : 0;
                vp = vp < 0 ? -vp : vp;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[k] = v[k] < 0 ? -v[k] : v[k];
                    if (v[k]) last = 4 * r + k;
                }
                last = max(last, qx1(last));
                last = max(last, qx2(last));
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int n = 4 * r + k;
                    const int pv = k ? v[k - 1] : vp;
                    const int ctx = n == 0 ? ctx0 : (pv >= 2 ? 2 : pv);
                    const int term = s_fixed[v[k]] + lc[(bandrow[k] + ctx) * kLevelTab + (v[k] > kMaxVarLevel ? kMaxVarLevel : v[k])];
                    rate_terms += n <= last ? term : 0;
                }
                rate_terms = qsum(rate_terms);
            }
            // the mode's score and terms on its lane r == 0 (4m)
            int myS = INT32_MAX, myD = 0, mySD = 0, myR = 0, myH = 0;
            if (act && r == 0) {
                // mode costs from the neighbouring sub-blocks' modes (frame edge: B_DC)
                const int left = bx ? s_modes4[i4 - 1] : s_nbm[by];
                const int topm = by ? s_modes4[i4 - 4] : s_nbm[4 + bx];
                myD = sse;
                mySD = Q.tlambda ? ((Q.tlambda * (xabs(tB - tA) >> 5) + 128) >> 8) : 0;
                myH = s_fi4[(topm * 10 + left) * 10 + m];
                myR = (m > 0 && cnt <= 3) ? 140 : 0;  // IsFlat(levels, 1, FLATNESS_LIMIT_I4)
                const int p0 = pr[(24 * 3 + ctx0) * 11];
                if (last < 0) {
                    myR += s_ent[p0];
                } else {
                    int vl = s_blv[m][last];
                    vl = vl < 0 ? -vl : vl;
                    myR += (ctx0 == 0 ? s_ent[255 - p0] : 0) + rate_terms;
                    if (last < 15) myR += s_ent[pr[((24 + s_bands[last + 1]) * 3 + (vl == 1 ? 1 : 2)) * 11]];
                }
                // (the i4 terms fit 32 bits: D <= 16 * 255^2, rates and lambdas small)
                myS = (myR + myH) * Q.lambda_i4 + 256 * (myD + mySD);
            }
            // lane 4m holds mode m's score: read the ten with v_readlane (wave-uniform
            // results, no LDS), strict "<" in mode order = ties to the lowest mode
            int bsc = INT32_MAX;
            int best = 0;
#pragma unroll
            for (int mm = 0; mm < 10; ++mm) {
                const int sc = __builtin_amdgcn_readlane(myS, 4 * mm);
                if (sc < bsc) { bsc = sc; best = mm; }
            }
            const int64_t sD = __builtin_amdgcn_readlane(myD, 4 * best), sSD = __builtin_amdgcn_readlane(mySD, 4 * best),
                          sR = __builtin_amdgcn_readlane(myR, 4 * best), sH = __builtin_amdgcn_readlane(myH, 4 * best);
            const int nzb = __builtin_amdgcn_readlane(nzl, 4 * best);
            aS += rd_score(sR, sH, sD, sSD, Q.lambda_mode);
            header_bits += (int)sH;
            if (l < 16) s_lv4[i4][l] = s_blv[best][l];
            if (l < 16) s_best4[off + (l & 3) + (l >> 2) * BPS] = s_blk[best][(l & 3) + (l >> 2) * BPS];
            IK_STAMP(16);
            tnz4[bx] = lnz4[by] = nzb;
            if (l == 0) s_modes4[i4] = (uint8_t)best;
            if (l < 4) {
                // VP8IteratorRotateI4, one position per lane (the writes [-4, 4) never
                // overlap another lane's reads: [4, 8) or the winner's block)
                uint8_t* top = s_bound + kTopLeftI4[i4];
                const uint8_t* blk = s_blk[best];
                const uint8_t b0 = blk[l + 3 * BPS];
                const uint8_t b1 = (i4 & 3) != 3 ? (l < 3 ? blk[3 + (2 - l) * BPS] : top[3]) : top[l + 4];
                top[-4 + l] = b0;
                top[l] = b1;
            }
            WSYNC();
            IK_STAMP(17);
        }
        if (l == 0) {
            S.aS4 = aS;
            S.hb4 = header_bits;
        }
    }
    IK_STAMP(3);
    };
    if (__builtin_amdgcn_readfirstlane(l >> 6)) run_i16_uv(l - 64);
    else run_i4(l);
    __syncthreads();

    // ---- outputs: the MB record, the edge record (reconstruction edges, contexts,
    // chroma errors, edge sub-block modes), built in LDS and stored write-through ----
    // intra-4 wins iff its running score never reached the i16 score nor its header
    // bits the limit (both only grow): libwebp's loop would not have stopped
    const bool i4 = S.aS4 < s_s16 && S.hb4 <= 256 * 16 * 16;
    const int b16 = s_b16, buv = s_buv;
    XMB& o = *reinterpret_cast<XMB*>(&s_tmp16[0][0][0]);
    XEdge& E = *reinterpret_cast<XEdge*>(&s_pred4[0][0]);
    const uint8_t* ry = i4 ? s_best4 : s_rec16[b16];
    const uint8_t* ruv = s_recuv[buv];
    for (int i = l; i < 16 * 16; i += kNT) o.ac[i >> 4][i & 15] = i4 ? s_lv4[i >> 4][i & 15] : s_lv16[b16][1 + (i >> 4)][i & 15];
    if (l < 8 * 16) o.uv[l >> 4][l & 15] = s_lvuv[buv][l >> 4][l & 15];
    if (l < 16) {
        o.dc[l] = i4 ? 0 : s_lv16[b16][0][l];
        o.bmodes[l] = i4 ? s_modes4[l] : (uint8_t)b16;
        E.ybot[l] = ry[15 * BPS + l];
        E.yright[l] = ry[l * BPS + 15];
    } else if (l < 24) {
        const int k = l - 16;
        E.ubot[k] = ruv[7 * BPS + k];
        E.vbot[k] = ruv[7 * BPS + 8 + k];
        E.uright[k] = ruv[k * BPS + 7];
        E.vright[k] = ruv[k * BPS + 15];
    } else if (l < 28) {
        const int k = l - 24;
        E.bmr[k] = i4 ? s_modes4[4 * k + 3] : (uint8_t)b16;
        E.bmb[k] = i4 ? s_modes4[12 + k] : (uint8_t)b16;
    } else if (l < 40) {
        o.pad2[l - 28] = 0;
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
        E.nz = nz;
        // StoreDiffusionErrors: [0..3] the top pair per channel (for the MB below), [4..7] the left pair
        for (int ch = 0; ch < 2; ++ch) {
            const int8_t* e = s_duv[buv][ch];
            const int8_t l1 = a.use_derr ? (int8_t)((3 * e[2]) >> 2) : 0;
            E.derr[4 + ch * 2 + 0] = a.use_derr ? e[0] : 0;
            E.derr[4 + ch * 2 + 1] = l1;
            E.derr[ch * 2 + 0] = a.use_derr ? e[1] : 0;
            E.derr[ch * 2 + 1] = a.use_derr ? (int8_t)(e[2] - l1) : 0;
        }
    }
    __syncthreads();
    store_wt(a.mbs + (size_t)img * nmb + mb, &o, sizeof(XMB), l);
    store_wt(a.edges + (size_t)img * nmb + mb, &E, sizeof(XEdge), l);
    IK_STAMP(5);
}

// One image's statistics fold after epoch [k0, k1): the epoch's token statistics in
// raster order, then the probabilities and level costs the next epoch's decisions use
// (and, after the last epoch, the file's probabilities), stored write-through.
__device__ __forceinline__ void fold_body(const XArgs& a, int img, int k0, int k1, FoldLds& F, int l) {
    const int nmb = a.mb_w * a.mb_h;
    const XMB* mbs = a.mbs + (size_t)img * nmb;
    const XEdge* edges = a.edges + (size_t)img * nmb;
    const uint32_t* stats = a.stats + (size_t)img * 1056;
    // the counters in LDS.  libwebp halves a counter pair when its total reaches 65534,
    // which makes the fold order-dependent; an epoch adds at most 25 blocks x 16
    // records per slot per MB, so when every total is below 65534 minus that bound no
    // counter can reach the halving point and the MBs fold in parallel (LDS atomics);
    // otherwise lane 0 walks them in raster order, staged in LDS.
    if (l == 0) F.serial = 0;
    __syncthreads();
    const uint32_t bound = (uint32_t)(k1 - k0) * 25u * 16u;
    for (int i = l; i < 1056; i += kNT) {
        F.st[i] = stats[i];
        if ((F.st[i] >> 16) + bound >= 0xfffeu) F.serial = 1;
    }
    __syncthreads();
    auto ctx_of = [&](int k, int* t, int* lf) {
        const int mx = k % a.mb_w, my = k / a.mb_w;
        const uint32_t tnz = my ? edges[k - a.mb_w].nz : 0u, lnz = mx ? edges[k - 1].nz : 0u;
        const int tb[9] = {12, 13, 14, 15, 18, 19, 22, 23, 24}, lb[8] = {3, 7, 11, 15, 17, 19, 21, 23};
        for (int i = 0; i < 9; ++i) t[i] = (int)((tnz >> tb[i]) & 1u);
        for (int i = 0; i < 8; ++i) lf[i] = (int)((lnz >> lb[i]) & 1u);
        lf[8] = (int)((lnz >> 25) & 1u);
    };
    if (!F.serial) {
        uint32_t* st = F.st;
        for (int k = k0 + l; k < k1; k += kNT) {
            int t[9], lf[9];
            ctx_of(k, t, lf);
            record_mb([st](uint32_t slot, int bit) { atomicAdd(st + slot, 0x00010000u + (uint32_t)bit); return bit; },
                      mbs[k], t, lf, [](int, uint32_t) {});
        }
        __syncthreads();
    } else {
        for (int k = k0; k < k1; ++k) {
            const uint4* src = reinterpret_cast<const uint4*>(mbs + k);
            for (int i = l; i < (int)(sizeof(XMB) / 16); i += kNT) reinterpret_cast<uint4*>(&F.mb)[i] = src[i];
            __syncthreads();
            if (l == 0) {
                int t[9], lf[9];
                ctx_of(k, t, lf);
                record_mb([&](uint32_t slot, int bit) { return record_stats(bit, F.st + slot); }, F.mb, t, lf,
                          [](int, uint32_t) {});
            }
            __syncthreads();
        }
    }
    for (int i = l; i < 1056; i += kNT) F.pr[i] = (uint8_t)finalize_proba(F.st[i], i);
    __syncthreads();
    for (int r = l; r < kCostRows; r += kNT) level_cost_row(F.pr + r * 11, r % 3, F.lc + r * kLevelTab);
    __syncthreads();
    for (int c = 0; c < 1056 * 4 / 16; c += kNT)
        store_wt(a.stats + (size_t)img * 1056 + 4 * c, F.st + 4 * c, min(1056 * 4 / 16 - c, kNT) * 16, l);
    store_wt(a.pr + (size_t)img * 1056, F.pr, 1056, l);
    constexpr int kLcWords = kCostRows * kLevelTab * 2 / 16;
    for (int c = 0; c < kLcWords; c += kNT)
        store_wt(a.lc + (size_t)img * kCostRows * kLevelTab + 8 * c, F.lc + 8 * c, min(kLcWords - c, kNT) * 16, l);
}

// lane 0: wait until *f >= want; false on a timeout (which sets the error word) or
// when another wait has failed
__device__ bool poll_ge(const uint32_t* f, uint32_t want, uint32_t* err, uint64_t t_end) {
    for (;;) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (__builtin_amdgcn_s_memrealtime() > t_end) {
            __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// The whole call's decisions and statistics folds, one launch (see the file header).
__global__ __launch_bounds__(kNT) void k_vp8x_run(XArgs a, XRun r) {
    __shared__ XLds S;
    __shared__ uint64_t s_task;
    __shared__ int s_ok;
    const int l = threadIdx.x;
    const int nmb = a.mb_w * a.mb_h;
    uint32_t* err = r.sync + 1;
    // the coder's waves win instruction issue on a SIMD they share with another batch's
    // decode waves: its MB chain is latency-bound, the decode throughput-bound
    __builtin_amdgcn_s_setprio(IK_VP8X_PRIO);
#ifdef IK_VP8X_STAMPS
    unsigned long long t_loop = clock64();
    __shared__ unsigned long long stm[32];
    if (l < 32) stm[l] = 0;
    __syncthreads();
#else
    unsigned long long* stm = nullptr;
#endif
    for (;;) {
        if (l == 0) {
            uint64_t task = ~0ull;
            bool ok = true;
            const uint32_t t = __hip_atomic_fetch_add(r.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t < r.ntasks) {
                task = r.tasks[t];
                const int img = (int)((task >> 32) & 0xffffu), e = (int)((task >> 48) & 0xffu);
                const int mb = (int)(uint32_t)task;
                // 4 s per wait (s_memrealtime counts at 100 MHz); a call takes tens of ms
                const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;
                if (task >> 63) {  // the fold of epoch e: its MBs decided, the previous fold's statistics in place
                    ok = poll_ge(r.cnt + (size_t)img * r.nep + e, (uint32_t)(r.bounds[e + 1] - r.bounds[e]), err, t_end);
                    if (ok && e > 0) ok = poll_ge(r.ready + (size_t)img * r.nep + e, 1u, err, t_end);
                } else {  // an MB: its epoch's level costs, its left and top-right (or top) neighbours
                    const int mx = mb % a.mb_w, my = mb / a.mb_w;
                    const uint32_t* done = r.done + (size_t)img * nmb;
                    if (e > 0) ok = poll_ge(r.ready + (size_t)img * r.nep + e, 1u, err, t_end);
                    if (ok && mx > 0) ok = poll_ge(done + mb - 1, 1u, err, t_end);
                    if (ok && my > 0) ok = poll_ge(done + mb - a.mb_w + (mx < a.mb_w - 1 ? 1 : 0), 1u, err, t_end);
                }
            }
            s_task = task;
            s_ok = ok;
        }
        __syncthreads();
        const uint64_t task = uniform_u64(s_task);
        const int ok = __builtin_amdgcn_readfirstlane(s_ok);
        if (task == ~0ull || !ok) {
#ifdef IK_VP8X_STAMPS
            if (l < 32) atomicAdd(&g_vp8x_stamps[l], stm[l]);
#endif
            return;
        }
        // the hand-off's acquire: this CU's L1 holds nothing older than the flags seen
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int img = (int)((task >> 32) & 0xffffu), e = (int)((task >> 48) & 0xffu);
#ifdef IK_VP8X_STAMPS
        if (l == 0 && img == 0 && !(task >> 63)) {  // stamp 20: ticket + dependency wait + acquire
            const unsigned long long t_ = clock64();
            atomicAdd(&stm[20], t_ - t_loop);
        }
#endif
        // the lane index made opaque per task: otherwise the compiler hoists every
        // lane-derived address of the MB body out of the task loop (255 VGPRs, not 98)
        int lt = threadIdx.x;
        asm volatile("" : "+v"(lt));
        if (task >> 63) fold_body(a, img, r.bounds[e], r.bounds[e + 1], S.f, lt);
        else mb_body(a, img, (int)(uint32_t)task, S.m, lt, stm);
        // the payload's write-through stores have completed before the flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (l == 0) {
            if (task >> 63) {
                if (e + 1 < (int)r.nep)
                    __hip_atomic_store(r.ready + (size_t)img * r.nep + e + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(r.done + (size_t)img * nmb + (uint32_t)task, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(r.cnt + (size_t)img * r.nep + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
#ifdef IK_VP8X_STAMPS
        if (l == 0) {
            const unsigned long long t_ = clock64();
            if (img == 0 && !(task >> 63)) atomicAdd(&stm[21], t_ - t_loop);  // stamp 21: the whole task
            t_loop = t_;
        }
#endif
    }
}

// The segment set-up (libwebp VP8SetSegmentParams + SimplifySegments + the segment
// map's tree probabilities; restated from the host's vp8_segment_setup) and the
// initial coding state of every image: one wave per image.  qtab[s_alpha + 127] is
// the segment quantiser for a segment alpha at this quality (libwebp's pow(), computed
// on the host with the same libm).
__global__ __launch_bounds__(64) void k_vp8x_setup(XArgs a, const vp8::SegRecord* recs, const uint8_t* kseg,
                                                   const int* qtab, ik_vp8_segment_header* hdrs) {
    constexpr int nb = 4, sns = 50, filter_strength = 60;
    const int img = blockIdx.x, l = threadIdx.x;
    const int nmb = a.mb_w * a.mb_h;
    __shared__ int s_map[nb], s_cnt[nb], s_nfinal, s_reset;
    __shared__ ik_vp8_segment_header s_hd;
    auto clip = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
    const vp8::SegRecord& r = recs[img];
    if (l == 0) {
        int mn = r.centers[0], mx = r.centers[0];
        for (int k = 0; k < nb; ++k) {
            mn = r.centers[k] < mn ? r.centers[k] : mn;
            mx = r.centers[k] > mx ? r.centers[k] : mx;
        }
        if (mx == mn) mx = mn + 1;
        int quant[nb], fstr[nb];
        for (int k = 0; k < nb; ++k) {
            const int s_alpha = clip(255 * (r.centers[k] - r.mid) / (mx - mn), -127, 127);
            const int s_beta = clip(255 * (r.centers[k] - mn) / (mx - mn), 0, 255);
            quant[k] = qtab[s_alpha + 127];
            const int qstep = vp8::kAcTable[clip(quant[k], 0, 127)] >> 2;
            const int base = qstep < 63 ? qstep : 63;
            const int f = base * (5 * filter_strength) / (256 + s_beta);
            fstr[k] = f < 2 ? 0 : (f > 63 ? 63 : f);  // FSTRENGTH_CUTOFF 2
        }
        const int total = r.nmb > 0 ? r.nmb : 1;
        const int uv_alpha = (int)(r.uv_alpha_sum / (unsigned long long)total);
        // MID_ALPHA 64, MIN_ALPHA 30, MAX_ALPHA 100; MIN/MAX_DQ_UV -4 / 6
        int dq_uv_ac = (uv_alpha - 64) * (6 - (-4)) / (100 - 30);
        dq_uv_ac = clip(dq_uv_ac * sns / 100, -4, 6);
        s_hd.base_quant = quant[0];
        int nfinal = 1;
        s_map[0] = 0;
        for (int s1 = 1; s1 < nb; ++s1) {
            int s2 = 0;
            bool found = false;
            for (; s2 < nfinal; ++s2)
                if (quant[s1] == quant[s2] && fstr[s1] == fstr[s2]) { found = true; break; }
            s_map[s1] = s2;
            if (!found) {
                if (nfinal != s1) { quant[nfinal] = quant[s1]; fstr[nfinal] = fstr[s1]; }
                ++nfinal;
            }
        }
        for (int k = nfinal; k < nb; ++k) { quant[k] = quant[nfinal - 1]; fstr[k] = fstr[nfinal - 1]; }
        for (int k = 0; k < nb; ++k) { s_hd.quant[k] = quant[k]; s_hd.fstrength[k] = fstr[k]; s_cnt[k] = 0; }
        s_hd.dq_uv_dc = clip(-4 * sns / 100, -15, 15);
        s_hd.dq_uv_ac = dq_uv_ac;
        s_hd.alpha = (int)(r.alpha_sum / (unsigned long long)total);
        s_hd.uv_alpha = uv_alpha;
        s_nfinal = nfinal;
    }
    __syncthreads();
    const int nfinal = s_nfinal;
    uint8_t* seg = a.seg + (size_t)img * nmb;
    const uint8_t* ks = kseg + (size_t)img * nmb;
    for (int i = l; i < nmb; i += 64) {
        const int v = nfinal < nb ? s_map[ks[i]] : ks[i];
        seg[i] = (uint8_t)v;
        atomicAdd(&s_cnt[v], 1);
    }
    __syncthreads();
    if (l == 0) {
        auto proba = [](int x, int y) { const int t = x + y; return t == 0 ? 255 : (255 * x + t / 2) / t; };
        s_hd.probs[0] = proba(s_cnt[0] + s_cnt[1], s_cnt[2] + s_cnt[3]);
        s_hd.probs[1] = proba(s_cnt[0], s_cnt[1]);
        s_hd.probs[2] = proba(s_cnt[2], s_cnt[3]);
        s_hd.num_segments = nfinal;
        s_hd.update_map = nfinal > 1 && (s_hd.probs[0] != 255 || s_hd.probs[1] != 255 || s_hd.probs[2] != 255);
        s_reset = nfinal > 1 && !s_hd.update_map;  // ResetSegments
        hdrs[img] = s_hd;
    }
    __syncthreads();
    if (s_reset)
        for (int i = l; i < nmb; i += 64) seg[i] = 0;
    if (l < nb) a.segs[(size_t)img * nb + l] = setup_segment(s_hd.quant[l], s_hd.dq_uv_dc, s_hd.dq_uv_ac, sns);
    // the initial coding state: default probabilities, their level costs, no statistics
    for (int i = l; i < 1056; i += 64) {
        a.pr[(size_t)img * 1056 + i] = kCoeffProbs0[i];
        a.stats[(size_t)img * 1056 + i] = 0;
    }
    for (int rr = l; rr < kCostRows; rr += 64)
        level_cost_row(kCoeffProbs0 + rr * 11, rr % 3, a.lc + ((size_t)img * kCostRows + rr) * kLevelTab);
    if (l < nb) a.max_edge[img * nb + l] = 0;
}

hipError_t launch_vp8x_setup(const XArgs& a, const vp8::SegRecord* rec, const uint8_t* kseg, const int* qtab,
                             ik_vp8_segment_header* hdr, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_vp8x_setup, dim3(n), dim3(64), 0, s, a, rec, kseg, qtab, hdr);
    return hipGetLastError();
}

hipError_t launch_vp8x_run(const XArgs& a, const XRun& r, int grid, hipStream_t s) {
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_vp8x_run, dim3(grid), dim3(kNT), 0, s, a, r);
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
