// ik_jsync.hip -- gfx950 kernels of the self-synchronising baseline JPEG entropy
// decoder (decode_image on a JPEG: reference src/transform.rs:31 -> image 0.25.8 ->
// zune-jpeg 0.4.21).  The algorithm and the per-lane code are in ik_jpeg_sync.h,
// shared with the CPU model the CPU tests run; the host side is
// ik_jpeg_decode.cpp (decode_jpeg_batch).
//
//   k_jsync_count    a workgroup per 4 KiB chunk of a scan: bytes kept by the
//                    unstuffing, restart markers, stray markers
//   k_jsync_scan     a workgroup per image: chunk bases (exclusive prefix sums),
//                    the interval table's ends and the zero padding
//   k_jsync_scatter  a workgroup per chunk: the kept bytes to their unstuffed
//                    position (big-endian words), interval starts
//   k_jsync_sync     a thread per lane: warm-up, START, EXIT, block count, DC sums
//   k_jsync_fix      a thread per lane: re-decode an inconsistent lane from its
//                    predecessor's EXIT (the first fix round, at full occupancy)
//   k_jsync_settle   a workgroup per image: the remaining fix rounds, over a list
//                    of the lanes whose predecessor changed, until none is left
//   k_jsync_seg1..3  per-lane block bases and DC predictions: a segmented prefix
//                    sum over each interval's lanes (a wave per 64 lanes, the carries
//                    between chunks per image, then per lane), the padding's blocks
//                    cut, inconsistent lanes and bad codes flagged
//   k_jsync_decode   a thread per lane: its blocks from START, coefficients out
//                    (each block staged in LDS and stored whole)
#include "ik_internal.h"
#include "ik_jpeg_sync.h"

namespace ik {
using namespace jsync;

namespace {

constexpr int kChunk = 4096;         // scan bytes per unstuffing workgroup
constexpr int kUT = 256;             // unstuffing threads (16 bytes each)
constexpr int kLanesPerWG = 256;     // decoder lanes per workgroup (one image's)

__device__ const uint8_t kZzNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int x = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, o, 64);
        if (x >= o) v += u;
    }
    return v;
}

// byte i of image I's scan (-1 outside)
__device__ __forceinline__ int scan_byte(const JsImageDev& I, long long i) {
    return i >= 0 && i < (long long)I.scan_len ? (int)I.scan[i] : -1;
}

// a thread's 16 bytes: keep mask (bit k), RST mask (marker FF at byte k), stray marker
struct Bytes16 {
    uint32_t keep, rst;
    bool bad;
    uint8_t b[16];
};
__device__ __forceinline__ Bytes16 classify(const JsImageDev& I, long long base) {
    Bytes16 r;
    r.keep = r.rst = 0;
    r.bad = false;
    int prev = scan_byte(I, base - 1);
    int cur = scan_byte(I, base);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const long long i = base + k;
        const int next = scan_byte(I, i + 1);
        r.b[k] = (uint8_t)(cur < 0 ? 0 : cur);
        if (cur >= 0) {
            const bool last = i + 1 == (long long)I.scan_len;
            if (unstuff_keep(prev, cur, next, last)) r.keep |= 1u << k;
            if (unstuff_rst(cur, next)) r.rst |= 1u << k;
            if (unstuff_bad(cur, next, last)) r.bad = true;
        }
        prev = cur;
        cur = next;
    }
    return r;
}

// workgroup exclusive scan of two counters (256 threads = 4 waves)
__device__ __forceinline__ void wg_scan2(uint32_t a, uint32_t b, uint32_t& ea, uint32_t& eb, uint32_t& ta, uint32_t& tb) {
    __shared__ uint32_t s_a[4], s_b[4];
    const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 63) { s_a[w] = ia; s_b[w] = ib; }
    __syncthreads();
    uint32_t pa = 0, pb = 0;
    ta = tb = 0;
    for (int k = 0; k < 4; ++k) {
        if (k < w) { pa += s_a[k]; pb += s_b[k]; }
        ta += s_a[k];
        tb += s_b[k];
    }
    ea = pa + ia - a;
    eb = pb + ib - b;
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(kUT) void k_jsync_count(const JsImageDev* imgs, const int2* chunks, uint2* counts) {
    const int2 ck = chunks[blockIdx.x];  // (image, chunk within the image)
    const JsImageDev I = imgs[ck.x];
    const long long base = (long long)ck.y * kChunk + 16 * threadIdx.x;
    const Bytes16 r = classify(I, base);
    uint32_t ea, eb, ta, tb;
    wg_scan2((uint32_t)__builtin_popcount(r.keep), (uint32_t)__builtin_popcount(r.rst), ea, eb, ta, tb);
    if (r.bad) atomicOr(I.status, 1);
    if (threadIdx.x == 0) counts[blockIdx.x] = make_uint2(ta, tb);
}

// one workgroup per image: the chunks' exclusive bases (in place), the totals, the
// last interval's end, the zero padding past the data
__global__ __launch_bounds__(kUT) void k_jsync_scan(JsImageDev* imgs, uint2* counts) {
    JsImageDev& I = imgs[blockIdx.x];
    uint32_t ka = 0, kb = 0;
    for (int c0 = 0; c0 < I.nchunks; c0 += kUT) {
        const int c = c0 + (int)threadIdx.x;
        const uint2 v = c < I.nchunks ? counts[I.chunk0 + c] : make_uint2(0, 0);
        uint32_t ea, eb, ta, tb;
        wg_scan2(v.x, v.y, ea, eb, ta, tb);
        if (c < I.nchunks) counts[I.chunk0 + c] = make_uint2(ka + ea, kb + eb);
        ka += ta;
        kb += tb;
    }
    if (threadIdx.x == 0) {
        I.totals[0] = ka;
        I.totals[1] = kb;
        if ((long long)kb + 2 > I.ivl_cap) atomicOr(I.status, 2);  // more restart markers than the frame has intervals
        else {
            I.ivl[0] = 0;
            I.ivl[kb + 1] = 8ll * ka;
        }
    }
    // zero words past the data (the readers' padding), bytes big-endian-swizzled
    uint8_t* out = I.out;
    const long long pad0 = ka, pad1 = (((long long)ka + 3) & ~3ll) + 4ll * kPadWords;
    for (long long i = pad0 + threadIdx.x; i < pad1; i += kUT) out[(i & ~3ll) | (3 - (i & 3))] = 0;
}

__global__ __launch_bounds__(kUT) void k_jsync_scatter(const JsImageDev* imgs, const int2* chunks, const uint2* bases) {
    const int2 ck = chunks[blockIdx.x];
    const JsImageDev I = imgs[ck.x];
    const long long base = (long long)ck.y * kChunk + 16 * threadIdx.x;
    const Bytes16 r = classify(I, base);
    uint32_t ea, eb, ta, tb;
    wg_scan2((uint32_t)__builtin_popcount(r.keep), (uint32_t)__builtin_popcount(r.rst), ea, eb, ta, tb);
    const uint2 cb = bases[blockIdx.x];
    long long o = (long long)cb.x + ea;       // unstuffed position of this thread's first kept byte
    long long m = (long long)cb.y + eb;       // restart markers before this thread's bytes
    uint8_t* out = I.out;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if ((r.rst >> k) & 1u) {  // the next interval starts at the next kept byte
            ++m;
            if (m < I.ivl_cap) I.ivl[m] = 8 * o;
        }
        if ((r.keep >> k) & 1u) {
            out[(o & ~3ll) | (3 - (o & 3))] = r.b[k];  // big-endian 32-bit words
            ++o;
        }
    }
}

// ---- decoding -----------------------------------------------------------------------
namespace {
// the workgroup's image tables in LDS
struct JsLds {
    JpegHuffTables T;
    uint8_t zz[64];
};
// the workgroup's Scan in LDS: the per-block reads of its component tables
// (comp_of, td, ta by a lane's own MCU phase) are LDS reads, not memory loads
__device__ __forceinline__ void load_scan(const Scan* g, Scan& s) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&s);
    for (int i = threadIdx.x; i < (int)(sizeof(Scan) / 4); i += blockDim.x) dst[i] = src[i];
}
__device__ __forceinline__ void load_tables(const JpegHuffTables* g, JsLds& L) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&L.T);
    for (int i = threadIdx.x; i < (int)(sizeof(JpegHuffTables) / 4); i += blockDim.x) dst[i] = src[i];
    if (threadIdx.x < 64) L.zz[threadIdx.x] = kZzNat[threadIdx.x];
}

}  // namespace

// wg: (image, first lane of the image's lanes this workgroup takes)
__global__ __launch_bounds__(kLanesPerWG) void k_jsync_sync(const Scan* scans, const int2* wgs, LaneRec* recs) {
    __shared__ JsLds L;
    __shared__ Scan S;
    const int2 w = wgs[blockIdx.x];
    load_scan(scans + w.x, S);
    load_tables(scans[w.x].tabs, L);
    __syncthreads();
    const int r = w.y + (int)threadIdx.x;
    if (r >= S.ivl_lane[S.nivl]) return;
    const int k = lane_interval(S, r);
    const LaneGeom g = lane_geom(S, k, r - S.ivl_lane[k]);
    LaneRec rec;
    run_lane(S, L.T, L.zz, g, warm_start(S, g), rec);
    recs[S.lane0 + r] = rec;
}

// the first fix round, over every lane of the batch at full occupancy: an
// inconsistent lane re-decodes from its predecessor's EXIT (a predecessor
// re-decoded in the same round may be read before or after its update -- either
// is a valid state of the chain, its EXIT one 8-byte word; k_jsync_settle checks
// every lane again)
__global__ __launch_bounds__(kLanesPerWG) void k_jsync_fix(const Scan* scans, const int2* wgs, LaneRec* recs) {
    __shared__ JsLds L;
    __shared__ Scan S;
    __shared__ int s_any;
    const int2 w = wgs[blockIdx.x];
    load_scan(scans + w.x, S);
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    const int r = w.y + (int)threadIdx.x;
    const long long l = S.lane0 + r;
    int k = 0, q = 0;
    uint64_t from = 0;
    bool todo = false;
    if (r < S.ivl_lane[S.nivl]) {
        k = lane_interval(S, r);
        q = r - S.ivl_lane[k];
        if (q > 0) {
            from = __hip_atomic_load(&recs[l - 1].exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            todo = from != 0 && recs[l].start != from;
        }
    }
    if (todo) s_any = 1;
    __syncthreads();
    if (!s_any) return;  // (the whole workgroup: nothing to redo, no tables to load)
    load_tables(S.tabs, L);
    __syncthreads();
    if (!todo) return;
    const LaneGeom g = lane_geom(S, k, q);
    LaneRec rec;
    run_lane(S, L.T, L.zz, g, from, rec);
    rec.work += recs[l].work;
    recs[l].start = rec.start;
    recs[l].nblk = rec.nblk;
    recs[l].err = rec.err;
    recs[l].work = rec.work;
    for (int c = 0; c < 4; ++c) recs[l].dc[c] = rec.dc[c];
    __hip_atomic_store(&recs[l].exit, rec.exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The remaining fix rounds, one workgroup per image, until its lanes are
// consistent -- no launch and no host round trip per round.  A round works a list
// of lanes in passes of kSettleThreads: a listed lane whose START differs from its
// predecessor's EXIT re-decodes from that EXIT, the results are committed, and
// then each re-decoded lane whose successor's START differs from its new EXIT
// appends the successor to the next round's list.  The barriers between the three
// steps keep a pass free of races: every EXIT a pass reads was committed before
// it, a lane is committed by one thread, and successors are checked against
// committed STARTs.  The first list is a scan of all the image's lanes, and so is
// the list after one that overflowed.  After kSettleMaxRounds rounds the rest is
// left inconsistent (the bases pass flags it; the host decoder takes the image).
namespace {
constexpr int kSettleThreads = 1024;
constexpr int kSettleList = 4096;
constexpr int kSettleMaxRounds = 8192;
struct SettleLds {
    int lane[2][kSettleList];
    int n[2];
    int full[2];
};
}  // namespace

__global__ __launch_bounds__(kSettleThreads) void k_jsync_settle(const Scan* scans, LaneRec* recs, int* rounds_out) {
    __shared__ JsLds L;
    __shared__ Scan S;
    __shared__ SettleLds Q;
    const int t = threadIdx.x;
    load_scan(scans + blockIdx.x, S);
    load_tables(scans[blockIdx.x].tabs, L);
    if (t == 0) { Q.n[0] = Q.n[1] = 0; Q.full[0] = 1; Q.full[1] = 0; }
    __syncthreads();
    const int nl = S.ivl_lane[S.nivl];
    if (nl <= 1) return;
    LaneRec* const R = recs + S.lane0;
    // lane r (not an interval's first) against its predecessor's committed EXIT
    auto behind = [&](int r, uint64_t& f) -> bool {
        f = R[r - 1].exit;
        return f != 0 && R[r].start != f;
    };
    int round = 0;
    for (; round < kSettleMaxRounds; ++round) {
        const int c = round & 1, nx = c ^ 1;
        if (Q.full[c]) {  // the list from a scan of every lane
            if (t == 0) Q.n[c] = 0;
            __syncthreads();
            for (int r = t; r < nl; r += kSettleThreads) {
                uint64_t f;
                if (r == S.ivl_lane[lane_interval(S, r)] || !behind(r, f)) continue;
                const int i = atomicAdd(&Q.n[c], 1);
                if (i < kSettleList) Q.lane[c][i] = r;
            }
            __syncthreads();
        }
        const int nc = Q.n[c];
        const int n = nc < kSettleList ? nc : kSettleList;
        if (n == 0) break;
        __syncthreads();  // (every thread has read n[c] and full[c] before the resets below)
        if (t == 0) { Q.n[nx] = 0; Q.full[nx] = nc > kSettleList ? 1 : 0; }
        __syncthreads();
        for (int p0 = 0; p0 < n; p0 += kSettleThreads) {
            const int i = p0 + t;
            bool did = false;
            int r = 0, k = 0;
            LaneRec rec;
            if (i < n) {
                r = Q.lane[c][i];
                uint64_t f;
                if (behind(r, f)) {
                    k = lane_interval(S, r);
                    const LaneGeom g = lane_geom(S, k, r - S.ivl_lane[k]);
                    const int wk = R[r].work;
                    run_lane(S, L.T, L.zz, g, f, rec);
                    rec.work += wk;
                    did = true;
                }
            }
            __syncthreads();  // every read of the pass done
            if (did) R[r] = rec;
            __syncthreads();  // every commit of the pass done
            if (did && r + 1 < S.ivl_lane[k + 1] && rec.exit && R[r + 1].start != rec.exit) {
                const int j = atomicAdd(&Q.n[nx], 1);
                if (j < kSettleList) Q.lane[nx][j] = r + 1;
                else Q.full[nx] = 1;
            }
            __syncthreads();
        }
    }
    if (t == 0) atomicMax(rounds_out, round);
}

// ---- bases: segmented prefix sums of (blocks, DC sums) over each interval's lanes --
// pass 1, a wave per 64 lanes: the segmented scan inside the chunk (segment heads:
// the lanes that start an interval), per-lane exclusive partials into `bases`,
// the chunk's tail sums into `cs`
namespace {
struct ChunkSum {
    long long blocks;
    int dc[4];
    int head;   // a segment head in the chunk
    int pad;
    long long cin_blocks;  // pass 2: the carry into the chunk
    int cin_dc[4];
};
constexpr int kBaseVals = 5;  // blocks, dc[4]
}  // namespace

__global__ __launch_bounds__(kLanesPerWG) void k_jsync_seg1(const Scan* scans, const int2* wgs, const LaneRec* recs,
                                                            LaneBase* bases, ChunkSum* cs) {
    const int2 w = wgs[blockIdx.x];
    const Scan& S = scans[w.x];
    const int r = w.y + (int)threadIdx.x;
    const long long l = S.lane0 + r;
    const int x = threadIdx.x & 63;
    const bool in = r < S.ivl_lane[S.nivl];
    int v[kBaseVals] = {0, 0, 0, 0, 0};
    int f = 0;
    if (in) {
        const int k = lane_interval(S, r);
        f = S.ivl_lane[k] == r;
        const LaneRec& rc = recs[l];
        v[0] = rc.nblk;
        for (int c = 0; c < 4; ++c) v[1 + c] = rc.dc[c];
    }
    int val[kBaseVals];
    for (int c = 0; c < kBaseVals; ++c) val[c] = v[c];
    int fl = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int fu = __shfl_up(fl, o, 64);
        int u[kBaseVals];
#pragma unroll
        for (int c = 0; c < kBaseVals; ++c) u[c] = __shfl_up(val[c], o, 64);
        if (x >= o) {
            if (!fl) {
#pragma unroll
                for (int c = 0; c < kBaseVals; ++c) val[c] += u[c];
            }
            fl |= fu;
        }
    }
    LaneBase b;
    b.block = val[0] - v[0];
    b.count = v[0];
    for (int c = 0; c < 4; ++c) b.dc[c] = val[1 + c] - v[1 + c];
    b.head = fl;
    bases[l] = b;
    if (x == 63) {
        ChunkSum& q = cs[l >> 6];
        q.blocks = val[0];
        for (int c = 0; c < 4; ++c) q.dc[c] = val[1 + c];
        q.head = fl;
    }
}

// pass 2, a thread per image: the carries into its chunks, in order
__global__ __launch_bounds__(64) void k_jsync_seg2(const Scan* scans, int nimg, ChunkSum* cs) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= nimg) return;
    const Scan& S = scans[i];
    const long long c0 = S.lane0 >> 6, c1 = (S.lane0 + S.ivl_lane[S.nivl] + 63) >> 6;
    long long cb = 0;
    int cd[4] = {0, 0, 0, 0};
    for (long long c = c0; c < c1; ++c) {
        ChunkSum& q = cs[c];
        q.cin_blocks = cb;
        for (int k = 0; k < 4; ++k) q.cin_dc[k] = cd[k];
        if (q.head) {
            cb = q.blocks;
            for (int k = 0; k < 4; ++k) cd[k] = q.dc[k];
        } else {
            cb += q.blocks;
            for (int k = 0; k < 4; ++k) cd[k] += q.dc[k];
        }
    }
}

// pass 3, a thread per lane: carries, the cut at the interval's block count,
// the consistency and error checks
__global__ __launch_bounds__(kLanesPerWG) void k_jsync_seg3(const Scan* scans, const int2* wgs, const LaneRec* recs,
                                                            LaneBase* bases, const ChunkSum* cs, int* status) {
    const int2 w = wgs[blockIdx.x];
    const Scan& S = scans[w.x];
    const int r = w.y + (int)threadIdx.x;
    if (r >= S.ivl_lane[S.nivl]) return;
    const long long l = S.lane0 + r;
    const int k = lane_interval(S, r);
    const int q = r - S.ivl_lane[k];
    LaneBase b = bases[l];
    if (!b.head) {
        const ChunkSum& c = cs[l >> 6];
        b.block += c.cin_blocks;
        for (int j = 0; j < 4; ++j) b.dc[j] += c.cin_dc[j];
    }
    const long long want = k + 1 < S.nivl ? S.ivl_blocks : S.total_blocks - (long long)k * S.ivl_blocks;
    const LaneRec rc = recs[l];
    const long long before = b.block;
    long long take = (long long)rc.nblk;
    if (before + take > want) take = want - before;
    if (take < 0) take = 0;
    bool bad = false;
    if (q > 0 && (recs[l - 1].exit == 0 || rc.start != recs[l - 1].exit)) bad = true;   // not synchronised
    if (rc.start == 0 && take > 0) bad = true;
    if (rc.err && (long long)(rc.err - 1) < take) bad = true;                         // a bad code in a real block
    if (r + 1 == S.ivl_lane[k + 1] && before + rc.nblk < want) bad = true;            // blocks missing
    if (bad) atomicOr(status + w.x, 4);
    b.block = (long long)k * S.ivl_blocks + before;
    b.count = (int)take;
    bases[l] = b;
}

// the decode pass: each lane's blocks from its START, the coefficients of each
// block staged in LDS and stored whole (eight 16-byte stores)
__global__ __launch_bounds__(kLanesPerWG) void k_jsync_decode(const Scan* scans, const int2* wgs, const LaneRec* recs,
                                                              const LaneBase* bases, int* status) {
    __shared__ JsLds L;
    __shared__ __attribute__((aligned(16))) int16_t s_blk[kLanesPerWG * 64];
    __shared__ Scan S;
    const int2 w = wgs[blockIdx.x];
    load_scan(scans + w.x, S);
    load_tables(scans[w.x].tabs, L);
    for (int i = threadIdx.x; i < kLanesPerWG * 8; i += kLanesPerWG)
        reinterpret_cast<uint4*>(s_blk)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int r = w.y + (int)threadIdx.x;
    if (r >= S.ivl_lane[S.nivl]) return;
    const long long l = S.lane0 + r;
    const LaneBase B = bases[l];
    if (B.count <= 0) return;
    const int k = lane_interval(S, r);
    const LaneGeom g = lane_geom(S, k, r - S.ivl_lane[k]);
    const uint64_t st = recs[l].start;
    Bits br;
    br.init(S.words, st_bit(st), g.e);
    int j = st_j(st);
    int pred[4];
    for (int c = 0; c < 4; ++c) pred[c] = B.dc[c];
    typedef __attribute__((address_space(3))) int16_t lds_i16;
    // may_alias: the block's 16-byte reads must see block()'s 2-byte stores (without
    // it type-based alias analysis lets the compiler move the reads above them)
    typedef int16_t s8 __attribute__((ext_vector_type(8), __may_alias__));
    lds_i16* blk = (lds_i16*)(s_blk + threadIdx.x * 64);
    for (int i = 0; i < B.count; ++i) {
        const int c = S.comp_of[j];
        int diff;
        if (!block<true>(br, L.T, L.zz, S.td[c], S.ta[c], &diff, blk)) {
            atomicOr(status + w.x, 8);
            return;
        }
        pred[c] += diff;
        blk[0] = (int16_t)pred[c];
        // (a global-address-space store: a flat store would also count in lgkmcnt, and
        // every LDS table read of the next block would wait for it)
        typedef __attribute__((address_space(1))) s8 gs8;
        gs8* gb = (gs8*)(S.coef + block_index(S, B.block + i) * 64);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            gb[p] = reinterpret_cast<const __attribute__((address_space(3))) s8*>(blk)[p];
            reinterpret_cast<__attribute__((address_space(3))) s8*>(blk)[p] = s8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        j = j + 1 == S.bpm ? 0 : j + 1;
    }
}

// ---- launchers ------------------------------------------------------------------------
hipError_t launch_jsync_unstuff(JsImageDev* imgs, int nimg, const int2* chunks, int nchunks, uint2* counts,
                                hipStream_t s) {
    if (nimg <= 0 || nchunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_jsync_count, dim3(nchunks), dim3(kUT), 0, s, imgs, chunks, counts);
    hipLaunchKernelGGL(k_jsync_scan, dim3(nimg), dim3(kUT), 0, s, imgs, counts);
    hipLaunchKernelGGL(k_jsync_scatter, dim3(nchunks), dim3(kUT), 0, s, imgs, chunks, counts);
    return hipGetLastError();
}

hipError_t launch_jsync_sync(const Scan* scans, const int2* wgs, int nwg, LaneRec* recs, hipStream_t s) {
    if (nwg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_jsync_sync, dim3(nwg), dim3(kLanesPerWG), 0, s, scans, wgs, recs);
    return hipGetLastError();
}

hipError_t launch_jsync_fix(const Scan* scans, int nimg, const int2* wgs, int nwg, LaneRec* recs, int* rounds,
                            hipStream_t s) {
    if (nwg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_jsync_fix, dim3(nwg), dim3(kLanesPerWG), 0, s, scans, wgs, recs);
    hipLaunchKernelGGL(k_jsync_settle, dim3(nimg), dim3(kSettleThreads), 0, s, scans, recs, rounds);
    return hipGetLastError();
}

hipError_t launch_jsync_bases_decode(const Scan* scans, int nimg, const int2* wgs, int nwg, const LaneRec* recs,
                                     LaneBase* bases, void* chunk_scratch, int* status, hipStream_t s) {
    if (nwg <= 0) return hipSuccess;
    ChunkSum* cs = reinterpret_cast<ChunkSum*>(chunk_scratch);
    hipLaunchKernelGGL(k_jsync_seg1, dim3(nwg), dim3(kLanesPerWG), 0, s, scans, wgs, recs, bases, cs);
    hipLaunchKernelGGL(k_jsync_seg2, dim3((nimg + 63) / 64), dim3(64), 0, s, scans, nimg, cs);
    hipLaunchKernelGGL(k_jsync_seg3, dim3(nwg), dim3(kLanesPerWG), 0, s, scans, wgs, recs, bases, cs, status);
    hipLaunchKernelGGL(k_jsync_decode, dim3(nwg), dim3(kLanesPerWG), 0, s, scans, wgs, recs, bases, status);
    return hipGetLastError();
}

size_t jsync_chunk_scratch_bytes(long long lanes) { return (size_t)((lanes + 63) / 64) * sizeof(ChunkSum); }

}  // namespace ik
