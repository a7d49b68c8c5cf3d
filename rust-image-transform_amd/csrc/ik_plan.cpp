// ik_plan.cpp -- resize plans: the host half of resize_image's resampler.
//
// Weights follow image 0.25.8 src/imageops/sample.rs (vertical_sample /
// horizontal_sample, called from reference src/transform.rs:85-89): per output
// index, centre (o + 0.5) * ratio, support * max(ratio, 1), window
// [floor(c - s), ceil(c + s)) clamped, kernel((i - (c - 0.5)) / sratio),
// normalised by the sequential f32 sum (w /= sum).  They are computed once per
// geometry on the host -- with glibc sinf/expf, as rustc's f32::sin/exp are --
// and uploaded, so the device kernels only multiply and add.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "ik_internal.h"
#include "ik_runtime.h"


namespace ik {
namespace {

constexpr float kPi = 3.14159265358979323846264338327950288f;

float sinc(float t) {
    const float a = t * kPi;
    if (t == 0.0f) return 1.0f;
    return sinf(a) / a;
}

float kernel_eval(int filter, float x) {
    const float ax = fabsf(x);
    switch (filter) {
    case 0: return 1.0f;                                   // box_kernel (Nearest)
    case 1: return ax < 1.0f ? 1.0f - ax : 0.0f;           // triangle_kernel
    case 2: {                                              // catmullrom = bc_cubic_spline(x, 0, 0.5)
        const float b = 0.0f, c = 0.5f;
        float k;
        if (ax < 1.0f) {
            const float a2 = ax * ax, a3 = a2 * ax;
            k = (12.0f - 9.0f * b - 6.0f * c) * a3 + (-18.0f + 12.0f * b + 6.0f * c) * a2 +
                (6.0f - 2.0f * b);
        } else if (ax < 2.0f) {
            const float a2 = ax * ax, a3 = a2 * ax;
            k = (-b - 6.0f * c) * a3 + (6.0f * b + 30.0f * c) * a2 + (-12.0f * b - 48.0f * c) * ax +
                (8.0f * b + 24.0f * c);
        } else {
            k = 0.0f;
        }
        return k / 6.0f;
    }
    case 3: {                                              // gaussian_kernel = gaussian(x, 0.5)
        const float r = 0.5f;
        const float cst = 1.0f / (sqrtf(2.0f * kPi) * r);
        return cst * expf(-(x * x) / (2.0f * (r * r)));
    }
    default:                                               // lanczos3_kernel
        return ax < 3.0f ? sinc(x) * sinc(x / 3.0f) : 0.0f;
    }
}

float support_of(int filter) {
    switch (filter) {
    case 0: return 0.0f;
    case 1: return 1.0f;
    case 2: return 2.0f;
    default: return 3.0f;
    }
}

}  // namespace

int axis_weights(int in, int out, int filter, std::vector<int>& left, std::vector<int>& cnt,
                 std::vector<float>& w) {
    const float ratio = (float)in / (float)out;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float src_support = support_of(filter) * sratio;
    left.assign(out, 0);
    cnt.assign(out, 0);
    std::vector<std::vector<float>> rows(out);
    int T = 1;
    for (int o = 0; o < out; ++o) {
        float c = ((float)o + 0.5f) * ratio;
        long long l = (long long)floorf(c - src_support);
        l = l < 0 ? 0 : (l > in - 1 ? in - 1 : l);
        long long r = (long long)ceilf(c + src_support);
        r = r < l + 1 ? l + 1 : (r > in ? in : r);
        c = c - 0.5f;
        std::vector<float>& ws = rows[o];
        float sum = 0.0f;
        for (long long i = l; i < r; ++i) {
            const float wv = kernel_eval(filter, ((float)i - c) / sratio);
            ws.push_back(wv);
            sum = sum + wv;
        }
        for (float& wv : ws) wv = wv / sum;
        left[o] = (int)l;
        cnt[o] = (int)(r - l);
        if (cnt[o] > T) T = cnt[o];
    }
    T = (T + 3) & ~3;  // the fused kernel's horizontal pass runs taps in groups
    w.assign((size_t)out * T, 0.0f);
    for (int o = 0; o < out; ++o) std::memcpy(&w[(size_t)o * T], rows[o].data(), sizeof(float) * cnt[o]);
    return T;
}

// smallest A with left[r + A] >= left[r] + cnt[r] for every r: no more than A
// output rows are ever open at once in a top-to-bottom sweep
int required_slots(const std::vector<int>& left, const std::vector<int>& cnt) {
    const int n = (int)left.size();
    int A = 1;
    for (int r = 0; r < n; ++r) {
        const int end = left[r] + cnt[r];
        while (r + A < n && left[r + A] < end) ++A;
    }
    return A;
}

namespace {

std::mutex g_plan_mu;
std::map<std::tuple<int, int, int, int, int, int, int, int, int>, ResizePlan*> g_plans;
// request -> plan (several requests can share one plan in g_plans)
std::map<std::tuple<int, int, int, int, int, int, int, int>, ResizePlan*> g_front;

template <typename T>
size_t put(std::vector<char>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 255) & ~size_t(255);
    blob.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

}  // namespace

ResizePlan* build_resize_plan(int device, int W, int H, int C, int nw, int nh, int filter, int n);

ResizePlan* get_resize_plan(int device, int W, int H, int C, int nw, int nh, int filter, int n) {
    // front cache on the request itself, so a repeated geometry costs a map
    // lookup, not a recomputation of the weights
    const auto fkey = std::make_tuple(device, W, H, C, nw, nh, filter, n);
    {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        auto it = g_front.find(fkey);
        if (it != g_front.end()) return it->second;
    }
    ResizePlan* p = build_resize_plan(device, W, H, C, nw, nh, filter, n);
    if (p) {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        g_front[fkey] = p;
    }
    return p;
}

ResizePlan* build_resize_plan(int device, int W, int H, int C, int nw, int nh, int filter, int n) {
    // band height depends on how many images share the launch: aim for >= 2048
    // workgroups (8 per CU) without cutting bands below 32 rows
    std::vector<int> lx, cx, ly, cy;
    std::vector<float> wx, wy;
    const int Tx = axis_weights(W, nw, filter, lx, cx, wx);
    const int Ty = axis_weights(H, nh, filter, ly, cy, wy);
    int A = required_slots(ly, cy);
    int slots = A <= 2 ? 2 : A <= 4 ? 4 : A <= 8 ? 8 : A <= 16 ? 16 : 0;

    // prefetch depth: source rows consumed per output row after the first
    int maxblk = 1;
    for (int r = 1; r < nh; ++r) {
        const int b = ly[r] + cy[r] - std::max(ly[r - 1] + cy[r - 1], ly[r]);
        maxblk = std::max(maxblk, b);
    }
    int rows = maxblk <= 4 ? 4 : maxblk <= 8 ? 8 : 16;
    // non-spilling instances: A=4,8 -> R<=8, A=16 -> R=4 (larger blocks
    // take the kernel's chunked path)
    if (slots <= 8 && rows > 8) rows = 8;
    if (slots == 16) rows = 4;
    // column strips: as many output columns as fit kStripBytes source bytes (and,
    // when possible, kMaxStripWeights horizontal weights in LDS)
    bool wl = (long)Tx <= kMaxStripWeights;
    std::vector<int> strips;
    for (int pass = 0; pass < 2 && slots; ++pass) {
        strips.clear();
        bool ok = true;
        for (int ox0 = 0; ox0 < nw;) {
            const int sb = (lx[ox0] * C) & ~127;  // strip rows start on a 128-B line
            int ox1 = ox0;
            while (ox1 < nw && (lx[ox1] + cx[ox1]) * C - sb <= kStripBytes && ox1 - ox0 < kMaxStripCols &&
                   (!wl || (long)(ox1 - ox0 + 1) * Tx <= kMaxStripWeights))
                ++ox1;
            if (ox1 == ox0) { ok = false; break; }  // one output column wider than a strip
            strips.push_back(ox0); strips.push_back(ox1); strips.push_back(sb);
            ox0 = ox1;
        }
        if (!ok) { slots = 0; break; }
        // weights in LDS only when that costs at most ~10% more strips
        if (wl && pass == 0) {
            std::vector<int> keep = strips;
            int ns_wl = (int)strips.size() / 3;
            wl = false;
            strips.clear();
            int ns_gl = 0;
            for (int ox0 = 0; ox0 < nw;) {
                const int sb = (lx[ox0] * C) & ~127;  // strip rows start on a 128-B line
                int ox1 = ox0;
                while (ox1 < nw && (lx[ox1] + cx[ox1]) * C - sb <= kStripBytes && ox1 - ox0 < kMaxStripCols) ++ox1;
                ++ns_gl;
                ox0 = ox1 > ox0 ? ox1 : ox0 + 1;
            }
            if (ns_wl * 10 <= ns_gl * 11) { wl = true; strips = keep; break; }
            continue;  // second pass without the LDS-weights limit
        }
        break;
    }
    const int NS = slots ? (int)strips.size() / 3 : 0;
    int band_h = nh;
    if (slots) {
        const long target = 8192;  // measured best on MI355X for 4096^2->512^2 batches (tools/sweep_resize.py)
        long per_img = (target + n - 1) / n;
        long nb = (per_img + NS - 1) / NS;
        if (nb < 1) nb = 1;
        band_h = (int)((nh + nb - 1) / nb);
        // halo rows re-read per band ~ taps - ratio: short filters afford short bands
        const int min_band = Ty <= 20 ? 16 : 32;
        if (band_h < min_band) band_h = min_band;
        band_h = ((band_h + slots - 1) / slots) * slots;
        if (band_h > nh) band_h = nh;
    }
    // flush depth F (vertical rows staged in LDS per horizontal pass): 3 measured
    // best on MI355X for both triangle and lanczos3 8x downscales (deeper costs
    // resident workgroups, shallower runs the barrier-bound horizontal pass more
    // often; tools/sweep_resize.py FLUSH=2,3,4)
    const int flush = 3;
    const auto key = std::make_tuple(device, W, H, C, nw, nh, filter, band_h, flush);
    std::lock_guard<std::mutex> lk(g_plan_mu);
    auto it = g_plans.find(key);
    if (it != g_plans.end()) return it->second;

    std::vector<int> bands;
    for (int y = 0; y < nh; y += band_h) { bands.push_back(y); bands.push_back(y + band_h < nh ? y + band_h : nh); }

    // step tables (see ResizeArgs): per band, output row r needs source rows
    // [max(consumed, ly[r]), ly[r]+cy[r]); cut into steps of <= rows rows, the last
    // step of r emits it.
    std::vector<int> hdr, band_step;
    std::vector<unsigned long long> smask;
    std::vector<float> sw;
    if (slots) {
        for (size_t bi = 0; bi < bands.size(); bi += 2) {
            const int oy0 = bands[bi], oy1 = bands[bi + 1];
            band_step.push_back((int)smask.size());
            int consumed = ly[oy0];
            for (int r = oy0; r < oy1; ++r) {
                const int end = ly[r] + cy[r];
                int st = std::max(consumed, ly[r]);
                do {
                    const int cnt = std::min(rows, std::max(0, end - st));
                    unsigned long long m = 0;
                    std::vector<float> w((size_t)rows * slots, 0.0f);
                    for (int j = 0; j < cnt; ++j)
                        for (int d = 0; d < slots && r + d < oy1; ++d) {
                            const int kk = st + j - ly[r + d];
                            if (kk >= 0 && kk < cy[r + d]) {
                                m |= 1ull << (j * slots + d);
                                w[(size_t)j * slots + d] = wy[(size_t)(r + d) * Ty + kk];
                            }
                        }
                    st += cnt;
                    const int emit = st >= end ? 1 : 0;
                    hdr.push_back(st - cnt); hdr.push_back(cnt); hdr.push_back(emit); hdr.push_back(0);
                    smask.push_back(m);
                    sw.insert(sw.end(), w.begin(), w.end());
                    if (emit) break;
                } while (true);
                consumed = std::max(consumed, end);
            }
            // the kernel runs steps in pairs: pad an odd band with a no-op step
            // (no rows, no taps, no emit; its prefetch re-reads a valid row)
            if ((smask.size() - band_step.back()) & 1) {
                const int last = hdr[hdr.size() - 4];
                hdr.push_back(last); hdr.push_back(0); hdr.push_back(0); hdr.push_back(0);
                smask.push_back(0);
                sw.insert(sw.end(), (size_t)rows * slots, 0.0f);
            }
        }
        band_step.push_back((int)smask.size());
    }

    // Periodic geometry (integer ratio R, every output window inside steps y .. y+A-1
    // of R rows each, step t starting at source row R*t + base): k_resize_periodic
    // sweeps it with A accumulators whose roles rotate at compile time -- no step
    // masks, no accumulator shifts.  Taps outside an output's own window carry weight
    // 0 (+0 added to the sum, so the f32 sequence of the reference is unchanged; the
    // first tap is assigned, not added to 0, which can differ only in the sign of a
    // zero sum and so never in an output byte).
    int per_A = 0, per_R = 0, per_base = 0;
    std::vector<float> per_w;
    std::vector<int> per_bands;
    if (slots && nh > 0 && H % nh == 0) {
        const int R = H / nh;
        int lo = 1 << 30, hi = -(1 << 30);
        for (int y = 0; y < nh; ++y) {
            lo = std::min(lo, ly[y] - R * y);
            hi = std::max(hi, ly[y] + cy[y] - R * y);
        }
        const int A = (hi - lo + R - 1) / R;
        if (periodic_instance(A, R)) {
            per_A = A; per_R = R; per_base = lo;
        }
    }
    if (per_A) {
        const int A = per_A, R = per_R, G = A % 2 ? 2 * A : A;  // steps per unrolled group
        // bands: ~kPerTarget workgroups; a band of h rows sweeps h + A - 1 steps,
        // rounded up to whole groups (the extra steps emit nothing)
        long per_img = (kPerTargetWG + n - 1) / n;
        long nb = std::max(1L, (per_img + NS - 1) / NS);
        int h = (int)((nh + nb - 1) / nb);
        h = std::max(h, std::min(nh, kPerMinBand));
        h = ((h + A - 1 + G - 1) / G) * G - (A - 1);  // h + A - 1 a whole number of groups
        if (h < 1) h = std::min(nh, G);
        for (int y = 0; y < nh; y += h) { per_bands.push_back(y); per_bands.push_back(std::min(nh, y + h)); }
        const int nsteps = nh + A - 1 + G;  // the last band's rounding included
        per_w.assign((size_t)nsteps * A * R, 0.0f);
        for (int t = 0; t < nsteps; ++t)
            for (int e = 0; e < A; ++e) {
                const int y = t - e;
                if (y < 0 || y >= nh) continue;
                for (int j = 0; j < R; ++j) {
                    const int kk = R * t + per_base + j - ly[y];
                    if (kk >= 0 && kk < cy[y]) per_w[((size_t)t * A + e) * R + j] = wy[(size_t)y * Ty + kk];
                }
            }
    }

    std::vector<char> blob;
    const size_t o_pw = put(blob, per_w), o_pb = put(blob, per_bands);
    const size_t o_ly = put(blob, ly), o_cy = put(blob, cy), o_wy = put(blob, wy);
    const size_t o_lx = put(blob, lx), o_cx = put(blob, cx), o_wx = put(blob, wx);
    const size_t o_st = put(blob, strips), o_bd = put(blob, bands);
    const size_t o_sh = put(blob, hdr), o_sm = put(blob, smask), o_sw = put(blob, sw), o_bst = put(blob, band_step);

    auto* p = new ResizePlan();
    p->W = W; p->H = H; p->C = C; p->nw = nw; p->nh = nh; p->filter = filter;
    p->slots = slots;
    p->rows = rows;
    p->weights_in_lds = wl;
    p->flush = flush;
    p->NS = NS;
    p->NB = (int)bands.size() / 2;
    p->per_A = per_A;
    p->per_R = per_R;
    p->table_bytes = blob.size();
    // upload on this thread's stream, synchronised there (copy_h2d_2d): done
    // before any stream launches with the plan, without a device-wide sync
    if (hipMalloc(&p->dev_tables, blob.size()) != hipSuccess) p->dev_tables = nullptr;
    if (!p->dev_tables ||
        copy_h2d_2d(static_cast<uint8_t*>(p->dev_tables), blob.size(), reinterpret_cast<const uint8_t*>(blob.data()),
                    blob.size(), blob.size(), 1,
                    thread_stream()) != IK_OK) {
        if (p->dev_tables) (void)hipFree(p->dev_tables);
        delete p;
        return nullptr;
    }
    mem_stat(kMemPlans, (int64_t)p->table_bytes);
    char* d = static_cast<char*>(p->dev_tables);
    ResizeArgs& a = p->args;
    a.W = W; a.H = H; a.C = C; a.nw = nw; a.nh = nh; a.row_bytes = W * C;
    a.ly = (const int*)(d + o_ly); a.ny = (const int*)(d + o_cy); a.wy = (const float*)(d + o_wy); a.Ty = Ty;
    a.lx = (const int*)(d + o_lx); a.nx = (const int*)(d + o_cx); a.wx = (const float*)(d + o_wx); a.Tx = Tx;
    a.strips = (const int*)(d + o_st); a.NS = p->NS;
    a.max_strip_cols = 0;
    for (int k = 0; k < p->NS; ++k) a.max_strip_cols = std::max(a.max_strip_cols, strips[3 * k + 1] - strips[3 * k]);
    a.max_strip_cols = (a.max_strip_cols + 3) & ~3;
    a.max_strip_weights = (a.max_strip_cols * Tx + 3) & ~3;
    a.bands = (const int*)(d + o_bd); a.NB = p->NB;
    a.step_hdr = (const int*)(d + o_sh);
    a.step_mask = (const unsigned long long*)(d + o_sm);
    a.step_w = (const float*)(d + o_sw);
    a.band_step = (const int*)(d + o_bst);
    a.per_w = (const float*)(d + o_pw);
    a.per_bands = (const int*)(d + o_pb);
    a.per_base = per_base;
    a.NBp = (int)per_bands.size() / 2;
    g_plans[key] = p;
    return p;
}

// ik_shutdown: every cached plan's device tables
void plans_shutdown() {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    for (auto& kv : g_plans) {
        if (kv.second->dev_tables) {
            (void)hipFree(kv.second->dev_tables);
            mem_stat(kMemPlans, -(int64_t)kv.second->table_bytes);
        }
        delete kv.second;
    }
    g_plans.clear();
    g_front.clear();
}

}  // namespace ik
