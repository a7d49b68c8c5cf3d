// ik_codec.cpp -- host entropy stages of encode_image (reference src/transform.rs:113-150).
//
// WebP: the reference calls webp 0.3.1 Encoder::from_rgb(..).encode(q) over
// libwebp-sys 0.9.6's libwebp (Cargo.lock:2811, 1168): WebPConfigInit, quality=q,
// lossless=0, WebPPictureImportRGB (RGB->YUV420), WebPEncode.  Here the
// RGB->YUV420 step has already run on the GPU (k_webp_yuv420, bit-identical to
// libwebp's import); the planes are handed to libwebp's WebPEncode as a YUV
// picture, so the VP8 analysis / RD / token coding is libwebp's own.  libwebp is
// reached with dlopen("libwebp.so.7") -- no headers: the WebPPicture offsets are
// those of WEBP_ENCODER_ABI_VERSION 0x020f and are checked once at load time.
//
// JPEG: image 0.25.8 JpegEncoder (src/codecs/jpeg/encoder.rs): JFIF APP0 1.02
// density 1:1, SOF0 8-bit 3 components all 1x1 (4:4:4), DQT luma/chroma in zigzag
// order, the four standard DHT tables, one scan, BitWriter with 0xFF stuffing
// and the pad_byte() = write_bits(0x7F, 7) tail.  The quantised coefficients come
// from the GPU (k_jpeg_coeffs).
//
// AVIF: the reference uses image's AvifEncoder (ravif 0.11.20 -> rav1e 0.7.1,
// speed 4, quality q; Cargo.lock:1796, 1761).  rav1e is not available here, so
// the AV1 coding is libavif 1.x with its aom encoder (the copy bundled with the
// image's Pillow, or a system libavif.so.16), fed BT.601 full-range 4:4:4 planes
// (+ alpha when not opaque) from the GPU (k_avif_yuv444), speed 4, quality q.
// Output bytes differ from rav1e's; parity is a decoded-PSNR bound
// (tests/test_gpu_encode.py).  The avifImage / avifEncoder field offsets are those
// of libavif 1.x and are checked against the library's defaults before use.
#include <dlfcn.h>
#include <glob.h>

#include <cstring>
#include <mutex>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {
namespace {

// ---- libwebp through dlopen -------------------------------------------------
struct WebPApi {
    void* lib = nullptr;
    int (*config_init)(void*, int, float, int) = nullptr;
    int (*picture_init)(void*, int) = nullptr;
    void (*picture_free)(void*) = nullptr;
    int (*encode)(const void*, void*) = nullptr;
    int (*memory_write)(const uint8_t*, size_t, const void*) = nullptr;
    void (*writer_init)(void*) = nullptr;
    void (*writer_clear)(void*) = nullptr;
    int version = 0;  // WebPGetEncoderVersion(): 0x010600 = 1.6.0
    std::string path;  // the file the loader mapped
    bool ok = false;
    std::string err;
};

// The codec libraries are explicit dependencies of the product library: the path
// in $IK_LIBWEBP (resp. $IK_LIBAVIF) when set, else the system soname through the
// dynamic loader.  Nothing is searched for in other packages' directories.  A
// libwebp >= 1.3 built as separate objects needs its libsharpyuv: a
// libsharpyuv*.so* next to $IK_LIBWEBP is loaded first (RTLD_GLOBAL).  libwebp
// 1.2.2 (system) and 1.6.0 give identical lossy bytes on every test input (both
// are checked against the oracle, which loads the system copy); 1.6.0 codes a
// 512^2 frame ~8 % faster.  ik_libwebp_version() reports the one loaded.
void* open_libwebp() {
    std::vector<std::string> cands;
    if (const char* e = getenv("IK_LIBWEBP")) {
        if (*e) cands.push_back(e);
    }
    cands.push_back("libwebp.so.7");
    for (const auto& c : cands) {
        const size_t slash = c.rfind('/');
        if (slash != std::string::npos) {
            glob_t g{};
            if (glob((c.substr(0, slash) + "/libsharpyuv*.so*").c_str(), 0, nullptr, &g) == 0 && g.gl_pathc)
                dlopen(g.gl_pathv[0], RTLD_NOW | RTLD_GLOBAL);
            globfree(&g);
        }
        if (void* lib = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL)) {
            if (dlsym(lib, "WebPEncode") && dlsym(lib, "WebPConfigInitInternal")) return lib;
            dlclose(lib);
        }
    }
    return nullptr;
}

constexpr int kAbi = 0x020f;
constexpr size_t kPicWidth = 8, kPicHeight = 12, kPicY = 16, kPicU = 24, kPicV = 32;
constexpr size_t kPicYStride = 40, kPicUVStride = 44, kPicWriter = 96, kPicCustom = 104;
constexpr size_t kPicErrorCode = 136;

const WebPApi& webp_api() {
    static WebPApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        api.lib = open_libwebp();
        if (!api.lib) { api.err = "libwebp.so.7 not found (set IK_LIBWEBP to a libwebp path)"; return; }
        if (Dl_info di{}; dladdr(dlsym(api.lib, "WebPEncode"), &di) && di.dli_fname) api.path = di.dli_fname;
        if (auto ver = (int (*)())dlsym(api.lib, "WebPGetEncoderVersion")) api.version = ver();
        api.config_init = (int (*)(void*, int, float, int))dlsym(api.lib, "WebPConfigInitInternal");
        api.picture_init = (int (*)(void*, int))dlsym(api.lib, "WebPPictureInitInternal");
        api.picture_free = (void (*)(void*))dlsym(api.lib, "WebPPictureFree");
        api.encode = (int (*)(const void*, void*))dlsym(api.lib, "WebPEncode");
        api.memory_write = (int (*)(const uint8_t*, size_t, const void*))dlsym(api.lib, "WebPMemoryWrite");
        api.writer_init = (void (*)(void*))dlsym(api.lib, "WebPMemoryWriterInit");
        api.writer_clear = (void (*)(void*))dlsym(api.lib, "WebPMemoryWriterClear");
        if (!api.config_init || !api.picture_init || !api.picture_free || !api.encode ||
            !api.memory_write || !api.writer_init || !api.writer_clear) {
            api.err = "libwebp.so.7 lacks the WebPEncode API";
            return;
        }
        // layout check: WebPPictureAlloc must fill y/u/v and the strides where expected
        auto alloc = (int (*)(void*))dlsym(api.lib, "WebPPictureAlloc");
        alignas(16) unsigned char pic[512] = {0};
        if (!alloc || !api.picture_init(pic, kAbi)) { api.err = "WebPPictureInit failed"; return; }
        int w = 6, h = 5;
        std::memcpy(pic + kPicWidth, &w, 4);
        std::memcpy(pic + kPicHeight, &h, 4);
        if (!alloc(pic)) { api.err = "WebPPictureAlloc failed"; return; }
        void *y, *u, *v;
        int ys, uvs;
        std::memcpy(&y, pic + kPicY, 8); std::memcpy(&u, pic + kPicU, 8); std::memcpy(&v, pic + kPicV, 8);
        std::memcpy(&ys, pic + kPicYStride, 4); std::memcpy(&uvs, pic + kPicUVStride, 4);
        const bool layout_ok = y && u && v && ys == 6 && uvs == 3;
        api.picture_free(pic);
        if (!layout_ok) { api.err = "unexpected WebPPicture layout"; return; }
        api.ok = true;
    });
    return api;
}

}  // namespace

extern "C" int ik_libwebp_version(void) {
    const WebPApi& api = webp_api();
    return api.ok ? api.version : -1;
}

namespace ik {
const std::string& libwebp_path() { return webp_api().path; }
}  // namespace ik

int webp_encode_yuv420(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h,
                       float quality, std::vector<uint8_t>& out) {
    const WebPApi& api = webp_api();
    if (!api.ok) return fail(IK_ERR_TRANSFORM, "WebP encoder unavailable: %s", api.err.c_str());
    alignas(16) unsigned char config[512] = {0};
    alignas(16) unsigned char pic[512] = {0};
    alignas(16) unsigned char wrt[64] = {0};
    // WebPConfigPreset(&config, WEBP_PRESET_DEFAULT, q) == WebPConfigInit + quality; lossless = 0
    if (!api.config_init(config, 0, quality, kAbi)) return fail(IK_ERR_TRANSFORM, "WebPConfigInit failed");
    if (!api.picture_init(pic, kAbi)) return fail(IK_ERR_TRANSFORM, "WebPPictureInit failed");
    const int uvs = (w + 1) / 2;
    std::memcpy(pic + kPicWidth, &w, 4);
    std::memcpy(pic + kPicHeight, &h, 4);
    std::memcpy(pic + kPicY, &y, 8);
    std::memcpy(pic + kPicU, &u, 8);
    std::memcpy(pic + kPicV, &v, 8);
    std::memcpy(pic + kPicYStride, &w, 4);
    std::memcpy(pic + kPicUVStride, &uvs, 4);
    api.writer_init(wrt);
    void* wfn = (void*)api.memory_write;
    void* wp = wrt;
    std::memcpy(pic + kPicWriter, &wfn, 8);
    std::memcpy(pic + kPicCustom, &wp, 8);
    const int ok = api.encode(config, pic);
    int code = 0;
    std::memcpy(&code, pic + kPicErrorCode, 4);
    uint8_t* mem;
    size_t size;
    std::memcpy(&mem, wrt, 8);
    std::memcpy(&size, wrt + 8, 8);
    if (ok) out.assign(mem, mem + size);
    api.writer_clear(wrt);
    api.picture_free(pic);  // planes are ours: memory_ is NULL, nothing of ours is freed
    if (!ok) return fail(IK_ERR_TRANSFORM, "WebPEncode failed (error %d)", code);
    return IK_OK;
}

// ---- JPEG -------------------------------------------------------------------
namespace {

const uint8_t kLumaQ[64] = {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                            14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                            18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                            49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChromaQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                              24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
const uint8_t kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// JPEG Annex K.3 tables (bits[16] then values)
const uint8_t kLumaDcBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kChromaDcBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kLumaAcBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kLumaAcVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
const uint8_t kChromaAcBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kChromaAcVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};

struct Huff { uint16_t code[256]; uint8_t size[256]; };

Huff make_huff(const uint8_t bits[16], const uint8_t* vals) {
    Huff h{};
    int k = 0;
    uint16_t code = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int j = 0; j < bits[l - 1]; ++j, ++k, ++code) { h.code[vals[k]] = code; h.size[vals[k]] = (uint8_t)l; }
        code <<= 1;
    }
    return h;
}

struct Tables {
    Huff ldc, lac, cdc, cac;
    Tables()
        : ldc(make_huff(kLumaDcBits, kDcVals)), lac(make_huff(kLumaAcBits, kLumaAcVals)),
          cdc(make_huff(kChromaDcBits, kDcVals)), cac(make_huff(kChromaAcBits, kChromaAcVals)) {}
};

const Tables& tables() {
    static const Tables t;
    return t;
}

// 64-bit accumulator bit writer; emits the same bytes as encoder.rs BitWriter
struct Bits {
    std::vector<uint8_t>& out;
    uint64_t acc = 0;
    int n = 0;  // bits pending in acc (low bits)
    explicit Bits(std::vector<uint8_t>& o) : out(o) {}
    inline void put(uint32_t bits, int size) {
        acc = (acc << size) | (bits & ((1u << size) - 1u));
        n += size;
        while (n >= 8) {
            const uint8_t b = (uint8_t)(acc >> (n - 8));
            out.push_back(b);
            if (b == 0xFF) out.push_back(0);
            n -= 8;
        }
    }
};

inline void coef_bits(int c, int& nb, uint32_t& val) {
    const uint32_t mag = (uint32_t)(c < 0 ? -c : c);
    nb = mag ? 32 - __builtin_clz(mag) : 0;
    const uint32_t mask = (1u << nb) - 1u;
    val = (c < 0 ? (uint32_t)(c - 1) : (uint32_t)c) & mask;
}

inline int write_block(Bits& b, const int16_t* blk, int prevdc, const Huff& dc, const Huff& ac) {
    const int dcv = blk[0];
    int nb;
    uint32_t v;
    coef_bits(dcv - prevdc, nb, v);
    b.put(dc.code[nb], dc.size[nb]);
    if (nb) b.put(v, nb);
    int zr = 0;
    for (int i = 1; i < 64; ++i) {
        const int c = blk[kZig[i]];
        if (c == 0) { ++zr; continue; }
        while (zr > 15) { b.put(ac.code[0xF0], ac.size[0xF0]); zr -= 16; }
        coef_bits(c, nb, v);
        const int sym = (zr << 4) | nb;
        b.put(ac.code[sym], ac.size[sym]);
        b.put(v, nb);
        zr = 0;
    }
    if (blk[kZig[63]] == 0) b.put(ac.code[0], ac.size[0]);
    return dcv;
}

void segment(std::vector<uint8_t>& o, uint8_t marker, const uint8_t* d, size_t n) {
    o.push_back(0xFF); o.push_back(marker);
    o.push_back((uint8_t)((n + 2) >> 8)); o.push_back((uint8_t)((n + 2) & 0xFF));
    o.insert(o.end(), d, d + n);
}

}  // namespace

void jpeg_quant_tables(int quality, uint8_t qt[128]) {
    uint32_t s = (uint32_t)(quality < 1 ? 1 : quality > 100 ? 100 : quality);
    s = s < 50 ? 5000 / s : 200 - s * 2;
    for (int i = 0; i < 64; ++i) {
        uint32_t a = (kLumaQ[i] * s + 50) / 100, c = (kChromaQ[i] * s + 50) / 100;
        qt[i] = (uint8_t)(a < 1 ? 1 : a > 255 ? 255 : a);
        qt[64 + i] = (uint8_t)(c < 1 ? 1 : c > 255 ? 255 : c);
    }
}

void jpeg_huff_u32(uint32_t t[4 * 256]) {
    const Tables& T = tables();
    const Huff* hs[4] = {&T.ldc, &T.lac, &T.cdc, &T.cac};
    for (int k = 0; k < 4; ++k)
        for (int i = 0; i < 256; ++i) t[k * 256 + i] = (uint32_t)hs[k]->code[i] << 8 | hs[k]->size[i];
}

void jpeg_header(int w, int h, const uint8_t qt[128], std::vector<uint8_t>& out) {
    out.clear();
    out.push_back(0xFF); out.push_back(0xD8);
    const uint8_t jfif[14] = {'J', 'F', 'I', 'F', 0, 1, 2, 0, 0, 1, 0, 1, 0, 0};
    segment(out, 0xE0, jfif, sizeof(jfif));
    const uint8_t sof[15] = {8, (uint8_t)(h >> 8), (uint8_t)h, (uint8_t)(w >> 8), (uint8_t)w, 3,
                             1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1};
    segment(out, 0xC0, sof, sizeof(sof));
    for (int t = 0; t < 2; ++t) {
        uint8_t d[65];
        d[0] = (uint8_t)t;
        for (int i = 0; i < 64; ++i) d[1 + i] = qt[t * 64 + kZig[i]];
        segment(out, 0xDB, d, 65);
    }
    struct { uint8_t tc; const uint8_t* bits; const uint8_t* vals; int nv; } dht[4] = {
        {0x00, kLumaDcBits, kDcVals, 12}, {0x10, kLumaAcBits, kLumaAcVals, 162},
        {0x01, kChromaDcBits, kDcVals, 12}, {0x11, kChromaAcBits, kChromaAcVals, 162}};
    for (auto& t : dht) {
        uint8_t seg[1 + 16 + 162];
        seg[0] = t.tc;
        std::memcpy(seg + 1, t.bits, 16);
        std::memcpy(seg + 17, t.vals, (size_t)t.nv);
        segment(out, 0xC4, seg, (size_t)(17 + t.nv));
    }
    const uint8_t sos[10] = {3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    segment(out, 0xDA, sos, sizeof(sos));
}

void jpeg_write(const int16_t* coef, int w, int h, const uint8_t qt[128], std::vector<uint8_t>& out) {
    const Tables& T = tables();
    const size_t nmcu = (size_t)((w + 7) / 8) * ((h + 7) / 8);
    jpeg_header(w, h, qt, out);
    out.reserve(out.size() + nmcu * 64);
    Bits b(out);
    int pdc[3] = {0, 0, 0};
    for (size_t m = 0; m < nmcu; ++m) {
        const int16_t* blk = coef + m * 192;
        pdc[0] = write_block(b, blk, pdc[0], T.ldc, T.lac);
        pdc[1] = write_block(b, blk + 64, pdc[1], T.cdc, T.cac);
        pdc[2] = write_block(b, blk + 128, pdc[2], T.cdc, T.cac);
    }
    b.put(0x7F, 7);  // pad_byte(); leftover bits (< 8) are dropped, as in BitWriter
    out.push_back(0xFF); out.push_back(0xD9);
}

// ---- AVIF through libavif (dlopen) ---------------------------------------------
namespace {

struct AvifApi {
    void* lib = nullptr;
    void* (*image_create)(uint32_t, uint32_t, uint32_t, int) = nullptr;
    int (*image_alloc)(void*, int) = nullptr;
    void (*image_destroy)(void*) = nullptr;
    void* (*encoder_create)() = nullptr;
    void (*encoder_destroy)(void*) = nullptr;
    int (*encoder_write)(void*, const void*, void*) = nullptr;
    void (*rwdata_free)(void*) = nullptr;
    std::string path;  // the file the loader mapped
    bool ok = false;
    std::string err;
};

// libavif 1.x layouts (include/avif/avif.h)
constexpr size_t kImgRange = 16, kImgPlanes = 24, kImgRowBytes = 48, kImgAlpha = 64, kImgAlphaRowBytes = 72;
constexpr size_t kImgCicp = 104;  // colorPrimaries, transferCharacteristics, matrixCoefficients (u16 each)
constexpr size_t kEncMaxThreads = 4, kEncSpeed = 8, kEncQuality = 32, kEncQualityAlpha = 36;
constexpr int kYuv444 = 1, kPlanesYuv = 1, kPlanesAll = 0xff;

const AvifApi& avif_api() {
    static AvifApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        std::vector<std::string> cands;
        // explicit dependency, as libwebp above: $IK_LIBAVIF, else the system soname
        if (const char* e = getenv("IK_LIBAVIF")) {
            if (*e) cands.push_back(e);
        }
        cands.push_back("libavif.so.16");
        for (const auto& c : cands)
            if ((api.lib = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL))) break;
        if (!api.lib) {
            api.err = "libavif (with an AV1 encoder) not found: install libavif.so.16 or set IK_LIBAVIF to its path";
            return;
        }
        if (Dl_info di{}; dladdr(dlsym(api.lib, "avifVersion"), &di) && di.dli_fname) api.path = di.dli_fname;
        api.image_create = (void* (*)(uint32_t, uint32_t, uint32_t, int))dlsym(api.lib, "avifImageCreate");
        api.image_alloc = (int (*)(void*, int))dlsym(api.lib, "avifImageAllocatePlanes");
        api.image_destroy = (void (*)(void*))dlsym(api.lib, "avifImageDestroy");
        api.encoder_create = (void* (*)())dlsym(api.lib, "avifEncoderCreate");
        api.encoder_destroy = (void (*)(void*))dlsym(api.lib, "avifEncoderDestroy");
        api.encoder_write = (int (*)(void*, const void*, void*))dlsym(api.lib, "avifEncoderWrite");
        api.rwdata_free = (void (*)(void*))dlsym(api.lib, "avifRWDataFree");
        auto version = (const char* (*)())dlsym(api.lib, "avifVersion");
        if (!api.image_create || !api.image_alloc || !api.image_destroy || !api.encoder_create ||
            !api.encoder_destroy || !api.encoder_write || !api.rwdata_free || !version || version()[0] != '1') {
            api.err = "libavif 1.x encoder API not found";
            return;
        }
        // layout check against the documented defaults of a fresh image / encoder
        void* img = api.image_create(291, 69, 8, kYuv444);
        void* enc = api.encoder_create();
        bool ok = img && enc;
        if (ok) {
            uint32_t whd[3]; int fmt_range[2]; uint16_t cicp[3]; int e[4];
            std::memcpy(whd, img, 12);
            std::memcpy(fmt_range, (char*)img + 12, 8);
            std::memcpy(cicp, (char*)img + kImgCicp, 6);
            std::memcpy(e, enc, 16);
            ok = whd[0] == 291 && whd[1] == 69 && whd[2] == 8 && fmt_range[0] == kYuv444 && fmt_range[1] == 1 &&
                 cicp[0] == 2 && cicp[1] == 2 && cicp[2] == 2 && e[1] == 1 && e[2] == -1;
            int qa[2];
            std::memcpy(qa, (char*)enc + kEncQuality, 8);
            ok = ok && qa[0] == -1 && qa[1] == -1;
        }
        if (img) api.image_destroy(img);
        if (enc) api.encoder_destroy(enc);
        if (!ok) { api.err = "unexpected libavif struct layout"; return; }
        api.ok = true;
    });
    return api;
}

}  // namespace

// the file behind an encoder, for reports: fmt IK_FORMAT_WEBP / IK_FORMAT_AVIF
extern "C" size_t ik_codec_library(int fmt, char* buf, size_t cap) {
    std::string p;
    if (fmt == IK_FORMAT_WEBP) p = webp_api().ok ? webp_api().path : std::string();
    else if (fmt == IK_FORMAT_AVIF) p = avif_api().ok ? avif_api().path : std::string();
    if (buf && cap) {
        const size_t n = p.size() < cap - 1 ? p.size() : cap - 1;
        std::memcpy(buf, p.data(), n);
        buf[n] = 0;
    }
    return p.size();
}

int avif_encode_yuv444(const uint8_t* planes, bool has_alpha, int w, int h, int quality, int speed,
                       std::vector<uint8_t>& out) {
    const AvifApi& api = avif_api();
    if (!api.ok) return fail(IK_ERR_UNSUPPORTED, "AVIF encoding unavailable: %s", api.err.c_str());
    void* img = api.image_create((uint32_t)w, (uint32_t)h, 8, kYuv444);
    void* enc = api.encoder_create();
    auto cleanup = [&] { if (img) api.image_destroy(img); if (enc) api.encoder_destroy(enc); };
    if (!img || !enc) { cleanup(); return fail(IK_ERR_NOMEM, "avif: out of memory"); }
    const int full = 1;
    const uint16_t cicp[3] = {1, 13, 6};  // BT.709 primaries, sRGB transfer, BT.601 matrix
    std::memcpy((char*)img + kImgRange, &full, 4);
    std::memcpy((char*)img + kImgCicp, cicp, 6);
    if (api.image_alloc(img, has_alpha ? kPlanesAll : kPlanesYuv) != 0) {
        cleanup();
        return fail(IK_ERR_NOMEM, "avif: cannot allocate planes");
    }
    const size_t n = (size_t)w * h;
    for (int pl = 0; pl < 4; ++pl) {
        if (pl == 3 && !has_alpha) break;
        uint8_t* dst;
        uint32_t rb;
        if (pl < 3) {
            std::memcpy(&dst, (char*)img + kImgPlanes + 8 * pl, 8);
            std::memcpy(&rb, (char*)img + kImgRowBytes + 4 * pl, 4);
        } else {
            std::memcpy(&dst, (char*)img + kImgAlpha, 8);
            std::memcpy(&rb, (char*)img + kImgAlphaRowBytes, 4);
        }
        if (!dst || rb < (uint32_t)w) { cleanup(); return fail(IK_ERR_TRANSFORM, "avif: bad plane layout"); }
        for (int y = 0; y < h; ++y) std::memcpy(dst + (size_t)y * rb, planes + pl * n + (size_t)y * w, (size_t)w);
    }
    const int threads = 1, q2[2] = {quality, quality};
    std::memcpy((char*)enc + kEncMaxThreads, &threads, 4);
    std::memcpy((char*)enc + kEncSpeed, &speed, 4);
    std::memcpy((char*)enc + kEncQuality, q2, 8);
    struct { uint8_t* data; size_t size; } rw{nullptr, 0};
    const int r = api.encoder_write(enc, img, &rw);
    if (r != 0 || !rw.data) {
        if (rw.data) api.rwdata_free(&rw);
        cleanup();
        return fail(IK_ERR_TRANSFORM, "Encoding error: avifEncoderWrite failed (%d)", r);
    }
    out.assign(rw.data, rw.data + rw.size);
    api.rwdata_free(&rw);
    cleanup();
    return IK_OK;
}

}  // namespace ik
