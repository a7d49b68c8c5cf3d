// ik_decode.cpp -- decode_image's format sniffing and the host entropy decoders
// (reference src/transform.rs:27-43: image::guess_format +
// load_from_memory_with_format with the crate features of Cargo.toml:20).
//
//  - guess_format: image 0.25.8's magic-byte table (src/image_reader/free_functions.rs)
//  - PNG  (png 0.18 via image, Transformations::EXPAND): zlib inflate, CRC check,
//         unfilter (None/Sub/Up/Average/Paeth), Adam7, palette/tRNS/low-bit
//         expansion.  Spec-exact; 16-bit PNGs are reported as unsupported.
//  - WebP (image-webp 0.2.4 in the reference): libwebp's decoder via dlopen.
//  - JPEG (zune-jpeg 0.4.21 in the reference): ik_jpeg_decode.cpp.
// Pixel results are uploaded to the device by ik_decode (ik_host.cpp).
#include <dlfcn.h>
#include <zlib.h>

#include <cstring>
#include <mutex>

#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {

Sniffed guess_format(const uint8_t* b, size_t n) {
    auto has = [&](const char* m, size_t k) { return n >= k && std::memcmp(b, m, k) == 0; };
    if (has("\x89PNG\r\n\x1a\n", 8)) return Sniffed::Png;
    if (n >= 3 && b[0] == 0xFF && b[1] == 0xD8 && b[2] == 0xFF) return Sniffed::Jpeg;
    if (has("GIF89a", 6) || has("GIF87a", 6)) return Sniffed::Gif;
    if (n >= 12 && std::memcmp(b, "RIFF", 4) == 0 && std::memcmp(b + 8, "WEBP", 4) == 0) return Sniffed::WebP;
    if (has("MM\x00*", 4) || has("II*\x00", 4)) return Sniffed::Tiff;
    if (has("DDS ", 4)) return Sniffed::Dds;
    if (has("BM", 2)) return Sniffed::Bmp;
    if (n >= 4 && b[0] == 0 && b[1] == 0 && b[2] == 1 && b[3] == 0) return Sniffed::Ico;
    if (has("#?RADIANCE", 10)) return Sniffed::Hdr;
    if (n >= 12 && std::memcmp(b + 4, "ftypavif", 8) == 0) return Sniffed::Avif;
    if (n >= 4 && b[0] == 0x76 && b[1] == 0x2f && b[2] == 0x31 && b[3] == 0x01) return Sniffed::OpenExr;
    if (has("qoif", 4)) return Sniffed::Qoi;
    if (has("farbfeld", 8)) return Sniffed::Farbfeld;
    if (n >= 2 && b[0] == 'P' && b[1] >= '1' && b[1] <= '7') return Sniffed::Pnm;
    return Sniffed::Unknown;
}

const char* format_name(Sniffed f) {
    switch (f) {
    case Sniffed::Png: return "Png";
    case Sniffed::Jpeg: return "Jpeg";
    case Sniffed::Gif: return "Gif";
    case Sniffed::WebP: return "WebP";
    case Sniffed::Tiff: return "Tiff";
    case Sniffed::Bmp: return "Bmp";
    case Sniffed::Ico: return "Ico";
    case Sniffed::Hdr: return "Hdr";
    case Sniffed::Avif: return "Avif";
    case Sniffed::OpenExr: return "OpenExr";
    case Sniffed::Qoi: return "Qoi";
    case Sniffed::Farbfeld: return "Farbfeld";
    case Sniffed::Pnm: return "Pnm";
    case Sniffed::Dds: return "Dds";
    default: return "Unknown";
    }
}

// ---- PNG --------------------------------------------------------------------
namespace {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

// libdeflate (system libdeflate.so.0, dlopen'd; about twice zlib's inflate rate on
// image data).  Only its one-shot zlib decompressor is used, and only when the
// stream inflates to exactly the expected size; anything else goes through zlib
// so that error and trailing-data behaviour stay those of the zlib path.
struct Deflate {
    void* (*alloc)() = nullptr;
    int (*zlib_decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*release)(void*) = nullptr;
    uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;  // same convention as zlib's crc32
    bool ok = false;
};
const Deflate& deflate_api() {
    static Deflate d;
    static std::once_flag once;
    std::call_once(once, [] {
        void* lib = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!lib) return;
        d.alloc = (void* (*)())dlsym(lib, "libdeflate_alloc_decompressor");
        d.zlib_decompress = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(lib, "libdeflate_zlib_decompress");
        d.release = (void (*)(void*))dlsym(lib, "libdeflate_free_decompressor");
        d.crc32 = (uint32_t (*)(uint32_t, const void*, size_t))dlsym(lib, "libdeflate_crc32");
        d.ok = d.alloc && d.zlib_decompress && d.release;
    });
    return d;
}

bool inflate_exact_libdeflate(const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
    const Deflate& d = deflate_api();
    if (!d.ok) return false;
    thread_local struct Holder {
        void* p = nullptr;
        ~Holder() { if (p) deflate_api().release(p); }
    } h;
    if (!h.p) h.p = d.alloc();
    if (!h.p) return false;
    size_t got = 0;
    return d.zlib_decompress(h.p, in.data(), in.size(), out.data(), out.size(), &got) == 0 && got == out.size();
}

}  // namespace

uint32_t png_chunk_crc(const uint8_t* type, const uint8_t* data, size_t len) {
    const Deflate& d = deflate_api();
    if (d.ok && d.crc32) return d.crc32(d.crc32(0, type, 4), data, len);
    return (uint32_t)crc32(crc32(0, type, 4), data, len);
}

namespace {

// Per-thread compressed/filtered buffers, kept between decodes (first-touch page
// faults cost as much as the unfiltering); released after images over 128 MiB.
struct PngScratch {
    std::vector<uint8_t> idat, raw, samp;  // samp trades buffers with the caller's px (swap)
};
struct PngScratchGuard {
    PngScratch& s;
    ~PngScratchGuard() {
        s.idat.clear();
        if (s.idat.capacity() > (128u << 20)) std::vector<uint8_t>().swap(s.idat);
        if (s.raw.capacity() > (128u << 20)) std::vector<uint8_t>().swap(s.raw);
        if (s.samp.capacity() > (128u << 20)) std::vector<uint8_t>().swap(s.samp);
    }
};

// unfilter one (sub)image of `h` rows of `rowbytes` bytes, bpp = bytes per complete pixel
bool unfilter(uint8_t* data, size_t h, size_t rowbytes, size_t bpp, std::vector<uint8_t>& out) {
    out.resize(h * rowbytes);
    std::vector<uint8_t> zero(rowbytes, 0);
    for (size_t y = 0; y < h; ++y) {
        const uint8_t ft = data[y * (rowbytes + 1)];
        const uint8_t* in = data + y * (rowbytes + 1) + 1;
        uint8_t* cur = out.data() + y * rowbytes;
        const uint8_t* prev = y ? out.data() + (y - 1) * rowbytes : zero.data();
        switch (ft) {
        case 0: std::memcpy(cur, in, rowbytes); break;
        case 1: {
            const size_t b0 = bpp < rowbytes ? bpp : rowbytes;
            for (size_t i = 0; i < b0; ++i) cur[i] = in[i];
            for (size_t i = b0; i < rowbytes; ++i) cur[i] = (uint8_t)(in[i] + cur[i - bpp]);
            break;
        }
        case 2:
            for (size_t i = 0; i < rowbytes; ++i) cur[i] = (uint8_t)(in[i] + prev[i]);
            break;
        case 3:
            for (size_t i = 0; i < rowbytes; ++i)
                cur[i] = (uint8_t)(in[i] + (((i >= bpp ? cur[i - bpp] : 0) + prev[i]) >> 1));
            break;
        case 4:
            for (size_t i = 0; i < rowbytes; ++i)
                cur[i] = (uint8_t)(in[i] + paeth(i >= bpp ? cur[i - bpp] : 0, prev[i], i >= bpp ? prev[i - bpp] : 0));
            break;
        default: return false;
        }
    }
    return true;
}

}  // namespace

int decode_png(const uint8_t* b, size_t n, uint32_t& W, uint32_t& H, uint32_t& C, std::vector<uint8_t>& px,
               uint32_t* depth_out) {
    size_t pos = 8;
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    thread_local PngScratch scratch;
    PngScratchGuard guard{scratch};
    std::vector<uint8_t>& idat = scratch.idat;
    idat.clear();
    std::vector<uint8_t> plte, trns;
    bool seen_ihdr = false, seen_iend = false;
    while (pos + 12 <= n) {
        const uint32_t len = be32(b + pos);
        if (len > n - pos - 12) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: truncated chunk");
        const uint8_t* type = b + pos + 4;
        const uint8_t* data = b + pos + 8;
        const uint32_t crc = be32(data + len);
        if (png_chunk_crc(type, data, len) != crc)
            return fail(IK_ERR_TRANSFORM, "Format error decoding Png: CRC error");
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: bad IHDR");
            w = be32(data); h = be32(data + 4); depth = data[8]; ctype = data[9]; interlace = data[12];
            seen_ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            seen_iend = true;
            break;
        }
        pos += 12 + len;
    }
    if (!seen_ihdr || idat.empty()) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: missing IHDR/IDAT");
    (void)seen_iend;
    if (!w || !h) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: zero dimension");
    int spp;  // samples per pixel
    switch (ctype) {
    case 0: spp = 1; break;
    case 2: spp = 3; break;
    case 3: spp = 1; break;
    case 4: spp = 2; break;
    case 6: spp = 4; break;
    default: return fail(IK_ERR_TRANSFORM, "Format error decoding Png: bad color type %d", ctype);
    }
    if (depth == 16 && ctype == 3) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: bad bit depth 16");
    if (depth == 16 && !depth_out) return fail(IK_ERR_UNSUPPORTED, "16-bit PNG decoding needs a 16-bit image");
    if (!(depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4))))
        return fail(IK_ERR_TRANSFORM, "Format error decoding Png: bad bit depth %d", depth);
    if (ctype == 3 && (plte.empty() || plte.size() % 3)) return fail(IK_ERR_TRANSFORM, "Format error decoding Png: bad palette");
    {  // image's default Limits: max_alloc 512 MiB of DECODED bytes (after EXPAND: palette,
       // tRNS alpha, low bit depths to 8; 16-bit samples take two bytes)
        const uint64_t out_c = ctype == 3 ? (trns.empty() ? 3 : 4)
                             : ctype == 0 ? (trns.size() >= 2 ? 2 : 1)
                             : ctype == 2 ? (trns.size() >= 6 ? 4 : 3) : (uint64_t)spp;
        if ((uint64_t)w * h * out_c * (depth == 16 ? 2 : 1) > (512ull << 20))
            return fail(IK_ERR_TRANSFORM, "Limits are exceeded");
    }

    const size_t bits_pp = (size_t)spp * depth;
    const size_t bpp = (bits_pp + 7) / 8;
    auto rowbytes_of = [&](size_t width) { return (width * bits_pp + 7) / 8; };
    // total raw size over the passes
    struct Pass { size_t x0, y0, dx, dy; };
    const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const Pass whole[1] = {{0, 0, 1, 1}};
    const Pass* passes = interlace ? adam7 : whole;
    const int npass = interlace ? 7 : 1;
    size_t raw_total = 0;
    for (int p = 0; p < npass; ++p) {
        const size_t pw = (w - passes[p].x0 + passes[p].dx - 1) / passes[p].dx;
        const size_t ph = (h - passes[p].y0 + passes[p].dy - 1) / passes[p].dy;
        if (passes[p].x0 >= w || passes[p].y0 >= h) continue;
        raw_total += ph * (rowbytes_of(pw) + 1);
    }
    std::vector<uint8_t>& raw = scratch.raw;
    raw.resize(raw_total);  // contents are overwritten by the inflate (or the decode fails)
    if (!inflate_exact_libdeflate(idat, raw)) {
        z_stream zs{};
        if (inflateInit(&zs) != Z_OK) return fail(IK_ERR_TRANSFORM, "zlib init failed");
        zs.next_in = idat.data();
        zs.avail_in = (uInt)idat.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        int zr = inflate(&zs, Z_FINISH);
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if (got != raw.size() || (zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK))
            return fail(IK_ERR_TRANSFORM, "Format error decoding Png: corrupt deflate stream");
    }

    if (depth == 16) {  // big-endian u16 samples -> native u16; tRNS -> alpha 0 / 65535
        const bool ka = (ctype == 0 && trns.size() >= 2) || (ctype == 2 && trns.size() >= 6);
        const uint32_t oc = (uint32_t)spp + (ka ? 1u : 0u);
        std::vector<uint16_t> s16((size_t)w * h * oc);
        std::vector<uint8_t> rows;
        size_t off16 = 0;
        for (int p = 0; p < npass; ++p) {
            if (passes[p].x0 >= w || passes[p].y0 >= h) continue;
            const size_t pw = (w - passes[p].x0 + passes[p].dx - 1) / passes[p].dx;
            const size_t ph = (h - passes[p].y0 + passes[p].dy - 1) / passes[p].dy;
            const size_t rb = rowbytes_of(pw);
            if (!unfilter(raw.data() + off16, ph, rb, bpp, rows))
                return fail(IK_ERR_TRANSFORM, "Format error decoding Png: unknown filter method");
            off16 += ph * (rb + 1);
            for (size_t y = 0; y < ph; ++y) {
                const uint8_t* r = rows.data() + y * rb;
                const size_t oy = passes[p].y0 + y * passes[p].dy;
                for (size_t x = 0; x < pw; ++x) {
                    const size_t ox = passes[p].x0 + x * passes[p].dx;
                    uint16_t* o = s16.data() + (oy * w + ox) * oc;
                    bool key = ka;
                    for (int k = 0; k < spp; ++k) {
                        const uint16_t v = (uint16_t)(r[2 * (x * spp + k)] << 8 | r[2 * (x * spp + k) + 1]);
                        o[k] = v;
                        if (ka) key = key && v == (uint16_t)(trns[2 * k] << 8 | trns[2 * k + 1]);
                    }
                    if (ka) o[spp] = key ? 0 : 65535;
                }
            }
        }
        W = w;
        H = h;
        C = oc;
        px.resize(s16.size() * 2);
        std::memcpy(px.data(), s16.data(), px.size());
        *depth_out = 2;
        return IK_OK;
    }
    if (depth_out) *depth_out = 1;
    // samples at 8 bits per sample (expanded), spp per pixel, full image
    std::vector<uint8_t>& samp = scratch.samp;  // every sample is written below
    size_t off = 0;
    std::vector<uint8_t> rows;
    if (depth == 8 && !interlace) {  // the unfiltered rows are the samples: no repacking
        if (!unfilter(raw.data(), h, rowbytes_of(w), bpp, samp))
            return fail(IK_ERR_TRANSFORM, "Format error decoding Png: unknown filter method");
    } else {
        samp.resize((size_t)w * h * spp);
    }
    for (int p = 0; p < (depth == 8 && !interlace ? 0 : npass); ++p) {
        if (passes[p].x0 >= w || passes[p].y0 >= h) continue;
        const size_t pw = (w - passes[p].x0 + passes[p].dx - 1) / passes[p].dx;
        const size_t ph = (h - passes[p].y0 + passes[p].dy - 1) / passes[p].dy;
        const size_t rb = rowbytes_of(pw);
        if (!unfilter(raw.data() + off, ph, rb, bpp, rows))
            return fail(IK_ERR_TRANSFORM, "Format error decoding Png: unknown filter method");
        off += ph * (rb + 1);
        for (size_t y = 0; y < ph; ++y) {
            const uint8_t* r = rows.data() + y * rb;
            const size_t oy = passes[p].y0 + y * passes[p].dy;
            for (size_t x = 0; x < pw; ++x) {
                const size_t ox = passes[p].x0 + x * passes[p].dx;
                uint8_t* o = samp.data() + (oy * w + ox) * spp;
                if (depth == 8) {
                    std::memcpy(o, r + x * spp, spp);
                } else {  // 1/2/4-bit single sample, MSB first
                    const size_t bit = x * depth;
                    const int v = (r[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
                    o[0] = (uint8_t)v;  // raw index / raw gray level, expanded below
                }
            }
        }
    }
    // EXPAND: palette -> RGB(A), low-bit gray -> 8-bit, tRNS -> alpha
    if (ctype == 3) {
        const size_t npal = plte.size() / 3;
        const bool alpha = !trns.empty();
        C = alpha ? 4 : 3;
        px.resize((size_t)w * h * C);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const size_t idx = samp[i];
            uint8_t* o = px.data() + i * C;
            if (idx < npal) { o[0] = plte[3 * idx]; o[1] = plte[3 * idx + 1]; o[2] = plte[3 * idx + 2]; }
            else { o[0] = o[1] = o[2] = 0; }
            if (alpha) o[3] = idx < trns.size() ? trns[idx] : 255;
        }
    } else if (ctype == 0) {
        const int scale = depth == 1 ? 255 : depth == 2 ? 85 : depth == 4 ? 17 : 1;
        const bool alpha = trns.size() >= 2;
        const int key = alpha ? (int)((trns[0] << 8) | trns[1]) : -1;
        C = alpha ? 2 : 1;
        px.resize((size_t)w * h * C);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const int v = samp[i];
            px[i * C] = (uint8_t)(v * scale);
            if (alpha) px[i * C + 1] = v == key ? 0 : 255;
        }
    } else if (ctype == 2 && trns.size() >= 6) {
        const int kr = (trns[0] << 8) | trns[1], kg = (trns[2] << 8) | trns[3], kb = (trns[4] << 8) | trns[5];
        C = 4;
        px.resize((size_t)w * h * 4);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const uint8_t* s = samp.data() + i * 3;
            uint8_t* o = px.data() + i * 4;
            o[0] = s[0]; o[1] = s[1]; o[2] = s[2];
            o[3] = (s[0] == kr && s[1] == kg && s[2] == kb) ? 0 : 255;
        }
    } else {
        C = (uint32_t)spp;
        px.swap(samp);
    }
    W = w;
    H = h;
    return IK_OK;
}

// ---- WebP via libwebp -------------------------------------------------------
namespace {
struct WebPDec {
    void* lib = nullptr;
    int (*features)(const uint8_t*, size_t, void*, int) = nullptr;
    uint8_t* (*rgb)(const uint8_t*, size_t, int*, int*) = nullptr;
    uint8_t* (*rgba)(const uint8_t*, size_t, int*, int*) = nullptr;
    void (*wfree)(void*) = nullptr;
};
const WebPDec& webp_dec() {
    static WebPDec d;
    static std::once_flag once;
    std::call_once(once, [] {
        d.lib = dlopen("libwebp.so.7", RTLD_NOW | RTLD_LOCAL);
        if (!d.lib) return;
        d.features = (int (*)(const uint8_t*, size_t, void*, int))dlsym(d.lib, "WebPGetFeaturesInternal");
        d.rgb = (uint8_t * (*)(const uint8_t*, size_t, int*, int*)) dlsym(d.lib, "WebPDecodeRGB");
        d.rgba = (uint8_t * (*)(const uint8_t*, size_t, int*, int*)) dlsym(d.lib, "WebPDecodeRGBA");
        d.wfree = (void (*)(void*))dlsym(d.lib, "WebPFree");
    });
    return d;
}
}  // namespace

int decode_webp(const uint8_t* b, size_t n, uint32_t& W, uint32_t& H, uint32_t& C, std::vector<uint8_t>& px) {
    const WebPDec& d = webp_dec();
    if (!d.features || !d.rgb || !d.rgba || !d.wfree) return fail(IK_ERR_TRANSFORM, "WebP decoder unavailable");
    int feat[16] = {0};  // WebPBitstreamFeatures: width, height, has_alpha, has_animation, format, pad[5]
    if (d.features(b, n, feat, 0x0209) != 0) return fail(IK_ERR_TRANSFORM, "Format error decoding WebP");
    if (feat[3]) return fail(IK_ERR_TRANSFORM, "animated WebP is not supported by decode_image");
    int w = 0, h = 0;
    const bool alpha = feat[2] != 0;
    uint8_t* p = alpha ? d.rgba(b, n, &w, &h) : d.rgb(b, n, &w, &h);
    if (!p) return fail(IK_ERR_TRANSFORM, "Format error decoding WebP: corrupt bitstream");
    C = alpha ? 4 : 3;
    px.assign(p, p + (size_t)w * h * C);
    d.wfree(p);
    W = (uint32_t)w;
    H = (uint32_t)h;
    return IK_OK;
}

}  // namespace ik
