/*
 * png_dec.c -- ORACLE PNG decoder (TEST INFRASTRUCTURE ONLY: tests/ and bench.py's
 * cpu_baseline leg; the product never links or loads it).
 *
 * Restates what decode_image does on a PNG (reference src/transform.rs:31 ->
 * image 0.25.8 load_from_memory_with_format -> png 0.18.0, Cargo.lock:1594,
 * with image's Transformations::EXPAND) for the non-interlaced 8-bit colour
 * types 0/2/4/6 (the synthetic configs[1] frames are RGBA8):
 *   - chunk walk with CRC-32 verification (png checks CRCs by default),
 *   - IDAT concatenation + zlib inflate (libdeflate when present, else zlib;
 *     png 0.18 itself inflates with fdeflate -- a different inflater, same bytes),
 *   - per-row unfiltering: None, Sub, Up, Average, Paeth (PNG spec 9.2-9.4).
 * Single-threaded, one image per call, as the reference decodes (no rayon).
 * Returns the pixel bytes in *out (malloc'd, iko_free) and w/h/channels, or a
 * negative code for anything outside that subset or malformed.
 */
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "ik_oracle.h"

static uint32_t be32(const uint8_t *p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

typedef int (*ldz_fn)(void *, const void *, size_t, void *, size_t, size_t *);
static void *ld_lib;
static void *(*ld_alloc)(void);
static ldz_fn ld_zlib;
static void (*ld_free)(void *);
static uint32_t (*ld_crc)(uint32_t, const void *, size_t);

static void ld_init(void) {
    static int done;
    if (done) return;
    ld_lib = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (ld_lib) {
        ld_alloc = (void *(*)(void))dlsym(ld_lib, "libdeflate_alloc_decompressor");
        ld_zlib = (ldz_fn)dlsym(ld_lib, "libdeflate_zlib_decompress");
        ld_free = (void (*)(void *))dlsym(ld_lib, "libdeflate_free_decompressor");
        ld_crc = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(ld_lib, "libdeflate_crc32");
    }
    done = 1;
}

static uint32_t crc_of(const uint8_t *type, const uint8_t *data, size_t len) {
    if (ld_crc) return ld_crc(ld_crc(0, type, 4), data, len);
    return (uint32_t)crc32(crc32(0, type, 4), data, (uInt)len);
}

static int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

long iko_png_decode(const uint8_t *b, size_t n, uint8_t **out, uint32_t *ow, uint32_t *oh, uint32_t *oc) {
    static __thread int inited;
    if (!inited) { ld_init(); inited = 1; }
    if (n < 8 || memcmp(b, "\x89PNG\r\n\x1a\n", 8)) return -1;
    size_t pos = 8, zlen = 0, zcap = 0;
    uint8_t *z = NULL;
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0, ihdr = 0;
    while (pos + 12 <= n) {
        const uint32_t len = be32(b + pos);
        if (len > n - pos - 12) { free(z); return -2; }
        const uint8_t *type = b + pos + 4, *data = b + pos + 8;
        if (crc_of(type, data, len) != be32(data + len)) { free(z); return -3; }
        if (!memcmp(type, "IHDR", 4) && len == 13) {
            w = be32(data); h = be32(data + 4); depth = data[8]; ctype = data[9]; interlace = data[12];
            ihdr = 1;
        } else if (!memcmp(type, "IDAT", 4)) {
            if (zlen + len > zcap) {
                zcap = (zlen + len) * 2;
                uint8_t *nz = realloc(z, zcap);
                if (!nz) { free(z); return -4; }
                z = nz;
            }
            memcpy(z + zlen, data, len);
            zlen += len;
        } else if (!memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    int c = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!ihdr || !z || depth != 8 || interlace || !c || !w || !h) { free(z); return -5; }
    const size_t rb = (size_t)w * c, raw_n = (rb + 1) * h;
    uint8_t *raw = malloc(raw_n), *px = malloc(rb * h);
    if (!raw || !px) { free(z); free(raw); free(px); return -4; }
    size_t got = 0;
    int ok = 0;
    if (ld_alloc && ld_zlib) {
        static __thread void *dec;
        if (!dec) dec = ld_alloc();
        ok = dec && ld_zlib(dec, z, zlen, raw, raw_n, &got) == 0 && got == raw_n;
    }
    if (!ok) {
        uLongf dl = (uLongf)raw_n;
        ok = uncompress(raw, &dl, z, (uLong)zlen) == Z_OK && dl == raw_n;
    }
    free(z);
    if (!ok) { free(raw); free(px); return -6; }
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t ft = raw[y * (rb + 1)];
        const uint8_t *in = raw + y * (rb + 1) + 1;
        uint8_t *cur = px + y * rb;
        const uint8_t *prev = y ? px + (y - 1) * rb : NULL;
        for (size_t i = 0; i < rb; ++i) {
            const int a = i >= (size_t)c ? cur[i - c] : 0;
            const int bb = prev ? prev[i] : 0;
            const int cc = (prev && i >= (size_t)c) ? prev[i - c] : 0;
            int p;
            switch (ft) {
            case 0: p = 0; break;
            case 1: p = a; break;
            case 2: p = bb; break;
            case 3: p = (a + bb) >> 1; break;
            case 4: p = paeth(a, bb, cc); break;
            default: free(raw); free(px); return -7;
            }
            cur[i] = (uint8_t)(in[i] + p);
        }
    }
    free(raw);
    *out = px;
    *ow = w;
    *oh = h;
    *oc = (uint32_t)c;
    return (long)(rb * h);
}
