// ik_png.h -- device-side descriptors and launchers of the GPU PNG decoder
// (kernels: ik_png.hip; host orchestration: ik_png_decode.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ik_inflate.h"
#include "ik_png_gather.h"

namespace ik {

constexpr int kPngInflateThreads = 64;     // decoder lanes per workgroup (one wave: LDS 320 B per lane)
constexpr int kPngExpandThreads = 64;      // expand lanes per workgroup (LDS: 256 B literal table each)
constexpr int kPngUnfilterThreads = 1024;  // 16 waves, one 64-row band each
constexpr int kPngUnfilterWaves = kPngUnfilterThreads / 64;
// workgroups per image for the unfilter pass: one per 16 bands of 64 rows, at
// most 32 (all of an image's workgroups must be resident together)
IK_HD int png_unfilter_groups(int h) {
    const int g = ((h + 63) / 64 + kPngUnfilterWaves - 1) / kPngUnfilterWaves;
    return g < 32 ? g : 32;
}
constexpr uint64_t kPngChunkBytes = 16384; // candidate-search chunk of the compressed stream
constexpr uint64_t kPngWaveChunkBytes = 65536; // the same, for the wave decoder (ik_png_decode.cpp png_chunk_bytes)
constexpr int kPngPageShift = 12;          // resolve: output page -> decoder table

// one image of a batch, as the kernels see it
struct PngImgDev {
    const uint32_t* words;   // zlib stream (little-endian words, zero padded)
    uint64_t bit0;           // first DEFLATE bit (after the 2-byte zlib header)
    uint64_t nbits;          // stream length in bits
    uint16_t* u16;           // expand pass output: raw_total symbols (+ padding)
    uint64_t raw_total;      // bytes of the filtered image (H rows of 1 + rowbytes)
    const int64_t* obase;    // output offset of each decoder lane (ascending)
    const int* page_lane;    // decoder holding the first byte of each output page
    int nlanes;
    int rowbytes, H, bpp;
    uint8_t* ft;             // filter type of every row
    uint8_t* dst;            // the image (pitched); filtered rows, then pixels in place
    size_t pitch;
    const int* flags;        // the image's resolve flags: 1 bad filter type, 2 bad marker, 4 Average/Paeth rows
};

struct PngLaneDev {
    uint64_t start, stop;    // decode: block boundary to start at; next lane's start (~0 = last)
    uint64_t tbase;          // token region: index into the batch's token area (a multiple of 8)
    int64_t obase;           // expand: output offset
    uint64_t out_len;        // expand: output bytes
    uint32_t ntok;           // decode: region capacity (tokens); expand: tokens to read
    uint32_t img;            // image of the batch
    uint32_t first;          // lane 0 of its image (no distance reaches before its output)
    uint32_t big;            // wave decoder: the region is sized by the exact bound (an overflow before)
    uint64_t pbase;          // wave decoder: its piece table, from entry pbase of the batch's
    uint32_t npieces;        // wave decoder: the table's entries; expand: pieces to read (0: one contiguous run)
    uint32_t ubase;          // expand (wave decoder): the lane's first unit in the batch
    uint32_t uimg;           // expand: its image's first unit in the batch
    uint32_t nunits;         // expand: the lane's units (LaneResult::units)
    uint32_t pad;
};

// Upload of whole PNG files (ik_png_decode.cpp png_upload_begin): each file lands
// byte for byte in a device "raw" area; k_png_gather then copies the IDAT payloads
// into the contiguous zlib stream the decoder reads (plus its zero padding) and
// computes every piece's CRC-32, and k_png_crc_check joins a chunk's pieces and
// compares the result with the chunk's stored CRC (png verifies every chunk).
// png's EXPAND of one image (k_png_px): its unfiltered rows (src, rowbytes wide)
// -> 8-bit pixels of out_c channels: palette indices through pal (RGBA), gray
// below 8 bits scaled to 8 bits, tRNS as alpha (key: gray level / RGB triple in
// the image's bit depth, -1 = none)
struct PngPxDev {
    const uint8_t* src;
    size_t sp;
    uint8_t* dst;
    size_t dp;
    int w, h, depth, ctype, out_c, scale, key;
    int key_rgb[3];
    uint32_t pal[256];  // r | g << 8 | b << 16 | a << 24
};
hipError_t launch_png_px(const PngPxDev& px, hipStream_t s);

// piece_crc[2 i] = finished CRC-32 of piece i's bytes, [2 i + 1] = its length.
// raw: the base address the pieces' src / the chunks' crc_at offsets are relative
// to (the upload area, or 0 when they are the caller's device addresses)
hipError_t launch_png_gather(uintptr_t raw, uint8_t* stream, const PngGatherPiece* pieces, int npieces,
                             uint32_t* piece_crc, hipStream_t s);
hipError_t launch_png_crc_check(uintptr_t raw, const PngCrcChunk* chunks, int nchunks, const uint32_t* piece_crc,
                                int* err, hipStream_t s);

// Chunk walk of PNG files already in device memory (the caller's request bodies
// in HBM): one wave per file follows the chunk lengths from byte 8, as png does,
// and records every chunk; the contents of the non-IDAT chunks (IHDR, PLTE, tRNS,
// ancillary: type + data + CRC) and the first bytes of each IDAT payload go to the
// file's side area, so the host can plan the stream from host memory alone.
struct PngWalkRec {
    uint64_t off;      // file offset of the chunk's length field
    uint32_t len;      // data length
    uint32_t side;     // offset of type + data + CRC in the file's side area (non-IDAT), ~0 if none
    uint8_t type[4];
    uint8_t head[4];   // first data bytes (IDAT: the zlib header lives in the first)
};
// out_n[f]: chunks recorded (>= 0), or -1 (record table full) / -2 (side area
// full): the host then copies the file back and decodes it there
constexpr int kPngWalkRecs = 4096;         // chunks recorded per file
constexpr uint32_t kPngWalkSide = 65536;   // side-area bytes per file
// out[64 f + t] = byte t of file f (0 past its end)
hipError_t launch_copy_heads(const uint64_t* files, const uint64_t* lens, int n, uint8_t* out, hipStream_t s);
hipError_t launch_png_walk(const uint64_t* files, const uint64_t* lens, int n, PngWalkRec* recs, uint8_t* side,
                           int* out_n, hipStream_t s);

// dst[i] = src[i] for n words, on the compute stream; one side may be pinned host
// memory (the small transfers of the PNG kernel phase: ik_png_decode.cpp Xfer)
hipError_t launch_copy_words(const uint32_t* src, uint32_t* dst, size_t n, hipStream_t s);
#ifdef IK_UNF_PROF
hipError_t png_unf_prof_read(unsigned long long* out);  // dev build: k_png_unfilter's segment clock sums (reset)
#endif
#ifdef IK_EXP_PROF
hipError_t png_exp_prof_read(unsigned long long* out);  // dev build: k_png_expand8's phase clock sums (reset)
#endif
#ifdef IK_WAVE_PROF
hipError_t png_wave_prof_read(unsigned long long* out);  // dev build: k_png_wave's phase clock sums (reset)
#endif
#ifdef IK_FIND_PROF
hipError_t png_find_prof_read(unsigned long long* out);  // dev build: k_png_find's phase clock sums (reset)
#endif
hipError_t launch_png_find(const PngImgDev* imgs, const int* chunk_img, const int* chunk_idx, int n,
                           uint64_t chunk_bits, int64_t* cand, hipStream_t s);
// order (nullable): launch slot -> lane index; lane t's result goes to res[t]
hipError_t launch_png_decode(const PngImgDev* imgs, const PngLaneDev* lanes, const uint32_t* order, int n,
                             uint16_t* tok, infl::LaneResult* res, hipStream_t s);
// The direct-rows expand (the wave decoder's default): expand writes the image's
// rows and filter types itself and lists the window markers (image << 40 | raw
// position) here; k_png_marks resolves them, k_png_ftflags checks the filter types.
// count > cap: the list overflowed -- the batch then takes k_png_resolve after all.
constexpr uint32_t kMarkLists = 256;  // sub-lists (unit % kMarkLists), cap / kMarkLists entries each
struct PngMarks {
    uint64_t* list = nullptr;  // nullptr: expand writes only the u16 symbols (k_png_resolve's input)
    uint32_t* count = nullptr; // kMarkLists counters
    uint32_t cap = 0;          // entries over all sub-lists
};
hipError_t launch_png_marks(const PngImgDev* imgs, PngMarks mk, const int2* rows, int nrows, int* err, hipStream_t s);
// expand: one wave per lane (units == nullptr; n lanes), or -- the wave decoder's
// lanes -- one wave per expand unit (n units; unit u of lane ulane[u], its record at
// units[lanes[l].pbase + u - lanes[l].ubase]); status: 2 ints per lane / unit
hipError_t launch_png_expand(const PngImgDev* imgs, const PngLaneDev* lanes, int n, const uint16_t* tok, int* status,
                             hipStream_t s, const uint2* pieces = nullptr, const uint2* units = nullptr,
                             const uint32_t* ulane = nullptr, PngMarks mk = PngMarks());
// the wave decoder (ik_png_wave.h): one wave per lane; pieces: (token base in the
// lane's region, first index in its virtual token stream) per piece, a table of
// lanes[t].npieces entries at lanes[t].pbase; units: the lane's expand-unit
// records (first piece, output bytes before it) at the same slots
hipError_t launch_png_wave(const PngImgDev* imgs, const PngLaneDev* lanes, const uint32_t* order, int n,
                           uint16_t* tok, uint2* pieces, uint2* units, infl::LaneResult* res, hipStream_t s);
// the expand units' tables from the verified lanes (n lanes, each with obase,
// out_len, pbase, ubase, uimg, nunits set): every unit's output offset into its
// image's obase table (imgs[].obase, as resolve reads it), its lane into ulane, and
// the image's page table (imgs[].page_lane: page -> the unit holding its first byte)
hipError_t launch_png_units(const PngImgDev* imgs, const PngLaneDev* lanes, int n, const uint2* units,
                            uint32_t* ulane, hipStream_t s);
hipError_t launch_png_resolve(const PngImgDev* imgs, const int2* rows, int nrows, int* err, hipStream_t s);
// groups[t] = (image, band group) of the workgroup holding ticket t; prog: one
// zeroed counter per band (the image's at prog_base[image]); ticket: zeroed
// The unfilter's scan path (k_png_unfilter_su): an RGBA8 image without Average /
// Paeth rows (flags bit 4 clear) and at most kSuThreads * 4 chunks of 16 bytes a row
// (4,096 pixels) is unfiltered by segments -- a None / Sub row and the Up rows under
// it -- instead of the diagonal wavefront (the Up rows' only dependency is the row
// above, byte for byte; a Sub row's is a prefix sum along the row).  k_png_unfilter
// skips those images.
constexpr int kSuThreads = 256, kSuChunks = 4, kSuChunksWide = 8, kSuRanges = 16;
IK_HD bool png_unfilter_scan_path(int bpp, int rowbytes, int flags) {
    return bpp == 4 && (rowbytes + 15) / 16 <= kSuThreads * kSuChunksWide && !(flags & 7);
}
// nimg images of one class (bpp 4): kSuRanges workgroups each
hipError_t launch_png_unfilter_su(const PngImgDev* imgs, int nimg, hipStream_t s);
hipError_t launch_png_unfilter(const PngImgDev* imgs, const int2* groups, int ngroups, const int* prog_base,
                               unsigned* prog, unsigned* ticket, int bpp, hipStream_t s);

}  // namespace ik
