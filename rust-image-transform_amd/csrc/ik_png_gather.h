// ik_png_gather.h -- the plan of the GPU PNG upload's gather pass (host side,
// no HIP): whole PNG files land byte for byte in a device "raw" area; every IDAT
// payload is cut into pieces of <= kPngGatherPiece bytes that k_png_gather copies
// into the contiguous zlib stream the decoder reads (followed by its zero
// padding) while computing each piece's CRC-32; k_png_crc_check joins a chunk's
// pieces after the CRC of its type and compares with the stored CRC.  Shared by
// ik_png_decode.cpp (the product) and ik_png_model.cpp (its CPU model, which
// executes the same plan on the host against zlib).
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace ik {

constexpr uint32_t kPngGatherPiece = 65536;  // bytes per piece (one 256-thread workgroup, 256 B per thread)
constexpr uint32_t kPngNoChunk = 0xFFFFFFFFu;
constexpr uint64_t kPngNoSrc = ~0ull;

struct PngGatherPiece {
    uint64_t src;    // byte offset in the raw area (kPngNoSrc: zero fill)
    uint64_t dst;    // byte offset in the stream area
    uint32_t len;    // <= kPngGatherPiece
    uint32_t chunk;  // chunk table index of the CRC it belongs to (kPngNoChunk: none)
};

struct PngCrcChunk {
    uint64_t crc_at;   // raw-area offset of the chunk's stored (big-endian) CRC
    uint32_t piece0;   // its pieces: piece0 .. piece0 + npieces - 1, in order
    uint32_t npieces;
    uint32_t stream;   // err[stream] = 1 on a mismatch
    uint32_t pad;
};

// One stream's share of the plan.  raw_off: where the file's first byte is in the
// raw address space the gather pass reads (an offset into the upload area, or the
// file's own device address when the caller's files are already in device
// memory); idat: its non-empty IDAT payloads in order (file offset, length);
// z_off: where its zlib stream starts in the stream area; tail: zero bytes to
// write after the stream's zlen payload bytes.
inline void png_gather_plan(uint64_t raw_off, const std::vector<std::pair<uint64_t, uint32_t>>& idat, uint64_t z_off,
                            uint32_t tail, uint32_t stream, std::vector<PngGatherPiece>& pieces,
                            std::vector<PngCrcChunk>& chunks) {
    uint64_t dst = z_off;
    for (const auto& seg : idat) {
        const uint64_t fo = seg.first;
        PngCrcChunk c{};
        c.crc_at = raw_off + fo + seg.second;
        c.piece0 = (uint32_t)pieces.size();
        c.stream = stream;
        for (uint32_t o = 0; o < seg.second; o += kPngGatherPiece) {
            const uint32_t n = seg.second - o < kPngGatherPiece ? seg.second - o : kPngGatherPiece;
            pieces.push_back(PngGatherPiece{raw_off + fo + o, dst, n, (uint32_t)chunks.size()});
            dst += n;
        }
        c.npieces = (uint32_t)pieces.size() - c.piece0;
        chunks.push_back(c);
    }
    for (uint32_t o = 0; o < tail; o += kPngGatherPiece) {
        const uint32_t n = tail - o < kPngGatherPiece ? tail - o : kPngGatherPiece;
        pieces.push_back(PngGatherPiece{kPngNoSrc, dst, n, kPngNoChunk});
        dst += n;
    }
}

}  // namespace ik
