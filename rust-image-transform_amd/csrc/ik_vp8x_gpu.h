// ik_vp8x_gpu.h -- launchers of the exact WebP coder's device half (ik_vp8x.hip); the
// host driver and bitstream writer are ik_vp8x_host.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "ik_vp8x.h"
#include "ik_vp8_gpu.h"
#include "../../include/imagekit_hip.h"

namespace ik {
namespace vp8x {

// What a macroblock hands to the MBs that predict from it (its right and bottom
// neighbours) and to the statistics fold: the edges of its reconstruction, its
// outgoing non-zero contexts, chroma DC errors and edge sub-block modes.  One
// 128-byte line per MB, written once per call with write-through stores.
struct alignas(16) XEdge {
    uint8_t ybot[16], yright[16];           // luma bottom row, right column
    uint8_t ubot[8], vbot[8], uright[8], vright[8];
    uint32_t nz;                            // RecordTokens' contexts after the MB (BytesToNz + bit 25 = left DC)
    int8_t derr[8];                         // chroma DC errors: [0..3] down (top pair per channel), [4..7] right
    uint8_t bmr[4], bmb[4];                 // sub-block modes: right column (4k+3), bottom row (12+k)
    uint8_t pad[44];
};
static_assert(sizeof(XEdge) == 128, "one line per MB");

struct XArgs {
    const uint8_t* yuv;  // per image: Y (w*h), U, V ((w+1)/2 * (h+1)/2)
    size_t yuv_stride;
    int w, h, mb_w, mb_h;
    XMB* mbs;            // per image mb_w*mb_h records
    XEdge* edges;        // per image mb_w*mb_h edge records
    uint8_t* seg;        // per image per MB: segment (written by the set-up kernel)
    XSeg* segs;          // per image 4
    uint16_t* lc;        // per image: level costs [96][68]
    uint8_t* pr;         // per image: coefficient probabilities [1056]
    uint32_t* stats;     // per image: token statistics [1056]
    int* max_edge;       // per image 4
    int use_derr;
};

// One call's schedule and hand-off words.  Tasks are taken in ticket order; a
// task's dependencies always hold smaller tickets (epoch, then diagonal, then
// image; an epoch's statistics fold after its MBs), so the lowest unfinished
// ticket can always run and the grid drains whatever the residency.
struct XRun {
    const uint64_t* tasks;  // ticket -> [63] fold, [48..55] epoch, [32..47] image, [0..31] MB / -
    uint32_t ntasks, nep;
    const int* bounds;      // nep + 1 raster bounds of the epochs
    uint32_t* sync;         // zeroed per call: [0] ticket, [1] error, then done / cnt / ready
    uint32_t* done;         // per image per MB: decided
    uint32_t* cnt;          // per image per epoch: MBs decided
    uint32_t* ready;        // per image per epoch: the epoch's level costs are in place
};

hipError_t launch_vp8x_setup(const XArgs& a, const vp8::SegRecord* rec, const uint8_t* kseg, const int* qtab,
                             ik_vp8_segment_header* hdr, int n, hipStream_t s);
hipError_t launch_vp8x_run(const XArgs& a, const XRun& r, int grid, hipStream_t s);

}  // namespace vp8x
}  // namespace ik
