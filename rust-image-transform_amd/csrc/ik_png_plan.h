// ik_png_plan.h -- host-side bookkeeping of the parallel inflate (ik_inflate.h):
// decoder lanes from chunk candidates, and the chain check that verifies them.
// Shared by the GPU PNG decoder (ik_png_decode.cpp) and its CPU model
// (ik_png_model.cpp, CPU tests only).
#pragma once
#include <cstdint>
#include <vector>

#include "ik_inflate.h"

namespace ik {
namespace pngplan {

// One image's decoder lanes: lane i decodes blocks from start[i] up to stop[i]
// (the next lane's start, ~0 for the last lane).
struct Lanes {
    std::vector<uint64_t> start, stop;
    std::vector<infl::LaneResult> res;
    std::vector<char> dirty;  // needs (re)decoding in the next decode round
    std::vector<uint64_t> tbase;  // token region (the caller's allocation)
    std::vector<uint32_t> tcap;   // its capacity (0: none yet)
    std::vector<char> big;        // overflowed once: the region is sized by the exact bound
    std::vector<int64_t> pslot;   // wave decoder: the lane's piece table (first entry; -1: none yet)
    std::vector<uint32_t> pcap;   // and its entries
    int rounds = 0;
    // a new dirty lane [b, stop[i]) after lane i, which now stops at b
    void split(size_t i, uint64_t b) {
        const size_t k = i + 1;
        start.insert(start.begin() + (long)k, b);
        stop.insert(stop.begin() + (long)k, stop[i]);
        stop[i] = b;
        res.insert(res.begin() + (long)k, infl::LaneResult{0, 0, 0, infl::kLaneCorrupt, 0, 0, 0, 0, 0, 0, 0});
        dirty.insert(dirty.begin() + (long)k, 1);
        tbase.insert(tbase.begin() + (long)k, 0);
        tcap.insert(tcap.begin() + (long)k, 0);
        big.insert(big.begin() + (long)k, 0);
        pslot.insert(pslot.begin() + (long)k, -1);
        pcap.insert(pcap.begin() + (long)k, 0);
    }
    void erase(size_t i) {
        start.erase(start.begin() + (long)i);
        stop.erase(stop.begin() + (long)i);
        res.erase(res.begin() + (long)i);
        dirty.erase(dirty.begin() + (long)i);
        tbase.erase(tbase.begin() + (long)i);
        tcap.erase(tcap.begin() + (long)i);
        big.erase(big.begin() + (long)i);
        pslot.erase(pslot.begin() + (long)i);
        pcap.erase(pcap.begin() + (long)i);
    }
};

// candidates per chunk (chunk 0 = the first block, always valid; -1 = none found)
inline void build(const std::vector<int64_t>& cand, Lanes& L) {
    L.start.clear();
    L.stop.clear();
    for (int64_t c : cand)
        if (c >= 0 && (L.start.empty() || (uint64_t)c > L.start.back())) L.start.push_back((uint64_t)c);
    L.stop.resize(L.start.size());
    for (size_t i = 0; i < L.start.size(); ++i) L.stop[i] = i + 1 < L.start.size() ? L.start[i + 1] : ~0ull;
    L.res.assign(L.start.size(), infl::LaneResult{0, 0, 0, infl::kLaneCorrupt, 0, 0, 0, 0, 0, 0, 0});
    L.dirty.assign(L.start.size(), 1);
    L.tbase.assign(L.start.size(), 0);
    L.tcap.assign(L.start.size(), 0);
    L.big.assign(L.start.size(), 0);
    L.pslot.assign(L.start.size(), -1);
    L.pcap.assign(L.start.size(), 0);
    L.rounds = 0;
}

// After a decode round: walk the chain from lane 0 (whose start is the stream's
// first block, so verified).  A lane whose start is verified and that stopped
// exactly on its successor's start verifies that start.  One that passed it
// (mismatch) shows the successor's candidate was not a block boundary: the
// successor is dropped and the lane decodes on to the next one next round.  A
// lane that split (kLaneSplit: whole blocks up to end_bit) gets a new lane from
// end_bit to its old stop.
// Returns 0 when every lane is verified (the output offsets are then valid),
// 1 when dirty lanes must be decoded again, -1 when a verified lane found the
// stream corrupt (or the rounds ran out).  A lane that overflowed its token
// region (kLaneOverflow) is decoded again; the caller gives it the large region.
inline int check(Lanes& L, int max_rounds = 24) {
    ++L.rounds;
    bool verified = true;  // lane i's start is verified by this round's results
    bool any_dirty = false;
    for (size_t i = 0; i < L.start.size();) {
        if (L.dirty[i]) {  // not decoded yet in this state: its successors wait
            verified = false;
            any_dirty = true;
            ++i;
            continue;
        }
        const infl::LaneResult& r = L.res[i];
        if (r.status == infl::kLaneOverflow) {  // token region too small: again, larger (the caller sizes it)
            L.dirty[i] = 1;
            verified = false;
            any_dirty = true;
            ++i;
            continue;
        }
        if (r.status == infl::kLaneSplit) {  // (wave decoder) whole blocks up to end_bit: a new lane from there
            if (r.end_bit <= L.start[i] || r.end_bit >= L.stop[i]) {
                if (verified) return -1;
                ++i;
                continue;
            }
            L.split(i, r.end_bit);
            L.res[i].status = infl::kLaneOk;
            any_dirty = true;
            verified = false;  // the new lane is not decoded yet: its successors wait
            i += 2;
            continue;
        }
        if (r.status == infl::kLaneOk) {
            ++i;
            continue;  // successor verified iff this one was
        }
        if (r.status == infl::kLaneCorrupt) {
            if (verified) return -1;
            ++i;  // its start may be false: the predecessor decides next round
            continue;
        }
        // mismatch: drop the successor, decode on to the one after it
        if (i + 1 >= L.start.size()) {  // cannot happen (the last lane has stop ~0); treat as corrupt
            if (verified) return -1;
            ++i;
            continue;
        }
        L.erase(i + 1);
        L.stop[i] = i + 1 < L.start.size() ? L.start[i + 1] : ~0ull;
        L.dirty[i] = 1;
        any_dirty = true;
        verified = false;
        ++i;
    }
    if (!any_dirty) return 0;
    return L.rounds >= max_rounds ? -1 : 1;
}

// output offsets of verified lanes (exclusive prefix sum); total in *total
inline void offsets(const Lanes& L, std::vector<int64_t>& obase, uint64_t* total) {
    obase.resize(L.start.size());
    uint64_t t = 0;
    for (size_t i = 0; i < L.start.size(); ++i) {
        obase[i] = (int64_t)t;
        t += L.res[i].out_len;
    }
    *total = t;
}

}  // namespace pngplan
}  // namespace ik
