// tick_regions.h -- the distinct bytes of a fan-out tick (host side, shared by the socket egress
// and the module adapter).
//
// A tick's arena is write-many: every sub-stream has its own copy of the packets it relays.
// Sub-streams flagged EDGPU_SUB_IDENTITY (UDP, no rewrite) of one sender carry the same bytes,
// each a suffix of the longest (they all end at the sender's newest packet), so a host that
// reads the tick back needs that longest region once per sender plus every other non-empty
// sub-stream's region -- the copy edgpu_arena_gather packs on the device before one PCIe copy.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "edgpu.h"

namespace edgpu_host {

struct TickRegions {
    std::vector<edgpu_region> reg;                      // regions to gather, in order
    std::vector<std::pair<uint32_t, uint64_t>> src;     // per sub-stream: (region, byte offset in it)
    std::vector<uint64_t> reg_off;                      // region i starts at reg_off[i] of the gather
    uint64_t bytes = 0;                                 // total gathered bytes
    static constexpr uint32_t kNone = 0xFFFFFFFFu;

    // Host address of sub-stream q's first byte in the gathered copy at `base` (q non-empty).
    const uint8_t* at(const uint8_t* base, uint32_t q) const { return base + reg_off[src[q].first] + src[q].second; }
};

// Per sender (engine sender ids are dense): the representative of its identity sub-streams -- the
// longest by bytes -- whose bytes and packet rows serve every other one of them as a suffix.  Both
// the gather (tick_regions) and the adapter's row sharing pick it here, so they agree; `skip` as
// below.  Senders without an identity sub-stream map to TickRegions::kNone.
inline std::vector<uint32_t> identity_reps(const edgpu_substream_out* subs, uint32_t nq, const uint8_t* skip = nullptr) {
    uint32_t nsend = 0;
    for (uint32_t q = 0; q < nq; q++)
        if (subs[q].desc_count && (subs[q].flags & EDGPU_SUB_IDENTITY)) nsend = std::max(nsend, subs[q].sender + 1);
    std::vector<uint32_t> rep(nsend, 0xFFFFFFFFu);
    for (uint32_t q = 0; q < nq; q++) {
        const edgpu_substream_out& s = subs[q];
        if (!s.desc_count || !(s.flags & EDGPU_SUB_IDENTITY) || (skip && skip[q])) continue;
        uint32_t& r = rep[s.sender];
        if (r == 0xFFFFFFFFu || subs[r].out_bytes < s.out_bytes) r = q;
    }
    return rep;
}

// `skip` (optional, per sub-stream): it needs no region (the host has its bytes elsewhere: an
// identity sub-stream whose packets all came with the batch the host still holds); its src is kNone.
inline TickRegions tick_regions(const edgpu_substream_out* subs, uint32_t nq, const uint8_t* skip = nullptr) {
    TickRegions t;
    t.src.assign(nq, {TickRegions::kNone, 0});
    // per sender: its longest identity sub-stream, its region
    const std::vector<uint32_t> rep = identity_reps(subs, nq, skip);
    std::vector<uint32_t> rep_reg(rep.size(), TickRegions::kNone);
    t.reg.reserve(nq);
    for (uint32_t q = 0; q < nq; q++) {
        const edgpu_substream_out& s = subs[q];
        if (!s.desc_count || (skip && skip[q])) continue;
        if (s.flags & EDGPU_SUB_IDENTITY) {
            const edgpu_substream_out& R = subs[rep[s.sender]];
            uint32_t& g = rep_reg[s.sender];
            if (g == TickRegions::kNone) {
                g = (uint32_t)t.reg.size();
                t.reg.push_back(edgpu_region{R.out_base, R.out_bytes});
            }
            t.src[q] = {g, R.out_bytes - s.out_bytes};      // q is a suffix of the longest
        } else {
            t.src[q] = {(uint32_t)t.reg.size(), 0};
            t.reg.push_back(edgpu_region{s.out_base, s.out_bytes});
        }
    }
    t.reg_off.assign(t.reg.size() + 1, 0);
    for (size_t i = 0; i < t.reg.size(); i++) t.reg_off[i + 1] = t.reg_off[i] + t.reg[i].bytes;
    t.bytes = t.reg_off.back();
    return t;
}

// The readback of a tick in up to K parts of the sub-stream table (Reflector::ReflectPackets
// gathers part k + 1 while its writers deliver part k): sub-streams [q[k-1], q[k]) need regions
// [0, r[k+1]) -- a sub-stream only uses regions created at or before its own index, so each part
// adds the regions [r[k], r[k+1]).  Parts are cut at even fractions of the gathered bytes; with
// k == 1 (or too few bytes) there is one part.
struct TickParts {
    static constexpr uint32_t kMax = 8;
    uint32_t n = 1;
    uint32_t q[kMax] = {};                      // part k holds the sub-streams below q[k]
    uint32_t r[kMax + 1] = {};                  // part k gathers regions [r[k], r[k + 1])
};

inline TickParts tick_parts(const TickRegions& tr, uint32_t nq, uint32_t k) {
    TickParts p;
    k = std::max<uint32_t>(1, std::min<uint32_t>(k, TickParts::kMax));
    for (uint32_t i = 0; i < TickParts::kMax; i++) p.q[i] = nq;
    p.n = k;
    uint32_t cut = 0, rend = 0;
    for (uint32_t q = 0; q < nq && cut + 1 < k; q++) {
        if (tr.src[q].first != TickRegions::kNone) rend = std::max(rend, tr.src[q].first + 1);
        if (tr.reg_off[rend] * k >= tr.bytes * (cut + 1)) { p.q[cut] = q + 1; p.r[cut + 1] = rend; cut++; }
    }
    for (; cut < k; cut++) { p.q[cut] = nq; p.r[cut + 1] = (uint32_t)tr.reg.size(); }
    for (uint32_t i = 1; i <= k; i++) p.r[i] = std::max(p.r[i], p.r[i - 1]);
    return p;
}

}  // namespace edgpu_host
