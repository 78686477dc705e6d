// Host-side check of tick_regions.h (CPU test, tests/test_tick_regions.py): random fan-out
// sub-stream tables -> the distinct-bytes regions and the readback parts must satisfy
//   * every non-empty sub-stream reads its bytes inside one region: an identity UDP sub-stream
//     is a suffix of its sender's longest one, any other sub-stream is its own region;
//   * regions are packed back to back (reg_off), their bytes sum to `bytes`;
//   * the parts cover the regions [0, nreg) contiguously and the sub-streams [0, nq) in order,
//     and a sub-stream of part k only uses regions gathered by parts 0..k.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "tick_regions.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "check failed at line %d: %s\n", __LINE__, #c); return 1; } } while (0)

int main() {
    std::mt19937_64 rng(7);
    for (int trial = 0; trial < 400; trial++) {
        const uint32_t nsend = 1 + (uint32_t)(rng() % 40);
        std::vector<edgpu_substream_out> subs;
        uint64_t base = 0;
        std::vector<uint64_t> longest(nsend, 0);
        for (uint32_t s = 0; s < nsend; s++) longest[s] = 16 * (1 + rng() % 200);
        const uint32_t nq = (uint32_t)(rng() % 300);
        for (uint32_t q = 0; q < nq; q++) {
            edgpu_substream_out o{};
            o.sender = (uint32_t)(rng() % nsend);
            const bool identity = rng() % 4 != 0;
            o.flags = identity ? EDGPU_SUB_IDENTITY : 0u;
            o.desc_count = rng() % 5 == 0 ? 0u : 1u + (uint32_t)(rng() % 30);
            if (o.desc_count) {
                // identity sub-streams of a sender end at its newest packet: suffixes of the longest
                o.out_bytes = identity ? longest[o.sender] - 16 * (rng() % (longest[o.sender] / 16)) : 16 * (1 + rng() % 100);
                o.out_base = base;
                base += o.out_bytes;
            }
            subs.push_back(o);
        }
        const edgpu_host::TickRegions tr = edgpu_host::tick_regions(subs.data(), nq);
        uint64_t sum = 0;
        for (size_t i = 0; i < tr.reg.size(); i++) {
            CHECK(tr.reg_off[i] == sum);
            sum += tr.reg[i].bytes;
        }
        CHECK(sum == tr.bytes && tr.reg_off.back() == tr.bytes);
        for (uint32_t q = 0; q < nq; q++) {
            const edgpu_substream_out& o = subs[q];
            if (!o.desc_count) { CHECK(tr.src[q].first == edgpu_host::TickRegions::kNone); continue; }
            const uint32_t r = tr.src[q].first;
            CHECK(r < tr.reg.size());
            const edgpu_region& g = tr.reg[r];
            CHECK(tr.src[q].second + o.out_bytes == g.bytes);                 // a suffix (or the whole)
            if (o.flags & EDGPU_SUB_IDENTITY) {
                CHECK(g.offset + tr.src[q].second >= g.offset);
                CHECK(g.bytes >= o.out_bytes);
            } else {
                CHECK(g.offset == o.out_base && g.bytes == o.out_bytes && tr.src[q].second == 0);
            }
        }
        for (uint32_t k = 1; k <= edgpu_host::TickParts::kMax; k++) {
            const edgpu_host::TickParts p = edgpu_host::tick_parts(tr, nq, k);
            CHECK(p.n == k);
            CHECK(p.r[0] == 0 && p.r[p.n] == tr.reg.size() && p.q[p.n - 1] == nq);
            for (uint32_t i = 0; i < p.n; i++) {
                CHECK(p.r[i] <= p.r[i + 1]);
                if (i) CHECK(p.q[i - 1] <= p.q[i]);
            }
            uint32_t part = 0;
            for (uint32_t q = 0; q < nq; q++) {
                while (part + 1 < p.n && q >= p.q[part]) part++;
                if (tr.src[q].first != edgpu_host::TickRegions::kNone) CHECK(tr.src[q].first < p.r[part + 1]);
            }
        }
    }
    printf("ok\n");
    return 0;
}
