// tests/tsan/edgpu_cpu_stub.cpp -- TEST INFRASTRUCTURE ONLY: a host-memory stand-in for the
// engine's C ABI (include/edgpu.h), just enough of it for the QTSS module and its adapter to run
// their threads -- the pushers' striped appends, the stager's edgpu_ingest_prestage, the tick
// thread, the gather thread, the write threads and the UDP reader -- under ThreadSanitizer on a
// machine without a GPU (tests/test_tsan.py).  It relays with simple rules (a subscriber gets
// every packet of its sender pushed after it joined, no key frames, no SSRC filter): the race
// check needs the calls and their threads, not the reference's bytes, which the GPU tests pin.
// "Device" memory is host memory here.  The stub does NOT lock the context: the engine's calls
// are externally serialised (include/edgpu.h conventions), so every context call writes a plain
// field, and two calls the host did not order show up as a ThreadSanitizer race.  The calls the
// ABI allows from any thread -- edgpu_ingest_prestage, edgpu_host_alloc / edgpu_host_free -- take
// the staging lock instead, as the engine's do (pin_mu).  The pinned-batch contracts the DMA relies
// on are checked where TSan cannot see them (the copy runs after the call returns): prestaged bytes
// must not change before their ingest, and a pinned batch must not change or be freed before the
// next ingest call or an edgpu_sync has returned.
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "edgpu.h"

namespace {

thread_local std::string g_err;
int fail(int code, const char* m) { g_err = m; return code; }

struct Pkt { std::string data; int64_t arrival; uint32_t slot, epoch; };   // epoch: its host ingest (0: none)
struct Sub { uint32_t handle, session, track; uint8_t kind, transport; size_t cursor; bool active, fresh; };
struct Sess { uint32_t ntracks; bool alive; std::vector<std::vector<Pkt>> q; };   // per sender (2 x track)

}  // namespace

struct edgpu_ctx {
    uint32_t ingest_epoch = 0, host_epoch_last = 0;   // edgpu_fanout_packet_info's batch sources
    uint64_t calls = 0;                     // written by every context call (unlocked, on purpose)
    std::mutex stage_mu;                    // prestage + host buffers, from any thread
    std::vector<uint8_t> staged;            // a copy of the prefix the stager pushed ahead
    std::map<const void*, uint64_t> pinned; // live edgpu_host_alloc buffers
    const uint8_t* last_blob = nullptr;     // the previous pinned batch: must stay intact until the
    std::vector<uint8_t> last_bytes;        // next ingest call returns
    edgpu_config cfg;
    std::vector<Sess> sessions;
    std::vector<Sub> subs;                  // sub-stream rows
    uint32_t next_handle = 0;
    bool pending = false;
    // the last tick
    std::vector<uint8_t> arena;
    std::vector<edgpu_out_desc> desc;
    std::vector<int64_t> arrivals;
    std::vector<uint32_t> sources;
    std::vector<edgpu_substream_out> table;
    uint64_t relayed = 0, relayed_bytes = 0;
};

static void touch(edgpu_ctx* x) { x->calls++; }

extern "C" {

const char* edgpu_version(void) { return "edgpu cpu stub (TSan)"; }
const char* edgpu_last_error(void) { return g_err.c_str(); }
void edgpu_config_default(edgpu_config* c) { memset(c, 0, sizeof(*c)); }

int edgpu_ctx_create(const edgpu_config* cfg, edgpu_ctx** out) {
    if (!out) return EDGPU_BAD_ARGUMENT;
    *out = new edgpu_ctx();
    if (cfg) (*out)->cfg = *cfg;
    return EDGPU_OK;
}
int edgpu_ctx_destroy(edgpu_ctx* x) { delete x; return EDGPU_OK; }
// the context stream waits for every pinned copy before the ingest kernel: a sync ends them all
static void pinned_copies_done(edgpu_ctx* x) {
    std::lock_guard<std::mutex> g(x->stage_mu);
    x->last_blob = nullptr;
    x->last_bytes.clear();
}
int edgpu_sync(edgpu_ctx* x) { touch(x); pinned_copies_done(x); return EDGPU_OK; }

int edgpu_sdp_parse(const char* sdp, uint32_t len, edgpu_sdp_track* out, uint32_t cap, uint32_t* n) {
    const std::string s(sdp, len);
    uint32_t k = 0;
    for (size_t p = 0; p < s.size();) {
        size_t e = s.find_first_of("\r\n", p);
        if (e == std::string::npos) e = s.size();
        const std::string line = s.substr(p, e - p);
        if (!line.empty() && line[0] == 'm') {
            if (k < cap) { memset(&out[k], 0, sizeof(out[k])); out[k].track_id = k + 1; }
            k++;
        } else if (line.rfind("a=control:trackID=", 0) == 0 && k && k - 1 < cap) {
            out[k - 1].track_id = (uint32_t)atoi(line.c_str() + 18);
        }
        p = e + 1;
    }
    *n = k;
    return k > cap ? EDGPU_BAD_ARGUMENT : EDGPU_OK;
}

int edgpu_session_add(edgpu_ctx* x, const char* sdp, uint32_t len, int, uint32_t* out) {
    touch(x);
    edgpu_sdp_track t[64];
    uint32_t n = 0;
    if (edgpu_sdp_parse(sdp, len, t, 64, &n) || !n) return fail(EDGPU_BAD_ARGUMENT, "bad SDP");
    Sess s;
    s.ntracks = n;
    s.alive = true;
    s.q.resize(2 * n);
    x->sessions.push_back(s);
    *out = (uint32_t)x->sessions.size() - 1;
    return EDGPU_OK;
}
int edgpu_session_tracks(edgpu_ctx* x, uint32_t s, uint32_t* n) {
    touch(x);
    if (s >= x->sessions.size()) return EDGPU_BAD_ARGUMENT;
    *n = x->sessions[s].ntracks;
    return EDGPU_OK;
}
int edgpu_session_ssrc_prefs(edgpu_ctx* x, uint32_t s, uint32_t, uint32_t) {
    touch(x);
    return s < x->sessions.size() ? EDGPU_OK : EDGPU_BAD_ARGUMENT;
}
int edgpu_session_remove(edgpu_ctx* x, uint32_t s, uint32_t flags) {
    touch(x);
    if (s >= x->sessions.size() || !x->sessions[s].alive) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    for (const Sub& q : x->subs)
        if (q.active && q.session == s && !(flags & EDGPU_SESSION_KILL_OUTPUTS)) return fail(EDGPU_ERR, "outputs attached");
    for (Sub& q : x->subs) if (q.session == s) q.active = false;
    x->sessions[s].alive = false;
    return EDGPU_OK;
}
int edgpu_source_identity(edgpu_ctx*, uint32_t, uint32_t, uint32_t, int64_t) { return EDGPU_OK; }
int edgpu_udp_sources(edgpu_ctx*, const edgpu_udp_source*, uint32_t) { return EDGPU_OK; }
int edgpu_source_reports(edgpu_ctx*, edgpu_source_report*, uint32_t, uint32_t* n) { *n = 0; return EDGPU_OK; }

static int add_sub(edgpu_ctx* x, uint32_t s, int transport, uint32_t* out) {
    if (s >= x->sessions.size() || !x->sessions[s].alive) return fail(EDGPU_BAD_ARGUMENT, "bad session");
    const uint32_t h = x->next_handle++;
    for (uint32_t t = 0; t < x->sessions[s].ntracks; t++)
        for (uint8_t k = 0; k < 2; k++)
            x->subs.push_back(Sub{h, s, t, k, (uint8_t)transport, x->sessions[s].q[2 * t + k].size(), true, true});
    *out = h;
    return EDGPU_OK;
}
int edgpu_subscriber_add(edgpu_ctx* x, uint32_t s, int transport, uint32_t* out) {
    touch(x);
    return add_sub(x, s, transport, out);
}
int edgpu_subscriber_play(edgpu_ctx* x, uint32_t s, int transport, uint32_t, int64_t, uint32_t* out,
                          edgpu_rtp_info* info) {
    touch(x);
    if (info && s < x->sessions.size()) memset(info, 0, sizeof(*info) * x->sessions[s].ntracks);
    return add_sub(x, s, transport, out);
}
int edgpu_subscriber_remove(edgpu_ctx* x, uint32_t h) {
    touch(x);
    for (Sub& q : x->subs) if (q.handle == h) q.active = false;
    return EDGPU_OK;
}

int edgpu_host_alloc(edgpu_ctx* x, uint64_t bytes, void** out) {
    *out = aligned_alloc(64, (bytes + 63) / 64 * 64 + 64);
    if (!*out) return EDGPU_OUT_OF_MEMORY;
    std::lock_guard<std::mutex> g(x->stage_mu);
    x->pinned[*out] = bytes;
    return EDGPU_OK;
}
int edgpu_host_free(edgpu_ctx* x, void* p) {
    if (!p) return EDGPU_OK;
    {
        std::lock_guard<std::mutex> g(x->stage_mu);
        if (!x->pinned.erase(p)) return fail(EDGPU_BAD_ARGUMENT, "not an edgpu_host_alloc buffer");
        if (p == x->last_blob) x->last_blob = nullptr;    // checked at the next ingest: see below
    }
    free(p);
    return EDGPU_OK;
}

int edgpu_ingest_prestage(edgpu_ctx* x, const uint8_t* blob, uint64_t off, uint64_t bytes) {
    std::lock_guard<std::mutex> g(x->stage_mu);
    if (!bytes && !off) { x->staged.clear(); return EDGPU_OK; }
    if (off != x->staged.size()) return fail(EDGPU_BAD_ARGUMENT, "a prestaged range must extend the staged prefix");
    x->staged.insert(x->staged.end(), blob + off, blob + off + bytes);   // the DMA's read of the blob
    return EDGPU_OK;
}

int edgpu_ingest(edgpu_ctx* x, const edgpu_pkt_desc* d, uint32_t n, const uint32_t* seg, const uint32_t* sess,
                 uint32_t nseg, const uint8_t* blob, uint64_t blob_bytes, int where) {
    touch(x);
    {
        std::lock_guard<std::mutex> g(x->stage_mu);
        // the previous pinned batch's copy may still be reading it until this call returns
        if (!x->last_bytes.empty() && (!x->last_blob || memcmp(x->last_blob, x->last_bytes.data(), x->last_bytes.size())))
            return fail(EDGPU_ERR, "a pinned batch changed or was freed before the next ingest returned");
        x->last_blob = nullptr;
        x->last_bytes.clear();
        if (where == EDGPU_PTR_PINNED) {
            if (!x->staged.empty() && (blob_bytes < x->staged.size() || memcmp(blob, x->staged.data(), x->staged.size())))
                return fail(EDGPU_ERR, "prestaged bytes changed before their ingest");
            if (!x->pinned.count(blob)) return fail(EDGPU_BAD_ARGUMENT, "EDGPU_PTR_PINNED blob not from edgpu_host_alloc");
            x->last_blob = blob;
            x->last_bytes.assign(blob, blob + blob_bytes);
        }
        x->staged.clear();
    }
    if (x->pending) return fail(EDGPU_ERR, "keyframe index pending");
    const uint32_t epoch = where == EDGPU_PTR_DEVICE ? 0u : ++x->ingest_epoch;
    if (!epoch) ++x->ingest_epoch;
    x->host_epoch_last = epoch;
    for (uint32_t k = 0; k < nseg; k++) {
        if (sess[k] >= x->sessions.size() || !x->sessions[sess[k]].alive) continue;
        Sess& S = x->sessions[sess[k]];
        for (uint32_t i = seg[k]; i < seg[k + 1] && i < n; i++) {
            const uint32_t len = std::min<uint32_t>(d[i].len, 2060);
            const uint32_t snd = d[i].channel;
            if (snd >= S.q.size()) continue;
            S.q[snd].push_back(Pkt{std::string((const char*)blob + (size_t)d[i].slot * 16 + 4, len), d[i].arrival_ms, d[i].slot,
                                   epoch});
        }
    }
    x->pending = true;
    return EDGPU_OK;
}
int edgpu_keyframe_index(edgpu_ctx* x) { touch(x); x->pending = false; return EDGPU_OK; }

int edgpu_fanout(edgpu_ctx* x, int64_t, edgpu_fanout_result* out) {
    touch(x);
    x->arena.clear(); x->desc.clear(); x->arrivals.clear(); x->sources.clear(); x->table.clear();
    x->relayed = x->relayed_bytes = 0;
    for (Sub& q : x->subs) {
        edgpu_substream_out o;
        memset(&o, 0, sizeof(o));
        o.subscriber = q.handle; o.track = (uint16_t)q.track; o.kind = q.kind; o.transport = q.transport;
        o.sender = 2 * q.track + q.kind;            // sessions' senders as distinct ids
        o.sender += 64 * q.session;
        // (every sub-stream has its own bytes here; UDP ones are identity: each a suffix of its
        // sender's longest, as the engine's)
        o.flags = (q.fresh ? EDGPU_SUB_NEW : 0u) | (q.transport ? 0u : EDGPU_SUB_IDENTITY);
        q.fresh = false;
        o.desc_base = (uint32_t)x->desc.size();
        o.out_base = x->arena.size();
        if (q.active && x->sessions[q.session].alive) {
            const std::vector<Pkt>& pk = x->sessions[q.session].q[2 * q.track + q.kind];
            for (size_t i = q.cursor; i < pk.size(); i++) {
                const uint64_t slot = x->arena.size();
                const uint32_t len = (uint32_t)pk[i].data.size();
                x->arena.resize(slot + ((len + 4 + 15) & ~15u), 0);
                x->arena[slot] = '$';
                x->arena[slot + 1] = (uint8_t)(2 * q.track + q.kind);
                x->arena[slot + 2] = (uint8_t)(len >> 8);
                x->arena[slot + 3] = (uint8_t)len;
                memcpy(&x->arena[slot + 4], pk[i].data.data(), len);
                x->desc.push_back(edgpu_out_desc{slot + (q.transport ? 0 : 4), len + (q.transport ? 4u : 0u), (uint32_t)i + 1});
                x->arrivals.push_back(pk[i].arrival);
                x->sources.push_back(x->host_epoch_last && pk[i].epoch == x->host_epoch_last ? pk[i].slot : EDGPU_NO_SOURCE);
                x->relayed++;
                x->relayed_bytes += len;
            }
            q.cursor = pk.size();
        }
        o.desc_count = (uint32_t)x->desc.size() - o.desc_base;
        o.out_bytes = x->arena.size() - o.out_base;
        x->table.push_back(o);
    }
    x->arena.resize(x->arena.size() + 16);
    out->arena = x->arena.data();
    out->desc = x->desc.data();
    out->substreams = x->table.data();
    out->n_substreams = (uint32_t)x->table.size();
    return EDGPU_OK;
}
int edgpu_fanout_next(edgpu_ctx*, edgpu_fanout_result*, uint32_t* launched) { *launched = 0; return EDGPU_OK; }

int edgpu_tick_stats_get(edgpu_ctx* x, edgpu_tick_stats* s) {
    touch(x);
    pinned_copies_done(x);                  // (it syncs)
    memset(s, 0, sizeof(*s));
    s->relayed_packets = x->relayed;
    s->relayed_bytes = x->relayed_bytes;
    s->arena_bytes = x->arena.size();
    s->pass_arena_bytes = x->arena.size();
    s->pass_packets = (uint32_t)x->desc.size();
    return EDGPU_OK;
}
int edgpu_fanout_arrivals(edgpu_ctx* x, int64_t* out, uint32_t n, int) {
    touch(x);
    if (n < x->arrivals.size()) return EDGPU_OUT_OVERFLOW;
    if (!x->arrivals.empty()) memcpy(out, x->arrivals.data(), x->arrivals.size() * sizeof(int64_t));
    return EDGPU_OK;
}
int edgpu_fanout_packet_info(edgpu_ctx* x, int64_t* arrivals, uint32_t* sources, uint32_t n, int) {
    touch(x);
    if (n < x->arrivals.size()) return EDGPU_OUT_OVERFLOW;
    if (arrivals && !x->arrivals.empty()) memcpy(arrivals, x->arrivals.data(), x->arrivals.size() * sizeof(int64_t));
    if (sources && !x->sources.empty()) memcpy(sources, x->sources.data(), x->sources.size() * sizeof(uint32_t));
    return EDGPU_OK;
}
int edgpu_fanout_rows(edgpu_ctx* x, const uint32_t* sel, uint32_t nsel, edgpu_packet_row* rows, uint64_t nrows, int) {
    touch(x);
    for (uint32_t k = 0; k < nsel; k++) {
        if (sel[2 * k] >= x->table.size()) continue;
        const edgpu_substream_out& o = x->table[sel[2 * k]];
        for (uint32_t i = 0; i < o.desc_count && sel[2 * k + 1] + (uint64_t)i < nrows; i++) {
            const size_t d = (size_t)o.desc_base + i;
            rows[sel[2 * k + 1] + i] = edgpu_packet_row{x->desc[d].offset, x->desc[d].len, x->desc[d].packet_id,
                                                        d < x->arrivals.size() ? x->arrivals[d] : -1,
                                                        d < x->sources.size() ? x->sources[d] : EDGPU_NO_SOURCE, 0};
        }
    }
    return EDGPU_OK;
}
int edgpu_fanout_active(edgpu_ctx* x, edgpu_substream_out* rows, uint32_t* q, uint32_t cap, uint32_t* n_out, int) {
    touch(x);
    uint32_t n = 0;
    for (uint32_t i = 0; i < x->table.size(); i++) {
        const edgpu_substream_out& o = x->table[i];
        if (!o.desc_count && !(o.flags & EDGPU_SUB_NEW)) continue;
        if (n < cap) { rows[n] = o; q[n] = i; }
        n++;
    }
    *n_out = n;
    return EDGPU_OK;
}
int edgpu_fanout_blocked(edgpu_ctx* x, const edgpu_blocked* r, uint32_t n) {
    touch(x);
    for (uint32_t i = 0; i < n; i++) {
        if (r[i].substream >= x->table.size() || r[i].substream >= x->subs.size()) return EDGPU_BAD_ARGUMENT;
        const edgpu_substream_out& o = x->table[r[i].substream];
        if (r[i].sent < o.desc_count) x->subs[r[i].substream].cursor -= o.desc_count - r[i].sent;
    }
    return EDGPU_OK;
}
int edgpu_debug_stall(edgpu_ctx* x, uint32_t) { touch(x); return EDGPU_OK; }   // no device to stall
int edgpu_device_local_cpus(int, uint32_t*, uint32_t, uint32_t* n) {   // no GPU: no placement
    if (n) *n = 0;
    return EDGPU_ERR;
}
int edgpu_copy_to_host(edgpu_ctx* x, void* dst, const void* src, uint64_t bytes) {
    touch(x);
    if (bytes) memcpy(dst, src, bytes);
    return EDGPU_OK;
}
int edgpu_arena_gather(edgpu_ctx* x, const edgpu_fanout_result* r, const edgpu_region* reg, uint32_t n, void* dst,
                       uint64_t cap) {
    touch(x);              // the gather thread calls this during the writes
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (off + reg[i].bytes > cap) return EDGPU_OUT_OVERFLOW;
        memcpy((uint8_t*)dst + off, r->arena + reg[i].offset, reg[i].bytes);
        off += reg[i].bytes;
    }
    return EDGPU_OK;
}
int edgpu_gop_copy(edgpu_ctx*, uint32_t, uint32_t, uint8_t*, uint64_t, uint64_t* len, uint32_t* k) {
    *len = 0; *k = 0;
    return EDGPU_OK;
}

// the stand-in's rings are unbounded: no stream ever loses a packet
int edgpu_stream_errors(edgpu_ctx* x, uint32_t* sessions, int32_t* codes, uint32_t cap, uint32_t* n) {
    (void)sessions; (void)codes; (void)cap;
    if (!x || !n) return EDGPU_BAD_ARGUMENT;
    touch(x);
    *n = 0;
    return EDGPU_OK;
}

}  // extern "C"

