// tools/adapter_replay.cpp -- drives the C++ module-side adapter (reflector_adapter.h) with an
// event trace, the way the reflector module would: PKT -> Reflector::PushPacket (track =
// channel/2, RTCP = channel&1, as ProcessRTPData does, QTSSReflectorModule.cpp:654-671),
// JOIN -> AddOutput, TICK -> ReflectPackets(now, sink), BLOCK -> the sink returns kWouldBlock
// after the scripted number of writes in the next tick, UPKT (UDP push) -> ProcessUDPPacket,
// LEAVE -> RemoveOutput; PUBLISH / UNPUBLISH (trace v3) -> the module's reference counting (the
// pusher's reference and one per output, QTSSReflectorModule.cpp:2133-2196): RemoveSession at 0
// (killOutputs for an UNPUBLISH with kill), SetupReflectorSession for a PUBLISH after that;
// PKT / UPKT of a session without a pusher are dropped, a JOIN of a removed session fails;
// receiver reports reach the sink's SendReceiverReport.  Writes the capture format of
// easydarwin_amd/trace.py so tests compare it with the reference harness byte for byte.
// Usage: adapter_replay <trace.edtr> <capture.edcp>
// EDGPU_ARENA_BYTES / EDGPU_MAX_OUT_PACKETS set the engine's fan-out capacities (a small arena
// splits ticks into copy passes); the copy passes are counted on stderr.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "reflector_adapter.h"
#include "trace_prefs.h"

using namespace edgpu_reflector;

struct Rec { uint32_t sub = 0, session = 0; bool tcp = false; std::string img[2]; uint64_t n[2] = {0, 0}; };

struct Report { int64_t t; uint32_t session; uint16_t track; uint32_t addr; uint16_t port; std::string bytes; };

class CaptureSink : public OutputSink {
public:
    std::vector<Report> reports;
    int64_t now = 0;
    void SendReceiverReport(uint32_t session, uint16_t track, uint32_t addr, uint16_t port, const uint8_t* rr,
                            uint32_t len) override {
        reports.push_back(Report{now, session, track, addr, port, std::string((const char*)rr, len)});
    }
    std::map<std::pair<uint32_t, uint16_t>, Rec>* recs;      // (handle, track)
    std::map<std::tuple<uint32_t, uint16_t, int>, int64_t> budget;   // BLOCK: writes left this tick
    // EDGPU_REPLAY_FAIL_PASS=1: the first write of a tick's second copy pass fails once (a sink
    // error), to check that the failed tick leaves the context usable (no owed pass)
    const Reflector* R = nullptr;
    bool failPass = false, failed = false;
    int WritePacket(uint32_t subscriber, uint16_t track, bool isRTCP, bool interleaved, const uint8_t* wire,
                    uint32_t wireLen, uint32_t) override {
        if (failPass && !failed && R && R->LastTick().passes >= 2) { failed = true; return kRequestFailed; }
        auto b = budget.find(std::make_tuple(subscriber, track, isRTCP ? 1 : 0));
        if (b != budget.end()) {
            if (b->second == 0) return kWouldBlock;
            b->second--;
        }
        Rec& r = (*recs)[{subscriber, track}];
        std::string& s = r.img[isRTCP ? 1 : 0];
        if (!interleaved) { s.push_back((char)(wireLen >> 8)); s.push_back((char)wireLen); }
        s.append((const char*)wire, wireLen);
        r.n[isRTCP ? 1 : 0]++;
        return kNoErr;
    }
};

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s trace capture\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    std::vector<uint8_t> d;
    fseek(f, 0, SEEK_END); d.resize(ftell(f)); fseek(f, 0, SEEK_SET);
    if (fread(d.data(), 1, d.size(), f) != d.size()) return 2;
    fclose(f);
    size_t p = 4;
    auto get = [&](auto& v) { memcpy(&v, &d[p], sizeof(v)); p += sizeof(v); };
    uint32_t ver, nsess;
    get(ver); get(nsess);
    std::vector<std::string> sdps(nsess);
    std::vector<uint8_t> udp(nsess, 0);
    for (uint32_t s = 0; s < nsess; s++) {
        uint32_t n; get(n);
        sdps[s].assign((const char*)&d[p], n);
        p += n;
        if (ver >= 2) get(udp[s]);
    }
    // the server's prefs (trace v4): the stream prefs configure the engine, the module prefs
    // are kept as the module keeps them (PREFS events: RereadPrefs)
    trace_prefs::Prefs prefs;
    if (ver >= 4) {
        uint32_t n; get(n);
        prefs = trace_prefs::Prefs::parse(&d[p], n);
        p += n;
    }
    edgpu_config cfg;
    edgpu_config_default(&cfg);
    cfg.reflector_buffer_size_sec = prefs.u32("reflector_buffer_size_sec");
    cfg.rtp_reflector_threshold_msec = std::max<uint32_t>(1000, prefs.u32("rtp_reflector_threshold_msec"));   // :101-102
    cfg.reflector_rtp_info_offset_msec = prefs.u32("reflector_rtp_info_offset_msec") ? prefs.u32("reflector_rtp_info_offset_msec")
                                                                                     : EDGPU_FALSE;
    cfg.reflector_use_in_packet_receive_time = prefs.flag("reflector_use_in_packet_receive_time") ? 1u : 0u;
    cfg.reflector_in_packet_max_receive_sec = prefs.u32("reflector_in_packet_max_receive_sec") ? prefs.u32("reflector_in_packet_max_receive_sec")
                                                                                               : EDGPU_FALSE;
    if (const char* v = getenv("EDGPU_ARENA_BYTES")) cfg.out_arena_bytes = strtoull(v, nullptr, 0);
    if (const char* v = getenv("EDGPU_INGEST_SPEC_MIN")) cfg.ingest_spec_min = (uint32_t)strtoul(v, nullptr, 0);
    if (const char* v = getenv("EDGPU_MAX_OUT_PACKETS")) cfg.max_out_packets = (uint32_t)strtoul(v, nullptr, 0);
    Reflector R(&cfg);
    uint64_t ticks = 0, passes = 0, stream_errors = 0;
    if (R.Status()) { fprintf(stderr, "edgpu: %s\n", edgpu_last_error()); return 3; }
    uint32_t rand_calls = 0;                  // the harness's deterministic rand() (trace.py rr_ssrc)
    std::vector<int64_t> sid_of(nsess, -1);   // engine session of each trace session (-1: removed)
    std::vector<bool> killAttr(nsess, false); // the pusher's kill-clients attribute (its RECORD)
    std::vector<bool> published(nsess, true);
    std::map<uint32_t, uint32_t> trace_of;    // engine session -> trace session
    auto create = [&](uint32_t s, int64_t cnameSecs) -> bool {
        uint32_t sid;
        if (R.SetupReflectorSession(sdps[s], (udp[s] & 1) != 0, &sid)) return false;
        if (R.SetSSRCFilter(sid, prefs.flag("use_one_SSRC_per_stream"), prefs.u32("timeout_stream_SSRC_secs"))) return false;
        killAttr[s] = prefs.flag("kill_clients_when_broadcast_stops");
        for (uint32_t x = 0; x < R.GetNumStreams(sid); x++) {
            const uint32_t k = rand_calls++;
            if (R.SetSourceIdentity(sid, x, ((k + 1) * 0x9E3779B1u + 0x7F4A7C15u) & 0x7FFFFFFFu, cnameSecs)) return false;
        }
        sid_of[s] = sid;
        trace_of[sid] = s;
        return true;
    };
    for (uint32_t s = 0; s < nsess; s++)
        if (!create(s, 0)) return 3;
    std::map<std::pair<uint32_t, uint16_t>, Rec> recs;
    std::map<uint32_t, std::tuple<uint32_t, uint32_t, bool>> handles;   // handle -> (sub, trace session, tcp)
    std::map<uint32_t, bool> live;                                      // handle -> still an output
    CaptureSink sink;
    sink.recs = &recs;
    sink.R = &R;
    sink.failPass = getenv("EDGPU_REPLAY_FAIL_PASS") && atoi(getenv("EDGPU_REPLAY_FAIL_PASS")) != 0;
    uint64_t failedTicks = 0, ticksAfterFailure = 0;
    int64_t now = 0;
    // a session without pusher or outputs ends (RemoveOutput's refcount-0 branch)
    auto release_check = [&](uint32_t s) -> bool {
        if (sid_of[s] < 0 || published[s]) return true;
        for (auto& kv : live)
            if (kv.second && std::get<1>(handles[kv.first]) == s) return true;
        if (R.RemoveSession((uint32_t)sid_of[s], false)) return false;
        sid_of[s] = -1;
        return true;
    };
    while (p < d.size()) {
        uint8_t type; get(type);
        if (type == 0) break;
        int64_t t; get(t);
        if (t > now) now = t;                 // the reflector's clock (max event time so far)
        if (type == 1) {
            uint32_t s, len; uint8_t ch;
            get(s); get(ch); get(len);
            if (published[s]) R.PushPacket((uint32_t)sid_of[s], ch / 2, (const char*)&d[p], len, ch & 1, t);
            p += len;
        } else if (type == 2) {
            uint32_t s, sub; uint8_t tr, ua;
            get(s); get(sub); get(tr); get(ua);
            if (sid_of[s] < 0) continue;      // no such session: the player's SETUP fails
            const uint32_t sid = (uint32_t)sid_of[s];
            uint32_t h;
            if (prefs.rtp_info_player(ua)) {  // RTP-Info player: PLAY now, or deferred
                const int err = R.PlayRTPInfo(sid, tr != 0, now, &h, nullptr);
                if (err == kWouldBlock) continue;
                if (err) return 3;
            } else if (R.AddOutput(sid, tr != 0, &h)) {
                return 3;
            }
            handles[h] = std::make_tuple(sub, s, tr != 0);
            live[h] = true;
            for (uint16_t x = 0; x < R.GetNumStreams(sid); x++) recs[{h, x}];
        } else if (type == 5) {               // UPKT: a UDP pusher's datagram
            uint32_t s, addr, len; uint8_t ch; uint16_t port;
            get(s); get(ch); get(addr); get(port); get(len);
            if (published[s]) R.ProcessUDPPacket((uint32_t)sid_of[s], ch / 2, ch & 1, (const char*)&d[p], len, addr, port, t);
            p += len;
        } else if (type == 7) {               // UNPUBLISH: the pusher's session closes
            uint32_t s; uint8_t kill;
            get(s); get(kill);
            if (!published[s]) continue;
            published[s] = false;
            kill = kill || killAttr[s] || prefs.flag("kill_clients_when_broadcast_stops");   // :2156
            if (kill && sid_of[s] >= 0) {     // TearDownAllOutputs: the session ends with them
                for (auto& kv : live)
                    if (kv.second && std::get<1>(handles[kv.first]) == s) kv.second = false;
                if (R.RemoveSession((uint32_t)sid_of[s], true)) return 3;
                sid_of[s] = -1;
            }
            if (!release_check(s)) return 3;
        } else if (type == 8) {               // PUBLISH: the existing session, or a fresh one
            uint32_t s; get(s);
            if (published[s]) continue;
            published[s] = true;
            if (sid_of[s] < 0 && !create(s, now / 1000)) return 3;
            killAttr[s] = prefs.flag("kill_clients_when_broadcast_stops");
        } else if (type == 9) {               // PREFS: the server's prefs rewritten (RereadPrefs)
            uint32_t n; get(n);
            prefs = trace_prefs::Prefs::parse(&d[p], n);
            p += n;
        } else if (type == 3) {
            sink.now = t;
            const size_t before = sink.reports.size();
            int err = R.ReflectPackets(t, &sink);
            for (size_t i = before; i < sink.reports.size(); i++) sink.reports[i].session = trace_of[sink.reports[i].session];
            if (err && sink.failed && failedTicks == 0) {
                fprintf(stderr, "adapter_replay: injected sink failure at tick %llu (%d)\n", (unsigned long long)ticks, err);
                failedTicks++;
            } else if (err) {
                fprintf(stderr, "ReflectPackets: %d %s\n", err, edgpu_last_error());
                return 3;
            } else if (failedTicks) {
                ticksAfterFailure++;
            }
            ticks++;
            passes += R.LastTick().passes;
            stream_errors += R.LastTick().stream_errors;
            sink.budget.clear();
        } else if (type == 6) {               // LEAVE: ReflectorSession::RemoveOutput
            uint32_t sub; get(sub);
            for (auto& kv : handles)
                if (std::get<0>(kv.second) == sub && live[kv.first]) {
                    if (R.RemoveOutput(kv.first)) return 3;
                    live[kv.first] = false;
                    if (!release_check(std::get<1>(kv.second))) return 3;
                    break;
                }
        } else if (type == 4) {               // BLOCK: the sub-stream's socket takes `budget` writes
            uint32_t sub, budget; uint16_t trk; uint8_t kind;
            get(sub); get(trk); get(kind); get(budget);
            for (auto& kv : handles)
                if (std::get<0>(kv.second) == sub) sink.budget[std::make_tuple(kv.first, trk, (int)(kind & 1))] = budget;
        } else return 3;
    }
    std::vector<std::tuple<uint32_t, uint16_t, Rec*>> out;
    for (auto& kv : recs) {
        Rec& r = kv.second;
        auto h = handles[kv.first.first];
        r.sub = std::get<0>(h); r.session = std::get<1>(h); r.tcp = std::get<2>(h);
        out.emplace_back(r.sub, kv.first.second, &r);
    }
    std::stable_sort(out.begin(), out.end(), [](auto& a, auto& b) {
        return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b); });
    FILE* o = fopen(argv[2], "wb");
    fwrite("EDCP", 1, 4, o);
    uint32_t n = (uint32_t)out.size() * 2;
    fwrite(&n, 4, 1, o);
    for (auto& e : out)
        for (int k = 0; k < 2; k++) {
            Rec& r = *std::get<2>(e);
            uint16_t tr = std::get<1>(e);
            uint8_t kind = (uint8_t)k, tcp = r.tcp;
            uint64_t np = r.n[k], nb = r.img[k].size();
            fwrite(&r.sub, 4, 1, o); fwrite(&r.session, 4, 1, o); fwrite(&tr, 2, 1, o);
            fwrite(&kind, 1, 1, o); fwrite(&tcp, 1, 1, o); fwrite(&np, 8, 1, o); fwrite(&nb, 8, 1, o);
            fwrite(r.img[k].data(), 1, nb, o);
        }
    if (!sink.reports.empty()) {              // EDRR trailer
        fwrite("EDRR", 1, 4, o);
        uint32_t m = (uint32_t)sink.reports.size();
        fwrite(&m, 4, 1, o);
        for (auto& rr : sink.reports) {
            uint32_t ln = (uint32_t)rr.bytes.size();
            fwrite(&rr.t, 8, 1, o); fwrite(&rr.session, 4, 1, o); fwrite(&rr.track, 2, 1, o);
            fwrite(&rr.addr, 4, 1, o); fwrite(&rr.port, 2, 1, o); fwrite(&ln, 4, 1, o);
            fwrite(rr.bytes.data(), 1, ln, o);
        }
    }
    fclose(o);
    fprintf(stderr, "adapter_replay: %llu ticks, %llu copy passes, %llu stream errors\n", (unsigned long long)ticks,
            (unsigned long long)passes, (unsigned long long)stream_errors);
    if (sink.failPass)
        fprintf(stderr, "adapter_replay: %llu failed ticks, %llu good ticks after the failure\n",
                (unsigned long long)failedTicks, (unsigned long long)ticksAfterFailure);
    return 0;
}
