// reflector_adapter.cpp -- see reflector_adapter.h.
#include "reflector_adapter.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace edgpu_reflector {

Reflector::Reflector(const edgpu_config* cfg) {
    fStatus = edgpu_ctx_create(cfg, &fCtx);
}

Reflector::~Reflector() {
    if (fCtx) edgpu_ctx_destroy(fCtx);
}

int Reflector::SetupReflectorSession(const std::string& sdp, bool udpPush, uint32_t* outSession) {
    if (!fCtx) return kRequestFailed;
    uint32_t s = 0, n = 0;
    int err = edgpu_session_add(fCtx, sdp.data(), (uint32_t)sdp.size(), udpPush ? 1 : 0, &s);
    if (err) return err;
    if ((err = edgpu_session_tracks(fCtx, s, &n))) return err;
    if (fTracks.size() <= s) fTracks.resize(s + 1, 0);
    fTracks[s] = n;
    if (outSession) *outSession = s;
    return kNoErr;
}

uint32_t Reflector::GetNumStreams(uint32_t session) const {
    return session < fTracks.size() ? fTracks[session] : 0;
}

int Reflector::AddOutput(uint32_t session, bool interleaved, uint32_t* outHandle) {
    if (!fCtx) return kRequestFailed;
    return edgpu_subscriber_add(fCtx, session, interleaved ? EDGPU_TRANSPORT_TCP : EDGPU_TRANSPORT_UDP, outHandle);
}

int Reflector::PlayRTPInfo(uint32_t session, bool interleaved, int64_t nowMs, uint32_t* outHandle,
                           std::vector<edgpu_rtp_info>* outInfo) {
    if (!fCtx) return kRequestFailed;
    int err = FlushIngest();
    if (err) return err;
    std::vector<edgpu_rtp_info> info(std::max<uint32_t>(GetNumStreams(session), 1));
    err = edgpu_subscriber_play(fCtx, session, interleaved ? EDGPU_TRANSPORT_TCP : EDGPU_TRANSPORT_UDP,
                                EDGPU_PLAY_RTP_INFO, nowMs, outHandle, info.data());
    if (!err && outInfo) *outInfo = info;
    return err;
}

int Reflector::RemoveOutput(uint32_t handle) {
    if (!fCtx) return kRequestFailed;
    return edgpu_subscriber_remove(fCtx, handle);
}

void Reflector::PushPacket(uint32_t session, uint32_t track, const char* packet, uint32_t packetLen,
                           bool isRTCP, int64_t nowMs) {
    // ReflectorStream::PushPacket ignores empty packets (ReflectorStream.cpp:533); the
    // '$' framing caps a pushed packet at 65535 bytes.
    if (packetLen == 0 || track >= GetNumStreams(session)) return;
    packetLen = std::min<uint32_t>(packetLen, 65535);
    Pushed p;
    p.session = session;
    p.channel = (uint8_t)(2 * track + (isRTCP ? 1 : 0));
    p.t = nowMs;
    p.off = (uint32_t)fBytes.size();
    p.len = packetLen;
    fBytes.insert(fBytes.end(), packet, packet + packetLen);
    fPushed.push_back(p);
}

void Reflector::ProcessUDPPacket(uint32_t session, uint32_t track, bool rtcpPort, const char* packet,
                                 uint32_t packetLen, uint32_t remoteAddr, uint16_t remotePort, int64_t nowMs) {
    if (packetLen == 0 || track >= GetNumStreams(session)) return;
    PushPacket(session, track, packet, packetLen, rtcpPort, nowMs);
    edgpu_udp_source u;
    memset(&u, 0, sizeof(u));
    u.session = session;
    u.channel = (uint8_t)(2 * track + (rtcpPort ? 1 : 0));
    u.port = remotePort;
    u.addr = remoteAddr;
    u.len = packetLen;
    memcpy(u.head, packet, std::min<uint32_t>(packetLen, 4));
    fSources.push_back(u);
}

int Reflector::SetSourceIdentity(uint32_t session, uint32_t track, uint32_t ssrc, int64_t cnameSecs) {
    if (!fCtx) return kRequestFailed;
    return edgpu_source_identity(fCtx, session, track, ssrc, cnameSecs);
}

int Reflector::FlushIngest() {
    int err;
    if (!fPushed.empty()) {
        // group by session (stable: arrival order within a session) into 16-B slots with the
        // packet 4 bytes in -- the edgpu_ingest batch layout
        std::vector<uint32_t> order(fPushed.size());
        for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return fPushed[a].session < fPushed[b].session; });
        std::vector<edgpu_pkt_desc> desc(order.size());
        std::vector<uint32_t> segOff, segSess;
        uint64_t blobBytes = 0;
        for (uint32_t i : order) {
            const uint32_t clamped = std::min<uint32_t>(fPushed[i].len, 2060);
            blobBytes += (clamped + 4 + 15) & ~15u;
        }
        std::vector<uint8_t> blob(std::max<uint64_t>(blobBytes, 16), 0);
        uint64_t off = 0;
        for (uint32_t k = 0; k < order.size(); k++) {
            const Pushed& p = fPushed[order[k]];
            if (segSess.empty() || segSess.back() != p.session) { segOff.push_back(k); segSess.push_back(p.session); }
            const uint32_t clamped = std::min<uint32_t>(p.len, 2060);   // bytes past 2060 are never read
            desc[k].slot = (uint32_t)(off / 16);
            desc[k].len = (uint16_t)p.len;
            desc[k].channel = p.channel;
            desc[k].flags = 0;
            desc[k].arrival_ms = p.t;
            memcpy(&blob[off + 4], &fBytes[p.off], clamped);
            off += (clamped + 4 + 15) & ~15u;
        }
        segOff.push_back((uint32_t)order.size());
        err = edgpu_ingest(fCtx, desc.data(), (uint32_t)desc.size(), segOff.data(), segSess.data(),
                           (uint32_t)segSess.size(), blob.data(), blobBytes, EDGPU_PTR_HOST);
        if (err) return err;
        if ((err = edgpu_keyframe_index(fCtx))) return err;
        fPushed.clear();
        fBytes.clear();
    }
    if (!fSources.empty()) {
        if ((err = edgpu_udp_sources(fCtx, fSources.data(), (uint32_t)fSources.size()))) return err;
        fSources.clear();
    }
    return kNoErr;
}

int Reflector::ReflectPackets(int64_t nowMs, OutputSink* sink) {
    if (!fCtx) return kRequestFailed;
    int err = FlushIngest();
    if (err) return err;
    edgpu_fanout_result res;
    if ((err = edgpu_fanout(fCtx, nowMs, &res))) return err;
    uint32_t nrr = 0;
    if ((err = edgpu_source_reports(fCtx, nullptr, 0, &nrr)) && nrr == 0) return err;
    if (nrr && sink) {
        std::vector<edgpu_source_report> rr(nrr);
        if ((err = edgpu_source_reports(fCtx, rr.data(), nrr, &nrr))) return err;
        for (const edgpu_source_report& r : rr)
            sink->SendReceiverReport(r.session, r.track, r.addr, r.port, r.bytes, r.len);
    }
    edgpu_tick_stats st;
    if ((err = edgpu_tick_stats_get(fCtx, &st))) return err;
    if (st.status) return st.status;
    if (!sink || st.relayed_packets == 0) return kNoErr;
    std::vector<edgpu_substream_out> subs(res.n_substreams);
    std::vector<edgpu_out_desc> d(st.relayed_packets);
    fArena.resize(st.arena_bytes);
    if ((err = edgpu_copy_to_host(fCtx, subs.data(), res.substreams, subs.size() * sizeof(subs[0])))) return err;
    if ((err = edgpu_copy_to_host(fCtx, d.data(), res.desc, d.size() * sizeof(d[0])))) return err;
    if ((err = edgpu_copy_to_host(fCtx, fArena.data(), res.arena, fArena.size()))) return err;
    std::vector<int64_t> arrival;
    if (sink->WantsArrivals()) {
        arrival.resize(d.size());
        if ((err = edgpu_fanout_arrivals(fCtx, arrival.data(), (uint32_t)arrival.size(), EDGPU_PTR_HOST))) return err;
    }
    sink->BeginTick(subs.data(), (uint32_t)subs.size());
    // SendPacketsToOutput (ReflectorStream.cpp:1138-1198): a write that would block stops this
    // output's sub-stream for the tick; the engine then bookmarks the blocked packet
    std::vector<edgpu_blocked> blocked;
    for (uint32_t s = 0; s < (uint32_t)subs.size(); s++) {
        const edgpu_substream_out& q = subs[s];
        for (uint32_t i = 0; i < q.desc_count; i++) {
            const edgpu_out_desc& o = d[q.desc_base + i];
            PacketWrite w;
            w.subscriber = q.subscriber;
            w.track = q.track;
            w.isRTCP = q.kind != 0;
            w.interleaved = q.transport == EDGPU_TRANSPORT_TCP;
            w.wire = &fArena[o.offset];
            w.wireLen = o.len;
            w.packetID = o.packet_id;
            w.arrivalMs = arrival.empty() ? -1 : arrival[q.desc_base + i];
            w.sender = q.sender;
            w.newOutput = (q.flags & EDGPU_SUB_NEW) != 0;
            err = sink->Write(w);
            if (err == kWouldBlock) { blocked.push_back(edgpu_blocked{s, i}); break; }
            if (err) return err;
        }
    }
    if (!blocked.empty()) return edgpu_fanout_blocked(fCtx, blocked.data(), (uint32_t)blocked.size());
    return kNoErr;
}

// ---------------------------------------------------------------------------------------
static const unsigned char kSTX = 0x28, kETX = 0x29;   // BUF_STX / BUF_ETX

CKeyFrameCache::CKeyFrameCache(int len) : mem_size(len) {
    _memory = (char*)malloc(mem_size);
    curdatalen = 0;
}

CKeyFrameCache::~CKeyFrameCache() {
    free(_memory);
    _memory = nullptr;
    mem_size = 0;
    curdatalen = 0;
}

bool CKeyFrameCache::PutOnePacket(char* buf, int len, int nalutype, int start) {
    if (buf == nullptr || len == 0) return false;
    if (nalutype == 7 && start == 1) curdatalen = 0;          // a new SPS starts a new GOP
    // the caller's packet is rewritten in place: byte 13 (the NAL header of an FU-A start
    // fragment after a 12-byte RTP header) becomes 0x67 (SPS) or 0x41 (keyframecache.cpp:
    // 27-40); the reference does it for any length (past the packet when len < 14) -- here
    // only inside the packet.  The reference's ./data.264 debug dump is not reproduced.
    if (start == 1 && len >= 14) buf[13] = (char)(nalutype == 7 ? 0x67 : 0x41);
    // the reference's 5 KiB TLV scratch: it overruns it for len > 5116 (FrameBuffer::Encode
    // ignores the capacity, keyframecache.h:24-45); refused here
    if (len < 0 || len + 4 > 5 * 1024) return false;
    unsigned char rec[5 * 1024];
    rec[0] = kSTX;
    rec[1] = (unsigned char)((unsigned)len >> 8);
    rec[2] = (unsigned char)len;
    memcpy(rec + 3, buf, len);
    rec[3 + len] = kETX;
    return SetBuf((char*)rec, len + 4);
}

bool CKeyFrameCache::GetOnePacket(char* outbuf, int& outLen, int curOffset) {
    if (curOffset >= curdatalen) return false;
    if ((unsigned char)_memory[curOffset] != kSTX) return false;
    const int pkgLen = ((unsigned char)_memory[curOffset + 1] << 8) | (unsigned char)_memory[curOffset + 2];
    if (pkgLen >= curdatalen) return false;
    if ((unsigned char)_memory[curOffset + 3 + pkgLen] != kETX) return false;
    memcpy(outbuf, _memory + curOffset + 3, pkgLen);
    outLen = pkgLen;
    return true;
}

bool CKeyFrameCache::SetBuf(char* frameBuf, int len) {
    if (frameBuf == nullptr || len == 0) return false;
    if (len + curdatalen > mem_size) return false;
    memcpy(_memory + curdatalen, frameBuf, len);
    curdatalen += len;
    return true;
}

int CKeyFrameCache::LoadGOP(Reflector& r, uint32_t session, uint32_t track, uint32_t* outPackets) {
    uint64_t n = 0;
    uint32_t k = 0;
    const int err = edgpu_gop_copy(r.Context(), session, track, (uint8_t*)_memory, (uint64_t)mem_size, &n, &k);
    if (err) return err;
    curdatalen = (int)n;
    if (outPackets) *outPackets = k;
    return kNoErr;
}

}  // namespace edgpu_reflector
