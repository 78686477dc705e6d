// edgpu_egress.cpp -- socket egress of a fan-out tick.
//
// The reference writes each packet from RTPStream::Write (Server.tproj/RTPStream.cpp:1084-1147):
//   * UDP: fSockets->GetSocketA()/B()->SendTo(remote addr, RTP/RTCP port, packet) with the result
//     ignored -- a full socket drops the datagram, it never blocks the output (:1145);
//   * TCP (RTSP-interleaved): InterleavedWrite (RTSPSessionInterface.cpp:255-344; the coalesce
//     buffer is bypassed, kTCPCoalesceDirectWriteSize = 0) -> RTSPResponseStream::WriteV with
//     kAllOrNothing (RTSPResponseStream.cpp:36-140): data left in the stream's output buffer
//     goes first; if it cannot all go, or none of the new frame goes, the write is EAGAIN ->
//     QTSS_WouldBlock; a frame that goes out partly counts as sent and its tail is buffered.
// Here one call sends a whole tick: the tick's DISTINCT bytes are brought to pinned host memory
// in one copy -- sub-streams flagged EDGPU_SUB_IDENTITY (UDP, no rewrite) of one sender carry the
// same bytes, each a suffix of the longest, so only that one region per sender crosses PCIe
// (edgpu_arena_gather packs the regions on the device first); TCP and rewritten sub-streams
// bring their own (EDGPU_EGRESS_DEDUP=0 copies the whole write-many arena instead).  Worker
// threads own disjoint subscribers (a TCP connection's frames keep the reference's
// per-connection order: track, RTP before RTCP), UDP datagrams leave in sendmmsg batches, TCP
// frames in sendmsg batches (MSG_NOSIGNAL: a reset peer raises no SIGPIPE), and the sub-streams
// that blocked are reported to the engine (edgpu_fanout_blocked) so the next tick resumes
// where the reference would.  Only EAGAIN blocks a TCP write; any other error marks the
// connection dead: like the reference, whose WritePacket counts a failed non-EAGAIN write as
// written (RTPSessionOutput.cpp:612-653), nothing is resent, and edgpu_egress_disconnected
// lists it for the host to tear down (ClientSessionClosing).
// Host code only: it uses the public C ABI of the engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <netinet/in.h>
#include <netinet/udp.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include "edgpu.h"
#include "edgpu_pacing.h"
#include "tick_regions.h"

namespace {

struct UdpDest {
    int fd[2] = {-1, -1};               // RTP, RTCP socket (-1: the worker's socket)
    sockaddr_in addr[2];
};

struct TcpConn {
    int fd = -1;
    std::string pending;                // RTSPResponseStream output buffer (unsent tail)
    int dead = 0;                       // errno of a failed (non-EAGAIN) write, 0 = alive
    bool reported = false;
};

#ifndef UDP_SEGMENT
#define UDP_SEGMENT 103
#endif

struct Worker {
    int udp_fd = -1;
    bool gso = true;                    // UDP generic segmentation offload still usable
    std::vector<edgpu_blocked> blocked;
    std::vector<edgpu_egress_block> why;   // per blocked sub-stream: writes that went, the cause
    std::vector<edgpu_out_desc> sel;       // a paced UDP sub-stream's packets that pass the gate
    uint64_t udp_datagrams = 0, udp_bytes = 0, udp_dropped = 0, tcp_frames = 0, tcp_bytes = 0, stale = 0;
    void block(uint32_t q, uint32_t sent, uint32_t written, uint32_t cause) {
        blocked.push_back(edgpu_blocked{q, sent});
        why.push_back(edgpu_egress_block{q, sent, written, cause});
    }
};

// A subscriber with the server's write gate (edgpu_egress_pacing).
struct Paced {
    Paced(const edpace::Config& c, bool tcp, const edgpu_pacing& p)
        : player(c, tcp, (p.flags & EDGPU_PACE_OVERBUFFER) != 0), video(p.video_tracks),
          overbuffer((p.flags & EDGPU_PACE_OVERBUFFER) != 0) {
        player.play_time_ms = p.play_time_ms;
    }
    edpace::Player player;
    uint32_t video;
    bool overbuffer;
    int32_t slot = 0;
};

}  // namespace

struct edgpu_egress {
    edgpu_ctx* ctx = nullptr;
    uint32_t nthreads = 1;
    bool dedup = true;
    bool gso = true;                    // EDGPU_EGRESS_GSO=0: one datagram per message
    std::map<uint64_t, UdpDest> udp;    // (subscriber << 16 | track)
    std::map<uint32_t, TcpConn> tcp;    // subscriber
    uint8_t* h_arena = nullptr;         // pinned: the tick's bytes (whole arena, or the gathered regions)
    size_t h_arena_cap = 0;
    edgpu_out_desc* desc = nullptr;     // pinned: the tick's descriptors
    uint64_t desc_cap = 0;
    std::vector<edgpu_substream_out> subs;
    std::vector<const uint8_t*> base;   // per sub-stream: host address of its arena region's start
    std::vector<Worker> workers;
    std::vector<edgpu_blocked> last_blocked;
    std::vector<edgpu_egress_block> last_why;
    std::vector<uint32_t> disconnected;
    // the write gate (Q20): config, paced subscribers, the tick's clock, the current pass's
    // arrivals and, per sender, the first bucket place of a new output this tick
    edpace::Config pcfg;
    std::map<uint32_t, Paced> paced;
    int64_t now = 0;
    std::vector<int64_t> arrival;
    std::map<uint32_t, int32_t> first_new;
    uint64_t copied_bytes = 0;
    std::atomic<int64_t> trace_left{0};     // EDGPU_PACE_TRACE=n: the first n gate decisions to stderr (debug)
    std::string err;
};

static int eg_fail(edgpu_egress* e, int code, const std::string& m) {
    if (e) e->err = m;
    return code;
}

// One UDP sub-stream: every datagram is offered to the socket once (errors ignored, like the
// reference's (void)SendTo); EAGAIN / ENOBUFS drop the datagram.
//
// With UDP GSO (UDP_SEGMENT, Linux >= 4.18) a run of datagrams of one length L to the
// sub-stream's destination -- FU-A fragments of one frame all have the same size -- goes down as
// ONE message whose kernel-side segmentation puts exactly the same datagrams on the wire, one
// per L bytes (the last may be shorter); up to 64 per message and 64 KiB.  The datagrams stay
// where they are in the pinned tick (one iovec each).  What changes is only failure
// granularity: a full socket drops a whole message instead of one datagram.  A message the
// route refuses (EINVAL, e.g. a smaller MTU) is resent one datagram at a time; a socket without
// GSO (EIO / EOPNOTSUPP) turns it off for that worker.  Datagrams over 1472 B go one per message.
static void send_udp_plain(Worker& w, int fd, const sockaddr_in* to, const uint8_t* base, const edgpu_out_desc* ds,
                           uint32_t count) {
    constexpr uint32_t kBatch = 256;
    mmsghdr msgs[kBatch];
    iovec iov[kBatch];
    uint32_t i = 0;
    while (i < count) {
        const uint32_t n = std::min(kBatch, count - i);
        for (uint32_t j = 0; j < n; j++) {
            iov[j].iov_base = const_cast<uint8_t*>(base + ds[i + j].offset);
            iov[j].iov_len = ds[i + j].len;
            memset(&msgs[j].msg_hdr, 0, sizeof(msgs[j].msg_hdr));
            msgs[j].msg_hdr.msg_name = const_cast<sockaddr_in*>(to);
            msgs[j].msg_hdr.msg_namelen = sizeof(sockaddr_in);
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
        }
        uint32_t done = 0;
        while (done < n) {
            const int r = sendmmsg(fd, msgs + done, n - done, MSG_DONTWAIT);
            if (r > 0) {
                for (int j = 0; j < r; j++) w.udp_bytes += iov[done + j].iov_len;
                w.udp_datagrams += (uint64_t)r;
                done += (uint32_t)r;
            } else {
                if (r < 0 && errno == EINTR) continue;
                w.udp_dropped++;                          // this datagram is lost; go on
                done++;
            }
        }
        i += n;
    }
}

static void send_udp_list(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, const UdpDest& d,
                          const edgpu_out_desc* ds, uint32_t count);
static void send_udp(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, const UdpDest& d) {
    send_udp_list(e, w, q, s, d, e->desc + s.desc_base, s.desc_count);
}
// `count` datagrams ds[0..count) of sub-stream q
static void send_udp_list(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, const UdpDest& d,
                          const edgpu_out_desc* ds, uint32_t count) {
    const int k = s.kind ? 1 : 0;
    const uint8_t* base = e->base[q] - s.out_base;
    const int fd = d.fd[k] >= 0 ? d.fd[k] : w.udp_fd;
    if (!e->gso || !w.gso) { send_udp_plain(w, fd, &d.addr[k], base, ds, count); return; }
    constexpr uint32_t kMsgs = 64, kSegs = 64, kMaxPayload = 65507, kMaxSeg = 1472;
    struct Msg { uint32_t first, n, seg; };
    mmsghdr msgs[kMsgs];
    Msg mi[kMsgs];
    iovec iov[kMsgs * kSegs];
    alignas(cmsghdr) char ctl[kMsgs][CMSG_SPACE(sizeof(uint16_t))];
    uint32_t i = 0;
    while (i < count) {
        // build up to kMsgs messages: runs of equal-length datagrams (+ one shorter tail)
        uint32_t nm = 0, niov = 0;
        while (nm < kMsgs && i < count) {
            const uint32_t L = ds[i].len;
            // a segment must fit the path MTU: only datagrams that fit a 1500-B Ethernet frame
            const uint32_t cap = (L && L <= kMaxSeg) ? std::min(kSegs, kMaxPayload / L) : 1;
            uint32_t n = 1;
            while (n < cap && i + n < count && ds[i + n].len == L) n++;
            if (n < cap && i + n < count && ds[i + n].len < L && ds[i + n].len > 0) n++;   // shorter last segment
            Msg& m = mi[nm];
            m.first = i; m.n = n; m.seg = L;
            mmsghdr& h = msgs[nm];
            memset(&h.msg_hdr, 0, sizeof(h.msg_hdr));
            h.msg_hdr.msg_name = const_cast<sockaddr_in*>(&d.addr[k]);
            h.msg_hdr.msg_namelen = sizeof(sockaddr_in);
            h.msg_hdr.msg_iov = &iov[niov];
            h.msg_hdr.msg_iovlen = n;
            for (uint32_t j = 0; j < n; j++) {
                iov[niov + j].iov_base = const_cast<uint8_t*>(base + ds[i + j].offset);
                iov[niov + j].iov_len = ds[i + j].len;
            }
            if (n > 1) {
                h.msg_hdr.msg_control = ctl[nm];
                h.msg_hdr.msg_controllen = CMSG_SPACE(sizeof(uint16_t));
                cmsghdr* c = CMSG_FIRSTHDR(&h.msg_hdr);
                c->cmsg_level = SOL_UDP;
                c->cmsg_type = UDP_SEGMENT;
                c->cmsg_len = CMSG_LEN(sizeof(uint16_t));
                const uint16_t seg = (uint16_t)L;
                memcpy(CMSG_DATA(c), &seg, sizeof(seg));
            }
            niov += n;
            i += n;
            nm++;
        }
        uint32_t done = 0;
        while (done < nm) {
            const int r = sendmmsg(fd, msgs + done, nm - done, MSG_DONTWAIT);
            if (r > 0) {
                for (int j = 0; j < r; j++) {
                    const Msg& m = mi[done + j];
                    for (uint32_t t = 0; t < m.n; t++) w.udp_bytes += ds[m.first + t].len;
                    w.udp_datagrams += m.n;
                }
                done += (uint32_t)r;
                continue;
            }
            if (r < 0 && errno == EINTR) continue;
            const Msg& m = mi[done];
            if (r < 0 && (errno == EIO || errno == EINVAL || errno == EOPNOTSUPP) && m.n > 1) {
                if (errno != EINVAL) w.gso = false;       // no GSO on this socket at all
                send_udp_plain(w, fd, &d.addr[k], base, ds + m.first, m.n);   // resend this one plainly
            } else {
                w.udp_dropped += m.n;                     // a full socket: the message is lost
            }
            done++;
        }
        if (!w.gso && i < count) { send_udp_plain(w, fd, &d.addr[k], base, ds + i, count - i); return; }
    }
}

// One TCP sub-stream, RTSPResponseStream::WriteV(kAllOrNothing) frame by frame, batched: the
// buffered tail goes first; frames the socket took (the last one possibly in part, its tail
// then buffered) are sent; the first frame that gets no byte blocks the sub-stream.
static void send_tcp(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, TcpConn& c) {
    const edgpu_out_desc* ds = e->desc + s.desc_base;
    const uint8_t* base = e->base[q] - s.out_base;
    if (c.dead) return;                                   // counted as written, never resent
    uint32_t i = 0;
    while (i < s.desc_count) {
        constexpr uint32_t kBatch = 512;
        iovec iov[kBatch + 1];
        uint32_t nv = 0;
        size_t plen = c.pending.size();
        if (plen) { iov[nv].iov_base = &c.pending[0]; iov[nv].iov_len = plen; nv++; }
        const uint32_t n = std::min(kBatch, s.desc_count - i);
        size_t total = plen;
        for (uint32_t j = 0; j < n; j++) {
            iov[nv].iov_base = const_cast<uint8_t*>(base + ds[i + j].offset);
            iov[nv].iov_len = ds[i + j].len;
            total += ds[i + j].len;
            nv++;
        }
        msghdr mh;
        memset(&mh, 0, sizeof(mh));
        mh.msg_iov = iov;
        mh.msg_iovlen = nv;
        ssize_t r = sendmsg(c.fd, &mh, MSG_NOSIGNAL);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) {   // peer gone: not backpressure
            c.dead = errno;
            c.pending.clear();
            return;
        }
        size_t wrote = r > 0 ? (size_t)r : 0;
        if (wrote < plen) {                               // the old tail is still not out
            c.pending.erase(0, wrote);
            w.block(q, i, i, 0);
            return;
        }
        c.pending.clear();
        wrote -= plen;
        uint32_t j = 0;
        while (j < n && wrote >= ds[i + j].len) { wrote -= ds[i + j].len; w.tcp_bytes += ds[i + j].len; j++; }
        w.tcp_frames += j;
        if (j < n && wrote > 0) {                         // partly out: counted sent, tail buffered
            const edgpu_out_desc& d = ds[i + j];
            c.pending.assign(reinterpret_cast<const char*>(base + d.offset) + wrote, d.len - wrote);
            w.tcp_bytes += d.len;
            w.tcp_frames++;
            j++;
            i += j;
            if (i < s.desc_count) w.block(q, i, i, 0);
            return;
        }
        i += j;
        if (j < n || (size_t)r < total) {                 // no byte of frame i went out
            w.block(q, i, i, 0);
            return;
        }
    }
}

// One frame of a paced TCP sub-stream, RTSPResponseStream::WriteV(kAllOrNothing): 1 = it went
// (a partial frame counts, its tail buffered, 2), 0 = no byte of it went (EAGAIN), -1 = dead peer.
static int tcp_frame(Worker& w, TcpConn& c, const uint8_t* p, uint32_t len) {
    for (;;) {
        iovec iov[2];
        uint32_t nv = 0;
        const size_t plen = c.pending.size();
        if (plen) { iov[nv].iov_base = &c.pending[0]; iov[nv].iov_len = plen; nv++; }
        iov[nv].iov_base = const_cast<uint8_t*>(p); iov[nv].iov_len = len; nv++;
        msghdr mh;
        memset(&mh, 0, sizeof(mh));
        mh.msg_iov = iov;
        mh.msg_iovlen = nv;
        const ssize_t r = sendmsg(c.fd, &mh, MSG_NOSIGNAL);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) { c.dead = errno; c.pending.clear(); return -1; }
        size_t wrote = r > 0 ? (size_t)r : 0;
        if (wrote < plen) { c.pending.erase(0, wrote); return 0; }
        c.pending.clear();
        wrote -= plen;
        if (wrote == 0) return 0;
        w.tcp_frames++;
        w.tcp_bytes += len;
        if (wrote < len) { c.pending.assign(reinterpret_cast<const char*>(p) + wrote, len - wrote); return 2; }
        return 1;
    }
}

// A paced sub-stream: RTPSessionOutput::WritePacket's transmit time, then RTPStream::Write's gate
// before each socket write (edgpu_pacing.h): the over-buffer window (RTP, and RTCP while
// overbuffering is off) holds the packet -> the sub-stream stops here (and a new output's first
// pass takes the packet's age as its buffer delay, RTPSessionOutput.cpp:612-622); a stale RTP
// packet of a TCP non-video stream is dropped (counted as written); a written RTP packet enters
// the window.
static void send_paced(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, Paced& P,
                       const UdpDest* ud, TcpConn* tc) {
    const edgpu_out_desc* ds = e->desc + s.desc_base;
    const uint8_t* base = e->base[q] - s.out_base;
    const int64_t* arr = e->arrival.data() + s.desc_base;
    const bool rtcp = s.kind != 0, tcp = s.transport == EDGPU_TRANSPORT_TCP;
    const bool video = s.track < 32 && ((P.video >> s.track) & 1u);
    const int64_t now = e->now;
    const int64_t lateness = e->pcfg.bucket_delay_ms * (int64_t)(P.slot / (int32_t)e->pcfg.bucket_size);
    auto fn = e->first_new.find(s.sender);
    const bool first = fn != e->first_new.end() && P.slot >= fn->second;   // ReflectPackets' firstPacket
    edpace::Player& pl = P.player;
    if (tcp && tc->dead) return;
    w.sel.clear();
    uint32_t written = 0;
    bool socket_full = false;                   // a frame went out in part: the next one waits
    for (uint32_t i = 0; i < s.desc_count; i++) {
        const uint32_t len = ds[i].len - (tcp ? 4u : 0u);           // the packet RTPStream::Write gets
        const int64_t tt = edpace::transmit_time(now, lateness, pl.buffer_delay_ms, arr[i]);
        if ((!rtcp || !P.overbuffer) && pl.win.CheckTransmitTime(tt, now, (int32_t)len) > now) {
            if (first) pl.buffer_delay_ms = now - arr[i];
            w.block(q, i, written, 1);
            break;
        }
        if (e->trace_left > 0 && tcp && !video && !rtcp && (now - tt > 800 || first)) {
            e->trace_left--;
            fprintf(stderr, "pace sub=%u tr=%u now=%lld arr=%lld bd=%lld tt=%lld first=%d slot=%d st=%d lc=%lld\n", s.subscriber,
                    s.track, (long long)now, (long long)arr[i], (long long)pl.buffer_delay_ms, (long long)tt, (int)first,
                    P.slot, (int)pl.started_thinning, (long long)pl.last_check);
        }
        if (!rtcp && !edpace::keep_packet(pl, s.track, video, tcp, tt, now - tt, now, e->pcfg)) {
            w.stale++;
            continue;
        }
        if (tcp) {
            const int r = socket_full ? 0 : tcp_frame(w, *tc, base + ds[i].offset, ds[i].len);
            if (r < 0) break;                                         // dead peer: counted as written
            if (r == 0) {
                if (first) pl.buffer_delay_ms = now - arr[i];
                w.block(q, i, written, 0);
                break;
            }
            if (r == 2) socket_full = true;
        } else {
            w.sel.push_back(ds[i]);
        }
        written++;
        if (!rtcp) pl.win.AddPacketToWindow((int32_t)len);
    }
    if (!tcp && !w.sel.empty()) send_udp_list(e, w, q, s, *ud, w.sel.data(), (uint32_t)w.sel.size());
}

extern "C" {

int edgpu_egress_create(edgpu_ctx* ctx, uint32_t threads, edgpu_egress** out) {
    if (!ctx || !out) return EDGPU_BAD_ARGUMENT;
    edgpu_egress* e = new edgpu_egress();
    e->ctx = ctx;
    e->nthreads = std::max(1u, std::min(threads, 64u));
    if (const char* v = getenv("EDGPU_EGRESS_DEDUP")) e->dedup = atoi(v) != 0;
    if (const char* v = getenv("EDGPU_EGRESS_GSO")) e->gso = atoi(v) != 0;
    if (const char* v = getenv("EDGPU_PACE_TRACE")) e->trace_left = atoll(v);
    e->workers.resize(e->nthreads);
    for (Worker& w : e->workers) {
        w.udp_fd = socket(AF_INET, SOCK_DGRAM, 0);
        if (w.udp_fd < 0) { edgpu_egress_destroy(e); return EDGPU_ERR; }
        int big = 8 << 20;
        setsockopt(w.udp_fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    }
    *out = e;
    return EDGPU_OK;
}

int edgpu_egress_destroy(edgpu_egress* e) {
    if (!e) return EDGPU_OK;
    for (Worker& w : e->workers) if (w.udp_fd >= 0) close(w.udp_fd);
    if (e->h_arena) (void)hipHostFree(e->h_arena);
    if (e->desc) (void)hipHostFree(e->desc);
    delete e;
    return EDGPU_OK;
}

const char* edgpu_egress_last_error(edgpu_egress* e) { return e ? e->err.c_str() : "egress is NULL"; }

int edgpu_egress_udp(edgpu_egress* e, uint32_t subscriber, uint32_t track, int rtp_fd, int rtcp_fd,
                     uint32_t ipv4_be, uint16_t rtp_port_be, uint16_t rtcp_port_be) {
    if (!e) return EDGPU_BAD_ARGUMENT;
    UdpDest d;
    d.fd[0] = rtp_fd;
    d.fd[1] = rtcp_fd;
    for (int k = 0; k < 2; k++) {
        memset(&d.addr[k], 0, sizeof(sockaddr_in));
        d.addr[k].sin_family = AF_INET;
        d.addr[k].sin_addr.s_addr = ipv4_be;
        d.addr[k].sin_port = k ? rtcp_port_be : rtp_port_be;
    }
    e->udp[(uint64_t)subscriber << 16 | track] = d;
    return EDGPU_OK;
}

int edgpu_egress_tcp(edgpu_egress* e, uint32_t subscriber, int fd) {
    if (!e || fd < 0) return EDGPU_BAD_ARGUMENT;
    e->tcp[subscriber].fd = fd;
    return EDGPU_OK;
}

// One copy pass of a tick (the whole tick unless it exceeded the arena, edgpu_fanout_next): its
// bytes to pinned memory, its sub-streams to the sockets; blocked sub-streams are appended.
static int send_pass(edgpu_egress* e, const edgpu_fanout_result* r, const edgpu_tick_stats& st,
                     std::vector<edgpu_blocked>& blocked, edgpu_egress_stats& s) {
    int rc;
    if (st.pass_packets > e->desc_cap) {
        if (e->desc) (void)hipHostFree(e->desc);
        e->desc = nullptr;
        e->desc_cap = 0;
        const uint64_t cap = std::max<uint64_t>((uint64_t)st.pass_packets + st.pass_packets / 2, 1 << 16);
        if (hipHostMalloc((void**)&e->desc, cap * sizeof(edgpu_out_desc), hipHostMallocDefault) != hipSuccess)
            return eg_fail(e, EDGPU_OUT_OF_MEMORY, "pinned descriptors");
        e->desc_cap = cap;
    }
    e->subs.resize(r->n_substreams);
    if ((rc = edgpu_copy_to_host(e->ctx, e->desc, r->desc, (uint64_t)st.pass_packets * sizeof(edgpu_out_desc))) ||
        (rc = edgpu_copy_to_host(e->ctx, e->subs.data(), r->substreams, r->n_substreams * sizeof(edgpu_substream_out))))
        return eg_fail(e, rc, "copy to host");
    // the distinct bytes: one region per identity sender (its longest sub-stream) + every other
    // non-empty sub-stream (tick_regions.h)
    const uint32_t nq = (uint32_t)e->subs.size();
    edgpu_host::TickRegions tr;
    uint64_t need = st.pass_arena_bytes;
    if (e->dedup) {
        tr = edgpu_host::tick_regions(e->subs.data(), nq);
        need = tr.bytes;
    }
    if (need > e->h_arena_cap) {
        if (e->h_arena) (void)hipHostFree(e->h_arena);
        e->h_arena = nullptr;
        const size_t cap = std::max<size_t>(need + need / 2, 1 << 20);   // geometric: pinning is slow
        if (hipHostMalloc((void**)&e->h_arena, cap, hipHostMallocDefault) != hipSuccess)
            return eg_fail(e, EDGPU_OUT_OF_MEMORY, "pinned arena");
        e->h_arena_cap = cap;
    }
    e->base.assign(nq, nullptr);
    if (e->dedup) {
        // gathered straight into the pinned buffer: the kernel's stores cross PCIe (one pass)
        if ((rc = edgpu_arena_gather(e->ctx, r, tr.reg.data(), (uint32_t)tr.reg.size(), e->h_arena, e->h_arena_cap)))
            return eg_fail(e, rc, "gather to host");
        for (uint32_t q = 0; q < nq; q++)
            if (tr.src[q].first != edgpu_host::TickRegions::kNone) e->base[q] = tr.at(e->h_arena, q);
    } else {
        if ((rc = edgpu_copy_to_host(e->ctx, e->h_arena, r->arena, st.pass_arena_bytes))) return eg_fail(e, rc, "copy to host");
        for (uint32_t q = 0; q < nq; q++) e->base[q] = e->h_arena + e->subs[q].out_base;
    }
    e->copied_bytes += need;
    if (!e->paced.empty()) {
        // the write gate's inputs: every descriptor's arrival, and (at the tick's first pass, whose
        // table flags every new output) the first bucket place of a new output per sender
        e->arrival.resize(std::max<uint64_t>(st.pass_packets, 1));
        if (st.pass_packets &&
            (rc = edgpu_fanout_arrivals(e->ctx, e->arrival.data(), st.pass_packets, EDGPU_PTR_HOST)))
            return eg_fail(e, rc, "arrivals (pacing needs serial ticks)");
        if (st.pass == 0) {
            e->first_new.clear();
            std::map<uint32_t, int32_t> slot_of;
            for (uint32_t q = 0; q < nq; q++) {
                const edgpu_substream_out& o = e->subs[q];
                if (!(o.flags & EDGPU_SUB_NEW)) continue;
                auto it = slot_of.find(o.subscriber);
                if (it == slot_of.end()) {
                    int32_t sl = -1;
                    if (edgpu_subscriber_slot(e->ctx, o.subscriber, &sl) != EDGPU_OK) sl = -1;
                    it = slot_of.emplace(o.subscriber, sl).first;
                }
                if (it->second < 0) continue;
                auto f = e->first_new.find(o.sender);
                if (f == e->first_new.end() || it->second < f->second) e->first_new[o.sender] = it->second;
            }
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    for (Worker& w : e->workers) {
        w.blocked.clear(); w.why.clear();
        w.udp_datagrams = w.udp_bytes = w.udp_dropped = w.tcp_frames = w.tcp_bytes = w.stale = 0;
    }
    // Which worker sends a row: a TCP connection's rows, and every row of a paced subscriber, on
    // the worker of their subscriber (one connection's frames in order, the pacing state without a
    // lock); plain UDP rows in blocks of consecutive rows -- a subscriber's rows are contiguous and
    // a session's subscribers mostly so -- so a worker sends whole sessions and reads their shared
    // regions of the pinned tick from its own caches instead of every worker reading every region.
    constexpr uint32_t kRowBlock = 64;
    const bool any_paced = !e->paced.empty();
    auto run = [&](uint32_t k) {
        Worker& w = e->workers[k];
        for (uint32_t q = 0; q < (uint32_t)e->subs.size(); q++) {
            const edgpu_substream_out& s = e->subs[q];
            if (s.desc_count == 0) continue;
            const bool by_sub = any_paced || s.transport == EDGPU_TRANSPORT_TCP;
            if ((by_sub ? s.subscriber : q / kRowBlock) % e->nthreads != k) continue;
            auto pc = e->paced.find(s.subscriber);
            if (pc != e->paced.end()) {                  // (one worker owns a subscriber: no lock)
                if (s.transport == EDGPU_TRANSPORT_TCP) {
                    auto it = e->tcp.find(s.subscriber);
                    if (it != e->tcp.end()) send_paced(e, w, q, s, pc->second, nullptr, &it->second);
                } else {
                    auto it = e->udp.find((uint64_t)s.subscriber << 16 | s.track);
                    if (it != e->udp.end()) send_paced(e, w, q, s, pc->second, &it->second, nullptr);
                }
                continue;
            }
            if (s.transport == EDGPU_TRANSPORT_TCP) {
                auto it = e->tcp.find(s.subscriber);
                if (it != e->tcp.end()) send_tcp(e, w, q, s, it->second);
            } else {
                auto it = e->udp.find((uint64_t)s.subscriber << 16 | s.track);
                if (it != e->udp.end()) send_udp(e, w, q, s, it->second);
            }
        }
    };
    if (e->nthreads == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (uint32_t k = 0; k < e->nthreads; k++) th.emplace_back(run, k);
        for (auto& t : th) t.join();
    }
    s.send_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    for (Worker& w : e->workers) {
        blocked.insert(blocked.end(), w.blocked.begin(), w.blocked.end());
        e->last_why.insert(e->last_why.end(), w.why.begin(), w.why.end());
        s.stale_dropped += w.stale;
        s.udp_datagrams += w.udp_datagrams; s.udp_bytes += w.udp_bytes; s.udp_dropped += w.udp_dropped;
        s.tcp_frames += w.tcp_frames; s.tcp_bytes += w.tcp_bytes;
    }
    return EDGPU_OK;
}

int edgpu_egress_send(edgpu_egress* e, const edgpu_fanout_result* r, edgpu_egress_stats* out) {
    if (!e || !r) return EDGPU_BAD_ARGUMENT;
    auto t0 = std::chrono::steady_clock::now();
    edgpu_egress_stats s;
    memset(&s, 0, sizeof(s));
    e->copied_bytes = 0;
    e->last_why.clear();
    std::vector<edgpu_blocked> blocked;
    // every copy pass of the tick, in sub-stream row order: a connection's frames keep their order
    edgpu_fanout_result cur = *r;
    int failed = EDGPU_OK;
    for (;;) {
        edgpu_tick_stats st;
        int rc = edgpu_tick_stats_get(e->ctx, &st);
        if (rc) { failed = eg_fail(e, rc, "tick stats"); break; }
        if (st.status) { failed = eg_fail(e, st.status, "device-side status after fan-out"); break; }
        if ((rc = send_pass(e, &cur, st, blocked, s))) { failed = rc; break; }
        if (!st.more_passes) break;
        uint32_t launched = 0;
        if ((rc = edgpu_fanout_next(e->ctx, &cur, &launched))) { failed = eg_fail(e, rc, "next copy pass"); break; }
        if (!launched) break;
    }
    if (failed) {
        // the context must not stay owing the rest of the tick (every later ingest / fan-out would
        // be refused): the remaining passes are launched unsent (counted in lost_passes), and the
        // blocked sub-streams of the passes already sent are still reported
        for (uint32_t guard = 0; guard < (1u << 20); guard++) {
            uint32_t launched = 0;
            if (edgpu_fanout_next(e->ctx, &cur, &launched) != EDGPU_OK || !launched) break;
        }
        if (!blocked.empty()) {
            std::sort(blocked.begin(), blocked.end(),
                      [](const edgpu_blocked& a, const edgpu_blocked& b) { return a.substream < b.substream; });
            (void)edgpu_fanout_blocked(e->ctx, blocked.data(), (uint32_t)blocked.size());
        }
        return failed;
    }
    std::sort(blocked.begin(), blocked.end(), [](const edgpu_blocked& a, const edgpu_blocked& b) { return a.substream < b.substream; });
    s.blocked_substreams = (uint32_t)blocked.size();
    s.copy_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - s.send_ms;
    e->last_blocked = blocked;
    std::sort(e->last_why.begin(), e->last_why.end(),
              [](const edgpu_egress_block& a, const edgpu_egress_block& b) { return a.substream < b.substream; });
    for (auto& kv : e->tcp)
        if (kv.second.dead && !kv.second.reported) { e->disconnected.push_back(kv.first); kv.second.reported = true; }
    s.copied_bytes = e->copied_bytes;
    int rc;
    if (!blocked.empty() && (rc = edgpu_fanout_blocked(e->ctx, blocked.data(), (uint32_t)blocked.size())))
        return eg_fail(e, rc, "backpressure report");
    if (out) *out = s;
    return EDGPU_OK;
}

int edgpu_egress_blocked(edgpu_egress* e, edgpu_blocked* out, uint32_t cap, uint32_t* n) {
    if (!e || !n || (cap && !out)) return EDGPU_BAD_ARGUMENT;
    const uint32_t k = (uint32_t)std::min<size_t>(cap, e->last_blocked.size());
    std::copy(e->last_blocked.begin(), e->last_blocked.begin() + k, out);
    *n = (uint32_t)e->last_blocked.size();
    return EDGPU_OK;
}

int edgpu_egress_disconnected(edgpu_egress* e, uint32_t* out, uint32_t cap, uint32_t* n) {
    if (!e || !n || (cap && !out)) return EDGPU_BAD_ARGUMENT;
    const uint32_t k = (uint32_t)std::min<size_t>(cap, e->disconnected.size());
    std::copy(e->disconnected.begin(), e->disconnected.begin() + k, out);
    *n = (uint32_t)e->disconnected.size();
    e->disconnected.erase(e->disconnected.begin(), e->disconnected.begin() + k);
    return EDGPU_OK;
}

int edgpu_egress_pacing_config(edgpu_egress* e, const edgpu_pacing_config* c) {
    if (!e || !c || c->bucket_size == 0) return EDGPU_BAD_ARGUMENT;
    e->pcfg.bucket_delay_ms = c->bucket_delay_ms;
    e->pcfg.over_buffer_ms = c->over_buffer_ms;
    e->pcfg.drop_all_packets_ms = c->drop_all_packets_ms;
    e->pcfg.thin_all_the_way_ms = c->thin_all_the_way_ms;
    e->pcfg.start_thinning_ms = c->start_thinning_ms;
    e->pcfg.bucket_size = c->bucket_size;
    e->pcfg.send_interval_ms = c->send_interval_ms;
    e->pcfg.max_send_ahead_s = c->max_send_ahead_s;
    e->pcfg.overbuffer_rate = c->overbuffer_rate;
    return EDGPU_OK;
}

int edgpu_egress_pacing(edgpu_egress* e, uint32_t subscriber, const edgpu_pacing* p) {
    if (!e) return EDGPU_BAD_ARGUMENT;
    if (!p) { e->paced.erase(subscriber); return EDGPU_OK; }
    int32_t slot = -1;
    if (edgpu_subscriber_slot(e->ctx, subscriber, &slot) != EDGPU_OK) return eg_fail(e, EDGPU_BAD_ARGUMENT, "bad subscriber");
    const bool tcp = e->tcp.count(subscriber) != 0;
    e->paced.erase(subscriber);
    Paced& P = e->paced.emplace(subscriber, Paced(e->pcfg, tcp, *p)).first->second;
    P.slot = slot;
    return EDGPU_OK;
}

int edgpu_egress_clock(edgpu_egress* e, int64_t now_ms) {
    if (!e) return EDGPU_BAD_ARGUMENT;
    e->now = now_ms;
    return EDGPU_OK;
}

int edgpu_egress_block_info(edgpu_egress* e, edgpu_egress_block* out, uint32_t cap, uint32_t* n) {
    if (!e || !n || (cap && !out)) return EDGPU_BAD_ARGUMENT;
    const uint32_t k = (uint32_t)std::min<size_t>(cap, e->last_why.size());
    std::copy(e->last_why.begin(), e->last_why.begin() + k, out);
    *n = (uint32_t)e->last_why.size();
    return EDGPU_OK;
}

int edgpu_egress_flush(edgpu_egress* e, uint64_t* out_pending) {
    if (!e) return EDGPU_BAD_ARGUMENT;
    uint64_t left = 0;
    for (auto& kv : e->tcp) {
        TcpConn& c = kv.second;
        while (!c.pending.empty() && !c.dead) {
            const ssize_t r = send(c.fd, c.pending.data(), c.pending.size(), MSG_NOSIGNAL);
            if (r < 0 && errno == EINTR) continue;
            if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) { c.dead = errno; c.pending.clear(); break; }
            if (r <= 0) break;
            c.pending.erase(0, (size_t)r);
        }
        left += c.pending.size();
        if (c.dead && !c.reported) { e->disconnected.push_back(kv.first); c.reported = true; }
    }
    if (out_pending) *out_pending = left;
    return EDGPU_OK;
}

}  // extern "C"
