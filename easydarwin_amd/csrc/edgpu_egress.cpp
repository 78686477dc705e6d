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
// Here one call sends a whole tick: the arena, descriptors and sub-stream table are copied to
// pinned host memory once, worker threads own disjoint subscribers (a TCP connection's frames
// keep the reference's per-connection order: track, RTP before RTCP), UDP datagrams leave in
// sendmmsg batches, TCP frames in writev batches, and the sub-streams that blocked are reported
// to the engine (edgpu_fanout_blocked) so the next tick resumes where the reference would.
// Host code only: it uses the public C ABI of the engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include "edgpu.h"

namespace {

struct UdpDest {
    int fd[2] = {-1, -1};               // RTP, RTCP socket (-1: the worker's socket)
    sockaddr_in addr[2];
};

struct TcpConn {
    int fd = -1;
    std::string pending;                // RTSPResponseStream output buffer (unsent tail)
};

struct Worker {
    int udp_fd = -1;
    std::vector<edgpu_blocked> blocked;
    uint64_t udp_datagrams = 0, udp_bytes = 0, udp_dropped = 0, tcp_frames = 0, tcp_bytes = 0;
};

}  // namespace

struct edgpu_egress {
    edgpu_ctx* ctx = nullptr;
    uint32_t nthreads = 1;
    std::map<uint64_t, UdpDest> udp;    // (subscriber << 16 | track)
    std::map<uint32_t, TcpConn> tcp;    // subscriber
    uint8_t* h_arena = nullptr;
    size_t h_arena_cap = 0;
    std::vector<edgpu_out_desc> desc;
    std::vector<edgpu_substream_out> subs;
    std::vector<Worker> workers;
    std::vector<edgpu_blocked> last_blocked;
    std::string err;
};

static int eg_fail(edgpu_egress* e, int code, const std::string& m) {
    if (e) e->err = m;
    return code;
}

// One UDP sub-stream: every datagram is offered to the socket once (errors ignored, like the
// reference's (void)SendTo); EAGAIN / ENOBUFS drop the datagram.
static void send_udp(edgpu_egress* e, Worker& w, const edgpu_substream_out& s, const UdpDest& d) {
    const int k = s.kind ? 1 : 0;
    const int fd = d.fd[k] >= 0 ? d.fd[k] : w.udp_fd;
    const edgpu_out_desc* ds = e->desc.data() + s.desc_base;
    constexpr uint32_t kBatch = 256;
    mmsghdr msgs[kBatch];
    iovec iov[kBatch];
    uint32_t i = 0;
    while (i < s.desc_count) {
        const uint32_t n = std::min(kBatch, s.desc_count - i);
        for (uint32_t j = 0; j < n; j++) {
            iov[j].iov_base = e->h_arena + ds[i + j].offset;
            iov[j].iov_len = ds[i + j].len;
            memset(&msgs[j].msg_hdr, 0, sizeof(msgs[j].msg_hdr));
            msgs[j].msg_hdr.msg_name = const_cast<sockaddr_in*>(&d.addr[k]);
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

// One TCP sub-stream, RTSPResponseStream::WriteV(kAllOrNothing) frame by frame, batched: the
// buffered tail goes first; frames the socket took (the last one possibly in part, its tail
// then buffered) are sent; the first frame that gets no byte blocks the sub-stream.
static void send_tcp(edgpu_egress* e, Worker& w, uint32_t q, const edgpu_substream_out& s, TcpConn& c) {
    const edgpu_out_desc* ds = e->desc.data() + s.desc_base;
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
            iov[nv].iov_base = e->h_arena + ds[i + j].offset;
            iov[nv].iov_len = ds[i + j].len;
            total += ds[i + j].len;
            nv++;
        }
        ssize_t r = writev(c.fd, iov, (int)nv);
        if (r < 0 && errno == EINTR) continue;
        size_t wrote = r > 0 ? (size_t)r : 0;
        if (wrote < plen) {                               // the old tail is still not out
            c.pending.erase(0, wrote);
            w.blocked.push_back(edgpu_blocked{q, i});
            return;
        }
        c.pending.clear();
        wrote -= plen;
        uint32_t j = 0;
        while (j < n && wrote >= ds[i + j].len) { wrote -= ds[i + j].len; w.tcp_bytes += ds[i + j].len; j++; }
        w.tcp_frames += j;
        if (j < n && wrote > 0) {                         // partly out: counted sent, tail buffered
            const edgpu_out_desc& d = ds[i + j];
            c.pending.assign(reinterpret_cast<const char*>(e->h_arena + d.offset) + wrote, d.len - wrote);
            w.tcp_bytes += d.len;
            w.tcp_frames++;
            j++;
            i += j;
            if (i < s.desc_count) w.blocked.push_back(edgpu_blocked{q, i});
            return;
        }
        i += j;
        if (j < n || (size_t)r < total) {                 // no byte of frame i went out
            w.blocked.push_back(edgpu_blocked{q, i});
            return;
        }
    }
}

extern "C" {

int edgpu_egress_create(edgpu_ctx* ctx, uint32_t threads, edgpu_egress** out) {
    if (!ctx || !out) return EDGPU_BAD_ARGUMENT;
    edgpu_egress* e = new edgpu_egress();
    e->ctx = ctx;
    e->nthreads = std::max(1u, std::min(threads, 64u));
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

int edgpu_egress_send(edgpu_egress* e, const edgpu_fanout_result* r, edgpu_egress_stats* out) {
    if (!e || !r) return EDGPU_BAD_ARGUMENT;
    auto t0 = std::chrono::steady_clock::now();
    edgpu_tick_stats st;
    int rc = edgpu_tick_stats_get(e->ctx, &st);
    if (rc) return eg_fail(e, rc, "tick stats");
    if (st.status) return eg_fail(e, st.status, "device-side status after fan-out");
    if (st.arena_bytes > e->h_arena_cap) {
        if (e->h_arena) (void)hipHostFree(e->h_arena);
        e->h_arena = nullptr;
        const size_t cap = std::max<size_t>(st.arena_bytes, 1 << 20);
        if (hipHostMalloc((void**)&e->h_arena, cap, hipHostMallocDefault) != hipSuccess)
            return eg_fail(e, EDGPU_OUT_OF_MEMORY, "pinned arena");
        e->h_arena_cap = cap;
    }
    e->desc.resize(st.relayed_packets);
    e->subs.resize(r->n_substreams);
    if ((rc = edgpu_copy_to_host(e->ctx, e->h_arena, r->arena, st.arena_bytes)) ||
        (rc = edgpu_copy_to_host(e->ctx, e->desc.data(), r->desc, st.relayed_packets * sizeof(edgpu_out_desc))) ||
        (rc = edgpu_copy_to_host(e->ctx, e->subs.data(), r->substreams, r->n_substreams * sizeof(edgpu_substream_out))))
        return eg_fail(e, rc, "copy to host");
    auto t1 = std::chrono::steady_clock::now();
    for (Worker& w : e->workers) { w.blocked.clear(); w.udp_datagrams = w.udp_bytes = w.udp_dropped = w.tcp_frames = w.tcp_bytes = 0; }
    auto run = [&](uint32_t k) {
        Worker& w = e->workers[k];
        for (uint32_t q = 0; q < (uint32_t)e->subs.size(); q++) {
            const edgpu_substream_out& s = e->subs[q];
            if (s.desc_count == 0 || s.subscriber % e->nthreads != k) continue;
            if (s.transport == EDGPU_TRANSPORT_TCP) {
                auto it = e->tcp.find(s.subscriber);
                if (it != e->tcp.end()) send_tcp(e, w, q, s, it->second);
            } else {
                auto it = e->udp.find((uint64_t)s.subscriber << 16 | s.track);
                if (it != e->udp.end()) send_udp(e, w, s, it->second);
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
    auto t2 = std::chrono::steady_clock::now();
    std::vector<edgpu_blocked> blocked;
    edgpu_egress_stats s;
    memset(&s, 0, sizeof(s));
    for (Worker& w : e->workers) {
        blocked.insert(blocked.end(), w.blocked.begin(), w.blocked.end());
        s.udp_datagrams += w.udp_datagrams; s.udp_bytes += w.udp_bytes; s.udp_dropped += w.udp_dropped;
        s.tcp_frames += w.tcp_frames; s.tcp_bytes += w.tcp_bytes;
    }
    std::sort(blocked.begin(), blocked.end(), [](const edgpu_blocked& a, const edgpu_blocked& b) { return a.substream < b.substream; });
    s.blocked_substreams = (uint32_t)blocked.size();
    s.copy_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    s.send_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    e->last_blocked = blocked;
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

int edgpu_egress_flush(edgpu_egress* e, uint64_t* out_pending) {
    if (!e) return EDGPU_BAD_ARGUMENT;
    uint64_t left = 0;
    for (auto& kv : e->tcp) {
        TcpConn& c = kv.second;
        while (!c.pending.empty()) {
            const ssize_t r = write(c.fd, c.pending.data(), c.pending.size());
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) break;
            c.pending.erase(0, (size_t)r);
        }
        left += c.pending.size();
    }
    if (out_pending) *out_pending = left;
    return EDGPU_OK;
}

}  // extern "C"
