// oracle/ref_deframe.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the
// product).  Drives the REAL RTSPRequestStream::ReadRequest (EasyDarwin Server.tproj/
// RTSPRequestStream.cpp, compiled from the read-only reference sources by oracle/_ref/Makefile)
// over one end of a socketpair, exactly as RTSPSession::Run does for a pusher's RTSP connection
// (RTSPSession.cpp:240-262, 431-433): each input read is written to the socket, then ReadRequest
// is called until it reports that it needs more data.  Every QTSS_RequestArrived that is a data
// packet is one '$' frame handed to QTSS_RTSPIncomingData_Role / ProcessRTPData
// (RTSPSession.cpp:2131-2178, QTSSReflectorModule.cpp:604-678).  The first non-data request (an
// RTSP message) or E2BIG (a frame longer than the 2 KiB request buffer, QTSS.h:47) ends the run.
//
// Usage: ref_deframe <reads.edrd> <events.eddf>
//   reads  := "EDRD" u32 n { u32 len bytes[len] }*              (one connection, in order)
//   events := "EDDF" u32 n { u8 kind u32 read u8 channel u32 a u32 blen bytes[blen] }*
//             kind 1 = frame completed by input read `read`: channel, a = payload length,
//                      bytes = payload;
//             kind 2 = RTSP message: a = stream bytes consumed before it, bytes = the request;
//             kind 3 = connection dropped (oversized frame) at read `read`: a = stream bytes
//                      consumed before the frame.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/socket.h>
#include <netinet/in.h>
#include <unistd.h>

#include "QTSS.h"
#include "TCPSocket.h"
#include "RTSPRequestStream.h"

// TCPSocket::Set (attach an accepted descriptor) is protected; TCPListenerSocket uses it the
// same way for accepted connections.
struct HarnessSocket : public TCPSocket {
    HarnessSocket() : TCPSocket(NULL, 0) {}
    void Attach(int fd, struct sockaddr_in* addr) { Set(fd, addr); }
};

struct Ev { unsigned char kind; unsigned read; unsigned char ch; std::string data; unsigned len; };

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s reads.edrd events.eddf\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    std::vector<unsigned char> d;
    fseek(f, 0, SEEK_END); d.resize(ftell(f)); fseek(f, 0, SEEK_SET);
    if (fread(d.data(), 1, d.size(), f) != d.size()) return 2;
    fclose(f);
    if (d.size() < 8 || memcmp(d.data(), "EDRD", 4) != 0) { fprintf(stderr, "bad reads\n"); return 2; }
    unsigned n; memcpy(&n, &d[4], 4);
    size_t p = 8;

    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) { perror("socketpair"); return 2; }
    int big = 1 << 22;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    fcntl(sv[1], F_SETFL, fcntl(sv[1], F_GETFL) | O_NONBLOCK);
    HarnessSocket sock;
    struct sockaddr_in peer;
    memset(&peer, 0, sizeof(peer));
    sock.Attach(sv[1], &peer);
    RTSPRequestStream stream(&sock);

    std::vector<Ev> evs;
    unsigned long consumed = 0;
    bool done = false;
    for (unsigned r = 0; r < n && !done; r++) {
        unsigned len; memcpy(&len, &d[p], 4); p += 4;
        size_t off = 0;
        while (off < len) {                                   // blocking writer end
            ssize_t w = write(sv[0], &d[p + off], len - off);
            if (w <= 0) { perror("write"); return 2; }
            off += (size_t)w;
        }
        p += len;
        while (true) {
            QTSS_Error err = stream.ReadRequest();
            if (err == QTSS_NoErr) break;                     // needs more data
            if (err == ENOTCONN || err == E2BIG) { evs.push_back({3, r, 0, std::string(), (unsigned)consumed}); done = true; break; }
            if (err != QTSS_RequestArrived) { fprintf(stderr, "ReadRequest: %d\n", (int)err); return 3; }
            StrPtrLen* req = stream.GetRequestBuffer();
            if (stream.IsDataPacket()) {
                Ev e{1, r, (unsigned char)req->Ptr[1], std::string(req->Ptr + 4, req->Len - 4), req->Len - 4};
                evs.push_back(e);
                consumed += req->Len;
            } else {
                evs.push_back({2, r, 0, std::string(req->Ptr, req->Len), (unsigned)consumed});
                done = true;
                break;
            }
        }
    }
    FILE* o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); return 2; }
    fwrite("EDDF", 1, 4, o);
    unsigned ne = (unsigned)evs.size();
    fwrite(&ne, 4, 1, o);
    for (const Ev& e : evs) {
        const unsigned blen = (unsigned)e.data.size();
        fwrite(&e.kind, 1, 1, o); fwrite(&e.read, 4, 1, o); fwrite(&e.ch, 1, 1, o);
        fwrite(&e.len, 4, 1, o); fwrite(&blen, 4, 1, o);
        fwrite(e.data.data(), 1, blen, o);
    }
    fclose(o);
    return 0;
}
