// oracle/ref_vectors.cpp -- TEST INFRASTRUCTURE ONLY.  Runs two cold-path parsers of the
// REAL reference, compiled from the read-only sources by oracle/_ref/Makefile, over input
// cases and prints their results as JSON, for the golden vectors in tests/golden/
// (tests/golden/make_vectors.py):
//
//   ref_vectors sdp <cases>   SDPSourceInfo::Parse (APICommonCode/SDPSourceInfo.cpp:172-420) on
//                             each SDP; per stream: payload type (video 1 / audio 2 / else 0),
//                             payload name (the rtpmap text the H.264 keyframe gate compares,
//                             ReflectorStream.cpp:1879), trackID, port, RTP/AVP/TCP flag
//   ref_vectors kfc <script>  CKeyFrameCache (CommonUtilitiesLib/keyframecache.cpp:6-118) driven
//                             by an op script; per op its result, the caller's buffer after the
//                             call (PutOnePacket rewrites buf[13]), and curdatalen
//
// Case file: u32 count, then per case u32 len + bytes.  Script: u32 count, then per op
// u8 code (0 new(len=a), 1 put(nalutype=a, start=b, bytes), 2 get(offset=a),
// 3 setbuf(bytes)) i32 a i32 b u32 len bytes.  Run it in a scratch directory: PutOnePacket
// appends to ./data.264.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "SDPSourceInfo.h"
#include "keyframecache.h"
#include "MyAssert.h"

struct NoopAssert : public AssertLogger {
    void LogAssert(char*) override {}
};

static std::vector<unsigned char> slurp(const char* path) {
    std::vector<unsigned char> d;
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    fseek(f, 0, SEEK_END); d.resize(ftell(f)); fseek(f, 0, SEEK_SET);
    if (fread(d.data(), 1, d.size(), f) != d.size()) exit(2);
    fclose(f);
    return d;
}

static FILE* J = nullptr;             // the JSON output: the reference prints diagnostics to stdout

static void hex(const unsigned char* p, size_t n) {
    fputc('"', J);
    for (size_t i = 0; i < n; i++) fprintf(J, "%02x", p[i]);
    fputc('"', J);
}

int main(int argc, char** argv) {
    static NoopAssert logger;
    SetAssertLogger(&logger);
    J = fdopen(dup(1), "w");
    if (!J || !freopen("/dev/null", "w", stdout)) return 2;
    if (argc != 3) { fprintf(stderr, "usage: %s sdp|kfc <file>\n", argv[0]); return 2; }
    std::vector<unsigned char> d = slurp(argv[2]);
    size_t p = 0;
    auto u32 = [&]() { unsigned v; memcpy(&v, &d[p], 4); p += 4; return v; };
    auto i32 = [&]() { int v; memcpy(&v, &d[p], 4); p += 4; return v; };
    const unsigned n = u32();
    fprintf(J, "[");
    if (strcmp(argv[1], "sdp") == 0) {
        for (unsigned c = 0; c < n; c++) {
            const unsigned len = u32();
            std::vector<char> sdp(d.begin() + p, d.begin() + p + len);
            p += len;
            SDPSourceInfo info(sdp.data(), len);
            fprintf(J, "%s[", c ? ",\n" : "");
            for (UInt32 s = 0; s < info.GetNumStreams(); s++) {
                SourceInfo::StreamInfo* si = info.GetStreamInfo(s);
                fprintf(J, "%s{\"type\": %u, \"name\": ", s ? ", " : "", (unsigned)si->fPayloadType);
                hex((const unsigned char*)si->fPayloadName.Ptr, si->fPayloadName.Ptr ? si->fPayloadName.Len : 0);
                fprintf(J, ", \"track_id\": %u, \"port\": %u, \"tcp\": %d}", (unsigned)si->fTrackID, (unsigned)si->fPort,
                       si->fIsTCP ? 1 : 0);
            }
            fprintf(J, "]");
        }
    } else if (strcmp(argv[1], "kfc") == 0) {
        CKeyFrameCache* k = nullptr;
        for (unsigned c = 0; c < n; c++) {
            const unsigned code = d[p++];
            const int a = i32(), b = i32();
            const unsigned len = u32();
            std::vector<char> buf(d.begin() + p, d.begin() + p + len);
            p += len;
            fprintf(J, "%s{\"op\": %u, ", c ? ",\n" : "", code);
            if (code == 0) {
                delete k;
                k = new CKeyFrameCache(a);
                fprintf(J, "\"ok\": 1");
            } else if (code == 1) {
                const bool ok = k->PutOnePacket(len ? buf.data() : nullptr, (int)len, a, b);
                fprintf(J, "\"ok\": %d, \"buf\": ", ok ? 1 : 0);
                hex((const unsigned char*)buf.data(), len);
            } else if (code == 2) {
                std::vector<char> out(70000, 0);
                int outLen = -1;
                const bool ok = k->GetOnePacket(out.data(), outLen, a);
                fprintf(J, "\"ok\": %d, \"out\": ", ok ? 1 : 0);
                hex((const unsigned char*)out.data(), ok ? (size_t)outLen : 0);
            } else if (code == 3) {
                const bool ok = k->SetBuf(len ? buf.data() : nullptr, (int)len);
                fprintf(J, "\"ok\": %d", ok ? 1 : 0);
            }
            fprintf(J, ", \"curdatalen\": %d}", k ? k->curdatalen : -1);
        }
        delete k;
    } else {
        return 2;
    }
    fprintf(J, "]\n");
    return 0;
}
