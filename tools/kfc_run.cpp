// tools/kfc_run.cpp -- runs the op scripts of tests/golden/keyframecache_vectors.json against
// the engine's CKeyFrameCache (edgpu_reflector::CKeyFrameCache, reflector_adapter.h) and prints
// the results in the format of oracle/ref_vectors.cpp kfc, so tests/test_cold_parsers.py compares
// them with the reference's.  Host code only (no GPU).  Usage: kfc_run <script>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "reflector_adapter.h"

using edgpu_reflector::CKeyFrameCache;

static void hex(const unsigned char* p, size_t n) {
    putchar('"');
    for (size_t i = 0; i < n; i++) printf("%02x", p[i]);
    putchar('"');
}

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<unsigned char> d;
    fseek(f, 0, SEEK_END); d.resize(ftell(f)); fseek(f, 0, SEEK_SET);
    if (fread(d.data(), 1, d.size(), f) != d.size()) return 2;
    fclose(f);
    size_t p = 0;
    auto u32 = [&]() { unsigned v; memcpy(&v, &d[p], 4); p += 4; return v; };
    auto i32 = [&]() { int v; memcpy(&v, &d[p], 4); p += 4; return v; };
    const unsigned n = u32();
    CKeyFrameCache* k = nullptr;
    printf("[");
    for (unsigned c = 0; c < n; c++) {
        const unsigned code = d[p++];
        const int a = i32(), b = i32();
        const unsigned len = u32();
        std::vector<char> buf(d.begin() + p, d.begin() + p + len);
        p += len;
        printf("%s{\"op\": %u, ", c ? ",\n" : "", code);
        if (code == 0) {
            delete k;
            k = new CKeyFrameCache(a);
            printf("\"ok\": 1");
        } else if (code == 1) {
            const bool ok = k->PutOnePacket(len ? buf.data() : nullptr, (int)len, a, b);
            printf("\"ok\": %d, \"buf\": ", ok ? 1 : 0);
            hex((const unsigned char*)buf.data(), len);
        } else if (code == 2) {
            std::vector<char> out(70000, 0);
            int outLen = -1;
            const bool ok = k->GetOnePacket(out.data(), outLen, a);
            printf("\"ok\": %d, \"out\": ", ok ? 1 : 0);
            hex((const unsigned char*)out.data(), ok ? (size_t)outLen : 0);
        } else if (code == 3) {
            const bool ok = k->SetBuf(len ? buf.data() : nullptr, (int)len);
            printf("\"ok\": %d", ok ? 1 : 0);
        }
        printf(", \"curdatalen\": %d}", k ? k->curdatalen : -1);
    }
    delete k;
    printf("]\n");
    return 0;
}
