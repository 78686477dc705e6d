// tests/pacing/pacing_runner.cpp -- TEST INFRASTRUCTURE: the egress's restated over-buffer window
// (easydarwin_amd/csrc/edgpu_pacing.h) over the op script oracle/ref_overbuffer.cpp reads.
#include <cstdio>
#include <cstring>
#include <memory>

#include "edgpu_pacing.h"

int main() {
    std::unique_ptr<edpace::OverbufferWindow> w;
    char op[8];
    while (scanf("%7s", op) == 1) {
        if (!strcmp(op, "N")) {
            unsigned si, ws, sa; float r;
            if (scanf("%u %u %u %f", &si, &ws, &sa, &r) != 4) return 2;
            w.reset(new edpace::OverbufferWindow(si, ws, sa, r));
        } else if (!w) {
            return 2;
        } else if (!strcmp(op, "C")) {
            long long t, n; int sz;
            if (scanf("%lld %lld %d", &t, &n, &sz) != 3) return 2;
            printf("%lld\n", (long long)w->CheckTransmitTime(t, n, sz));
        } else if (!strcmp(op, "A")) {
            int sz;
            if (scanf("%d", &sz) != 1) return 2;
            w->AddPacketToWindow(sz);
        } else if (!strcmp(op, "W")) {
            unsigned b;
            if (scanf("%u", &b) != 1) return 2;
            w->SetWindowSize(b);
        } else if (!strcmp(op, "R")) {
            w->ResetOverBufferWindow();
        } else if (!strcmp(op, "O")) {
            int on;
            if (scanf("%d", &on) != 1) return 2;
            if (on) w->TurnOnOverbuffering(); else w->TurnOffOverbuffering();
        } else {
            return 2;
        }
    }
    return 0;
}
