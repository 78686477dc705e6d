/* tools/udp_drain.c -- loopback UDP receivers that drain while the egress sends (test
 * infrastructure, easydarwin_amd/egress.py SocketSink).  A tick that replays a whole GOP to a new
 * UDP player (the `highrate` golden: ~9,600 datagrams / 13.5 MB in one tick) outruns any receive
 * buffer net.core.rmem_max allows, and loopback UDP drops what does not fit, as UDP does; so each
 * receiver socket gets a thread that takes datagrams (recvmmsg) as they arrive, from before the
 * egress starts sending until after it returns.  Each socket's datagrams are kept in arrival
 * order as BE16(len) + bytes, the capture's UDP wire image (easydarwin_amd/trace.py).  A TCP
 * player's socket (stream[i] != 0: the reader end of its socketpair) is drained the same way, its
 * bytes kept as they come: a GOP replay past the socket buffer would otherwise block the egress.
 *   udpd_start(fds, stream, n) -> handle;  udpd_stop(handle) (joins, then drains what is left);
 *   udpd_size(handle, i) / udpd_count(handle, i) / udpd_take(handle, i, out): the image of fds[i],
 *   its datagram count;  udpd_free(handle). */
#define _GNU_SOURCE
#include <errno.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>

enum { kBatch = 64, kMax = 65536, kSpinMax = 16 };

typedef struct {
    int fd, stream, spin;
    uint8_t* slots;                 /* kBatch receive buffers of kMax bytes */
    uint8_t* buf;
    size_t len, cap, count;
    volatile int stop;
    pthread_t th;
} Rx;

typedef struct { Rx* rx; int n; } Drain;

static void put(Rx* r, const uint8_t* d, size_t n) {
    if (r->len + n + 2 > r->cap) {
        size_t c = r->cap ? r->cap * 2 : (1 << 20);
        while (c < r->len + n + 2) c *= 2;
        r->buf = (uint8_t*)realloc(r->buf, c);
        r->cap = c;
    }
    r->buf[r->len++] = (uint8_t)(n >> 8);
    r->buf[r->len++] = (uint8_t)n;
    memcpy(r->buf + r->len, d, n);
    r->len += n;
    r->count++;
}

static void put_raw(Rx* r, const uint8_t* d, size_t n) {
    if (r->len + n > r->cap) {
        size_t c = r->cap ? r->cap * 2 : (1 << 20);
        while (c < r->len + n) c *= 2;
        r->buf = (uint8_t*)realloc(r->buf, c);
        r->cap = c;
    }
    memcpy(r->buf + r->len, d, n);
    r->len += n;
}

/* every datagram (stream: every byte) waiting now; returns how many reads took something */
static int take(Rx* r) {
    uint8_t* bufs = r->slots;
    if (r->stream) {
        int total = 0;
        for (;;) {
            const ssize_t n = recv(r->fd, bufs, (size_t)kBatch * kMax, MSG_DONTWAIT);
            if (n <= 0) return total;
            put_raw(r, bufs, (size_t)n);
            total++;
        }
    }
    struct mmsghdr m[kBatch];
    struct iovec io[kBatch];
    int total = 0;
    for (;;) {
        for (int k = 0; k < kBatch; k++) {
            io[k].iov_base = bufs + (size_t)k * kMax;
            io[k].iov_len = kMax;
            memset(&m[k].msg_hdr, 0, sizeof(m[k].msg_hdr));
            m[k].msg_hdr.msg_iov = &io[k];
            m[k].msg_hdr.msg_iovlen = 1;
        }
        const int n = recvmmsg(r->fd, m, kBatch, MSG_DONTWAIT, NULL);
        if (n <= 0) return total;
        for (int k = 0; k < n; k++) put(r, bufs + (size_t)k * kMax, m[k].msg_len);
        total += n;
    }
}

/* Spins while datagrams keep coming and for 20 ms after the last one: a sleeping (or yielding)
 * receiver gets the CPU back later than the sender needs to fill a receive buffer clamped to
 * net.core.rmem_max (a sched_yield measured 1.6 ms beside a sending thread); then waits in poll.
 * Needs a core per receiver beside the sender's (the GPU box's CPU share has them): with more than
 * kSpinMax receivers (a fleet of slow players, e.g. the `udppush` golden's 520 sockets) every one
 * waits in poll instead. */
static void* loop(void* arg) {
    Rx* r = (Rx*)arg;
    struct pollfd p = {r->fd, POLLIN, 0};
    struct timespec last, now;
    clock_gettime(CLOCK_MONOTONIC, &last);
    while (!r->stop) {
        if (take(r) > 0) { clock_gettime(CLOCK_MONOTONIC, &last); continue; }
        if (!r->spin) { (void)poll(&p, 1, 1); continue; }
        clock_gettime(CLOCK_MONOTONIC, &now);
        const long idle_us = (now.tv_sec - last.tv_sec) * 1000000L + (now.tv_nsec - last.tv_nsec) / 1000;
        if (idle_us >= 20000) (void)poll(&p, 1, 1);
    }
    return NULL;
}

void* udpd_start(const int* fds, const int* stream, int n) {
    Drain* d = (Drain*)calloc(1, sizeof(Drain));
    d->rx = (Rx*)calloc((size_t)n, sizeof(Rx));
    d->n = n;
    for (int i = 0; i < n; i++) {
        d->rx[i].fd = fds[i];
        d->rx[i].stream = stream ? stream[i] : 0;
        d->rx[i].spin = n <= kSpinMax;
        d->rx[i].slots = (uint8_t*)malloc((size_t)kBatch * kMax);
        pthread_create(&d->rx[i].th, NULL, loop, &d->rx[i]);
    }
    return d;
}

void udpd_stop(void* h) {
    Drain* d = (Drain*)h;
    for (int i = 0; i < d->n; i++) d->rx[i].stop = 1;
    for (int i = 0; i < d->n; i++) {
        pthread_join(d->rx[i].th, NULL);
        (void)take(&d->rx[i]);
    }
}

size_t udpd_size(void* h, int i) { return ((Drain*)h)->rx[i].len; }
size_t udpd_count(void* h, int i) { return ((Drain*)h)->rx[i].count; }   /* datagrams */

void udpd_take(void* h, int i, uint8_t* out) {
    Rx* r = &((Drain*)h)->rx[i];
    if (r->len) memcpy(out, r->buf, r->len);
}

void udpd_free(void* h) {
    Drain* d = (Drain*)h;
    for (int i = 0; i < d->n; i++) { free(d->rx[i].buf); free(d->rx[i].slots); }
    free(d->rx);
    free(d);
}
