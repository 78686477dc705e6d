"""tools/libudp_drain.so (the loopback UDP receivers SocketSink drains while the egress sends):
every datagram arrives, in order, framed BE16(len) + bytes.  The burst here fits the receive
buffers: this container gives its threads ~2 cores, so a receiver cannot keep pace beside a
full-speed sender here; the GPU box's egress tests (the `highrate` GOP burst) exercise that."""
import ctypes as C
import socket
import struct

from easydarwin_amd.egress import _drain


def test_drain_keeps_a_burst_in_order():
    lib = _drain()
    rx = []
    for _ in range(2):
        r = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        r.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
        r.bind(("127.0.0.1", 0))
        r.setblocking(False)
        rx.append(r)
    fds = (C.c_int * 2)(*[r.fileno() for r in rx])
    h = lib.udpd_start(fds, None, 2)
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    n = 1000
    try:
        for i in range(n):
            for r in rx:
                tx.sendto(struct.pack(">I", i) + bytes(1000 + i % 300), r.getsockname())
    finally:
        lib.udpd_stop(h)
    for i, r in enumerate(rx):
        size = lib.udpd_size(h, i)
        b = C.create_string_buffer(max(size, 1))
        lib.udpd_take(h, i, b)
        raw, o, seq = b.raw[:size], 0, []
        while o < size:
            ln = (raw[o] << 8) | raw[o + 1]
            assert ln == 4 + 1000 + len(seq) % 300
            seq.append(struct.unpack(">I", raw[o + 2:o + 6])[0])
            o += 2 + ln
        assert lib.udpd_count(h, i) == len(seq)
        assert seq == list(range(n)), f"socket {i}: {len(seq)} of {n} datagrams"
        r.close()
    lib.udpd_free(h)
    tx.close()
