"""GPU + sockets: the engine's socket egress (edgpu_egress_*).

* Every golden scenario's ticks leave through edgpu_egress_send to loopback UDP receivers and
  RTSP-interleaved socketpairs; the capture rebuilt from the bytes the receivers read equals
  the reference reflector's capture.
* TCP backpressure over real sockets: small send buffers and readers held back for a while
  make the socket refuse writes (EAGAIN); the egress reports each blocked sub-stream to the
  engine (edgpu_fanout_blocked), and the bytes that finally arrive equal what the reference
  harness and the restatement produce when their sinks block at exactly the same writes
  (the reports replayed as BLOCK events).
"""
import hashlib
import json
import os
import subprocess

import pytest

from easydarwin_amd.replay import replay
from easydarwin_amd.trace import BLOCK, TICK, TCP, Trace, capture_summary, read_capture
from scenarios import SCENARIOS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in SCENARIOS if n not in ("backpressure", "leave")])   # scripted BLOCKs
def test_socket_egress_matches_reference(name):
    cap, _ = replay(SCENARIOS[name](), sockets={"threads": 3})
    fix = _fixture(name)
    got = capture_summary(read_capture(cap))
    bad = [k for k in fix["substreams"] if got.get(k) != fix["substreams"][k]]
    assert not bad, f"{len(bad)} sub-streams differ over sockets, e.g. {bad[:3]}"
    assert hashlib.sha256(cap).hexdigest() == fix["capture_sha256"]


def _with_blocks(tr: Trace, blocked) -> Trace:
    by_t = {}
    for t, sub, trk, kind, sent in blocked:
        by_t.setdefault(t, []).append((sub, trk, kind, sent))
    out = Trace(sdps=list(tr.sdps))
    for ev in tr.events:
        if ev[0] == TICK:
            for sub, trk, kind, sent in by_t.get(ev[1], []):
                out.events.append((BLOCK, ev[1], sub, trk, kind, sent))
        out.events.append(ev)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["stall", "anchor", "mixed"])
def test_tcp_backpressure_over_sockets(name, oracle_bins, tmp_path):
    tr = SCENARIOS[name]()
    tcp_subs = {ev[3] for ev in tr.events if ev[0] == 2 and ev[4] == TCP}
    ticks = [ev[1] for ev in tr.events if ev[0] == TICK]
    # hold every TCP reader for a stretch of ticks in the middle of the run
    lo, hi = ticks[len(ticks) // 4], ticks[len(ticks) // 2]
    hold = {t: tcp_subs for t in ticks if lo <= t < hi}
    report = []
    cap, _ = replay(tr, sockets={"threads": 2, "tcp_sndbuf": 4096, "hold": hold, "report": report})
    assert report, "no write blocked: the test did not exercise backpressure"
    tb = _with_blocks(tr, report)
    p = tmp_path / "bp.edtr"
    tb.write(str(p))
    for which in ("port", "ref"):
        exe = oracle_bins[which]
        if exe is None:
            continue
        c = tmp_path / f"{which}.edcp"
        subprocess.run([exe, str(p), str(c)], check=True, stderr=subprocess.DEVNULL)
        want = capture_summary(read_capture(c.read_bytes()))
        got = capture_summary(read_capture(cap))
        bad = [k for k in want if got.get(k) != want[k]]
        assert not bad, f"{which}: {len(bad)} sub-streams differ, e.g. {bad[:3]}"
