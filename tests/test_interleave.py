"""CPU: the RTSP-interleaved '$'-deframe restatement (oracle/interleave.py) is pinned to the
reference framing code.

* tests/golden/deframe.json holds the events the REAL RTSPRequestStream::ReadRequest
  (oracle/_ref/ref_deframe, compiled from the reference sources) produced for the seeded
  connections of tests/interleave_cases.py; the restatement must reproduce them.
* Where the reference harness is present it is re-run on further random connections.

RTSP messages: the reference reports one only once its whole header has arrived (the read
index can be later than the one that brought its first byte), so for kind 2 the read index
is not compared -- the bytes consumed before it are.
"""
import hashlib
import json
import os
import random
import subprocess

import pytest

from interleave_cases import CASES, RTSP_REQ, case, _frame, _split
from oracle.interleave import FRAME, MESSAGE, deframe, read_events, write_reads

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deframe.json")
REF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "ref_deframe")


def _digest(reads):
    h = hashlib.sha256()
    for r in reads:
        h.update(len(r).to_bytes(4, "little") + r)
    return h.hexdigest()


def _summ(events):
    out = []
    for k, r, ch, a, b in events:
        out.append([k, None if k == MESSAGE else r, ch, a,
                    hashlib.sha256(b or b"").hexdigest()[:16] if k != MESSAGE else None])
    return out


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


@pytest.mark.parametrize("name", CASES)
def test_restatement_matches_reference_golden(name, gold):
    reads = case(name)
    assert _digest(reads) == gold[name]["reads_sha256"]
    want = [[k, None if k == MESSAGE else r, ch, a, None if k == MESSAGE else h]
            for k, r, ch, a, h in gold[name]["events"]]
    assert _summ(deframe(reads)) == want


def test_golden_covers_the_edges(gold):
    kinds = {name: [e[0] for e in gold[name]["events"]] for name in CASES}
    assert kinds["rtsp_tail"][-1] == MESSAGE and kinds["oversize"][-1] == 3
    assert all(k == FRAME for k in kinds["oversize_short"])
    assert max(e[3] for e in gold["max_frame"]["events"]) == 2043


def _ref(reads, tmp_path):
    i, o = tmp_path / "r.edrd", tmp_path / "e.eddf"
    write_reads(str(i), reads)
    subprocess.run([REF, str(i), str(o)], check=True)
    return read_events(str(o))


@pytest.mark.parametrize("seed", range(16))
def test_restatement_matches_live_reference(seed, tmp_path):
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/ref_deframe not built (reference tree absent)")
    rng = random.Random(seed)
    parts = []
    for _ in range(rng.randint(0, 120)):
        n = rng.choice([0, 1, 12, rng.randint(0, 1500), 2043, 2042])
        parts.append(_frame(rng.randrange(256), rng.randbytes(n) if rng.random() < 0.7 else b"$" * n))
    tail = rng.random()
    if tail < 0.25:
        parts.append(RTSP_REQ)
    elif tail < 0.5:
        parts.append(_frame(0, rng.randbytes(rng.randint(2044, 5000))))
    elif tail < 0.6:
        parts.append(_frame(0, rng.randbytes(3000))[: rng.randint(1, 2046)])
    data = b"".join(parts)
    reads = _split(rng, data, 1, rng.choice([3, 200, 4096, 70000]), zero=0.05)
    assert _summ(deframe(reads)) == _summ(_ref(reads, tmp_path))


# ---- the boundary's per-read report (oracle.interleave.ingest_reads) vs the framing ----

def _rows(reads, session=0, t0=0):
    rows, off = [], 0
    for k, r in enumerate(reads):
        rows.append((session, len(r), off, t0 + k))
        off += len(r)
    return rows, b"".join(reads)


@pytest.mark.parametrize("name", CASES)
def test_ingest_report_agrees_with_framing(name):
    from oracle.interleave import TCP_DROPPED, TCP_MESSAGE, ingest_reads
    reads = case(name)
    ev = deframe(reads)
    # one call
    rows, blob = _rows(reads)
    res, frames = ingest_reads({}, rows, blob)
    fr = [e for e in ev if e[0] == FRAME]
    assert [(f[1], f[3]) for f in frames] == [(e[2], e[4]) for e in fr]
    assert [f[2] for f in frames] == [e[1] for e in fr]             # arrival = completing read
    per_read = [0] * len(reads)
    for e in fr:
        per_read[e[1]] += 1
    assert [r[0] for r in res] == per_read
    last = ev[-1] if ev else None
    if last and last[0] == MESSAGE:
        k = next(i for i, r in enumerate(res) if r[2])
        assert res[k][2] == TCP_MESSAGE and sum(len(x) for x in reads[:k]) + res[k][1] == last[3]
    elif last and last[0] == 3:
        k = next(i for i, r in enumerate(res) if r[2])
        assert res[k][2] == TCP_DROPPED and k == last[1]
    else:
        assert not any(r[2] for r in res)
    # the same reads over several calls (device carry between them)
    rng = random.Random(name)
    carry, frames2, k = {}, [], 0
    while k < len(reads):
        m = rng.randint(1, 40)
        rows, blob = _rows(reads[k:k + m], t0=k)
        r2, f2 = ingest_reads(carry, rows, blob)
        frames2 += f2
        if any(x[2] for x in r2):
            break
        k += m
    assert [(f[1], f[3], f[2]) for f in frames2] == [(f[1], f[3], f[2]) for f in frames]


# ---- the replay's pusher model (easydarwin_amd/replay.py tcp_plan / ingest_tcp) on CPU ----

class _RestatedCtx:
    """Answers ingest_interleaved from the restatement, so the host-side replay logic
    (read splitting, carried prefixes, RTSP keep-alives) is checked without a GPU."""

    def __init__(self):
        self.carry, self.frames = {}, []

    def ingest_interleaved(self, rows, data):
        import numpy as np
        from easydarwin_amd import edgpu
        from oracle.interleave import ingest_reads
        rr = [(int(r["session"]), int(r["len"]), int(r["offset"]), int(r["arrival_ms"])) for r in rows]
        res, fr = ingest_reads(self.carry, rr, data)
        self.frames += fr
        return np.array([tuple(r) for r in res], dtype=edgpu.TCP_RESULT_DTYPE)

    def keyframe_index(self):
        pass


def _scenario_names():
    from scenarios import SCENARIOS
    return list(SCENARIOS)


@pytest.mark.parametrize("name", _scenario_names())
def test_replay_pusher_model_delivers_every_packet(name):
    from easydarwin_amd.replay import _batches, ingest_tcp, tcp_plan
    from easydarwin_amd.trace import PKT
    from scenarios import SCENARIOS
    tr = SCENARIOS[name]()
    if any(len(ev[4]) > 2043 for ev in tr.events if ev[0] == PKT):
        pytest.skip("packets above 2043 bytes cannot travel RTSP-interleaved (connection dropped)")
    batches, barriers = _batches(tr, True)
    plan = tcp_plan(batches, seed=7, barriers=barriers)
    ctx = _RestatedCtx()
    calls = 0
    for b, p in zip(batches, plan):
        ctx.frames = []
        calls += ingest_tcp(ctx, p)
        got, want = {}, {}
        for s, ch, t, data in ctx.frames:
            got.setdefault(s, []).append((ch, t, data))
        for s, ch, t, data in b:
            want.setdefault(s, []).append((ch, t, data))
        assert got == want
    assert calls >= sum(1 for b in batches if b)    # more when keep-alives were answered
    assert not any(ctx.carry.values())


@pytest.mark.parametrize("name", ["tiny", "nal", "clamp", "ssrc"])
def test_interleaved_output_parses_back_through_reference_reader(name, tmp_path):
    """The subscriber-side '$' ch BE16(len) framing of every RTSP-interleaved sub-stream in the
    committed reference captures (the engine reproduces them byte for byte) is read back by the
    reference's own RTSPRequestStream (oracle/_ref/ref_deframe): the same packets, in order, on
    the channel RTPStream assigns (2 * track + RTCP, RTPStream.cpp:472-473).  The capture's
    framing is the harness's restatement of RTSPSessionInterface::InterleavedWrite
    (RTSPSessionInterface.cpp:329-344), whose class needs the server singleton to construct;
    this pins it against compiled reference code from the other side of the wire."""
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/ref_deframe not built (reference tree absent)")
    from easydarwin_amd.trace import read_capture, split_wire_image
    gold_dir = os.path.dirname(GOLD)
    cap = read_capture(open(os.path.join(gold_dir, name + ".edcp"), "rb").read())
    rng = random.Random(name)
    checked = 0
    for (sub, track, kind), v in cap.items():
        if not v.tcp or not v.data:
            continue
        pkts = split_wire_image(v.data, 1)
        fits = []
        for p in pkts:                       # the reader's 2047-byte request buffer (QTSS.h:47)
            if len(p) + 4 > 2047:
                break
            fits.append(p)
        data = v.data[:sum(len(p) + 4 for p in fits)]
        reads = _split(rng, data, 1, 3000, zero=0.0)
        ev = _ref(reads, tmp_path)
        got = [(ch, b) for k, _r, ch, _a, b in ev if k == FRAME]
        assert got == [(2 * track + kind, p) for p in fits], (sub, track, kind)
        checked += len(fits)
    assert checked > 0
