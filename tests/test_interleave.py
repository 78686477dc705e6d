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
