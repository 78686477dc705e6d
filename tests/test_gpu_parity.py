"""GPU parity: the HIP engine (through the C ABI) must reproduce the reference reflector's
per-subscriber output byte for byte on every golden scenario."""
import hashlib
import json
import os

import pytest

from easydarwin_amd.replay import replay
from easydarwin_amd.trace import Trace, capture_summary, read_capture
from scenarios import MODULE_SCENARIOS, SCENARIOS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def _trace(name):
    p = os.path.join(GOLD, name + ".edtr")
    if os.path.exists(p):
        with open(p, "rb") as f:
            return Trace.from_bytes(f.read())
    tr = SCENARIOS[name]() if name in SCENARIOS else MODULE_SCENARIOS[name]()
    assert hashlib.sha256(tr.to_bytes()).hexdigest() == _fixture(name)["trace_sha256"], \
        "trace generator drifted from the golden fixture"
    return tr


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_engine_matches_reference(name):
    tr = _trace(name)
    cap, stats = replay(tr)
    fix = _fixture(name)
    got = capture_summary(read_capture(cap))
    want = fix["substreams"]
    assert got.keys() == want.keys()
    bad = [k for k in want if got[k] != want[k]]
    assert not bad, f"{len(bad)} sub-streams differ, e.g. {bad[:3]}"
    assert hashlib.sha256(cap).hexdigest() == fix["capture_sha256"]
    full = os.path.join(GOLD, name + ".edcp")
    if os.path.exists(full):
        with open(full, "rb") as f:
            assert cap == f.read()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mixed", "c1", "backpressure", "rtpinfo", "leave", "repush"])
def test_pinned_host_ingest_matches_reference(name):
    """Batches written into pinned host buffers (edgpu_host_alloc, two sets alternating) and
    ingested asynchronously (EDGPU_PTR_PINNED: copy stream + event) give the reference bytes."""
    cap, _ = replay(_trace(name), pinned=True)
    assert hashlib.sha256(cap).hexdigest() == _fixture(name)["capture_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_speculative_ingest_matches_reference(name):
    """Every golden with k_ingest's speculative copy forced on every descriptor batch
    (edgpu_config.ingest_spec_min = 1; by default only 1-s-sized batches take it):
    refused, emptied and trailer-stripped packets change no output byte."""
    cap, _ = replay(_trace(name), ingest_spec_min=1)
    assert hashlib.sha256(cap).hexdigest() == _fixture(name)["capture_sha256"]
