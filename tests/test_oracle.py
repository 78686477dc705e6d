"""CPU: the oracle is pinned to the reference.

* The committed golden fixtures were produced by the REAL reference reflector
  (oracle/_ref/ref_harness, compiled from the read-only reference sources); the clean-room
  restatement (oracle/relay_model) must reproduce them byte for byte.
* Where the reference harness is available (this container, or a GPU box that received the
  prebuilt binary) it is re-run and compared too.
"""
import hashlib
import json
import os
import subprocess

import pytest

from easydarwin_amd.trace import capture_summary, read_capture
from scenarios import SCENARIOS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FULL = ["tiny", "nal", "clamp", "ssrc"]


def _fix(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def _run(binary, trace_bytes, tmp_path, tag):
    t = tmp_path / f"{tag}.edtr"
    c = tmp_path / f"{tag}.edcp"
    t.write_bytes(trace_bytes)
    subprocess.run([binary, str(t), str(c)], check=True, stderr=subprocess.DEVNULL)
    return c.read_bytes()


@pytest.mark.parametrize("name", FULL)
def test_port_matches_committed_reference_capture(name, oracle_bins, tmp_path):
    trace = open(os.path.join(GOLD, name + ".edtr"), "rb").read()
    want = open(os.path.join(GOLD, name + ".edcp"), "rb").read()
    got = _run(oracle_bins["port"], trace, tmp_path, name)
    assert got == want


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_generator_reproduces_golden_trace(name):
    tr = SCENARIOS[name]()
    assert hashlib.sha256(tr.to_bytes()).hexdigest() == _fix(name)["trace_sha256"]


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_port_matches_golden_digests(name, oracle_bins, tmp_path):
    cap = _run(oracle_bins["port"], SCENARIOS[name]().to_bytes(), tmp_path, name)
    fix = _fix(name)
    assert capture_summary(read_capture(cap)) == fix["substreams"]
    assert hashlib.sha256(cap).hexdigest() == fix["capture_sha256"]


@pytest.mark.parametrize("name", ["tiny", "nal", "ssrc", "anchor", "rtpinfo", "backpressure", "udppush", "leave",
                                  "prefs_buffer", "prefs_reread"])
def test_reference_harness_reproduces_fixture(name, oracle_bins, tmp_path):
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built (reference tree absent)")
    tt = tmp_path / f"{name}.edtt"
    os.environ["EDGPU_TT_OUT"] = str(tt)
    try:
        cap = _run(oracle_bins["ref"], SCENARIOS[name]().to_bytes(), tmp_path, name)
    finally:
        del os.environ["EDGPU_TT_OUT"]
    assert hashlib.sha256(cap).hexdigest() == _fix(name)["capture_sha256"]
    assert hashlib.sha256(tt.read_bytes()).hexdigest() == _fix(name)["transmit_sha256"]


def test_key_pointer_skips_sps_pps_on_join():
    """Q4/Q7: a subscriber that joins at t=0 starts at the IDR's first FU-A fragment; the SPS
    and PPS packets that precede it are not replayed (c1 fixture, reference output)."""
    fix = _fix("c1")
    tr = SCENARIOS["c1"]()
    pushed = sum(1 for e in tr.events if e[0] == 1)
    n_sub1 = fix["substreams"]["1/0/0"][0]
    assert n_sub1 == pushed - 2


def test_golden_index_counts():
    idx = json.load(open(os.path.join(GOLD, "index.json")))
    for name in SCENARIOS:
        fix = _fix(name)
        assert idx[name]["relayed_packets"] == sum(v[0] for v in fix["substreams"].values())


def test_rtp_info_players_start_later_and_deferred_plays_drop():
    """Q10 from the reference's own output (rtpinfo fixture): an RTP-Info player (UA vlc)
    joining mid-GOP starts at the packet ~500 ms back (GetFirstPacketInfo) rather than at the
    key pointer a plain player starts from; PLAYs with nothing buffered (before the first
    packet, during a stall) never become subscribers."""
    sub = _fix("rtpinfo")["substreams"]
    subs = {int(k.split("/")[0]) for k in sub}
    assert not subs & {10, 13, 14}
    assert {1, 2, 3, 4, 5, 6, 11, 12, 15, 20, 21, 22, 23} <= subs
    assert sub["3/0/0"][0] < sub["4/0/0"][0]          # same join tick, vlc vs plain (video)
    assert sub["3/1/0"][0] < sub["4/1/0"][0]          # and the audio anchor start
    assert sub["1/0/0"][0] == sub["2/0/0"][0]          # at the first packets both see everything


def test_udppush_reports_pin_reference_quirks():
    """The reference's receiver reports to UDP pushers (fixture from the real reflector):
    the 5-s timer, the NAT_WORKAROUND address moves, the SR-only gate and the eye-count
    masking all show in the committed reports."""
    rr = _fix("udppush")["source_reports"]
    by = {(t, s, trk): (addr, port, bytes.fromhex(h)) for t, s, trk, addr, port, h in rr}
    assert sorted({t for t, *_ in rr}) == [5100, 10200, 15300]      # now > last + 5000
    assert not any(s == 2 for _, s, *_ in rr)                       # TCP push: no address
    assert (5100, 1, 0) not in by and (10200, 1, 0) in by           # timer ran before the 1st packet
    src0 = 10 << 24 | 5
    assert by[(5100, 0, 0)][:2] == (src0, 6001)                     # even RTP port + 1
    assert by[(10200, 0, 0)][:2] == (src0, 7001)                    # SRs moved it (NAT)
    assert by[(15300, 0, 0)][:2] == (src0, 8001)                    # foreign-SSRC SR still moves it
    assert by[(10200, 1, 0)][1] == 5001                             # odd RTP port: no + 1
    eye = lambda b: int.from_bytes(b[-12:-8], "big")               # noqa: E731
    assert [eye(by[(t, 0, 0)][2]) for t in (5100, 10200, 15300)] == [2, 3, 3]
    assert eye(by[(5100, 3, 0)][2]) == 130 & ~0x80                  # htonl(n) & 0x7fffffff on LE
    b = by[(5100, 0, 0)][2]
    assert b[:4] == bytes.fromhex("80c90001") and b[16:24] == b"\x01\x05QTSS0\x00"
    assert len(b) == 16 + 36 + 12


def test_reference_bench_modes_relay_the_same_packets(oracle_bins, tmp_path):
    """bench.py's CPU baselines: --bench (memcpy sinks) and --bench-udp (one sendto() per
    subscriber packet to loopback) replay the same trace and relay the same packets."""
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built (reference tree absent)")
    t = tmp_path / "mixed.edtr"
    t.write_bytes(SCENARIOS["mixed"]().to_bytes())
    out = {}
    for mode in ("--bench", "--bench-udp"):
        r = subprocess.run([oracle_bins["ref"], mode, str(t), "2"], check=True, capture_output=True, text=True)
        out[mode] = json.loads(r.stdout)
    assert out["--bench"]["relayed_packets"] > 0
    for k in ("relayed_packets", "relayed_bytes", "repeat"):
        assert out["--bench"][k] == out["--bench-udp"][k]
