"""GPU: differential parity on fresh random traces (tests/scenarios.py random_scenario: random
sessions, codecs, UDP / interleaved pushers, UDP / TCP / RTP-Info players, leaves and socket
budgets).  The oracle is the clean-room restatement, which test_random_parity.py pins to the
real reference on the same seeds; where the prebuilt reference harness travelled with the
tree it is run too (the QTSS module's transmit times).  Every path the golden scenarios take
is taken here: the C ABI replay, the same with the pushers' packets sent RTSP-interleaved
through the GPU deframer, the C++ adapter, and the QTSS module in the fake server."""
import os
import subprocess

import pytest

from easydarwin_amd.replay import replay
from easydarwin_amd.trace import PKT
from scenarios import random_scenario

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADAPTER = os.path.join(ROOT, "tools", "adapter_replay")
MODULE = os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so")
QREPLAY = os.path.join(ROOT, "tools", "qtss_replay")
SEEDS = range(24)


def _oracle(binary, trace_bytes, tmp_path, tag, env=None):
    t, c = tmp_path / f"{tag}.edtr", tmp_path / f"{tag}.edcp"
    t.write_bytes(trace_bytes)
    subprocess.run([binary, str(t), str(c)], check=True, stderr=subprocess.DEVNULL,
                   env=dict(os.environ, **(env or {})))
    return c.read_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_engine_paths_match_oracle_on_random_traces(seed, oracle_bins, tmp_path):
    tr = random_scenario(seed)
    tb = tr.to_bytes()
    want = _oracle(oracle_bins["port"], tb, tmp_path, "port")
    cap, _ = replay(tr)
    assert cap == want, "C ABI replay"
    if all(len(ev[4]) <= 2043 for ev in tr.events if ev[0] == PKT):
        cap, _ = replay(tr, interleaved=1 + seed % 2)
        assert cap == want, "interleaved push"
    t, c = tmp_path / "a.edtr", tmp_path / "a.edcp"
    t.write_bytes(tb)
    subprocess.run([ADAPTER, str(t), str(c)], check=True, timeout=120)
    assert c.read_bytes() == want, "C++ adapter"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_module_matches_reference_on_random_traces(seed, oracle_bins, tmp_path):
    """Every random trace through the QTSS module -- RTSP-interleaved pushers as RTSPIncomingData,
    UDP pushers as loopback datagrams to the socket pairs the module bound: the capture
    (receiver reports included), and (with the reference harness at hand) every write's
    transmit time."""
    tr = random_scenario(seed)
    tb = tr.to_bytes()
    want = _oracle(oracle_bins["port"], tb, tmp_path, "port")
    t, c, tt = tmp_path / "m.edtr", tmp_path / "m.edcp", tmp_path / "m.edtt"
    t.write_bytes(tb)
    r = subprocess.run([QREPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_TT_OUT=str(tt)))
    assert r.returncode == 0, r.stderr[-2000:]
    assert c.read_bytes() == want
    if oracle_bins["ref"] is not None:
        rtt = tmp_path / "r.edtt"
        _oracle(oracle_bins["ref"], tb, tmp_path, "ref", env={"EDGPU_TT_OUT": str(rtt)})
        assert tt.read_bytes() == rtt.read_bytes()


def _heavy_trace():
    """Six 8 Mb/s H.264 + AAC pushers at 1000-ms ticks: a tick's batch fills many 64-KiB slabs
    of the module's pinned blob, so its stager copies finished slabs ahead of the tick."""
    from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
    from easydarwin_amd.trace import TCP, UDP, Trace
    from scenarios import _assemble
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=8_000_000, gop=30, idr_bytes=80_000),
              TrackSpec("audio", "MPEG4-GENERIC/48000/2", 97)]
    tr = Trace()
    per = []
    for s in range(6):
        tr.add_session(make_sdp(tracks))
        per.append(session_packets(tracks, 3000, 0x5EA0 + s, t0=13 * s))
    joins = [(0, s, 10 * s + k, UDP if k < 2 else TCP) for s in range(6) for k in range(3)]
    joins += [(1500, s, 10 * s + 5, UDP) for s in range(6)]
    return _assemble(tr, per, 1000, 3000, joins)


@pytest.mark.gpu
@pytest.mark.parametrize("prestage", ["65536", "0"])
def test_module_streams_batches_ahead_of_the_tick(prestage, oracle_bins, tmp_path):
    """The module's batch copied to the device slab by slab while it fills
    (edgpu_ingest_prestage from the adapter's stager thread; EDGPU_PRESTAGE_BYTES the least it
    copies at once, 0 = the whole batch at the tick) relays the reference's bytes and transmit
    times either way."""
    tr = _heavy_trace()
    tb = tr.to_bytes()
    want = _oracle(oracle_bins["port"], tb, tmp_path, "port")
    t, c, tt = tmp_path / "m.edtr", tmp_path / "m.edcp", tmp_path / "m.edtt"
    t.write_bytes(tb)
    r = subprocess.run([QREPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_TT_OUT=str(tt), EDGPU_PRESTAGE_BYTES=prestage))
    assert r.returncode == 0, r.stderr[-2000:]
    ahead = int(r.stderr.rsplit(" bytes copied ahead", 1)[0].rsplit(" ", 1)[1])
    assert (ahead > 0) == (prestage != "0"), r.stderr[-300:]
    assert c.read_bytes() == want
    if oracle_bins["ref"] is not None:
        rtt = tmp_path / "r.edtt"
        _oracle(oracle_bins["ref"], tb, tmp_path, "ref", env={"EDGPU_TT_OUT": str(rtt)})
        assert tt.read_bytes() == rtt.read_bytes()
