"""GPU: the QTSS reflector module as a drop-in.

tools/qtss_replay is a fake EasyDarwin server: it dlopens libQTSSReflectorModule.so, calls
QTSSReflectorModule_Main with a QTSS_PrivateArgs block and a callback table, and drives the
module through its roles -- ANNOUNCE / SETUP (record, interleaved) / RECORD for every pusher,
RTSPIncomingData for every pushed '$' frame, SETUP + PLAY for every player (UA "vlc" for an
RTP-Info player), ClientSessionClosing for a leave -- with a virtual clock and manual reflect
ticks.  The module's QTSS_Write calls on the players' RTP stream objects, framed as
RTPStream::Write frames them, must reproduce the REFERENCE reflector's per-subscriber capture
byte for byte (the golden fixtures, tests/golden/*.json), and the QTSS_PacketStruct transmit
time of every write must be the one the reference's RTPSessionOutput::WritePacket computed
(RTPSessionOutput.cpp:603-622: bucket delay, buffer delay, its reset on a blocked first-packet
pass) -- the input of the server's own thinning and over-buffer logic under QTSS_Write
(RTPStream.cpp:936-1045, 1119-1137; Q20).  UDP pushers SETUP over UDP: the module binds each
track's socket pair and answers with its port; the replay sends every UPKT datagram over
loopback from a socket bound to the trace's source port, and the receiver reports the module
sends back (eye counts included) are part of the capture (its EDRR trailer).

The session lifecycle (``repush``): pushers leaving with and without kill_clients, players
keeping a session alive, fresh sessions after the last reference went -- the replay checks the
module's reference counting at every player SETUP.  And the module's default mode
(``threaded``): its own 5-ms tick thread and UDP reader thread, two pusher threads feeding
RTSPIncomingData and loopback datagrams while the ticks run.
"""
import hashlib
import os
import subprocess

import pytest

from test_gpu_parity import _fixture, _trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODULE = os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so")
REPLAY = os.path.join(ROOT, "tools", "qtss_replay")
TCP_PUSH = ["tiny", "c1", "mixed", "clamp", "ssrc", "nal", "nokey", "stall", "anchor", "rtpinfo", "backpressure"]
UDP_PUSH = ["udppush", "leave", "repush"]   # UDP pushers (with interleaved ones beside them)
PREFS = ["prefs_buffer", "prefs_reread", "prefs_push"]   # the server's prefs objects, RereadPrefs
ACCESS = ["access"]                           # RTSPAuthorize / RTSPRoute / allow_broadcasts (module-only fixture)
KEEPALIVE = ["keepalive"]                     # 70 s: the pushers' timeouts and the module's refreshes
RETENTION = ["highrate", "longbuffer"]        # retention past the default ring capacities (ring growth)
RECEIVE_TIME = ["aktt"]                       # reflector_use_in_packet_receive_time: the "aktt" trailer


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["whole", "parts"])
@pytest.mark.parametrize("name", TCP_PUSH + UDP_PUSH + PREFS + KEEPALIVE + RETENTION + RECEIVE_TIME + ACCESS)
def test_module_matches_reference(name, gather, tmp_path):
    """`parts`: every tick's readback gathered in parts, overlapped with the write threads
    (EDGPU_GATHER_SPLIT_BYTES=0; by default only ticks of 8 MiB and more are split).  The
    keep-alive log -- the timeout set at every push SETUP, every QTSS_RefreshTimeOut, the server's
    timeouts -- is the reference's too (QTSSReflectorModule.cpp:1644, ReflectorStream.cpp:
    1779-1786).  `prefs_push`'s fixture is the reference module's own output."""
    t, c, tt, ka, rq = (tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "t.edtt", tmp_path / "ka.log",
                        tmp_path / "rq.log")
    t.write_bytes(_trace(name).to_bytes())
    env = dict(os.environ, EDGPU_TT_OUT=str(tt), EDGPU_KEEPALIVE_LOG=str(ka), EDGPU_REQ_LOG=str(rq))
    if gather == "parts":
        env["EDGPU_GATHER_SPLIT_BYTES"] = "0"
    r = subprocess.run([REPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "lost packets" not in r.stderr, r.stderr[-2000:]          # no stream error at default capacities
    if name in UDP_PUSH:                 # name the part that differs before the whole-file hash
        from easydarwin_amd.trace import capture_summary, read_capture, read_source_reports
        fx = _fixture(name)
        assert capture_summary(read_capture(c.read_bytes())) == fx["substreams"]
        assert len(read_source_reports(c.read_bytes())) == len(fx["source_reports"])
    assert hashlib.sha256(c.read_bytes()).hexdigest() == _fixture(name)["capture_sha256"]
    assert hashlib.sha256(tt.read_bytes()).hexdigest() == _fixture(name)["transmit_sha256"]
    assert hashlib.sha256(ka.read_bytes()).hexdigest() == _fixture(name)["keepalive_log_sha256"]
    if "request_log" in _fixture(name):   # the reference module's own routes, authorizations, responses
        assert rq.read_text().splitlines() == _fixture(name)["request_log"]


@pytest.mark.gpu
def test_module_udp_pusher_times_out_without_refresh(tmp_path):
    """The same 70-s trace with the server ignoring QTSS_RefreshTimeOut: the UDP pusher times out
    at 30 s and kill_clients tears its players down -- exactly as the reference does (the
    fixture's no-refresh capture and log); with the refreshes it is fed for 70 s."""
    t, c, ka = tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "ka.log"
    t.write_bytes(_trace("keepalive").to_bytes())
    r = subprocess.run([REPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, EDGPU_REPLAY_NO_REFRESH="1", EDGPU_KEEPALIVE_LOG=str(ka)))
    assert r.returncode == 0, r.stderr[-2000:]
    fx = _fixture("keepalive")["no_refresh"]
    assert ka.read_text().splitlines() == fx["keepalive_log"]
    assert hashlib.sha256(c.read_bytes()).hexdigest() == fx["capture_sha256"]


REF_MODULE = os.path.join(ROOT, "oracle", "_ref", "libQTSSReflectorModule_ref.so")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["repush", "rtpinfo", "leave", "threaded", "udppush", "prefs_reread", "backpressure",
                                  "keepalive", "prefs_push", "aktt", "access", "c1", "mixed", "nokey", "ssrc"])
@pytest.mark.parametrize("refresh", ["on", "off"])
def test_module_equals_reference_module(name, refresh, tmp_path):
    """The drop-in and the REFERENCE QTSSReflectorModule (compiled from its own sources,
    oracle/_ref/Makefile; tests/test_ref_module.py) driven by the same fake server through the same
    roles: equal QTSS_Write streams and transmit times (QTSSReflectorModule.cpp:604-678,
    1379-1545, 1597-2023, 2070-2196)."""
    if not os.path.exists(REF_MODULE):
        pytest.skip("oracle/_ref/libQTSSReflectorModule_ref.so not built")
    if refresh == "off" and name not in ("keepalive", "prefs_push", "udppush"):
        pytest.skip("no pusher outlives its timeout in this trace either way")
    t = tmp_path / "t.edtr"
    t.write_bytes(_trace(name).to_bytes())
    out = {}
    for tag, so in (("gpu", MODULE), ("ref", REF_MODULE)):
        c, tt, ka, rq = tmp_path / f"{tag}.edcp", tmp_path / f"{tag}.edtt", tmp_path / f"{tag}.ka", tmp_path / f"{tag}.rq"
        env = dict(os.environ, EDGPU_TT_OUT=str(tt), EDGPU_KEEPALIVE_LOG=str(ka), EDGPU_REQ_LOG=str(rq))
        if refresh == "off":
            env["EDGPU_REPLAY_NO_REFRESH"] = "1"
        r = subprocess.run([REPLAY, so, str(t), str(c)], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, (tag, r.stderr[-2000:])
        out[tag] = (c.read_bytes(), tt.read_bytes(), ka.read_text(), rq.read_text())
    assert out["gpu"][2] == out["ref"][2], "keep-alive logs differ"
    assert out["gpu"][3].splitlines() == out["ref"][3].splitlines(), "request logs (routes, authorizations, responses) differ"
    assert out["gpu"][0] == out["ref"][0]
    assert out["gpu"][1] == out["ref"][1]


@pytest.mark.gpu
@pytest.mark.parametrize("arrival", ["0", "1", "2"])
def test_module_threaded_default_mode_matches_reference(tmp_path, arrival):
    """Tick thread + UDP reader thread + two pusher threads: the per-sub-stream bytes (tick
    invariant for this trace) equal the reference capture's.  Transmit times and receiver-report
    times depend on when the ticks ran and are not compared.  arrival: "0" a tick every 5 ms; "1"
    and "2" (the default) the ticker reflects as soon as a packet waits, at most every 1 / 2 ms
    (EDGPU_QTSS_REFLECT_ON_ARRIVAL)."""
    from easydarwin_amd.trace import capture_summary, read_capture
    t, c = tmp_path / "t.edtr", tmp_path / "c.edcp"
    t.write_bytes(_trace("threaded").to_bytes())
    env = dict(os.environ, EDGPU_QTSS_REFLECT_ON_ARRIVAL=arrival)
    for attempt in range(2):             # the same bytes whatever the tick timing: run it twice
        r = subprocess.run([REPLAY, MODULE, str(t), str(c), "--threaded"], capture_output=True, text=True,
                           timeout=120, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        got = capture_summary(read_capture(c.read_bytes()))
        want = _fixture("threaded")["substreams"]
        assert got.keys() == want.keys()
        bad = {k: (got[k][:2], want[k][:2]) for k in want if got[k] != want[k]}
        assert not bad, f"run {attempt}: {len(bad)} sub-streams differ: {dict(list(bad.items())[:6])}"


def _watchdog_trace():
    """One RTSP-interleaved H.264 push for 4 s, ticks every 100 ms; player 1 from the start, player 2
    joining at 2.5 s (after the stall below is over)."""
    from easydarwin_amd.trace import UDP, Trace
    from scenarios import SEED_BASE, TrackSpec, _assemble, make_sdp, session_packets
    v = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=30, idr_bytes=4_000)]
    tr = Trace()
    tr.add_session(make_sdp(v))
    pk = session_packets(v, 4000, SEED_BASE + 170)
    return _assemble(tr, [pk], 100, 4000, [(0, 0, 1, UDP), (2500, 0, 2, UDP)])


@pytest.mark.gpu
def test_module_gpu_watchdog(tmp_path):
    """SURVEY §5's GPU watchdog through the module (VERDICT r5 missing #2): before its 10th tick the
    engine stream gets a wave that waits 0.9 s (EDGPU_QTSS_TEST_STALL), the watchdog is 0.3 s.  The
    tick returns the timeout; the module logs it through the server's error log, tears every player
    down (QTSS_Teardown, as kill_clients does) and answers a SETUP made meanwhile at once with 503;
    the fake server retries the tick every 50 ms; once the wave has exited the tick succeeds, the
    module logs the recovery, and a player joining later gets exactly the reference's bytes."""
    from easydarwin_amd.trace import capture_summary, read_capture
    tr = _watchdog_trace()
    t, c, el, rq = tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "err.log", tmp_path / "rq.log"
    t.write_bytes(tr.to_bytes())
    env = dict(os.environ, EDGPU_QTSS_WATCHDOG_MS="300", EDGPU_QTSS_TEST_STALL="10:900", EDGPU_REPLAY_TICK_RETRY="1",
               EDGPU_ERROR_LOG=str(el), EDGPU_REQ_LOG=str(rq))
    r = subprocess.run([REPLAY, MODULE, str(t), str(c)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    log = el.read_text()
    assert "GPU watchdog: the device did not finish a reflect tick in time" in log, log
    assert "tearing down 1 players" in log and "the device recovered" in log, log
    assert "T 900 tick failed" in log and "P probe SETUP refused in <50 ms" in log, log
    assert any(" player 999999 " in l and l.endswith("-> 503 hdr+0 close") for l in rq.read_text().splitlines())
    got = capture_summary(read_capture(c.read_bytes()))
    # the reference (the port oracle of the same trace): player 2's bytes equal; player 1 stopped at the stall
    port = os.path.join(ROOT, "oracle", "relay_model")
    ref_t, ref_c = tmp_path / "r.edtr", tmp_path / "r.edcp"
    ref_t.write_bytes(tr.to_bytes())
    subprocess.run([port, str(ref_t), str(ref_c)], check=True)
    want = capture_summary(read_capture(ref_c.read_bytes()))
    assert got["2/0/0"] == want["2/0/0"] and got["2/0/0"][0] > 0
    assert 0 < got["1/0/0"][0] < want["1/0/0"][0]
