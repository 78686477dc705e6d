"""CPU: the REFERENCE QTSSReflectorModule itself, hosted by the fake server.

oracle/_ref/Makefile compiles QTSSReflectorModule.cpp with everything the reflector links, from the
read-only reference sources, into a loadable QTSS module (libQTSSReflectorModule_ref.so); what the
server process gives it -- the server object's session map, the socket event set-up, the clock,
the reflect tick and UDP reads its task threads would run -- is oracle/ref_module_host.cpp.
tools/qtss_replay, the fake server the GPU drop-in is tested with (tests/test_gpu_qtss_module.py),
loads it and replays every golden trace through its roles: ANNOUNCE / SETUP / RECORD / PLAY,
RTSPIncomingData, loopback UDP pushes, ClientSessionClosing, RereadPrefs.

Its captures and transmit times must equal the golden fixtures byte for byte.  The fixtures come
from oracle/ref_harness, which restates the module's role logic around the same reference runtime;
so this pins that restatement to the module's own code, and pins the fake server's emulation of
the server (request attributes, stream dictionaries, callbacks) to what the reference module
expects of it.  The GPU drop-in, driven by the same fake server, must reproduce the same fixtures,
so the two modules agree with each other.
"""
import hashlib
import json
import os
import subprocess

import pytest

from scenarios import MODULE_SCENARIOS, SCENARIOS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REPLAY = os.path.join(ROOT, "tools", "qtss_replay")


def _fix(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def refmod(oracle_bins):
    if oracle_bins["refmod"] is None:
        pytest.skip("oracle/_ref/libQTSSReflectorModule_ref.so not built (reference tree absent)")
    if not os.path.exists(REPLAY):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "easydarwin_amd", "csrc"), REPLAY], check=True)
    return oracle_bins["refmod"]


@pytest.mark.parametrize("name", sorted(SCENARIOS) + sorted(MODULE_SCENARIOS))
def test_reference_module_reproduces_fixture(name, refmod, tmp_path):
    """Captures, transmit times and the keep-alive log (the pushers' timeouts the module set,
    its QTSS_RefreshTimeOut calls, the server's timeouts: ReflectorStream.cpp:1779-1786,
    QTSSReflectorModule.cpp:1644) as the harness restated them -- or, for the module-only
    scenarios, as this same module produced them when the fixture was made."""
    t, c, tt, ka, rq = (tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "t.edtt", tmp_path / "ka.log",
                        tmp_path / "rq.log")
    fn = SCENARIOS.get(name) or MODULE_SCENARIOS[name]
    t.write_bytes(fn().to_bytes())
    from conftest import udp_port_lock
    with udp_port_lock():                # UDP pushers bind fixed loopback source ports
        r = subprocess.run([REPLAY, refmod, str(t), str(c)], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, EDGPU_TT_OUT=str(tt), EDGPU_KEEPALIVE_LOG=str(ka), EDGPU_REQ_LOG=str(rq)))
    assert r.returncode == 0, r.stderr[-3000:]
    assert hashlib.sha256(c.read_bytes()).hexdigest() == _fix(name)["capture_sha256"]
    assert hashlib.sha256(tt.read_bytes()).hexdigest() == _fix(name)["transmit_sha256"]
    assert hashlib.sha256(ka.read_bytes()).hexdigest() == _fix(name)["keepalive_log_sha256"]
    if "request_log" in _fix(name):        # module scenarios: every request's route, authorization, response
        assert rq.read_text().splitlines() == _fix(name)["request_log"]


def test_reference_module_udp_pusher_times_out_without_refresh(refmod, tmp_path):
    """The keepalive trace with the server ignoring the module's QTSS_RefreshTimeOut calls
    (EDGPU_REPLAY_NO_REFRESH): the UDP pusher's session times out at 30 s, its players are torn
    down (kill_clients) and the session ends -- the outcome the refreshes prevent."""
    t, c, ka = tmp_path / "t.edtr", tmp_path / "c.edcp", tmp_path / "ka.log"
    t.write_bytes(SCENARIOS["keepalive"]().to_bytes())
    from conftest import udp_port_lock
    with udp_port_lock():
        r = subprocess.run([REPLAY, refmod, str(t), str(c)], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, EDGPU_REPLAY_NO_REFRESH="1", EDGPU_KEEPALIVE_LOG=str(ka)))
    assert r.returncode == 0, r.stderr[-3000:]
    fx = _fix("keepalive")
    assert hashlib.sha256(c.read_bytes()).hexdigest() == fx["no_refresh"]["capture_sha256"]
    assert ka.read_text().splitlines() == fx["no_refresh"]["keepalive_log"]
    assert "X 30000 push 0.0" in fx["no_refresh"]["keepalive_log"]
    fed, starved = fx["substreams"]["1/0/0"][0], fx["no_refresh"]["substreams"]["1/0/0"][0]
    assert starved < fed / 2


def test_reference_module_registers_its_roles(refmod):
    r = subprocess.run([REPLAY, refmod, "--register"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["module"] == "QTSSReflectorModule"
