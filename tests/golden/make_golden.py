"""Regenerates the golden parity fixtures in tests/golden/ from the REAL reference.

For every scenario in tests/scenarios.py:
  1. write the trace;
  2. replay it through oracle/_ref/ref_harness (EasyDarwin's reflector compiled from the
     read-only reference sources, oracle/_ref/Makefile) -> capture;
  3. replay it through oracle/relay_model (the clean-room restatement) -> capture, and
     require byte equality with (2);
  4. commit <name>.json = {trace sha256, per sub-stream [packets, bytes, sha256], sha256 of the
     QTSS_PacketStruct transmit times RTPSessionOutput::WritePacket gave every accepted write
     (EDGPU_TT_OUT, pinned for the QTSS module drop-in), the pushers' keep-alive log (the module's
     qtssCliSesTimeoutMsec settings, QTSS_RefreshTimeOut calls and the server's timeouts,
     EDGPU_KEEPALIVE_LOG) and, for ``keepalive``, the same replay with the refreshes ignored
     (EDGPU_REPLAY_NO_REFRESH: the UDP pusher times out); for the module scenarios also every RTSP
     request's route, authorization and response (EDGPU_REQ_LOG)} and, for the small scenarios, the
     trace and the reference capture themselves (<name>.edtr/.edcp).

Run here (needs /root/reference):  python tests/golden/make_golden.py
The fixtures are data only (inputs + expected outputs); nothing here is reference source.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from easydarwin_amd.trace import capture_summary, read_capture, read_source_reports  # noqa: E402
from scenarios import MODULE_SCENARIOS, SCENARIOS  # noqa: E402

FULL = {"tiny", "nal", "clamp", "ssrc"}          # small enough to commit byte for byte
KEEPALIVE = {"keepalive"}                       # the log itself and a no-refresh replay


def main():
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    port = os.path.join(ROOT, "oracle", "relay_model")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    index = {}
    with tempfile.TemporaryDirectory() as td:
        for name, fn in SCENARIOS.items():
            trace = fn().to_bytes()
            tpath = os.path.join(td, name + ".edtr")
            with open(tpath, "wb") as f:
                f.write(trace)
            rc, pc = tpath + ".ref", tpath + ".port"
            tt = tpath + ".edtt"
            ka = tpath + ".ka"
            subprocess.run([ref, tpath, rc], check=True, stderr=subprocess.DEVNULL,
                           env=dict(os.environ, EDGPU_TT_OUT=tt, EDGPU_KEEPALIVE_LOG=ka))
            subprocess.run([port, tpath, pc], check=True)
            rb, pb = open(rc, "rb").read(), open(pc, "rb").read()
            if rb != pb:
                raise SystemExit(f"{name}: port oracle disagrees with the reference")
            cap = read_capture(rb)
            fix = {
                "scenario": name,
                "trace_sha256": hashlib.sha256(trace).hexdigest(),
                "trace_bytes": len(trace),
                "capture_sha256": hashlib.sha256(rb).hexdigest(),
                "generator": "tests/scenarios.py:%s (numpy PCG64, seed base 0xEA5D)" % name,
                "source": "oracle/_ref/ref_harness (EasyDarwin reference reflector)",
                "substreams": capture_summary(cap),
                "transmit_sha256": hashlib.sha256(open(tt, "rb").read()).hexdigest(),
            }
            ka_lines = open(ka).read().splitlines()
            fix["keepalive_log_sha256"] = hashlib.sha256(open(ka, "rb").read()).hexdigest()
            if name in KEEPALIVE:
                fix["keepalive_log"] = ka_lines
                nc = tpath + ".noref"
                subprocess.run([ref, tpath, nc], check=True, stderr=subprocess.DEVNULL,
                               env=dict(os.environ, EDGPU_REPLAY_NO_REFRESH="1", EDGPU_KEEPALIVE_LOG=ka + "n"))
                nb = open(nc, "rb").read()
                fix["no_refresh"] = {"capture_sha256": hashlib.sha256(nb).hexdigest(),
                                     "substreams": capture_summary(read_capture(nb)),
                                     "keepalive_log": open(ka + "n").read().splitlines()}
            rr = read_source_reports(rb)
            if rr:                       # receiver reports to UDP pushers (EDRR trailer)
                fix["source_reports"] = [[t, s, trk, addr, port, data.hex()] for t, s, trk, addr, port, data in rr]
            with open(os.path.join(HERE, name + ".json"), "w") as f:
                json.dump(fix, f, indent=1, sort_keys=True)
            if name in FULL:
                with open(os.path.join(HERE, name + ".edtr"), "wb") as f:
                    f.write(trace)
                with open(os.path.join(HERE, name + ".edcp"), "wb") as f:
                    f.write(rb)
            index[name] = {"relayed_packets": sum(v.n_packets for v in cap.values()),
                           "substreams": len(cap)}
            print(f"{name:8s} ok  {index[name]}")
        # scenarios for the QTSS module alone (ANNOUNCE refusals, second pushers): the REFERENCE
        # QTSSReflectorModule compiled from its sources, in the fake server tools/qtss_replay
        refmod = os.path.join(ROOT, "oracle", "_ref", "libQTSSReflectorModule_ref.so")
        replay = os.path.join(ROOT, "tools", "qtss_replay")
        for name, fn in MODULE_SCENARIOS.items():
            trace = fn().to_bytes()
            tpath = os.path.join(td, name + ".edtr")
            with open(tpath, "wb") as f:
                f.write(trace)
            rc, tt, ka, rq = tpath + ".ref", tpath + ".edtt", tpath + ".ka", tpath + ".req"
            subprocess.run([replay, refmod, tpath, rc], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=dict(os.environ, EDGPU_TT_OUT=tt, EDGPU_KEEPALIVE_LOG=ka, EDGPU_REQ_LOG=rq))
            rb = open(rc, "rb").read()
            cap = read_capture(rb)
            fix = {
                "scenario": name,
                "trace_sha256": hashlib.sha256(trace).hexdigest(),
                "trace_bytes": len(trace),
                "capture_sha256": hashlib.sha256(rb).hexdigest(),
                "generator": "tests/scenarios.py:%s (numpy PCG64, seed base 0xEA5D)" % name,
                "source": "oracle/_ref/libQTSSReflectorModule_ref.so (the reference QTSSReflectorModule) "
                          "in tools/qtss_replay",
                "substreams": capture_summary(cap),
                "transmit_sha256": hashlib.sha256(open(tt, "rb").read()).hexdigest(),
                "keepalive_log_sha256": hashlib.sha256(open(ka, "rb").read()).hexdigest(),
                "keepalive_log": open(ka).read().splitlines(),
                # every RTSP request: route, authorization, response (tools/qtss_replay EDGPU_REQ_LOG)
                "request_log_sha256": hashlib.sha256(open(rq, "rb").read()).hexdigest(),
                "request_log": open(rq).read().splitlines(),
            }
            with open(os.path.join(HERE, name + ".json"), "w") as f:
                json.dump(fix, f, indent=1, sort_keys=True)
            index[name] = {"relayed_packets": sum(v.n_packets for v in cap.values()), "substreams": len(cap),
                           "module_only": True}
            print(f"{name:8s} ok  {index[name]}")
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
