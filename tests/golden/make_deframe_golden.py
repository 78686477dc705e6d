#!/usr/bin/env python3
"""Writes tests/golden/deframe.json: the events the REAL reference framing code
(oracle/_ref/ref_deframe = RTSPRequestStream::ReadRequest compiled from the reference
sources) produces for each seeded connection in tests/interleave_cases.py.

Per case: sha256 of the reads, and per event [kind, read, channel, a, sha256(bytes)[:16]]
(kind 1 frame / 2 RTSP message / 3 connection dropped, see oracle/ref_deframe.cpp).
Run here, where /root/reference exists:  python tests/golden/make_deframe_golden.py
"""
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

from interleave_cases import CASES, case  # noqa: E402
from oracle.interleave import read_events, write_reads  # noqa: E402


def reads_digest(reads):
    h = hashlib.sha256()
    for r in reads:
        h.update(len(r).to_bytes(4, "little") + r)
    return h.hexdigest()


def ref_events(binary, reads):
    with tempfile.TemporaryDirectory() as d:
        i, o = os.path.join(d, "r.edrd"), os.path.join(d, "e.eddf")
        write_reads(i, reads)
        subprocess.run([binary, i, o], check=True)
        return read_events(o)


def summarize(events):
    return [[k, r, ch, a, hashlib.sha256(b or b"").hexdigest()[:16]] for k, r, ch, a, b in events]


def main():
    binary = os.path.join(ROOT, "oracle", "_ref", "ref_deframe")
    out = {}
    for name in CASES:
        reads = case(name)
        out[name] = {"reads_sha256": reads_digest(reads), "events": summarize(ref_events(binary, reads))}
    with open(os.path.join(HERE, "deframe.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    for name in CASES:
        ev = out[name]["events"]
        print(name, len(ev), "events; last", ev[-1][:4] if ev else None)


if __name__ == "__main__":
    main()
