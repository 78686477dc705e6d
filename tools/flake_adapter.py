#!/usr/bin/env python3
"""Runs tools/adapter_replay N times per scenario and saves any capture that differs from the
golden fixture (debugging an intermittent mismatch).  Usage: flake_adapter.py N name..."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from scenarios import SCENARIOS  # noqa: E402

n = int(sys.argv[1])
out = os.path.join(ROOT, "gpurun_out", "flake")
os.makedirs(out, exist_ok=True)
for name in sys.argv[2:]:
    fix = json.load(open(os.path.join(ROOT, "tests", "golden", name + ".json")))
    t = os.path.join(out, name + ".edtr")
    SCENARIOS[name]().write(t)
    bad = 0
    for k in range(n):
        c = os.path.join(out, f"{name}_{k}.edcp")
        subprocess.run(["timeout", "-k", "5", "60", os.path.join(ROOT, "tools", "adapter_replay"), t, c], check=True)
        h = hashlib.sha256(open(c, "rb").read()).hexdigest()
        if h == fix["capture_sha256"]:
            os.remove(c)
        else:
            bad += 1
    print(name, "mismatches", bad, "of", n, flush=True)
