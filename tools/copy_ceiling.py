#!/usr/bin/env python3
"""Device-to-device copy and fill ceilings on this GPU (the ingest's bound: k_ingest reads each
packet once and writes its slot once).  torch's copy_ / zero_ on 16-B-aligned buffers of the
C2 ingest's size, timed with HIP events over repeated launches; prints one JSON line."""
import json
import torch

dev = torch.device("cuda", 0)
out = {}
for mb in (512, 1024):
    n = mb << 20
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    a.random_(0, 255)
    for name, fn, traffic in (("copy", lambda: b.copy_(a), 2 * n), ("fill", lambda: b.zero_(), n)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[f"{name}_{mb}MiB"] = {"ms": round(ms, 4), "GBps": round(traffic / ms / 1e6, 1)}
print(json.dumps(out))
