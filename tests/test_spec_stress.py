"""Refusals inside large ingest rounds (tests/scenarios.py spec_stress): k_ingest's speculative
copy copies a descriptor batch before the headers decide, so every packet the SSRC
filter empties or the SR gate refuses leaves a hole in its ring, and a stripped receive-time
trailer leaves slack.  Output bytes must not change.  CPU: the oracle restatement equals the
compiled reference on the trace (its pin).  GPU: the C ABI replay, the same pushers through the
GPU deframer (the header-first path) and the C++ adapter equal the oracle."""
import os
import subprocess

import pytest

from easydarwin_amd.trace import PKT
from scenarios import spec_stress

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADAPTER = os.path.join(ROOT, "tools", "adapter_replay")
TICKS = [1000, 100]


def _run(binary, trace_bytes, tmp_path, tag):
    t, c = tmp_path / f"{tag}.edtr", tmp_path / f"{tag}.edcp"
    t.write_bytes(trace_bytes)
    subprocess.run([binary, str(t), str(c)], check=True, stderr=subprocess.DEVNULL, timeout=300)
    return c.read_bytes()


@pytest.mark.parametrize("tick", TICKS)
def test_oracle_matches_reference_on_spec_stress(tick, oracle_bins, tmp_path):
    if oracle_bins["ref"] is None:
        pytest.skip("the reference harness is built only where /root/reference is")
    tb = spec_stress(tick).to_bytes()
    want = _run(oracle_bins["ref"], tb, tmp_path, "ref")
    assert len(want) > 1 << 20
    same = _run(oracle_bins["port"], tb, tmp_path, "port") == want     # (no pytest diff of MBs)
    assert same


@pytest.mark.gpu
@pytest.mark.parametrize("tick", TICKS)
def test_engine_matches_oracle_on_spec_stress(tick, oracle_bins, tmp_path):
    from easydarwin_amd.replay import replay
    tr = spec_stress(tick)
    tb = tr.to_bytes()
    want = _run(oracle_bins["port"], tb, tmp_path, "port")
    for spec_min in (1, 0xFFFFFFFF):     # the speculative copy on every batch / never
        cap, _ = replay(tr, ingest_spec_min=spec_min)
        same = cap == want               # (a bool: pytest would diff megabytes of bytes)
        assert same, f"C ABI replay (ingest_spec_min {spec_min:#x})"
    assert all(len(ev[4]) <= 2043 for ev in tr.events if ev[0] == PKT)
    cap, _ = replay(tr, interleaved=1)
    same = cap == want
    assert same, "interleaved push (header-first copy)"
    for spec_min in ("1", "0xFFFFFFFF"):
        t, c = tmp_path / "a.edtr", tmp_path / "a.edcp"
        t.write_bytes(tb)
        subprocess.run([ADAPTER, str(t), str(c)], check=True, stderr=subprocess.DEVNULL, timeout=300,
                       env=dict(os.environ, EDGPU_INGEST_SPEC_MIN=spec_min))
        same = c.read_bytes() == want
        assert same, f"C++ adapter (ingest_spec_min {spec_min})"
