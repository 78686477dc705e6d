"""Diagnostic: prefs_buffer replayed on the owner and on a replica (all / late), EDGPU_DEBUG_PLAY on:
the RTP-Info PLAY inputs / results and the per-sub-stream capture differences."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
os.environ["EDGPU_DEBUG_PLAY"] = "1"
from scenarios import SCENARIOS
from easydarwin_amd.replay import replay
from easydarwin_amd.trace import capture_summary, read_capture
from test_gpu_parity import _fixture

tr = SCENARIOS["prefs_buffer"]()
gold = _fixture("prefs_buffer")["substreams"]
for mode in (None, "all", "late"):
    print("=== mode", mode, flush=True)
    cap, _ = replay(tr, replica=mode)
    g = capture_summary(read_capture(cap))
    bad = [k for k in gold if g.get(k) != gold[k]]
    print("mode", mode, "differs:", [(k, g.get(k, [None])[:2], gold[k][:2]) for k in bad], flush=True)
