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
for mode in (None, "all"):
    print("=== mode", mode, flush=True)
    cap, _ = replay(tr, replica=mode)
    g = capture_summary(read_capture(cap))
    bad = [k for k in gold if g.get(k) != gold[k]]
    print("mode", mode, "differs:", [(k, g.get(k, [None])[:2], gold[k][:2]) for k in bad], flush=True)

# the sequence numbers / arrival order of sub-stream 21's writes in each mode
import struct
os.environ.pop("EDGPU_DEBUG_PLAY", None)
for mode in (None, "all"):
    cap, _ = replay(tr, replica=mode)
    recs = read_capture(cap)
    for key, ss in recs.items():
        if ss.sub != 21:
            continue
        seqs, p = [], 0
        while p + 2 <= len(ss.data):
            (ln,) = struct.unpack_from(">H", ss.data, p)
            pk = ss.data[p + 2:p + 2 + ln]
            seqs.append(struct.unpack_from(">H", pk, 2)[0] if ss.kind == 0 and ln >= 4 else ln)
            p += 2 + ln
        print("mode", mode, key, len(seqs), seqs[:6], seqs[-3:], flush=True)
