"""Diagnostic: the reference harness on the udppush scenario, with and without the server gate,
against the committed golden summary (is the harness's UDP-push path the same on this host?)."""
import os, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from scenarios import SCENARIOS
from easydarwin_amd.trace import capture_summary, read_capture
from test_gpu_parity import _fixture

for name in ("udppush", "repush"):
    tr = SCENARIOS[name]()
    d = tempfile.mkdtemp()
    tr.write(os.path.join(d, "t.edtr"))
    gold = _fixture(name)["substreams"]
    for gate in ("0", "1"):
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness"), os.path.join(d, "t.edtr"),
                            os.path.join(d, "c.edcp")], capture_output=True, text=True,
                           env=dict(os.environ, EDTR_SERVER_GATE=gate))
        g = capture_summary(read_capture(open(os.path.join(d, "c.edcp"), "rb").read()))
        bad = [k for k in gold if g.get(k) != gold[k]]
        print(name, "gate", gate, "rc", r.returncode, "differs from golden:", len(bad),
              [(k, g.get(k, [None])[0], gold[k][0]) for k in bad[:6]], r.stderr[-300:])
