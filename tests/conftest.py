import contextlib
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libedgpu.so")


@pytest.fixture(scope="session")
def oracle_bins():
    """Builds (here) or reuses (GPU box) the oracle binaries."""
    port = os.path.join(ROOT, "oracle", "relay_model")
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(port) or os.path.exists("/root/reference/EasyDarwin"):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    refmod = os.path.join(ROOT, "oracle", "_ref", "libQTSSReflectorModule_ref.so")
    return {"port": port, "ref": ref if os.path.exists(ref) else None,
            "refmod": refmod if os.path.exists(refmod) else None}


@contextlib.contextmanager
def udp_port_lock():
    """tools/qtss_replay binds the traces' fixed loopback source ports for UDP pushers: runs of it
    on the CPU take turns under pytest -n (one machine-wide lock file)."""
    import fcntl
    with open(os.path.join(tempfile.gettempdir(), "edgpu_udp_ports.lock"), "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        yield
