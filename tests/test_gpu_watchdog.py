"""GPU: the watchdog (per-stream error isolation and a GPU watchdog; VERDICT r5 missing #2).

Every wait of the engine on the device is bounded by edgpu_config.watchdog_ms.  A wait that runs out
returns EDGPU_TIMEOUT and wedges the context: calls that would enqueue work or wait return
EDGPU_TIMEOUT at once, enqueueing nothing, until the work it timed out on has finished -- then the
context serves ticks as before.  The stuck work is edgpu_debug_stall: one wave that waits on the
device clock for three times the watchdog and exits."""
import hashlib
import os
import time

import pytest

from easydarwin_amd import edgpu
from easydarwin_amd.replay import replay
from easydarwin_amd.trace import Trace

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
WATCHDOG_MS = 300


def _tiny():
    with open(os.path.join(GOLD, "tiny.edtr"), "rb") as f:
        return Trace.from_bytes(f.read())


@pytest.mark.gpu
def test_watchdog_times_out_a_stuck_kernel_and_the_context_recovers():
    want = open(os.path.join(GOLD, "tiny.edcp"), "rb").read()
    with edgpu.Context(watchdog_ms=WATCHDOG_MS) as ctx:
        ctx.sync()                                   # (the context's first work: code objects loaded)
        t0 = time.monotonic()
        ctx.debug_stall(3 * WATCHDOG_MS * 1000)
        with pytest.raises(edgpu.EdgpuError) as e:
            ctx.sync()
        waited = time.monotonic() - t0
        assert e.value.code == edgpu.TIMEOUT
        assert WATCHDOG_MS / 1000 * 0.9 <= waited < 3 * WATCHDOG_MS / 1000, waited
        # wedged: every call that would enqueue work or wait is refused at once
        t1 = time.monotonic()
        for call in (ctx.sync, lambda: ctx.fanout(0)):
            with pytest.raises(edgpu.EdgpuError) as e2:
                call()
            assert e2.value.code == edgpu.TIMEOUT
        assert time.monotonic() - t1 < 0.1
        with pytest.raises(edgpu.EdgpuError) as e3:           # (reading counters waits too)
            ctx.counters()
        assert e3.value.code == edgpu.TIMEOUT
        time.sleep(3 * WATCHDOG_MS / 1000)           # the wave has exited by now
        ctx.sync()                                   # and the context is itself again
        assert ctx.counters()["watchdog_timeouts"] == 1
        cap, _ = replay(_tiny(), ctx=ctx)            # the next ticks are clean
    assert hashlib.sha256(cap).hexdigest() == hashlib.sha256(want).hexdigest()


@pytest.mark.gpu
def test_watchdog_off_waits_without_a_bound():
    """watchdog_ms = EDGPU_FALSE: the wait outlasts a stall far longer than the default would allow
    a tick (here 0.5 s) and returns normally."""
    with edgpu.Context(watchdog_ms=edgpu.FALSE) as ctx:
        ctx.sync()
        ctx.debug_stall(500_000)
        t0 = time.monotonic()
        ctx.sync()
        assert time.monotonic() - t0 >= 0.4
        assert ctx.counters()["watchdog_timeouts"] == 0
