"""CPU: the QTSS module and its adapter under ThreadSanitizer.

tests/tsan/Makefile builds the module (qtss_reflector_module.cpp + reflector_adapter.cpp) and
the fake server (tools/qtss_replay) with LLVM's -fsanitize=thread, over a host-memory stand-in
of the engine's C ABI (tests/tsan/edgpu_cpu_stub.cpp).  The stand-in leaves the context
unlocked, so two engine calls the host did not order race in it; it also checks the pinned-batch
contracts the DMA relies on.  The runs cover every thread the module starts: its tick thread and
UDP reader (``--threaded``), the pusher threads' striped appends and blob growth, the stager's
edgpu_ingest_prestage, the gather thread and four write threads (``--bench`` with concurrent
pushes), and session teardown / prefs rereads / backpressure with manual ticks.  The relayed bytes
are the stand-in's and are not compared (the GPU tests pin them); any ThreadSanitizer report, or a
non-zero exit, fails.

The same runs also go through an AddressSanitizer + UndefinedBehaviorSanitizer build (``make
SAN=address``, leak checking on): out-of-bounds and use-after-free in the striped push path, the
pinned blob's growth, the gather parts and the teardown paths, and undefined behaviour.
"""
import os
import shutil
import subprocess

import pytest

from test_gpu_parity import _trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "tsan", "_build")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG) or not shutil.which("make"),
                                reason="LLVM clang++ (TSan runtime) not in this image")


@pytest.fixture(scope="module", params=["thread", "address"])
def tsan_build(request):
    san = request.param
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "tsan"), "-j4", f"SAN={san}"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    b = BUILD if san == "thread" else f"{BUILD}_{san}"
    return os.path.join(b, "qtss_replay"), os.path.join(b, "libQTSSReflectorModule.so")


def _run(args, env_extra, tmp_path):
    from conftest import udp_port_lock
    with udp_port_lock():                  # traces with UDP pushers bind fixed loopback source ports
        return _run_locked(args, env_extra, tmp_path)


def _run_locked(args, env_extra, tmp_path):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66 second_deadlock_stack=1",
               # (verify_asan_link_order=0: a preloaded library may come before the ASan runtime)
               ASAN_OPTIONS="detect_leaks=1 exitcode=67 verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1 halt_on_error=1", **env_extra)
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env, cwd=tmp_path)
    for tool in ("ThreadSanitizer", "AddressSanitizer", "LeakSanitizer", "runtime error:"):
        assert tool not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, r.stderr[-3000:]
    return r


@pytest.mark.parametrize("arrival", ["0", "2"])
@pytest.mark.parametrize("name", ["threaded"])
def test_tsan_threaded_default_mode(tsan_build, name, arrival, tmp_path):
    """The module's own tick thread and UDP reader, two pusher threads of the fake server: a tick
    every 5 ms, and the reflect-on-arrival ticker (woken by the pushes, at most every 2 ms)."""
    replay, module = tsan_build
    (tmp_path / "t.edtr").write_bytes(_trace(name).to_bytes())
    _run([replay, module, "t.edtr", "c.edcp", "--threaded"], {"EDGPU_QTSS_REFLECT_ON_ARRIVAL": arrival}, tmp_path)


@pytest.mark.parametrize("sessions,subs,tick_ms", [(16, 8, 20), (64, 2, 200)])
def test_tsan_concurrent_push_prestage_gather(tsan_build, sessions, subs, tick_ms, tmp_path):
    """Eight pusher threads pushing while the tick runs; the stager copying sealed slabs ahead
    (64-KiB prestage); every tick's readback gathered in parts by the gather thread while four
    write threads deliver; at 200-ms ticks a batch outgrows its 4-MiB blob (GrowBlob under every
    stripe lock while the stager holds the blob pointer)."""
    replay, module = tsan_build
    r = _run([replay, module, "--bench", str(sessions), str(subs), "2.0", str(tick_ms), "8"],
             {"EDGPU_BENCH_CONCURRENT_PUSH": "1", "EDGPU_PRESTAGE_BYTES": "65536", "EDGPU_GATHER_SPLIT_BYTES": "0",
              "EDGPU_QTSS_WRITE_THREADS": "4"}, tmp_path)
    assert '"relayed_packets": 0,' not in r.stdout
    if tick_ms == 200:
        assert '"prestaged": 0}' not in r.stdout, r.stdout


@pytest.mark.parametrize("name", ["repush", "udppush", "prefs_reread", "backpressure", "mixed"])
def test_tsan_manual_ticks(tsan_build, name, tmp_path):
    """Session teardown with and without kill_clients, UDP pushers, RereadPrefs, blocked writes:
    the tick's write threads and gather parts against the RTSP-role calls."""
    replay, module = tsan_build
    (tmp_path / "t.edtr").write_bytes(_trace(name).to_bytes())
    _run([replay, module, "t.edtr", "c.edcp"], {"EDGPU_GATHER_SPLIT_BYTES": "0", "EDGPU_QTSS_WRITE_THREADS": "4"},
         tmp_path)


@pytest.mark.parametrize("writers", ["1", "4"])
def test_tsan_rtsp_churn_during_concurrent_writes(tsan_build, writers, tmp_path):
    """The module's own ticker reflecting a real-time push load while a churn thread SETs UP, PLAYs
    and TEARs DOWN a player every 5 ms: the tick's writes run without `mu` and without the engine
    lock (SetConcurrentDelivery), so AddOutput / RemoveOutput meet the write threads, the gather
    thread and the handle table's readers; a teardown waits only for its own output's write."""
    replay, module = tsan_build
    r = _run([replay, module, "--bench", "16", "4", "2.0", "20", "2"],
             {"EDGPU_BENCH_REALTIME": "1", "EDGPU_QTSS_TICK_MSEC": "5", "EDGPU_GATHER_SPLIT_BYTES": "0",
              "EDGPU_QTSS_WRITE_THREADS": writers}, tmp_path)
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["relayed_per_s"] > 0
    assert line["rtsp_ms"]["setup_play"]["n"] > 50 and line["rtsp_ms"]["teardown"]["n"] > 50, line
