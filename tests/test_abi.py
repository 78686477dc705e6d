"""CPU: the C-ABI library loads, exports every entry point include/edgpu.h declares, and its
struct layouts agree with the ctypes / numpy mirrors.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from easydarwin_amd import edgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "edgpu.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(edgpu_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = edgpu.load()
    declared = _declared()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(edgpu.EXPORTED) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", edgpu.LIB_PATH], capture_output=True, text=True).stdout
    for s in declared:
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", edgpu.LIB_PATH],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "edgpu.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(edgpu_config), sizeof(edgpu_pkt_desc),
         sizeof(edgpu_out_desc), sizeof(edgpu_substream_out), sizeof(edgpu_fanout_result),
         sizeof(edgpu_tick_stats));
  printf("%zu %zu %zu %zu\n", offsetof(edgpu_config, video_ring_bytes), offsetof(edgpu_config, max_batch_bytes),
         offsetof(edgpu_pkt_desc, arrival_ms), offsetof(edgpu_substream_out, out_base));
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(edgpu_udp_source), offsetof(edgpu_udp_source, addr),
         offsetof(edgpu_udp_source, head), sizeof(edgpu_source_report), offsetof(edgpu_source_report, len),
         offsetof(edgpu_source_report, bytes));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    a, b, c = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")[:3]
    sizes = [int(x) for x in a.split()]
    offs = [int(x) for x in b.split()]
    assert sizes == [ctypes.sizeof(edgpu.Config), ctypes.sizeof(edgpu.PktDesc), ctypes.sizeof(edgpu.OutDesc),
                     ctypes.sizeof(edgpu.SubstreamOut), ctypes.sizeof(edgpu.FanoutResult),
                     ctypes.sizeof(edgpu.TickStats)]
    assert offs == [edgpu.Config.video_ring_bytes.offset, edgpu.Config.max_batch_bytes.offset,
                    edgpu.PktDesc.arrival_ms.offset, edgpu.SubstreamOut.out_base.offset]
    assert sizes[1] == edgpu.PKT_DTYPE.itemsize and sizes[2] == edgpu.OUT_DTYPE.itemsize
    assert sizes[3] == edgpu.SUB_DTYPE.itemsize
    u, r = edgpu.UDP_SOURCE_DTYPE, edgpu.SOURCE_REPORT_DTYPE
    assert [int(x) for x in c.split()] == [u.itemsize, u.fields["addr"][1], u.fields["head"][1],
                                           r.itemsize, r.fields["len"][1], r.fields["bytes"][1]]


def test_no_device_fails_loudly():
    """Without a visible gfx950 device the engine refuses to start (no CPU fallback)."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(edgpu.EdgpuError) as ei:
        edgpu.Context()
    assert ei.value.code == edgpu.NO_DEVICE


def test_build_batch_layout():
    pk = [(1, 0, 10, b"\x80" + bytes(30)), (0, 2, 11, b"\x80" + bytes(99)), (1, 1, 12, bytes(5))]
    desc, seg_off, seg_sess, blob = edgpu.build_batch(pk)
    assert list(seg_sess) == [0, 1] and list(seg_off) == [0, 1, 3]
    assert list(desc["len"]) == [100, 31, 5]
    assert list(desc["arrival_ms"]) == [11, 10, 12]
    for d, (_, _, _, data) in zip(desc, [pk[1], pk[0], pk[2]]):
        off = int(d["slot"]) * 16 + 4
        assert blob[off:off + len(data)].tobytes() == data
    assert np.all(desc["slot"][1:] > desc["slot"][:-1])


def test_engine_reads_back_only_through_readback():
    """every device->host copy of the engine goes through Readback (pinned
    bounce buffer for small reads, one stream synchronize before the host reads the
    destination) or the pinned RTP-Info staging -- no bare async copy into caller / stack memory."""
    src = open(os.path.join(ROOT, "easydarwin_amd", "csrc", "edgpu_engine.cpp")).read()
    body = src[src.index("struct Readback {"):]
    body = body[body.index("\n};\n") + 4:]                 # everything after the helper
    lines = [ln for ln in body.splitlines() if "DeviceToHost" in ln]
    assert lines == ["    HIP_CHECK(hipMemcpyAsync(x->h_fpi_r, x->d_fpi_r, q.size() * sizeof(FirstInfoResult), "
                     "hipMemcpyDeviceToHost, x->stream));"], lines


def test_no_stream_ordered_pool_allocations():
    """host->device copies into recycled hipMallocAsync blocks were lost on this
    stack, so the engine allocates nothing from the stream-ordered pool."""
    csrc = os.path.join(ROOT, "easydarwin_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".cpp", ".hip", ".h")):
            src = open(os.path.join(csrc, f)).read()
            assert "hipMallocAsync" not in src and "hipFreeAsync" not in src, f
