"""CPU: the QTSS module drop-in -- ABI and registration.

* include/qtss_module_abi.h restates the QTSS plugin ABI the reflector module uses; compiled
  beside the reference's own QTSS.h / QTSS_Private.h, every constant, structure size and
  field offset must match (tests/abi/qtss_abi_check.cpp, static_asserts).  Needs the
  reference tree (this container); skipped where it is absent (the GPU box).
* libQTSSReflectorModule.so exports QTSSReflectorModule_Main (the symbol the server resolves,
  QTSSReflectorModule.cpp:228-231) and, loaded by a fake server through that entry point
  (tools/qtss_replay --register), hands back a dispatch function that registers the roles
  of the relay path and names itself "QTSSReflectorModule" -- no GPU needed for Register.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
MODULE = os.path.join(ROOT, "easydarwin_amd", "libQTSSReflectorModule.so")
REPLAY = os.path.join(ROOT, "tools", "qtss_replay")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "EasyDarwin")), reason="reference headers absent")
def test_abi_matches_reference_headers():
    cmd = ["g++", "-std=gnu++11", "-w", "-fpermissive", "-fsyntax-only",
           "-DDSS_USE_API_CALLBACKS", "-D_REENTRANT", "-D__USE_POSIX", "-D__linux__",
           "-include", f"{REF}/Include/PlatformHeader.h",
           f"-I{REF}/CommonUtilitiesLib", f"-I{REF}/EasyDarwin/APIStubLib", f"-I{REF}/RTSPUtilitiesLib",
           f"-I{REF}/HTTPUtilitiesLib", f"-I{REF}/Include", f"-I{ROOT}/include",
           os.path.join(ROOT, "tests", "abi", "qtss_abi_check.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_module_exports_entry_points():
    out = subprocess.run(["nm", "-D", "--defined-only", MODULE], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert "QTSSReflectorModule_Main" in syms
    assert "EDGPU_QTSSReflectorModule_Tick" in syms


def test_module_registers_through_the_plugin_abi():
    r = subprocess.run([REPLAY, MODULE, "--register"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout)
    assert info["module"] == "QTSSReflectorModule"
    # the reference's roles (QTSSReflectorModule.cpp:268-276) but EasyCMS's Easy_GetDeviceStream
    assert info["roles"] == 8 and info["attributes"] == 8
