"""CPU: the host-side readback plan of a fan-out tick (easydarwin_amd/csrc/tick_regions.h) --
the distinct-bytes regions the socket egress and the module adapter gather, and the parts the
adapter gathers while its write threads deliver the earlier ones -- checked on random
sub-stream tables by tests/abi/tick_regions_check.cpp (compiled here with g++)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tick_regions_and_parts(tmp_path):
    exe = tmp_path / "tick_regions_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", f"-I{ROOT}/include", f"-I{ROOT}/easydarwin_amd/csrc",
                    os.path.join(ROOT, "tests", "abi", "tick_regions_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
