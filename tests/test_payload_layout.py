"""Host logic of the RBF payload layout (csrc/pd_common.h): the 25-slot map of a neighbourhood's
50 terms, checked exhaustively over every split of the 50 points across the five AoA columns
(tests/native/slot_map_check.cpp, compiled with hipcc for the host; no GPU needed)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "psso-sac-for-powered-descent_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_slot_map_every_column_split(tmp_path):
    exe = str(tmp_path / "slot_map_check")
    subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17", "-I", CSRC,
                    os.path.join(HERE, "native", "slot_map_check.cpp"), "-o", exe], check=True,
                   capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout and "combos 316251" in r.stdout
