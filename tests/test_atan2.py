"""atan2_fd (csrc/pd_common.h), the step kernel's flight-path angle gamma = atan2(vy, vx)
(rockets_physics.py:631): within 1 ulp of glibc's atan2 -- what the reference's math.atan2 calls
-- over 4e6 arguments (tests/native/atan2_check.cpp, compiled for the host; the function is
IEEE-only, so the device gives the same bits: tools/atan2_gpu_check.hip checks that on the
GPU).  No GPU needed."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "psso-sac-for-powered-descent_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_atan2_fd_within_one_ulp_of_glibc(tmp_path):
    exe = str(tmp_path / "atan2_check")
    subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "native", "atan2_check.cpp"), "-o", exe], check=True, capture_output=True,
                   timeout=300)
    r = subprocess.run([exe, "1000000"], capture_output=True, text=True, timeout=120)
    m = re.search(r"total (\d+) differ (\d+) worst_ulp (\d+)", r.stdout)
    assert r.returncode == 0 and m, r.stdout + r.stderr
    total, differ, worst = map(int, m.groups())
    assert total == 4000000 and worst <= 1
    assert differ / total < 0.02          # correctly rounded in > 98 % of the arguments
