"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU oracle (the
oracle is plain C; a memory error in the checker would void every parity claim built on it).

`make -C oracle sanitize` builds oracle/san_driver.c + pd_oracle.c with
-fsanitize=address,undefined (host code only); the driver reads the ctypes image of
oracle.make_params() and runs the atmosphere / aero / Philox known-answer grids, Philox
rollouts of all seven phases under every reward mode with wind, tilt and auto-reset, the
multi-threaded rollout and PSO actor rollouts.  Any sanitizer report aborts with a non-zero
exit."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no host C compiler")
def test_oracle_under_asan_ubsan(tmp_path):
    import oracle

    r = subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    p = oracle.make_params()
    img = tmp_path / "params.bin"
    img.write_bytes(ctypes.string_at(ctypes.addressof(p), ctypes.sizeof(p)))
    env = dict(os.environ)

    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:exitcode=23"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([os.path.join(ORACLE, "build", "san_driver"), str(img)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.startswith("ok "), r.stdout
