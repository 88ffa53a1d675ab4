"""div_known (csrc/pd_physics.h): the step kernel's divisions by literals and per-handle constants
through correctly rounded reciprocals (Markstein's correction step) are IEEE quotients, bit for
bit, in binary64 and binary32 -- checked on the host (tests/native/markstein_check.c; the host
fma and gfx950's v_fma are both IEEE fused multiply-adds) for every divisor the kernel replaces.
No GPU needed."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PACK = os.path.join(os.path.dirname(HERE), "psso-sac-for-powered-descent_amd", "data", "param_pack.json")


def divisors():
    pk = json.load(open(PACK))
    nm = pk["norm"]
    s0 = pk["state0"]
    # literals of pd_step_impl.h (wind km, g-load window, rtd_rl reward) and the handle's
    # m_prop0, y0, m0 and observation normalisers
    lit = [1000.0, 0.1, 9.81, 10.0, 50.0, 5000.0]
    return lit + [pk["sizing"]["m_prop0"], s0[1], s0[8], nm["y"], nm["vy"], nm["x"], nm["vx"]]


def test_div_known_is_ieee_division(tmp_path):
    exe = str(tmp_path / "markstein_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(HERE, "native", "markstein_check.c"), "-o", exe,
                    "-lm"], check=True)
    r = subprocess.run([exe, "2000000"] + [repr(float(b)) for b in divisors()], capture_output=True, text=True)
    bad, tried = map(int, r.stdout.split())
    assert r.returncode == 0 and bad == 0, r.stderr[:2000]
    assert tried == 2000000 * len(divisors())
