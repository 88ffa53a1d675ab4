"""div_known (csrc/pd_physics.h): the step kernel's divisions by literals and per-handle constants
through correctly rounded reciprocals (Markstein's correction step, with one more correction for
divisors whose reciprocal is not accurate enough for the first quotient to be faithful) are IEEE
quotients, bit for bit, in binary64 and binary32.  Checked on the host (tests/native/
markstein_check.c; the host fma and gfx950's v_fma are both IEEE fused multiply-adds):
  - the classification: a divisor takes one correction only if eps = b RN(1/b) - 1 satisfies
    |eps| <= 2^-(p+1), in exact rational arithmetic here -- then RN(a RN(1/b)) is faithful for every
    a (pd_physics.h) and Markstein's theorem gives RN(a/b); the kernel's own constexpr classifier
    (pd::one_step_ok, compiled for the host) agrees with the C one;
  - every signed binary32 mantissa of every divisor at five exponents across the domain (the
    quotient, the remainder and the corrections scale exactly by powers of two while they stay
    normal); the full 2^32-numerator sweep of the same domain (numerators and quotients 0 or of
    magnitude >= 2^-100: below, the remainder is subnormal and the theorem does not apply; no
    quantity of the step is that small) is tools/markstein_exhaustive.sh's, its output committed
    in profiles/r05_markstein_exhaustive32.txt;
  - sampled binary64 numerators (wide exponents, integers, multiples of b, near powers of two,
    quotients at the top of a binade, the physics range).
No GPU needed."""
import json
import os
import shutil
import subprocess
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PACK = os.path.join(os.path.dirname(HERE), "psso-sac-for-powered-descent_amd", "data", "param_pack.json")
CSRC = os.path.join(os.path.dirname(HERE), "psso-sac-for-powered-descent_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def divisors():
    pk = json.load(open(PACK))
    nm = pk["norm"]
    s0 = pk["state0"]
    # literals of pd_step_impl.h (wind km, g-load window, rtd_rl reward) and the handle's
    # m_prop0, y0, m0 and observation normalisers
    lit = [1000.0, 0.1, 9.81, 10.0, 50.0, 5000.0]
    return lit + [pk["sizing"]["m_prop0"], s0[1], s0[8], nm["y"], nm["vy"], nm["x"], nm["vx"]]


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("mk") / "markstein_check")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", os.path.join(HERE, "native", "markstein_check.c"),
                    "-o", path, "-lm"], check=True)
    return path


def classify(exe):
    r = subprocess.run([exe, "classify"] + [repr(float(b)) for b in divisors()], capture_output=True, text=True,
                       check=True)
    return [(float(b), int(o64), int(o32)) for b, o64, o32 in (ln.split() for ln in r.stdout.split("\n") if ln)]


def test_classification_is_sound(exe):
    """One correction only where |b RN(1/b) - 1| <= 2^-(p+1) exactly (the faithfulness bound)."""
    two = 0
    for b, o64, o32 in classify(exe):
        e64 = Fraction(b) * Fraction(1.0 / b) - 1
        bf = np.float32(b)
        e32 = Fraction(float(bf)) * Fraction(float(np.float32(1) / bf)) - 1
        if o64:
            assert abs(e64) <= Fraction(1, 2 ** 54), b
        if o32:
            assert abs(e32) <= Fraction(1, 2 ** 25), b
        two += (1 - o64) + (1 - o32)
    assert two > 0          # (the parameter pack has divisors that need the second correction)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_kernel_classifier_matches(exe, tmp_path):
    """pd::one_step_ok (Dekker's product, the compile-time / pd_create classifier) gives the C
    check's (exact fma) classification for every divisor."""
    kx = str(tmp_path / "one_step_check")
    subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "native", "one_step_check.cpp"), "-o", kx], check=True, capture_output=True,
                   timeout=300)
    r = subprocess.run([kx] + [repr(float(b)) for b in divisors()], capture_output=True, text=True, check=True)
    mine = [(float(b), int(o64), int(o32)) for b, o64, o32 in (ln.split() for ln in r.stdout.split("\n") if ln)]
    assert mine == classify(exe)


def test_div_known_every_binary32_mantissa(exe):
    r = subprocess.run([exe, "mantissas32"] + [repr(float(b)) for b in divisors()], capture_output=True, text=True,
                       timeout=600, env={**os.environ, "OMP_NUM_THREADS": str(min(8, os.cpu_count() or 1))})
    bad, tried = map(int, r.stdout.split())
    assert r.returncode == 0 and bad == 0, r.stderr[:2000]
    assert tried > 0.75 * 5 * 2 ** 24 * len(divisors())


def test_exhaustive_record():
    """The committed full sweep (every binary32 numerator of the domain, every divisor) found no
    mismatch."""
    rec = os.path.join(os.path.dirname(HERE), "profiles", "r05_markstein_exhaustive32.txt")
    bad, tried = map(int, open(rec).read().split()[-2:])
    assert bad == 0 and tried > 0.8 * 2 ** 32 * len(divisors())   # (the domain: ~85 % of the patterns)


def test_div_known_sampled_binary64(exe):
    r = subprocess.run([exe, "sample", "2000000"] + [repr(float(b)) for b in divisors()], capture_output=True,
                       text=True)
    bad, tried = map(int, r.stdout.split())
    assert r.returncode == 0 and bad == 0, r.stderr[:2000]
    assert tried == 2000000 * len(divisors())
