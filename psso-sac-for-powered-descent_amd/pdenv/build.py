"""Compile libpdenv.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRCS = [os.path.join(ROOT, "csrc", f) for f in ("pdenv.hip", "pdpso.hip")]
OUT = os.path.join(PKG, "libpdenv.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: no FMA contraction, so binary64 arithmetic follows the reference's
# (CPython/NumPy) operation-by-operation rounding.
# -disable-machine-licm: machine LICM hoists the literal constants of the inlined libm
# polynomials out of the sub-step loop into VGPRs (>60 VGPRs, a 2x occupancy loss).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wno-unused-result", "-mllvm", "-disable-machine-licm"]


def sources():
    d = os.path.join(ROOT, "csrc")
    return [os.path.join(d, f) for f in os.listdir(d)] + [os.path.join(os.path.dirname(ROOT), "include", "pdenv.h")]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + SRCS
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
