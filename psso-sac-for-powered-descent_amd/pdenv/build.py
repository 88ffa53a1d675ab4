"""Compile libpdenv.so for gfx950 in-tree (hipcc cross-compiles without a GPU).

The step kernel is instantiated per (precision, phase family, wind) in 12 objects from
csrc/kstep.hip, compiled in parallel with the host unit (pdenv.hip) and the PSO kernels
(pdpso.hip) and the SAC actor (pdsac.hip), then linked into one shared library.  Objects are rebuilt when any source is
newer than them."""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG, "libpdenv.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: no FMA contraction, so binary64 arithmetic follows the reference's
# (CPython/NumPy) operation-by-operation rounding.
# -disable-machine-licm: machine LICM hoists the literal constants of the inlined libm
# polynomials out of the sub-step loop into VGPRs (>60 VGPRs, a 2x occupancy loss).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
         "-Wno-unused-result", "-mllvm", "-disable-machine-licm"]
KSTEP = [(r, ph, w) for r in (0, 1) for ph in (0, 1, 2) for w in (0, 1)]


# per-unit compiler flags: the c3 unit (binary64, pure throttle, wind) is scheduled for memory
# clauses -- c3 -1.0 %, c3-descent -1.3 % against the default scheduler, two interleaved rounds
# (profiles/r05_exp_sched.jsonl; max-ilp -1.2 / -1.0 %, iterative-ilp +0.8 %, metric bias 0 +-0),
# the same registers and no scratch
KSTEP_FLAGS = {(0, 0, 1): ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]}


def units():
    """(object path, source, defines) of every translation unit."""
    u = [(os.path.join(OBJ, "pdenv.o"), "pdenv.hip", []), (os.path.join(OBJ, "pdpso.o"), "pdpso.hip", []),
         (os.path.join(OBJ, "pdsac.o"), "pdsac.hip", [])]
    for r, ph, w in KSTEP:
        u.append((os.path.join(OBJ, f"kstep_r{r}_p{ph}_w{w}.o"), "kstep.hip",
                  [f"-DPD_KR={r}", f"-DPD_KPH={ph}", f"-DPD_KW={w}"] + KSTEP_FLAGS.get((r, ph, w), [])))
    for r in (0, 1):   # the non-parity RK4 kernels (pure throttle, no wind) in units of their own
        u.append((os.path.join(OBJ, f"kstep_r{r}_rk4.o"), "kstep.hip", [f"-DPD_KR={r}", "-DPD_KPH=0", "-DPD_KW=0",
                                                                        "-DPD_KRK4=1"]))
    return [(o, os.path.join(CSRC, s), list(d)) for o, s, d in u]


def sources():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(os.path.dirname(ROOT), "include", "pdenv.h")]


def _newest_source():
    return max(os.path.getmtime(s) for s in sources())


def up_to_date():
    if not os.path.exists(OUT):
        return False
    return _newest_source() <= os.path.getmtime(OUT)


def _compile(job, verbose):
    obj, src, defs = job
    cmd = [HIPCC] + FLAGS + defs + ["-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(obj)}:\n{r.stderr}")
    return obj


def build(force=False, verbose=True, jobs=None):
    """Compile stale objects in parallel (at most `jobs`, default the CPU count capped at 16) and
    link libpdenv.so.  (Experiment builds go through build_variant, into their own directory
    and library, never into these objects.)"""
    if not force and up_to_date():
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    newest = _newest_source()
    todo = [u for u in units() if force or not os.path.exists(u[0]) or os.path.getmtime(u[0]) < newest]
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda j: _compile(j, verbose), todo))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + [u[0] for u in units()]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)


def build_variant(name, defines, unit=(0, 0, 1), patch=None, host=False):
    """Experiments: libpdenv_<name>.so with the step-kernel object of `unit` (precision, phase
    family, wind; default the c3 one) compiled with extra `defines` -- and, given `patch` (a
    unified diff against csrc/, e.g. tools/experiments/*.patch), from a patched copy of the
    sources, so that experiments stay out of the product source -- the other objects shared with
    the main build (which must be current); host=True also compiles the host unit (pdenv.hip)
    with them.  Returns the library path."""
    import shutil
    import tempfile
    build(verbose=False)
    r, ph, w = unit
    odir = os.path.join(ROOT, "build", "obj_" + name)
    os.makedirs(odir, exist_ok=True)
    obj = os.path.join(odir, f"kstep_r{r}_p{ph}_w{w}.o")
    src = os.path.join(CSRC, "kstep.hip")
    tmp = None
    if patch:
        # the copy keeps the tree shape (csrc/ next to ../../include) so that includes resolve
        tmp = tempfile.mkdtemp(prefix="pdvar_")
        shutil.copytree(CSRC, os.path.join(tmp, "p", "csrc"))
        shutil.copytree(os.path.join(os.path.dirname(ROOT), "include"), os.path.join(tmp, "include"))
        subprocess.run(["patch", "-s", "-t", "-p2", "-d", os.path.join(tmp, "p", "csrc"), "-i", os.path.abspath(patch)],
                       check=True)
        src = os.path.join(tmp, "p", "csrc", "kstep.hip")
    hobj = os.path.join(odir, "pdenv.o")
    try:
        _compile((obj, src, [f"-DPD_KR={r}", f"-DPD_KPH={ph}", f"-DPD_KW={w}"] + list(defines)), False)
        if host:
            _compile((hobj, os.path.join(os.path.dirname(src), "pdenv.hip"), list(defines)), False)
    finally:
        if tmp:
            shutil.rmtree(tmp, ignore_errors=True)
    out = os.path.join(PKG, f"libpdenv_{name}.so")
    objs = [obj if os.path.basename(u[0]) == os.path.basename(obj) else
            (hobj if host and os.path.basename(u[0]) == "pdenv.o" else u[0]) for u in units()]
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    return out
