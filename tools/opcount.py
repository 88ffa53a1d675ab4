#!/usr/bin/env python3
"""The exact algorithmic operation count of one env-step (tools/opcount.cpp) as
profiles/opcount.json: per unit (physics sub-step, wind, gust band, each aero query path, the
step tail) the counted +, *, /, fma, sqrt, comparisons and transcendentals, and the FLOPs (add,
sub, mul, div, sqrt 1; fma 2).  bench.py turns them into the line's flop_roofline with the
timed launches' workload counts.  Test infrastructure: builds tools/opcount.cpp against the
oracle library (the restatement's check), writes the JSON.
  python tools/opcount.py [out.json]"""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
COLS = ["add", "mul", "div", "fma", "sqrt", "cmp", "log", "exp", "sin", "cos", "atan2", "hypot", "tanh", "f32"]
ROWS = ["substep", "substep_first", "wind_profile", "gust", "q_line", "q_piece", "q_bisect", "q_payload",
        "step_tail", "atmosphere"]
TRANS = ["log", "exp", "sin", "cos", "atan2", "hypot", "tanh"]


def build(out_dir):
    import oracle
    oracle.build()
    lib = os.path.join(out_dir, "libopcount.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(REPO, "tools", "opcount.cpp"), "-I", os.path.join(REPO, "oracle"), "-o", lib,
                    os.path.join(REPO, "oracle", "build", "liborc.so")], check=True)
    return C.CDLL(lib)


def counts(L):
    import oracle
    out = (C.c_double * (len(ROWS) * len(COLS)))()
    L.oc_counts.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.oc_counts(C.byref(oracle.params()), out)
    res = {}
    for i, r in enumerate(ROWS):
        row = {c: int(out[i * len(COLS) + k]) for k, c in enumerate(COLS)}
        row["flops"] = row["add"] + row["mul"] + row["div"] + row["sqrt"] + 2 * row["fma"]
        row["transcendentals"] = sum(row[t] for t in TRANS)
        res[r] = row
    return res


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "opcount.json")
    with tempfile.TemporaryDirectory() as d:
        res = counts(build(d))
    doc = {"source": "tools/opcount.cpp (the step kernel's arithmetic restated over a counting scalar type; "
                     "checked against oracle/pd_oracle.c by tests/test_opcount.py)",
           "flop_rule": "add, sub, mul, div, sqrt = 1; fma = 2; transcendentals, comparisons and binary32 "
                        "operations apart",
           "units": res}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({k: v["flops"] for k, v in res.items()}))


if __name__ == "__main__":
    main()
