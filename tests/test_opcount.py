"""The exact algorithmic operation count (SURVEY 8(d) "ALGORITHMIC FLOPs", tools/opcount.cpp):
the step kernel's arithmetic restated over a counting scalar type.  Its binary64 instantiation
must compute the env step -- one env-step from 40 perturbed states with random float32 actions
equals the oracle's (orc_step; C_D / C_L from the oracle's exact RBF) to the per-step parity
tolerances -- and its counts must equal the committed profiles/opcount.json that bench.py's
flop_roofline reads.  No GPU needed."""
import ctypes as C
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def test_opcount_restatement_and_committed_counts(tmp_path):
    import oracle
    import opcount
    L = opcount.build(str(tmp_path))
    D = C.c_double
    L.oc_step.restype = D
    L.oc_step.argtypes = [C.c_void_p, C.POINTER(D), C.c_float, D, C.POINTER(D), C.c_int, C.POINTER(C.c_int),
                          C.POINTER(C.c_int), C.POINTER(D)]
    P = oracle.params()
    rng = np.random.default_rng(0)
    worst, wrew, wobs = np.zeros(11), 0.0, 0.0
    for t in range(40):
        s0 = np.array(P.state0[:])
        s0[4] += rng.normal(0, 0.02)
        s0[7] = s0[4] - s0[6]
        s0[1] *= rng.uniform(0.3, 1.0)
        s0[3] *= rng.uniform(0.3, 1.0)
        a = np.float32(rng.uniform(-1, 1))
        o = oracle.Oracle(phase=0, rtd=0)
        o.reset(s0)
        so, r, d, tr, tid, ob, info = o.step([a])
        s, ring, dn, tc, obs = (D * 11)(*s0), (D * 10)(), C.c_int(), C.c_int(), (D * 2)()
        rr = L.oc_step(C.byref(P), s, a, math.sqrt(s0[2] ** 2 + s0[3] ** 2), ring, 0, C.byref(dn), C.byref(tc), obs)
        worst = np.maximum(worst, np.abs(np.array(s[:]) - so) / np.maximum(np.abs(so), 1e-3))
        wrew = max(wrew, abs(rr - r))
        wobs = max(wobs, float(np.abs(np.array(obs[:]) - ob[:2]).max()))
        assert dn.value == d and tc.value == tr, t
    tol = np.full(11, 1e-10)
    tol[5] = 1e-8
    assert (worst <= tol).all(), worst
    assert wrew <= 1e-9 and wobs <= 1e-12
    got = opcount.counts(L)
    ref = json.load(open(os.path.join(REPO, "profiles", "opcount.json")))["units"]
    assert got == ref, {k: (got[k]["flops"], ref.get(k, {}).get("flops")) for k in got}
