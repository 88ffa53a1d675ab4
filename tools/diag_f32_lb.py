#!/usr/bin/env python3
"""Diagnostic: the binary32 handle against the binary64 handle on the reference's recorded
landing_burn teacher-forced states (tests/golden/ref_teacher_forced.npz): one step each, the
state and every info field's worst relative difference, and the worst env's inputs."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import pdenv  # noqa: E402
from pdenv import _lib as L  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "ref_teacher_forced.npz"), allow_pickle=False)
tag = os.environ.get("TAG", "lb")
phase = "landing_burn" if tag == "lb" else "landing_burn_pure_throttle"
S0, A = d[f"{tag}_state_in"], d[f"{tag}_action"]
res = {}
outs = {}
for prec in ("f64", "f32"):
    env = pdenv.PoweredDescentEnv(len(S0), flight_phase=phase, mode="pso", precision=prec)
    env.set_state(torch.tensor(S0))
    if tag == "lb":
        env.set_actuators(torch.tensor(d["lb_prevs"]))
    *_, ex = env.step(torch.tensor(A), info=True)
    outs[prec] = (env.state.double().cpu().numpy(), {k: ex[k].double().cpu().numpy() for k in L.INFO_FIELDS})
s64, i64 = outs["f64"]
s32, i32 = outs["f32"]
ref = d[f"{tag}_state_out"]
st_err = np.abs(s32 - ref) / np.maximum(np.abs(ref), 1.0)
res["state_err_vs_ref"] = dict(zip(["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "m", "mp", "t"],
                                   st_err.max(0).tolist()))
w = int(np.argmax(st_err[:, 5]))
res["worst_env"] = w
res["worst_state_in"] = S0[w].tolist()
res["worst_action"] = np.asarray(A[w]).tolist()
res["worst_prevs"] = d["lb_prevs"][w].tolist() if tag == "lb" else None
res["info_rel_f32_vs_f64_worst_env"] = {k: [float(i32[k][w]), float(i64[k][w])] for k in L.INFO_FIELDS}
res["info_maxrel"] = {k: float(np.max(np.abs(i32[k] - i64[k]) / np.maximum(np.abs(i64[k]), 1e-3))) for k in L.INFO_FIELDS}
print(json.dumps(res, indent=0))
