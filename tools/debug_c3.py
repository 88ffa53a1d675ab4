"""GPU diagnostic: follow a few envs of the c3 stochastic workload (Philox wind + tilt) step by step
against the oracle and report the first divergence (step, channel) per env.  Usage on the box:
python tools/debug_c3.py"""
import ctypes as C
import math
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
import pdenv  # noqa: E402

ST = ["x", "y", "vx", "vy", "th", "thd", "ga", "al", "m", "mp", "t"]


def run(tag, n, T, seed, stoch, tilt, fixed, fused=False):
    L = oracle.lib()
    P = oracle.params()
    env = pdenv.PoweredDescentEnv(n, flight_phase="landing_burn_pure_throttle", mode="rl", enable_wind=True,
                                  stochastic_wind=stoch, wind_percentile=None if fixed < 0 else fixed + 50,
                                  auto_reset=True, tilt_sigma_rad=tilt, seed=seed)
    A = (torch.rand(T, n, 1, generator=torch.Generator().manual_seed(seed)) * 2 - 1).contiguous()
    Es = [oracle.OrcEnv() for _ in range(n)]
    eps = [0] * n
    for i in range(n):
        L.orc_reset_philox(C.byref(P), C.byref(Es[i]), 0, seed, i, 0, 1, int(stoch), fixed, tilt)
    f, s, pr = env.wind_state()
    S = env.state.cpu().numpy()
    for i in range(n):
        E = Es[i]
        d = dict(state=np.abs(S[i] - np.array(E.s[:])).max(), su=float(s[i, 0]) - E.sigma_u,
                 sv=float(s[i, 1]) - E.sigma_v, prof=int(pr[i]) - 50 - E.wind_prof)
        if any(abs(v) > 0 for v in d.values()):
            print(f"[{tag}] env {i} reset mismatch {d}", flush=True)
    first = {}
    if fused:
        env.step_n(A.cuda())
        Sg = None
    o = oracle.OrcOut()
    for t in range(T):
        if not fused:
            _, rew, dn, tr, ex = env.step(A[t].cuda())
            Sg = env.state.cpu().numpy()
            fg = env.wind_state()[0].cpu().numpy()
        for i in range(n):
            u = (C.c_double * 4)(float(A[t, i, 0]), 0, 0, 0)
            L.orc_step(C.byref(P), C.byref(Es[i]), 0, 0, u, 1, None, C.byref(o))
            so = np.array(Es[i].s[:])
            fo = np.array([Es[i].fu[0], Es[i].fu[1], Es[i].fv[0], Es[i].fv[1]])
            ended = o.done or o.trunc
            if not fused and i not in first:
                err = np.abs(Sg[i] - so) / np.maximum(np.abs(so), 1e-3)
                ferr = np.abs(fg[i] - fo).max() if not ended else 0.0
                if err.max() > 1e-9 or ferr > 1e-12 or bool(dn[i]) != bool(o.done) or bool(tr[i]) != bool(o.trunc):
                    k = int(err.argmax())
                    first[i] = t
                    print(f"[{tag}] env {i} diverges at step {t}: {ST[k]} gpu {Sg[i][k]!r} orc {so[k]!r} rel {err[k]:.2e};"
                          f" filt err {ferr:.2e}; done {bool(dn[i])}/{o.done} trunc {bool(tr[i])}/{o.trunc}"
                          f" rew {float(rew[i])!r}/{o.reward!r}; orc ep {eps[i]} ts {Es[i].rng_ts} y {so[1]:.1f}",
                          flush=True)
                    print(f"    gpu filt {fg[i]} orc filt {fo}", flush=True)
            if ended:
                eps[i] += 1
                L.orc_reset_philox(C.byref(P), C.byref(Es[i]), 0, seed, i, eps[i], 1, int(stoch), fixed, tilt)
    if fused:
        Sg = env.state.cpu().numpy()
        for i in range(n):
            so = np.array(Es[i].s[:])
            err = np.abs(Sg[i] - so) / np.maximum(np.abs(so), 1e-3)
            print(f"[{tag}] fused env {i} final max rel err {err.max():.2e} ({ST[int(err.argmax())]})", flush=True)
    ep, st, _ = env.episode_counters()
    print(f"[{tag}] done: diverged envs {sorted(first.items())}; gpu episodes {ep.tolist()} orc {eps}", flush=True)


if __name__ == "__main__":
    T = int(os.environ.get("T", "150"))
    run("det", 4, T, 5, False, 0.0, 0)
    run("tilt", 4, T, 5, False, math.radians(1.0), 0)
    run("stoch", 4, T, 5, True, 0.0, 0)
    run("stoch+tilt", 4, T, 5, True, math.radians(1.0), 0)
    run("randprof", 4, T, 5, True, math.radians(1.0), -1)
    run("fused", 4, T, 5, True, math.radians(1.0), 0, fused=True)
