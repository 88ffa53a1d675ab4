#!/usr/bin/env python3
"""Time the c3 workload through pd_step_n (F fused env-steps per launch, FUSE, default 16) with the
library named by PDENV_LIB (default the in-tree one): one JSON line with the event-timed k_step
launch average, the wall ms per env-step and the step kernel's workload counters over the timed
launches.  N, LAUNCHES, PREC, LPE, PHASE from the environment; DESCENT=1: the c3-descent action
mix (bench.py c3_actions) after bench.py's burn-in; BURN overrides the untimed burn-in steps."""
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
import pdenv  # noqa: E402

n = int(os.environ.get("N", "65536"))
launches = int(os.environ.get("LAUNCHES", "24"))
F = int(os.environ.get("FUSE", "16"))
descent = os.environ.get("DESCENT") == "1"
sys.path.insert(0, REPO)
import bench  # noqa: E402
burn = int(os.environ.get("BURN", bench.DESCENT_BURN_IN if descent else 0))
phase = os.environ.get("PHASE", "landing_burn_pure_throttle")
t_c = time.perf_counter()
wind = os.environ.get("WIND", "1") == "1"      # WIND=0 TILT=0: the c2 workload (INTEG=rk4: its RK4 mode)
env = pdenv.PoweredDescentEnv(n, flight_phase=phase, mode="rl" if phase == "landing_burn_pure_throttle" else "pso",
                              precision=os.environ.get("PREC", "f64"), enable_wind=wind, stochastic_wind=wind,
                              wind_percentile=None, auto_reset=True,
                              tilt_sigma_rad=math.radians(1.0) if os.environ.get("TILT", "1") == "1" else 0.0, seed=1234,
                              lanes_per_env=int(os.environ.get("LPE", "0")), integrator=os.environ.get("INTEG", "reference"),
                              table_flags=int(os.environ.get("TABLE_FLAGS", "0")))
t_create = time.perf_counter() - t_c
env.set_tuning(step_fuse=F)
g = torch.Generator(device="cuda").manual_seed(42)
acts = bench.c3_actions(burn + (launches + 8) * F, n, g, "cuda", descent)
kw = dict(device="cuda")
outs = (torch.empty(F, n, env.obs_dim, dtype=env.dtype, **kw), torch.empty(F, n, dtype=env.dtype, **kw),
        torch.empty(F, n, dtype=torch.uint8, **kw), torch.empty(F, n, dtype=torch.uint8, **kw),
        torch.empty(F, n, dtype=torch.int8, **kw))
for t0 in range(0, burn + 8 * F, F):
    env.step_n_raw(acts[t0:min(t0 + F, burn + 8 * F)], outs)
torch.cuda.synchronize()
acts = acts[burn:]
env.count_work(os.environ.get("COUNT") == "1")   # counting costs a few per cent: off unless asked
w0 = env.stats()
if os.environ.get("STATS"):      # the counters after the warmup launches (to difference)
    import ctypes as C
    from pdenv import _lib as L
    v0 = (L.I64 * 32)()
    L.check(env.lib.pd_stats(env.h, v0, 32))
    print(json.dumps({"stats_warm": list(v0)}), flush=True)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
t0 = time.perf_counter()
for k in range(launches):
    ev[k][0].record()
    env.step_n_raw(acts[(8 + k) * F:(9 + k) * F], outs)
    ev[k][1].record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
ms = sorted(a.elapsed_time(b) for a, b in ev)
w1 = env.stats()
work = {k: w1[k] - w0[k] for k in env.WORK_COUNTERS}
work["gust_steps_frac"] = work["gust_substeps"] / (n * launches * F * 4)
print(json.dumps({"lib": os.path.basename(os.environ.get("PDENV_LIB", "libpdenv.so")), "n": n, "fuse": F,
                  "lpe": int(os.environ.get("LPE", "0")), "wind": wind, "integrator": os.environ.get("INTEG", "reference"), "table_flags": int(os.environ.get("TABLE_FLAGS", "0")),
                  "descent": descent, "work": work,
                  "launch_ms_avg": sum(ms) / len(ms), "launch_ms_med": ms[len(ms) // 2],
                  "ms_per_step": sum(ms) / len(ms) / F, "wall_ms_per_step": wall * 1e3 / (launches * F),
                  "misses": env.counters()["rbf_misses"], "create_s": round(t_create, 2)}), flush=True)
if os.environ.get("STATS"):
    import ctypes as C
    from pdenv import _lib as L
    v = (L.I64 * 32)()
    L.check(env.lib.pd_stats(env.h, v, 32))
    print(json.dumps({"stats": list(v)}), flush=True)
