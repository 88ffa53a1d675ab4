#!/usr/bin/env python3
"""Wave-lifetime spread of the c3 step kernel (diagnostic build tools/experiments/wave_times.patch,
PDENV_LIB=.../libpdenv_wave_times.so): per wave of a 64-step launch its start and end
(s_memrealtime, 100 MHz) and its hardware slot (XCC, SE, CU, SIMD).  Reports how long the launch
is against its waves and its SIMDs: the time a SIMD's last wave ends before the launch does is
idle silicon that balancing envs across waves could recover.  DESCENT=1: c3-descent."""
import ctypes as C
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import pdenv  # noqa: E402
import bench  # noqa: E402

F = int(os.environ.get("FUSE", "64"))
descent = os.environ.get("DESCENT") == "1"
n = 65536
env = pdenv.PoweredDescentEnv(n, enable_wind=True, stochastic_wind=True, wind_percentile=None, auto_reset=True,
                              tilt_sigma_rad=math.radians(1.0), seed=1234)
env.set_tuning(step_fuse=F)
burn = bench.DESCENT_BURN_IN if descent else 32
L = 6
g = torch.Generator(device="cuda").manual_seed(42)
acts = bench.c3_actions(burn + L * F, n, g, "cuda", descent)
for t0 in range(0, burn, F):
    env.step_n_raw(acts[t0:min(t0 + F, burn)])
torch.cuda.synchronize()
fn = env.lib.pd_debug_wave_times
fn.argtypes = [C.c_void_p, C.c_int]
W = n * 2 // 64
out = []
for k in range(L):
    env.step_n_raw(acts[burn + k * F:burn + (k + 1) * F])
    torch.cuda.synchronize()
    rec = np.zeros((W, 4), dtype=np.uint64)
    assert fn(rec.ctypes.data, W) == 0
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    hw, xcc = rec[:, 2].astype(np.int64), rec[:, 3].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    slot = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    span = (t1.max() - t0.min()) * 10e-9 * 1e3        # ms
    dur = (t1 - t0) * 10e-9 * 1e3
    ends = {}
    for s_, e_ in zip(slot, t1):
        ends[s_] = max(ends.get(s_, 0), e_)
    simd_end = (np.array(list(ends.values())) - t0.min()) * 10e-9 * 1e3
    out.append({"launch_span_ms": round(float(span), 4), "wave_ms_mean": round(float(dur.mean()), 4),
                "wave_ms_max": round(float(dur.max()), 4), "wave_ms_min": round(float(dur.min()), 4),
                "wave_mean_over_span": round(float(dur.mean() / span), 4),
                "simds": len(ends), "simd_end_mean_over_span": round(float(simd_end.mean() / span), 4),
                "simd_end_p10_over_span": round(float(np.percentile(simd_end, 10) / span), 4),
                "start_spread_ms": round(float((t0.max() - t0.min()) * 10e-9 * 1e3), 4)})
print(json.dumps({"descent": descent, "fuse": F, "launches": out}))
