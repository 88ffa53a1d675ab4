"""Interior-grid resolution experiment (PDENV_GRID): untrusted-query rate (COUNT build) or
step time (normal build) on the c3 workload."""
import math, os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
os.environ["PDENV_DEBUG_COUNTERS"] = "1"
n = 65536
t0 = time.perf_counter()
e = pdenv.PoweredDescentEnv(n, mode="rl", enable_wind=True, stochastic_wind=True, wind_percentile=None,
                            auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234)
print("grid", os.environ.get("PDENV_GRID", "default"), "create s", round(time.perf_counter() - t0, 2), flush=True)
g = torch.Generator(device="cuda").manual_seed(0)
acts = (torch.rand(120, n, 1, generator=g, device="cuda") * 2 - 1).contiguous()
for t in range(60):
    e.step_raw(acts[t])
torch.cuda.synchronize(); t0 = time.perf_counter()
for t in range(60, 120):
    e.step_raw(acts[t])
torch.cuda.synchronize()
print("ms/step", round((time.perf_counter() - t0) / 60 * 1e3, 4), e.counters(), flush=True)
