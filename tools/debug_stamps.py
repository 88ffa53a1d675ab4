"""Wave-clock breakdown of k_step on the bench workload (c3), with a PD_STAMP build:
PDENV_LIB=.../libpdenv_stamp.so python tools/debug_stamps.py  (prints from pd_counters)."""
import math, os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
os.environ["PDENV_DEBUG_COUNTERS"] = "1"
for prec in ("f64", "f32"):
    n = 65536
    e = pdenv.PoweredDescentEnv(n, mode="rl", precision=prec, enable_wind=True, stochastic_wind=True, wind_percentile=None,
                                auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234)
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = (torch.rand(100, n, 1, generator=g, device="cuda") * 2 - 1).contiguous()
    for t in range(100):
        e.step_raw(acts[t])
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for t in range(100):
        e.step_raw(acts[t])
    torch.cuda.synchronize()
    print(prec, "ms/step", (time.perf_counter() - t0) * 10, e.counters(), flush=True)
    e.close()
