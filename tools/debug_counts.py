import math, os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
os.environ["PDENV_DEBUG_COUNTERS"] = "1"
for wind in (True, False):
    n = 65536
    e = pdenv.PoweredDescentEnv(n, mode="rl", enable_wind=wind, stochastic_wind=wind, wind_percentile=None,
                                auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234, lanes_per_env=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    for phase in range(3):
        for t in range(60):
            e.step_raw((torch.rand(n, 1, generator=g, device="cuda") * 2 - 1).contiguous())
        torch.cuda.synchronize()
        print("wind", wind, "after", 60 * (phase + 1), "steps", e.counters(), flush=True)
