"""Counts, in a PD_EXP_TRUSTCHECK build, how often a trusted line-interval key differs from the
verified 50-NN key (printed by pd_counters with PDENV_DEBUG_COUNTERS: 'knn calls' = trusted
lookups, 'probes' = mismatches)."""
import math, os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
os.environ["PDENV_DEBUG_COUNTERS"] = "1"
for prec in ("f64", "f32"):
    for wind in (True, False):
        n = 65536
        e = pdenv.PoweredDescentEnv(n, mode="rl", precision=prec, enable_wind=wind, stochastic_wind=wind,
                                    wind_percentile=None, auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234)
        g = torch.Generator(device="cuda").manual_seed(0)
        for t in range(300):
            e.step_raw((torch.rand(n, 1, generator=g, device="cuda") * 2 - 1).contiguous())
        torch.cuda.synchronize()
        print(prec, "wind", wind, e.counters(), flush=True)
        e.close()
