import math, os, sys, time, torch
sys.path.insert(0, "psso-sac-for-powered-descent_amd")
import pdenv
n=65536
env = pdenv.PoweredDescentEnv(n, mode="rl", enable_wind=True, stochastic_wind=True, wind_percentile=None,
                              auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234)
env.flush_every = 16
T=220
acts=(torch.rand(T,n,1,device="cuda")*2-1).contiguous()
for t in range(20): env.step_raw(acts[t])
torch.cuda.synchronize()
for mode in ("events","noevents","events","noevents"):
    torch.cuda.synchronize(); t0=time.perf_counter()
    if mode=="events":
        ev=[(torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)) for _ in range(200)]
        for k in range(200):
            ev[k][0].record(); env.step_raw(acts[20+k]); ev[k][1].record()
    else:
        for k in range(200): env.step_raw(acts[20+k])
    torch.cuda.synchronize(); w=(time.perf_counter()-t0)/200*1e3
    extra = "" if mode!="events" else f" kern {sum(a.elapsed_time(b) for a,b in ev)/200:.4f}"
    print(mode, f"{w:.4f} ms/step", extra)
# host-side cost of one step_raw call
t0=time.perf_counter()
for k in range(200): env.step_raw(acts[20+k])
t1=time.perf_counter(); torch.cuda.synchronize()
print("host enqueue per step", (t1-t0)/200*1e3, "ms")
