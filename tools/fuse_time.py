"""Time pd_step_n (fused launches) against the per-step pd_step loop on the c3 workload
(65 536 envs, pure throttle, RL, wind), both with per-step outputs written."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "psso-sac-for-powered-descent_amd"))
import torch
import pdenv

N, T = 65536, 320
res = {}
for prec in ("f64", "f32"):
    kw = dict(precision=prec, enable_wind=True, stochastic_wind=True, auto_reset=True, seed=1)
    A = (torch.rand(T, N, 1, device="cuda") * 2 - 1).contiguous()
    e1 = pdenv.PoweredDescentEnv(N, flight_phase="landing_burn_pure_throttle", mode="rl", **kw)
    e1.flush_every = 16
    for t in range(T): e1.step_raw(A[t])
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for t in range(T): e1.step_raw(A[t])
    torch.cuda.synchronize(); loop = (time.perf_counter() - t0) / T
    e2 = pdenv.PoweredDescentEnv(N, flight_phase="landing_burn_pure_throttle", mode="rl", **kw)
    e2.step_n(A)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    e2.step_n(A)
    torch.cuda.synchronize(); fused = (time.perf_counter() - t0) / T
    res[prec] = {"loop_ms_per_step": loop * 1e3, "fused_ms_per_step": fused * 1e3,
                 "fused_env_steps_per_s": N / fused, "PDENV_FUSE": os.environ.get("PDENV_FUSE", "16")}
print(json.dumps(res))
