"""c4 diagnostics: per-launch k_step time and aero-table misses over one PSO generation."""
import os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
P = int(os.environ.get("P", "32768"))
for lpe in (2, 4):
    env = pdenv.PoweredDescentEnv(P, "landing_burn", mode="pso", seed=1, lanes_per_env=lpe)
    W = (torch.rand(P, 372, device="cuda") * 3 - 1.5)
    for rep in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        fit, steps = env.rollout_policy(W, max_steps=2200, check_every=64)
        torch.cuda.synchronize(); dt = time.perf_counter() - t0
        print(f"lpe {lpe} rep {rep}: {dt*1e3:.2f} ms, max len {int(steps.max())}, mean {float(steps.float().mean()):.1f}, counters {env.counters()}", flush=True)
    env.close()
