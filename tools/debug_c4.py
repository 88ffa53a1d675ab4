"""c4 diagnostics: per-generation rollout time, episode-length distribution and aero-table
misses of one PSO evaluation (random swarm U(-1.5, 1.5))."""
import os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
P = int(os.environ.get("P", "32768"))
for lpe in [int(x) for x in os.environ.get("LPES", "2,4").split(",")]:
    env = pdenv.PoweredDescentEnv(P, "landing_burn", mode="pso", seed=1, lanes_per_env=lpe)
    W = (torch.rand(P, 372, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0)) * 3 - 1.5)
    for ce in [int(x) for x in os.environ.get("CES", "4,8,16,64").split(",")]:
        for rep in range(3):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            fit, steps = env.rollout_policy(W, max_steps=2200, check_every=ce)
            torch.cuda.synchronize(); dt = time.perf_counter() - t0
            print(f"lpe {lpe} check_every {ce} rep {rep}: {dt*1e3:.2f} ms, max len {int(steps.max())}, mean {float(steps.float().mean()):.1f}, counters {env.counters()}", flush=True)
    q = torch.quantile(steps.float(), torch.tensor([0.5, 0.9, 0.99, 0.999, 1.0], device=steps.device))
    print("len quantiles 50/90/99/99.9/100:", [round(float(v), 1) for v in q], flush=True)
    h = torch.bincount(steps.long().clamp(max=256) // 16)
    print("len histogram (16-step bins, last = >=256):", h.tolist(), flush=True)
    env.close()
