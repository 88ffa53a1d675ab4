"""Sub-batches on concurrent HIP streams: the c3 batch (65 536 envs) as S handles of 65536/S
envs, each stepped on its own stream, against one handle on one stream (median ms per step of
all 65 536 envs)."""
import math, os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
import pdenv
N = 65536
res = {}
for S in [int(x) for x in os.environ.get("SPLITS", "1,2,4").split(",")]:
    n = N // S
    envs = [pdenv.PoweredDescentEnv(n, mode="rl", enable_wind=True, stochastic_wind=True, wind_percentile=None,
                                    auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=1234, env_offset=k * n,
                                    lanes_per_env=int(os.environ.get("LPE", "2")))
            for k in range(S)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = (torch.rand(200, N, 1, generator=g, device="cuda") * 2 - 1).contiguous()
    def step(t):
        for k in range(S):
            with torch.cuda.stream(streams[k]):
                envs[k].step_raw(acts[t, k * n:(k + 1) * n])
    for t in range(40):
        step(t)
    torch.cuda.synchronize()
    times = []
    for r in range(5):
        t0 = time.perf_counter()
        for t in range(40 + 30 * r, 70 + 30 * r):
            step(t)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) / 30 * 1e3)
    times.sort()
    print(f"splits {S}: ms/step median {times[2]:.4f} min {times[0]:.4f} -> {N / times[2] * 1e3:.3e} env-steps/s", flush=True)
    for e in envs:
        e.close()
