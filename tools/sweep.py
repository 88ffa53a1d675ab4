#!/usr/bin/env python3
"""Kernel-variant sweep on one GPU, interleaved rounds in one process (guide rule 24):
lanes-per-env x precision on the bench workload (c3).  Prints one JSON line per variant."""
import itertools
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
import pdenv  # noqa: E402


def main():
    n = int(os.environ.get("N", "65536"))
    steps = int(os.environ.get("STEPS", "60"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    lpes = [int(x) for x in os.environ.get("LPES", "1,2,4,8").split(",")]
    precs = os.environ.get("PRECS", "f64,f32").split(",")
    wind = os.environ.get("WIND", "1") == "1"
    phase = os.environ.get("PHASE", "landing_burn_pure_throttle")
    mode = "rl" if phase == "landing_burn_pure_throttle" else "pso"
    envs = {}
    for lpe, p in itertools.product(lpes, precs):
        e = pdenv.PoweredDescentEnv(n, flight_phase=phase, mode=mode, precision=p, enable_wind=wind,
                                    stochastic_wind=wind, wind_percentile=None, auto_reset=True,
                                    tilt_sigma_rad=math.radians(1.0), seed=1234, lanes_per_env=lpe)
        e.flush_every = 16
        envs[(lpe, p)] = e
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = (torch.rand(steps * (rounds + 1), n, envs[(lpes[0], precs[0])].action_dim, generator=g, device="cuda") * 2 - 1).contiguous()
    res = {k: [] for k in envs}
    for k, e in envs.items():           # warm-up: fills neighbourhood caches
        for t in range(steps):
            e.step_raw(acts[t])
    torch.cuda.synchronize()
    for r in range(rounds):
        for k, e in envs.items():
            base = steps * (r + 1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(steps):
                e.step_raw(acts[base + t])
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / steps)
    for k, v in res.items():
        v = sorted(v)
        print(json.dumps({"lpe": k[0], "precision": k[1], "n": n, "ms_per_step_min": v[0] * 1e3,
                          "ms_per_step_med": v[len(v) // 2] * 1e3, "env_steps_per_s": n / v[len(v) // 2],
                          "misses": envs[k].counters()["rbf_misses"]}))


if __name__ == "__main__":
    main()
