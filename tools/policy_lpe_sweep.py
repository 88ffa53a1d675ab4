#!/usr/bin/env python3
"""Lanes-per-env sweep of the c4 policy rollouts (pd_rollout_policy: fused actor + landing_burn
env + done-mask compaction) at P particles, interleaved rounds in one process: pd_tuning.policy_lanes 2/4/8
(read by the library at every rollout).  The same swarm (U(-1.5, 1.5) per parameter, as
initialize_swarms draws it) each time.  Prints one JSON line per LPE: median rollout ms, the mean
episode length, and the largest fitness difference against LPE 2 (LPE 4/8 evaluate the tables by
split payload sums, LPE 2 by Taylor lines and cell pieces: equal to rounding, not bits)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pdenv  # noqa: E402


def main():
    P = int(os.environ.get("P", "32768"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    lpes = [int(x) for x in os.environ.get("PLPES", "2,4,8").split(",")]
    env = pdenv.PoweredDescentEnv(P, flight_phase="landing_burn", mode="pso", device=0)
    W = torch.from_numpy(np.random.default_rng(0).uniform(-1.5, 1.5, (P, 372)).astype(np.float32)).cuda()
    times = {l: [] for l in lpes}
    fits = {}
    for r in range(rounds + 1):
        for l in lpes:
            env.set_tuning(policy_lanes=l)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fit, steps = env.rollout_policy(W)
            torch.cuda.synchronize()
            if r > 0:                        # round 0 warms the tables and the kernels
                times[l].append((time.perf_counter() - t0) * 1e3)
            fits[l] = (fit.cpu().numpy(), steps.cpu().numpy())
    f2 = fits[lpes[0]][0]
    for l in lpes:
        t = sorted(times[l])
        f, s = fits[l]
        print(json.dumps({"plpe": l, "particles": P, "rollout_ms_med": t[len(t) // 2], "rollout_ms_min": t[0],
                          "mean_episode_len": float(s.mean()),
                          "episode_len_p50_p90_p99_max": [float(np.percentile(s, q)) for q in (50, 90, 99, 100)],
                          # (the longest episode of each wave's 64 / LPE particles: the wave's life)
                          "wave_life_mean": float(s[:len(s) // (64 // l) * (64 // l)].reshape(-1, 64 // l).max(1).mean()),
                          "max_rel_fitness_diff_vs_first": float(np.max(np.abs(f - f2) / (np.abs(f2) + 1.0)))}))


if __name__ == "__main__":
    main()
