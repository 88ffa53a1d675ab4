#!/usr/bin/env python3
"""Where c5's collection step goes: the SAC actor and the step kernel timed
apart and together at c5's per-GPU size (4 096 envs, landing_burn_pure_throttle, rtd_rl, no wind,
auto-reset, 16 lanes per env), each as the median of REPS event-timed launches on the launch
stream, after WARM untimed ones:
  actor        pd_sac_actor alone (the reference Actor 2-256-256-1 on the envs' observations)
  sac_ring     pd_step_sac_ring from given heads: eps drawn in the kernel, ring rows + priorities
  sac_det      the same, deterministic (no eps draw)
  sac_slab     the same, transition rows into a slab instead of the ring
  fused        pd_step_sac_fused: the actor in the step kernel's prologue + sac_ring's work
  step1        pd_step with uniform random float32 actions (one launch per env-step)
  step128      pd_step_n at 128 steps per launch, per env-step (the c2 line's launch shape)
One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
import pdenv  # noqa: E402
from pdenv.sac import Actor, ActorKernel, DevicePrioritizedReplayBuffer  # noqa: E402

N = int(os.environ.get("N", "4096"))
REPS, WARM = int(os.environ.get("REPS", "100")), 10


def timed(fn, reps=REPS, per=1):
    for _ in range(WARM):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) / per for a, b in ev)
    return {"med_us": 1e3 * ms[len(ms) // 2], "min_us": 1e3 * ms[0], "mean_us": 1e3 * sum(ms) / len(ms)}


def main():
    torch.manual_seed(0)
    env = pdenv.PoweredDescentEnv(N, flight_phase="landing_burn_pure_throttle", mode="rl", device=0, auto_reset=True,
                                  seed=1234)
    env.flush_every = 1 << 30
    actor = Actor(2, 1).to(env.device)
    k = ActorKernel(actor)
    S, A = env.obs_dim, env.action_dim
    obs = env.reset().float().contiguous()
    heads = torch.empty(N, 2 * A, device="cuda")
    buf = DevicePrioritizedReplayBuffer(1_000_000, S, A, env.device)
    act = torch.empty(N, A, device="cuda")
    slab = torch.empty(N, 2 * S + A + 2, device="cuda")
    out = {"envs": N, "lanes_per_env": 16, "reps": REPS}
    out["actor"] = timed(lambda: k(obs, heads))
    common = dict(log_std_min=actor.log_std_min, log_std_max=actor.log_std_max, max_action=actor.max_action,
                  action=act, obs32=obs)
    ring = dict(ring=buf.data, capacity=buf.capacity, ring_state=buf.state_dev, priorities=buf.priorities,
                max_priority=buf.max_prio_dev)
    out["sac_ring"] = timed(lambda: env.step_sac_ring(heads, **common, **ring))
    out["sac_det"] = timed(lambda: env.step_sac_ring(heads, deterministic=True, **common, **ring))
    out["sac_slab"] = timed(lambda: env.step_sac_ring(heads, ring=slab, **common))
    out["fused"] = timed(lambda: env.step_sac_fused(k.S, k.A, k.H, k.nl, k.ptrs(), **common, **ring))
    g = torch.Generator(device="cuda").manual_seed(3)
    U = (torch.rand(200, N, 1, generator=g, device="cuda") * 2 - 1).contiguous()
    it = iter(range(10 ** 9))
    out["step1"] = timed(lambda: env.step_raw(U[next(it) % 200]))
    env.set_tuning(step_fuse=128)
    outs = (torch.empty(128, N, S, dtype=env.dtype, device="cuda"), torch.empty(128, N, dtype=env.dtype, device="cuda"),
            torch.empty(128, N, dtype=torch.uint8, device="cuda"), torch.empty(128, N, dtype=torch.uint8, device="cuda"),
            torch.empty(128, N, dtype=torch.int8, device="cuda"))
    U128 = (torch.rand(128, N, 1, generator=g, device="cuda") * 2 - 1).contiguous()
    out["step128_per_step"] = timed(lambda: env.step_n_raw(U128, outs), reps=12, per=128)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
