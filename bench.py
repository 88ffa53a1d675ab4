#!/usr/bin/env python3
"""Benchmark: env-steps/s of the MI355X powered-descent env (BASELINE.json metric).

Workload (BASELINE config c3, one GPU): 65 536 parallel envs per GPU, phase
landing_burn_pure_throttle with the SAC driver's reward (rtd_rl), the horizontal wind
profile + von Karman gusts (percentile drawn per reset, as WindModel(given_percentile=None)),
initial pitch perturbation N(0, 1 deg), synthetic uniform float32 random actions resident in
HBM, auto-reset on done/truncated.  One timed "step" = one env.step() of all envs (4 physics
sub-steps + g-load window + truncated/done/reward + obs written per step); by default 128
consecutive steps run in one k_step launch (pd_step_n, --fuse 128), --fuse 1 launches per step.

Multi-GPU: one process per GPU (torchrun), each rank steps its own contiguous env shard
(env_offset = rank * N); the env batch shards with no data-path collective, so scaling is
weak; the timed region is bracketed by barriers and the max over ranks is reported.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))


def algorithmic_bytes(precision, phase, wind):
    """SURVEY.md 8(d) ALGORITHMIC bytes per env-step (the roofline's per-unit figure): step-mode
    SoA, binary32 base 163 B (reads: 11 state + prev speed + 10 g-window + 1 action = 92 B;
    writes: 11 state + prev speed + window slot + head + 2 obs + reward = 68 B, + done, trunc,
    trunc_id 3 B); binary64 state +88 B; wind +56 B (4 filter values r/w, 2 sigmas, RNG counter);
    landing_burn +48 B.  c3 (f64, wind, pure throttle) = 307 B."""
    b = 163 + (88 if precision == "f64" else 0)
    if wind:
        b += 56
    if phase == "landing_burn":
        b += 48
    return b


def implementation_bytes(precision, phase, wind, obs_dim, act_dim, fuse):
    """Bytes k_step actually moves per env-step in a launch of `fuse` fused steps: the per-env
    state is read and written once per launch (registers in between), the per-step I/O every
    step (action in; obs, reward, done/trunc/trunc_id out)."""
    r = 8 if precision == "f64" else 4
    state = 11 * r + r + 10 * r + 2 + 16 + 8 + 8 + 1          # state, |v_prev|, g-window, head/len, keys, slots, counters, tid
    if phase == "landing_burn":
        state += 3 * r
    if wind:
        state += 6 * r + 1                                      # filters, sigmas, percentile
    per_step = 4 * act_dim + obs_dim * r + r + 3
    return 2 * state / fuse + per_step


def valu_roofline(mix, steps, kern_ms, simds=1024, clock_hz=2.4e9, fp64_peak_tflops=78.6):
    """The bound that actually limits k_step: vector-ALU issue.  `mix` is the
    instruction mix per env-step (all envs) of the same workload from rocprofv3 PMC passes
    (profiles/pmc_traffic.json), counted here over the `steps` env-steps of the timed launches,
    whose kernel time `kern_ms` is the one measured live.  Issue model of a SIMD-32 (MI355X
    guide): a wave64 VALU instruction occupies 2 cycles, a binary64 one 4."""
    f64 = steps * sum(mix.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
    valu = steps * mix["SQ_INSTS_VALU"]
    issue_cycles = 4.0 * f64 + 2.0 * (valu - f64)
    sec = kern_ms * 1e-3
    flop = 64.0 * steps * (mix.get("SQ_INSTS_VALU_ADD_F64", 0.0) + mix.get("SQ_INSTS_VALU_MUL_F64", 0.0)
                           + mix.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + 2.0 * mix.get("SQ_INSTS_VALU_FMA_F64", 0.0))
    return {"bound": "valu", "achieved": issue_cycles / sec / 1e12, "peak": simds * clock_hz / 1e12,
            "unit": "T SIMD-issue-cycles/s", "frac": issue_cycles / (simds * clock_hz * sec),
            "valu_insts_per_env_step": mix["SQ_INSTS_VALU"], "f64_insts_per_env_step": f64 / steps,
            "env_steps": steps, "kernel_ms": kern_ms,
            "fp64_tflops": flop / sec / 1e12, "fp64_peak_tflops": fp64_peak_tflops,
            "waves_per_launch": mix.get("SQ_WAVES"),
            "source": "profiles/pmc_traffic.json f64_valu_mix_per_launch (rocprofv3 --pmc, 2 passes), "
                      "per env-step"}


def flop_roofline(oc, wc, n, steps, kern_ms, peak_tflops=78.6):
    """Algorithmic binary64 FLOPs of the timed launches over their kernel time, against the FP64
    vector peak: profiles/opcount.json's exact counts per unit (tools/opcount.cpp: the step's
    arithmetic over a counting scalar type; add/sub/mul/div/sqrt 1, fma 2) weighted by what the
    launches did (workload_counts: gust-band sub-steps and the table queries by path).  Per
    env-step: 3 sub-steps with their own atmosphere and one reusing the rtd's, the wind profile
    on each, the gust block on the gust-band ones, 8 table queries (2 tables x 4 sub-steps) by
    path (clamped line: Taylor piece; interior: cell piece, + the side test in a bisector
    sub-cell; verified: payload sums), and the step tail (g-load window, rtd, observation)."""
    u = oc["units"]
    f = lambda k, key="flops": u[k][key]
    per_q = {key: wc["q_taylor_frac"] * f("q_line", key) + wc["q_cell_frac"] * f("q_piece", key)
             + wc["q_bisect_frac"] * (f("q_bisect", key) - f("q_piece", key)) + wc["q_balanced_frac"] * f("q_payload", key)
             for key in ("flops", "transcendentals")}
    per = {key: 3 * f("substep", key) + f("substep_first", key) + 4 * f("wind_profile", key)
                + 4 * wc["gust_steps_frac"] * f("gust", key) + 8 * per_q[key] + f("step_tail", key)
           for key in ("flops", "transcendentals")}
    achieved = per["flops"] * n * steps / (kern_ms * 1e-3) / 1e12
    return {"bound": "fp64", "achieved": achieved, "peak": peak_tflops, "unit": "TFLOP/s",
            "frac": achieved / peak_tflops, "flops_per_env_step": per["flops"],
            "transcendentals_per_env_step": per["transcendentals"],
            "query_flops_mean": per_q["flops"],
            "source": "profiles/opcount.json (tools/opcount.cpp, checked by tests/test_opcount.py) x this "
                      "window's workload_counts; the algorithm's arithmetic, not the instructions issued"}


def shard_offset(rank, n_per_rank):
    """Global index of a rank's first env: contiguous shards, disjoint Philox streams."""
    return rank * n_per_rank


def whole_job_rate(n_per_rank, world, steps, wall_max):
    """env-steps/s of the whole job: every rank's envs x steps over the slowest rank's time."""
    return n_per_rank * world * steps / wall_max


def timed_region(step_fn, steps, sync, dist=None, device="cpu", pre=None, post=None):
    """barrier + sync, exactly `steps` calls of step_fn(k), sync + barrier; max wall over ranks.
    pre()/post() run right after the clock starts / before the closing sync (stream events)."""
    import torch
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if pre:
        pre()
    for k in range(steps):
        step_fn(k)
    if post:
        post()
    sync()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist:
        w = torch.tensor([wall], device=device, dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    return wall


def bench_sac(args, world, rank, local, dist):
    """Config c5: SAC data collection, 4096 envs per GPU (32 768 on 8 GPUs), pure throttle, RL
    reward, auto-reset.  One timed step = the reference's Actor (256x2, sampled, PyTorch-ROCm)
    on every env's observation + one env step + transition slab + all_gather over RCCL + append
    to the learner rank's device replay buffer."""
    import torch
    import pdenv
    from pdenv.sac import Actor, DevicePrioritizedReplayBuffer, SACCollector
    n = args.envs if args.envs != 65536 else 4096
    env = pdenv.PoweredDescentEnv(n, flight_phase="landing_burn_pure_throttle", mode="rl",
                                  precision=args.precision, device=local, auto_reset=True, seed=1234,
                                  env_offset=shard_offset(rank, n))
    torch.manual_seed(0)
    actor = Actor(2, 1).to(env.device)
    # the driver's buffer: PrioritizedReplayBuffer, 1e6 transitions (sac_pytorch_powered_descent.py:62-70)
    buf = DevicePrioritizedReplayBuffer(1_000_000, 2, 1, env.device) if rank == 0 else None
    col = SACCollector(env, actor, buf, dist, use_graph=args.graph == 1)
    for _ in range(args.warmup):
        col.step()
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall = timed_region(lambda k: col.step(), args.steps, torch.cuda.synchronize, dist, env.device,
                        pre=r0.record, post=r1.record)
    region_ms = r0.elapsed_time(r1) / args.steps
    # the dominant kernel's device time.  Eager (the default): the timed region's own event pair
    # on the stream the k_step<SAC> launches run on, per step -- the launches run back to back
    # there (rocprofv3: no gap between them), so this is their average duration with the miss
    # flush every 16th step included (an upper bound).  With a graph the region also holds the
    # gaps its replays leave, so the kernel time is the same step run again with a HIP event pair
    # per step (the flush outside the pairs).  The pairs are reported in both modes.
    kern = []
    for _ in range(min(args.steps, 64)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        col.step()
        e1.record()
        kern.append((e0, e1))
    torch.cuda.synchronize()
    kern_ms = sorted(a.elapsed_time(b) for a, b in kern)
    # a pair also spans any host stall between its first event and the launch (the GPU idles
    # there): pairs beyond 1.5x the median are such stalls (rocprofv3's k_step average agrees with
    # the rest), left out of the average and counted
    kern_med = kern_ms[len(kern_ms) // 2]
    kern_in = [k for k in kern_ms if k <= 1.5 * kern_med]
    pairs_avg = sum(kern_in) / len(kern_in)
    kern_avg = pairs_avg if args.graph == 1 else region_ms
    if rank != 0:
        return None
    # per env-step: the env's algorithmic bytes (f64 pure throttle, no wind: SURVEY 8(d)), the
    # transition row (2 S + A + 2 floats) and the next float32 observation, plus the actor's
    # parameters once per launch shared by the n envs; FLOPs: the actor's three GEMMs (2 per MAC)
    S, A, H = env.obs_dim, env.action_dim, actor.mean.in_features
    n_par = sum(p.numel() for p in actor.parameters())
    bpe = algorithmic_bytes(args.precision, "landing_burn_pure_throttle", False) + 4 * (2 * S + A + 2) + 4 * S \
        + 4.0 * n_par / n
    fpe = 2.0 * (S * H + H * H + 2 * H * A)
    out = {
        "metric": ("SAC collection env-steps/sec (c5: actor + env + RCCL all_gather of the transition rows + "
                   "prioritized replay buffer)" if dist else
                   "SAC collection env-steps/sec (c5: actor + env + prioritized replay buffer, one launch per step; "
                   "one process, no collective)"),
        "value": whole_job_rate(n, world, args.steps, wall), "unit": "env-steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (random-init SAC actor 2-256-256-1, reference initial state, no wind)",
        "config": {"workload": "c5: SAC collection, landing_burn_pure_throttle, rtd_rl, auto-reset",
                   "envs_per_gpu": n, "global_envs": n * world,
                   "parallelism": f"env-shard x{world} + all_gather" if dist else "one process (no process group)"},
        "replay_buffer_size": len(buf), "hip_graph": args.graph == 1,
        "roofline": {"bound": "hbm", "achieved": bpe * n / (kern_avg * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": bpe * n / (kern_avg * 1e-3) / 1e9 / 8000.0,
                     "traffic": pmc_traffic("c5", n) if n == 4096 else None,
                     "traffic_bytes_per_env_step": pmc_traffic("c5", 1) if n == 4096 else None,
                     "traffic_source": PMC_C4C5 + " (case c5: 2 FETCH_SIZE + WRITE_SIZE of the k_step<SAC> launch, "
                                       "per launch of n env-steps)",
                     "bytes_per_env_step": round(bpe, 1), "kernel": "k_step<SAC> (pd_step_sac_fused: actor MLP + step)",
                     "kernel_avg_ms": kern_avg, "kernel_launches": args.steps if args.graph != 1 else len(kern_in),
                     "kernel_timing": ("the timed region's HIP event pair per step (back-to-back launches)"
                                       if args.graph != 1 else
                                       "HIP events around each replayed step (pairs beyond 1.5x the median, host "
                                       "stalls, left out)"),
                     "event_pairs": {"avg_ms": pairs_avg, "med_ms": kern_med, "pairs": len(kern_in),
                                     "host_stalled": len(kern_ms) - len(kern_in),
                                     "note": "a HIP event pair around each step run again: each pair adds its "
                                             "events' own device time"},
                     "bytes_source": "SURVEY 8(d) env bytes + transition row + next obs32 + actor parameters / n"},
        "mfma_roofline": {"bound": "mfma", "achieved": fpe * n / (kern_avg * 1e-3) / 1e12, "peak": 157.3,
                          "unit": "TFLOP/s", "frac": fpe * n / (kern_avg * 1e-3) / 1e12 / 157.3,
                          "flops_per_env_step": fpe, "note": "the actor's GEMMs (fp32 MFMA peak) over the whole kernel "
                                                             "time, which also steps the env"},
    }
    if args.cpu_baseline and world == 1:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle
        thr = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1, 64))
        ps = [p.detach().float().cpu().numpy() for p in actor.parameters()]
        L_ = sum(1 for m in actor.shared_net if isinstance(m, torch.nn.Linear))
        ne, ns = 64 * thr, 600          # (about 10 s of host work at 16 threads)
        t0 = time.perf_counter()
        _, nsteps = oracle.sac_collect(ne, ns, ps, H, L_, S, A, seed=1234, threads=thr)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": nsteps / dt, "unit": "env-steps/s", "cores": thr, "kind": "port",
                               "sample": f"oracle/pd_oracle.c orc_sac_collect_mt: the same actor (binary32, sequential "
                                         f"sums) + sampling + env step + transition row, {ne} envs x {ns} steps on "
                                         f"{thr} host threads, {dt:.1f} s"}
    return out


def bench_pso(args, world, rank, local, dist):
    """Config c4: generations of the particle subswarm optimisation over P particles per GPU
    (phase landing_burn, 372-parameter simple_actor per particle, swarm initialised U(-1.5, 1.5)
    as initialize_swarms does).  One timed step = one generation: every particle's episode with
    the actor fused into the step kernel (pd_rollout_policy_chunked, until done/truncated, cap
    2200), subswarm/global bests with the per-subswarm minima exchanged across ranks, and the
    velocity/position update (pd_pso_step_chunked, which writes the next rollout's weights)."""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    P = args.particles
    opt = ParticleSubswarmOptimisationGPU("landing_burn", pop_size=P * world, device=local, seed=1234,
                                          precision=args.precision, dist=dist,
                                          tuning=dict(policy_list=args.policy_list, policy_refill=args.policy_refill,
                                                      policy_refill_own=args.policy_refill_own),
                                          pso_params=dict(generations=args.warmup + args.steps,
                                                          re_initialise_generation=-1))
    for g in range(args.warmup):
        opt.generation(g)
    torch.cuda.synchronize()
    tot = torch.zeros((), dtype=torch.int64, device=opt.device)

    def one(k):
        opt.generation(args.warmup + k)
    # episode lengths of the timed generations (a separate evaluation pass is not timed)
    wall = timed_region(one, args.steps, torch.cuda.synchronize, dist, opt.device)
    # the dominant kernel: the policy rollout of the swarm's current positions
    # (pd_rollout_policy_chunked: k_step<POL> launches until every episode ended), replayed with a
    # HIP event pair per rollout
    kern = []
    for _ in range(max(1, min(args.steps, 8))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _, steps = opt.evaluate(opt.x32c)
        e1.record()
        kern.append((e0, e1))
    torch.cuda.synchronize()
    kern_ms = sorted(a.elapsed_time(b) for a, b in kern)
    kern_avg = sum(kern_ms) / len(kern_ms)
    tot += steps.sum()
    if dist:
        dist.all_reduce(tot)
    if rank != 0:
        return None
    mean_len = int(tot.item()) / (P * world)
    eps = whole_job_rate(P, world, args.steps, wall)
    # per particle-episode: the env's algorithmic bytes per env-step (f64 landing_burn, no wind:
    # SURVEY 8(d)) x the episode's steps, + its 372 float32 actor parameters read once
    bpp = mean_len * algorithmic_bytes(args.precision, "landing_burn", False) + 4 * 372
    out = {
        "metric": "PSO particle-episodes/sec (c4: fused actor rollouts + device swarm update)", "value": eps,
        "unit": "particle-episodes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (swarm initialised U(-1.5,1.5) per parameter, nominal initial state, no wind)",
        "config": {"workload": "c4: PSO generation, landing_burn, 372-param simple_actor fused in k_step, "
                               "2 subswarms", "particles_per_gpu": P, "global_particles": P * world,
                   "parallelism": f"particle-shard x{world} + subswarm-minimum all_gather"},
        "env_steps_per_s_est": eps * mean_len, "mean_episode_len_after": mean_len,
        "global_best_fitness": opt.gbf,
        "roofline": {"bound": "hbm", "achieved": bpp * P / (kern_avg * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": bpp * P / (kern_avg * 1e-3) / 1e9 / 8000.0,
                     "traffic": pmc_traffic(f"c4_{P}", P), "traffic_bytes_per_particle_episode": pmc_traffic(f"c4_{P}", 1),
                     "traffic_source": PMC_C4C5 + f" (case c4_{P}: 2 FETCH_SIZE + WRITE_SIZE of the policy k_step "
                                       f"launches of one rollout, per rollout of {P} particles; null: no pass at this size)",
                     "bytes_per_particle_episode": round(bpp, 1), "kernel": "k_step<POL> (pd_rollout_policy_chunked)",
                     "kernel_avg_ms": kern_avg, "kernel_med_ms": kern_ms[len(kern_ms) // 2], "rollouts": len(kern_ms),
                     "kernel_timing": "HIP events around each replayed rollout of the swarm's positions "
                                      "(k_policy_init, the k_step launches, k_policy_finish)",
                     "bytes_source": "SURVEY 8(d) landing_burn env bytes x mean episode length + the actor's parameters"},
    }
    if args.cpu_baseline and world == 1:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import numpy as np
        import oracle
        thr = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1, 64))
        Wc = np.random.default_rng(0).uniform(-1.5, 1.5, (1024 * thr, 372)).astype(np.float32)
        t0 = time.perf_counter()
        _, st = oracle.rollout_policy(1, Wc, 2200, threads=thr)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": len(Wc) / dt, "unit": "particle-episodes/s", "cores": thr, "kind": "port",
                               "sample": f"oracle/pd_oracle.c orc_rollout_policy_mt, {len(Wc)} particles of the same "
                                         f"U(-1.5, 1.5) swarm law ({int(st.sum())} env-steps), {thr} host threads, "
                                         f"{dt:.1f} s"}
    return out


def other_workloads(args, local):
    """BASELINE configs c4 and c5 at their per-GPU sizes, run after the c3 line's measurement in
    the same process (one GPU, no process group), so that the default run records them too:
    short runs, summarised beside the headline line (`python bench.py --workload c4|c5` gives
    the full lines)."""
    res = {}
    for wl, kw in (("c5", dict(steps=192, warmup=32)), ("c4", dict(steps=16, warmup=2, cpu_baseline=0))):
        sub = argparse.Namespace(**{**vars(args), **kw, "workload": wl})
        try:
            o = (bench_pso if wl == "c4" else bench_sac)(sub, 1, 0, local, None)
            res[wl] = {k: o[k] for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype")}
            res[wl]["size_per_gpu"] = o["config"].get("particles_per_gpu", o["config"].get("envs_per_gpu"))
        except Exception as exc:      # reported, never hides the headline line
            res[wl] = {"error": repr(exc)[:300]}
    return res


KERNEL_REPLAYS = 3      # replays of the timed launches for the kernel time (per-launch median)
DESCENT_BURN_IN = 640   # c3-descent: untimed steps before the warmup (a steady mix of episode phases)
# c3: untimed steps before the warmup, so that the timed window sees resets at their stationary
# rate; --c3-burn-in 0 gives the fresh-episode window of rounds 1-3, which the line also reports as
# `c3_fresh`
C3_BURN_IN = 640
# Staggered starts (--stagger K, off by default): under the uniform-action law every episode lasts
# 131 +- 2.4 steps (oracle, 1 024 envs x 3 000 steps), so envs that all start at step 0 keep
# resetting together for thousands of steps -- a 20-step window lands on a reset wave (47 resets
# per 1 000 env-steps in the driver's window) or between two (0; the stationary rate is 7.6).
# With --stagger K env i is reset once more at prologue step i mod K before the burn-in (pd_reset
# with a mask, rocket_environment_pre_wrap.reset of that env), which spreads the episodes' phases
# over the period as a training run's independent envs are.  Measured (round 6): resets cost
# little, but a wave's 32 envs then sit at 32 different phases of their descent and take more
# divergent paths: c3 3 % slower than with the synchronized starts (profiles/r06_bench_stagger.jsonl).
# The default keeps the synchronized starts (every env reset together, as pd_reset / the
# reference's reset() leave a batch); the line reports the staggered window as `c3_staggered`.
C3_STAGGER = 0
C3_STAGGER_SUB = 128


def c3_actions(T, n, gen, device, descent):
    """Synthetic float32 actions [T, n, 1] resident in HBM.  c3: U(-1, 1) for every env (under
    this law every episode truncates on max-q near 17 km, rtd_rl.py:229-231, id 4).  c3-descent:
    the 3:1 high-throttle mix of tests/test_gpu_c3.py -- U(0.5, 1) on three envs in four (they
    descend through the 15 km gust ceiling, full_wind_model.py:37, towards the landing logic,
    rtd_rl.py:194-206), U(-1, 1) on every fourth."""
    import torch
    u = torch.rand(T, n, 1, generator=gen, device=device)
    if not descent:
        return (u * 2 - 1).contiguous()
    hi = (torch.arange(n, device=device) % 4 != 0).view(1, n, 1)
    return torch.where(hi, 0.5 + 0.5 * u, 2 * u - 1).contiguous()


def workload_counts(d, n, steps, lpe):
    """What the timed launches did, from the step kernel's counters (pd_stats words 32-39) over a
    counting replay of exactly the timed launches (pd_count_work; the replay starts from the
    timed region's checkpoint with the same actions, so it steps the same envs through the same
    states): gust-band sub-steps, resets, table queries by path."""
    sub = n * steps * 4
    out = {"env_substeps": sub, "gust_substeps": d["gust_substeps"], "gust_steps_frac": d["gust_substeps"] / sub,
           "resets": d["resets"], "resets_per_1k_env_steps": 1e3 * d["resets"] / (n * steps),
           "rbf_misses_solved": d["rbf_misses"]}
    if lpe == 2:
        q = 2 * sub      # one C_D and one C_L query per env sub-step
        out.update({"table_queries": q, "q_line_frac": d["q_line"] / q, "q_interior_frac": 1 - d["q_line"] / q,
                    "q_verified_frac": d["q_verified"] / q, "q_taylor_frac": d["q_taylor"] / q,
                    "q_cell_frac": d["q_cell"] / q,
                    "q_balanced_frac": d["q_balanced"] / q, "q_miss_frac": d["q_miss"] / q,
                    "balanced_rounds_per_wave_substep": d["balanced_rounds"] / (sub * 2 / 64),
                    "q_refined_frac": d["q_refined"] / q, "q_bisect_frac": d["q_bisect"] / q,
                    "wave_substeps_refined_frac": d["wave_substeps_refined"] / (sub * 2 / 64),
                    "wave_substeps_bisect_frac": d["wave_substeps_bisect"] / (sub * 2 / 64),
                    # wave sub-steps whose lanes hold both clamped-line and interior queries (each
                    # such wave runs both evaluation paths one after the other)
                    "wave_substeps_mixed_frac": d["wave_substeps_mixed"] / (sub * 2 / 64)})
    return out


def run_c3(args, precision, local, rank, dist, descent=False, launch_base=0, burn=None, stagger=None):
    """One c3 (or c3-descent) measurement on this rank's handle, after the staggered prologue
    (`stagger` steps, default --stagger when there is a burn-in) and `burn` untimed steps
    (default: c3-descent's, or --c3-burn-in).  Returns the raw timings."""
    import torch
    import pdenv
    n = args.envs
    mode = "rl" if args.phase == "landing_burn_pure_throttle" else "pso"
    env = pdenv.PoweredDescentEnv(
        n, flight_phase=args.phase, mode=mode, precision=precision, device=local,
        enable_wind=not args.no_wind, stochastic_wind=not args.no_wind, wind_percentile=None,
        auto_reset=True, tilt_sigma_rad=0.0 if args.workload == "c2" else math.radians(1.0), seed=1234,
        env_offset=shard_offset(rank, n), integrator=args.integrator)
    if burn is None:
        burn = DESCENT_BURN_IN if descent else args.c3_burn_in
    stagger = args.stagger if (stagger is None and burn > 0) else (stagger or 0)
    W = burn + args.warmup
    T = W + args.steps
    F = max(1, args.fuse)
    g = torch.Generator(device=env.device).manual_seed(42 + rank)
    if stagger > 0:
        # the staggered prologue (C3_STAGGER): one step of every env, then the envs of phase t
        # reset, for t = 0 .. stagger - 1 (untimed; its own draws of the same action law)
        ph = torch.arange(n, device=env.device) % stagger
        pro = c3_actions(stagger, n, g, env.device, descent)
        for t in range(stagger):
            env.step_raw(pro[t].contiguous())
            env.reset(mask=ph == t)
        torch.cuda.synchronize()
        del pro, ph
    acts = c3_actions(T, n, g, env.device, descent)
    launches = [0]
    if F > 1:
        # pd_step_n: F env-steps per launch, every step's outputs written (rows of [F, N, ...]
        # buffers reused chunk to chunk, as the per-step loop reuses one [N, ...] buffer)
        kw = dict(device=env.device)
        outs = (torch.empty(F, n, env.obs_dim, dtype=env.dtype, **kw), torch.empty(F, n, dtype=env.dtype, **kw),
                torch.empty(F, n, dtype=torch.uint8, **kw), torch.empty(F, n, dtype=torch.uint8, **kw),
                torch.empty(F, n, dtype=torch.int8, **kw))
        env.set_tuning(step_fuse=F)

        def chunk(t0, t1):
            env.step_n_raw(acts[t0:t1], tuple(o[:t1 - t0] for o in outs))
            launches[0] += 1
    else:
        def chunk(t0, t1):
            env.step_raw(acts[t0])
            launches[0] += 1
    bounds = lambda a, b: [(t, min(t + F, b)) for t in range(a, b, F)]
    for t0, t1 in bounds(0, W):
        chunk(t0, t1)
    torch.cuda.synchronize()
    # timed region: exactly K env-steps (ceil(K / F) launches), nothing else on the stream but
    # the miss flush after each launch and one event at either end (device time of the region)
    tb = bounds(W, T)
    blob = env.checkpoint()          # every per-env buffer at the start of the timed region
    s0 = env.stats()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    first_timed = launch_base + launches[0]
    timed = lambda k: chunk(*tb[k])
    if F > 1:
        # the timed launches' C arguments (device pointers of the action / output rows, the
        # stream) prepared before the clock starts: inside it, exactly one pd_step_n call per
        # launch -- the tensor slicing and pointer boxing of step_n_raw cost ~16 us of host time
        # per call, which the short driver window (one 20-step launch) would otherwise time
        import ctypes as C
        from pdenv import _lib as PL
        stream = C.c_void_p(torch.cuda.current_stream(env.device).cuda_stream)
        cargs = [(env.h, C.c_void_p(acts[t0:t1].data_ptr()), t1 - t0) +
                 tuple(C.c_void_p(o[:t1 - t0].data_ptr()) for o in outs) + (stream,) for t0, t1 in tb]
        step_n = env.lib.pd_step_n

        def timed(k):
            PL.check(step_n(*cargs[k]))
            launches[0] += 1
    wall = timed_region(timed, len(tb), torch.cuda.synchronize, dist, env.device, pre=e0.record, post=e1.record)
    dev_ms = e0.elapsed_time(e1)
    s1 = env.stats()
    # kernel duration: the timed region's launches replayed from the checkpoint (the same
    # actions and per-env state; the aero tables keep what the timed region inserted, so the
    # replay solves fewer misses -- both counts are reported), each launch with its miss flush
    # between a pair of HIP events on the stream the kernel runs on
    # (three replays; each launch's median: one launch of the driver's 20-step window varies by
    # up to 20 % between identical replays -- clocks, the chip's other traffic)
    first_replay = launch_base + launches[0]
    reps = []
    for _ in range(KERNEL_REPLAYS):
        env.restore(blob)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in tb]
        for k, b in enumerate(tb):
            ev[k][0].record()
            chunk(*b)
            ev[k][1].record()
        torch.cuda.synchronize()
        reps.append([a.elapsed_time(b) for a, b in ev])
    s2 = env.stats()
    # workload counts: the same launches once more with the step kernel's counters on (counting
    # costs a few per cent, so neither timed pass counts)
    env.restore(blob)
    env.count_work(True)
    for b in tb:
        chunk(*b)
    torch.cuda.synchronize()
    env.count_work(False)
    s3 = env.stats()
    kern = [sorted(r[k] for r in reps)[len(reps) // 2] for k in range(len(tb))]
    full = [m for m, (t0, t1) in zip(kern, tb) if t1 - t0 == F]
    d = {k: s3[k] - s2[k] for k in env.WORK_COUNTERS}
    d["rbf_misses"] = s1["rbf_misses"] - s0["rbf_misses"]     # solved in the timed region itself
    res = dict(wall=wall, dev_ms=dev_ms, kern_total_ms=sum(kern), kern_launches=len(kern), kern_replays=KERNEL_REPLAYS,
               kern_avg_full_ms=(sum(full) / len(full)) if full else None, fuse=F, n=n,
               obs_dim=env.obs_dim, act_dim=env.action_dim, burn_in=burn, stagger=stagger,
               # (lanes per env: pd_create's default, 2 above 8 192 envs)
               counts=workload_counts(d, n, args.steps, 2 if n > 8192 else 0),
               replay_misses=s2["rbf_misses"] - s1["rbf_misses"],
               launch_index={"kernel": f"k_step<{'double' if precision == 'f64' else 'float'}>",
                             "timed": [first_timed, first_timed + len(tb)],
                             "replay": [first_replay, first_replay + KERNEL_REPLAYS * len(tb)],
                             "replays": KERNEL_REPLAYS},
               nan_events=s3["nan_events"], descent=descent)
    res["launches_total"] = launches[0]   # (every launch of this handle: the replays included)
    env.close()
    return res


def c3_summary(args, r, world, precision, pmc=None):
    """The measured quantities of one run_c3 result (the headline line's fields)."""
    wind = not args.no_wind
    bpe = algorithmic_bytes(precision, args.phase, wind)
    F, n, K = r["fuse"], r["n"], args.steps
    ibpe = implementation_bytes(precision, args.phase, wind, r["obs_dim"], r["act_dim"], F)
    kern_s = r["kern_total_ms"] * 1e-3
    achieved = bpe * n * K / kern_s / 1e9
    traffic = per_step = None
    mix = None
    if pmc:
        # counter bytes per env-step, times the env-steps of the average timed launch
        # (like `achieved`: the driver's short timed region may be one partial launch)
        per_step = pmc.get(f"{precision}_bytes_per_launch")
        per_step = per_step / float(pmc.get("env_steps_per_launch", 1)) if per_step is not None else None
        traffic = per_step * K / r["kern_launches"] if per_step is not None else None
        mix = pmc.get("f64_valu_mix_per_launch") if precision == "f64" else None
        if mix:   # per env-step (the wave count is per launch)
            ps = float(pmc.get("env_steps_per_launch", 1))
            mix = {k: (v / ps if k != "SQ_WAVES" else v) for k, v in mix.items()}
    out = {
        "value": whole_job_rate(n, world, K, r["wall"]),
        "ms_per_step": r["wall"] / K * 1e3,
        "device_ms_per_step": r["dev_ms"] / K,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                     "frac": achieved / 8000.0, "traffic": traffic,
                     "traffic_bytes_per_env_step": per_step / n if per_step is not None else None,
                     "bytes_per_env_step": bpe, "bytes_source": "SURVEY.md 8(d) algorithmic count",
                     "implementation_bytes_per_env_step": round(ibpe, 1),
                     "kernel": "k_step", "kernel_ms_per_step": r["kern_total_ms"] / K,
                     # (the average over the timed launches; a short timed region may be one
                     # partial launch of K < F env-steps)
                     "kernel_avg_ms": r["kern_total_ms"] / r["kern_launches"],
                     "kernel_avg_full_launch_ms": r["kern_avg_full_ms"], "kernel_launches_timed": r["kern_launches"],
                     "env_steps_per_launch": F, "env_steps_per_timed_launch": K / r["kern_launches"],
                     "envs_per_launch": n,
                     "kernel_timing": "the timed region's launches replayed from its checkpoint three times, HIP events "
                                      "per launch (k_step + its miss flush) on the launch stream, each launch's median",
                     "note": "VALU/latency-bound elementwise ODE (no MFMA); see DESIGN.md"},
        "workload_counts": r["counts"],
        "replay_rbf_misses": r["replay_misses"],
        "launch_index": r["launch_index"],
    }
    if mix and n == 65536:
        # over exactly the timed launches' env-steps and kernel time (a short timed region may be
        # one partial launch)
        out["valu_roofline"] = valu_roofline(mix, K, r["kern_total_ms"])
        cm = load_pmc("r06_pmc_c3_mix.json")
        case = (cm or {}).get("cases", {}).get("c3_descent" if r.get("descent") else "c3")
        if case and precision == "f64":
            # rocprof's VALUUtilization: the share of a VALU instruction's 64 lanes
            # active, SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU), and the VALU stream by type
            out["valu_roofline"]["lane_utilisation"] = case["valu_lane_utilisation"]
            out["valu_roofline"]["valu_shares"] = case["valu_shares"]
            out["valu_roofline"]["class_source"] = "profiles/r06_pmc_c3_mix.json (rocprofv3 --pmc, the same workload)"
    oc = load_pmc("opcount.json")
    if oc and precision == "f64" and args.phase == "landing_burn_pure_throttle" and not args.no_wind \
            and "q_taylor_frac" in r["counts"]:
        out["flop_roofline"] = flop_roofline(oc, r["counts"], n, K, r["kern_total_ms"])
    return out


PMC_C4C5 = "profiles/r06_pmc_c4c5.json"


def pmc_traffic(case, units):
    """HBM-side bytes of `units` units of a c4 / c5 case from the committed rocprofv3 PMC passes
    (tools/pmc_r06.sh, reduced by tools/pmc_r06.py: bytes per unit); None without a pass."""
    d = load_pmc(os.path.basename(PMC_C4C5))
    c = (d or {}).get("cases", {}).get(case)
    if not c or c.get("bytes_per_unit") is None:
        return None
    return c["bytes_per_unit"] * units


def load_pmc(name):
    p = os.path.join(REPO, "profiles", name)
    try:
        return json.load(open(p)) if os.path.exists(p) else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=192)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--precision", choices=["f64", "f32"], default="f64")
    ap.add_argument("--phase", default="landing_burn_pure_throttle")
    ap.add_argument("--no-wind", action="store_true")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--secondary", type=int, default=0,
                    help="also time the other precision (off by default: the binary32 handle is 1.2x binary64 on c3 "
                         "and slower on c2, DESIGN.md s8)")
    ap.add_argument("--descent", type=int, default=1, help="c3: also measure c3-descent (nested in the line)")
    ap.add_argument("--workload", choices=["c2", "c3", "c3-descent", "c4", "c5"], default="c3",
                    help="c3: env-steps/s headline (uniform random actions); c3-descent: c3 with the 3:1 "
                         "high-throttle action mix after a burn-in (gust band, landings); c2: 4096 envs, no "
                         "wind, no tilt (--integrator); c4: PSO generations with the fused actor; "
                         "c5: SAC collection (actor + env + RCCL transition gather + replay buffer)")
    ap.add_argument("--integrator", choices=["reference", "rk4"], default="reference",
                    help="rk4: BASELINE c2's RK4 dt=0.01 s, NOT the reference's integrator (non-parity)")
    ap.add_argument("--particles", type=int, default=32768, help="c4: particles per GPU")
    ap.add_argument("--fuse", type=int, default=128,
                    help="c3: env-steps per k_step launch (pd_step_n; 1 = one pd_step launch per step)")
    ap.add_argument("--policy-list", type=int, default=-1, choices=[-1, 0, 1],
                    help="c4: the policy rollouts' live-list launches (pd_tuning.policy_list: -1 auto, 0 off, 1 on)")
    ap.add_argument("--policy-refill", type=int, default=-1,
                    help="c4: refill rollouts (pd_tuning.policy_refill: -1 auto, 0 off, k = batch of k waiting slots)")
    ap.add_argument("--policy-refill-own", type=int, default=-1,
                    help="c4: percent of the swarm refilled from the waves' own ranges (pd_tuning.policy_refill_own; -1 auto)")
    ap.add_argument("--graph", type=int, default=0,
                    help="c5: replay the collection step as a HIP graph (off: each replay left an 8.6 us gap "
                         "between step kernels, eager launches none -- 0.0434 against 0.0392 ms per step, "
                         "profiles/r05_exp_c5_graph.jsonl)")
    ap.add_argument("--stagger", type=int, default=C3_STAGGER,
                    help="c3: staggered starts before the burn-in (env i reset at prologue step i mod STAGGER; "
                         "0 = every env starts at step 0, the synchronized starts, the default)")
    ap.add_argument("--staggered", type=int, default=C3_STAGGER_SUB,
                    help="c3: also measure the window with staggered starts (this K), reported as c3_staggered "
                         "(0: not measured)")
    ap.add_argument("--c3-burn-in", type=int, default=C3_BURN_IN,
                    help="c3: untimed env-steps before the warmup (steady state: resets at their stationary rate)")
    ap.add_argument("--fresh", type=int, default=1,
                    help="c3: also measure the fresh-episode window (no burn-in), reported as c3_fresh")
    ap.add_argument("--others", type=int, default=1,
                    help="c3 at one GPU: also run short c4 and c5 measurements (summarised in the line)")
    args = ap.parse_args()
    if args.workload == "c2":
        args.no_wind = True
        if args.envs == 65536:
            args.envs = 4096
    if args.integrator == "rk4" and args.workload != "c2":
        ap.error("--integrator rk4 is the non-parity c2 mode: use --workload c2")

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; PD_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks
    # sharing fewer GPUs (ranks map onto the visible devices round-robin)
    backend = os.environ.get("PD_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    dist = None
    # PD_BENCH_DIST=1: initialise the process group (and run every collective) even at one rank,
    # to exercise the RCCL path on a single GPU
    if world > 1 or os.environ.get("PD_BENCH_DIST") == "1":
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    if args.workload in ("c4", "c5"):
        out = (bench_pso if args.workload == "c4" else bench_sac)(args, world, rank, local, dist)
        if out is not None:
            print(json.dumps(out))
        if dist:
            dist.destroy_process_group()
        return

    descent_main = args.workload == "c3-descent"
    main_res = run_c3(args, args.precision, local, rank, dist, descent=descent_main)
    base = main_res["launches_total"]
    desc = None
    if args.workload == "c3" and args.descent:
        desc = run_c3(args, args.precision, local, rank, dist, descent=True, launch_base=base)
        base += desc["launches_total"]
    fresh = None
    if args.workload == "c3" and args.fresh and args.c3_burn_in > 0:
        fresh = run_c3(args, args.precision, local, rank, dist, launch_base=base, burn=0)
        base += fresh["launches_total"]
    stag = None
    if args.workload == "c3" and args.staggered > 0 and args.stagger == 0 and args.c3_burn_in > 0:
        stag = run_c3(args, args.precision, local, rank, dist, launch_base=base, stagger=args.staggered)
        base += stag["launches_total"]
    other = None
    if args.secondary:
        other = run_c3(args, "f32" if args.precision == "f64" else "f64", local, rank, dist, descent=descent_main)
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    n_total = main_res["n"] * world
    wind = not args.no_wind
    pmc = None
    if args.workload == "c3":
        pmc = load_pmc("pmc_traffic.json")          # the committed PMC passes of the c3 workload
    elif descent_main:
        pmc = load_pmc("pmc_c3_descent.json")
    summ = c3_summary(args, main_res, world, args.precision, pmc)
    wl = {"c3": "c3: 65536 envs/GPU, landing_burn_pure_throttle, rtd_rl reward, wind (percentile profile drawn "
                "per reset + VK gusts below 15 km) + tilt, auto-reset, uniform random actions" +
                ((f"; timed after {args.stagger} staggered-start steps" if args.stagger > 0 else "; synchronized starts") +
                 f", {args.c3_burn_in} untimed burn-in + {args.warmup} warmup steps" if args.c3_burn_in > 0
                 else "; timed on fresh episodes (no burn-in)"),
          "c3-descent": f"c3-descent: the c3 configuration with the 3:1 high-throttle action mix, timed after "
                        f"{DESCENT_BURN_IN} burn-in + {args.warmup} warmup steps (episodes in every phase of the "
                        f"descent: gust band, landing logic)",
          "c2": f"c2: {main_res['n']} envs/GPU, landing_burn_pure_throttle, rtd_rl reward, no wind, no tilt, "
                f"auto-reset, integrator {args.integrator}" +
                (" (RK4 dt=0.01 s: NOT the reference's integrator, non-parity)" if args.integrator == "rk4"
                 else " (semi-implicit Euler 4 x 0.025 s)")}[args.workload]
    metric = "env-steps/sec at 65 536 parallel envs; achieved HBM GB/s vs peak"    # BASELINE.json's (c3)
    if args.workload == "c2":
        metric = (f"env-steps/sec at {main_res['n']} parallel envs (c2, no wind" +
                  (", RK4 dt=0.01 s: non-parity" if args.integrator == "rk4" else "") + "); achieved HBM GB/s vs peak")
    out = {
        "metric": metric,
        "value": summ["value"],
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": summ["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (float32 actions in HBM; reference initial state" +
                (" + N(0,1deg) pitch tilt)" if args.workload != "c2" else ")"),
        "config": {"workload": wl, "envs_per_gpu": main_res["n"], "global_envs": n_total,
                   "parallelism": f"env-shard x{world}"},
    }
    out.update({k: v for k, v in summ.items() if k not in ("value", "ms_per_step")})
    out["rbf_table_misses"] = main_res["counts"]["rbf_misses_solved"]
    if desc is not None:
        ds = c3_summary(args, desc, world, args.precision, load_pmc("pmc_c3_descent.json"))
        ds["workload"] = (f"c3-descent: 3:1 high-throttle action mix, {DESCENT_BURN_IN} burn-in + {args.warmup} "
                          f"warmup steps, then {args.steps} timed")
        out["c3_descent"] = ds
    if fresh is not None:
        fs = c3_summary(args, fresh, world, args.precision)
        out["c3_fresh"] = {"value": fs["value"], "ms_per_step": fs["ms_per_step"],
                           "kernel_ms_per_step": fs["roofline"]["kernel_ms_per_step"],
                           "roofline_frac": fs["roofline"]["frac"], "workload_counts": fs["workload_counts"],
                           "launch_index": fs["launch_index"],
                           "workload": f"c3 on fresh episodes: no burn-in, {args.warmup} warmup steps, then "
                                       f"{args.steps} timed (every env's first episode, 30 km down)"}
    if stag is not None:
        ss = c3_summary(args, stag, world, args.precision)
        out["c3_staggered"] = {"value": ss["value"], "ms_per_step": ss["ms_per_step"],
                               "kernel_ms_per_step": ss["roofline"]["kernel_ms_per_step"],
                               "roofline_frac": ss["roofline"]["frac"], "workload_counts": ss["workload_counts"],
                               "launch_index": ss["launch_index"],
                               "workload": f"c3 with staggered starts: env i reset once more at prologue step i mod "
                                           f"{args.staggered}, then {args.c3_burn_in} burn-in + {args.warmup} warmup steps, "
                                           f"then {args.steps} timed (resets at their stationary rate; each wave's envs at "
                                           f"different phases of their episodes)"}
    if other is not None:
        op = "f32" if args.precision == "f64" else "f64"
        out["secondary"] = {"dtype": op, "value": whole_job_rate(other["n"], world, args.steps, other["wall"]),
                            "kernel_ms_per_step": other["kern_total_ms"] / args.steps,
                            "launch_index": other["launch_index"]}
    # (before the CPU baseline: its host threads must not share the CPU with these launch-bound runs)
    if args.others and world == 1 and args.workload == "c3" and args.envs == 65536:
        out["other_workloads"] = other_workloads(args, local)
    if args.cpu_baseline and world == 1 and args.workload == "c2" and args.integrator == "rk4":
        out["cpu_baseline"] = None
        out["cpu_baseline_note"] = ("the RK4 mode is not the reference's integrator and the oracle's threaded rollout "
                                    "runs the reference integrator only: no CPU line for it")
    elif args.cpu_baseline and world == 1 and args.workload in ("c2", "c3", "c3-descent"):
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import numpy as np
        import oracle
        # all host threads this job may use (the GPU box exports OMP_NUM_THREADS = its CPU share)
        thr = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1, 64))
        c2 = args.workload == "c2"
        tilt = 0.0 if c2 else math.radians(1.0)
        ne, ns = 64 * thr, 600
        acts = np.random.default_rng(0).uniform(-1, 1, (ns, ne, 1)).astype(np.float32)
        oracle.rollout(0, 0, 2, 2, acts[:2, :2], True, wind, tilt)
        t0 = time.perf_counter()
        _, nsteps = oracle.rollout(0, 0, ne, ns, acts, True, wind, tilt, threads=thr)
        dt = time.perf_counter() - t0
        what = ("the c2 workload (no wind, no tilt, auto-reset, uniform random actions)" if c2 else
                "the c3 workload (wind+tilt+auto-reset, uniform random actions)")
        out["cpu_baseline"] = {"value": nsteps / dt, "unit": "env-steps/s", "cores": thr, "kind": "port",
                               "sample": f"oracle/pd_oracle.c scalar port on {thr} host threads (static env "
                                         f"partition), {ne} envs x {ns} steps of {what}, {dt:.1f} s"}
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
