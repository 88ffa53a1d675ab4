#!/usr/bin/env python3
"""Benchmark: env-steps/s of the MI355X powered-descent env (BASELINE.json metric).

Workload (BASELINE config c3, one GPU): 65 536 parallel envs per GPU, phase
landing_burn_pure_throttle with the SAC driver's reward (rtd_rl), the horizontal wind
profile + von Karman gusts (percentile drawn per reset, as WindModel(given_percentile=None)),
initial pitch perturbation N(0, 1 deg), synthetic uniform float32 random actions resident in
HBM, auto-reset on done/truncated.  One timed "step" = one env.step() of all envs (4 physics
sub-steps + g-load window + truncated/done/reward + obs written per step); by default 16
consecutive steps run in one k_step launch (pd_step_n, --fuse 16), --fuse 1 launches per step.

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


def valu_roofline(mix, kern_avg_ms, simds=1024, clock_hz=2.4e9, fp64_peak_tflops=78.6):
    """The bound that actually limits k_step: vector-ALU issue.  `mix` is the
    per-launch instruction mix of the same workload from rocprofv3 PMC passes
    (profiles/pmc_traffic.json); the launch time is the one measured live.  Issue model of a
    SIMD-32 (MI355X guide): a wave64 VALU instruction occupies 2 cycles, a binary64 one 4."""
    f64 = sum(mix.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
    valu = mix["SQ_INSTS_VALU"]
    issue_cycles = 4.0 * f64 + 2.0 * (valu - f64)
    sec = kern_avg_ms * 1e-3
    flop = 64.0 * (mix.get("SQ_INSTS_VALU_ADD_F64", 0.0) + mix.get("SQ_INSTS_VALU_MUL_F64", 0.0)
                   + mix.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + 2.0 * mix.get("SQ_INSTS_VALU_FMA_F64", 0.0))
    return {"bound": "valu", "achieved": issue_cycles / sec / 1e12, "peak": simds * clock_hz / 1e12,
            "unit": "T SIMD-issue-cycles/s", "frac": issue_cycles / (simds * clock_hz * sec),
            "valu_insts_per_launch": valu, "f64_insts_per_launch": f64,
            "fp64_tflops": flop / sec / 1e12, "fp64_peak_tflops": fp64_peak_tflops,
            "waves_per_launch": mix.get("SQ_WAVES"),
            "source": "profiles/pmc_traffic.json f64_valu_mix_per_launch (rocprofv3 --pmc, 2 passes)"}


def shard_offset(rank, n_per_rank):
    """Global index of a rank's first env: contiguous shards, disjoint Philox streams."""
    return rank * n_per_rank


def whole_job_rate(n_per_rank, world, steps, wall_max):
    """env-steps/s of the whole job: every rank's envs x steps over the slowest rank's time."""
    return n_per_rank * world * steps / wall_max


def timed_region(step_fn, steps, sync, dist=None, device="cpu"):
    """barrier + sync, exactly `steps` calls of step_fn(k), sync + barrier; max wall over ranks."""
    import torch
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step_fn(k)
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
    env.flush_every = 16
    torch.manual_seed(0)
    actor = Actor(2, 1).to(env.device)
    # the driver's buffer: PrioritizedReplayBuffer, 1e6 transitions (sac_pytorch_powered_descent.py:62-70)
    buf = DevicePrioritizedReplayBuffer(1_000_000, 2, 1, env.device) if rank == 0 else None
    col = SACCollector(env, actor, buf, dist, use_graph=args.graph == 1)
    for _ in range(args.warmup):
        col.step()
    wall = timed_region(lambda k: col.step(), args.steps, torch.cuda.synchronize, dist, env.device)
    if rank != 0:
        return None
    out = {
        "metric": "SAC collection env-steps/sec (c5: actor + env + RCCL gather + prioritized replay buffer)",
        "value": whole_job_rate(n, world, args.steps, wall), "unit": "env-steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (random-init SAC actor 2-256-256-1, reference initial state, no wind)",
        "config": {"workload": "c5: SAC collection, landing_burn_pure_throttle, rtd_rl, auto-reset",
                   "envs_per_gpu": n, "global_envs": n * world, "parallelism": f"env-shard x{world} + all_gather"},
        "replay_buffer_size": len(buf), "hip_graph": args.graph == 1,
    }
    return out


def bench_pso(args, world, rank, local, dist):
    """Config c4: generations of the particle subswarm optimisation over P particles per GPU
    (phase landing_burn, 372-parameter simple_actor per particle, swarm initialised U(-1.5, 1.5)
    as initialize_swarms does).  One timed step = one generation: every particle's episode with
    the actor fused into the step kernel (pd_rollout_policy, until done/truncated, cap 2200),
    subswarm/global bests with the per-subswarm minima exchanged across ranks, and the
    velocity/position update (pd_pso_step)."""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    P = args.particles
    opt = ParticleSubswarmOptimisationGPU("landing_burn", pop_size=P * world, device=local, seed=1234,
                                          precision=args.precision, dist=dist,
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
    _, steps = opt.evaluate(opt.x32)
    tot += steps.sum()
    if dist:
        dist.all_reduce(tot)
    if rank != 0:
        return None
    mean_len = int(tot.item()) / (P * world)
    eps = whole_job_rate(P, world, args.steps, wall)
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
    }
    if args.cpu_baseline and world == 1:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import numpy as np
        import oracle
        Wc = np.random.default_rng(0).uniform(-1.5, 1.5, (2048, 372)).astype(np.float32)
        t0 = time.perf_counter()
        _, st = oracle.rollout_policy(1, Wc, 2200)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": len(Wc) / dt, "unit": "particle-episodes/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/pd_oracle.c orc_rollout_policy, {len(Wc)} particles "
                                         f"({int(st.sum())} env-steps), 1 host thread, {dt:.1f} s"}
    return out


def other_workloads(args, local):
    """BASELINE configs c4 and c5 at their per-GPU sizes, run after the c3 line's measurement in
    the same process (one GPU, no process group), so that the default run records them too:
    short runs, summarised beside the headline line (`python bench.py --workload c4|c5` gives
    the full lines)."""
    res = {}
    for wl, kw in (("c5", dict(steps=192, warmup=32)), ("c4", dict(steps=4, warmup=2, cpu_baseline=0))):
        sub = argparse.Namespace(**{**vars(args), **kw, "workload": wl})
        try:
            o = (bench_pso if wl == "c4" else bench_sac)(sub, 1, 0, local, None)
            res[wl] = {k: o[k] for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype")}
            res[wl]["size_per_gpu"] = o["config"].get("particles_per_gpu", o["config"].get("envs_per_gpu"))
        except Exception as exc:      # reported, never hides the headline line
            res[wl] = {"error": repr(exc)[:300]}
    return res


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
    ap.add_argument("--secondary", type=int, default=1, help="also time the other precision")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c3",
                    help="c3: env-steps/s headline; c2: 4096 envs, no wind, no tilt (--integrator); "
                         "c4: PSO generations with the fused actor; "
                         "c5: SAC collection (actor + env + RCCL transition gather + replay buffer)")
    ap.add_argument("--integrator", choices=["reference", "rk4"], default="reference",
                    help="rk4: BASELINE c2's RK4 dt=0.01 s, NOT the reference's integrator (non-parity)")
    ap.add_argument("--particles", type=int, default=32768, help="c4: particles per GPU")
    ap.add_argument("--fuse", type=int, default=16,
                    help="c3: env-steps per k_step launch (pd_step_n; 1 = one pd_step launch per step)")
    ap.add_argument("--graph", type=int, default=1, help="c5: replay the collection step as a HIP graph")
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
    import pdenv
    if args.workload in ("c4", "c5"):
        out = (bench_pso if args.workload == "c4" else bench_sac)(args, world, rank, local, dist)
        if out is not None:
            print(json.dumps(out))
        if dist:
            dist.destroy_process_group()
        return

    def run(precision):
        n = args.envs
        mode = "rl" if args.phase == "landing_burn_pure_throttle" else "pso"
        env = pdenv.PoweredDescentEnv(
            n, flight_phase=args.phase, mode=mode, precision=precision, device=local,
            enable_wind=not args.no_wind, stochastic_wind=not args.no_wind, wind_percentile=None,
            auto_reset=True, tilt_sigma_rad=0.0 if args.workload == "c2" else math.radians(1.0), seed=1234,
            env_offset=shard_offset(rank, n), integrator=args.integrator)
        env.flush_every = 16
        T = args.warmup + args.steps
        F = max(1, args.fuse)
        KT = 8                  # full launches of the separate kernel-duration pass
        g = torch.Generator(device=env.device).manual_seed(42 + rank)
        acts = (torch.rand(max(T, args.warmup + KT * F), n, env.action_dim, generator=g, device=env.device) * 2 - 1).contiguous()
        if F > 1:
            # pd_step_n: F env-steps per launch, every step's outputs written (rows of [F, N, ...]
            # buffers reused chunk to chunk, as the per-step loop reuses one [N, ...] buffer)
            kw = dict(device=env.device)
            outs = (torch.empty(F, n, env.obs_dim, dtype=env.dtype, **kw), torch.empty(F, n, dtype=env.dtype, **kw),
                    torch.empty(F, n, dtype=torch.uint8, **kw), torch.empty(F, n, dtype=torch.uint8, **kw),
                    torch.empty(F, n, dtype=torch.int8, **kw))
            os.environ["PDENV_FUSE"] = str(F)

            def chunk(t0, t1):
                k = t1 - t0
                env.step_n_raw(acts[t0:t1], tuple(o[:k] for o in outs))
        else:
            def chunk(t0, t1):
                env.step_raw(acts[t0])
        bounds = lambda a, b: [(t, min(t + F, b)) for t in range(a, b, F)]
        for t0, t1 in bounds(0, args.warmup):
            chunk(t0, t1)
        torch.cuda.synchronize()
        # timed region: exactly K env-steps (ceil(K / F) launches), nothing else on the stream (a
        # per-launch event pair costs ~10 us of GPU time, so the kernel-duration pass is separate)
        tb = bounds(args.warmup, T)
        blob = env.checkpoint()          # every per-env buffer at the start of the timed region
        wall = timed_region(lambda k: chunk(*tb[k]), len(tb), torch.cuda.synchronize, dist, env.device)
        # kernel duration: the timed region's launches replayed from the checkpoint (the same
        # work, bit for bit), extended by the following actions to at least KT full launches,
        # with HIP events around each launch (and its miss flush) on the stream the kernel runs on
        env.restore(blob)
        nfull = max(KT, args.steps // F)
        full = [(args.warmup + k * F, args.warmup + (k + 1) * F) for k in range(nfull)]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in full]
        for k, b in enumerate(full):
            ev[k][0].record()
            chunk(*b)
            ev[k][1].record()
        torch.cuda.synchronize()
        kern_ms = sorted(a.elapsed_time(b) for a, b in ev)
        c = env.counters()
        res = dict(wall=wall, kern_avg_ms=sum(kern_ms) / len(kern_ms), kern_med_ms=kern_ms[len(kern_ms) // 2], fuse=F,
                   kern_launches=len(kern_ms),
                   n=n, obs_dim=env.obs_dim, act_dim=env.action_dim, counters=c)
        env.close()
        return res

    main_res = run(args.precision)
    other = None
    if args.secondary:
        other = run("f32" if args.precision == "f64" else "f64")
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    n_total = main_res["n"] * world
    value = whole_job_rate(main_res["n"], world, args.steps, main_res["wall"])
    wind = not args.no_wind
    bpe = algorithmic_bytes(args.precision, args.phase, wind)
    F = main_res["fuse"]
    ibpe = implementation_bytes(args.precision, args.phase, wind, main_res["obs_dim"], main_res["act_dim"], F)
    achieved = bpe * main_res["n"] * F / (main_res["kern_avg_ms"] * 1e-3) / 1e9
    traffic = None
    mix = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc) and args.workload == "c3":   # the committed PMC passes profile c3
        try:
            summ = json.load(open(pmc))
            # PMC figures are per launch of the profiled run's env-steps-per-launch: rescale to F
            scale = F / float(summ.get("env_steps_per_launch", 1))
            traffic = summ.get(f"{args.precision}_bytes_per_launch")
            traffic = traffic * scale if traffic is not None else None
            mix = summ.get("f64_valu_mix_per_launch") if args.precision == "f64" else None
            if mix:
                mix = {k: v * scale for k, v in mix.items()}
        except Exception:
            traffic = None
    out = {
        "metric": "env-steps/sec at 65 536 parallel envs; achieved HBM GB/s vs peak",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_res["wall"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (uniform float32 random actions in HBM; reference initial state" +
                (" + N(0,1deg) pitch tilt)" if args.workload == "c3" else ")"),
        "config": {"workload": "c3: 65536 envs/GPU, landing_burn_pure_throttle, rtd_rl reward, wind (VK gusts + "
                               "percentile profile) + tilt, auto-reset" if args.workload == "c3" else
                               f"c2: {main_res['n']} envs/GPU, landing_burn_pure_throttle, rtd_rl reward, no wind, "
                               f"no tilt, auto-reset, integrator {args.integrator}" +
                               (" (RK4 dt=0.01 s: NOT the reference's integrator, non-parity)"
                                if args.integrator == "rk4" else " (semi-implicit Euler 4 x 0.025 s)"),
                   "envs_per_gpu": main_res["n"], "global_envs": n_total, "parallelism": f"env-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                     "frac": achieved / 8000.0, "traffic": traffic,
                     "bytes_per_env_step": bpe, "bytes_source": "SURVEY.md 8(d) algorithmic count",
                     "implementation_bytes_per_env_step": round(ibpe, 1),
                     "kernel": "k_step", "kernel_avg_ms": main_res["kern_avg_ms"],
                     "kernel_launches_timed": main_res["kern_launches"],
                     "env_steps_per_launch": F, "envs_per_launch": main_res["n"],
                     "note": "VALU/transcendental-bound elementwise ODE (no MFMA); see DESIGN.md"},
        "rbf_table_misses": main_res["counters"]["rbf_misses"],
    }
    if mix and args.envs == 65536 and args.phase == "landing_burn_pure_throttle" and not args.no_wind:
        out["valu_roofline"] = valu_roofline(mix, main_res["kern_avg_ms"])
    if other is not None:
        op = "f32" if args.precision == "f64" else "f64"
        out["secondary"] = {"dtype": op, "value": whole_job_rate(other["n"], world, args.steps, other["wall"]),
                            "kernel_avg_ms": other["kern_avg_ms"]}
    # (before the CPU baseline: its host threads must not share the CPU with these launch-bound runs)
    if args.others and world == 1 and args.workload == "c3" and args.envs == 65536:
        out["other_workloads"] = other_workloads(args, local)
    if args.cpu_baseline and world == 1 and args.workload == "c3":
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import numpy as np
        import oracle
        # all host threads this job may use (the GPU box exports OMP_NUM_THREADS = its CPU share)
        thr = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1, 64))
        ne, ns = 64 * thr, 600
        acts = np.random.default_rng(0).uniform(-1, 1, (ns, ne, 1)).astype(np.float32)
        oracle.rollout(0, 0, 2, 2, acts[:2, :2], True, wind, math.radians(1.0))
        t0 = time.perf_counter()
        _, nsteps = oracle.rollout(0, 0, ne, ns, acts, True, wind, math.radians(1.0), threads=thr)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": nsteps / dt, "unit": "env-steps/s", "cores": thr, "kind": "port",
                               "sample": f"oracle/pd_oracle.c scalar port on {thr} host threads (static env "
                                         f"partition), {ne} envs x {ns} steps of the same workload "
                                         f"(wind+tilt+auto-reset), {dt:.1f} s"}
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
