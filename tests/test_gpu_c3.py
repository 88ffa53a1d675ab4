"""GPU parity of the headline workload (BASELINE config c3) and of the per-env bookkeeping.

c3 = 65 536 envs, landing_burn_pure_throttle with the SAC driver's reward, the horizontal wind
profile of a percentile drawn per reset (WindModel(given_percentile=None),
full_wind_model.py:27-33) plus von Karman gusts (vonkarman.py:33-36), a pitch tilt N(0, 1 deg)
at every reset, and auto-reset.  The reference draws its randomness from np.random with
seed(None) (vonkarman.py:88), so no run of it can be replayed; the oracle instead restates the
device's Philox4x32-10 draw scheme (oracle/pd_oracle.c orc_reset_philox / orc_gauss_pair).  The
env is chaotic (a 1-ulp pitch change moves the oracle's own rewards by 4e-3 within an episode,
tests/test_oracle_golden.py::test_oracle_episode_chaos_bound), so sampled envs of the full-size
run are teacher-forced against the oracle at every step (tests/shadow.py) instead of being
compared after hundreds of free-running steps.  The oracle's wind model itself is pinned to the
reference by tests/test_oracle_golden.py (recorded normals, every percentile).

Tolerances (f64 handle, per env-step): state <= 1e-10 relative (theta_dot 1e-8), reward <= 1e-9
absolute, done/truncated/trunc_id exact, obs <= 1e-6 (float32-cast state), gust filters <= 1e-12,
auto-resets bit-identical.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ST = ["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass", "mass_propellant", "time"]


@pytest.fixture(scope="module")
def pd():
    import torch
    import pdenv
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return pdenv


def c3_env(pd, n, seed=1234, **kw):
    args = dict(flight_phase="landing_burn_pure_throttle", mode="rl", enable_wind=True, stochastic_wind=True,
                wind_percentile=None, auto_reset=True, tilt_sigma_rad=math.radians(1.0), seed=seed)
    args.update(kw)
    return pd.PoweredDescentEnv(n, **args)


def c3_actions(T, N, seed):
    """Random actions U(-1, 1) on every 4th env (episodes end by truncation after ~130 steps and
    auto-reset), U(0.5, 1) elsewhere (high throttle: the vehicles get below the 15 km gust
    ceiling, vonkarman.py / full_wind_model.py:39-41, where the Philox gust draws act)."""
    import torch
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(T, N, 1, generator=g)
    hi = torch.arange(N) % 4 != 0
    a = torch.where(hi.view(1, N, 1), 0.5 + 0.5 * u, 2 * u - 1)
    return a.contiguous()


def c3_sample(N):
    return np.unique(np.concatenate([np.arange(16), np.arange(N - 16, N), np.linspace(16, N - 17, 64).astype(int)]))


def test_c3_full_size_shadowed(pd, oracle_mod):
    """65 536 envs x 400 steps of the c3 workload (wind with a percentile drawn per reset, gusts,
    tilt, auto-reset), stepped by pd_step; 96 sampled envs (both ends of the batch and spread
    through it) teacher-forced against the oracle at every step (tests/shadow.py): state <= 1e-10
    rel (theta_dot 1e-8), reward <= 1e-9, done/truncated/trunc_id exact, obs <= 1e-6, gust filters
    <= 1e-12, every auto-reset bit-identical.  Then the same 400 steps through pd_step_n (16 fused
    steps per launch, state in registers) from a fresh handle: every output and the final state
    bit-identical to the per-step run."""
    import torch
    from shadow import shadow_run, check_stats
    N, T, seed = 65536, 400, 1234
    A = c3_actions(T, N, 7).cuda()
    idx = c3_sample(N)
    env = c3_env(pd, N, seed=seed)
    st = shadow_run(oracle_mod, env, A, idx, 0, 0, seed, math.radians(1.0))
    check_stats(st)
    # coverage: resets, gusts, many percentiles, the truncations random actions reach
    assert st["resets"] >= len(idx), st["resets"]
    assert st["gust_steps"] >= 20 * len(idx), st["gust_steps"]
    assert len(st["profiles"]) >= 20, sorted(st["profiles"])
    assert env.counters()["nan_events"] == 0
    S_loop = env.state
    ref = st["outs"]
    env2 = c3_env(pd, N, seed=seed)
    obs, rew, dn, tr, tid = env2.step_n(A)
    assert torch.equal(obs, ref["obs"]) and torch.equal(rew, ref["rew"])
    assert torch.equal(dn, ref["done"]) and torch.equal(tr, ref["trunc"]) and torch.equal(tid, ref["tid"])
    assert torch.equal(env2.state, S_loop)
    assert torch.equal(env2.checkpoint(), env.checkpoint())


def test_c3_full_size_properties(pd):
    """The whole 65 536-env batch of the c3 workload, per step: time advances by exactly 0.1 s,
    propellant never grows, and every env that ended is back at the initial state with its own
    tilt (theta perturbed, alpha = theta - gamma, all other channels the nominal ones)."""
    import torch
    N, T = 65536, 300
    env = c3_env(pd, N, seed=99)
    g = torch.Generator(device="cuda").manual_seed(0)
    s_nom = torch.tensor(env.params.state0, dtype=torch.float64, device="cuda")
    ended_total = 0
    prev = env.state
    for t in range(T):
        a = torch.rand(N, 1, device="cuda", generator=g) * 2 - 1
        obs, r, dn, trc, ex = env.step(a)
        cur = env.state
        ended = dn | trc
        ended_total += int(ended.sum())
        live = ~ended
        assert torch.allclose(cur[live, 10] - prev[live, 10], torch.full_like(cur[live, 10], 0.1), rtol=0, atol=1e-9)
        assert bool((cur[live, 9] <= prev[live, 9]).all())
        if ended.any():
            keep = [0, 1, 2, 3, 5, 6, 8, 9, 10]
            assert torch.equal(cur[ended][:, keep], s_nom[keep].expand(int(ended.sum()), -1))
            assert torch.equal(cur[ended][:, 7], cur[ended][:, 4] - cur[ended][:, 6])
            assert float((cur[ended][:, 4] - s_nom[4]).abs().max()) < math.radians(6)
        prev = cur
    assert ended_total > N
    assert env.counters()["nan_events"] == 0


@pytest.mark.parametrize("percentile", [50, 57, 63, 75, 88, 98, 99])
def test_fixed_percentile_profiles_shadowed(pd, oracle_mod, percentile):
    """Each percentile's horizontal profile (HorizontalWindSpeed.py:44-114) with gusts, 64 envs x
    300 steps (mostly high throttle, so the vehicles descend through the gust band), every step
    teacher-forced against the oracle (tests/shadow.py; the profiles are pinned to the reference
    by tests/test_oracle_golden.py::test_wind_profiles_every_percentile)."""
    from shadow import shadow_run, check_stats
    N, T = 64, 300
    A = c3_actions(T, N, percentile).cuda()
    env = c3_env(pd, N, seed=5, wind_percentile=percentile)
    st = shadow_run(oracle_mod, env, A, np.arange(N), 0, 0, 5, math.radians(1.0), fixed_prof=percentile - 50)
    check_stats(st)
    assert st["gust_steps"] >= 20 * N and st["resets"] >= N // 4
    assert st["profiles"] == {percentile - 50}
    assert (env.wind_state()[2].cpu().numpy() == percentile).all()


def test_landing_burn_wind_shadowed(pd, oracle_mod):
    """The PSO driver's phase (landing_burn, 4 actions, actuator memory) with the c3 wind and
    tilt: 128 envs x 120 steps, every step teacher-forced against the oracle (PSO reward)."""
    import torch
    from shadow import shadow_run, check_stats
    N, T = 128, 120
    A = (torch.rand(T, N, 4, generator=torch.Generator().manual_seed(3)) * 2 - 1).contiguous().cuda()
    env = c3_env(pd, N, seed=11, flight_phase="landing_burn", mode="pso")
    st = shadow_run(oracle_mod, env, A, np.arange(N), 1, 1, 11, math.radians(1.0))
    check_stats(st)
    assert st["resets"] >= N // 2


def test_checkpoint_restore_continues_bit_identically(pd):
    """Stop a wind + tilt + random-percentile run mid-episode, checkpoint every per-env buffer
    (state, g-load window, actuators, wind filters/sigmas/percentile, episode and step counters,
    aero caches), restore into a fresh handle, and continue: outputs and state bit-identical."""
    import torch
    N, T1, T2 = 4096, 150, 45
    A = (torch.rand(T1 + T2, N, 4, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2)) * 2 - 1)
    for phase, adim in (("landing_burn_pure_throttle", 1), ("landing_burn", 4)):
        a = A[..., :adim].contiguous()
        src = c3_env(pd, N, seed=21, flight_phase=phase)
        src.step_n(a[:T1])
        blob = src.checkpoint()
        ep, st, _ = src.episode_counters()
        assert int(st.max()) > 0 and int(ep.max()) > 0      # mid-episode, after resets
        ref = src.step_n(a[T1:])
        dst = c3_env(pd, N, seed=21, flight_phase=phase)
        dst.restore(blob)
        got = dst.step_n(a[T1:])
        for x, y in zip(ref, got):
            assert torch.equal(x, y), phase
        assert torch.equal(src.state, dst.state)
        assert torch.equal(src.checkpoint(), dst.checkpoint())
        # the getters see the same bookkeeping
        for x, y in zip(src.wind_state(), dst.wind_state()):
            assert torch.equal(x, y)
        for x, y in zip(src.gload_window(), dst.gload_window()):
            assert torch.equal(x, y)


FORCE_KEYS = ("drag", "lift", "aero_force_x", "aero_force_y")
A_FRONT = 107.5131545874767   # sizing_results.csv frontal area (param_pack.json)


def test_info_tap_vs_oracle(pd, oracle_mod):
    """pd_step's info tap (the last sub-step's quantities of rockets_physics.py:649-702) against
    the oracle's info for teacher-forced steps of both landing phases."""
    import torch
    from conftest import golden
    d = golden("ref_teacher_forced.npz")
    names = ["air_density", "atmospheric_pressure", "speed_of_sound", "mach_number", "dynamic_pressure", "CL", "CD",
             "mass_flow", "x_cog", "inertia", "d_thrust_cg", "alpha_effective", "throttle", "control_force_parallel",
             "control_force_perpendicular", "control_moment_z", "aero_force_x", "aero_force_y", "drag", "lift",
             "C_a", "C_n_L", "gimbal_angle_deg", "delta_command_left_rad", "delta_command_right_rad"]
    for tag, phase, pidx in (("pt", "landing_burn_pure_throttle", 0), ("lb", "landing_burn", 1)):
        S0, A = d[f"{tag}_state_in"][:128], d[f"{tag}_action"][:128]
        env = pd.PoweredDescentEnv(len(S0), flight_phase=phase, mode="pso")
        env.set_state(torch.tensor(S0))
        prevs = d[f"{tag}_prevs"][:128]
        if phase == "landing_burn":
            env.set_actuators(torch.tensor(prevs))
        _, _, _, _, ex = env.step(torch.tensor(A), info=True)
        for i in range(0, len(S0), 8):
            o = oracle_mod.Oracle(phase=pidx, rtd=1)
            _, info = o.physics(S0[i], A[i], f32=True, prevs=tuple(prevs[i]) if pidx else (0.0, 0.0, 0.0))
            for k in names:
                if k not in ex:
                    continue
                gv, ov = float(ex[k][i]), info[k]
                # forces built from C_L/C_D carry their absolute 1e-9 tolerance times q A_front
                scale = max(1.0, abs(ov))
                if k in FORCE_KEYS:
                    scale = max(scale, info["dynamic_pressure"] * A_FRONT)
                assert abs(gv - ov) <= 1e-9 * scale, (tag, i, k, gv, ov)


def test_c3_f32_handle_shadowed(pd, oracle_mod):
    """The binary32 handle (the throughput precision: Taylor lines and binary32 cell pieces
    through the fine index) on the c3 workload at full size, 65 536 envs x 240
    steps; 96 sampled envs teacher-forced against the binary64 oracle at every step from the
    handle's own (binary32) state: every channel within 1e-5 of max(|x|, 1) (SURVEY 8(d)'s fp32
    tolerance; the handle integrates the state chain in binary64 within the env-step) and
    theta_dot within 2.5e-4 (see the bounds below), reward within 1e-4,
    done/truncated/trunc_id equal in >= 99.5 % of the sampled steps (a binary32 quantity can sit
    on the other side of a threshold); auto-resets within 1e-6 of the oracle's (the same Philox
    draws; the binary32 reset adds the tilt in binary32) with the same wind percentile."""
    import ctypes as C
    import torch
    from shadow import snapshot, _load
    N, T, seed = 65536, 240, 1234
    A = c3_actions(T, N, 7).cuda()
    idx = c3_sample(N)
    env = c3_env(pd, N, seed=seed, precision="f32")
    L, P = oracle_mod.lib(), oracle_mod.params()
    E, E2, o = oracle_mod.OrcEnv(), oracle_mod.OrcEnv(), oracle_mod.OrcOut()
    it = torch.as_tensor(idx, device="cuda")
    snap = snapshot(env, it)
    keep = [1, 3, 8, 9, 10]
    worst = np.zeros(11)
    wrew, flips, n, resets = 0.0, 0, 0, 0
    for t in range(T):
        obs, rew, dn, tr, ex = env.step(A[t])
        after = snapshot(env, it)
        g_rew, g_dn, g_tr = rew[it].double().cpu().numpy(), dn[it].cpu().numpy(), tr[it].cpu().numpy()
        a = A[t][it].cpu().numpy().astype(np.float64)
        for j, g in enumerate(idx):
            _load(L, P, E, snap, j, 0, seed, g, -1, math.radians(1.0))
            u = (C.c_double * 4)(float(a[j, 0]), 0.0, 0.0, 0.0)
            L.orc_step(C.byref(P), C.byref(E), 0, 0, u, 1, None, C.byref(o))
            n += 1
            if bool(g_dn[j]) != bool(o.done) or bool(g_tr[j]) != bool(o.trunc):
                flips += 1
                continue
            wrew = max(wrew, abs(float(g_rew[j]) - o.reward))
            if o.done or o.trunc:
                resets += 1
                L.orc_reset_philox(C.byref(P), C.byref(E2), 0, seed, int(g), (int(snap["ep"][j]) + 1) & 0xFFFFFFFF, 1, 1,
                                   -1, math.radians(1.0))
                ref = np.array(E2.s[:])   # (the binary32 reset adds the tilt in binary32)
                assert (np.abs(after["s"][j] - ref) <= 1e-6 * np.maximum(np.abs(ref), 1.0)).all(), (t, g)
                assert int(after["prof"][j]) == E2.wind_prof and int(after["ep"][j]) == int(snap["ep"][j]) + 1
            else:
                so = np.array(E.s[:])
                worst = np.maximum(worst, np.abs(after["s"][j].astype(np.float64) - so) / np.maximum(np.abs(so), 1.0))
        snap = after
    # Bounds.  The attitude channels are where binary32 rounding is amplified most: an env near
    # max-q with |alpha_eff| ~ 1e-3 has alpha_eff = gamma - theta - pi as the difference of two
    # O(1) angles, and the aerodynamic moment over the step turns its error into theta_dot.  With
    # the angles in binary32 (round 4) one step lost theta_dot 9.3e-3, theta 1.5e-4, alpha
    # 6.9e-5, vx 4.5e-5; the handle now carries the state chain in binary64 through the env-step
    # and rounds it once, so only the binary32 forces and tables are left: measured theta_dot
    # 1.8e-4, theta 3.3e-6, every other channel <= 4e-7 (the binary32 cell pieces hold C_L to
    # 2e-6 of sum |c_j phi_j|, DESIGN.md s4, which the aerodynamic moment of an env near max-q
    # turns into theta_dot).
    att = [0, 2, 4, 6, 7]     # x, vx, theta, gamma, alpha
    res = dict(keep=float(worst[keep].max()), attitude=float(worst[att].max()), theta_dot=float(worst[5]),
               reward=wrew, flips=flips, steps=n, resets=resets, per_channel=dict(zip(ST, worst.tolist())))
    print("f32 shadow:", res)
    assert (res["keep"] <= 1e-5 and res["attitude"] <= 1e-5 and res["theta_dot"] <= 2.5e-4 and wrew <= 1e-4
            and flips <= 0.005 * n and resets >= len(idx) // 2), res
    assert env.counters()["nan_events"] == 0
