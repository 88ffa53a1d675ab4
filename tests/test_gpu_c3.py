"""GPU parity of the headline workload (BASELINE config c3) and of the per-env bookkeeping.

c3 = 65 536 envs, landing_burn_pure_throttle with the SAC driver's reward, the horizontal wind
profile of a percentile drawn per reset (WindModel(given_percentile=None),
full_wind_model.py:27-33) plus von Karman gusts (vonkarman.py:33-36), a pitch tilt N(0, 1 deg)
at every reset, and auto-reset.  The reference draws its randomness from np.random with
seed(None) (vonkarman.py:88), so no run of it can be replayed; the oracle instead restates the
device's Philox4x32-10 draw scheme (oracle/pd_oracle.c orc_reset_philox / orc_gauss_pair), and
sampled envs of the full-size GPU run are followed env for env.  The oracle's wind model itself
is pinned to the reference by tests/test_oracle_golden.py (recorded normals, every percentile).

Tolerances (f64 handle): per-step reward <= 1e-9 absolute, done/truncated/trunc_id exact, obs
<= 1e-6 (float32-cast state), final state <= 1e-8 relative on y, vy, masses, time, <= 1e-6 on the
attitude channels (chaotic).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ST = ["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass", "mass_propellant", "time"]
TOL_STATE = np.array([1e-6, 1e-8, 1e-6, 1e-8, 1e-6, 1e-6, 1e-6, 1e-6, 1e-10, 1e-10, 1e-12])


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


def test_c3_full_size_vs_oracle(pd, oracle_mod):
    """65 536 envs x 200 steps of the c3 workload through pd_step_n (16 steps per launch, state in
    registers across the fused steps); 96 sampled envs (both ends of the batch, and spread
    through it) followed by the oracle under the same draws: every step's reward, done,
    truncated, trunc_id and observation, and the final state."""
    import torch
    N, T = 65536, 200
    g = torch.Generator().manual_seed(7)
    A = (torch.rand(T, N, 1, generator=g) * 2 - 1).contiguous()
    env = c3_env(pd, N)
    _, _, prof0 = env.wind_state()
    obs, rew, dn, tr, tid = env.step_n(A.cuda())
    idx = np.unique(np.concatenate([np.arange(16), np.arange(N - 16, N), np.linspace(16, N - 17, 64).astype(int)]))
    it = torch.tensor(idx, device=obs.device)
    got = dict(reward=rew[:, it].cpu().numpy(), done=dn[:, it].cpu().numpy(), trunc=tr[:, it].cpu().numpy(),
               trunc_id=tid[:, it].cpu().numpy(), obs=obs[:, it].cpu().numpy())
    S = env.state[it].cpu().numpy()
    prof = prof0[it].cpu().numpy()
    o = oracle_mod.rollout_philox(0, 0, idx, np.zeros(len(idx)), A[:, idx].numpy(), auto_reset=True, wind=True,
                                  stochastic=True, fixed_prof=-1, tilt=math.radians(1.0), seed=1234, obs_dim=2)
    # coverage: resets happened, the sample spans many percentiles
    assert (got["done"] | got["trunc"]).sum() >= len(idx), "every sampled env should end an episode"
    assert len(set(prof.tolist())) >= 20, sorted(set(prof.tolist()))
    assert np.array_equal(got["done"].astype(bool), o["done"].astype(bool))
    assert np.array_equal(got["trunc"].astype(bool), o["trunc"].astype(bool))
    assert np.array_equal(got["trunc_id"], o["trunc_id"])
    assert np.abs(got["reward"] - o["reward"]).max() <= 1e-9
    assert np.abs(got["obs"] - o["obs"]).max() <= 1e-6
    err = np.abs(S - o["state"]) / np.maximum(np.abs(o["state"]), 1e-3)
    assert (err.max(0) <= TOL_STATE).all(), dict(zip(ST, err.max(0)))
    assert env.counters()["nan_events"] == 0


def test_c3_full_size_properties(pd):
    """The whole 65 536-env batch of the c3 workload, per step: time advances by exactly 0.1 s,
    propellant never grows, and every env that ended is back at the initial state with its own
    tilt (theta perturbed, alpha = theta - gamma, all other channels the nominal ones)."""
    import torch
    N, T = 65536, 200
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
def test_fixed_percentile_profiles_vs_oracle(pd, oracle_mod, percentile):
    """Each percentile's horizontal profile (HorizontalWindSpeed.py:44-114) with gusts, 64 envs x
    150 steps, against the oracle on the same draws (the profiles are pinned to the reference by
    tests/test_oracle_golden.py::test_wind_profiles_every_percentile)."""
    import torch
    N, T = 64, 150
    A = (torch.rand(T, N, 1, generator=torch.Generator().manual_seed(percentile)) * 2 - 1).contiguous()
    env = c3_env(pd, N, seed=5, wind_percentile=percentile)
    obs, rew, dn, tr, tid = env.step_n(A.cuda())
    o = oracle_mod.rollout_philox(0, 0, np.arange(N), np.zeros(N), A.numpy(), wind=True, stochastic=True,
                                  fixed_prof=percentile - 50, tilt=math.radians(1.0), seed=5, obs_dim=2)
    assert np.array_equal(dn.cpu().numpy().astype(bool), o["done"].astype(bool))
    assert np.array_equal(tid.cpu().numpy(), o["trunc_id"])
    assert np.abs(rew.cpu().numpy() - o["reward"]).max() <= 1e-9
    S = env.state.cpu().numpy()
    err = np.abs(S - o["state"]) / np.maximum(np.abs(o["state"]), 1e-3)
    assert (err.max(0) <= TOL_STATE).all(), dict(zip(ST, err.max(0)))
    assert (env.wind_state()[2].cpu().numpy() == percentile).all()


def test_landing_burn_wind_vs_oracle(pd, oracle_mod):
    """The PSO driver's phase (landing_burn, 4 actions, actuator memory) with the c3 wind and
    tilt: 256 envs x 60 steps against the oracle under the same draws."""
    import torch
    N, T = 256, 60
    A = (torch.rand(T, N, 4, generator=torch.Generator().manual_seed(3)) * 2 - 1).contiguous()
    env = c3_env(pd, N, seed=11, flight_phase="landing_burn", mode="pso")
    obs, rew, dn, tr, tid = env.step_n(A.cuda())
    o = oracle_mod.rollout_philox(1, 1, np.arange(N), np.zeros(N), A.numpy(), wind=True, stochastic=True,
                                  fixed_prof=-1, tilt=math.radians(1.0), seed=11, obs_dim=5)
    d_ok = (dn.cpu().numpy().astype(bool) == o["done"].astype(bool)).all(0) & \
        (tid.cpu().numpy() == o["trunc_id"]).all(0)
    # tumbling landing_burn vehicles amplify last-ulp differences: bounds on the ensemble
    assert d_ok.mean() >= 0.95, d_ok.mean()
    r_ok = (np.abs(rew.cpu().numpy() - o["reward"]) <= 1e-6 * np.maximum(1, np.abs(o["reward"]))).all(0)
    assert r_ok.mean() >= 0.95, r_ok.mean()


def test_checkpoint_restore_continues_bit_identically(pd):
    """Stop a wind + tilt + random-percentile run mid-episode, checkpoint every per-env buffer
    (state, g-load window, actuators, wind filters/sigmas/percentile, episode and step counters,
    aero caches), restore into a fresh handle, and continue: outputs and state bit-identical."""
    import torch
    N, T1, T2 = 4096, 37, 45
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
                assert abs(gv - ov) <= 1e-9 * max(1.0, abs(ov)), (tag, i, k, gv, ov)
