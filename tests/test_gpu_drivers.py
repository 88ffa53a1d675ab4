"""GPU tests of the drop-in facade as the two north-star drivers call it, and of the driver-side
device components at their per-GPU sizes (SURVEY configs c4 and c5).

The drivers' call sequences are restated here (the reference itself is not imported on the GPU
box): sac_pytorch_powered_descent.py:355-374 (visualize_trajectory) + :253-352
(save_trajectory_to_csv's info flattening), and particle_swarm_optimisation.py:499-506,
759-833 (plot_results, collect_trajectory_data, save_trajectory_data).
"""
import math

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pd():
    import torch
    import pdenv
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return pdenv


class _DeterministicAgent:
    """Stands in for SACPyTorch.select_action(state, deterministic=True) (sac_pytorch.py:404-409):
    a float32 action of shape (1,)."""

    def __init__(self, seq):
        self.seq, self.t = seq, 0

    def select_action(self, state, deterministic=False):
        a = np.array([self.seq[self.t % len(self.seq)]], dtype=np.float32)
        self.t += 1
        return a


def test_sac_driver_visualize_trajectory_sequence(pd, oracle_mod):
    """visualize_trajectory's loop over the facade, with the driver's imports swapped to pdenv:
    info['state'], info['dynamic_pressure'], info['action_info']['throttle'] and
    maximum_velocity_lambda(y, vy) per step; then save_trajectory_to_csv's flattening of every
    scalar and nested info key.  maximum_velocity equals the oracle ISA's sqrt(2p/rho)."""
    from pdenv.wrappers import maximum_velocity as maximum_velocity_lambda
    from pdenv.wrappers import rl_wrapped_env_pytorch
    env = rl_wrapped_env_pytorch(flight_phase="landing_burn_pure_throttle", enable_wind=False,
                                 stochastic_wind=False, trajectory_length=1, discount_factor=0.99)
    agent = _DeterministicAgent(np.random.default_rng(3).uniform(-1, 1, 4000))
    state = env.reset()
    states, rewards, dynamic_pressure, throttle_command, maximum_velocity, infos = [], [], [], [], [], []
    done = truncated = False
    while not (done or truncated):
        action = agent.select_action(state, deterministic=True)
        next_state, reward, done, truncated, info = env.step(action)
        raw_state = info["state"]
        states.append(raw_state)
        rewards.append(reward)
        dynamic_pressure.append(info["dynamic_pressure"])
        throttle_command.append(info["action_info"]["throttle"])
        maximum_velocity.append(maximum_velocity_lambda(raw_state[1], raw_state[3]))
        infos.append(info)
        state = next_state
    assert len(states) > 10
    for k in (0, len(states) // 2, len(states) - 1):
        rho, p, a = oracle_mod.atmosphere(states[k][1])
        ref = math.sqrt(2 * p / rho) if a != 0 else states[k][3]
        assert abs(maximum_velocity[k] - ref) <= 1e-12 * ref
    # save_trajectory_to_csv (sac_pytorch_powered_descent.py:300-341): scalar and nested keys
    scalar, nested = set(), {}
    for info in infos:
        for key, value in info.items():
            if key in ("state", "actions"):
                continue
            if isinstance(value, dict):
                nested.setdefault(key, set()).update(k for k, v in value.items() if k != "throttle" and np.isscalar(v))
            elif np.isscalar(value):
                scalar.add(key)
    cols = scalar | {f"{k}_{s}" for k, ss in nested.items() for s in ss}
    for c in ("air_density", "mach_number_max", "drag", "lift", "fuel_percentage_consumed", "gravity_force_y",
              "g_load_1_sec_window", "acceleration_dict_acceleration_x_component_drag",
              "acceleration_dict_acceleration_y_component_wind", "moment_dict_theta_dot_dot"):
        assert c in cols, c
    assert len(cols) >= 40, sorted(cols)


def test_info_tap_vs_recorded_sac_trajectory(pd):
    """The info tap against the reference's own recorded SAC runs (data/agent_saves/.../
    trajectory.csv columns): each recorded row teacher-forced from the previous row's state with
    the recorded action, every env of one batched pd_step; air density, speed of sound, Mach,
    C_D, C_L, mass flow, dynamic pressure, x_cog, inertia, d_thrust_cg, alpha_effective,
    control force, throttle."""
    import torch
    from pdenv.wrappers import info_dict
    d = golden("recorded_sac_trajectories.npz")
    names = list(d["info_names"])
    S, A, I = d["run0_state"], d["run0_action"], d["run0_info"]
    rows = np.arange(1, min(len(S), 400))
    env = pd.PoweredDescentEnv(len(rows), flight_phase="landing_burn_pure_throttle", mode="rl")
    env.set_state(torch.tensor(S[rows - 1]))
    _, _, _, _, ex = env.step(torch.tensor(A[rows].astype(np.float32)[:, None]), info=True)
    st = env.state.cpu().numpy()
    exc = {k: v.cpu() for k, v in ex.items() if k != "trunc_id"}
    for j, t in enumerate(rows[::7]):
        i = int(np.nonzero(rows == t)[0][0])
        info = info_dict("landing_burn_pure_throttle", exc, st[i], A[t], env.params, i=i)
        for k in names:
            if k in ("g_load_1_sec_window",):
                continue
            ref = I[t, names.index(k)]
            got = info["action_info"]["throttle"] if k == "throttle" else info[k]
            assert abs(got - ref) <= 1e-8 * max(1.0, abs(ref)), (t, k, got, ref)


def test_pso_driver_collect_trajectory_and_plot_results(pd, tmp_path):
    """The PSO driver's save-interval block against the facade: model.plot_results(best, dir + '/')
    writes the episode (trajectory.csv, Simulation.png); collect_trajectory_data's loop over
    model.env.reset/step with model.actor.forward; save_trajectory_data's flatten_dict of the
    info into info_data columns."""
    import pandas as pd_
    from pdenv.wrappers import pso_wrapped_env
    model = pso_wrapped_env(flight_phase="landing_burn")
    ind = np.random.default_rng(2).uniform(-0.3, 0.3, len(model.bounds))
    rows = model.plot_results(ind, str(tmp_path) + "/")
    assert (tmp_path / "trajectory.csv").exists()
    df = pd_.read_csv(tmp_path / "trajectory.csv")
    assert len(df) == len(rows) > 0 and "action_info_acs_info_F_parallel" in df.columns
    # collect_trajectory_data (particle_swarm_optimisation.py:759-784)
    model.individual_update_model(ind)
    state = model.env.reset()
    traj = {"states": [], "actions": [], "rewards": [], "info": []}
    done_or_truncated = False
    while not done_or_truncated:
        action = model.actor.forward(state)
        next_state, reward, done, truncated, info = model.env.step(action)
        traj["states"].append(state.tolist() if hasattr(state, "tolist") else state)
        traj["actions"].append(action.detach().numpy().tolist())
        traj["rewards"].append(reward)
        traj["info"].append(info)
        done_or_truncated = done or truncated
        state = next_state
    assert len(traj["rewards"]) == len(rows)
    assert np.allclose(traj["rewards"], df["reward"].values, rtol=0, atol=0)
    # save_trajectory_data's flatten_dict (:800-807)
    flat = []
    for info in traj["info"]:
        fi = {}

        def flatten_dict(dd, prefix=""):
            for key, value in dd.items():
                if isinstance(value, dict):
                    flatten_dict(value, f"{prefix}{key}_")
                else:
                    fi[f"{prefix}{key}"] = value
        flatten_dict(info)
        flat.append(fi)
    cols = set(flat[0])
    for c in ("action_info_gimbal_angle_deg", "action_info_delta_command_left_rad", "action_info_acs_info_Mz",
              "acceleration_dict_acceleration_x_component_control", "moment_dict_control_moment_z", "state"):
        assert c in cols, c


def test_prioritized_buffer_on_device(pd):
    """DevicePrioritizedReplayBuffer on the GPU (the SAC driver's buffer, sac_pytorch.py:51-127):
    pair probabilities of np.random.choice(size, 2, replace=False, p=prio**alpha) by Gumbel-top-k,
    importance weights (size p)^-beta / max, beta annealing, priority updates and max tracking."""
    import itertools
    import torch
    from pdenv.sac import DevicePrioritizedReplayBuffer
    buf = DevicePrioritizedReplayBuffer(8, 1, 1, "cuda", alpha=0.6, beta=0.4, beta_annealing_steps=10)
    buf.add_batch(torch.arange(25, dtype=torch.float32, device="cuda").reshape(5, 5))
    assert torch.equal(buf.priorities[:5].cpu(), torch.ones(5))
    buf.update_priorities(torch.arange(5, device="cuda"), torch.tensor([0.5, 1.0, 2.0, 4.0, 8.0], device="cuda"))
    assert buf.max_priority == pytest.approx(8.0 + 1e-6)
    p = (np.array([0.5, 1.0, 2.0, 4.0, 8.0]) + 1e-6) ** 0.6
    p /= p.sum()
    exact = {(i, j): p[i] * p[j] / (1 - p[i]) for i, j in itertools.permutations(range(5), 2)}
    g = torch.Generator(device="cuda").manual_seed(0)
    T = 20000
    idxs = []
    beta0 = buf.beta
    for _ in range(T):
        s, a, r, s2, d, w, idx = buf.sample(2, generator=g)
        idxs.append(idx)
    assert buf.beta == pytest.approx(min(1.0, beta0 + T * (1 - 0.4) / 10))
    I = torch.stack(idxs).cpu().numpy()
    for k, e in exact.items():
        f = np.mean((I[:, 0] == k[0]) & (I[:, 1] == k[1]))
        assert abs(f - e) < 5 * np.sqrt(e * (1 - e) / T) + 1e-3, (k, f, e)
    wr = (5 * p[idx.cpu().numpy()]) ** (-1.0)
    assert np.allclose(w.cpu().numpy().ravel(), wr / wr.max(), rtol=1e-6)
    # new transitions enter at the current max priority (sac_pytorch.py:84-85)
    buf.add_batch(torch.zeros(2, 5, device="cuda"))
    assert torch.allclose(buf.priorities[5:7].cpu(), torch.full((2,), 8.0 + 1e-6))


def test_c5_collector_4096_envs_prioritized(pd):
    """c5's per-GPU share: 4 096 envs, the reference Actor (2-256-256-1), HIP-graph collection into
    the device prioritized buffer (1e6, the driver's size): 220 steps with auto-resets, then the
    learner's sample -> update_priorities round trip."""
    import torch
    from pdenv.sac import Actor, DevicePrioritizedReplayBuffer, SACCollector
    torch.manual_seed(0)
    N = 4096
    env = pd.PoweredDescentEnv(N, flight_phase="landing_burn_pure_throttle", mode="rl", auto_reset=True, seed=8)
    actor = Actor(2, 1).cuda()
    buf = DevicePrioritizedReplayBuffer(1_000_000, 2, 1, "cuda")
    col = SACCollector(env, actor, buf, use_graph=True)
    for _ in range(220):
        col.step()
    torch.cuda.synchronize()
    assert len(buf) == 220 * N
    assert torch.isfinite(buf.data[:len(buf)]).all()
    assert (buf.data[:len(buf), 2].abs() <= 1).all()                 # tanh-squashed actions
    assert float(buf.data[:len(buf), 6].sum()) >= 0                   # done flags are 0/1
    g = torch.Generator(device="cuda").manual_seed(1)
    s, a, r, s2, d, w, idx = buf.sample(256, generator=g)
    assert s.shape == (256, 2) and w.shape == (256, 1) and len(torch.unique(idx)) == 256
    assert float(w.max()) == pytest.approx(1.0) and float(w.min()) > 0
    buf.update_priorities(idx, torch.linspace(0, 5, 256, device="cuda"))
    assert buf.max_priority == pytest.approx(5 + 1e-6)
    t = env.state[:, 10]
    assert (t < t.max() - 1.0).any()                                  # episodes ended and restarted


def test_c4_per_gpu_share_32768_particles(pd, oracle_mod):
    """c4's per-GPU share: 32 768 particles, landing_burn, 372-parameter actors ~ U(-1.5, 1.5),
    max_steps 2200: every episode ends within the cap, fitness finite, and 48 sampled particles
    equal the oracle's objective; then one device swarm update.  (At this size N x LPE fits one
    chip round, so the compacted list is not used; test_gpu_parity.py forces it.)"""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    opt = ParticleSubswarmOptimisationGPU("landing_burn", pop_size=32768, seed=3,
                                          pso_params=dict(generations=4, re_initialise_generation=-1))
    fit, steps = opt.evaluate(opt.x32)
    f, s = fit.cpu().numpy(), steps.cpu().numpy()
    assert np.isfinite(f).all() and (s >= 1).all() and (s <= 2200).all()
    pick = np.linspace(0, 32767, 48).astype(int)
    W = opt.x32[:, pick].t().contiguous().cpu().numpy()
    of, os_ = oracle_mod.rollout_policy(1, W, 2200)
    rel = np.abs(f[pick] - of) / np.abs(of)
    # tumbling landing_burn vehicles amplify 1e-13 RBF differences: ensemble bounds (as the
    # 64-particle test in test_gpu_parity.py)
    assert (s[pick] == os_).mean() >= 0.8 and (rel < 1e-6).mean() >= 0.8 and np.median(rel) < 1e-9, rel
    x0 = opt.x.clone()
    opt.generation(0)
    assert not torch.equal(x0, opt.x) and bool((opt.x.abs() <= 1.5).all())


def test_c4_policy_rollout_shadowed(pd, oracle_mod):
    """c4's per-GPU share (32 768 landing_burn particles ~ U(-1.5, 1.5), the fused actor +
    compaction kernel) teacher-forced at EVERY policy step until every sampled episode ends: 128
    sampled particles (both ends of the batch and spread through it); per step the oracle's
    actor + env step from the device's complete state must equal the device's next state,
    reward, done/truncated and truncation id (tests/shadow.py shadow_policy).  The ensemble
    bounds of test_c4_per_gpu_share_32768_particles stay as a secondary, free-running check."""
    import torch
    from shadow import policy_snapshots, shadow_policy, TOL_STEP, ST
    N = 32768
    W = np.random.default_rng(17).uniform(-1.5, 1.5, (N, 372)).astype(np.float32)
    env = pd.PoweredDescentEnv(N, flight_phase="landing_burn", mode="pso")
    _, steps = env.rollout_policy(torch.tensor(W), max_steps=2200)
    idx = np.unique(np.concatenate([np.arange(16), np.arange(N - 16, N), np.linspace(16, N - 17, 96).astype(int)]))
    K = int(steps.cpu().numpy()[idx].max()) + 1
    assert K <= 400, K                      # (the sampled episodes all end: snapshots cost O(K^2) steps)
    snaps = policy_snapshots(env, W, K)
    assert (snaps[K]["steps"][idx] < K).all()
    st = shadow_policy(oracle_mod, snaps, W, idx, 1)
    bad = {ST[k]: float(st["max_err"][k]) for k in range(11) if st["max_err"][k] > TOL_STEP[k]}
    assert not bad, bad
    assert st["ended"] == len(idx), (st["ended"], len(idx))     # every sampled episode followed to its end
    assert st["steps"] >= 10 * len(idx), st["steps"]
