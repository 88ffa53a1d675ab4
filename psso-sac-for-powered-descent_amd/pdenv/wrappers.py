"""Drop-in facades with the reference's class names, constructor kwargs and return types.

    from pdenv.wrappers import rl_wrapped_env_pytorch      # was src.envs.rl.env_wrapped_rl_pytorch
    from pdenv.wrappers import pso_wrapped_env             # was src.envs.pso.env_wrapped_ea

With one env they return exactly what the reference returns (numpy observations, Python
float/bool, an info dict); all physics runs in libpdenv.so on the GPU.  The batched entry
points (`PoweredDescentEnv`, `pso_wrapped_env.objective_function_batch`) keep everything on
the device for thousands of envs / particles.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .env import PoweredDescentEnv


def _acs_info(v, q_s):
    """acs_model.py:62-86 from the kernel's ACS quantities (qS = dynamic_pressure * grid_fin_area)."""
    dl, dr, ca, cnl, cnr = v["delta_left_rad"], v["delta_right_rad"], v["C_a"], v["C_n_L"], v["C_n_R"]
    th, ae = v["theta_in"], v["alpha_effective"]
    fpar, fperp = v["gf_F_parallel"], v["gf_F_perpendicular"]
    return {
        "alpha_local_left_rad": ae - dl, "alpha_local_right_rad": ae - dr,
        "C_n_L": cnl, "C_a_L": ca, "C_n_R": cnr, "C_a_R": ca,
        "F_n_L": cnl * q_s, "F_a_L": ca * q_s, "F_n_R": cnr * q_s, "F_a_R": ca * q_s,
        "F_perpendicular_L": q_s * (cnl * math.cos(dl) - ca * math.sin(dl)),
        "F_perpendicular_R": q_s * (cnr * math.cos(dr) - ca * math.sin(dr)),
        "F_perpendicular": fperp,
        "F_parallel_L": q_s * (ca * math.cos(dl) + cnl * math.sin(dl)),
        "F_parallel_R": q_s * (ca * math.cos(dr) + cnr * math.sin(dr)),
        "F_parallel": fpar,
        "Fx": fpar * math.cos(th) + fperp * math.sin(th),
        "Fy": fpar * math.sin(th) - fperp * math.cos(th),
        "Mz": v["gf_Mz"], "d_fin_cg": v["_d_base_gf"] - v["x_cog"],
        "delta_left_rad": dl, "delta_right_rad": dr,
    }


def info_dict(flight_phase, ex, state, actions, params, i=0):
    """The info dict of rocket_physics_fcn (rockets_physics.py:649-702) + the env's keys
    (base_environment.py:134-149) for env i, built from pd_step's info tap (the last sub-step's
    quantities, include/pdenv.h pd_info_field) and the post-step state.  Entries that are
    arithmetic of those (accelerations, F_n = C_n qS, ...) are formed here as the reference forms
    them; trigonometric ones may differ from the reference's in the last ulp."""
    v = {k: float(ex[k][i]) for k in L.INFO_FIELDS if k in ex}
    v["_d_base_gf"] = float(params.struct.d_base_grid_fin)
    s = [float(x) for x in state]
    mass, gamma = s[8], s[6]
    g, drag, lift = v["gravity"], v["drag"], v["lift"]
    acc = {
        "acceleration_x_component_control": v["control_force_x"] / mass,
        "acceleration_y_component_control": v["control_force_y"] / mass,
        "acceleration_x_component_drag": -drag * math.cos(gamma) / mass,
        "acceleration_y_component_drag": -drag / mass * math.sin(gamma) / mass,
        "acceleration_x_component_lift": -lift * math.cos(math.pi - gamma) / mass,
        "acceleration_y_component_lift": lift * math.sin(math.pi - gamma) / mass,
        "acceleration_x_component_gravity": 0,
        "acceleration_y_component_gravity": -g,
        "acceleration_x_component": v["vx_dot"],
        "acceleration_y_component": v["vy_dot"],
        "acceleration_x_component_wind": v["F_wind_x"] / mass,
        "acceleration_y_component_wind": v["F_wind_y"] / mass,
    }
    mom = {"control_moment_z": v["control_moment_z"], "aero_moment_z": v["aero_moment_z"],
           "moments_z": v["moments_z"], "theta_dot_dot": v["theta_dot_dot"], "M_wind_z": v["M_wind_z"]}
    q_s = v["dynamic_pressure"] * float(params.struct.grid_fin_area)
    if flight_phase in ("landing_burn_pure_throttle", "landing_burn_pure_throttle_Pcontrol"):
        ai = {"throttle": v["throttle"], "acs_info": _acs_info(v, q_s)}
    elif flight_phase == "landing_burn":
        ai = {"throttle": v["throttle"], "delta_command_left_rad": v["delta_command_left_rad"],
              "delta_command_right_rad": v["delta_command_right_rad"], "gimbal_angle_deg": v["gimbal_angle_deg"],
              "acs_info": _acs_info(v, q_s)}
    elif flight_phase in ("subsonic", "supersonic"):
        ai = {"gimbal_angle_deg": v["gimbal_angle_deg"], "throttle": v["throttle"]}
    elif flight_phase == "flip_over_boostbackburn":
        ai = {"gimbal_angle_deg": v["gimbal_angle_deg"]}
    else:
        ai = {"RCS_throttle": actions}
    info = {
        "inertia": v["inertia"], "acceleration_dict": acc, "mach_number": v["mach_number"],
        "mach_number_max": v["mach_number_max"], "CL": v["CL"], "CD": v["CD"], "drag": drag, "lift": lift,
        "moment_dict": mom, "d_cp_cg": v["d_cp_cg"], "d_thrust_cg": v["d_thrust_cg"], "x_cog": v["x_cog"],
        "dynamic_pressure": v["dynamic_pressure"], "mass_flow": v["mass_flow"],
        "fuel_percentage_consumed": v["fuel_percentage_consumed"],
        "control_force_parallel": v["control_force_parallel"],
        "control_force_perpendicular": v["control_force_perpendicular"],
        "control_force_x": v["control_force_x"], "control_force_y": v["control_force_y"],
        "aero_force_x": v["aero_force_x"], "aero_force_y": v["aero_force_y"], "gravity_force_y": -g * mass,
        "atmospheric_pressure": v["atmospheric_pressure"], "air_density": v["air_density"],
        "speed_of_sound": v["speed_of_sound"], "action_info": ai, "ug": v["ug"], "vg": v["vg"],
        "alpha_effective": v["alpha_effective"],
        "state": s, "actions": actions, "g_load_1_sec_window": v["g_load_1_sec_window"],
    }
    return info


_ATM = {}


def _atm_env(device):
    """One 1-env handle per device for the scalar ISA helper, closed at interpreter exit."""
    if device not in _ATM:
        if not _ATM:
            import atexit
            atexit.register(lambda: [e.close() for e in _ATM.values()])
        _ATM[device] = PoweredDescentEnv(1, "landing_burn_pure_throttle", mode="rl", device=device)
    return _ATM[device]


def maximum_velocity(y, vy, device=None):
    """env_wrapped_rl_pytorch.py:60-66: sqrt(2 p / rho) of the ISA at altitude y (the handle's
    device atmosphere, pd_atmosphere), or vy above the ISA's top.  The SAC driver imports it as
    maximum_velocity_lambda (sac_pytorch_powered_descent.py:11, used at :370).  Evaluated on
    `device` (default: the current torch device, so each rank of a multi-GPU job uses its own)."""
    dev = torch.cuda.current_device() if device is None else int(device)
    rho, p, a = _atm_env(dev).atmosphere(torch.tensor([float(y)], dtype=torch.float64))
    rho, p, a = float(rho[0]), float(p[0]), float(a[0])
    if a != 0:
        return math.sqrt(2 * p / rho)
    return vy


# state_dim / action_dim per phase (env_wrapped_rl_pytorch.py:87-104)
RL_DIMS = {"subsonic": (8, 2), "supersonic": (8, 2), "flip_over_boostbackburn": (2, 1),
           "ballistic_arc_descent": (4, 1), "landing_burn": (5, 4), "landing_burn_ACS": (5, 3),
           "landing_burn_pure_throttle": (2, 1), "landing_burn_pure_throttle_Pcontrol": (1, 1)}


def augment_action(flight_phase, actions, speed0=None):
    """rl_wrapped_env_pytorch.augment_action (env_wrapped_rl_pytorch.py:120-165) on a batch of
    float32 policy actions [N, A] (device tensor) -> the actions the env receives.

    landing_burn: u' = sign(u) log(1 + c|u|)/log(1 + c), c = 10 (gimbal) / 5 (fins), u1 as is.
        NumPy keeps c*|u| and 1 + c|u| in float32 (NEP 50); math.log and the division are
        binary64, and np.array([...]) of the mix is float64 -> float64 actions.
    landing_burn_pure_throttle_Pcontrol: v_ref = (u + 1)/2 * speed0, all float32.
    other phases: unchanged (float32)."""
    a = actions.to(torch.float32)
    if flight_phase == "landing_burn":
        def comp(u, c):
            t = 1.0 + c * u.abs()                                   # float32 (NEP 50)
            return torch.copysign(torch.log(t.double()) / math.log(1 + c), u.double())
        return torch.stack([comp(a[:, 0], 10.0), a[:, 1].double(), comp(a[:, 2], 5.0), comp(a[:, 3], 5.0)], 1)
    if flight_phase == "landing_burn_pure_throttle_Pcontrol":
        return (a + 1.0) / 2.0 * torch.tensor(speed0, dtype=torch.float32, device=a.device)
    return a


class rl_wrapped_env_pytorch:
    """env_wrapped_rl_pytorch.py:68-205 for every flight phase (the SAC driver's is
    landing_burn_pure_throttle).

    step(action) -> (obs float64[state_dim], float reward, bool done, bool truncated, info dict).
    Actions are taken as float32, the dtype SACPyTorch.select_action returns
    (sac_pytorch.py:404-409), and augmented as the reference's wrapper does (augment_action);
    pass action_f64=True to reproduce float64 callers of the pure-throttle phase.
    flip_over_boostbackburn and landing_burn_ACS construct, and raise TypeError at step() as the
    reference's do."""

    def __init__(self, flight_phase="subsonic", enable_wind=False, stochastic_wind=True,
                 horiontal_wind_percentile=50, trajectory_length=None, discount_factor=None,
                 precision="f64", device=0, seed=0, action_f64=False):
        if flight_phase not in RL_DIMS:
            raise AssertionError(f"unknown flight_phase {flight_phase!r}")
        self.flight_phase = flight_phase
        self.enable_wind = enable_wind
        self.state_dim, self.action_dim = RL_DIMS[flight_phase]
        # landing_burn's augmented actions are float64 arrays (np.array of Python floats)
        f64 = action_f64 or flight_phase == "landing_burn"
        self.env = PoweredDescentEnv(1, flight_phase, mode="rl", precision=precision, device=device,
                                     enable_wind=enable_wind, stochastic_wind=stochastic_wind,
                                     wind_percentile=horiontal_wind_percentile, seed=seed,
                                     action_f64=f64, discount_factor=discount_factor,
                                     trajectory_length=trajectory_length)
        self.speed0 = self.env.params.speed0_pcontrol if not self.env.unsteppable else None
        self._state = None

    def reset(self):
        obs = self.env.reset()
        return None if obs is None else obs[0].double().cpu().numpy()

    def augment_action(self, actions):
        return augment_action(self.flight_phase, actions, self.speed0)

    def step(self, action):
        self.env._check_steppable()
        if isinstance(action, torch.Tensor):
            a = action.detach()
        else:
            a = torch.as_tensor(np.asarray(action))
        a = a.reshape(-1)[:self.action_dim].reshape(1, self.action_dim).to(self.env.device)
        if self.flight_phase in ("landing_burn", "landing_burn_pure_throttle_Pcontrol"):
            a = self.augment_action(a)
        obs, r, d, tr, ex = self.env.step(a, info=True)
        state = self.env.state[0].cpu().numpy()
        self._tid = int(ex["trunc_id"][0])
        info = info_dict(self.flight_phase, {k: v.cpu() for k, v in ex.items() if k != "trunc_id"}, state,
                         a.cpu().numpy(), self.env.params)
        return obs[0].double().cpu().numpy(), float(r[0]), bool(d[0]), bool(tr[0]), info

    def truncation_id(self):
        return getattr(self, "_tid", 0)

    def render(self):
        pass

    def close(self):
        self.env.close()


class simple_actor:
    """env_wrapped_ea.py:18-75: Linear(in,h)-ReLU-[Linear(h,h)-ReLU]xL-Linear(h,out)-Tanh."""

    def __init__(self, number_of_hidden_layers=15, hidden_dim=10, output_dim=2, input_dim=7, flight_phase="subsonic"):
        self.number_of_hidden_layers, self.hidden_dim = number_of_hidden_layers, hidden_dim
        self.output_dim, self.input_dim = output_dim, input_dim
        self.network = nn.Sequential(
            nn.Linear(input_dim, hidden_dim), nn.ReLU(),
            *[nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.ReLU()) for _ in range(number_of_hidden_layers)],
            nn.Linear(hidden_dim, output_dim), nn.Tanh())
        self.number_of_network_parameters = sum(p.numel() for p in self.network.parameters())

    def forward(self, state):
        if not isinstance(state, torch.Tensor):
            state = torch.tensor(state, dtype=torch.float32)
        return self.network(state)

    def update_individiual(self, individual):
        idx = 0
        for name, param in self.network.named_parameters():
            n = param.numel()
            param.data = torch.tensor(individual[idx:idx + n], dtype=torch.float32).view(param.shape)
            idx += n

    def return_setup_vals(self):
        d, bounds = {}, []
        for name, param in self.network.named_parameters():
            for j, v in enumerate(param.data.flatten().tolist()):
                d[f'{name.replace(".", "_")}_{j}'] = v
                bounds.append((-1.5, 1.5))
        return d, bounds

    def shapes(self):
        """(out, in) of every Linear in forward order."""
        return [(m.out_features, m.in_features) for m in self.network.modules() if isinstance(m, nn.Linear)]


_ACTOR = {"landing_burn_pure_throttle": dict(input_dim=2, output_dim=1, number_of_hidden_layers=3, hidden_dim=8),
          "landing_burn": dict(input_dim=5, output_dim=4, number_of_hidden_layers=4, hidden_dim=8)}


class pso_wrapper:
    """env_wrapped_ea.py:77-134 (one env)."""

    def __init__(self, flight_phase="landing_burn", enable_wind=False, stochastic_wind=False,
                 horiontal_wind_percentile=95, device=0, precision="f64", seed=0):
        if flight_phase not in _ACTOR:
            raise NotImplementedError("PSO facade covers 'landing_burn' and 'landing_burn_pure_throttle'")
        self.flight_phase, self.enable_wind = flight_phase, enable_wind
        self.env = PoweredDescentEnv(1, flight_phase, mode="pso", precision=precision, device=device,
                                     enable_wind=enable_wind, stochastic_wind=stochastic_wind,
                                     wind_percentile=horiontal_wind_percentile, seed=seed)
        self.initial_mass = float(self.env.params.state0[9])

    def truncation_id(self):
        return getattr(self, "_tid", 0)

    def step(self, action):
        """env_wrapped_ea.py:125-129: (augmented state, reward, done, truncated, info) with the full
        info dict of rocket_physics_fcn (the PSO driver's collect_trajectory_data /
        save_trajectory_data flatten it, particle_swarm_optimisation.py:759-833)."""
        a = action.detach().reshape(1, -1).float()
        obs, r, d, tr, ex = self.env.step(a, info=True)
        self._tid = int(ex["trunc_id"][0])
        state = self.env.state[0].cpu().numpy()
        info = info_dict(self.flight_phase, {k: v.cpu() for k, v in ex.items() if k != "trunc_id"}, state,
                         action.detach().cpu().numpy(), self.env.params)
        return obs[0].double().cpu().numpy(), float(r[0]), bool(d[0]), bool(tr[0]), info

    def reset(self):
        return self.env.reset()[0].double().cpu().numpy()


class pso_wrapped_env:
    """env_wrapped_ea.py:137-229: objective_function(individual) = -sum(rewards) of one episode
    driven by the particle's actor; objective_function_batch evaluates P particles at once on
    the device (P envs, batched actor)."""

    def __init__(self, flight_phase="landing_burn", enable_wind=False, stochastic_wind=False,
                 horiontal_wind_percentile=50, device=0, precision="f64", seed=0):
        self.enable_wind, self.flight_phase = enable_wind, flight_phase
        self.device, self.precision, self.seed = device, precision, seed
        self.wind = (enable_wind, stochastic_wind, horiontal_wind_percentile)
        self.env = pso_wrapper(flight_phase, enable_wind, stochastic_wind, horiontal_wind_percentile,
                               device=device, precision=precision, seed=seed)
        self.actor = simple_actor(flight_phase=flight_phase, **_ACTOR[flight_phase])
        self.mock_dictionary_of_opt_params, self.bounds = self.actor.return_setup_vals()
        self.experience_buffer = []
        self.episode_idx = 0
        self._batch_env = None

    def individual_update_model(self, individual):
        self.actor.update_individiual(individual)

    def reset(self):
        self.env.reset()
        self.experience_buffer = []

    def objective_function(self, individual, max_steps=None):
        """env_wrapped_ea.py:199-222, including its experience_buffer tuples: from the second step
        on, (state after the previous step, previous action, previous reward, state after this
        step, this action) -- the reference's own pairing, kept as is."""
        self.individual_update_model(individual)
        state = self.env.reset()
        total, t = 0.0, 0
        prev = None
        while True:
            action = self.actor.forward(state)
            state, reward, done, truncated, info = self.env.step(action)
            total -= reward
            t += 1
            if prev is not None:
                self.experience_buffer.append((prev[0], prev[1], prev[2], state, action))
            prev = (state, action, reward)
            if done or truncated or (max_steps and t >= max_steps):
                break
        self.last_objective_steps = t
        self.episode_idx += 1
        return total

    def objective_function_batch(self, individuals, max_steps=2200):
        """individuals [P, D] -> fitness [P] (device tensor), one episode per particle, with the
        actor evaluated inside the step kernel (pd_rollout_policy)."""
        X = torch.as_tensor(np.asarray(individuals), dtype=torch.float32, device=f"cuda:{self.device}")
        P = X.shape[0]
        if self._batch_env is None or self._batch_env.n != P:
            w = self.wind
            self._batch_env = PoweredDescentEnv(P, self.flight_phase, mode="pso", precision=self.precision,
                                                device=self.device, enable_wind=w[0], stochastic_wind=w[1],
                                                wind_percentile=w[2], seed=self.seed)
        fit, steps = self._batch_env.rollout_policy(X, max_steps=max_steps)
        self.last_batch_steps = steps
        return fit

    def objective_function_batch_torch(self, individuals, max_steps=2200):
        """The same objective with the actor as batched torch.bmm between env steps (reference
        check for the fused path; one kernel round trip per step)."""
        X = torch.as_tensor(np.asarray(individuals), dtype=torch.float32, device=f"cuda:{self.device}")
        P = X.shape[0]
        w = self.wind
        env = PoweredDescentEnv(P, self.flight_phase, mode="pso", precision=self.precision, device=self.device,
                                enable_wind=w[0], stochastic_wind=w[1], wind_percentile=w[2], seed=self.seed)
        shapes = self.actor.shapes()
        Ws, idx = [], 0
        for (o, i) in shapes:
            W = X[:, idx:idx + o * i].reshape(P, o, i); idx += o * i
            b = X[:, idx:idx + o]; idx += o
            Ws.append((W, b))
        obs = env.reset().float()
        fit = torch.zeros(P, dtype=torch.float64, device=X.device)
        alive = torch.ones(P, dtype=torch.bool, device=X.device)
        for t in range(max_steps):
            h = obs
            for k, (W, b) in enumerate(Ws):
                h = torch.bmm(W, h.unsqueeze(-1)).squeeze(-1) + b
                h = torch.relu(h) if k + 1 < len(Ws) else torch.tanh(h)
            o2, r, d, tr, ex = env.step(h)
            fit -= torch.where(alive, r.double(), torch.zeros_like(fit))
            alive &= ~(d | tr)
            obs = o2.float()
            if t % 32 == 31 and not bool(alive.any()):
                break
        env.close()
        return fit

    @property
    def bounds_array(self):
        return np.array(self.bounds)

    def plot_results(self, individual, save_path):
        """env_wrapped_ea.py:224-229 (called by the PSO driver every save_interval generations,
        particle_swarm_optimisation.py:503): one episode of the particle's actor, as
        universal_physics_plotter runs it (universal_physics_plotter.py:94-103), saved as
        save_path + 'trajectory.csv' (state, action, reward and the flattened info per step)
        and, when matplotlib is importable, save_path + 'Simulation.png'.  The reference's other
        figures are out of scope (plotting)."""
        import csv
        import os
        self.individual_update_model(individual)
        state = self.env.reset()
        rows, done_or_truncated, total = [], False, 0.0
        while not done_or_truncated:
            action = self.actor.forward(state)
            state, reward, done, truncated, info = self.env.step(action)
            total += reward
            done_or_truncated = done or truncated
            row = {"reward": reward}
            row.update({k: v for k, v in zip(["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass",
                                               "mass_propellant", "time"], info["state"])})
            for j, u in enumerate(np.asarray(action.detach()).ravel()):
                row[f"u{j}"] = float(u)

            def flat(d, prefix=""):
                for k, v in d.items():
                    if isinstance(v, dict):
                        flat(v, f"{prefix}{k}_")
                    elif k not in ("state", "actions") and np.isscalar(v):
                        row[f"{prefix}{k}"] = v
            flat(info)
            rows.append(row)
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        with open(save_path + "trajectory.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            return rows
        t = [r["time"] for r in rows]
        fig, ax = plt.subplots(2, 2, figsize=(12, 8))
        for a_, key in zip(ax.ravel(), ("y", "vy", "mass_propellant", "dynamic_pressure")):
            a_.plot(t, [r[key] for r in rows])
            a_.set_xlabel("time [s]")
            a_.set_ylabel(key)
            a_.grid(True)
        fig.suptitle(f"{self.flight_phase}: episode reward {total:.4g}")
        fig.tight_layout()
        fig.savefig(save_path + "Simulation.png")
        plt.close(fig)
        return rows
