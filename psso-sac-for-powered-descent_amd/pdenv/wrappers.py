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


def _info_dict(env, ex, state, action):
    """The info keys the drivers read (sac_pytorch_powered_descent.py:253-374), last sub-step."""
    info = {k: float(ex[k][0]) for k in L.INFO_FIELDS if k in ex}
    info["state"] = [float(v) for v in state]
    info["actions"] = action
    info["action_info"] = {"throttle": info.get("throttle", float("nan"))}
    if env.flight_phase == "landing_burn":
        info["action_info"]["gimbal_angle_deg"] = info.get("gimbal_angle_deg", float("nan"))
    return info


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
        info = _info_dict(self.env, {k: v.cpu() for k, v in ex.items() if k != "trunc_id"}, state, a.cpu().numpy())
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
        a = action.detach().reshape(1, -1).float()
        obs, r, d, tr, ex = self.env.step(a)
        self._tid = int(ex["trunc_id"][0])
        return obs[0].double().cpu().numpy(), float(r[0]), bool(d[0]), bool(tr[0]), {"state": self.env.state[0].tolist()}

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
        self.individual_update_model(individual)
        state = self.env.reset()
        total, t = 0.0, 0
        while True:
            action = self.actor.forward(state)
            state, reward, done, truncated, info = self.env.step(action)
            total -= reward
            t += 1
            if done or truncated or (max_steps and t >= max_steps):
                break
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
