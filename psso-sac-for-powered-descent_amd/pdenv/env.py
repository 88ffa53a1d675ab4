"""Batched powered-descent environment over HBM-resident torch tensors.

`PoweredDescentEnv(n_envs, ...)` is the vectorised counterpart of the reference's
`rocket_environment_pre_wrap` (src/envs/base_environment.py:12-154) for every flight phase of
compile_physics: the two the north-star drivers use, 'landing_burn_pure_throttle' (SAC driver)
and 'landing_burn' (PSO driver), and 'landing_burn_pure_throttle_Pcontrol',
'ballistic_arc_descent', 'flip_over_boostbackburn', 'subsonic', 'supersonic'.
'landing_burn_ACS' is accepted by the constructor (as the reference's is) and raises TypeError
at the first step, as the reference does.  All compute runs in libpdenv.so (HIP kernels); torch
only provides device memory and the current stream.
"""
import ctypes as C

import torch

from . import _lib as L
from .params import Params

PHASES = {"landing_burn_pure_throttle": L.PURE_THROTTLE, "landing_burn": L.LANDING_BURN,
          "landing_burn_pure_throttle_Pcontrol": L.PCONTROL, "ballistic_arc_descent": L.BALLISTIC_ARC,
          "flip_over_boostbackburn": L.FLIP_OVER, "subsonic": L.SUBSONIC, "supersonic": L.SUPERSONIC,
          "landing_burn_ACS": L.LANDING_BURN_ACS}
# 'physics': compile_physics stepping only (reward 0, never done/truncated)
MODES = {"rl": L.RTD_RL, "pso": L.RTD_PSO, "physics": L.RTD_NONE}
INTEGRATORS = {"reference": 0, "rk4": 1}   # pd_integrator (PD_INTEG_REFERENCE, PD_INTEG_RK4)
# (phase, mode) pairs whose reference env raises TypeError at the first step (include/pdenv.h)
UNSTEPPABLE = {("landing_burn_ACS", m) for m in MODES} | {("flip_over_boostbackburn", "rl")} | \
    {(p, "pso") for p in PHASES if p not in ("landing_burn_pure_throttle", "landing_burn")}


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class PoweredDescentEnv:
    def __init__(self, n_envs, flight_phase="landing_burn_pure_throttle", mode="rl", precision="f64",
                 device=0, enable_wind=False, stochastic_wind=False, wind_percentile=50,
                 auto_reset=False, tilt_sigma_rad=0.0, seed=0, env_offset=0, action_f64=False,
                 params=None, lanes_per_env=0, dt=0.0, discount_factor=0.99, trajectory_length=100,
                 integrator="reference", table_flags=0):
        # integrator "rk4": NOT the reference's (semi-implicit Euler) -- BASELINE config c2's
        # "RK4 dt=0.01 s", pure throttle without wind only; see include/pdenv.h pd_integrator
        if flight_phase not in PHASES:
            raise ValueError(f"flight_phase must be one of {list(PHASES)} (got {flight_phase!r})")
        if mode not in MODES:
            raise ValueError(f"mode must be one of {list(MODES)} (got {mode!r})")
        if mode == "pso" and flight_phase in ("landing_burn_ACS", "landing_burn_pure_throttle_Pcontrol"):
            # compile_rtd_pso asserts its phase list (rtd_pso.py:321) at construction
            raise AssertionError(f"compile_rtd_pso has no {flight_phase!r}")
        self.flight_phase, self.mode = flight_phase, mode
        self.n = int(n_envs)
        self.unsteppable = (flight_phase, mode) in UNSTEPPABLE
        if self.unsteppable:
            # the reference constructs these envs and raises TypeError at their first step
            self.h = None
            self.obs_dim, self.action_dim = 0, 0
            return
        self.lib = L.load()
        if self.lib.pd_device_count() <= 0 or not torch.cuda.is_available():
            raise L.PdError("no HIP device visible: the powered-descent env runs on MI355X only")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.dtype = torch.float64 if precision == "f64" else torch.float32
        self.params = params or Params()
        cfg = L.PdConfig()
        cfg.n_envs = self.n
        cfg.device = self.device.index or 0
        cfg.phase = PHASES[flight_phase]
        cfg.rtd = MODES[mode]
        cfg.precision = L.F64 if precision == "f64" else L.F32
        cfg.seed = int(seed)
        cfg.env_offset = int(env_offset)
        cfg.enable_wind = int(bool(enable_wind))
        cfg.stochastic_wind = int(bool(stochastic_wind))
        cfg.wind_percentile = -1 if wind_percentile is None else int(wind_percentile)
        cfg.auto_reset = int(bool(auto_reset))
        cfg.tilt_sigma_rad = float(tilt_sigma_rad)
        cfg.action_f64 = int(bool(action_f64))
        cfg.lanes_per_env = int(lanes_per_env)
        cfg.dt = float(dt)
        cfg.discount_factor = float(discount_factor) if discount_factor is not None else 0.0
        cfg.trajectory_length = int(trajectory_length) if trajectory_length is not None else 0
        if integrator not in INTEGRATORS:
            raise ValueError(f"integrator must be one of {list(INTEGRATORS)} (got {integrator!r})")
        cfg.integrator = INTEGRATORS[integrator]
        cfg.table_flags = int(table_flags)   # pd_table_flags (L.TABLES_*): 0 = the defaults
        self.integrator = integrator
        self.cfg = cfg
        handle = C.c_void_p()
        with torch.cuda.device(self.device):
            L.check(self.lib.pd_create(C.byref(self.params.struct), C.byref(cfg), C.byref(handle)))
        self.h = handle
        self.obs_dim = self.lib.pd_obs_dim(self.h)
        self.action_dim = self.lib.pd_action_dim(self.h)
        self.action_dtype = torch.float64 if action_f64 else torch.float32
        kw = dict(device=self.device)
        self._obs = torch.empty(self.n, self.obs_dim, dtype=self.dtype, **kw)
        self._rew = torch.empty(self.n, dtype=self.dtype, **kw)
        self._done = torch.empty(self.n, dtype=torch.uint8, **kw)
        self._trunc = torch.empty(self.n, dtype=torch.uint8, **kw)
        self._tid = torch.empty(self.n, dtype=torch.int8, **kw)
        self._steps = 0
        # pd_flush_misses every flush_every steps (0: never -- since ABI 10 every step launch inserts
        # the neighbourhoods it solved itself; the call is kept for ABI <= 9 habits)
        self.flush_every = 0

    # ------------------------------------------------------------------ reference surface
    def reset(self, mask=None):
        """base_environment.py:80-97 for all envs (or a bool/uint8 mask [N]); returns obs [N, O]."""
        if self.unsteppable:
            return None
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        L.check(self.lib.pd_reset(self.h, _ptr(m), _ptr(self._obs), _stream(self.device)))
        return self._obs.clone()

    def step(self, actions, noise=None, info=False):
        """base_environment.py:99-154 for every env.  actions: [N, A] float32 (float64 with
        action_f64).  Returns (obs, reward, done, truncated, extras) as device tensors; with
        auto_reset the obs is the post-step (terminal) observation."""
        self._check_steppable()
        a = actions.to(device=self.device, dtype=self.action_dtype).reshape(self.n, self.action_dim).contiguous()
        nz = None
        if noise is not None:
            nz = noise.to(device=self.device, dtype=torch.float64).reshape(self.n, 8).contiguous()
        inf = torch.empty(L.N_INFO, self.n, dtype=self.dtype, device=self.device) if info else None
        L.check(self.lib.pd_step(self.h, _ptr(a), _ptr(self._obs), _ptr(self._rew), _ptr(self._done),
                                 _ptr(self._trunc), _ptr(self._tid), _ptr(nz), _ptr(inf), _stream(self.device)))
        self._steps += 1
        if self.flush_every and self._steps % self.flush_every == 0:
            self.flush()
        extras = {"trunc_id": self._tid.clone()}
        if info:
            extras.update({k: inf[j] for j, k in enumerate(L.INFO_FIELDS)})
        return self._obs.clone(), self._rew.clone(), self._done.bool(), self._trunc.bool(), extras

    def _check_steppable(self):
        if self.unsteppable:
            raise TypeError(f"{self.flight_phase!r} with mode {self.mode!r} cannot be stepped: the reference "
                            "raises TypeError here (argument-count mismatch, see include/pdenv.h pd_phase/pd_rtd)")

    def step_raw(self, actions):
        """Hot-loop step: launches pd_step into the handle's preallocated output buffers
        (obs_buf, reward_buf, done_buf, trunc_buf, trunc_id_buf) without copies or syncs.
        actions must already be a contiguous [N, A] tensor of action_dtype on the device."""
        L.check(self.lib.pd_step(self.h, C.c_void_p(actions.data_ptr()), _ptr(self._obs), _ptr(self._rew),
                                 _ptr(self._done), _ptr(self._trunc), _ptr(self._tid), None, None,
                                 _stream(self.device)))
        self._steps += 1
        if self.flush_every and self._steps % self.flush_every == 0:
            self.flush()

    def step_raw_noflush(self, actions):
        """step_raw without any pd_flush_misses call (graph capture)."""
        L.check(self.lib.pd_step(self.h, C.c_void_p(actions.data_ptr()), _ptr(self._obs), _ptr(self._rew),
                                 _ptr(self._done), _ptr(self._trunc), _ptr(self._tid), None, None,
                                 _stream(self.device)))

    def step_sac(self, mean, log_std, eps, log_std_min=-20.0, log_std_max=2.0, max_action=1.0, action=None,
                 slab=None, obs32=None, heads=None):
        """One SAC collection step in one launch (pd_step_sac): the action sampled in the kernel
        from the actor's heads (mean, log_std, eps: contiguous float32 [N, A] device tensors; or
        heads [N, 2A] = mean | log_std of one GEMM, with mean = log_std = None; eps None =
        deterministic), the env step, and float32 outputs written by the kernel epilogue into the
        given tensors: action [N, A], slab [N, 2S + A + 2] (state | action | reward | next_state |
        done) and obs32 [N, S] (the next observation, after any auto-reset).
        No copies, allocations or syncs."""
        hs = 0
        if heads is not None:
            A = self.action_dim
            mean = C.c_void_p(heads.data_ptr())
            log_std = C.c_void_p(heads.data_ptr() + 4 * A)
            hs = 2 * A
        else:
            mean, log_std = _ptr(mean), _ptr(log_std)
        L.check(self.lib.pd_step_sac(self.h, mean, log_std, hs, _ptr(eps), float(log_std_min),
                                     float(log_std_max), float(max_action), _ptr(action), _ptr(slab), _ptr(obs32),
                                     _stream(self.device)))
        self._steps += 1

    def step_sac_ring(self, heads, log_std_min=-20.0, log_std_max=2.0, max_action=1.0, deterministic=False,
                      ring=None, capacity=0, ring_state=None, priorities=None, max_priority=None, action=None,
                      obs32=None, eps_out=None):
        """One SAC collection step in one launch (pd_step_sac_ring): the action sampled in the
        kernel from heads [N, 2A] (mean | log_std, unclamped; eps drawn in the kernel unless
        deterministic), the env step, and the transition rows written into `ring` -- the replay
        buffer's [capacity, 2S + A + 2] rows at its device-held position ring_state (int64 [3]:
        position, size, 0), with priorities[row] = max_priority[0] -- or, ring_state None, into
        ring as a [N, 2S + A + 2] slab.  action [N, A], obs32 [N, S] (next observation) and
        eps_out [N, A] as given.  No copies, allocations or syncs."""
        L.check(self.lib.pd_step_sac_ring(self.h, _ptr(heads), int(bool(deterministic)), float(log_std_min),
                                          float(log_std_max), float(max_action), _ptr(eps_out), _ptr(action),
                                          _ptr(ring), int(capacity), _ptr(ring_state), _ptr(priorities),
                                          _ptr(max_priority), _ptr(obs32), _stream(self.device)))
        self._steps += 1

    def step_sac_fused(self, state_dim, action_dim, hidden, n_hidden_layers, params, log_std_min=-20.0, log_std_max=2.0, max_action=1.0,
                       deterministic=False, ring=None, capacity=0, ring_state=None, priorities=None,
                       max_priority=None, action=None, obs32=None, eps_out=None, heads=None):
        """The whole SAC collection step in one launch (pd_step_sac_fused): the actor's forward pass
        in the step kernel's prologue on obs32 [N, S] (the observation the previous step left
        there), then step_sac_ring's sampling, env step and transition rows, and the next
        observation back into obs32.  params: a ctypes array of the actor's 2 (n_hidden_layers +
        2) parameter pointers (pd_sac_actor's order) of an actor with state_dim inputs and action_dim
        outputs (the library refuses widths other than the handle's); heads [N, 2A] receives the
        heads if given.
        Handles that do not step 16 lanes per env run the actor as its own launch (same bits).
        No copies, allocations or syncs."""
        L.check(self.lib.pd_step_sac_fused(self.h, int(state_dim), int(action_dim), int(hidden), int(n_hidden_layers),
                                           params, _ptr(heads),
                                           int(bool(deterministic)), float(log_std_min), float(log_std_max),
                                           float(max_action), _ptr(eps_out), _ptr(action), _ptr(ring), int(capacity),
                                           _ptr(ring_state), _ptr(priorities), _ptr(max_priority), _ptr(obs32),
                                           _stream(self.device)))
        self._steps += 1

    def tuning(self):
        """The handle's launch tuning (pd_get_tuning) as a dict."""
        t = L.PdTuning()
        L.check(self.lib.pd_get_tuning(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in L.PdTuning._fields_}

    def set_tuning(self, **kw):
        """Change launch tuning fields (pd_set_tuning: step_fuse, policy_fuse, policy_lanes,
        policy_list, policy_list_at, policy_refill, policy_slots, policy_refill_own); results never
        depend on them."""
        cur = self.tuning()
        bad = set(kw) - set(cur)
        if bad:
            raise ValueError(f"unknown tuning fields {sorted(bad)}")
        cur.update(kw)
        t = L.PdTuning(**cur)
        L.check(self.lib.pd_set_tuning(self.h, C.byref(t)))

    def observe_raw(self):
        """pd_observe into the preallocated obs buffer (no copy); returns that buffer."""
        L.check(self.lib.pd_observe(self.h, _ptr(self._obs), _stream(self.device)))
        return self._obs

    @property
    def obs_buf(self):
        return self._obs

    @property
    def reward_buf(self):
        return self._rew

    @property
    def done_buf(self):
        return self._done

    @property
    def trunc_buf(self):
        return self._trunc

    @property
    def trunc_id_buf(self):
        return self._tid

    def _check_actions(self, a):
        """[T, N, A] with A the handle's action width: the kernel reads row t of env i at
        (t N + i) A + k, so anything narrower would be read past its end."""
        if a.dim() != 3 or a.shape[1] != self.n or a.shape[2] != self.action_dim:
            raise ValueError(f"actions must be [T, {self.n}, {self.action_dim}] (got {list(a.shape)})")

    def rollout(self, actions, reward_sum=None):
        """T step launches over device-resident actions [T, N, A]; returns summed rewards [N]."""
        self._check_steppable()
        a = actions.to(device=self.device, dtype=self.action_dtype).contiguous()
        self._check_actions(a)
        T = a.shape[0]
        rs = reward_sum if reward_sum is not None else torch.zeros(self.n, dtype=self.dtype, device=self.device)
        L.check(self.lib.pd_rollout(self.h, _ptr(a), int(T), _ptr(rs), _stream(self.device)))
        return rs

    def step_n(self, actions, outputs=True, info_keys=None):
        """T consecutive env-steps over device-resident actions [T, N, A] (pd_step_n: fused
        launches of up to 128 steps each, each inserting its solved misses), the same results as T step()
        calls.  Landing-burn phases only.  outputs=True returns per-step
        (obs [T, N, O], reward [T, N], done [T, N], truncated [T, N], trunc_id [T, N]);
        outputs=False writes nothing per step and returns None.  info_keys: names of
        L.INFO_FIELDS to tap in the fused launches (pd_step_n_info); the result then ends with a
        dict of [T, N] tensors, one per key."""
        self._check_steppable()
        a = actions.to(device=self.device, dtype=self.action_dtype).contiguous()
        self._check_actions(a)
        T = int(a.shape[0])
        if outputs:
            kw = dict(device=self.device)
            obs = torch.empty(T, self.n, self._obs.shape[-1], dtype=self.dtype, **kw)
            rew = torch.empty(T, self.n, dtype=self.dtype, **kw)
            dn = torch.empty(T, self.n, dtype=torch.uint8, **kw)
            tr = torch.empty(T, self.n, dtype=torch.uint8, **kw)
            tid = torch.empty(T, self.n, dtype=torch.int8, **kw)
            ptrs = [_ptr(x) for x in (obs, rew, dn, tr, tid)]
        else:
            ptrs = [None] * 5
        if info_keys:
            keys = list(info_keys)
            bad = [k for k in keys if k not in L.INFO_FIELDS]
            if bad:
                raise ValueError(f"unknown info keys {bad} (pdenv._lib.INFO_FIELDS)")
            if len(set(keys)) != len(keys):
                raise ValueError(f"info_keys holds a key more than once: {keys}")
            idx = sorted(L.INFO_FIELDS.index(k) for k in keys)
            mask = 0
            for j in idx:
                mask |= 1 << j
            inf = torch.empty(T, len(idx), self.n, dtype=self.dtype, device=self.device)
            L.check(self.lib.pd_step_n_info(self.h, _ptr(a), T, *ptrs, _ptr(inf), mask, _stream(self.device)))
        else:
            L.check(self.lib.pd_step_n(self.h, _ptr(a), T, *ptrs, _stream(self.device)))
        self._steps += T
        tap = {L.INFO_FIELDS[j]: inf[:, r] for r, j in enumerate(idx)} if info_keys else None
        if outputs:
            if T > 0:   # the handle's step buffers (obs_buf, ...) hold the last step, as after step()
                for dst, src in zip((self._obs, self._rew, self._done, self._trunc, self._tid), (obs, rew, dn, tr, tid)):
                    dst.copy_(src[-1])
            res = (obs, rew, dn.bool(), tr.bool(), tid)
            return res + (tap,) if info_keys else res
        return tap

    def step_n_raw(self, actions, outputs=None):
        """Hot-loop pd_step_n: actions a contiguous [T, N, A] device tensor of action_dtype (the
        caller guarantees the shape: nothing is checked here); outputs None or preallocated
        (obs [T,N,O], reward [T,N], done, truncated uint8 [T,N], trunc_id int8 [T,N]).  No copies,
        allocations or syncs; the handle's obs_buf/... are not updated."""
        ptrs = [None] * 5 if outputs is None else [_ptr(x) for x in outputs]
        L.check(self.lib.pd_step_n(self.h, C.c_void_p(actions.data_ptr()), int(actions.shape[0]), *ptrs,
                                   _stream(self.device)))
        self._steps += int(actions.shape[0])

    def flush(self):
        """Insert queued device-solved aero neighbourhoods into the tables (pd_flush_misses; since
        ABI 10 the step launches insert their own, so the queue is normally empty)."""
        L.check(self.lib.pd_flush_misses(self.h, _stream(self.device)))

    def observe(self):
        L.check(self.lib.pd_observe(self.h, _ptr(self._obs), _stream(self.device)))
        return self._obs.clone()

    @property
    def state(self):
        """[N, 11] x y vx vy theta theta_dot gamma alpha mass mass_propellant time."""
        soa = torch.empty(11, self.n, dtype=self.dtype, device=self.device)
        L.check(self.lib.pd_get_state(self.h, _ptr(soa), _stream(self.device)))
        return soa.t().contiguous()

    def set_state(self, state):
        soa = state.to(device=self.device, dtype=self.dtype).reshape(self.n, 11).t().contiguous()
        L.check(self.lib.pd_set_state(self.h, _ptr(soa), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def actuators(self):
        soa = torch.empty(3, self.n, dtype=self.dtype, device=self.device)
        L.check(self.lib.pd_get_actuators(self.h, _ptr(soa), _stream(self.device)))
        return soa.t().contiguous()

    def set_actuators(self, act):
        soa = act.to(device=self.device, dtype=self.dtype).reshape(self.n, 3).t().contiguous()
        L.check(self.lib.pd_set_actuators(self.h, _ptr(soa), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def set_gload_window(self, vprev, window, length):
        """g-load history (base_environment.py:137-149): |v| of the previous state [N], the
        window [N, 10] oldest first, and its valid length [N] (0..10)."""
        vp = torch.as_tensor(vprev, dtype=self.dtype).to(self.device).reshape(self.n).contiguous()
        w = torch.as_tensor(window, dtype=self.dtype).to(self.device).reshape(self.n, 10).t().contiguous()
        ln = torch.as_tensor(length, dtype=torch.uint8).to(self.device).reshape(self.n).contiguous()
        L.check(self.lib.pd_set_gload_window(self.h, _ptr(vp), _ptr(w), _ptr(ln), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def set_wind_sigmas(self, sigma_u, sigma_v):
        sig = torch.stack([torch.as_tensor(sigma_u, dtype=torch.float64).expand(self.n),
                           torch.as_tensor(sigma_v, dtype=torch.float64).expand(self.n)]).to(self.device).contiguous()
        L.check(self.lib.pd_set_wind_sigmas(self.h, _ptr(sig), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def rollout_policy(self, weights, max_steps=2200, check_every=8):
        """PSO objective of N particles on the device (pd_rollout_policy): every env is reset and
        driven by its own simple_actor until done/truncated or max_steps.
        weights: [N, P] per-particle parameter vectors (named_parameters() order).
        Returns (fitness [N] = -sum(reward), steps [N] int32) device tensors."""
        w = torch.as_tensor(weights, dtype=torch.float32, device=self.device)
        if w.dim() != 2 or w.shape[0] != self.n:
            raise ValueError(f"weights must be [{self.n}, P]")
        wt = w.t().contiguous()                       # parameter-major [P][N]: coalesced loads
        fit = torch.empty(self.n, dtype=self.dtype, device=self.device)
        steps = torch.empty(self.n, dtype=torch.int32, device=self.device)
        L.check(self.lib.pd_rollout_policy(self.h, _ptr(wt), int(w.shape[1]), int(max_steps), _ptr(fit),
                                           _ptr(steps), int(check_every), _stream(self.device)))
        self._keep = wt                               # alive until the stream has consumed it
        return fit, steps

    # ------------------------------------------------------------------ checkpoint / restore
    def checkpoint(self):
        """Every per-env buffer (state, g-load window, actuators, wind, counters, aero caches)
        as one device uint8 tensor (pd_checkpoint_save)."""
        blob = torch.empty(int(self.lib.pd_checkpoint_size(self.h)), dtype=torch.uint8, device=self.device)
        L.check(self.lib.pd_checkpoint_save(self.h, _ptr(blob), _stream(self.device)))
        return blob

    def restore(self, blob):
        """Load a checkpoint() of a handle with the same configuration; stepping then continues
        bit-identically to the saved handle."""
        b = blob.to(device=self.device, dtype=torch.uint8).contiguous()
        if b.numel() != int(self.lib.pd_checkpoint_size(self.h)):
            raise ValueError("checkpoint size does not match this handle's configuration")
        L.check(self.lib.pd_checkpoint_load(self.h, _ptr(b), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def gload_window(self):
        """(vprev [N], ring [N, 10], len [N], head [N]) of the g-load window (base_environment.py:136-149)."""
        kw = dict(device=self.device)
        vp = torch.empty(self.n, dtype=self.dtype, **kw)
        w = torch.empty(10, self.n, dtype=self.dtype, **kw)
        ln = torch.empty(self.n, dtype=torch.uint8, **kw)
        hd = torch.empty(self.n, dtype=torch.uint8, **kw)
        L.check(self.lib.pd_get_gload_window(self.h, _ptr(vp), _ptr(w), _ptr(ln), _ptr(hd), _stream(self.device)))
        return vp, w.t().contiguous(), ln, hd

    def wind_state(self):
        """(filters [N, 4] = u0 u1 v0 v1, sigmas [N, 2], percentile [N] int) of the wind model."""
        kw = dict(device=self.device)
        f = torch.empty(4, self.n, dtype=self.dtype, **kw)
        s = torch.empty(2, self.n, dtype=self.dtype, **kw)
        pr = torch.empty(self.n, dtype=torch.uint8, **kw)
        L.check(self.lib.pd_get_wind_state(self.h, _ptr(f), _ptr(s), _ptr(pr), _stream(self.device)))
        return f.t().contiguous(), s.t().contiguous(), pr.to(torch.int32) + 50

    def set_wind_state(self, filters=None, sigmas=None, percentile=None):
        kw = dict(device=self.device)
        f = None if filters is None else torch.as_tensor(filters, dtype=self.dtype).to(**kw).reshape(self.n, 4).t().contiguous()
        s = None if sigmas is None else torch.as_tensor(sigmas, dtype=self.dtype).to(**kw).reshape(self.n, 2).t().contiguous()
        pr = None
        if percentile is not None:
            p = torch.as_tensor(percentile).to(**kw).reshape(self.n)
            if bool(((p < 50) | (p > 99)).any()):
                raise ValueError("percentile must be in 50..99 (full_wind_model.py:29 draws randint(50, 99))")
            pr = (p - 50).to(torch.uint8).contiguous()
        L.check(self.lib.pd_set_wind_state(self.h, _ptr(f), _ptr(s), _ptr(pr), _stream(self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def episode_counters(self):
        """(episode [N], step within episode [N], truncation id [N]) -- the Philox counter words."""
        kw = dict(device=self.device)
        ep = torch.empty(self.n, dtype=torch.int32, **kw)
        st = torch.empty(self.n, dtype=torch.int32, **kw)
        tid = torch.empty(self.n, dtype=torch.int8, **kw)
        L.check(self.lib.pd_get_counters(self.h, _ptr(ep), _ptr(st), _ptr(tid), _stream(self.device)))
        return ep, st, tid

    def atmosphere(self, altitude):
        """The handle's ISA (pd_atmosphere) at altitudes [n]: (density, pressure, speed_of_sound)."""
        alt = torch.as_tensor(altitude, dtype=self.dtype).to(self.device).reshape(-1).contiguous()
        out = torch.empty(3, alt.numel(), dtype=self.dtype, device=self.device)
        L.check(self.lib.pd_atmosphere(self.h, _ptr(alt), _ptr(out), int(alt.numel()), _stream(self.device)))
        return out[0], out[1], out[2]

    def count_work(self, enable=True):
        """Workload counting of the following step launches on/off (pd_count_work; a diagnostic
        that costs the launches a few per cent): stats() then reports what they did."""
        L.check(self.lib.pd_count_work(self.h, int(bool(enable))))

    WORK_COUNTERS = ("gust_substeps", "resets", "q_line", "q_verified", "q_taylor", "q_balanced", "q_miss",
                     "balanced_rounds", "q_refined", "q_bisect", "wave_substeps_refined", "wave_substeps_bisect",
                     "q_cell", "wave_substeps_mixed")

    def stats(self):
        """Device statistics words (pd_stats): misses, NaN events, table entries, dropped queue
        entries, and the step kernel's workload counters since create (include/pdenv.h pd_stats)."""
        v = (L.I64 * 48)()
        L.check(self.lib.pd_stats(self.h, v, 48))
        out = {"rbf_misses": v[0], "nan_events": v[1], "table_entries_cd": v[2], "table_entries_cl": v[3],
               "miss_queue_dropped": v[16]}
        out.update({k: v[32 + j] for j, k in enumerate(self.WORK_COUNTERS)})
        return out

    def counters(self):
        v = [L.I64() for _ in range(4)]
        L.check(self.lib.pd_counters(self.h, *[C.byref(x) for x in v]))
        return {"rbf_misses": v[0].value, "table_entries_cd": v[1].value, "table_entries_cl": v[2].value,
                "nan_events": v[3].value}

    def close(self):
        if getattr(self, "h", None):
            self.lib.pd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
