"""The non-parity RK4 mode on the device (PD_INTEG_RK4, BASELINE config c2's "RK4 dt=0.01 s",
k_step<..., RK4>).  NOT the reference's integrator: it is checked against the oracle's
restatement of the same scheme (ORC_INTEG_RK4, pinned by tests/test_oracle_rk4.py), with the
tolerances of the reference-integrator batch test (test_gpu_parity.test_batched_random_vs_oracle):
the transcendentals differ in the last ulp (device atan2/exp vs libm), everything else is the same
operations in the same order."""
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


@pytest.mark.parametrize("lpe", [2, 16])
def test_rk4_batch_vs_oracle(pd, oracle_mod, lpe):
    """c2 shape (4096 envs, no wind, no tilt), random float32 actions, 40 steps: 16 sampled envs
    free-running against the oracle's RK4 (state <= 1e-8 rel, attitude 1e-7/1e-6, reward 1e-9)."""
    import torch
    rng = np.random.default_rng(7)
    N, T = 4096, 40
    A = rng.uniform(-1, 1, (T, N, 1)).astype(np.float32)
    env = pd.PoweredDescentEnv(N, mode="rl", lanes_per_env=lpe, integrator="rk4")
    at = torch.tensor(A).cuda()
    rews = []
    for t in range(T):
        obs, r, dn, tr, ex = env.step(at[t])
        rews.append(r.cpu().numpy())
    S = env.state.cpu().numpy()
    rews = np.array(rews)
    s0 = np.array(oracle_mod.Oracle(phase=0, rtd=0).state)
    assert abs(S[0, 10] - (s0[10] + 4.0)) < 1e-9   # 40 x 10 x 0.01 s
    for i in rng.choice(N, 16, replace=False):
        o = oracle_mod.Oracle(phase=0, rtd=0, integrator=oracle_mod.INTEG_RK4)
        rr = []
        for t in range(T):
            s, r, dn_, tr_, tid, ob, info = o.step(A[t, i], f32=True)
            rr.append(r)
        err = np.abs(o.state - S[i]) / (np.abs(o.state) + 1e-3)
        tol = np.full(11, 1e-8); tol[[4, 6, 7]] = 1e-7; tol[5] = 1e-6   # attitude: chaotic
        assert (err < tol).all(), (i, dict(zip(ST, err)))
        assert np.abs(np.array(rr) - rews[:, i]).max() < 1e-9


def test_rk4_differs_from_reference_integrator(pd):
    """The mode is really selected: after one step the RK4 and reference handles differ (by the
    integrators' error, far above rounding) while sharing the initial state."""
    import torch
    A = torch.full((64, 1), 0.3, device="cuda")
    a = pd.PoweredDescentEnv(64, mode="rl")
    b = pd.PoweredDescentEnv(64, mode="rl", integrator="rk4")
    a.step(A); b.step(A)
    d = (a.state - b.state).abs()[:, 3]
    assert float(d.min()) > 1e-7 and float(d.max()) < 1e-2


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_rk4_fused_equals_step_loop(pd, precision):
    """pd_step_n (16 env-steps per launch) with RK4 and auto-reset equals the per-step loop bit for bit."""
    import torch
    N, T = 1000, 37
    g = torch.Generator(device="cuda").manual_seed(3)
    A = (torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1).contiguous()
    kw = dict(mode="rl", precision=precision, integrator="rk4", auto_reset=True)
    loop = pd.PoweredDescentEnv(N, **kw)
    fused = pd.PoweredDescentEnv(N, **kw)
    rows = [loop.step(A[t]) for t in range(T)]
    obs, rew, dn, tr, tid = fused.step_n(A)
    for t, (o, r, d, tt, ex) in enumerate(rows):
        assert torch.equal(o, obs[t]) and torch.equal(r, rew[t]) and torch.equal(d, dn[t]), t
    assert torch.equal(loop.state, fused.state)
    assert bool(torch.isfinite(fused.state).all())


def test_rk4_refused_outside_c2(pd):
    """RK4 exists for landing_burn_pure_throttle without wind only; policy rollouts refuse it."""
    import torch
    with pytest.raises(pd.PdError):
        pd.PoweredDescentEnv(8, flight_phase="landing_burn", mode="pso", integrator="rk4")
    with pytest.raises(pd.PdError):
        pd.PoweredDescentEnv(8, mode="rl", integrator="rk4", enable_wind=True)
    with pytest.raises(ValueError):
        pd.PoweredDescentEnv(8, mode="rl", integrator="rk2")
    env = pd.PoweredDescentEnv(8, mode="pso", integrator="rk4")
    w = torch.zeros(8, 249, device="cuda")
    with pytest.raises(pd.PdError):
        env.rollout_policy(w, max_steps=10)
