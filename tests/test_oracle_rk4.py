"""The non-parity RK4 mode of the oracle (ORC_INTEG_RK4, BASELINE config c2's "RK4 dt=0.01 s").
It is not the reference's integrator (semi-implicit Euler, rockets_physics.py:909-957), so it has
no reference fixture: these tests pin the restatement itself -- fourth-order convergence on a
smooth stretch, agreement with the reference integrator to the integrators' own error, and the
mode's restriction to pure throttle without wind."""
import numpy as np

ST = ["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass", "mass_propellant", "time"]


def _run(O, acts, h, f32=False, integrator=1):
    o = O.Oracle(phase=O.PURE_THROTTLE, rtd=O.RTD_RL, integrator=integrator, dt=h)
    out = []
    for a in acts:
        s, r, d, tr, tid, ob, info = o.step(a, f32=f32)
        out.append(s)
        if d or tr:
            break
    return np.array(out)


def test_rk4_fourth_order_one_step(oracle_mod):
    """One 0.1 s env step from the reference initial state with binary64 actions (float32 actions
    quantise the thrust at 1e-7 relative, which caps any integrator's observable order): halving
    h cuts the error against h = 0.1/80 by ~16 on vx, vy, theta, theta_dot."""
    O = oracle_mod
    for u in (-0.7, 0.1, 0.9):
        acts = np.array([[u]])
        ref = _run(O, acts, 0.1 / 80)[-1]
        e1 = np.abs(_run(O, acts, 0.01)[-1] - ref)
        e2 = np.abs(_run(O, acts, 0.005)[-1] - ref)
        for k in (2, 3, 4, 5):
            assert e1[k] / max(e2[k], 1e-300) > 10.0, (u, ST[k], e1[k], e2[k])
        assert e1[[2, 3]].max() < 1e-8


def test_rk4_tracks_reference_integrator(oracle_mod):
    """A random-action episode under RK4 dt 0.01 and under the reference's Euler 4 x 0.025 s: the
    two approximate the same ODE, so the translational channels agree to the Euler error
    (O(dt), metres over a ~13 s episode), masses and time exactly (constant mass flow within a step)."""
    O = oracle_mod
    acts = np.random.default_rng(1).uniform(-1, 1, (300, 1)).astype(np.float32)
    a = _run(O, acts, 0.0, f32=True, integrator=0)
    b = _run(O, acts, 0.0, f32=True, integrator=1)
    n = min(len(a), len(b))
    assert n > 100
    assert np.abs(a[:n, 1] - b[:n, 1]).max() < 5.0          # y (m), ~17 km altitude
    assert np.abs(a[:n, 3] - b[:n, 3]).max() < 0.5          # vy (m/s), ~950 m/s
    assert np.abs(a[:n, 8] - b[:n, 8]).max() / a[0, 8] < 1e-8
    assert np.abs(a[:n, 10] - b[:n, 10]).max() < 1e-9


def test_rk4_only_pure_throttle_without_wind(oracle_mod):
    """orc_physics refuses the mode (returns -1, state untouched) outside pure throttle / no wind."""
    import ctypes as C
    O = oracle_mod
    o = O.Oracle(phase=O.LANDING_BURN, rtd=O.RTD_PSO, integrator=1)
    s0 = o.state.copy()
    u = (C.c_double * 4)(0.1, 0.2, 0.0, 0.0)
    rc = o.L.orc_physics(C.byref(o.P), C.byref(o.E), O.LANDING_BURN, u, 1, None, None)
    assert rc == -1 and np.array_equal(o.state, s0)
    w = O.Oracle(phase=O.PURE_THROTTLE, rtd=O.RTD_RL, wind=True, integrator=1)
    rc = w.L.orc_physics(C.byref(w.P), C.byref(w.E), O.PURE_THROTTLE, u, 1, None, None)
    assert rc == -1
