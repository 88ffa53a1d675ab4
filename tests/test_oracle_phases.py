"""CPU oracle vs the reference for the flight phases besides the two landing burns (SURVEY 8f
rank 4): landing_burn_pure_throttle_Pcontrol, ballistic_arc_descent, flip_over_boostbackburn,
subsonic and supersonic ascent, plus the RL reward of landing_burn.

Pinned by (tests/golden/make_golden.py):
  * recorded_phases.npz -- the reference's own recorded classical-controller runs of the
    flip-over and both ascent phases (data/reference_trajectory/*), replayed open loop;
  * ref_phases.npz -- compile_physics steps and rl_wrapped_env_pytorch episodes produced by
    importing the reference.
"""
import math
import os

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
Z = np.load(os.path.join(HERE, "golden", "ref_phases.npz"))
REC = np.load(os.path.join(HERE, "golden", "recorded_phases.npz"))
INFO = ["air_density", "mach_number", "CL", "CD", "mass_flow", "dynamic_pressure", "x_cog", "inertia",
        "gimbal_angle_deg"]
TAGS = {"pc": O.PCONTROL, "ba": O.BALLISTIC, "fl": O.FLIP, "sub": O.SUBSONIC, "sup": O.SUPERSONIC}
EP_TAGS = {"lb": O.LANDING_BURN, "pc": O.PCONTROL, "ba": O.BALLISTIC, "sub": O.SUBSONIC, "sup": O.SUPERSONIC}


def rel(a, b):
    e = np.abs(np.asarray(a) - np.asarray(b)) / (np.abs(np.asarray(b)) + 1e-300)
    e[np.asarray(a) == np.asarray(b)] = 0
    return e


def augment(tag, a, speed0):
    """rl_wrapped_env_pytorch.augment_action (env_wrapped_rl_pytorch.py:120-165) on a float32
    policy action -> (env action, float32?)."""
    a = np.asarray(a, np.float32)
    if tag == "lb":   # log compression; 10*|u| and 1+. stay float32 (NEP 50), math.log in binary64
        f = lambda u, c: math.copysign(math.log(1 + c * abs(u)) / math.log(1 + c), u)
        return np.array([f(a[0], 10), a[1], f(a[2], 5), f(a[3], 5)]), False
    if tag == "pc":   # v_ref = (u + 1)/2 * speed0 in float32
        return ((a + np.float32(1)) / np.float32(2) * np.float32(speed0)).astype(np.float64), True
    return a.astype(np.float64), True


@pytest.mark.parametrize("tag", list(TAGS))
def test_teacher_forced_physics(tag):
    """compile_physics(0.1, phase) from recorded states, float32 and float64 actions."""
    o = O.Oracle(phase=TAGS[tag], rtd=O.RTD_NONE)
    S, A, F, PV, SO, INF = (Z[f"{tag}_{k}"] for k in ("state_in", "action", "f32", "prev", "state_out", "info"))
    for i in range(len(S)):
        f32 = bool(F[i])
        prev = float(np.float32(PV[i])) if f32 else float(PV[i])
        s, info = o.physics(S[i], A[i], f32=f32, prevs=(prev, 0.0, 0.0))
        e = rel(s, SO[i])
        assert e[5] < 1e-9 and np.delete(e, 5).max() < 1e-10, (tag, i, e)
        iv = np.array([info[k] for k in INFO])
        ei = rel(iv, INF[i])
        assert ei[[2, 3]].max() < 1e-9, (tag, i, "CL/CD", ei)          # RBF solve order
        assert np.delete(ei, [2, 3]).max() < 1e-14, (tag, i, ei)        # mass flow bit-level incl. f32 islands


@pytest.mark.parametrize("tag", list(EP_TAGS))
@pytest.mark.parametrize("k", [0, 1])
def test_teacher_forced_rl_episodes(tag, k):
    """rl_wrapped_env_pytorch episodes, each step started from the reference's previous state and
    g-load window: next state, reward, done/truncated/id and observation."""
    p = f"ep_{tag}{k}_"
    S, R, Dn, T, TI, OB, A = (Z[p + n] for n in ("state", "reward", "done", "trunc", "trunc_id", "obs", "actions"))
    o = O.Oracle(phase=EP_TAGS[tag], rtd=O.RTD_RL, discount_factor=0.99, trajectory_length=100)
    allS = np.vstack([np.array(o.P.state0_ph[EP_TAGS[tag]][:])[None], S])
    v = np.hypot(allS[:, 2], allS[:, 3])
    g = np.abs(np.diff(v)) / 0.1 / 9.81
    prevs = (0.0, 0.0, 0.0)
    for t in range(len(R)):
        o.reset(allS[t])
        o.E.gimbal_prev, o.E.dl_prev, o.E.dr_prev = prevs
        win = g[max(0, t - 9):t]
        for i, gv in enumerate(win):
            o.E.gwin[i] = gv
        o.E.gwin_len = len(win)
        u, f32 = augment(tag, A[t], o.P.speed0_pc)
        s, r, d, tr, tid, ob, info = o.step(u, f32=f32)
        prevs = (info["gimbal_angle_deg"], info["delta_command_left_rad"], info["delta_command_right_rad"])
        assert rel(s, S[t]).max() < 1e-9, (tag, t, rel(s, S[t]))
        assert abs(r - R[t]) <= 1e-10 * max(1.0, abs(R[t])), (tag, t, r, R[t])
        assert (d, tr, tid) == (bool(Dn[t]), bool(T[t]), int(TI[t])), (tag, t)
        assert np.abs(ob - OB[t]).max() < 1e-12, (tag, t, ob, OB[t])


@pytest.mark.parametrize("tag,phase,skip", [("fl", O.FLIP, []), ("sub", O.SUBSONIC, [6]), ("sup", O.SUPERSONIC, [])])
def test_recorded_runs_open_loop(tag, phase, skip):
    """The reference's recorded runs of the phase, replayed open loop from the phase's initial
    state with the recorded float64 controls.  (The subsonic CSV's gamma column holds degrees.)"""
    S, U = REC[f"{tag}_state"], REC[f"{tag}_u"]
    o = O.Oracle(phase=phase, rtd=O.RTD_NONE)
    st = np.array(o.P.state0_ph[phase][:])
    prevs = (0.0, 0.0, 0.0)
    span = S.max(0) - S.min(0) + 1e-300
    worst = np.zeros(11)
    for t in range(len(S)):
        st, info = o.physics(st, U[t], f32=False, prevs=prevs)
        prevs = (info["gimbal_angle_deg"], 0.0, 0.0)
        worst = np.maximum(worst, np.abs(st - S[t]) / span)
    worst[skip] = 0
    assert worst.max() < 1e-10, worst


def test_unsteppable_pairs_recorded():
    """landing_burn_ACS and the flip-over RL env raise TypeError at their first step in the
    reference (arity mismatches, rockets_physics.py:867-891 / rtd_rl.py:134 vs
    base_environment.py:150); the facade reproduces that (tests/test_gpu_parity.py)."""
    assert list(Z["raises"]) == ["landing_burn_ACS/rl: TypeError", "flip_over_boostbackburn/rl: TypeError"]
