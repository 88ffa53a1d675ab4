"""GPU parity: the HIP kernels (through the C ABI) against the reference's recorded runs,
the fixtures made by importing the reference, and the CPU oracle.

Tolerances (fp64 handle): teacher-forced single env-step <= 1e-10 relative per channel
(theta_dot: 1e-8 with a 1e-3 rad/s floor); full episodes: TOL_EPISODE (fraction of
per-channel range; the attitude channels are chaotic).  fp32 handle:
teacher-forced <= 1e-4 relative on non-attitude channels.
"""
import math
import os

import numpy as np
import pytest

from conftest import golden
from pdenv import _lib as L

pytestmark = pytest.mark.gpu

ST = ["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass", "mass_propellant", "time"]
TOL_EPISODE = np.array([1e-6, 1e-9, 1e-6, 1e-9, 1e-6, 1e-6, 1e-6, 1e-6, 1e-12, 1e-12, 1e-12])


@pytest.fixture(scope="module")
def pd():
    import torch
    import pdenv
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return pdenv


def make(pd, n, phase="landing_burn_pure_throttle", mode="rl", **kw):
    return pd.PoweredDescentEnv(n, flight_phase=phase, mode=mode, **kw)


@pytest.mark.parametrize("lpe", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("tag,phase", [("pt", "landing_burn_pure_throttle"), ("lb", "landing_burn")])
def test_teacher_forced_step_vs_reference(pd, tag, phase, lpe):
    import torch
    d = golden("ref_teacher_forced.npz")
    S0, A = d[f"{tag}_state_in"], d[f"{tag}_action"]
    env = make(pd, len(S0), phase, mode="pso", lanes_per_env=lpe)
    env.set_state(torch.tensor(S0))
    if phase == "landing_burn":
        env.set_actuators(torch.tensor(d[f"{tag}_prevs"]))
    obs, r, dn, tr, ex = env.step(torch.tensor(A), info=True)
    S = env.state.cpu().numpy()
    ref = d[f"{tag}_state_out"]
    err = np.abs(S - ref) / np.maximum(np.abs(ref), 1e-3)
    tol = np.full(11, 1e-10); tol[5] = 1e-8
    assert (err.max(0) < tol).all(), dict(zip(ST, err.max(0)))
    names = list(d["info_names"])
    md = ex["mass_flow"].cpu().numpy()
    assert np.array_equal(md, d[f"{tag}_info"][:, names.index("mass_flow")]), "float32 mass-flow island"
    cd = ex["CD"].cpu().numpy(); cl = ex["CL"].cpu().numpy()
    assert np.abs(cd - d[f"{tag}_info"][:, names.index("CD")]).max() < 1e-11
    assert np.abs(cl - d[f"{tag}_info"][:, names.index("CL")]).max() < 1e-9   # |CL| <= 2.2


def test_reference_trajectory_config1(pd):
    """Config c1: the classical controller's u0 as f64 [[u0]] from the nominal initial state."""
    import torch
    d = golden("recorded_reference_trajectory.npz")
    env = make(pd, 1, mode="pso", action_f64=True)
    got, last = [], None
    for u in d["u0"]:
        obs, r, dn, tr, ex = env.step(torch.tensor([[u]], dtype=torch.float64))
        got.append(env.state.cpu().numpy()[0])
        last = (float(r[0]), bool(dn[0]), bool(tr[0]))
    got = np.array(got)
    err = np.abs(got - d["state"]).max(0) / np.ptp(d["state"], 0)
    assert (err < TOL_EPISODE).all(), dict(zip(ST, err))
    assert last[1] and not last[2] and last[0] == pytest.approx(474318.950426, rel=1e-9)


EPISODES = [("rl_land", "landing_burn_pure_throttle", "rl"), ("rl_rand0", "landing_burn_pure_throttle", "rl"),
            ("rl_rand1", "landing_burn_pure_throttle", "rl"), ("rl_hi", "landing_burn_pure_throttle", "rl"),
            ("pso_pt_land", "landing_burn_pure_throttle", "pso"), ("pso_pt_rand", "landing_burn_pure_throttle", "pso"),
            ("pso_lb_rand0", "landing_burn", "pso"), ("pso_lb_rand1", "landing_burn", "pso")]


@pytest.mark.parametrize("name,phase,mode", EPISODES)
def test_episode_vs_reference(pd, name, phase, mode):
    """Whole episodes with float32 actions, as the SAC / PSO wrappers feed them."""
    import torch
    d = golden("ref_episodes.npz")
    acts = d[f"{name}_actions"]
    T = len(acts)
    env = make(pd, 1, phase, mode=mode)
    S, R, DN, TR, TID, OBS = [], [], [], [], [], []
    at = torch.tensor(acts, dtype=torch.float32).cuda()
    for t in range(T):
        obs, r, dn, tr, ex = env.step(at[t:t + 1])
        S.append(env.state); R.append(r); DN.append(dn); TR.append(tr); TID.append(ex["trunc_id"]); OBS.append(obs)
    S = torch.cat(S).cpu().numpy(); R = torch.cat(R).cpu().numpy()
    DN = torch.cat(DN).cpu().numpy(); TR = torch.cat(TR).cpu().numpy(); TID = torch.cat(TID).cpu().numpy()
    OBS = torch.cat(OBS).cpu().numpy()
    rs = d[f"{name}_state"]
    err = np.abs(S - rs).max(0) / (np.ptp(rs, 0) + 1e-12)
    tol = TOL_EPISODE if phase == "landing_burn_pure_throttle" else np.maximum(TOL_EPISODE, 1e-6 * (TOL_EPISODE > 1e-12))
    assert (err < tol).all(), dict(zip(ST, err))
    assert np.abs(R - d[f"{name}_reward"]).max() <= 1e-9 * max(1.0, np.abs(d[f"{name}_reward"]).max())
    assert list(DN.astype(bool)) == list(d[f"{name}_done"])
    assert list(TR.astype(bool)) == list(d[f"{name}_trunc"])
    assert TID[-1] == d[f"{name}_trunc_id"][-1]
    ref_obs = d[f"{name}_obs"]
    assert np.abs(OBS - ref_obs).max() < 1e-6   # bounded by the (chaotic) state drift


@pytest.mark.parametrize("lpe", [1, 4, 8, 16])
def test_batched_random_vs_oracle(pd, oracle_mod, lpe):
    """4096 envs (config c2 size), random float32 actions, 40 steps: every env against the
    scalar oracle on a sampled subset, and batch-invariance (env i does not depend on N)."""
    import torch
    rng = np.random.default_rng(5)
    N, T = 4096, 40
    A = rng.uniform(-1, 1, (T, N, 1)).astype(np.float32)
    env = make(pd, N, mode="rl", lanes_per_env=lpe)
    at = torch.tensor(A).cuda()
    rews = []
    for t in range(T):
        obs, r, dn, tr, ex = env.step(at[t])
        rews.append(r.cpu().numpy())
    S = env.state.cpu().numpy()
    rews = np.array(rews)
    for i in rng.choice(N, 16, replace=False):
        o = oracle_mod.Oracle(phase=0, rtd=0)
        rr = []
        for t in range(T):
            s, r, dn_, tr_, tid, ob, info = o.step(A[t, i], f32=True)
            rr.append(r)
        err = np.abs(o.state - S[i]) / (np.abs(o.state) + 1e-3)
        tol = np.full(11, 1e-8); tol[[4, 6, 7]] = 1e-7; tol[5] = 1e-6   # attitude: chaotic
        assert (err < tol).all(), (i, dict(zip(ST, err)))
        assert np.abs(np.array(rr) - rews[:, i]).max() < 1e-9


@pytest.mark.parametrize("precision,lpe", [("f64", 1), ("f64", 2), ("f32", 2)])
def test_device_solve_bit_identical(pd, precision, lpe):
    """Neighbourhoods missing from the pre-enumerated tables are solved on the device (wave-
    cooperative LU in LDS).  With the tables cut to 4 entries nearly every query goes through
    that path; the trajectories must equal the full-table run bit for bit, i.e. the device
    solve reproduces the host-built payloads exactly."""
    import torch
    N, T = 2048, 60
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1
    kw = dict(precision=precision, lanes_per_env=lpe, enable_wind=True, stochastic_wind=True,
              wind_percentile=None, auto_reset=True, tilt_sigma_rad=0.02, seed=9)
    # payload sums only: with cell pieces (binary64, the default) interior queries of both handles
    # would take the pieces whatever the tables hold
    kw["table_flags"] = L.TABLES_NO_CELL_PIECES
    full = make(pd, N, **kw)
    cut = make(pd, N, params=pd.Params().restrict_keys(4, 4), **kw)
    for t in range(T):
        o1, r1, d1, *_ = full.step(A[t])
        o2, r2, d2, *_ = cut.step(A[t])
        assert torch.equal(r1, r2) and torch.equal(d1, d2) and torch.equal(o1, o2), t
    assert torch.equal(full.state, cut.state)
    assert cut.counters()["rbf_misses"] > 100
    assert full.counters()["rbf_misses"] < cut.counters()["rbf_misses"]


def test_step_launch_inserts_its_misses(pd):
    """The misses a step launch solves are inserted by the launch's last workgroup (k_step's tail:
    a ticket per workgroup), with no k_insert launch or pd_flush_misses call after pd_step_n: with
    the tables cut to 4 keys, the first launch of 10 fused steps already grows them (the pd_stats
    entry counts, which only the inserter raises), every later launch keeps growing them up to
    the tables' load-factor cap, and the trajectory equals the full-table handle's bit for bit."""
    import torch
    N, T, F = 2048, 40, 10
    g = torch.Generator(device="cuda").manual_seed(12)
    A = (torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1).contiguous()
    kw = dict(lanes_per_env=2, enable_wind=True, stochastic_wind=True, wind_percentile=None, auto_reset=True,
              tilt_sigma_rad=0.02, seed=9, table_flags=L.TABLES_NO_CELL_PIECES)
    full = make(pd, N, **kw)
    cut = make(pd, N, params=pd.Params().restrict_keys(4, 4), **kw)
    misses, entries = [], []
    for c in range(T // F):
        c0 = cut.counters()
        for env in (full, cut):
            env.set_tuning(step_fuse=F)
            env.step_n_raw(A[c * F:(c + 1) * F])
        c1 = cut.counters()
        misses.append(c1["rbf_misses"] - c0["rbf_misses"])
        entries.append(c1["table_entries_cd"] + c1["table_entries_cl"])
    assert misses[0] > 100, misses
    assert entries[0] > 8 and all(b >= a for a, b in zip(entries, entries[1:])), (entries, misses)
    assert torch.equal(full.state, cut.state)


def test_cell_pieces_match_payload_sums(pd):
    """Binary64 handles evaluate trusted interior queries from cell pieces: the
    same first steps with the pieces (default) and with the payload sums only
    (PD_TABLES_NO_CELL_PIECES) from the same seeded states, |alpha| mostly inside the interior band
    (pitch tilt sigma 0.002 rad): C_D and C_L agree to rounding (1e-12 relative) on the first
    step, the states to the per-step tolerance after it; the counting launches report the piece
    path taken."""
    import torch
    N, T = 8192, 6
    g = torch.Generator(device="cuda").manual_seed(21)
    A = torch.rand(T, N, 1, device="cuda", generator=g) * 0.5 + 0.5
    kw = dict(lanes_per_env=2, enable_wind=False, auto_reset=False, tilt_sigma_rad=0.002, seed=5)
    pc = make(pd, N, **kw)
    ps = make(pd, N, table_flags=L.TABLES_NO_CELL_PIECES, **kw)
    pc.count_work(True)
    for t in range(T):
        _, r1, _, _, x1 = pc.step(A[t], info=True)
        _, r2, _, _, x2 = ps.step(A[t], info=True)
        # the first step from identical states: the coefficients to rounding; later steps start
        # from states that differ by that rounding (the per-step tolerances of s3)
        for k in ("CD", "CL"):
            d = (x1[k] - x2[k]).abs() / x2[k].abs().clamp_min(1e-3)
            assert float(d.max()) <= (1e-12 if t == 0 else 1e-9), (t, k, float(d.max()))
        ds = (pc.state - ps.state).abs() / ps.state.abs().clamp_min(1e-3)
        assert float(ds.max()) <= 1e-9, (t, float(ds.max()))
    st = pc.stats()
    interior = 2 * 4 * N * T - st["q_line"]        # 2 tables x 4 sub-steps per env step
    assert interior > 0.1 * 2 * 4 * N * T, st
    assert st["q_cell"] >= 0.99 * interior - st["q_verified"], st   # every trusted interior query
    assert ps.stats()["q_cell"] == 0


def test_fine_index_bit_identical(pd):
    """The fine index (one word per sub-cell naming the piece or bisector that settles the query,
    read in place of the cell record) picks the same piece as the cell / sub-cell records, so
    with and without it (PD_TABLES_NO_FINE_INDEX) the c3 workload -- wind, gusts below 15 km, tilt,
    auto-reset -- is bit-identical over 2 fused launches of 64 steps."""
    import torch
    N, T = 16384, 128
    g = torch.Generator(device="cuda").manual_seed(31)
    A = torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1
    A[:, : 3 * N // 4] = A[:, : 3 * N // 4] * 0.25 + 0.75      # 3/4 of the envs fly high throttle
    kw = dict(lanes_per_env=2, enable_wind=True, stochastic_wind=True, wind_percentile=None,
              auto_reset=True, tilt_sigma_rad=0.02, seed=13)
    fine = make(pd, N, **kw)
    rec = make(pd, N, table_flags=L.TABLES_NO_FINE_INDEX, **kw)
    for t0 in range(0, T, 64):
        o1 = fine.step_n(A[t0:t0 + 64])
        o2 = rec.step_n(A[t0:t0 + 64])
        for x, y in zip(o1, o2):
            assert torch.equal(x, y), t0
    assert torch.equal(fine.state, rec.state)


def test_fine_index_cell_edge_margins(pd):
    """Queries placed a fraction of the 1e-9 trust margin inside an interior cell's Mach edge
    (2e-10 .. 8e-10 cell widths, both edges, 120 cells): the fine index applies the record
    path's margin in the coordinates the record path uses (cell coordinates for a non-refined
    cell), so one step from these states is bit-identical with and without it (PD_TABLES_NO_FINE_INDEX).
    With the sub-cell margin on every word (round 3) the queries in (1.25e-10, 1e-9] cell widths
    of a non-refined cell's edge took its piece with the index and the payload sums without."""
    import torch
    probe = make(pd, 1)
    y = 12000.0
    a = float(probe.atmosphere(torch.tensor([y], dtype=torch.float64, device="cuda"))[2][0])
    w = 10.0 / 800.0                                            # C_D / C_L interior cells in Mach
    cells = np.arange(40, 760, 6)
    frac = np.array([2e-10, 5e-10, 8e-10, 1 - 2e-10, 1 - 5e-10, 1 - 8e-10])
    M = ((cells[:, None] + frac[None, :]) * w).ravel()
    n = len(M)
    s = np.tile(probe.state.cpu().numpy()[0], (n, 1))
    s[:, 1], s[:, 2], s[:, 3] = y, 0.0, -M * a                  # speed = |vy| exactly, Mach ~ M
    s[:, 6] = 1.5 * np.pi                                       # gamma of a vertical descent
    ae = np.radians(0.05)                                       # both tables interior (|deg(ae)| < radians(10))
    s[:, 4] = s[:, 6] - np.pi - ae                              # alpha_eff = gamma - theta - pi
    s[:, 7] = s[:, 4] - s[:, 6]
    outs = []
    for flags in (0, L.TABLES_NO_FINE_INDEX):
        env = make(pd, n, lanes_per_env=2, table_flags=flags)
        env.set_state(torch.tensor(s, device="cuda"))
        o = env.step(torch.zeros(n, 1, device="cuda"))
        outs.append((env.state.clone(), o[1].clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_env_shards_equal_single_handle(pd):
    """Multi-GPU layout on one device: two handles over contiguous shards (env_offset = rank*n,
    as bench.py assigns them) reproduce the single N-env handle bit for bit, wind + tilt +
    random percentile + auto-reset included (the Philox streams depend on the global env)."""
    import torch
    N, T = 4096, 50
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1
    kw = dict(enable_wind=True, stochastic_wind=True, wind_percentile=None, auto_reset=True,
              tilt_sigma_rad=0.02, seed=77)
    whole = make(pd, N, **kw)
    half = N // 2
    shards = [make(pd, half, env_offset=r * half, **kw) for r in range(2)]
    for t in range(T):
        o, r, d, *_ = whole.step(A[t])
        parts = [s.step(A[t, k * half:(k + 1) * half]) for k, s in enumerate(shards)]
        assert torch.equal(r, torch.cat([p[1] for p in parts])), t
        assert torch.equal(d, torch.cat([p[2] for p in parts])), t
    assert torch.equal(whole.state, torch.cat([s.state for s in shards], dim=0))


def test_auto_reset_and_full_size_properties(pd):
    """65 536 envs (config c3 size): auto-reset keeps every env in a valid episode; time
    advances by exactly 0.1 s per step; mass never increases; counters sane."""
    import torch
    N = 65536
    env = make(pd, N, mode="rl", auto_reset=True, seed=3)
    g = torch.Generator(device="cuda").manual_seed(0)
    s0 = env.state
    done_total = 0
    for t in range(200):
        a = torch.rand(N, 1, device="cuda", generator=g) * 2 - 1
        prev = env.state
        obs, r, dn, tr, ex = env.step(a)
        cur = env.state
        ended = (dn | tr)
        done_total += int(ended.sum())
        live = ~ended
        dt = (cur[live, 10] - prev[live, 10]).cpu().numpy()
        assert np.allclose(dt, 0.1, rtol=0, atol=1e-9)
        assert bool((cur[live, 9] <= prev[live, 9]).all())
        if ended.any():
            assert torch.equal(cur[ended], s0[ended])
    assert done_total > 0
    c = env.counters()
    assert c["nan_events"] == 0


def test_wind_injected_noise_vs_oracle(pd, oracle_mod):
    """Stochastic wind with the same injected normals (slotted per sub-step) on both sides.
    The oracle's own reference parity on the reference's recorded noise stream is
    tests/test_oracle_golden.py::test_wind_episode_injected_noise."""
    import torch
    d = golden("ref_episodes.npz")
    acts = d["rl_land_actions"][:500]
    rng = np.random.default_rng(17)
    noise = rng.standard_normal((len(acts), 8))
    su, sv = 1.3, 1.7
    env = make(pd, 1, mode="rl", enable_wind=True, stochastic_wind=True, wind_percentile=50)
    env.set_wind_sigmas(su, sv)
    o = oracle_mod.Oracle(phase=0, rtd=0, wind=True, stochastic=True, sigma_u=su, sigma_v=sv)
    o.E.noise_slotted = 1
    for t, a in enumerate(acts):
        obs, r, dn, tr, ex = env.step(torch.tensor(a[None]), noise=torch.tensor(noise[t][None]))
        s_o, r_o, dn_o, tr_o, tid, ob, info = o.step(a, f32=True, noise=noise[t])
        if dn_o or tr_o:
            break
    s = env.state.cpu().numpy()[0]
    err = np.abs(s - s_o) / (np.abs(s_o) + 1e-3)
    assert err.max() < 1e-8, dict(zip(ST, err))


def test_f32_teacher_forced(pd):
    """fp32 handle: one step from the reference's recorded states vs the reference, every channel
    (SURVEY 8(d)'s fp32 tolerance, 1e-5 of max(|x|, 1); theta_dot 2.5e-4, test_c3_f32_handle_shadowed).  The handle computes its
    forces in binary32 and integrates the state chain in binary64 within the step (alpha_eff =
    gamma - theta - pi from binary64 angles), so what is left is the binary32 rounding of the
    inputs and the forces.

    landing_burn's recorded states include tumbling ones (theta_ddot ~16 rad/s^2 with the
    aerodynamic moment's slope ~200 rad/s^2 per rad: an error grows ~2x per 0.1 s sub-step) and
    queries near a change of the 50-nearest set (the reference's k-NN RBF is discontinuous there),
    where no binary32 computation can hold 1e-5: the bound is the larger of the tolerance and 8x
    the step's own conditioning -- the binary64 handle's spread over inputs perturbed by one
    binary32 rounding (2^-24 relative, four draws).  Measured (profiles/r05_f32_teacher_forced.log):
    for 71 % of the 600 recorded landing_burn states that input rounding alone moves the binary64
    step beyond the tolerance (theta_dot spread: median 6.7e-5, 90 % 2.2e-3, max 0.35); the
    binary32 handle stays within 0.32 of 16x the spread on every channel, i.e. within ~5x what
    rounding its inputs costs; the states the rounding leaves within the tolerance hold it on every
    channel but theta (1.4e-5).  pure throttle: every state, every channel, at the tolerance."""
    import torch
    d = golden("ref_teacher_forced.npz")
    rng = np.random.default_rng(5)
    for tag, phase in (("pt", "landing_burn_pure_throttle"), ("lb", "landing_burn")):
        S0, A = d[f"{tag}_state_in"], d[f"{tag}_action"]
        prevs = d["lb_prevs"] if phase == "landing_burn" else None

        def run(prec, s0, pv):
            env = make(pd, len(S0), phase, mode="pso", precision=prec)
            env.set_state(torch.tensor(s0))
            if pv is not None:
                env.set_actuators(torch.tensor(pv).float() if prec == "f32" else torch.tensor(pv))
            env.step(torch.tensor(A))
            return env.state.double().cpu().numpy()

        ref = d[f"{tag}_state_out"]
        scale = np.maximum(np.abs(ref), 1.0)
        err = np.abs(run("f32", S0, prevs) - ref) / scale
        tol = np.full(11, 1e-5)
        tol[5] = 2.5e-4
        bound = np.broadcast_to(tol, err.shape).copy()
        if tag == "lb":
            s64 = run("f64", S0, prevs)
            spread = np.zeros_like(err)
            for _ in range(4):
                sg = lambda x: x * (1.0 + rng.choice([-1.0, 1.0], x.shape) * 2.0 ** -24)
                spread = np.maximum(spread, np.abs(run("f64", sg(S0), sg(prevs)) - s64) / scale)
            ill = (spread > tol).any(1)
            bound = np.maximum(bound, 8 * spread)
            print(f"f32 teacher-forced lb: {int(ill.sum())} of {len(S0)} states whose binary32 input rounding alone "
                  f"moves the binary64 step beyond the fp32 tolerance; spread quantiles (50/90/99/100 %) per channel:")
            for k, q in zip(ST, np.quantile(spread, [0.5, 0.9, 0.99, 1.0], axis=0).T):
                print(f"   {k:10s} spread {q}  err/bound max {np.max(err[:, ST.index(k)] / bound[:, ST.index(k)]):.3g}")
            wc = dict(zip(ST, err[~ill].max(0).tolist()))
            print("f32 teacher-forced lb, the other states:", wc)
        worst = dict(zip(ST, err.max(0).tolist()))
        print(f"f32 teacher-forced {tag}:", worst)
        bad = np.argwhere(err > bound)
        assert bad.size == 0, (tag, worst, bad[:8].tolist())


def test_rl_facade_matches_reference_episode(pd):
    """The drop-in rl_wrapped_env_pytorch facade replays the reference SAC-wrapper episode
    (float32 actions, float64 observations, Python float/bool returns)."""
    from pdenv.wrappers import rl_wrapped_env_pytorch
    d = golden("ref_episodes.npz")
    env = rl_wrapped_env_pytorch(flight_phase="landing_burn_pure_throttle", enable_wind=False,
                                 stochastic_wind=False, trajectory_length=1, discount_factor=0.99)
    assert env.state_dim == 2 and env.action_dim == 1
    obs0 = env.reset()
    assert obs0.shape == (2,)
    acts = d["rl_rand0_actions"]
    for t, a in enumerate(acts):
        obs, r, dn, tr, info = env.step(a.astype(np.float32))
        assert isinstance(r, float) and isinstance(dn, bool) and isinstance(tr, bool)
        assert abs(r - d["rl_rand0_reward"][t]) < 1e-9
        assert np.abs(obs - d["rl_rand0_obs"][t]).max() < 1e-6
        for k in ("state", "dynamic_pressure", "action_info"):
            assert k in info
    assert tr and env.truncation_id() == d["rl_rand0_trunc_id"][-1]


def test_pso_facade_batch_objective(pd):
    """pso_wrapped_env: batched particle evaluation on the device (landing_burn, 372-param actors)."""
    from pdenv.wrappers import pso_wrapped_env
    w = pso_wrapped_env(flight_phase="landing_burn")
    assert len(w.bounds) == 372
    rng = np.random.default_rng(0)
    X = rng.uniform(-1.5, 1.5, (256, 372)).astype(np.float32)
    fit = w.objective_function_batch(X, max_steps=400).cpu().numpy()
    assert fit.shape == (256,) and np.isfinite(fit).all()
    f0 = w.objective_function(X[0], max_steps=400)
    assert np.isfinite(f0)
    # experience_buffer as env_wrapped_ea.py:209-218 fills it: one tuple per step after the first,
    # each pairing the previous step's (state, action, reward) with this step's (state, action)
    import torch
    buf = w.experience_buffer
    n = w.last_objective_steps
    assert len(buf) == n - 1
    for later, earlier in zip(buf[1:], buf[:-1]):
        assert np.array_equal(later[0], earlier[3]) and torch.equal(later[1], earlier[4])
        assert isinstance(later[2], float)
    w.reset()
    assert w.experience_buffer == []


@pytest.mark.parametrize("phase,pidx", [("landing_burn_pure_throttle", 0), ("landing_burn", 1)])
def test_policy_first_step_vs_oracle(pd, oracle_mod, phase, pidx):
    """pd_rollout_policy with max_steps = 1: the in-kernel actor (binary32, sequential sums)
    drives one env-step from the nominal state for 256 particles; the resulting states and
    -reward equal the oracle actor + oracle env to the teacher-forced tolerance."""
    import torch
    rng = np.random.default_rng(21 + pidx)
    npar = 249 if pidx == 0 else 372
    W = np.concatenate([rng.uniform(-1.5, 1.5, (128, npar)), rng.uniform(-0.3, 0.3, (128, npar))]).astype(np.float32)
    env = make(pd, len(W), phase=phase, mode="pso")
    fit, steps = env.rollout_policy(torch.tensor(W), max_steps=1)
    S = env.state.cpu().numpy()
    assert (steps.cpu().numpy() == 1).all()
    for i in range(0, len(W), 8):
        o = oracle_mod.Oracle(phase=pidx, rtd=1)
        a = oracle_mod.actor(pidx, W[i], o.state)
        s, r, *_ = o.step(a, f32=True)
        np.testing.assert_allclose(S[i], s, rtol=1e-10, atol=1e-9)
        assert float(fit[i]) == pytest.approx(-r, rel=1e-12, abs=1e-9)


@pytest.mark.parametrize("phase,pidx", [("landing_burn_pure_throttle", 0), ("landing_burn", 1)])
def test_policy_rollout_vs_oracle_and_reference(pd, oracle_mod, phase, pidx):
    """Whole PSO objectives on the device against the oracle's (same actor arithmetic) for 64
    seeded particles, and against the reference's objective_function for its 8 recorded
    particles.  Saturated landing_burn actors tumble the vehicle (chaotic attitude),
    so the landing_burn bounds are on fitness (the quantity PSO consumes), not on states."""
    import torch
    rng = np.random.default_rng(5 + pidx)
    npar = 249 if pidx == 0 else 372
    d = golden("ref_pso_objective.npz")
    tag = "pt" if pidx == 0 else "lb"
    W = np.concatenate([d[f"{tag}_individuals"], rng.uniform(-1.5, 1.5, (28, npar)),
                        rng.uniform(-0.4, 0.4, (28, npar))]).astype(np.float32)
    env = make(pd, len(W), phase=phase, mode="pso")
    fit, steps = env.rollout_policy(torch.tensor(W), max_steps=2200)
    fit, steps = fit.cpu().numpy(), steps.cpu().numpy()
    ofit, osteps = oracle_mod.rollout_policy(pidx, W, 2200)
    rel = np.abs(fit - ofit) / np.abs(ofit)
    if pidx == 0:
        assert (steps == osteps).all() and rel.max() < 1e-7, (steps, osteps, rel)
    else:
        # tumbling vehicles amplify 1e-13 RBF differences ~3x per step: bounds on the ensemble
        assert (steps == osteps).mean() >= 0.8 and (rel < 1e-6).mean() >= 0.8 and np.median(rel) < 1e-9, rel
    ref = d[f"{tag}_fitness"]
    rref = np.abs(fit[:8] - ref) / np.abs(ref)
    if pidx == 0:
        assert list(steps[:8]) == list(d["pt_length"]) and rref.max() < 1e-7, rref
    else:
        assert (rref < 1e-6).sum() >= 6, rref    # actor ulps vs torch's MKL sgemv order


def test_policy_trajectory_teacher_forced(pd, oracle_mod):
    """landing_burn, 96 particles: the device's policy trajectory, step by step.  The state and
    actuator memory after k policy steps (a rollout with max_steps = k; the rollout is
    deterministic) are fed to the oracle's actor + physics; the result must equal the device's
    state after k + 1 steps to the teacher-forced tolerance, for k = 0..7 and every particle
    still flying.  This checks the fused actor and the env along the actual policy trajectory
    without the chaotic amplification of free-running comparisons."""
    import torch
    rng = np.random.default_rng(31)
    W = rng.uniform(-1.5, 1.5, (96, 372)).astype(np.float32)
    env = make(pd, len(W), phase="landing_burn", mode="pso")
    S, A, NS = [], [], []
    for k in range(9):
        _, steps = env.rollout_policy(torch.tensor(W), max_steps=k)
        S.append(env.state.cpu().numpy()); A.append(env.actuators.cpu().numpy()); NS.append(steps.cpu().numpy())
    checked = 0
    for k in range(8):
        for i in range(len(W)):
            if NS[k + 1][i] != k + 1:          # finished before step k + 1
                continue
            a = oracle_mod.actor(1, W[i], S[k][i])
            o = oracle_mod.Oracle(phase=1, rtd=1)
            s, _ = o.physics(S[k][i], a, f32=True, prevs=tuple(A[k][i]))
            err = np.abs(s - S[k + 1][i]) / np.maximum(np.abs(S[k + 1][i]), 1e-3)
            tol = np.full(11, 1e-10); tol[5] = 1e-8
            assert (err < tol).all(), (k, i, dict(zip(ST, err)))
            checked += 1
    assert checked > 300


def test_pso_facade_fused_vs_torch_actor(pd):
    """pso_wrapped_env.objective_function_batch (actor fused in the step kernel) against the
    same objective with the actor as torch.bmm between pd_step launches."""
    from pdenv.wrappers import pso_wrapped_env
    rng = np.random.default_rng(8)
    m = pso_wrapped_env(flight_phase="landing_burn_pure_throttle")
    X = rng.uniform(-0.5, 0.5, (256, len(m.bounds)))
    a = m.objective_function_batch(X).cpu().numpy()
    b = m.objective_function_batch_torch(X).cpu().numpy()
    rel = np.abs(a - b) / np.abs(b)
    assert np.median(rel) < 1e-9 and (rel < 1e-3).mean() >= 0.95, rel


def test_sac_collector_single_rank(pd):
    """c5 data path on one rank: actor -> pd_step -> transition slab -> device replay buffer.
    Every stored transition is (obs the actor saw, its action, reward, post-step obs, done), and
    the next step's input is the post-auto-reset observation."""
    import torch
    from pdenv.sac import Actor, DeviceReplayBuffer, SACCollector
    torch.manual_seed(0)
    N = 2048
    env = make(pd, N, mode="rl", auto_reset=True, seed=4)
    actor = Actor(2, 1).cuda()
    buf = DeviceReplayBuffer(4 * N, 2, 1, "cuda")
    col = SACCollector(env, actor, buf, generator=torch.Generator(device="cuda").manual_seed(1))
    obs0 = col.obs.clone()
    full = col.step()
    assert full.shape == (N, 7) and len(buf) == N
    assert torch.equal(buf.data[:N, :2], obs0)
    assert (buf.data[:N, 2].abs() <= 1).all()
    # replay the same actions on a twin env: identical rewards / next obs / done
    twin = make(pd, N, mode="rl", auto_reset=True, seed=4)
    twin.reset()
    o, r, d, tr, _ = twin.step(buf.data[:N, 2:3])
    assert torch.equal(buf.data[:N, 3], r.float()) and torch.equal(buf.data[:N, 4:6], o.float())
    assert torch.equal(buf.data[:N, 6], d.float())
    for _ in range(300):
        col.step()
    assert len(buf) == 4 * N
    t = env.state[:, 10]
    assert (t < t.max() - 1.0).any()        # some episodes ended (truncated) and were auto-reset
    assert torch.isfinite(buf.data).all()


def _np_pso_step(x, v, pb, pbf, fit, sb, swarm, lo, hi, w, c1, c2, seed, gen, offset):
    """particle_swarm_optimisation.py:437-441, 515-519, 112-118 in NumPy, parameter-major."""
    from philox_np import philox, u01
    P = x.shape[1]
    g = np.arange(offset, offset + P, dtype=np.uint64)
    r = philox(g & np.uint64(0xFFFFFFFF), g >> np.uint64(32), np.full(P, gen), np.full(P, 32),
               seed & 0xFFFFFFFF, seed >> 32)
    r1, r2 = u01(r[0], r[1]), u01(r[2], r[3])
    better = fit < pbf
    pb = np.where(better[None, :], x, pb)
    inertia = w * v
    cognitive = c1 * r1[None, :] * (pb - x)
    social = c2 * r2[None, :] * (sb[swarm].T - x)
    v = inertia + cognitive + social
    xn = x + v
    xn = np.where(xn < lo[:, None], lo[:, None], np.where(xn > hi[:, None], hi[:, None], xn))
    return xn, v, pb, np.where(better, fit, pbf)


def test_pso_step_matches_numpy(pd):
    """pd_pso_step (binary64, one r1/r2 per particle from Philox) is bit-identical to the
    reference's update written in NumPy with the same uniforms."""
    import torch
    from pdenv import _lib as L
    from pdenv.env import _ptr
    rng = np.random.default_rng(3)
    P, D, S = 300, 372, 3
    x = rng.uniform(-1.5, 1.5, (D, P)); v = rng.normal(0, 0.2, (D, P)); pb = rng.uniform(-1.5, 1.5, (D, P))
    pbf = rng.uniform(0, 10, P); pbf[::7] = np.inf
    fit = rng.uniform(0, 10, P); sb = rng.uniform(-1.5, 1.5, (S, D))
    swarm = rng.integers(0, S, P).astype(np.int32)
    lo, hi = np.full(D, -1.5), np.full(D, 1.5)
    w, c1, c2, seed, gen, off = 0.83, 1.0, 1.0, 0x123456789A, 7, 1000
    T = {k: torch.tensor(a).cuda() for k, a in dict(x=x, v=v, pb=pb, pbf=pbf, fit=fit, sb=sb, swarm=swarm,
                                                      lo=lo, hi=hi).items()}
    x32 = torch.empty(D, P, dtype=torch.float32, device="cuda")
    lib = L.load()
    L.check(lib.pd_pso_step(P, D, _ptr(T["fit"]), _ptr(T["pbf"]), _ptr(T["x"]), _ptr(T["v"]), _ptr(T["pb"]),
                            _ptr(T["sb"]), _ptr(T["swarm"]), _ptr(T["lo"]), _ptr(T["hi"]), w, c1, c2, seed, gen,
                            off, _ptr(x32), None))
    torch.cuda.synchronize()
    xn, vn, pbn, pbfn = _np_pso_step(x, v, pb, pbf, fit, sb, swarm, lo, hi, w, c1, c2, seed, gen, off)
    assert np.array_equal(T["x"].cpu().numpy(), xn) and np.array_equal(T["v"].cpu().numpy(), vn)
    assert np.array_equal(T["pb"].cpu().numpy(), pbn) and np.array_equal(T["pbf"].cpu().numpy(), pbfn)
    assert np.array_equal(x32.cpu().numpy(), xn.astype(np.float32))


@pytest.mark.parametrize("D", [372, 249, 10])
def test_pso_step_chunked_matches_numpy(pd, D):
    """pd_pso_step_chunked: the same update bit for bit (one thread per four parameters), its
    float32 copy in the chunked layout [ceil(D/4)][P][4] with zeros past D (D = 249, the pure
    throttle actor, and 10 end inside a chunk)."""
    import torch
    from pdenv import _lib as L
    from pdenv.env import _ptr
    from pdenv.pso import chunk4, unchunk4
    rng = np.random.default_rng(5)
    P, S = 777, 4
    x = rng.uniform(-1.5, 1.5, (D, P)); v = rng.normal(0, 0.2, (D, P)); pb = rng.uniform(-1.5, 1.5, (D, P))
    pbf = rng.uniform(0, 10, P); pbf[::5] = np.inf
    fit = rng.uniform(0, 10, P); fit[::11] = np.nan
    sb = rng.uniform(-1.5, 1.5, (S, D))
    swarm = rng.integers(0, S, P).astype(np.int32)
    lo, hi = np.full(D, -1.5), np.full(D, 1.5)
    w, c1, c2, seed, gen, off = 0.61, 1.0, 1.0, 0xABCDEF01234, 3, 77
    T = {k: torch.tensor(a).cuda() for k, a in dict(x=x, v=v, pb=pb, pbf=pbf, fit=fit, sb=sb, swarm=swarm,
                                                      lo=lo, hi=hi).items()}
    C = (D + 3) // 4
    x32c = torch.full((C, P, 4), 7.0, dtype=torch.float32, device="cuda")   # (the pad lanes must be written)
    lib = L.load()
    L.check(lib.pd_pso_step_chunked(P, D, _ptr(T["fit"]), _ptr(T["pbf"]), _ptr(T["x"]), _ptr(T["v"]), _ptr(T["pb"]),
                                    _ptr(T["sb"]), _ptr(T["swarm"]), _ptr(T["lo"]), _ptr(T["hi"]), w, c1, c2, seed,
                                    gen, off, _ptr(x32c), None))
    torch.cuda.synchronize()
    xn, vn, pbn, pbfn = _np_pso_step(x, v, pb, pbf, fit, sb, swarm, lo, hi, w, c1, c2, seed, gen, off)
    assert np.array_equal(T["x"].cpu().numpy(), xn) and np.array_equal(T["v"].cpu().numpy(), vn)
    assert np.array_equal(T["pb"].cpu().numpy(), pbn)
    assert np.array_equal(T["pbf"].cpu().numpy(), pbfn, equal_nan=True)
    ref = chunk4(torch.tensor(xn.astype(np.float32)))
    assert torch.equal(x32c.cpu(), ref)
    assert np.array_equal(unchunk4(x32c, D).cpu().numpy(), xn.astype(np.float32))


@pytest.mark.parametrize("phase,wind", [("landing_burn", False), ("landing_burn_pure_throttle", False),
                                        ("landing_burn", True)])
def test_rollout_policy_chunked_same_bits(pd, phase, wind):
    """pd_rollout_policy_chunked on chunk4'd weights gives pd_rollout_policy's fitness and
    episode lengths bit for bit (refill launch and the compacted list; with stochastic wind the
    per-check launches)."""
    import torch
    from pdenv.env import _ptr, _stream
    from pdenv import _lib as L
    from pdenv.pso import chunk4
    n = 3000
    env = pd.PoweredDescentEnv(n, flight_phase=phase, mode="pso", device=0, enable_wind=wind, stochastic_wind=wind)
    D = 372 if phase == "landing_burn" else 249
    W = torch.from_numpy(np.random.default_rng(11).uniform(-1.5, 1.5, (D, n)).astype(np.float32)).cuda()
    W4 = chunk4(W)
    lib = L.load()
    for tune in (dict(), dict(policy_refill=-1, policy_list=1)):
        if tune:
            env.set_tuning(**tune)
        out = []
        for fn, w in ((lib.pd_rollout_policy, W), (lib.pd_rollout_policy_chunked, W4)):
            fit = torch.empty(n, dtype=torch.float64, device="cuda")
            steps = torch.empty(n, dtype=torch.int32, device="cuda")
            L.check(fn(env.h, _ptr(w), D, 400, _ptr(fit), _ptr(steps), 8, _stream(env.device)))
            torch.cuda.synchronize()
            out.append((fit.cpu().numpy(), steps.cpu().numpy()))
        assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1]), tune
        assert (out[0][1] >= 1).all()
    env.close()


def test_rollout_policy_repeat_and_null_steps(pd):
    """A policy rollout starts from nothing its handle's previous rollouts left (k_policy_init:
    every env reset, fitness zeroed, live list and counts re-initialised): the same weights on
    the same handle give the same bits after a rollout of other weights, with and without the
    episode-length output (k_policy_finish skips the copy when steps is NULL), on the refill
    launch and on the per-check list launches."""
    import torch
    from pdenv.env import _ptr, _stream
    from pdenv import _lib as L
    from pdenv.pso import chunk4
    n, D = 2500, 372
    env = pd.PoweredDescentEnv(n, flight_phase="landing_burn", mode="pso", device=0)
    g = np.random.default_rng(21)
    W = chunk4(torch.from_numpy(g.uniform(-1.5, 1.5, (D, n)).astype(np.float32)).cuda())
    W2 = chunk4(torch.from_numpy(g.uniform(-1.5, 1.5, (D, n)).astype(np.float32)).cuda())
    lib = L.load()

    def roll(w, with_steps=True):
        fit = torch.full((n,), 123.0, dtype=torch.float64, device="cuda")
        steps = torch.empty(n, dtype=torch.int32, device="cuda") if with_steps else None
        L.check(lib.pd_rollout_policy_chunked(env.h, _ptr(w), D, 400, _ptr(fit), _ptr(steps) if with_steps else None,
                                              8, _stream(env.device)))
        torch.cuda.synchronize()
        return fit.cpu().numpy(), (steps.cpu().numpy() if with_steps else None)

    for tune in (dict(), dict(policy_refill=-1, policy_list=1)):
        if tune:
            env.set_tuning(**tune)
        f0, s0 = roll(W)
        roll(W2)
        f1, s1 = roll(W)
        f2, _ = roll(W, with_steps=False)
        assert np.array_equal(f0, f1) and np.array_equal(s0, s1) and np.array_equal(f0, f2), tune
        assert (s0 >= 1).all() and np.isfinite(f0).all()
    env.close()


def test_pso_swarm_minima_and_bests_vs_numpy(pd):
    """pd_pso_swarm_minima (the reference's sequential `if fitness < subswarm_best` per subswarm,
    particle_swarm_optimisation.py:437-441: a NaN never wins, ties keep the lower index, +inf for
    a subswarm with no particle of non-NaN fitness) and pd_pso_update_bests (strictly better
    replaces; the first subswarm holding the minimum feeds the global best) against a Python
    restatement of that loop.  Sizes cross the 1 024-particle blocks of the two-pass argmin."""
    import torch
    from pdenv import _lib as L
    from pdenv.env import _ptr
    lib = L.load()
    rng = np.random.default_rng(12)
    for trial in range(8):
        P, D, S = int(rng.integers(1, 5000)), int(rng.integers(1, 400)), int(rng.integers(1, 6))
        if trial == 6:
            P = 40000                                           # 40 pass-1 blocks
        fit = np.round(rng.normal(size=P), 1)                  # many ties
        if trial % 2:
            fit[rng.integers(0, P, 3)] = np.nan
            fit[0] = np.nan                                     # a NaN first in its subswarm
        sw = rng.integers(0, S, P).astype(np.int32)
        if trial == 3:
            sw[sw == S - 1] = 0                                 # an empty subswarm
        if trial == 5 and S > 1:
            fit[sw == 1] = np.nan                               # a subswarm of NaNs only
        x = rng.normal(size=(D, P))
        T = {k: torch.tensor(v, device="cuda") for k, v in dict(fit=fit, sw=sw, x=x).items()}
        mf = torch.empty(S, dtype=torch.float64, device="cuda")
        mp = torch.empty(S, D, dtype=torch.float64, device="cuda")
        nb = int(lib.pd_pso_swarm_minima_scratch_bytes(P, S))
        scratch = torch.empty(nb, dtype=torch.uint8, device="cuda")
        if trial == 0:   # the caller's scratch is checked: missing or too small is refused
            assert lib.pd_pso_swarm_minima(P, D, S, _ptr(T["fit"]), _ptr(T["sw"]), _ptr(T["x"]), _ptr(mf), _ptr(mp),
                                           None, 0, None) == L.PD_ERR_INVALID
            assert lib.pd_pso_swarm_minima(P, D, S, _ptr(T["fit"]), _ptr(T["sw"]), _ptr(T["x"]), _ptr(mf), _ptr(mp),
                                           _ptr(scratch), nb - 8, None) == L.PD_ERR_INVALID
        L.check(lib.pd_pso_swarm_minima(P, D, S, _ptr(T["fit"]), _ptr(T["sw"]), _ptr(T["x"]), _ptr(mf), _ptr(mp),
                                        _ptr(scratch), nb, None))
        sbf = torch.tensor(rng.normal(size=S), device="cuda"); sb = torch.tensor(rng.normal(size=(S, D)), device="cuda")
        gbf = torch.tensor(0.5, dtype=torch.float64, device="cuda"); gb = torch.zeros(D, dtype=torch.float64, device="cuda")
        sbf0, sb0 = sbf.cpu().numpy().copy(), sb.cpu().numpy().copy()
        L.check(lib.pd_pso_update_bests(S, D, _ptr(mf), _ptr(mp), _ptr(sbf), _ptr(sb), _ptr(gbf), _ptr(gb), None))
        torch.cuda.synchronize()
        ef, ep = np.full(S, np.inf), np.zeros((S, D))
        for s in range(S):
            best, bi = np.inf, -1
            for p in np.flatnonzero(sw == s):                   # the reference's loop
                if bi < 0 and not np.isnan(fit[p]) or fit[p] < best:
                    best, bi = fit[p], p
            if bi >= 0:
                ef[s], ep[s] = best, x[:, bi]
        assert np.array_equal(mf.cpu().numpy(), ef) and np.array_equal(mp.cpu().numpy(), ep)
        for s in range(S):
            if ef[s] < sbf0[s]:
                sbf0[s], sb0[s] = ef[s], ep[s]
        assert np.array_equal(sbf.cpu().numpy(), sbf0) and np.array_equal(sb.cpu().numpy(), sb0)
        g, gv = 0.5, np.zeros(D)
        for s in range(S):
            if sbf0[s] < g:
                g, gv = sbf0[s], sb0[s]
        assert float(gbf) == g and np.array_equal(gb.cpu().numpy(), gv)


def test_pso_share_merged_into_next_rollout(pd):
    """share_information's candidates ride along with the next generation's rollout (S - 1 more
    envs): with a share every generation, the run equals one that evaluates every share's
    candidates on their own handle, bit for bit (candidate fitness, bests, swarm state)."""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    prm = dict(generations=6, communication_freq=1, migration_freq=2, num_sub_swarms=3, re_initialise_generation=99)
    runs, sizes = [], []
    for merge in (True, False):
        opt = ParticleSubswarmOptimisationGPU("landing_burn", pso_params=prm, pop_size=96, seed=7, max_steps=300)
        if not merge:
            opt._mergeable = lambda: False
        seen = []
        ev = opt.evaluate
        opt.evaluate = lambda x32, ev=ev, seen=seen: (seen.append(x32.shape[1]), ev(x32))[1]
        for g in range(6):
            opt.generation(g)
        opt.flush_share()
        runs.append(opt)
        sizes.append(seen)
    a, b = runs
    assert 96 + 2 in sizes[0] and 96 + 2 not in sizes[1]       # the merged rollout ran (and only there)
    assert len(a.share_history) == len(b.share_history) >= 3
    for (ga, ma, fa), (gb, mb, fb) in zip(a.share_history, b.share_history):
        assert ga == gb and ma == mb and torch.equal(fa, fb)
    for k in ("x", "v", "pb", "pbf", "swarm", "sb", "sbf_t", "gbf_t", "gb_t"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_pso_driver_stochastic_wind_host_share_path(pd):
    """The PSO driver on a windy swarm with stochastic gusts: its share candidates cannot ride
    with the next rollout (a candidate's gusts depend on its env index), so share_information
    takes the host path and evaluates them on the share handle; the policy rollouts run the windy
    kernels' per-check launches.  Two runs of the same seed agree bit for bit; every share that
    moved a subswarm is logged with its candidates' finite fitness."""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    prm = dict(generations=5, communication_freq=1, migration_freq=2, num_sub_swarms=3, re_initialise_generation=99)
    runs = []
    for _ in range(2):
        opt = ParticleSubswarmOptimisationGPU("landing_burn", pso_params=prm, pop_size=96, seed=11, max_steps=300,
                                              enable_wind=True, stochastic_wind=True)
        assert not opt._mergeable()
        for g in range(5):
            opt.generation(g)
        opt.flush_share()
        runs.append(opt)
    a, b = runs
    ha, hb = a.share_history, b.share_history
    assert len(ha) == len(hb) >= 1
    for (ga, ma, fa), (gb, mb, fb) in zip(ha, hb):
        assert ga == gb and ma == mb and torch.equal(fa, fb) and bool(torch.isfinite(fa).all())
    for k in ("x", "v", "pb", "pbf", "swarm", "sb", "sbf_t", "gbf_t", "gb_t"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert math.isfinite(a.gbf)


def test_pso_driver_generations_vs_numpy(pd):
    """Three generations of the device subswarm PSO (evaluation, subswarm/global bests, inertia
    schedule, update, share_information and migrate_particles at generation 2) against a NumPy
    restatement of ParticleSubswarmOptimisation.run fed the same fitness values."""
    import random
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU
    prm = dict(generations=3, communication_freq=2, migration_freq=2, re_initialise_generation=99)
    opt = ParticleSubswarmOptimisationGPU("landing_burn_pure_throttle", pso_params=prm, pop_size=64, seed=5,
                                          max_steps=400)
    x = opt.x.cpu().numpy().copy(); v = np.zeros_like(x); pb = np.zeros_like(x)
    pbf = np.full(opt.P, np.inf); swarm = opt.swarm.cpu().numpy().copy()
    S, D = opt.S, opt.D
    sb = np.zeros((S, D)); sbf = [np.inf] * S; gbf = np.inf
    lo, hi = np.full(D, -1.5), np.full(D, 1.5)
    rng = random.Random(5)
    for gen in range(3):
        opt.generation(gen)
        fit = opt.last_fitness.cpu().numpy()
        for s in range(S):
            idx = np.nonzero(swarm == s)[0]
            i = idx[np.argmin(fit[idx])]
            if fit[i] < sbf[s]:
                sbf[s], sb[s] = fit[i], x[:, i].copy()
        for s in range(S):
            gbf = min(gbf, sbf[s])
        w = 0.9 - (0.9 - 0.4) * gen / 3
        x, v, pb, pbf = _np_pso_step(x, v, pb, pbf, fit, sb, swarm, lo, hi, w, 1, 1, 5, gen, 0)
        if gen == 2:
            best = int(np.argmin(sbf))
            moved = [i for i in range(S) if i != best and rng.random() < 0.5]
            if moved:
                assert opt.share_log[0] == moved
                for k, i in enumerate(moved):
                    sb[i] = (1 - 0.3) * sb[i] + 0.3 * sb[best]
                    f = float(opt.share_log[1][k])
                    if f < sbf[i]:
                        sbf[i] = f
            members = [list(np.nonzero(swarm == s)[0]) for s in range(S)]
            for i in range(S):
                if len(members[i]) > 1:
                    k = rng.randrange(len(members[i]))
                    g = members[i].pop(k)
                    t = rng.choice([j for j in range(S) if j != i])
                    members[t].append(g)
                    swarm[g] = t
    assert np.array_equal(opt.x.cpu().numpy(), x) and np.array_equal(opt.v.cpu().numpy(), v)
    assert np.array_equal(opt.pb.cpu().numpy(), pb) and np.array_equal(opt.pbf.cpu().numpy(), pbf)
    assert np.array_equal(opt.sb.cpu().numpy(), sb) and opt.sbf == sbf and opt.gbf == gbf
    assert np.array_equal(opt.swarm.cpu().numpy(), swarm)


def test_sac_step_fused_sampling_and_slab(pd):
    """pd_step_sac (c5's fused step): the action sampled in the kernel from the actor heads equals
    torch's Actor.sample arithmetic (clamp, exp, mean + std eps, tanh, x max_action) to 3 float32
    ulps, and with that action a twin env stepped by pd_step gives the slab's reward, next
    observation and done and the next observation bit for bit (the slab's state is the float32
    observation the actor saw)."""
    import torch
    from pdenv.sac import Actor
    torch.manual_seed(3)
    N = 2048
    actor = Actor(2, 1).cuda()
    env = make(pd, N, mode="rl", auto_reset=True, seed=9, tilt_sigma_rad=0.05)
    twin = make(pd, N, mode="rl", auto_reset=True, seed=9, tilt_sigma_rad=0.05)
    obs = env.reset().float().contiguous()
    twin.reset()
    g = torch.Generator(device="cuda").manual_seed(5)
    act = torch.empty(N, 1, device="cuda")
    slab = torch.empty(N, 7, device="cuda")
    for t in range(60):
        with torch.no_grad():
            f = actor.shared_net(obs)
            mean, ls = actor.mean(f), actor.log_std(f)
        eps = torch.randn(mean.shape, device="cuda", generator=g)
        ref = torch.tanh(mean + torch.clamp(ls, -20.0, 2.0).exp() * eps) * 1.0
        seen = obs.clone()
        if t % 2:
            env.step_sac(mean, ls, eps, -20.0, 2.0, 1.0, action=act, slab=slab, obs32=obs)
        else:                               # both heads in one [N, 2] array (head_stride 2)
            env.step_sac(None, None, eps, -20.0, 2.0, 1.0, action=act, slab=slab, obs32=obs,
                         heads=torch.cat([mean, ls], dim=1).contiguous())
        assert (act - ref).abs().max() <= 2e-7, (t, float((act - ref).abs().max()))
        o, r, d, _, _ = twin.step(act)
        assert torch.equal(slab[:, :2], seen) and torch.equal(slab[:, 2:3], act)
        assert torch.equal(slab[:, 3], r.float()) and torch.equal(slab[:, 4:6], o.float())
        assert torch.equal(slab[:, 6], d.float())
        assert torch.equal(obs, twin.observe().float()), t        # post-auto-reset observation
    assert int(twin.episode_counters()[0].max()) >= 1 or bool(d.any())


@pytest.mark.parametrize("S,A,H,L", [(2, 1, 256, 2), (5, 4, 256, 3), (2, 1, 128, 1), (5, 4, 512, 2)])
def test_sac_actor_kernel_vs_torch(pd, S, A, H, L):
    """pd_sac_actor (the Actor's shared MLP on MFMA and both heads in one launch) against the
    reference Actor's forward in PyTorch (sac_pytorch.py:129-159): f32 heads equal to f32
    rounding (the sums run in another order; max |d| <= 2e-5 + 1e-4 |ref|), over observations
    spanning the normalised range and a batch that is not a multiple of the 16-env tile."""
    import torch
    from pdenv.sac import Actor, ActorKernel
    torch.manual_seed(11)
    n = 4096 + 5
    actor = Actor(S, A, hidden_dim=H, n_hidden_layers=L).cuda()
    assert ActorKernel.supported(actor)
    obs = (torch.rand(n, S, device="cuda") * 4 - 2).contiguous()
    heads = torch.full((n, 2 * A), float("nan"), device="cuda")
    ActorKernel(actor)(obs, heads)
    with torch.no_grad():
        f = actor.shared_net(obs)
        ref = torch.cat([actor.mean(f), actor.log_std(f)], dim=1)
    d = (heads - ref).abs()
    assert torch.isfinite(heads).all()
    assert (d <= 2e-5 + 1e-4 * ref.abs()).all(), float(d.max())


def test_sac_ring_step_draws_rows_priorities(pd):
    """pd_step_sac_ring (c5's step kernel): eps is drawn in the kernel (N(0, 1): moments and a
    KS bound over 64 k draws; new draws every step), the action equals torch's Actor.sample
    arithmetic on the kernel's heads and eps to 2e-7, the transition rows land in the replay
    ring at the device-held position -- wrapping, since the capacity is 1.5 N + 7 -- with the
    buffer's max priority, the position and size advance, and a twin env stepped by pd_step
    with the same actions gives the rows' reward, next observation and done bit for bit."""
    import torch
    from scipy import stats
    from pdenv.sac import Actor, ActorKernel, DevicePrioritizedReplayBuffer
    torch.manual_seed(5)
    N = 4096
    actor = Actor(2, 1).cuda()
    env = make(pd, N, mode="rl", auto_reset=True, seed=21, tilt_sigma_rad=0.05)
    twin = make(pd, N, mode="rl", auto_reset=True, seed=21, tilt_sigma_rad=0.05)
    cap = N + N // 2 + 7
    buf = DevicePrioritizedReplayBuffer(cap, 2, 1, "cuda")
    buf.max_prio_dev.fill_(2.5)
    obs = env.reset().float().contiguous()
    twin.reset()
    kern = ActorKernel(actor)
    heads = torch.empty(N, 2, device="cuda")
    act = torch.empty(N, 1, device="cuda")
    eps = torch.empty(N, 1, device="cuda")
    draws, prev = [], None
    for t in range(16):
        seen = obs.clone()
        kern(obs, heads)
        h = heads.clone()
        pos = buf.position
        env.step_sac_ring(heads, -20.0, 2.0, 1.0, ring=buf.data, capacity=cap, ring_state=buf.state_dev,
                          priorities=buf.priorities, max_priority=buf.max_prio_dev, action=act, obs32=obs,
                          eps_out=eps)
        buf.note_appended(N)
        st = buf.state_dev.cpu().tolist()
        assert st == [buf.position, buf.size, 0], (t, st)
        ref = torch.tanh(h[:, :1] + torch.clamp(h[:, 1:], -20.0, 2.0).exp() * eps)
        assert (act - ref).abs().max() <= 2e-7, (t, float((act - ref).abs().max()))
        rows = buf.rows(pos, N)
        o, r, d, _, _ = twin.step(act)
        assert torch.equal(rows[:, :2], seen) and torch.equal(rows[:, 2:3], act)
        assert torch.equal(rows[:, 3], r.float()) and torch.equal(rows[:, 4:6], o.float())
        assert torch.equal(rows[:, 6], d.float())
        idx = (torch.arange(N, device="cuda") + pos) % cap
        assert (buf.priorities[idx] == 2.5).all()
        assert torch.equal(obs, twin.observe().float()), t
        if prev is not None:
            assert not torch.equal(eps, prev)
        prev = eps.clone()
        draws.append(eps.cpu().numpy().ravel())
    z = np.concatenate(draws)
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    assert stats.kstest(z, "norm").pvalue > 1e-4
    assert len(buf) == cap


@pytest.mark.parametrize("S,A,H,L,lpe", [(2, 1, 256, 2, 0), (2, 1, 128, 3, 0), (5, 4, 256, 2, 16),
                                          (2, 1, 256, 2, 2), (2, 1, 512, 2, 0)])
def test_sac_fused_step_equals_two_launches(pd, S, A, H, L, lpe):
    """pd_step_sac_fused (the Actor's MLP in the step kernel's prologue: c5's whole collection step
    in one launch) against pd_sac_actor + pd_step_sac_ring on a twin env: the same heads, eps,
    actions, replay-ring rows, priorities, ring position and next observations, bit for bit,
    over 12 steps with auto-resets (ring wrapping: capacity 1.5 N + 3); a batch that is not a
    multiple of the 16-env tile.  The handles that cannot take the one launch (2 lanes per env,
    hidden 512) run the two launches inside pd_step_sac_fused: the same bits too."""
    import torch
    from pdenv.sac import Actor, ActorKernel, DevicePrioritizedReplayBuffer
    torch.manual_seed(3)
    N = 4096 - 9
    phase = "landing_burn_pure_throttle" if A == 1 else "landing_burn"
    actor = Actor(S, A, hidden_dim=H, n_hidden_layers=L).cuda()
    assert ActorKernel.supported(actor)
    kern = ActorKernel(actor)
    envs, bufs, outs = [], [], []
    for fused in (True, False):
        env = make(pd, N, phase=phase, mode="rl", auto_reset=True, seed=17, tilt_sigma_rad=0.05, lanes_per_env=lpe)
        cap = N + N // 2 + 3
        buf = DevicePrioritizedReplayBuffer(cap, S, A, "cuda")
        buf.max_prio_dev.fill_(1.75)
        obs = env.reset().float().contiguous()
        heads = torch.empty(N, 2 * A, device="cuda")
        act = torch.empty(N, A, device="cuda")
        eps = torch.empty(N, A, device="cuda")
        rec = []
        for t in range(12):
            kw = dict(ring=buf.data, capacity=cap, ring_state=buf.state_dev, priorities=buf.priorities,
                      max_priority=buf.max_prio_dev, action=act, obs32=obs, eps_out=eps)
            if fused:
                env.step_sac_fused(S, A, H, L, kern.ptrs(), actor.log_std_min, actor.log_std_max, actor.max_action,
                                   heads=heads, **kw)
            else:
                kern(obs, heads)
                env.step_sac_ring(heads, actor.log_std_min, actor.log_std_max, actor.max_action, **kw)
            buf.note_appended(N)
            rec.append((heads.clone(), eps.clone(), act.clone(), obs.clone(), buf.state_dev.clone()))
        torch.cuda.synchronize()
        envs.append(env); bufs.append(buf); outs.append(rec)
    for t, (a, b) in enumerate(zip(*outs)):
        for x, y in zip(a, b):
            assert torch.equal(x, y), t
    assert torch.equal(bufs[0].data, bufs[1].data) and torch.equal(bufs[0].priorities, bufs[1].priorities)
    assert torch.equal(envs[0].state, envs[1].state)
    assert int(envs[0].episode_counters()[0].max()) >= 1      # auto-resets happened


@pytest.mark.parametrize("deterministic", [True, False])
def test_sac_collector_graph_equals_eager(pd, deterministic):
    """The HIP-graph collection step stores exactly the transitions of the eager step (twin envs,
    40 steps including auto-resets and miss flushes; the stochastic actor too, its eps being
    drawn in the kernel from the env's counters)."""
    import torch
    from pdenv.sac import Actor, DeviceReplayBuffer, SACCollector
    torch.manual_seed(0)
    N = 1024
    actor = Actor(2, 1).cuda()
    bufs = []
    for g in (False, True):
        env = make(pd, N, mode="rl", auto_reset=True, seed=6, tilt_sigma_rad=0.05)
        buf = DeviceReplayBuffer(64 * N, 2, 1, "cuda")
        col = SACCollector(env, actor, buf, deterministic=deterministic, use_graph=g)
        for _ in range(40):
            col.step()
        torch.cuda.synchronize()
        bufs.append(buf)
    assert len(bufs[0]) == len(bufs[1]) == 40 * N
    assert torch.equal(bufs[0].data, bufs[1].data)


def test_policy_rollout_compaction_invariant(pd):
    """Done-mask compaction: the live-env list is rebuilt inside every launch and, with the list
    in use (pd_tuning.policy_list 1; by default only for grids larger than one chip round), later
    launches are sized to the live count read back every check_every steps, each launch copying
    its envs' actor parameters into list order once (policy_wc).  Fitness, episode lengths and
    final states must be bit-identical with and without the list, with the list switched on
    mid-rollout (policy_list_at), whatever the check interval (0 = never) and the steps per launch,
    and equal to those of envs stepped in their own handle (the order of the list is irrelevant)."""
    import torch
    rng = np.random.default_rng(77)
    W = np.concatenate([rng.uniform(-1.5, 1.5, (700, 372)), rng.uniform(-0.3, 0.3, (324, 372))]).astype(np.float32)
    env = make(pd, len(W), phase="landing_burn", mode="pso")
    res = []
    cases = ((0, 8, 0.0, 64, 0, 0), (1, 0, 0.0, 64, 0, 0), (1, 1, 0.0, 64, 0, 0),
             (1, 3, 0.0, 8, 0, 0), (1, 8, 0.0, 4, 0, 0), (1, 64, 0.0, 64, 0, 0),
             (-1, 8, 0.0, 64, -1, 0), (0, 8, 0.5, 8, 0, 0), (0, 8, 0.05, 2, 0, 0),
             (0, 8, 0.0, 1, 0, 0), (0, 8, 0.0, 64, 1, 256), (0, 8, 0.0, 64, 8, 97),
             (0, 8, 0.0, 64, 32, 0), (0, 8, 0.0, 64, 3, 1), (0, 8, 0.0, 64, 24, 64, 0), (0, 8, 0.0, 64, 24, 64, 100),
             (0, 8, 0.0, 64, 5, 96, 50))
    for c in cases:
        lst, ce, at, pf, rf, sl = c[:6]
        own = c[6] if len(c) > 6 else -1
        # (policy_list_at: switched on mid-rollout at that live fraction; policy_refill with
        # policy_slots env slots (rounded down to whole waves, at least one), each wave's own
        # particles (policy_refill_own percent of the swarm) without atomics, then the shared pool in
        # batches of policy_refill waiting slots of a wave -- 97 slots round to 96 (three waves, less
        # than one workgroup), 32 waits for a whole wave, 1 is one wave; own 0 / 100: pool / own only)
        env.set_tuning(policy_list=lst, policy_list_at=at, policy_fuse=pf, policy_refill=rf, policy_slots=sl,
                       policy_refill_own=own)
        fit, steps = env.rollout_policy(torch.tensor(W), max_steps=300, check_every=ce)
        res.append((fit.cpu().numpy(), steps.cpu().numpy(), env.state.cpu().numpy()))
    for c, (f, s, S) in zip(cases[1:], res[1:]):
        bad = np.flatnonzero((f != res[0][0]) | (s != res[0][1]))
        assert bad.size == 0 and np.array_equal(S, res[0][2]), (c, bad[:8], s[bad[:8]], res[0][1][bad[:8]])
    assert len(set(res[0][1].tolist())) > 5            # ragged episode lengths: compaction exercised
    sub = np.arange(0, len(W), 97)
    env2 = make(pd, len(sub), phase="landing_burn", mode="pso")
    env2.set_tuning(policy_refill=8)   # (11 particles: fewer than a wave's slots, refill cannot run)
    f2, s2 = env2.rollout_policy(torch.tensor(W[sub]), max_steps=300)
    assert np.array_equal(s2.cpu().numpy(), res[0][1][sub])
    np.testing.assert_allclose(f2.cpu().numpy(), res[0][0][sub], rtol=1e-12)


@pytest.mark.parametrize("P", [65536, 262144])
def test_policy_rollout_compaction_invariant_full_swarm(pd, P):
    """Done-mask compaction in the regime it is built for (N x 2 lanes beyond one chip round):
    BASELINE c4's whole 262 144-particle swarm on one device, and a quarter of it, through the
    refill rollout (the default beyond the chip's resident env slots: one launch, the lanes of an
    ended episode take the next particle -- first from their wave's own range, then from the shared
    pool by a wave ballot and prefix count in batches of waiting slots; own share 100 % (default),
    0 and 90 %, batches 24 (the auto batch at two lanes per env), 1, 32), the live list (from
    the first launch; from 50 % live) and neither, at 64 and at 8 policy steps per launch, check
    every 8 steps: fitness, episode lengths and final states bit-identical."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(5)
    W = (torch.rand(P, 372, generator=g, device="cuda") * 3 - 1.5).contiguous()
    env = make(pd, P, phase="landing_burn", mode="pso")
    assert env.tuning()["policy_list"] == -1 and env.tuning()["policy_refill"] == -1
    res = []
    for lst, at, pf, rf, sl, own in ((0, 0.0, 64, 0, 0, -1), (-1, 0.0, 64, -1, 0, -1), (1, 0.0, 8, 0, 0, -1),
                                     (0, 0.5, 8, 0, 0, -1), (0, 0.0, 64, 1, 0, 0), (0, 0.0, 64, 32, 20000, 90)):
        env.set_tuning(policy_list=lst, policy_list_at=at, policy_fuse=pf, policy_refill=rf, policy_slots=sl,
                       policy_refill_own=own)
        fit, steps = env.rollout_policy(W, max_steps=400, check_every=8)
        res.append((fit.clone(), steps.clone(), env.state.clone()))
    for f, s, S in res[1:]:
        assert torch.equal(f, res[0][0]) and torch.equal(s, res[0][1]) and torch.equal(S, res[0][2])
    assert int(res[0][1].max()) > 2 * int(res[0][1].float().mean())     # ragged: the list shrinks


@pytest.mark.parametrize("lpe", [1, 2, 4, 8, 16])
def test_ragged_batch_sizes_bit_identical(pd, lpe):
    """Batch sizes that are not multiples of a wave or a workgroup (1, 3, 63, 65, 257, 1000):
    lanes past the end recompute the last env and write nothing, so env i's trajectory is
    bit-identical whatever N (same lanes per env), including the aero-table misses solved on
    device and the truncation/auto-reset path."""
    import torch
    rng = np.random.default_rng(11)
    T, NMAX = 12, 1000
    A = torch.tensor(rng.uniform(-1, 1, (T, NMAX, 1)).astype(np.float32)).cuda()
    ref = make(pd, NMAX, mode="rl", auto_reset=True, lanes_per_env=lpe)
    R_ = []
    for t in range(T):
        obs, r, dn, tr, ex = ref.step(A[t])
        R_.append(r.clone())
    S_ref, R_ = ref.state, torch.stack(R_)
    for n in (1, 3, 63, 65, 257):
        env = make(pd, n, mode="rl", auto_reset=True, lanes_per_env=lpe)
        rr = []
        for t in range(T):
            obs, r, dn, tr, ex = env.step(A[t, :n].contiguous())
            rr.append(r.clone())
        assert torch.equal(env.state, S_ref[:n]), (n, lpe)
        assert torch.equal(torch.stack(rr), R_[:, :n]), (n, lpe)


def test_n_envs_range_rejected(pd):
    """pd_create validates the batch size: 1 .. 2^25 envs per handle (32-bit per-lane offsets);
    0 or 2^25 + 1 fail loudly with the reason, before any allocation."""
    for n in (0, 2 ** 25 + 1):
        with pytest.raises(pd.PdError, match="n_envs"):
            make(pd, n, mode="rl")


def test_maximum_handle_size(pd):
    """The largest handle, 2^25 envs (16.8 GB of per-env state in binary64 on one MI355X): two
    steps; sampled envs are bit-identical to the same envs in a small handle (same lanes per
    env), and every env's clock advanced by exactly 0.1 s per step."""
    import torch
    N = 2 ** 25
    g = torch.Generator(device="cuda").manual_seed(9)
    A = (torch.rand(2, N, 1, generator=g, device="cuda") * 2 - 1).contiguous()
    big = make(pd, N, mode="rl", lanes_per_env=2)
    for t in range(2):
        big.step_raw(A[t])
    torch.cuda.synchronize()
    idx = torch.tensor([0, 1, 63, 64, 12345, N // 2, N - 65, N - 2, N - 1], device="cuda")
    S = big.state[idx]
    tt = big.state[:, 10]
    assert bool(torch.all(torch.abs(tt - (tt[0])) == 0)), "every env's time must be equal"
    big.close()
    del tt
    small = make(pd, len(idx), mode="rl", lanes_per_env=2)
    for t in range(2):
        small.step(A[t, idx].contiguous())
    assert torch.equal(small.state, S)
    assert abs(float(S[0, 10]) - (float(small.state[0, 10]))) == 0.0


@pytest.mark.parametrize("phase,precision,lpe", [("landing_burn_pure_throttle", "f64", 2),
                                                 ("landing_burn_pure_throttle", "f64", 1),
                                                 ("landing_burn_pure_throttle", "f32", 4),
                                                 ("landing_burn", "f64", 2)])
def test_step_n_fused_equals_step_loop(pd, phase, precision, lpe):
    """pd_step_n runs up to 16 env-steps per launch (state through memory between the fused
    steps, miss flush after each launch).  Every per-step output row and the final state must
    equal T separate pd_step calls bit for bit: wind + tilt + auto-reset + device-solved
    misses (tables cut to 4 entries) + a ragged batch, T not a multiple of the chunk."""
    import torch
    N, T = 1000, 37
    A_dim = 1 if phase == "landing_burn_pure_throttle" else 4
    g = torch.Generator(device="cuda").manual_seed(5)
    A = (torch.rand(T, N, A_dim, device="cuda", generator=g) * 2 - 1).contiguous()
    kw = dict(precision=precision, lanes_per_env=lpe, enable_wind=True, stochastic_wind=True,
              wind_percentile=None, auto_reset=True, tilt_sigma_rad=0.02, seed=21,
              params=pd.Params().restrict_keys(4, 4))
    loop = make(pd, N, phase=phase, **kw)
    fused = make(pd, N, phase=phase, **kw)
    rows = [loop.step(A[t]) for t in range(T)]
    obs, rew, dn, tr, tid = fused.step_n(A)
    for t, (o, r, d, tt, ex) in enumerate(rows):
        assert torch.equal(o, obs[t]) and torch.equal(r, rew[t]), t
        assert torch.equal(d, dn[t]) and torch.equal(tt, tr[t]) and torch.equal(ex["trunc_id"], tid[t]), t
    assert torch.equal(loop.state, fused.state)
    # the reward-only fused rollout matches the per-step rewards' sum
    r2 = make(pd, N, phase=phase, **kw).rollout(A)
    torch.testing.assert_close(r2, rew.sum(0), rtol=1e-12 if precision == "f64" else 1e-5, atol=1e-9)


def test_launcher_refuses_mismatched_inputs(pd):
    """Every launch checks its inputs before any kernel runs (the round-4 fault class: a launch
    reaching the plain step kernel with a NULL action pointer): a step without actions, a SAC
    step without heads, a SAC launch on a handle with no SAC kernel, a fused SAC step whose actor
    widths differ from the handle's or whose parameters are misaligned, out-of-range tuning.
    Each is refused with its status and the handle steps on unharmed."""
    import ctypes as C
    import torch
    from pdenv.env import _ptr
    env = make(pd, 256, lanes_per_env=16)
    lib, h = env.lib, env.h
    vp = C.c_void_p
    assert lib.pd_step(h, None, None, None, None, None, None, None, None, None) == L.PD_ERR_INVALID
    assert lib.pd_step_n(h, None, 4, None, None, None, None, None, None) == L.PD_ERR_INVALID
    assert lib.pd_step_sac(h, None, None, 0, None, -20.0, 2.0, 1.0, None, None, None, None) == L.PD_ERR_INVALID
    assert lib.pd_step_sac_ring(h, None, 0, -20.0, 2.0, 1.0, None, None, None, 0, None, None, None, None,
                                None) == L.PD_ERR_INVALID
    pso = make(pd, 256, mode="pso")
    heads = torch.zeros(256, 2, device="cuda")
    assert pso.lib.pd_step_sac_ring(pso.h, _ptr(heads), 1, -20.0, 2.0, 1.0, None, None, None, 0, None, None, None,
                                    None, None) == L.PD_ERR_UNSUPPORTED
    # a 2-256-256-1 actor: the right widths step, wrong ones and a misaligned parameter do not
    H, S, A = 256, env.obs_dim, env.action_dim
    ts = [torch.zeros(H, S), torch.zeros(H), torch.zeros(H, H), torch.zeros(H), torch.zeros(A, H), torch.zeros(A),
          torch.zeros(A, H), torch.zeros(A)]
    ts = [t.cuda() for t in ts]
    params = (vp * 8)(*[t.data_ptr() for t in ts])
    obs32 = torch.zeros(256, S, device="cuda")
    act = torch.zeros(256, A, device="cuda")

    def fused(s, a, p):
        return lib.pd_step_sac_fused(h, s, a, H, 2, p, None, 1, -20.0, 2.0, 1.0, None, _ptr(act), None, 0, None, None,
                                     None, _ptr(obs32), None)
    assert fused(S + 1, A, params) == L.PD_ERR_INVALID
    assert fused(S, A + 1, params) == L.PD_ERR_INVALID
    bad = torch.zeros(A * H + 1, device="cuda")
    params2 = (vp * 8)(*([t.data_ptr() for t in ts[:6]] + [bad.data_ptr() + 4, ts[7].data_ptr()]))
    assert fused(S, A, params2) == L.PD_ERR_UNSUPPORTED
    L.check(fused(S, A, params))
    for kw in (dict(step_fuse=0), dict(step_fuse=257), dict(policy_fuse=3), dict(policy_lanes=16), dict(policy_list=2),
               dict(policy_list_at=1.5), dict(policy_refill=65), dict(policy_refill_own=101)):
        with pytest.raises(L.PdError):
            env.set_tuning(**kw)
    assert env.tuning() == dict(step_fuse=128, policy_fuse=64, policy_lanes=2, policy_list=-1, policy_list_at=0.0,
                                policy_refill=-1, policy_slots=0, policy_refill_own=-1, pad_tuning=0)
    env.step(torch.zeros(256, 1, device="cuda"))
    torch.cuda.synchronize()
    assert torch.isfinite(env.state).all()


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_step_n_info_tap_matches_step(pd, precision):
    """The info tap in fused launches (pd_step_n_info, a key mask): 40 steps of 512 envs with wind,
    gusts, tilt and auto-reset through two fused launches (step_fuse 24) with a subset of the keys
    equal, bit for bit, to the same keys of 40 pd_step calls with the full tap; the states too."""
    import torch
    N, T = 512, 40
    g = torch.Generator(device="cuda").manual_seed(41)
    A = torch.rand(T, N, 1, device="cuda", generator=g) * 2 - 1
    A[:, : N // 2] = A[:, : N // 2] * 0.25 + 0.75
    kw = dict(precision=precision, lanes_per_env=2, enable_wind=True, stochastic_wind=True, wind_percentile=None,
              auto_reset=True, tilt_sigma_rad=0.02, seed=17)
    keys = ["air_density", "mach_number", "CL", "CD", "alpha_effective", "g_load_1_sec_window", "ug", "vg",
            "theta_dot_dot", "gf_Mz", "theta_in"]
    one, fused = make(pd, N, **kw), make(pd, N, **kw)
    fused.set_tuning(step_fuse=24)
    ref = {k: [] for k in keys}
    for t in range(T):
        *_, ex = one.step(A[t], info=True)
        for k in keys:
            ref[k].append(ex[k].clone())
    obs, rew, dn, tr, tid, tap = fused.step_n(A, info_keys=keys)
    assert set(tap) == set(keys)
    for k in keys:
        assert torch.equal(tap[k], torch.stack(ref[k])), k
    assert torch.equal(one.state, fused.state)
    #  a repeated or unknown key is refused before any launch: a repeated key's bit
    # would carry into the next field's and the tap would return unwritten rows
    for bad in (["mach_number", "mach_number"], ["no_such_key"]):
        with pytest.raises(ValueError):
            fused.step_n(A[:2], info_keys=bad)
