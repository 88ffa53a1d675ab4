"""Teacher-forced ("shadowing") parity of a free-running GPU env against the oracle.

The powered-descent env is chaotic: in the oracle itself (and so in the reference, which it
restates), a 1-ulp change of the initial pitch changes a random-action episode's per-step reward
by up to 4e-3 before it ends (tests/test_oracle_golden.py::test_oracle_episode_chaos_bound).  A
GPU trajectory and an oracle trajectory started from the same state therefore part after a few
dozen steps through last-ulp differences of the transcendental functions alone, and comparing
them far into an episode tests nothing.  Instead, at EVERY step of the GPU run, the complete
per-env state of sampled envs is read back (state, g-load window, actuators, wind filters,
sigmas, percentile, episode/step counters -- the checkpoint getters), the oracle takes that
state through one env step with the same action and the same Philox draws, and its result must
equal the GPU's next state and outputs at the per-step tolerances; every auto-reset must equal
the oracle's reset (orc_reset_philox) bit for bit.  This covers the whole trajectory of every
sampled env: resets, percentiles, gust draws, truncations.
"""
import ctypes as C

import numpy as np
import torch

ST = ["x", "y", "vx", "vy", "theta", "theta_dot", "gamma", "alpha", "mass", "mass_propellant", "time"]
# per env-step, f64 handle: relative to max(|oracle|, 1e-3); theta_dot is a small difference
# of large moments
TOL_STEP = np.array([1e-10] * 5 + [1e-8] + [1e-10] * 5)


def snapshot(env, it):
    """The sampled envs' complete per-env state (host numpy)."""
    vp, ring, ln, hd = env.gload_window()
    f, sg, pr = env.wind_state()
    ep, ts, tid = env.episode_counters()
    out = dict(s=env.state[it], vprev=vp[it], ring=ring[it], len=ln[it], head=hd[it], filt=f[it], sig=sg[it],
               prof=pr[it] - 50, ep=ep[it], ts=ts[it], tid=tid[it])
    if env.action_dim == 4:
        out["act"] = env.actuators[it]
    return {k: v.cpu().numpy() for k, v in out.items()}


def _load(L, P, E, snap, j, phase, seed, g, fixed_prof, tilt):
    """OrcEnv E := sampled env j of the snapshot (orc_reset_philox sets the draw scheme)."""
    L.orc_reset_philox(C.byref(P), C.byref(E), phase, seed, int(g), int(snap["ep"][j]) & 0xFFFFFFFF, 1, 1,
                       fixed_prof, tilt)
    for k in range(11):
        E.s[k] = float(snap["s"][j, k])
        E.prev_s[k] = 0.0
    E.prev_s[2] = float(snap["vprev"][j])        # |v_prev| = sqrt(fl(vprev^2)) exactly
    n, h = int(snap["len"][j]), int(snap["head"][j])
    for k in range(10):
        E.gwin[k] = float(snap["ring"][j, k if n < 10 else (h + k) % 10])
    E.gwin_len = n
    E.trunc_id = int(snap["tid"][j])
    if "act" in snap:
        E.gimbal_prev, E.dl_prev, E.dr_prev = (float(v) for v in snap["act"][j])
    E.sigma_u, E.sigma_v = (float(v) for v in snap["sig"][j])
    E.fu[0], E.fu[1], E.fv[0], E.fv[1] = (float(v) for v in snap["filt"][j])
    E.wind_prof = int(snap["prof"][j])
    E.rng_ts = int(snap["ts"][j]) & 0xFFFFFFFF


def shadow_run(oracle_mod, env, actions, idx, phase, rtd, seed, tilt, fixed_prof=-1, y_gust=15000.0):
    """Step `env` through actions [T, N, A] (device tensor) one pd_step at a time; teacher-force
    the oracle on envs `idx` at every step.  Returns coverage statistics and the per-step
    outputs of the whole batch (for the fused-launch identity check)."""
    L = oracle_mod.lib()
    P = oracle_mod.params()
    it = torch.as_tensor(idx, device=env.device)
    T = actions.shape[0]
    o = oracle_mod.OrcOut()
    E, E2 = oracle_mod.OrcEnv(), oracle_mod.OrcEnv()
    nobs = env.obs_dim
    stats = dict(steps=0, resets=0, gust_steps=0, profiles=set(), max_err=np.zeros(11), max_rew=0.0, max_obs=0.0,
                 max_filt=0.0, trunc_ids=set())
    outs = dict(obs=[], rew=[], done=[], trunc=[], tid=[])
    snap = snapshot(env, it)
    for t in range(T):
        obs, rew, dn, tr, ex = env.step(actions[t])
        for k, v in zip(("obs", "rew", "done", "trunc", "tid"), (obs, rew, dn, tr, ex["trunc_id"])):
            outs[k].append(v)
        after = snapshot(env, it)
        g_obs, g_rew = obs[it].cpu().numpy(), rew[it].cpu().numpy()
        g_dn, g_tr, g_tid = dn[it].cpu().numpy(), tr[it].cpu().numpy(), ex["trunc_id"][it].cpu().numpy()
        a = actions[t][it].cpu().numpy().astype(np.float64)
        for j, g in enumerate(idx):
            _load(L, P, E, snap, j, phase, seed, g, fixed_prof, tilt)
            stats["profiles"].add(int(snap["prof"][j]))
            if E.s[1] < y_gust:
                stats["gust_steps"] += 1
            u = (C.c_double * 4)(*(list(a[j]) + [0.0] * (4 - a.shape[1])))
            L.orc_step(C.byref(P), C.byref(E), phase, rtd, u, 1, None, C.byref(o))
            ctx = f"step {t} env {g}"
            assert bool(g_dn[j]) == bool(o.done) and bool(g_tr[j]) == bool(o.trunc), ctx
            assert int(g_tid[j]) == o.trunc_id, ctx
            stats["max_rew"] = max(stats["max_rew"], abs(float(g_rew[j]) - o.reward))
            ob = np.array(o.obs[:nobs])
            stats["max_obs"] = max(stats["max_obs"], float(np.abs(g_obs[j] - ob).max()))
            stats["steps"] += 1
            if o.done or o.trunc:
                # auto-reset into the next episode: the oracle's reset, bit for bit
                stats["resets"] += 1
                stats["trunc_ids"].add(o.trunc_id)
                _ = L.orc_reset_philox(C.byref(P), C.byref(E2), phase, seed, int(g), (int(snap["ep"][j]) + 1) & 0xFFFFFFFF,
                                       1, 1, fixed_prof, tilt)
                assert np.array_equal(after["s"][j], np.array(E2.s[:])), ctx
                assert after["sig"][j][0] == E2.sigma_u and after["sig"][j][1] == E2.sigma_v, ctx
                assert int(after["prof"][j]) == E2.wind_prof, ctx
                assert int(after["ep"][j]) == int(snap["ep"][j]) + 1 and int(after["ts"][j]) == 0, ctx
                assert (after["filt"][j] == 0).all() and int(after["len"][j]) == 0, ctx
            else:
                so = np.array(E.s[:])
                err = np.abs(after["s"][j] - so) / np.maximum(np.abs(so), 1e-3)
                stats["max_err"] = np.maximum(stats["max_err"], err)
                fo = np.array([E.fu[0], E.fu[1], E.fv[0], E.fv[1]])
                stats["max_filt"] = max(stats["max_filt"], float(np.abs(after["filt"][j] - fo).max()))
                assert int(after["ts"][j]) == int(snap["ts"][j]) + 1, ctx
        snap = after
    stats["outs"] = {k: torch.stack(v) for k, v in outs.items()}
    return stats


def check_stats(stats, tol_rew=1e-9, tol_obs=1e-6, tol_filt=1e-12):
    bad = {ST[k]: float(stats["max_err"][k]) for k in range(11) if stats["max_err"][k] > TOL_STEP[k]}
    assert not bad, bad
    assert stats["max_rew"] <= tol_rew, stats["max_rew"]
    assert stats["max_obs"] <= tol_obs, stats["max_obs"]
    assert stats["max_filt"] <= tol_filt, stats["max_filt"]


def policy_snapshots(env, W, K):
    """pd_rollout_policy with max_steps = k for k = 0..K (the rollout is deterministic: the state
    after k policy steps of a longer rollout): per k the handle's complete per-env state, the
    fitness (-sum of rewards) and the episode lengths, host numpy, all particles."""
    import torch
    out = []
    Wt = torch.as_tensor(W, device=env.device)
    for k in range(K + 1):
        fit, steps = env.rollout_policy(Wt, max_steps=k)
        vp, ring, ln, hd = env.gload_window()
        _, _, tid = env.episode_counters()
        out.append({"s": env.state.cpu().numpy(), "act": env.actuators.cpu().numpy(), "vprev": vp.cpu().numpy(),
                     "ring": ring.cpu().numpy(), "len": ln.cpu().numpy(), "head": hd.cpu().numpy(),
                     "tid": tid.cpu().numpy(), "fit": fit.cpu().numpy(), "steps": steps.cpu().numpy()})
    return out


def shadow_policy(oracle_mod, snaps, W, idx, phase):
    """Teacher-forced parity of a policy rollout (fused actor + env step + PSO reward, no wind)
    on particles `idx`: for every policy step k -> k + 1 a particle takes, the oracle loads the
    device's complete state after k steps, runs its actor (orc_actor: the same binary32 order)
    and one env step (orc_step, rtd_pso), and must equal the device after k + 1 steps: state per
    TOL_STEP, reward (fitness difference) <= 1e-9 + 1e-12 |fitness|, done/truncated (an ended
    episode is frozen: its length stops growing) and the truncation id exactly."""
    L = oracle_mod.lib()
    P = oracle_mod.params()
    o = oracle_mod.OrcOut()
    E = oracle_mod.OrcEnv()
    stats = dict(steps=0, ended=0, max_err=np.zeros(11), max_rew=0.0, trunc_ids=set())
    K = len(snaps) - 1
    for j in idx:
        for k in range(K - 1):
            a, b, c = snaps[k], snaps[k + 1], snaps[k + 2]
            if int(b["steps"][j]) != k + 1:      # the episode ended before this step
                break
            L.orc_reset(C.byref(P), C.byref(E), None, 0, 0, C.c_double(1.0), C.c_double(1.0))
            for q in range(11):
                E.s[q] = float(a["s"][j, q])
                E.prev_s[q] = 0.0
            E.prev_s[2] = float(a["vprev"][j])           # |v_prev| = sqrt(fl(vprev^2)) exactly
            n, h = int(a["len"][j]), int(a["head"][j])
            for q in range(10):
                E.gwin[q] = float(a["ring"][j, q if n < 10 else (h + q) % 10])
            E.gwin_len = n
            E.trunc_id = int(a["tid"][j])
            E.gimbal_prev, E.dl_prev, E.dr_prev = (float(v) for v in a["act"][j])
            u = oracle_mod.actor(phase, W[j], a["s"][j]).astype(np.float64)
            ua = (C.c_double * 4)(*(list(u) + [0.0] * (4 - len(u))))
            L.orc_step(C.byref(P), C.byref(E), phase, 1, ua, 1, None, C.byref(o))
            ctx = f"particle {j} step {k}"
            so = np.array(E.s[:])
            err = np.abs(b["s"][j] - so) / np.maximum(np.abs(so), 1e-3)
            stats["max_err"] = np.maximum(stats["max_err"], err)
            rew = float(a["fit"][j]) - float(b["fit"][j])
            stats["max_rew"] = max(stats["max_rew"], abs(rew - o.reward))
            assert abs(rew - o.reward) <= 1e-9 + 1e-12 * abs(float(b["fit"][j])), (ctx, rew, o.reward)
            ended = bool(o.done or o.trunc)
            assert (int(c["steps"][j]) == k + 1) == ended, (ctx, int(c["steps"][j]), ended)
            assert int(b["tid"][j]) == o.trunc_id, ctx
            stats["steps"] += 1
            if ended:
                stats["ended"] += 1
                stats["trunc_ids"].add(o.trunc_id)
                break
    return stats
