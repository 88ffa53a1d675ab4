"""CPU checks of the PSO driver's host-side decisions (pdenv/pso.py)."""
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))


def _moves_lists(swarm, n_swarms, n_migrants, rng):
    """particle_swarm_optimisation.py:545-553 with Python lists, as the reference keeps them."""
    members = [list(np.flatnonzero(np.asarray(swarm) == s)) for s in range(n_swarms)]
    moves = []
    for i in range(n_swarms):
        if len(members[i]) > 1:
            for _ in range(n_migrants):
                k = rng.randrange(len(members[i]))
                g = members[i].pop(k)
                t = rng.choice([j for j in range(n_swarms) if j != i])
                members[t].append(g)
                moves.append((int(g), t))
    return moves


def test_migration_moves_equal_list_restatement():
    """The NumPy member arrays take the same decisions as the reference's lists (pop/append
    order, rng stream) for random memberships, subswarm counts and migrant numbers, including
    subswarms with one member or none (and, like the reference, fail when a subswarm's own
    migrants empty it: the len > 1 check precedes the migrant loop)."""
    from pdenv.pso import migration_moves
    for seed in range(200):
        r = np.random.default_rng(seed)
        S = int(r.integers(2, 6))
        n = int(r.integers(0, 40))
        sw = torch.tensor(r.integers(0, S, n), dtype=torch.int32)
        k = int(r.integers(1, 4))
        out = []
        for f, arg in ((migration_moves, sw), (_moves_lists, sw.numpy())):
            try:
                out.append(f(arg, S, k, random.Random(seed)))
            except ValueError as e:    # a subswarm emptied by its own migrants: both raise
                out.append(type(e))
        assert out[0] == out[1], seed


def test_chunk4_layout_and_inverse():
    """chunk4: chunk c of column i holds parameters 4c .. 4c+3 (zeros past D), the layout
    pd_rollout_policy_chunked reads; unchunk4 inverts it; concatenating chunked batches along
    the particle axis equals chunking the concatenation (the merged share rollout relies on it)."""
    from pdenv.pso import chunk4, unchunk4
    g = torch.Generator().manual_seed(0)
    for D, n in ((372, 33), (249, 5), (10, 7), (4, 1)):
        w = torch.rand(D, n, generator=g)
        w4 = chunk4(w)
        C = (D + 3) // 4
        assert w4.shape == (C, n, 4) and w4.is_contiguous()
        for c in range(C):
            for k in range(4):
                d = 4 * c + k
                exp = w[d] if d < D else torch.zeros(n)
                assert torch.equal(w4[c, :, k], exp)
        assert torch.equal(unchunk4(w4, D), w)
        v = torch.rand(D, 3, generator=g)
        assert torch.equal(torch.cat([w4, chunk4(v)], dim=1), chunk4(torch.cat([w, v], dim=1)))


def test_share_decisions_on_device_equal_the_list_restatement():
    """share_information's device path (_share_on_device, CPU tensors here) takes the reference's
    decisions (particle_swarm_optimisation.py:521-543 as the host path states them): best = the
    first minimum of the subswarm bests, one uniform per subswarm but the best, in order, moved
    when below 1/2, moved positions 30 % toward the best's; the candidates are the moved subswarms
    ascending, padded with the first; and the strictly-better replacement leaves nothing changed
    when nothing moved (ties, +inf bests and S = 2..6 included)."""
    from pdenv.pso import ParticleSubswarmOptimisationGPU, chunk4
    rng = np.random.default_rng(3)
    opt = object.__new__(ParticleSubswarmOptimisationGPU)
    for trial in range(300):
        S = int(rng.integers(2, 7))
        D = int(rng.choice([5, 8, 372]))
        opt.S, opt.device = S, torch.device("cpu")
        opt._cols = torch.arange(S)
        sbf = rng.choice([1.0, 2.0, 3.0, np.inf], S) if trial % 3 == 0 else rng.uniform(0, 10, S)
        sb = rng.uniform(-1.5, 1.5, (S, D))
        u = rng.uniform(0, 1, S - 1)
        # the host path's list restatement, drawing the same uniforms in order
        draws = iter(u.tolist())
        best = int(np.argmin(sbf))
        moved = [i for i in range(S) if i != best and next(draws) < 0.5]
        sb_ref = sb.copy()
        for i in moved:
            sb_ref[i] = (1 - 0.3) * sb_ref[i] + 0.3 * sb_ref[best]
        sb_t, sbf_t = torch.tensor(sb), torch.tensor(sbf)
        pad, count, cand = opt._share_on_device(sb_t, sbf_t, torch.tensor(u))
        assert int(count) == len(moved)
        assert np.array_equal(sb_t.numpy(), sb_ref)
        if moved:
            want = moved + [moved[0]] * (S - 1 - len(moved))
            assert pad.tolist() == want
            assert torch.equal(cand, chunk4(torch.tensor(sb_ref[want]).t().float()))
        fit = torch.tensor(rng.uniform(0, 10, S - 1))
        if moved:                               # the padded entries repeat the first candidate
            fit[len(moved):] = fit[0]
        sbf_ref = sbf.copy()
        for k, i in enumerate(moved):
            if fit[k] < sbf_ref[i]:
                sbf_ref[i] = float(fit[k])
        opt._flush_on_device(sbf_t, pad, count, fit)
        assert np.array_equal(sbf_t.numpy(), sbf_ref)
