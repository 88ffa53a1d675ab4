"""The N > 1 path on CPU: world_size-2 `gloo` process groups (no GPU).

bench.py shards the env batch contiguously (`shard_offset`), steps each shard with no data-path
collective, brackets the timed region with barriers and reports the max over ranks
(`timed_region`, `whole_job_rate`).  These tests run those helpers on two gloo ranks, and
check with the CPU oracle that sharding does not change any env's result: the per-rank shards,
all-gathered (the transition gather of SURVEY config c5), equal the single-process batch.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _timing_worker(rank, world, port, out):
    import time
    import bench
    _init(rank, world, port)
    wall = bench.timed_region(lambda k: time.sleep(0.004 * (rank + 1)), 5, lambda: None, dist, "cpu")
    out[rank] = wall
    dist.destroy_process_group()


def test_timed_region_reports_max_over_ranks():
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_timing_worker, args=(world, port, out), nprocs=world, join=True)
        walls = [out[r] for r in range(world)]
    import bench
    assert walls[0] == walls[1]                 # every rank reports the same (max) time
    assert walls[0] >= 5 * 0.008                # at least the slow rank's own work
    assert bench.whole_job_rate(100, world, 5, walls[0]) == pytest.approx(1000 / walls[0])
    assert [bench.shard_offset(r, 100) for r in range(world)] == [0, 100]


def _episode(global_env, n_steps):
    """The oracle run of one env whose actions depend only on its GLOBAL index."""
    import oracle
    rng = np.random.default_rng(1000 + global_env)
    acts = rng.uniform(-1, 1, (n_steps, 1)).astype(np.float32)
    o = oracle.Oracle(phase=0, rtd=0)
    rew = 0.0
    for t in range(n_steps):
        s, r, d, tr, tid, ob, info = o.step(acts[t], f32=True)
        rew += r
        if d or tr:
            break
    return np.concatenate([o.state, [rew]])


def _shard_worker(rank, world, port, n_per_rank, n_steps, out):
    import bench
    _init(rank, world, port)
    off = bench.shard_offset(rank, n_per_rank)
    mine = torch.tensor(np.stack([_episode(off + i, n_steps) for i in range(n_per_rank)]))
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    if rank == 0:
        out["all"] = torch.cat(gathered).numpy()
    dist.destroy_process_group()


def test_sharded_envs_equal_single_batch(oracle_mod):
    world, n_per_rank, n_steps = 2, 3, 25
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_shard_worker, args=(world, port, n_per_rank, n_steps, out), nprocs=world, join=True)
        got = out["all"]
    ref = np.stack([_episode(g, n_steps) for g in range(world * n_per_rank)])
    assert np.array_equal(got, ref)


def _sac_gather_worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
    from pdenv.sac import DeviceReplayBuffer, gather_slabs, transition_slab
    _init(rank, world, port)
    n = 5
    obs = torch.full((n, 2), float(rank)) + torch.arange(n)[:, None] * 0.1
    act = torch.full((n, 1), -float(rank))
    rew = torch.arange(n, dtype=torch.float64) + 100 * rank
    nxt = obs + 1
    done = torch.tensor([0, 1, 0, 0, 1], dtype=torch.uint8)
    buf = DeviceReplayBuffer(12, 2, 1, "cpu")
    for k in range(3):                              # 3 steps x 2 ranks x 5 = 30 > capacity 12
        full = gather_slabs(transition_slab(obs + k, act, rew, nxt + k, done), dist)
        if rank == 0:
            buf.add_batch(full)
    if rank == 0:
        out["data"] = buf.data.clone().numpy()
        out["pos"], out["size"] = buf.position, buf.size
        out["sample"] = [t.shape for t in buf.sample(7, generator=torch.Generator().manual_seed(0))]
    dist.destroy_process_group()


def test_sac_transition_gather_into_replay_buffer():
    """c5 data path on two gloo ranks: per-rank transition slabs all-gathered in rank order and
    appended to the learner rank's ring buffer (oldest entries overwritten)."""
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_sac_gather_worker, args=(world, port, out), nprocs=world, join=True)
        data, pos, size, shapes = out["data"], out["pos"], out["size"], out["sample"]
    # expected stream: for k in 0..2, rank 0 rows then rank 1 rows
    rows = []
    for k in range(3):
        for r in range(2):
            for i in range(5):
                s = np.array([r + 0.1 * i + k, r + 0.1 * i + k], dtype=np.float32)
                rows.append(np.concatenate([s, [-r], [i + 100 * r], s + 1, [[0, 1, 0, 0, 1][i]]]).astype(np.float32))
    rows = np.array(rows)
    assert size == 12 and pos == 30 % 12
    ring = np.roll(rows[-12:], 30 % 12, axis=0)     # row t lands at t % 12
    assert np.array_equal(data, ring)
    assert [tuple(s) for s in shapes] == [(7, 2), (7, 1), (7, 1), (7, 2), (7, 1)]


def test_prioritized_buffer_sampling_distribution():
    """Device PER (Gumbel-top-k) draws pairs with the probabilities of
    np.random.choice(size, 2, replace=False, p) and reproduces the reference's weights and
    priority bookkeeping (sac_pytorch.py:77-124)."""
    import itertools
    sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
    from pdenv.sac import DevicePrioritizedReplayBuffer
    buf = DevicePrioritizedReplayBuffer(8, 1, 1, "cpu", alpha=0.6, beta=0.4, beta_annealing_steps=10)
    buf.add_batch(torch.arange(5 * 5, dtype=torch.float32).reshape(5, 5))
    assert torch.equal(buf.priorities[:5], torch.ones(5))
    buf.update_priorities(torch.arange(5), torch.tensor([0.5, 1.0, 2.0, 4.0, 8.0]))
    assert buf.max_priority == pytest.approx(8.0 + 1e-6)
    p = (np.array([0.5, 1.0, 2.0, 4.0, 8.0]) + 1e-6) ** 0.6
    p /= p.sum()
    exact = {}
    for i, j in itertools.permutations(range(5), 2):
        exact[(i, j)] = p[i] * p[j] / (1 - p[i])
    g = torch.Generator().manual_seed(0)
    counts = {k: 0 for k in exact}
    T = 40000
    beta0 = buf.beta
    for _ in range(T):
        s, a, r, s2, d, w, idx = buf.sample(2, generator=g)
        counts[tuple(int(v) for v in idx)] += 1
    assert buf.beta == pytest.approx(min(1.0, beta0 + T * (1 - 0.4) / 10))
    for k, e in exact.items():
        assert abs(counts[k] / T - e) < 5 * np.sqrt(e * (1 - e) / T) + 1e-3, (k, counts[k] / T, e)
    # weights of the last draw: (size * p)^-beta / max, beta as it was before the last anneal
    wr = (5 * p[idx.numpy()]) ** (-1.0)
    assert np.allclose(w.numpy().ravel(), wr / wr.max(), rtol=1e-6)


def _pso_uneven_worker(rank, world, port, out):
    """After re_initialise_swarms the ranks hold different numbers of particles (rank 1 none):
    the variable-size gathers and the migration decisions must still agree on every rank."""
    import random
    sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
    from pdenv.pso import all_gather_var, local_moves, migration_moves, reinit_keep
    _init(rank, world, port)
    # global population of 12 in 2 subswarms; rank 0 holds 0..5, rank 1 holds 6..11
    g = torch.Generator().manual_seed(4)
    pbf_all = torch.rand(12, generator=g, dtype=torch.float64)
    sw_all = torch.tensor([0] * 6 + [1] * 6, dtype=torch.int32)
    mine = slice(0, 6) if rank == 0 else slice(6, 12)
    keep = reinit_keep(all_gather_var(pbf_all[mine].contiguous(), dist),
                       all_gather_var(sw_all[mine].contiguous(), dist), 2, 3)
    assert torch.equal(keep, reinit_keep(pbf_all, sw_all, 2, 3))
    # uneven shards: rank 0 keeps 5 particles of both subswarms, rank 1 none (an empty shard)
    local = torch.tensor([0, 1, 0, 1, 1], dtype=torch.int32) if rank == 0 else torch.empty(0, dtype=torch.int32)
    sw = all_gather_var(local, dist)
    moves = migration_moves(sw, 2, 1, random.Random(9))
    # each rank applies the moves that hit its own particles, a later move of a particle winning
    offset, n = (0, 5) if rank == 0 else (5, 0)
    applied = sw.clone()
    for g, t in moves:
        applied[g] = t
    mine = local_moves(moves, offset, n)
    assert all(applied[offset + i] == t for i, t in mine.items())
    assert set(mine) == {g - offset for g, _ in moves if offset <= g < offset + n}
    out[rank] = (sw.tolist(), moves)
    dist.destroy_process_group()


def test_pso_uneven_shards_gather_and_migrate():
    """after re-initialisation shards differ in size; migrate_particles and a second
    re-initialisation gather with all_gather_var (sizes first, padded, trimmed) on two gloo ranks."""
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_pso_uneven_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == out[1]
    assert out[0][0] == [0, 1, 0, 1, 1]
    assert len(out[0][1]) == 2


def test_pso_local_moves_later_move_wins():
    """migrate_particles applies the moves that hit this rank's shard in one indexed write: a
    particle the decisions move twice ends in its last subswarm (the reference edits its member
    lists in order), and moves of other ranks' particles are left to them."""
    sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
    from pdenv.pso import local_moves
    moves = [(3, 1), (7, 0), (3, 2), (12, 1), (5, 0)]
    assert local_moves(moves, 2, 5) == {1: 2, 3: 0}          # particles 2..6: 3 -> 1 -> 2, 5 -> 0
    assert local_moves(moves, 7, 6) == {0: 0, 5: 1}          # particles 7..12
    assert local_moves(moves, 20, 0) == {}
