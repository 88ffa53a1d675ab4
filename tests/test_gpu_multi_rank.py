"""The N > 1 product path on the GPU: the c4 and c5 drivers on two ranks sharing cuda:0.

SURVEY configs c4 (PSO, 262 144 particles over 8 GPUs) and c5 (SAC collection, 32 768 envs over
8 GPUs) shard their units over ranks and exchange data only at the drivers' collectives:
- c4: the per-subswarm minima every generation, the membership / personal bests at
  re_initialise_swarms (particle_swarm_optimisation.py:413-552);
- c5: the transition rows, all-gathered in rank order onto the learner rank's replay buffer
  (sac_pytorch_powered_descent.py:160-183).
Here both run on two `gloo` ranks that share cuda:0 and must reproduce the world-1 run bit for
bit: the global best and every subswarm best, the membership, the positions and personal bests,
the share-candidate fitness, and every replay-buffer row and priority.

RCCL refuses two ranks on one device, and gloo has no all_gather of device tensors, so
`HostStagedGroup` (test-only) stages those collectives through host tensors; the drivers call it
exactly as they call torch.distributed.  The RCCL path itself runs in bench.py under
PD_BENCH_DIST=1 (profiles/r06_rccl_1rank.jsonl).
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "psso-sac-for-powered-descent_amd")

# c4: 2 048 particles (2 subswarms), 16 generations: migrations at 5, 10 and 15, a share at 10,
# the re-initialisation at 12 keeps 300 per subswarm -- the ranks then hold different numbers of
# particles (possibly fewer than a refill wave's slots), and generation 15 migrates across them
PSO_POP, PSO_GENS = 2048, 16
PSO_KW = dict(generations=400, re_initialise_generation=12, re_initialise_number_of_particles=600)
# c5: 1 024 envs per rank (2 048 at world 1: both at 16 lanes per env, the fused actor kernel);
# the ring (15 336 rows) wraps every 7.5 steps; 256 steps: the random-init actor's episodes end
# (truncated or done) and auto-reset inside the window
SAC_ENVS, SAC_STEPS, SAC_CAP = 1024, 256, 7 * 2048 + 1000


class HostStagedGroup:
    """The torch.distributed calls the drivers make (is_initialized, get_rank, get_world_size,
    all_gather, all_gather_into_tensor, barrier) on a gloo group, device tensors staged through
    host memory.  Test infrastructure only."""

    def __init__(self, dist):
        self.d = dist

    def is_initialized(self):
        return True

    def get_rank(self):
        return self.d.get_rank()

    def get_world_size(self):
        return self.d.get_world_size()

    def barrier(self):
        self.d.barrier()

    def all_gather(self, outs, t):
        host = [o.new_empty(o.shape, device="cpu") for o in outs]
        self.d.all_gather(host, t.detach().cpu().contiguous())
        for o, h in zip(outs, host):
            o.copy_(h)

    def all_gather_into_tensor(self, out, t):
        host = [t.new_empty(t.shape, device="cpu") for _ in range(self.get_world_size())]
        self.d.all_gather(host, t.detach().cpu().contiguous())
        out.copy_(torch_cat(host))


def torch_cat(xs):
    import torch
    return torch.cat(xs)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_pso(dist):
    """The c4 driver's generations; returns the GLOBAL swarm (rank order) and the bests."""
    import torch
    from pdenv.pso import ParticleSubswarmOptimisationGPU, all_gather_var
    opt = ParticleSubswarmOptimisationGPU("landing_burn", pop_size=PSO_POP, seed=7, dist=dist, pso_params=PSO_KW)
    sizes = []
    for g in range(PSO_GENS):
        opt.generation(g)
        sizes.append(opt.P)
    opt.flush_share()
    torch.cuda.synchronize()
    D = opt.D
    x = all_gather_var(opt.x.t().contiguous().reshape(-1), opt.dist).reshape(-1, D)
    pb = all_gather_var(opt.pb.t().contiguous().reshape(-1), opt.dist).reshape(-1, D)
    out = {
        "gbf": float(opt.gbf_t), "gb": opt.gb_t.cpu().numpy(), "sbf": opt.sbf_t.cpu().numpy(),
        "sb": opt.sb.cpu().numpy(), "x": x.cpu().numpy(), "pb": pb.cpu().numpy(),
        "pbf": all_gather_var(opt.pbf, opt.dist).cpu().numpy(),
        "swarm": all_gather_var(opt.swarm, opt.dist).cpu().numpy(), "swarm_host": np.array(opt.swarm_host),
        "fit": all_gather_var(opt.last_fitness, opt.dist).cpu().numpy(),
        "share": [(g, list(m), f.cpu().numpy()) for g, m, f in opt.share_history],
        "sizes": sizes, "offset": opt.offset,
    }
    return out


def run_sac(dist, n_envs, offset):
    """The c5 collection: the reference Actor (same init on every rank) drives this rank's envs;
    the learner rank's prioritized device buffer receives every rank's rows."""
    import torch
    import pdenv
    from pdenv.sac import Actor, DevicePrioritizedReplayBuffer, SACCollector
    rank = dist.get_rank() if dist else 0
    env = pdenv.PoweredDescentEnv(n_envs, flight_phase="landing_burn_pure_throttle", mode="rl", auto_reset=True,
                                  seed=1234, env_offset=offset)
    torch.manual_seed(0)
    actor = Actor(2, 1).to(env.device)
    buf = DevicePrioritizedReplayBuffer(SAC_CAP, 2, 1, env.device) if rank == 0 else None
    col = SACCollector(env, actor, buf, dist)
    assert col.kernel is not None                   # the fused actor + step kernel
    rows = []
    for _ in range(SAC_STEPS):
        rows.append(col.step().cpu().numpy().copy())
    torch.cuda.synchronize()
    out = {"rows": np.stack(rows), "ring": col.ring}
    if buf is not None:
        out.update(data=buf.data.cpu().numpy(), prio=buf.priorities.cpu().numpy(), position=buf.position,
                   size=buf.size, dev_state=buf.state_dev.cpu().numpy())
    return out


def _worker(rank, world, port, out):
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = HostStagedGroup(dist)
    try:
        pso = run_pso(g)
        sac = run_sac(g, SAC_ENVS, rank * SAC_ENVS)
        out[rank] = {"pso": pso, "sac": sac}
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def runs():
    import torch
    import torch.multiprocessing as mp
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    sys.path.insert(0, PKG)
    one = {"pso": run_pso(None), "sac": run_sac(None, 2 * SAC_ENVS, 0)}
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, _free_port(), res), nprocs=2, join=True)
        two = [dict(res[0]), dict(res[1])]
    return one, two


@pytest.mark.timeout(600)
def test_pso_two_ranks_equal_world_one(runs):
    """c4 on two ranks: the same generations as one rank, bit for bit, through migrations (5, 10,
    15), a share (10) and the re-initialisation (12) that leaves the ranks uneven shards."""
    one, two = runs
    a = one["pso"]
    for r in (0, 1):
        b = two[r]["pso"]
        assert b["gbf"] == a["gbf"] and np.array_equal(b["gb"], a["gb"])
        assert np.array_equal(b["sbf"], a["sbf"]) and np.array_equal(b["sb"], a["sb"])
        for k in ("x", "pb", "pbf", "swarm", "swarm_host", "fit"):
            assert b[k].shape == a[k].shape and np.array_equal(b[k], a[k]), k
        assert len(b["share"]) == len(a["share"]) >= 1
        for (g1, m1, f1), (g2, m2, f2) in zip(a["share"], b["share"]):
            assert g1 == g2 and m1 == m2 and np.array_equal(f1, f2)
    # the shards: even before the re-initialisation, uneven after it
    s0, s1 = two[0]["pso"]["sizes"], two[1]["pso"]["sizes"]
    assert s0[:12] == s1[:12] == [PSO_POP // 2] * 12
    assert s0[-1] + s1[-1] == 600 == a["sizes"][-1]
    assert two[1]["pso"]["offset"] == s0[-1]
    assert np.isfinite(a["gbf"])


@pytest.mark.timeout(600)
def test_sac_two_ranks_equal_world_one(runs):
    """c5 on two ranks: every step's gathered transition rows and the learner's replay ring
    (rows, priorities, position, size; the ring wraps every 7.5 steps) equal the world-1 ring bit for bit."""
    one, two = runs
    a = one["sac"]
    assert a["ring"] and not two[0]["sac"]["ring"]   # world 1 writes the ring in the kernel
    for r in (0, 1):
        assert np.array_equal(two[r]["sac"]["rows"], a["rows"])
    b = two[0]["sac"]
    assert b["position"] == a["position"] == (SAC_STEPS * 2 * SAC_ENVS) % SAC_CAP
    assert b["size"] == a["size"] == SAC_CAP
    assert np.array_equal(b["data"], a["data"]) and np.array_equal(b["prio"], a["prio"])
    assert list(a["dev_state"][:2]) == [a["position"], a["size"]]
    # episodes ended and auto-reset inside the window: a row's next state differs from the next
    # step's state only where the env was reset in between
    nxt, cur = a["rows"][:-1, :, 3:5], a["rows"][1:, :, 0:2]
    assert (nxt != cur).any(axis=-1).sum() > 0
