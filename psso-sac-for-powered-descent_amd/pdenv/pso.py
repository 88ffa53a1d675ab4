"""Device-resident particle subswarm optimisation.

ParticleSubswarmOptimisation.run (src/particle_swarm_optimisation/particle_swarm_optimisation.py
:285-520) with the swarm kept on the GPU between generations: particles are evaluated by
pd_rollout_policy_chunked (the actor fused into the step kernel), the personal-best / velocity /
position update is pd_pso_step_chunked (binary64, parameter-major [D][P]; its float32 copy is
written in the rollout's chunked weight layout, so a generation makes no copy pass), and only
per-subswarm minima cross ranks.  The reference's parameters
(configs/evolutionary_algorithms_config.py) are the defaults; the population can be scaled to config c4's 262 144 particles.

Randomness: positions U(bounds) at init, r1/r2 per particle and generation (Philox, in the
kernel), and a seeded Python `random.Random` for the share/migrate decisions that the reference
draws from `random` -- the same on every rank, so all ranks take identical decisions.
"""
import math
import random

import numpy as np
import torch

from . import _lib as L
from .env import PoweredDescentEnv, _ptr, _stream

# configs/evolutionary_algorithms_config.py:69-101
PSO_PARAMS = {
    "landing_burn_pure_throttle": dict(pop_size=150, generations=400, c1=1, c2=1, w_start=0.9, w_end=0.4,
                                       num_sub_swarms=2, communication_freq=10, migration_freq=5,
                                       number_of_migrants=1, re_initialise_number_of_particles=600,
                                       re_initialise_generation=90),
    "landing_burn": dict(pop_size=200, generations=400, c1=1, c2=1, w_start=0.9, w_end=0.7,
                         num_sub_swarms=2, communication_freq=10, migration_freq=5, number_of_migrants=1,
                         re_initialise_number_of_particles=600, re_initialise_generation=90),
}
ACTOR_DIM = {"landing_burn_pure_throttle": 249, "landing_burn": 372}


def _to_device(values, dtype, device):
    """A host list as a device tensor through pinned staging, copied on the current stream (a
    pageable copy would wait for the queue: a generation that draws host-side decisions must not
    drain it)."""
    return torch.tensor(values, dtype=dtype).pin_memory().to(device, non_blocking=True)


def chunk4(w):
    """float32 actor weights [D][n] -> the chunked layout [ceil(D/4)][n][4] (chunk c of column i
    holds parameters 4c .. 4c+3, zeros past D) that pd_rollout_policy_chunked reads and
    pd_pso_step_chunked writes."""
    D, n = w.shape
    C = (D + 3) // 4
    if C * 4 != D:
        w = torch.cat([w, torch.zeros(C * 4 - D, n, dtype=w.dtype, device=w.device)])
    return w.reshape(C, 4, n).permute(0, 2, 1).contiguous()


def unchunk4(w4, D):
    """The inverse of chunk4: [C][n][4] -> [D][n]."""
    C, n, _ = w4.shape
    return w4.permute(0, 2, 1).reshape(C * 4, n)[:D].contiguous()


def all_gather_var(t, dist):
    """Every rank's 1-D tensor `t` concatenated in rank order, for shards of DIFFERENT lengths
    (after re_initialise_swarms the ranks keep different numbers of particles, possibly none):
    the lengths are gathered first, each shard padded to the longest, gathered, and trimmed."""
    if dist is None:
        return t
    world = dist.get_world_size()
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x) for x in ns]
    m = max(ns)
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[:t.numel()] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([parts[r][:ns[r]] for r in range(world)])


def reinit_keep(pbf, swarm, n_swarms, keep_n):
    """re_initialise_swarms' selection (particle_swarm_optimisation.py:360-370) on the global
    population: per subswarm the keep_n particles with the best personal-best fitness (stable,
    the lowest index first on ties).  Returns the boolean keep mask."""
    keep = torch.zeros_like(pbf, dtype=torch.bool)
    for s in range(n_swarms):
        idx = torch.nonzero(swarm == s).flatten()
        order = torch.argsort(pbf[idx], stable=True)[:keep_n]
        keep[idx[order]] = True
    return keep


def migration_moves(swarm, n_swarms, n_migrants, rng):
    """migrate_particles' decisions (particle_swarm_optimisation.py:545-553) on the global
    membership `swarm` (subswarm id per global particle): [(particle, new subswarm)].  The member
    lists are NumPy index arrays (one read-back of the membership; pop = delete, append = concat,
    the same order as the reference's Python lists)."""
    sw = swarm.cpu().numpy() if torch.is_tensor(swarm) else np.asarray(swarm)
    members = [np.flatnonzero(sw == s) for s in range(n_swarms)]
    moves = []
    for i in range(n_swarms):
        if len(members[i]) > 1:
            for _ in range(n_migrants):
                k = rng.randrange(len(members[i]))
                g = int(members[i][k])
                members[i] = np.delete(members[i], k)
                t = rng.choice([j for j in range(n_swarms) if j != i])
                members[t] = np.append(members[t], g)
                moves.append((g, t))
    return moves


def local_moves(moves, offset, n_local):
    """The migration moves [(global particle, new subswarm)] that hit this rank's particles
    [offset, offset + n_local), as {local index: subswarm}: a particle moved twice in one
    migration ends in its last subswarm, as the reference's sequential list edits leave it."""
    mine = {}
    for g, t in moves:
        if offset <= g < offset + n_local:
            mine[g - offset] = t
    return mine


class ParticleSubswarmOptimisationGPU:
    """One rank's shard of the swarm.  Global particle g belongs to subswarm g // (pop / S)
    (initialize_swarms, :372-389); rank r holds particles [r*P_local, (r+1)*P_local)."""

    def __init__(self, flight_phase="landing_burn", pso_params=None, pop_size=None, enable_wind=False,
                 stochastic_wind=False, horiontal_wind_percentile=50, device=0, precision="f64", seed=0,
                 dist=None, max_steps=2200, tuning=None):
        self.flight_phase = flight_phase
        self.tuning = dict(tuning or {})     # pd_tuning fields of the rollout handles (PoweredDescentEnv.set_tuning)
        self.p = dict(PSO_PARAMS[flight_phase])
        if pso_params:
            self.p.update(pso_params)
        if pop_size:
            self.p["pop_size"] = int(pop_size)
        self.dist = dist if dist is not None and dist.is_initialized() else None
        self.world = self.dist.get_world_size() if self.dist else 1
        self.rank = self.dist.get_rank() if self.dist else 0
        self.device = torch.device("cuda", device)
        self.D = ACTOR_DIM[flight_phase]
        self.S = self.p["num_sub_swarms"]
        pop = self.p["pop_size"]
        self.sub_size = pop // self.S
        pop = self.sub_size * self.S                      # the reference builds S * (pop // S)
        if pop % self.world:
            raise ValueError("pop_size must split evenly over the ranks")
        self.P = pop // self.world
        self.offset = self.rank * self.P
        self.seed = int(seed)
        self.max_steps = max_steps
        self.env_kw = dict(mode="pso", precision=precision, device=device, enable_wind=enable_wind,
                           stochastic_wind=stochastic_wind, wind_percentile=horiontal_wind_percentile, seed=seed)
        self.rng = random.Random(seed)                    # share/migrate decisions, same on all ranks
        self.lib = L.load()
        b = torch.tensor([[-1.5, 1.5]] * self.D, dtype=torch.float64)   # simple_actor.return_setup_vals bounds
        self.lower = b[:, 0].contiguous().to(self.device)
        self.upper = b[:, 1].contiguous().to(self.device)
        self.initialize_swarms()

    # ------------------------------------------------------------------ state
    def initialize_swarms(self):
        # the GLOBAL swarm's uniforms from one seed on every rank, this rank's columns kept: a
        # particle's start position depends on its global index only, so any world size starts
        # from the same swarm (and world 1 draws exactly what it always drew)
        g = torch.Generator(device=self.device).manual_seed(self.seed * 1000003)
        u = torch.rand(self.D, self.P * self.world, generator=g, device=self.device, dtype=torch.float64)
        u = u[:, self.offset:self.offset + self.P]
        self.x = (self.lower[:, None] + (self.upper - self.lower)[:, None] * u).contiguous()
        del u
        self.v = torch.zeros_like(self.x)
        self.pb = torch.zeros_like(self.x)
        self.pbf = torch.full((self.P,), math.inf, dtype=torch.float64, device=self.device)
        # the float32 actor weights in the rollout's chunked layout (pd_pso_step_chunked keeps it)
        self.x32c = chunk4(self.x.float())
        gid = torch.arange(self.offset, self.offset + self.P, device=self.device)
        self.swarm = (gid // self.sub_size).to(torch.int32).contiguous()
        # the GLOBAL membership mirrored on the host: only migrate_particles (host-drawn moves) and
        # re_initialise_swarms (which reads the device anyway) change it, so a migration draws its
        # moves without reading the device back (that read drained the queue every fifth
        # generation: c4 generations 5 / 10 / 15 took 1.7-1.9 ms against 1.37)
        self.swarm_host = (np.arange(self.P * self.world) // self.sub_size).astype(np.int32)
        # subswarm / global bests stay on the device: a generation reads nothing back
        self.sb = torch.zeros(self.S, self.D, dtype=torch.float64, device=self.device)
        self.sbf_t = torch.full((self.S,), math.inf, dtype=torch.float64, device=self.device)
        self.gbf_t = torch.full((), math.inf, dtype=torch.float64, device=self.device)
        self.gb_t = torch.zeros(self.D, dtype=torch.float64, device=self.device)
        self._cols = torch.arange(self.S, device=self.device)
        self.w = self.p["w_start"]
        self.env = self._new_env(self.P, self.offset) if self.P > 0 else None
        # share_information evaluates 1..S-1 moved subswarm bests: one handle of S - 1 envs made
        # here (creating a handle inside a generation costs tens of ms), candidates padded to it
        self._aux = {self.S - 1: self._new_env(self.S - 1)} if self.S > 1 else {}
        self.last_fitness = None
        self._pending = None           # a share's candidates, evaluated with the next generation
        # every completed share: (generation, moved subswarms, count, candidates' fitness), the
        # moved subswarms a host list (count None) or, for a share decided on the device, the padded
        # device index tensor and a device count (share_history / share_log read them back)
        self._share_raw = []
        self._make_merged_handle()
        self._warm_share_path()

    def _new_env(self, n, offset=0):
        """A rollout handle of n envs whose env i is global particle offset + i (the Philox key
        of a stochastic-wind episode: the same draws at any world size)."""
        env = PoweredDescentEnv(n, self.flight_phase, env_offset=offset, **self.env_kw)
        if self.tuning:
            env.set_tuning(**self.tuning)
        return env

    def _mergeable(self):
        """share_information's candidates ride along with the next generation's rollout (S - 1 more
        envs in one launch sequence instead of a latency-bound rollout of their own) unless the
        wind is stochastic: a candidate's noise then depends on its env index, which must be the
        same on every rank."""
        return self.S > 1 and self.P > 0 and not (self.env_kw["enable_wind"] and self.env_kw["stochastic_wind"])

    def _make_merged_handle(self):
        n = self.P + self.S - 1
        for k in [k for k in self._aux if k not in (self.S - 1, n)]:   # (a merged handle of an earlier P)
            self._aux.pop(k).close()
        if self._mergeable() and n not in self._aux:
            self._aux[n] = self._new_env(n, self.offset)

    def _warm_share_path(self):
        """share_information's tensor operations once on scratch copies (no rng draws, no state
        change): the first launch of a kernel in a process loads its code object, which cost a
        timed generation 50-180 ms when the first non-empty share came."""
        if self.S < 2:
            return
        if self._mergeable():
            sb, sbf = self.sb.clone(), self.sbf_t.clone()
            u = _to_device([0.25] * (self.S - 1), torch.float64, self.device)
            pad, count, _ = self._share_on_device(sb, sbf, u)
            self._flush_on_device(sbf, pad, count, torch.zeros(self.S - 1, dtype=torch.float64, device=self.device))
        sb, sbf = self.sb.clone(), self.sbf_t.clone()
        moved = [0]
        sb[0] = (1 - 0.3) * sb[0] + 0.3 * sb[self.S - 1]
        pad = moved + [moved[0]] * (self.S - 1 - len(moved))
        cand = chunk4(sb[pad].t().float())
        fit = torch.zeros(cand.shape[1], dtype=torch.float64, device=self.device)[:len(moved)]
        mv = _to_device(moved, torch.int64, self.device)
        old = sbf[mv]
        sbf[mv] = torch.where(fit < old, fit, old)
        sb[mv] = (1 - 0.3) * sb[mv] + 0.3 * sb[self.S - 1]
        if self._mergeable():
            torch.cat([self.x32c, cand], dim=1)
        if self.P > 0:
            sw = self.swarm.clone()
            sw.index_put_((_to_device([0], torch.int64, self.device),), _to_device([0], torch.int32, self.device))
        torch.cuda.synchronize(self.device)

    def _env_for(self, n):
        if self.env is not None and self.env.n == n:
            return self.env
        if n not in self._aux:                                  # share_information's candidates
            self._aux[n] = self._new_env(n)
        return self._aux[n]

    @property
    def x32(self):
        """The swarm's float32 positions [D][P] (a copy of the chunked weights the rollouts read)."""
        return unchunk4(self.x32c, self.D)

    def evaluate(self, x32):
        """pso_wrapped_env.objective_function for every particle of x32 (fused actor): chunked
        weights [ceil(D/4)][n][4] (chunk4; pd_rollout_policy_chunked) or plain [D][n]
        (pd_rollout_policy, which chunks them itself)."""
        n = x32.shape[1]
        if n == 0:
            return torch.empty(0, dtype=torch.float64, device=self.device), torch.empty(0, dtype=torch.int32)
        env = self._env_for(n)
        fit = torch.empty(n, dtype=env.dtype, device=self.device)
        steps = torch.empty(n, dtype=torch.int32, device=self.device)
        roll = self.lib.pd_rollout_policy_chunked if x32.dim() == 3 else self.lib.pd_rollout_policy
        L.check(roll(env.h, _ptr(x32), self.D, self.max_steps, _ptr(fit), _ptr(steps), 8, _stream(self.device)))
        return fit.double(), steps

    # ------------------------------------------------------------------ one generation
    # host views of the device bests (each read synchronises; the generation itself never reads);
    # a read first completes a pending share, so that what it shows is what the reference's
    # share_information leaves behind
    @property
    def sbf(self):
        self.flush_share()
        return [float(v) for v in self.sbf_t.cpu()]

    @property
    def gbf(self):
        self.flush_share()
        return float(self.gbf_t)

    @property
    def gb(self):
        return None if not math.isfinite(self.gbf) else self.gb_t.clone()

    @property
    def share_history(self):
        """[(generation, moved subswarms, their candidates' fitness)] of every share_information
        that moved a subswarm (reads the device decisions back)."""
        self.flush_share()
        out = []
        for gen, moved, count, fit in self._share_raw:
            if count is not None:
                c = int(count)
                if c == 0:
                    continue
                moved = [int(i) for i in moved[:c].tolist()]
                fit = fit[:c]
            out.append((gen, moved, fit))
        return out

    @property
    def share_log(self):
        """(moved subswarms, their candidates' fitness) of the last share_information that moved
        a subswarm."""
        h = self.share_history
        return (h[-1][1], h[-1][2]) if h else None

    def flush_share(self, fit=None):
        """Complete a pending share_information (:533-541): the candidates' fitness (`fit`, from
        the merged rollout; else evaluated now on the share handle) replaces a subswarm's best
        fitness when strictly better."""
        if self._pending is None:
            return
        gen, moved, count, cand = self._pending
        self._pending = None
        if count is not None:                                    # decided on the device
            if fit is None:
                if int(count) == 0:                              # (a read: nothing moved)
                    return
                fit, _ = self.evaluate(cand)
            fit = fit[:self.S - 1].clone()
            self._share_raw.append((gen, moved, count, fit))
            self._flush_on_device(self.sbf_t, moved, count, fit)
            return
        if fit is None:
            fit, _ = self.evaluate(cand)
        fit = fit[:len(moved)].clone()
        self._share_raw.append((gen, moved, None, fit))
        mv = _to_device(moved, torch.int64, self.device)
        old = self.sbf_t[mv]
        self.sbf_t[mv] = torch.where(fit < old, fit, old)

    @staticmethod
    def _flush_on_device(sbf, pad, count, fit):
        """The strictly-better replacement of a device-decided share: every padded entry repeats
        the first moved subswarm with its (same) candidate, so the duplicate writes agree; nothing
        changes when nothing moved."""
        old = sbf.index_select(0, pad)
        sbf.index_put_((pad,), torch.where((count > 0) & (fit < old), fit, old))

    def _swarm_minima(self, fit):
        """Per subswarm: (min fitness, its position) over all ranks, first particle on ties, a NaN
        fitness never chosen (the reference's sequential strict '<') -- a two-pass segmented
        argmin on the device (pd_pso_swarm_minima), no host synchronisation.  A subswarm with no
        particle of non-NaN fitness here reports +inf (so a rank's minima never hold a NaN, and
        torch.argmin over the ranks picks the lowest rank among equal minima)."""
        f = torch.empty(self.S, dtype=torch.float64, device=self.device)
        pos = torch.empty(self.S, self.D, dtype=torch.float64, device=self.device)
        need = int(self.lib.pd_pso_swarm_minima_scratch_bytes(self.P, self.S))
        if getattr(self, "_min_scratch", None) is None or self._min_scratch.numel() < need:
            self._min_scratch = torch.empty(need, dtype=torch.uint8, device=self.device)   # the first pass's partials
        L.check(self.lib.pd_pso_swarm_minima(self.P, self.D, self.S, _ptr(fit) if self.P else None,
                                             _ptr(self.swarm) if self.P else None, _ptr(self.x) if self.P else None,
                                             _ptr(f), _ptr(pos), _ptr(self._min_scratch), need, _stream(self.device)))
        if self.dist:
            fa = [torch.empty_like(f) for _ in range(self.world)]
            pa = [torch.empty_like(pos) for _ in range(self.world)]
            self.dist.all_gather(fa, f)
            self.dist.all_gather(pa, pos)
            F, Pz = torch.stack(fa), torch.stack(pa)            # [world, S], [world, S, D]
            r = torch.argmin(F, dim=0)                          # lowest rank on ties
            cols = torch.arange(self.S, device=self.device)
            f = F[r, cols]
            pos = Pz[r, cols]
        return f, pos

    def generation(self, gen):
        if self._pending is not None and self._mergeable():
            # the previous generation's share candidates as S - 1 more envs of this rollout (each
            # env's episode is independent of the batch: the same fitness bits as on their own);
            # their bests are updated before this generation's (the reference's order)
            cand = self._pending[3]
            fit_all, _ = self.evaluate(torch.cat([self.x32c, cand], dim=1))
            fit = fit_all[:self.P]
            self.flush_share(fit_all[self.P:])
        else:
            self.flush_share()
            fit, _ = self.evaluate(self.x32c)
        self.last_fitness = fit
        f, pos = self._swarm_minima(fit)
        # :442-444 per subswarm: a strictly better minimum replaces the subswarm best; :474-477
        # subswarms in order, strictly better replaces: the first subswarm holding the minimum,
        # if it beats the global best (pd_pso_update_bests, one workgroup)
        L.check(self.lib.pd_pso_update_bests(self.S, self.D, _ptr(f), _ptr(pos), _ptr(self.sbf_t), _ptr(self.sb),
                                             _ptr(self.gbf_t), _ptr(self.gb_t), _stream(self.device)))
        self.w = self.p["w_start"] - (self.p["w_start"] - self.p["w_end"]) * gen / self.p["generations"]
        if self.P > 0:
            L.check(self.lib.pd_pso_step_chunked(self.P, self.D, _ptr(fit), _ptr(self.pbf), _ptr(self.x),
                                                 _ptr(self.v), _ptr(self.pb), _ptr(self.sb), _ptr(self.swarm),
                                                 _ptr(self.lower), _ptr(self.upper), float(self.w), float(self.p["c1"]),
                                                 float(self.p["c2"]), self.seed, gen, self.offset, _ptr(self.x32c),
                                                 _stream(self.device)))
        self._gen = gen
        if gen % self.p["communication_freq"] == 0 and gen > 0:
            self.share_information()
        if gen % self.p["migration_freq"] == 0 and gen > 0:
            self.migrate_particles()
        if gen == self.p["re_initialise_generation"]:
            self.re_initialise_swarms()
        return fit

    def run(self, generations=None):
        for gen in range(generations if generations is not None else self.p["generations"]):
            self.generation(gen)
        self.flush_share()
        return self.gb, self.gbf

    # ------------------------------------------------------------------ share / migrate / re-init
    def _share_on_device(self, sb, sbf, u):
        """share_information's decisions on the device, from the S - 1 uniforms the reference's
        loop draws (one per subswarm but the best, in order -- the count does not depend on which
        is best): best = the first minimum of sbf (np.argmin), subswarm i != best moves when its
        uniform (draw i, or i - 1 past best) is below 1/2, and moves 30 % toward the best's
        position.  Returns the moved subswarms ascending, padded to S - 1 with the first (the
        share handle's size), their count, and the candidates in the rollout's chunked layout."""
        S = self.S
        i = self._cols
        best = torch.argmin(sbf)
        k = (i - (i > best).long()).clamp(max=S - 2)
        moved = (i != best) & (u.index_select(0, k) < 0.5)
        toward = 0.3 * sb.index_select(0, best.view(1))
        sb.copy_(torch.where(moved[:, None], (1 - 0.3) * sb + toward, sb))
        order = torch.argsort(torch.where(moved, i, i + S))
        count = moved.sum()
        pos = torch.arange(S - 1, device=self.device)
        pad = torch.where(pos < count, order[:S - 1], order[0])
        return pad, count, chunk4(sb.index_select(0, pad).t().float())

    def share_information(self):
        """:521-543: for every subswarm but the best, with probability 1/2 its best position moves
        30 % toward the best subswarm's; the moved position is re-evaluated and its fitness kept
        only if better (the position is kept either way, as in the reference).  When the
        candidates ride along with the next rollout the decisions are taken on the device from
        the host's uniforms (no read-back: the host used to wait for the queue to read the bests,
        idling the GPU ~250 us every communication_freq generations)."""
        if self._mergeable():
            self.flush_share()
            u = _to_device([self.rng.random() for _ in range(self.S - 1)], torch.float64, self.device)
            pad, count, cand = self._share_on_device(self.sb, self.sbf_t, u)
            self._pending = (getattr(self, "_gen", None), pad, count, cand)
            return
        best = int(np.argmin(self.sbf))                         # (one read-back: the rng draws depend on it)
        moved = [i for i in range(self.S) if i != best and self.rng.random() < 0.5]
        if not moved:
            return
        mv = _to_device(moved, torch.int64, self.device)
        self.sb[mv] = (1 - 0.3) * self.sb[mv] + 0.3 * self.sb[best]
        pad = moved + [moved[0]] * (self.S - 1 - len(moved))  # (padded to the share handle's size)
        cand = chunk4(self.sb[pad].t().float())                 # [ceil(D/4)][S-1][4]
        # evaluated with the next generation's rollout (or on the next read of the bests)
        self._pending = (getattr(self, "_gen", None), moved, None, cand)

    def migrate_particles(self):
        """:545-553: number_of_migrants random particles of every subswarm (with > 1 member) move
        to a random other subswarm.  Decisions are taken on the global membership (all ranks
        draw the same choices); each rank applies those that hit its own particles."""
        moves = migration_moves(self.swarm_host, self.S, self.p["number_of_migrants"], self.rng)
        for g, t in moves:
            self.swarm_host[g] = t
        mine = local_moves(moves, self.offset, self.P)
        if mine:
            # one pinned, stream-ordered copy of the (index, subswarm) pairs and one scatter: a
            # Python-int item write is a pageable 4-byte copy, which waits for the queue (two of
            # them idled the GPU 30-37 us each per migration, profiles/r06_exp_policy_init.json)
            idx = _to_device(list(mine.keys()), torch.int64, self.device)
            val = _to_device(list(mine.values()), torch.int32, self.device)
            self.swarm.index_put_((idx,), val)

    def re_initialise_swarms(self):
        """:360-370: every subswarm keeps its re_initialise_number_of_particles // S best
        particles (by personal best fitness); the rest are dropped."""
        keep_n = self.p["re_initialise_number_of_particles"] // self.S
        pbf = all_gather_var(self.pbf, self.dist)
        sw = all_gather_var(self.swarm, self.dist)
        keep = reinit_keep(pbf, sw, self.S, keep_n)
        self.swarm_host = sw.cpu().numpy()[keep.cpu().numpy()].astype(np.int32)
        mine = keep[self.offset:self.offset + self.P]
        sel = torch.nonzero(mine).flatten()
        self.x, self.v, self.pb = (t[:, sel].contiguous() for t in (self.x, self.v, self.pb))
        self.pbf, self.swarm = self.pbf[sel].contiguous(), self.swarm[sel].contiguous()
        self.x32c = chunk4(self.x.float())
        gids = torch.nonzero(keep).flatten()
        self.offset = int((gids < self.offset).sum()) if self.P else 0
        self.P = int(sel.numel())
        if self.env is not None:
            self.env.close()
        self.env = self._new_env(self.P, self.offset) if self.P > 0 else None
        self._make_merged_handle()
