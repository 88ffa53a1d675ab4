#!/usr/bin/env python3
"""c4 generations with the chunked swarm copy (pd_pso_step_chunked + pd_rollout_policy_chunked,
the product path since ABI 11) against the previous path (pd_pso_step's plain float32 copy
[D][P], which pd_rollout_policy chunks in a pass of its own), interleaved in one process: two
swarms of the same seed, blocks of G generations each in turn.  Shares, migrations and the
re-initialisation are off so that a generation is rollout + minima + bests + update in both.
Prints the median generation wall time of each path and checks that the two swarms stay bit-identical.
Env: P (particles, default 32768), G (generations per block, 8), ROUNDS (4)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
from pdenv import _lib as L  # noqa: E402
from pdenv.env import _ptr, _stream  # noqa: E402
from pdenv.pso import ParticleSubswarmOptimisationGPU  # noqa: E402


class PlainCopy(ParticleSubswarmOptimisationGPU):
    """The round-6 generation before ABI 11: a plain float32 copy, chunked by the rollout."""

    def generation(self, gen):
        if not hasattr(self, "x32p"):
            self.x32p = self.x.float().contiguous()
        fit, _ = self.evaluate(self.x32p)
        self.last_fitness = fit
        f, pos = self._swarm_minima(fit)
        L.check(self.lib.pd_pso_update_bests(self.S, self.D, _ptr(f), _ptr(pos), _ptr(self.sbf_t), _ptr(self.sb),
                                             _ptr(self.gbf_t), _ptr(self.gb_t), _stream(self.device)))
        self.w = self.p["w_start"] - (self.p["w_start"] - self.p["w_end"]) * gen / self.p["generations"]
        L.check(self.lib.pd_pso_step(self.P, self.D, _ptr(fit), _ptr(self.pbf), _ptr(self.x), _ptr(self.v),
                                     _ptr(self.pb), _ptr(self.sb), _ptr(self.swarm), _ptr(self.lower),
                                     _ptr(self.upper), float(self.w), float(self.p["c1"]), float(self.p["c2"]),
                                     self.seed, gen, self.offset, _ptr(self.x32p), _stream(self.device)))
        return fit


def main():
    P = int(os.environ.get("P", "32768"))
    G = int(os.environ.get("G", "8"))
    rounds = int(os.environ.get("ROUNDS", "4"))
    total = G * (rounds + 1)
    pp = dict(generations=total, communication_freq=10 ** 9, migration_freq=10 ** 9, re_initialise_generation=-1)
    opts = {"chunked": ParticleSubswarmOptimisationGPU("landing_burn", pop_size=P, seed=1234, pso_params=pp),
            "plain": PlainCopy("landing_burn", pop_size=P, seed=1234, pso_params=pp)}
    times = {k: [] for k in opts}
    gens = {k: 0 for k in opts}
    for r in range(rounds + 1):
        for k, o in opts.items():
            for _ in range(G):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o.generation(gens[k])
                torch.cuda.synchronize()
                if r > 0:                            # round 0: code objects, tables
                    times[k].append((time.perf_counter() - t0) * 1e3)
                gens[k] += 1
    a, b = opts["chunked"], opts["plain"]
    same = all(torch.equal(x, y) for o in opts.values()
               for x, y in ((a.x, o.x), (a.v, o.v), (a.pb, o.pb), (a.pbf, o.pbf), (a.gb_t, o.gb_t)))
    for k in opts:
        t = sorted(times[k])
        print(json.dumps({"path": k, "particles": P, "generations": len(t), "gen_ms_med": t[len(t) // 2],
                          "gen_ms_mean": sum(t) / len(t), "gen_ms_min": t[0]}))
    print(json.dumps({"bit_identical_swarms": bool(same), "gbf": [float(a.gbf_t), float(b.gbf_t)]}))


if __name__ == "__main__":
    main()
