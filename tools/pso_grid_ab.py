#!/usr/bin/env python3
"""The swarm update alone: pd_pso_step (k_pso_step, plain float32 copy) against pd_pso_step_chunked
(k_pso_step4, the copy in the rollout's chunked layout), one swarm state restored before each,
HIP events around each call, rounds interleaved.  (The plain path's rollout adds k_wchunk, the
copy pass; see the kernel traces.)  The round-6 experiment build also had a PD_PSO_GRID switch for
k_pso_step4's grid order (0 = particle range fastest, kept; 1 = chunk fastest; 2 = tiles of 4 096
particles), the "grid0/1/2" lines of profiles/r06_exp_pso_chunked.jsonl."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
from pdenv import _lib as L  # noqa: E402
from pdenv.env import _ptr, _stream  # noqa: E402


def main():
    P = int(os.environ.get("P", "262144"))
    D, S, rounds = 372, 8, int(os.environ.get("ROUNDS", "6"))
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    dev = dict(device="cuda", dtype=torch.float64)
    x0 = torch.rand(D, P, generator=g, **dev) * 3 - 1.5
    v0 = torch.randn(D, P, generator=g, **dev) * 0.1
    pb0 = torch.rand(D, P, generator=g, **dev) * 3 - 1.5
    pbf0 = torch.rand(P, generator=g, **dev) * 10
    fit = torch.rand(P, generator=g, **dev) * 10
    sb = torch.rand(S, D, generator=g, **dev) * 3 - 1.5
    sw = torch.randint(0, S, (P,), device="cuda", dtype=torch.int32)
    lo, hi = torch.full((D,), -1.5, **dev), torch.full((D,), 1.5, **dev)
    x, v, pb, pbf = x0.clone(), v0.clone(), pb0.clone(), pbf0.clone()
    x32 = torch.empty(D, P, device="cuda", dtype=torch.float32)
    x32c = torch.empty((D + 3) // 4, P, 4, device="cuda", dtype=torch.float32)
    times = {}
    for r in range(rounds + 1):
        for var in ("plain", "chunked"):
            for t, t0 in ((x, x0), (v, v0), (pb, pb0), (pbf, pbf0)):
                t.copy_(t0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            args = (P, D, _ptr(fit), _ptr(pbf), _ptr(x), _ptr(v), _ptr(pb), _ptr(sb), _ptr(sw), _ptr(lo), _ptr(hi),
                    0.7, 1.0, 1.0, 5, r, 0)
            if var == "plain":
                L.check(lib.pd_pso_step(*args, _ptr(x32), None))
            else:
                L.check(lib.pd_pso_step_chunked(*args, _ptr(x32c), None))
            e1.record()
            torch.cuda.synchronize()
            if r > 0:
                times.setdefault(var, []).append(e0.elapsed_time(e1))
    for var, t in times.items():
        t = sorted(t)
        print(json.dumps({"variant": var, "particles": P, "update_ms_med": t[len(t) // 2], "update_ms_min": t[0]}))


if __name__ == "__main__":
    main()
