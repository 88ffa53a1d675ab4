#!/usr/bin/env python3
"""Per-generation wall times of the c4 PSO driver (bench.py's configuration), each generation
bracketed by device syncs: which generations (share every 10, migrate every 5) cost what."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
import torch  # noqa: E402
from pdenv.pso import ParticleSubswarmOptimisationGPU  # noqa: E402

G = int(os.environ.get("GENS", "34"))
opt = ParticleSubswarmOptimisationGPU("landing_burn", pop_size=int(os.environ.get("P", "32768")), device=0,
                                      seed=1234, pso_params=dict(generations=G, re_initialise_generation=-1))
out = []
for g in range(G):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    opt.generation(g)
    torch.cuda.synchronize()
    out.append(round((time.perf_counter() - t0) * 1e3, 3))
print(json.dumps({"gen_ms": out, "mean_ms_from_2": sum(out[2:]) / len(out[2:])}))
# the share handle's work: episode length of its last evaluation, misses solved on device, and
# one more timed evaluation of the same candidate (tables now warm)
aux = opt._aux.get(opt.S - 1)
if aux is not None and getattr(opt, "share_log", None):
    moved = opt.share_log[0]
    cand = opt.sb[moved + [moved[0]] * (opt.S - 1 - len(moved))].t().float().contiguous()
    c0 = aux.counters()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    fit, steps = opt.evaluate(cand)
    torch.cuda.synchronize(); dt = time.perf_counter() - t0
    c1 = aux.counters()
    print(json.dumps({"share_eval_ms": dt * 1e3, "steps": steps.cpu().tolist(), "misses_before": c0["rbf_misses"],
                      "misses_during": c1["rbf_misses"] - c0["rbf_misses"], "main_misses": opt.env.counters()["rbf_misses"]}))
