"""How long does an env stay on one table path?  (regime-coherent waves.)

The step kernel's lookup takes one of two paths per sub-step: the clamped lines (|alpha_eff| >
radians(10) in degrees, both tables clamp; Taylor pieces) or the interior grids (fine index ->
cell piece).  A wave whose lanes take both runs both, one after the other.  Binning the envs by
path at each launch boundary (a permutation applied at launch, every F fused steps) only helps if
an env keeps its path for most of the next F steps.  This tool measures that on the oracle (the
CPU restatement; test/analysis infrastructure, never the product path), under the c3 and
c3-descent action laws of bench.py, after their burn-in, with the oracle's per-sub-step path log
(orc_set_qlog):

- the workgroup query exchange instead (csrc/pd_step_impl.h rbf2_exchange): every sub-step the
  256 queries of a workgroup's 128 envs (both tables take an env's path) are sorted by path over
  its four waves, so a wave sub-step is mixed only where the line / interior boundary falls
  inside it;
- flips: the share of env sub-steps (and env-steps) whose path differs from the previous one;
- mixed wave sub-steps (32 envs per wave at 2 lanes per env; sub-steps with envs on both paths)
  in the natural env order, and after sorting the envs by their path at each launch boundary,
  for F = 1 .. 128 steps per launch -- plus a clairvoyant sort by the majority path of the
  coming launch, which bounds any launch-boundary binning.

    python tools/regime_persistence.py [--envs 1024] [--window 256] [--out profiles/...json]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

BURN_IN = 640      # bench.py C3_BURN_IN / DESCENT_BURN_IN
ENVS_PER_WAVE = 32


def actions(T, n, descent, rng):
    """bench.py c3_actions in numpy: U(-1, 1); descent: U(0.5, 1) on three envs in four."""
    u = rng.random((T, n, 1), dtype=np.float32)
    if not descent:
        return (u * 2 - 1).astype(np.float32)
    hi = (np.arange(n) % 4 != 0).reshape(1, n, 1)
    return np.where(hi, 0.5 + 0.5 * u, 2 * u - 1).astype(np.float32)


def mixed_share(q, order_of_launch, F):
    """q [T, n, 4] path per sub-step (1 line, 2 interior, 0 none); order_of_launch(t0) -> env
    permutation for the launch starting at step t0.  Share of wave sub-steps with both paths."""
    T, n, _ = q.shape
    W = n // ENVS_PER_WAVE
    mixed = total = 0
    for t0 in range(0, T, F):
        perm = order_of_launch(t0)
        blk = q[t0:t0 + F][:, perm, :]                       # [F, n, 4]
        blk = blk.reshape(blk.shape[0], W, ENVS_PER_WAVE, 4)
        has_line = (blk == 1).any(axis=2)
        has_int = (blk == 2).any(axis=2)
        mixed += int((has_line & has_int).sum())
        total += has_line.size
    return mixed / total


def analyse(descent, n, window, threads, seed):
    T = BURN_IN + window
    rng = np.random.default_rng(seed)
    acts = actions(T, n, descent, rng)
    q = np.zeros((T, n, 4), np.uint8)
    t0 = time.time()
    O.rollout_philox(O.PURE_THROTTLE, O.RTD_RL, np.arange(n, dtype=np.uint64), np.zeros(n, np.uint32), acts,
                     auto_reset=True, wind=True, stochastic=True, tilt=math.radians(1.0), seed=1234,
                     threads=threads, qclass=q)
    cpu_s = time.time() - t0
    q = q[BURN_IN:]
    flat = q.transpose(0, 2, 1).reshape(-1, n)              # [window * 4, n], sub-steps in time order
    prev, cur = flat[:-1], flat[1:]
    valid = (prev != 0) & (cur != 0)
    flips_sub = float(((prev != cur) & valid).sum() / max(valid.sum(), 1))
    last = q[:, :, 3]
    flips_step = float(((q[1:] != q[:-1, :, 3:4]).any(axis=2) & (last[:-1] != 0)).mean())
    line_share = float((q == 1).sum() / max((q != 0).sum(), 1))
    res = dict(workload="c3-descent" if descent else "c3", envs=n, burn_in=BURN_IN, window=window,
               oracle_seconds=round(cpu_s, 1), line_share=round(line_share, 4),
               flips_per_env_substep=round(flips_sub, 4), env_steps_with_a_flip=round(flips_step, 4), by_F={})
    # the exchange: per sub-step and workgroup of 128 envs, 2 * n_line line queries from slot 0
    wg = q.reshape(window, n // 128, 128, 4)
    nl2 = 2 * (wg == 1).sum(axis=2)                            # [window, WG, 4] line queries
    res["exchange_mixed_wave_substeps"] = round(float((nl2 % 64 != 0).sum() / (nl2.size * 4)), 4)
    natural = lambda t0: np.arange(n)
    for F in (1, 2, 8, 32, 128):
        def at_boundary(t0):
            # the path each env took in the last sub-step before the launch (the state the
            # launch-boundary pass would see), stable sort
            key = q[t0 - 1, :, 3] if t0 > 0 else q[0, :, 0]
            return np.argsort(key, kind="stable")

        def clairvoyant(t0):
            blk = q[t0:t0 + F]
            return np.argsort((blk == 1).sum(axis=(0, 2)) - (blk == 2).sum(axis=(0, 2)), kind="stable")
        res["by_F"][str(F)] = dict(natural=round(mixed_share(q, natural, F), 4),
                                   sorted_at_boundary=round(mixed_share(q, at_boundary, F), 4),
                                   clairvoyant=round(mixed_share(q, clairvoyant, F), 4))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--window", type=int, default=256)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r04_regime_persistence.json"))
    a = ap.parse_args()
    assert a.envs % ENVS_PER_WAVE == 0
    out = dict(tool="tools/regime_persistence.py", note=__doc__.split("\n\n")[0],
               results=[analyse(d, a.envs, a.window, a.threads, 7 + d) for d in (False, True)])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["results"], indent=1))


if __name__ == "__main__":
    main()
