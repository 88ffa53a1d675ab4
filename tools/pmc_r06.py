#!/usr/bin/env python3
"""Reduce tools/pmc_r06.sh's passes: per case, the last LAUNCHES k_step dispatches' FETCH_SIZE,
WRITE_SIZE (KiB per dispatch), TCC hits/misses, and the HBM-side bytes per unit, 2 FETCH_SIZE +
WRITE_SIZE (the MI355X guide's gfx950 reading of FETCH_SIZE; Infinity-Cache hits are counted):
c4_P: one refill rollout of P particles per dispatch (bytes per particle-episode), c5: one
collection step of 4 096 envs per dispatch (bytes per env-step).
Usage: python tools/pmc_r06.py > profiles/r06_pmc_c4c5.json"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_r05 import OUT, last_dispatches  # noqa: E402

UNITS = {"c4_32768": 32768, "c4_262144": 262144, "c5": 4096}
# dispatches averaged: the line's kernel-timing replays (c4: min(steps, 8) rollouts; c5: 64 steps)
K = {"c4_32768": 4, "c4_262144": 2, "c5": 16}


def main():
    res = {}
    for case, units in UNITS.items():
        r = {}
        for pn in ("fetch_size", "write_size", "tcc_hit_sum"):
            f = glob.glob(os.path.join(OUT, f"pmc6_{case}_{pn}", "**", "*counter_collection.csv"), recursive=True)
            if f:
                v, used = last_dispatches(f[0], K[case])
                r.update(v)
                r["dispatches_averaged"] = used
            lg = os.path.join(OUT, f"pmc6_{case}_{pn}.log")
            if os.path.exists(lg):
                for line in open(lg):
                    if line.startswith("{") and "ms_per_step" in line:
                        j = json.loads(line)
                        r.setdefault("line_under_profiler", {"value": j["value"], "ms_per_step": j["ms_per_step"],
                                                            "mean_episode_len": j.get("mean_episode_len_after")})
        if not r:
            continue
        r["units_per_dispatch"] = units
        r["unit"] = "particle-episode" if case.startswith("c4") else "env-step"
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["bytes_per_unit"] = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024.0 / units
            r["read_bytes_per_unit"] = 2 * r["FETCH_SIZE"] * 1024.0 / units
            r["write_bytes_per_unit"] = r["WRITE_SIZE"] * 1024.0 / units
        if "TCC_HIT_sum" in r:
            r["l2_hit_rate"] = r["TCC_HIT_sum"] / max(1.0, r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
        res[case] = r
    json.dump({"source": "tools/pmc_r06.sh + tools/pmc_r06.py (rocprofv3 --pmc over bench.py --workload c4 / c5; "
                         "the last k_step dispatches: the line's kernel-timing replays)", "cases": res},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
