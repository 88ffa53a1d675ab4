#!/usr/bin/env python3
"""Per-generation breakdown of a c4 rocprofv3 kernel trace (bench.py --workload c4): a
generation ends with its k_pso_step; wall = end of one k_pso_step to the end of the next, busy =
summed kernel durations inside, k_step = the fused actor + env rollout launches.
  python tools/trace_gens.py <run_kernel_trace.csv> [last_n] [out.json]"""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    ends = [i for i, r in enumerate(rows) if "k_pso_step" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    gens = []
    for a, b in zip(ends[:-1], ends[1:]):
        seg = rows[a + 1:b + 1]
        wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) * 1e-6
        ks = [r for r in seg if "k_step" in r["Kernel_Name"]]
        gens.append({"wall_ms": wall, "busy_ms": sum(map(dur, seg)), "k_step_ms": sum(map(dur, ks)),
                     "k_step_launches": len(ks), "kernels": len(seg)})
    gens = gens[-last:]
    tot = {k: sum(g[k] for g in gens) for k in ("wall_ms", "busy_ms", "k_step_ms")}
    out = {"generations": len(gens), "per_generation": gens, "total": tot,
           "wall_over_busy": tot["wall_ms"] / tot["busy_ms"], "wall_over_k_step": tot["wall_ms"] / tot["k_step_ms"],
           "mean_wall_ms": tot["wall_ms"] / len(gens), "mean_busy_ms": tot["busy_ms"] / len(gens)}
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
