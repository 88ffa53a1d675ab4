#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of a GPU session (tools/gpu_session.sh, under gpurun_out/) into
profiles/ and reduce the PMC passes to per-launch figures for k_step.

  FETCH_SIZE, WRITE_SIZE: KiB per dispatch (rocprofv3 derived counters).  Per
  /opt/skills/guides/MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports half the bytes of
  wide coalesced reads on gfx950, so traffic = 2 * FETCH_SIZE + WRITE_SIZE (x 1024 B).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def per_launch(path, kernel="k_step"):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}, {k: len(v) for k, v in d.items()}


def kernel_avg_ns(stats_csv, kernel="k_step"):
    for r in csv.DictReader(open(stats_csv)):
        if kernel in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def main(tag="r01"):
    os.makedirs(PROF, exist_ok=True)
    # merge into the existing summary: a session that ran only some stages keeps the others
    prev = os.path.join(PROF, "pmc_traffic.json")
    summary = json.load(open(prev)) if os.path.exists(prev) else {}
    summary["source"] = ("tools/gpu_session.sh stages prof/prof32/pmc/pmc32/pmcv on one MI355X; "
                         "workload = bench.py defaults (c3, 65536 envs, 16 env-steps per k_step launch)")
    summary["env_steps_per_launch"] = int(os.environ.get("FUSE", "16"))
    for prec, d in (("f64", "prof"), ("f32", "prof32")):
        src = os.path.join(OUT, d, "run_kernel_stats.csv")
        if os.path.exists(src):
            rows = list(csv.DictReader(open(src)))
            with open(os.path.join(PROF, f"{tag}_kernel_stats_{prec}.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=rows[0].keys())
                w.writeheader()
                for r in rows:
                    if len(r["Name"]) > 160:
                        r["Name"] = r["Name"][:157] + "..."
                    w.writerow(r)
            avg, calls = kernel_avg_ns(src)
            summary[f"{prec}_k_step_avg_ns"] = avg
            summary[f"{prec}_k_step_calls"] = calls
    for prec, suf in (("f64", ""), ("f32", "32")):
        fp = os.path.join(OUT, f"pmc_fetch{suf}", "run_counter_collection.csv")
        wp = os.path.join(OUT, f"pmc_write{suf}", "run_counter_collection.csv")
        if os.path.exists(fp) and os.path.exists(wp):
            fetch, nf = per_launch(fp)
            write, nw = per_launch(wp)
            fk, wk = fetch["FETCH_SIZE"], write["WRITE_SIZE"]
            summary[f"{prec}_fetch_kib_per_launch"] = fk
            summary[f"{prec}_write_kib_per_launch"] = wk
            summary[f"{prec}_launches_averaged"] = nf["FETCH_SIZE"]
            summary[f"{prec}_bytes_per_launch"] = (2 * fk + wk) * 1024.0
    vp = os.path.join(OUT, "pmc_valu", "run_counter_collection.csv")
    if os.path.exists(vp):
        v, n = per_launch(vp)
        summary["f64_pmc_per_launch"] = v
    # instruction mix of k_step (stage pmcmix: two passes, <= 8 SQ counters each)
    mix = {}
    for d in ("pmc_mix", "pmc_mix2"):
        p = os.path.join(OUT, d, "run_counter_collection.csv")
        if os.path.exists(p):
            mix.update(per_launch(p)[0])
    if mix:
        summary["f64_valu_mix_per_launch"] = mix
    for extra in ("pmc_f64ops",):
        p = os.path.join(OUT, extra, "run_counter_collection.csv")
        if os.path.exists(p):
            summary[f"{extra}_per_launch"] = per_launch(p)[0]
    json.dump(summary, open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=1)
    for name in ("bench.log", "bench32.log"):
        p = os.path.join(OUT, name)
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                open(os.path.join(PROF, f"{tag}_{name.replace('.log', '.json')}"), "w").write(lines[-1])
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
