#!/usr/bin/env python3
"""Copy a round-3 measurement session (tools/r03_final.sh, under gpurun_out/) into profiles/:
the bench lines, the rocprofv3 kernel-stats summaries, the line-vs-trace checks
(tools/prof_check.py), the c4 per-generation breakdown (tools/trace_gens.py), and the PMC passes
(tools/pmc_r03b.sh) reduced to per-launch figures of the timed k_step launches:

  FETCH_SIZE, WRITE_SIZE: KiB per dispatch.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM
  section) FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950, so
  traffic = (2 FETCH_SIZE + WRITE_SIZE) x 1024 B.

profiles/pmc_traffic.json (c3) and profiles/pmc_c3_descent.json are what bench.py reads for the
line's roofline.traffic and valu_roofline."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")
TAG = sys.argv[1] if len(sys.argv) > 1 else "r03"
LAUNCHES = int(os.environ.get("LAUNCHES", "3"))
FUSE = int(os.environ.get("FUSE", "128"))


def timed_dispatch_means(path):
    """Counter means over the last LAUNCHES k_step<double> dispatches (time_fused's timed ones)."""
    per = {}
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("void pd::k_step<double,"):
            continue
        per.setdefault(int(r["Dispatch_Id"]), {}).setdefault(r["Counter_Name"], 0.0)
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(per)[-LAUNCHES:]
    keys = per[ids[0]].keys()
    return {k: sum(per[i][k] for i in ids) / len(ids) for k in keys}, len(ids)


def pmc_summary(wl):
    d = {}
    for p in (1, 2, 3, 4):
        f = os.path.join(OUT, f"pmcF_{wl}_p{p}", "run_counter_collection.csv")
        if os.path.exists(f):
            m, n = timed_dispatch_means(f)
            d.update(m)
            d["launches_averaged"] = n
    if not d:
        return None
    s = {"env_steps_per_launch": FUSE, "source": f"tools/pmc_r03b.sh (rocprofv3 --pmc, one counter set per run) over "
                                              f"tools/time_fused.py {'DESCENT=1 ' if wl == 'desc' else ''}FUSE={FUSE}; means "
                                              f"of the {d.get('launches_averaged')} timed k_step launches"}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        s["f64_fetch_kib_per_launch"] = d["FETCH_SIZE"]
        s["f64_write_kib_per_launch"] = d["WRITE_SIZE"]
        s["f64_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
    mixk = [k for k in d if k.startswith("SQ_INSTS_VALU") or k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")]
    if mixk:
        s["f64_valu_mix_per_launch"] = {k: d[k] for k in mixk}
    st = {k: d[k] for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                            "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE") if k in d}
    if st:
        s["stall_counters_per_launch"] = st
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            s["wave_cycle_fractions"] = {"waitcnt (SQ_WAIT_ANY)": st.get("SQ_WAIT_ANY", 0) / wc,
                                         "issue stall (SQ_WAIT_INST_ANY)": st.get("SQ_WAIT_INST_ANY", 0) / wc,
                                         "issuing (SQ_ACTIVE_INST_ANY)": st.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                         "issuing VALU (SQ_ACTIVE_INST_VALU)": st.get("SQ_ACTIVE_INST_VALU", 0) / wc}
        if "SQ_LDS_IDX_ACTIVE" in st:
            s["lds_bank_conflict_share"] = st["SQ_LDS_BANK_CONFLICT"] / st["SQ_LDS_IDX_ACTIVE"]
    return s


def copy_stats(src_dir, name):
    f = os.path.join(OUT, src_dir, "run_kernel_stats.csv")
    if not os.path.exists(f):
        return
    rows = list(csv.DictReader(open(f)))
    with open(os.path.join(PROF, f"{TAG}_{name}.csv"), "w", newline="") as fo:
        w = csv.DictWriter(fo, fieldnames=rows[0].keys())
        w.writeheader()
        for r in rows:
            if len(r["Name"]) > 160:
                r["Name"] = r["Name"][:157] + "..."
            w.writerow(r)


def last_json(log):
    p = os.path.join(OUT, log)
    if not os.path.exists(p):
        return None
    lines = [l for l in open(p) if l.startswith("{")]
    return lines[-1] if lines else None


def main():
    os.makedirs(PROF, exist_ok=True)
    for log, name in (("bench.log", "bench"), ("benchdrv.log", "bench_driver_cmd"), ("prof.log", "bench_prof"),
                      ("profdrv.log", "bench_profdrv"), ("profc4.log", "bench_c4_prof"), ("profc5.log", "bench_c5_prof")):
        j = last_json(log)
        if j:
            open(os.path.join(PROF, f"{TAG}_{name}.json"), "w").write(j)
    for d, name in (("prof", "kernel_stats_f64"), ("profdrv", "kernel_stats_driver_cmd"), ("profc4", "kernel_stats_c4"),
                    ("profc5", "kernel_stats_c5")):
        copy_stats(d, name)
    for d, log, name in (("prof", "prof.log", "prof_check"), ("profdrv", "profdrv.log", "prof_check_driver_cmd")):
        tr = os.path.join(OUT, d, "run_kernel_trace.csv")
        if os.path.exists(tr) and os.path.exists(os.path.join(OUT, log)):
            subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_check.py"), tr, os.path.join(OUT, log),
                            os.path.join(PROF, f"{TAG}_{name}.json")], check=True, capture_output=True)
    tr = os.path.join(OUT, "profc4", "run_kernel_trace.csv")
    if os.path.exists(tr):
        subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_gens.py"), tr, "16",
                        os.path.join(PROF, f"{TAG}_c4_generations.json")], check=True, capture_output=True)
    for wl, name in (("c3", "pmc_traffic.json"), ("desc", "pmc_c3_descent.json")):
        s = pmc_summary(wl)
        if s:
            json.dump(s, open(os.path.join(PROF, name), "w"), indent=1)
            print(name, json.dumps({k: v for k, v in s.items() if k != "source"})[:600])


if __name__ == "__main__":
    main()
