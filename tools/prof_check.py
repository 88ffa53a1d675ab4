#!/usr/bin/env python3
"""Check a bench.py line against the rocprofv3 kernel trace of the same command.

  python tools/prof_check.py <kernel_trace.csv> <bench log with the JSON line> [out.json]

bench.py numbers its k_step launches per precision in issue order and reports, for the headline
and for the nested c3-descent measurement, the index ranges of the timed launches and of their
replay (`launch_index`).  This tool takes the k_step dispatches of that precision from the trace
in dispatch order, averages the kernel durations over each range, and sets them beside the line's
own event-timed figures: the rocprof average per launch of the timed range must agree with the
line's kernel time, and the per-step kernel time must not exceed the wall time per step."""
import csv
import json
import sys


def dispatches(trace, tag):
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].startswith(f"void pd::k_step<{tag},")]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]   # ms


def check(trace, line):
    out = {}
    parts = [("headline", line)]
    if "c3_descent" in line:
        parts.append(("c3_descent", line["c3_descent"]))
    steps = line["steps"]
    for name, part in parts:
        li = part["launch_index"]
        tag = li["kernel"].split("<")[1].rstrip(">")
        d = dispatches(trace, tag)
        res = {}
        for rng in ("timed", "replay"):
            a, b = li[rng]
            sel = d[a:b]
            reps = li.get("replays", 1) if rng == "replay" else 1     # (the replay range holds every replay)
            res[rng] = {"launches": len(sel), "rocprof_total_ms": sum(sel),
                        "rocprof_ms_per_step": sum(sel) / steps / reps,
                        "rocprof_avg_ms_per_launch": sum(sel) / len(sel) if sel else None}
        rf = part["roofline"]
        res["line_kernel_ms_per_step"] = rf["kernel_ms_per_step"]
        res["line_kernel_avg_ms"] = rf["kernel_avg_ms"]
        res["line_ms_per_step"] = part["ms_per_step"]
        res["line_device_ms_per_step"] = part.get("device_ms_per_step")
        res["rocprof_timed_vs_line_kernel"] = res["timed"]["rocprof_ms_per_step"] / rf["kernel_ms_per_step"]
        res["kernel_per_step_le_wall"] = res["timed"]["rocprof_ms_per_step"] <= part["ms_per_step"] and \
            rf["kernel_ms_per_step"] <= part["ms_per_step"]
        out[name] = res
    return out


def main():
    trace, log = sys.argv[1], sys.argv[2]
    line = json.loads([l for l in open(log) if l.startswith("{")][-1])
    res = check(trace, line)
    res["source"] = {"trace": trace, "bench_log": log}
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
