#!/usr/bin/env python3
"""Registers, scratch and LDS of every step-kernel instantiation, from the compiler
(hipcc -Rpass-analysis=kernel-resource-usage on each kstep translation unit of pdenv/build.py).
  python tools/resource_usage.py [out.txt]
Prints one row per kernel: precision, phase family, rtd, wind, lanes per env, policy, RK4,
counting, SAC; VGPRs, spilled VGPRs, scratch bytes per lane, LDS bytes, waves per SIMD."""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
from pdenv import build as b  # noqa: E402

FIELDS = {"VGPRs": "vgpr", "VGPRs Spill": "vgpr_spill", "ScratchSize [bytes/lane]": "scratch",
          "LDS Size [bytes/block]": "lds", "Occupancy [waves/SIMD]": "waves"}


def unit_report(job):
    obj, src, defs = job
    cmd = [b.HIPCC] + b.FLAGS + defs + ["-c", "-o", os.devnull, src, "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +([A-Za-z \[\]/]+): (\d+)", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[FIELDS[m.group(1).strip()]] = int(m.group(2))
    return rows


def decode(name):
    m = re.match(r"_ZN2pd6k_stepI([df])Li(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELi(\d+)ELb(\d)ELb(\d)ELb(\d)E", name)
    if not m:
        return None
    r, ph, rt, w, lpe, pol, rk, cnt, sac = m.groups()
    return (("f64" if r == "d" else "f32"), int(ph), int(rt), int(w), int(lpe), int(pol), int(rk), int(cnt), int(sac))


def main():
    jobs = [u for u in b.units() if "kstep" in u[0]]
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        allrows = [r for rows in ex.map(unit_report, jobs) for r in rows]
    out = ["prec phase rtd wind lpe pol rk4 cnt sac | vgpr spill scratch lds waves"]
    seen = set()
    for r in sorted(allrows, key=lambda r: decode(r["name"]) or ()):
        k = decode(r["name"])
        if k is None or k in seen:
            continue
        seen.add(k)
        out.append(" ".join(str(v) for v in k) + f" | {r.get('vgpr')} {r.get('vgpr_spill')} {r.get('scratch')} "
                   f"{r.get('lds')} {r.get('waves')}")
    txt = "\n".join(out)
    print(txt)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
