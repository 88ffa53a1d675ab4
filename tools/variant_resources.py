#!/usr/bin/env python3
"""Registers / scratch of the c3 step kernel (k_step<double,0,0,true,2,...>) built from a patched copy
of csrc/ (tools/experiments/*.patch), as tools/resource_usage.py reports the product's:
  python tools/variant_resources.py tools/experiments/<name>.patch"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "psso-sac-for-powered-descent_amd"))
from pdenv import build as b  # noqa: E402

with tempfile.TemporaryDirectory() as td:
    shutil.copytree(os.path.join(REPO, "psso-sac-for-powered-descent_amd", "csrc"), os.path.join(td, "p", "csrc"))
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(td, "include"))
    if len(sys.argv) > 1:
        subprocess.run(["patch", "-s", "-t", "-p2", "-d", os.path.join(td, "p", "csrc"), "-i", os.path.abspath(sys.argv[1])],
                       check=True)
    cmd = [b.HIPCC] + b.FLAGS + ["-DPD_KR=0", "-DPD_KPH=0", "-DPD_KW=1", "-c", "-o", os.devnull,
                                 os.path.join(td, "p", "csrc", "kstep.hip"), "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    lines = r.stderr.splitlines()
    for i, l in enumerate(lines):
        if re.search(r"Function Name: _ZN2pd6k_stepIdLi0ELi0ELb1ELi2ELi0ELb0ELb[01]ELb0E", l):
            print(l.split("remark: ")[-1])
            for x in lines[i + 1:i + 11]:
                print("   ", x.split("remark: ")[-1].replace(" [-Rpass-analysis=kernel-resource-usage]", ""))
