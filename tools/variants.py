#!/usr/bin/env python3
"""Build experiment variants of libpdenv (c3 step-kernel object only) in parallel:
python tools/variants.py name=-DFOO,-DBAR name2=patch:tools/experiments/no_gust.patch ...
(patch:<file> compiles a patched copy of csrc/; the product sources are never modified; the item
"host" also compiles the host unit from it, e.g.
idx2=patch:tools/experiments/two_level_index.patch,-DPD_IDX2=1,host; the item unit:R.P.W builds that
step-kernel object instead of the c3 one -- precision 0/1, phase family 0/1/2, wind 0/1 -- e.g.
pnt=patch:tools/experiments/policy_nt.patch,unit:0.1.0 for the f64 landing_burn windless (c4) unit)"""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "psso-sac-for-powered-descent_amd"))
from pdenv import build as b  # noqa: E402

if __name__ == "__main__":
    b.build(verbose=False)
    specs = [a.split("=", 1) for a in sys.argv[1:]]
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        def one(sp):
            items = [d for d in sp[1].split(",") if d]
            patch = next((d[6:] for d in items if d.startswith("patch:")), None)
            unit = next((tuple(int(x) for x in d[5:].split(".")) for d in items if d.startswith("unit:")), (0, 0, 1))
            defs = [d for d in items if not d.startswith("patch:") and not d.startswith("unit:") and d != "host"]
            return b.build_variant(sp[0], defs, unit=unit, patch=patch, host="host" in items)
        for p in ex.map(one, specs):
            print(p)
