#!/usr/bin/env python3
"""Run bench.py in this process after choosing how the host waits for the GPU.

    python tools/spin_probe.py --spin 0|1 -- <bench.py arguments>

--spin 1 calls hipSetDeviceFlags(hipDeviceScheduleSpin) on the HIP runtime torch loaded, before
anything touches the device: torch.cuda.synchronize() then polls the completion signal instead
of sleeping on it.  Used to attribute the driver window's launch/sync gap."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

argv = sys.argv[1:]
spin = 0
if argv[:1] == ["--spin"]:
    spin = int(argv[1])
    argv = argv[2:]
if argv[:1] == ["--"]:
    argv = argv[1:]

import torch  # noqa: E402,F401

if spin:
    hip = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                hip = line.split()[-1]
                break
    lib = ctypes.CDLL(hip or "libamdhip64.so")
    rc = lib.hipSetDeviceFlags(ctypes.c_uint(1))      # hipDeviceScheduleSpin
    print(f"spin_probe: hipSetDeviceFlags(spin) = {rc} ({hip})", file=sys.stderr, flush=True)

import bench  # noqa: E402

sys.argv = ["bench.py"] + argv
bench.main()
