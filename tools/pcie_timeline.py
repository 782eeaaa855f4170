#!/usr/bin/env python3
"""Streamed host-buffer encode timeline from a rocprofv3 --kernel-trace --memory-copy-trace run:
per batch, the H2D / D2H copies (> 1 MiB-ish: > 0.2 ms) and each encode's first global-pass
histogram to its last pack kernel. usage: python tools/pcie_timeline.py <rocprof_out_dir> [last_ms]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
ks, mc = [], []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e - s > 200000:
            mc.append((s, e, "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H"))
ks.sort()
mc.sort()
# the pcie section: the last g1_hist launches within last_ms of the end of the last pack_write
end = max(e for s, e, n in ks if n == "k_pack_write")
t0 = end - last_ms * 1e6
ev = [(s, e, "H2D/D2H " + n) for s, e, n in mc if s >= t0 and n == "H2D"]
ev += [(s, e, "D2H") for s, e, n in mc if s >= t0 and n == "D2H"]
hist = [s for s, e, n in ks if n == "k_g1_hist" and s >= t0]
packs = [e for s, e, n in ks if n == "k_pack_write" and s >= t0]
for s in hist:
    ev.append((s, s, "encode start (g1_hist)"))
for e in packs:
    ev.append((e, e, "pack_write end"))
ev.sort()
base = ev[0][0]
for s, e, n in ev:
    print(f"{(s - base) / 1e6:9.3f} {(e - s) / 1e6:7.3f} {n}")
