#!/usr/bin/env python3
"""Summary of tools/ctx_pmc.sh: dispatches split into contexts at idle gaps > 100 ms; per context,
for the big kernels, the mean duration (kernel trace) and the mean of each PMC counter.
usage: python tools/ctx_pmc_sum.py DIR [DIR ...]   (each a rocprofv3 -d directory)"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

KERNELS = ["k_g1_scatter", "k_finish_dense", "k_mtf_encode", "k_g1_hist", "k_pack_write", "k_mtf_recency"]


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:30]


for d in sys.argv[1:]:
    disp = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            disp[r["Dispatch_Id"]] = [short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), {}]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            x = disp.setdefault(r["Dispatch_Id"], [short(r["Kernel_Name"]), int(r.get("Start_Timestamp", 0) or 0),
                                                  int(r.get("End_Timestamp", 0) or 0), {}])
            x[3][r["Counter_Name"]] = float(r["Counter_Value"])
    ds = sorted(disp.values(), key=lambda x: x[1])
    ctxs, last = [], None
    for x in ds:
        if last is None or x[1] - last > 100_000_000:
            ctxs.append([])
        ctxs[-1].append(x)
        last = max(last or 0, x[2])
    print(f"== {d}: {len(ds)} dispatches, {len(ctxs)} groups")
    for ci, c in enumerate(ctxs):
        by = defaultdict(list)
        for x in c:
            by[x[0]].append(x)
        parts = []
        for k in KERNELS:
            xs = by.get(k)
            if not xs or len(xs) < 3:
                continue
            xs = xs[1:]  # first (warm-up) step dropped
            dur = sum(x[2] - x[1] for x in xs) / len(xs) / 1e6
            cn = defaultdict(float)
            for x in xs:
                for a, v in x[3].items():
                    cn[a] += v / len(xs)
            mhz = f" clock={cn['GRBM_GUI_ACTIVE'] / 8 / (dur * 1e-3) / 1e6:.0f}MHz" if "GRBM_GUI_ACTIVE" in cn else ""
            parts.append(f"{k[2:]} {dur:.3f}ms{mhz} " + " ".join(f"{a.replace('_sum', '')}={v:.3g}" for a, v in sorted(cn.items())))
        if parts:
            print(f" group {ci}: " + " | ".join(parts))
