#!/usr/bin/env python3
"""Aggregate rocprofv3 CSV outputs (kernel stats, PMC passes) per kernel name.

usage: python tools/prof_summary.py <pmc_dir> [--steps K]
Prints per kernel: calls, avg duration, and each counter summed over dispatches / per call.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"::(k_[A-Za-z0-9_]+)", name) or re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    d = sys.argv[1]
    counters = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(int)
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            counters[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (k, r.get("Dispatch_Id"))
            if key not in seen and "p1" in f.split(os.sep)[-4:-1][0] if False else False:
                pass
    for f in glob.glob(os.path.join(d, "p1", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            calls[k] += 1
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    names = sorted(counters, key=lambda k: -dur.get(k, 0))
    for k in names:
        c = counters[k]
        n = max(1, calls.get(k, 1))
        line = f"{k:22s} calls={calls.get(k,0):4d} ms/call={dur.get(k,0)/n:8.3f}"
        fs = c.get("FETCH_SIZE", 0) / n
        ws = c.get("WRITE_SIZE", 0) / n
        if fs or ws:
            line += f" FETCH(x2)={2*fs/1e6:8.1f}MB WRITE={ws/1e6:8.1f}MB"
        print(line)
        for cn in sorted(c):
            if cn in ("FETCH_SIZE", "WRITE_SIZE"):
                continue
            print(f"    {cn:28s} {c[cn]/n:16.0f}")


if __name__ == "__main__":
    main()
