#!/usr/bin/env python3
"""Per-launch durations of the BWT list kernels from a rocprofv3 kernel trace, in launch order
(diagnostics). usage: python tools/launch_times.py <run_kernel_trace.csv>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    m = re.search(r"k_(\w+?)(<[^>]*>)?\(", n)
    nm = (m.group(1) + (m.group(2) or "")) if m else n[:30]
    if any(x in nm for x in ["finish", "dcp", "dhist", "dscatter", "dscan", "dcopy", "dtiles", "g1_"]):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{nm:28s} {d:8.1f} us grid {r.get('Grid_Size', '')} wg {r.get('Workgroup_Size', '')}")
