#!/usr/bin/env python3
"""Per-dispatch durations from a rocprofv3 kernel trace, in launch order (short names).
usage: python tools/trace_summary.py run_kernel_trace.csv [filter]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
tot = {}
for r in rows:
    nm = r["Kernel_Name"]
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>]*>)?", nm)
    short = (m.group(1) + (m.group(2) or "")) if m else nm[:40]
    if flt and flt not in short:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[short] = tot.get(short, 0.0) + d
    print(f"{d:9.3f} ms  {short}")
print("--- totals")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.3f} ms  {k}")
