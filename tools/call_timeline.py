#!/usr/bin/env python3
"""Timeline of the LAST encode call in a rocprofv3 --kernel-trace of tools/trace_run.py (calls are
separated by >= 10 ms of host sleep): every kernel's start offset, duration and queue, the union
busy time, and the idle gaps between kernels, so a call's serial latency shows.
usage: python tools/call_timeline.py <trace dir> [min_gap_us]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
mingap = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
ks = []
for r in rows:
    m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:28], q))
ks.sort()
# the last call: kernels after the last gap >= 10 ms
start = 0
end_max = ks[0][1]
for i in range(1, len(ks)):
    if ks[i][0] - end_max >= 10_000_000:
        start = i
    end_max = max(end_max, ks[i][1])
call = ks[start:]
t0 = call[0][0]
busy, cur_s, cur_e, gaps = 0, call[0][0], call[0][1], []
for s, e, _, _ in call[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        if (s - cur_e) / 1e3 >= mingap:
            gaps.append(((cur_e - t0) / 1e3, (s - cur_e) / 1e3))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = (max(e for _, e, _, _ in call) - t0) / 1e3
print(f"last call: {len(call)} kernels, span {span:.1f} us, union busy {busy / 1e3:.1f} us, "
      f"idle {span - busy / 1e3:.1f} us; gaps >= {mingap} us: " + ", ".join(f"@{a:.0f}+{g:.1f}" for a, g in gaps))
for s, e, n, q in call:
    print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {n}")
