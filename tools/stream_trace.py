#!/usr/bin/env python3
"""Per-stream view of the LAST of the encode calls in a rocprofv3 --kernel-trace run of
tools/cal_trace_run.py (calls = the N equal calls the script makes; default 3): per stream its
first / last kernel, busy time, launches and top kernels, so the critical pipeline shows.
usage: python tools/stream_trace.py <trace dir> [ncalls]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
ks = []
for r in rows:
    m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:24],
               int(r["Stream_Id"]), int(r["Thread_Id"])))
ks.sort()
# calls: split at the ncalls-1 largest gaps between consecutive kernel starts (after the upload)
gaps = sorted(range(1, len(ks)), key=lambda i: ks[i][0] - max(k[1] for k in ks[max(0, i - 64):i]))[-(ncalls - 1):]
start = max(gaps) if gaps else 0
c = ks[start:]
t0, t1 = c[0][0], max(k[1] for k in c)
print(f"last call: {len(c)} kernels, span {(t1 - t0) / 1e3:.1f} us")
by = {}
for k in c:
    by.setdefault(k[3], []).append(k)
for sid, kk in sorted(by.items()):
    busy = sum(b - a for a, b, *_ in kk) / 1e3
    top = {}
    for a, b, n, *_ in kk:
        top[n] = top.get(n, 0) + (b - a) / 1e3
    tops = ", ".join(f"{n} {v:.0f}" for n, v in sorted(top.items(), key=lambda kv: -kv[1])[:5])
    print(f"stream {sid}: {len(kk):4d} launches, {(kk[0][0] - t0) / 1e3:7.1f} .. {(max(k[1] for k in kk) - t0) / 1e3:7.1f} us, "
          f"busy {busy:7.1f} us  [{tops}]")

# union of busy intervals (any stream) and the idle gaps inside the call
iv = sorted((a, b) for a, b, *_ in c)
busy, cur_a, cur_b, gaps = 0, iv[0][0], iv[0][1], []
for a, b in iv[1:]:
    if a > cur_b:
        busy += cur_b - cur_a
        gaps.append((cur_b - t0, a - cur_b))
        cur_a, cur_b = a, b
    else:
        cur_b = max(cur_b, b)
busy += cur_b - cur_a
print(f"device busy (union) {busy / 1e3:.1f} us of {(t1 - t0) / 1e3:.1f}; idle gaps > 5 us: " +
      ", ".join(f"@{g0 / 1e3:.0f}+{g / 1e3:.0f}" for g0, g in gaps if g > 5000))
