#!/usr/bin/env python3
"""Per-phase / per-round breakdown of the LAST encode call in a rocprofv3 --kernel-trace run
(calls are separated by > 1 ms of GPU idle): kernel time, idle gaps, and the doubling rounds
(each starts at a k_classify launch). usage: python tools/round_trace.py <dir> [--all]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
ks = []
for r in rows:
    m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:24]))
ks.sort()
calls = [[ks[0]]]
for k in ks[1:]:
    if k[0] - max(x[1] for x in calls[-1]) > 1_000_000:
        calls.append([k])
    else:
        calls[-1].append(k)
c = calls[-1]
t0, t1 = c[0][0], max(x[1] for x in c)
busy, s, e = 0, c[0][0], c[0][1]
for a, b, _ in c[1:]:
    if a > e:
        busy += e - s
        s, e = a, b
    else:
        e = max(e, b)
busy += e - s
print(f"call: {len(c)} kernels, span {(t1 - t0) / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us, "
      f"idle {(t1 - t0 - busy) / 1e3:.1f} us")
# phases: everything before the first k_classify = data phase; rounds start at each k_classify
marks = [i for i, k in enumerate(c) if k[2] == "k_classify"]
segs = []
if marks:
    segs.append(("data+fill", 0, marks[0]))
    for j, i in enumerate(marks):
        nxt = marks[j + 1] if j + 1 < len(marks) else None
        if nxt is None:  # the last round ends at the first kernel after the doubling phase
            nxt = next((q for q in range(i, len(c)) if c[q][2].startswith("k_mtf")), len(c))
        segs.append((f"round {j}", i, nxt))
    segs.append(("mtf+huffman+pack", segs[-1][2], len(c)))
else:
    segs.append(("all", 0, len(c)))
for name, i, j in segs:
    if i >= j:
        continue
    ks_ = c[i:j]
    span = (max(x[1] for x in ks_) - ks_[0][0]) / 1e3
    kt = sum(b - a for a, b, _ in ks_) / 1e3
    top = {}
    for a, b, n in ks_:
        top[n] = top.get(n, 0) + (b - a) / 1e3
    tops = ", ".join(f"{n} {v:.0f}" for n, v in sorted(top.items(), key=lambda kv: -kv[1])[:4])
    print(f"{name:18s} launches {len(ks_):4d} span {span:8.1f} us  kernel {kt:8.1f} us  [{tops}]")
