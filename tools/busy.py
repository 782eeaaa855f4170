#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 --kernel-trace run of bench.py: the union of kernel
intervals over the timed steps (2 sub-batches per step, so 2 `k_g1_hist` launches per step;
steps counted from the first encode, skipping `warmup`), and the largest idle gaps inside.
usage: python tools/busy.py <rocprof_out_dir> [steps] [warmup] [subbatches]"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


d = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 2
sub = int(sys.argv[4]) if len(sys.argv) > 4 else 2
ks = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
ks.sort()
starts = [i for i, k in enumerate(ks) if k[2] == "k_g1_hist"]
steps = starts[::sub]
if len(steps) < warm + nsteps + 1:
    sys.exit("not enough steps in the trace")
lo, hi = steps[warm], steps[warm + nsteps]
win = ks[lo:hi]
t0, t1 = win[0][0], max(e for _, e, _ in win)
busy, cur_s, cur_e, gaps = 0, win[0][0], win[0][1], []
for s, e, n in win[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print(f"{nsteps} steps: span {span / 1e6 / nsteps:.3f} ms/step, busy {busy / span * 100:.1f} %, "
      f"idle {(span - busy) / 1e6 / nsteps:.3f} ms/step in {len(gaps)} gaps")
for g, n in sorted(gaps, reverse=True)[:12]:
    print(f"  gap {g / 1e3:8.1f} us before {n}")
