#!/usr/bin/env python3
"""Timeline gaps from a rocprofv3 --kernel-trace --hip-trace run: for the last N kernels,
print every idle gap > threshold between consecutive kernels and the HIP API calls that
ran on the host during it.

usage: python tools/timeline.py <rocprof_out_dir> [--last 200] [--gap-us 200]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 200
    gap_us = float(sys.argv[sys.argv.index("--gap-us") + 1]) if "--gap-us" in sys.argv else 200
    ks = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    api = []
    for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    ks.sort()
    api.sort()
    ks = ks[-last:]
    t0 = ks[0][0]
    busy = sum(e - s for s, e, _ in ks)
    print(f"{len(ks)} kernels over {(ks[-1][1] - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms")
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        g = (s1 - e0) / 1e3
        if g > gap_us:
            calls = {}
            for a, b, fn in api:
                if b >= e0 and a <= s1:
                    calls.setdefault(fn, [0, 0.0])
                    calls[fn][0] += 1
                    calls[fn][1] += (min(b, s1) - max(a, e0)) / 1e3
            top = sorted(calls.items(), key=lambda kv: -kv[1][1])[:5]
            print(f"  +{(e0 - t0) / 1e6:8.3f} ms gap {g:9.1f} us  {n0} -> {n1}  " +
                  ", ".join(f"{fn} x{c} {us:.0f}us" for fn, (c, us) in top))


if __name__ == "__main__":
    main()
