#!/usr/bin/env python3
"""Per-kernel L2 summary of tools/text_tcc.sh: hit rate, read requests (64 B; 32-B requests
counted half) and DRAM reads per call, for the config-3 text encode (5 calls under the profiler:
the warm-up, 3 timed, 1 kernel-timing call)."""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
calls = 5
rows = []
for k, c in acc.items():
    hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    rd = c.get("TCC_EA0_RDREQ_sum", 0)
    r32 = c.get("TCC_EA0_RDREQ_32B_sum", 0)
    rd_bytes = (rd - r32) * 64 + r32 * 32  # gfx950: FETCH_SIZE-style tally
    rows.append((rd_bytes, k, hit, miss, c.get("TCC_EA0_RDREQ_DRAM_sum", 0), c.get("TCC_EA0_WRREQ_sum", 0)))
print(f"{'kernel':28s} {'L2 hit':>7s} {'reqs/call (M)':>13s} {'EA read GB/call':>15s} {'DRAM rd req/call (M)':>21s} {'EA wr req/call (M)':>19s}")
for rd_bytes, k, hit, miss, dram, wr in sorted(rows, reverse=True)[:25]:
    tot = hit + miss
    print(f"{k:28s} {hit / tot if tot else 0:7.3f} {tot / calls / 1e6:13.2f} {rd_bytes / calls / 1e9:15.3f} {dram / calls / 1e6:21.2f} {wr / calls / 1e6:19.2f}")
