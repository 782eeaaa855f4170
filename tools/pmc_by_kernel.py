#!/usr/bin/env python3
"""Sum rocprofv3 PMC counters per kernel from one or more run_counter_collection.csv files
(diagnostics). usage: python tools/pmc_by_kernel.py file.csv [...]; prints counters and, when
present, the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS) (MI355X_MICROARCH.md)."""
import collections
import csv
import re
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        m = re.search(r"k_(\w+?)(<[^>]*>)?\(", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:30]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -sum(kv[1].values())):
    s = "  ".join(f"{n} {v:.3g}" for n, v in sorted(c.items()))
    h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        s += f"  L2hit {h / (h + m):.3f}"
    print(f"{k:28s} {s}")
