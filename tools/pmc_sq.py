#!/usr/bin/env python3
"""Per-kernel SQ counter summary from rocprofv3 PMC passes (tools/pmc_run.sh output): where the
wave cycles go (parked on waitcnt/barrier, issue-stalled, issuing), instruction mix per wave
and LDS bank-conflict share. SQ_* cycle counters count quad-cycles (MI355X_MICROARCH.md).
usage: python tools/pmc_sq.py <pmc_dir> [kernel-filter]"""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>]*>)?", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if flt and flt not in k:
        continue
    wc = c.get("SQ_WAVE_CYCLES", 0)
    waves = c.get("SQ_WAVES", 0) or 1
    if wc == 0:
        continue
    pct = lambda x: f"{100 * c.get(x, 0) / wc:5.1f}%"
    lds = c.get("SQ_ACTIVE_INST_LDS", 0) or 1
    print(f"{k:30s} waves {waves:10.0f}  wait {pct('SQ_WAIT_ANY')} stall {pct('SQ_WAIT_INST_ANY')} "
          f"active {pct('SQ_ACTIVE_INST_ANY')} (valu {pct('SQ_ACTIVE_INST_VALU')} lds {pct('SQ_ACTIVE_INST_LDS')} "
          f"vmem {pct('SQ_ACTIVE_INST_VMEM')})  per wave: valu {c.get('SQ_INSTS_VALU', 0) / waves:7.0f} "
          f"lds {c.get('SQ_INSTS_LDS', 0) / waves:6.0f} vmem_rd {c.get('SQ_INSTS_VMEM_RD', 0) / waves:5.0f} "
          f"vmem_wr {c.get('SQ_INSTS_VMEM_WR', 0) / waves:5.0f}  bank-conflict/lds-active "
          f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:5.2f}")
