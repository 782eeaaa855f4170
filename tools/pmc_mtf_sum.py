#!/usr/bin/env python3
"""Summary of tools/pmc_mtf.sh: per kernel, each counter averaged over its dispatches in its own
pass (no double counting across passes), cycle shares of SQ_WAVE_CYCLES (quad-cycles), LDS array
busy share, and the effective shader clock GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH
'DVFS give-back').  usage: tools/pmc_mtf_sum.py <dir> [kernel-substring ...]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
want = sys.argv[2:] or ["k_mtf_encode", "k_g1_scatter", "k_finish_dense", "k_pack_write"]
out = {}
for p in sorted(glob.glob(os.path.join(d, "p*"))):
    if not os.path.isdir(p):
        continue
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(dict)
    for f in glob.glob(f"{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            vals[k][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    for f in glob.glob(f"{p}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            durs[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    for k, cs in vals.items():
        if not any(w in k for w in want):
            continue
        e = out.setdefault(k, {})
        for cn, lst in cs.items():
            per = defaultdict(float)
            for di, v in lst:
                per[di] += v
            e[cn] = sum(per.values()) / len(per)
            if cn == "GRBM_GUI_ACTIVE":
                ds = [durs[k][di] for di in per if di in durs[k]]
                if ds:
                    e["clock_GHz"] = round(sum(per.values()) / 8 / sum(ds) / 1e9, 3)
                    e["kernel_ms_in_clock_pass"] = round(1e3 * sum(ds) / len(ds), 4)
for k, e in out.items():
    wc = e.get("SQ_WAVE_CYCLES") or 0
    if wc:
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                   "SQ_WAIT_INST_LDS"):
            if cn in e:
                e[cn + "_share"] = round(e[cn] / wc, 4)
    if e.get("SQ_WAVES"):
        e["valu_per_wave"] = round(e.get("SQ_INSTS_VALU", 0) / e["SQ_WAVES"], 1)
        e["lds_per_wave"] = round(e.get("SQ_INSTS_LDS", 0) / e["SQ_WAVES"], 1)
    if e.get("SQ_LDS_IDX_ACTIVE") and e.get("SQ_BUSY_CYCLES"):
        e["lds_idx_active_per_busy_cycle"] = round(e["SQ_LDS_IDX_ACTIVE"] / e["SQ_BUSY_CYCLES"], 4)
print(json.dumps(out, indent=1))
