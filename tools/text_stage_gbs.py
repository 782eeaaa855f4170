#!/usr/bin/env python3
"""Per-stage HBM table of a text encode (VERDICT r4 item 3 / Missing 2): kernel time from a plain
rocprofv3 --kernel-trace pass, HBM bytes from FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md
HBM: 2 * FETCH_SIZE + WRITE_SIZE kilobytes), summed over all dispatches of each kernel and
divided by the number of encode calls the traced script made.
usage: python tools/text_stage_gbs.py <dir with kt/ pf/ pw/> <input bytes per call> <calls> [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def kname(s: str) -> str:
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:40]


def rows(d: str, pat: str):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    d, nbytes, calls = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ms, disp = defaultdict(float), defaultdict(int)
    for r in rows(os.path.join(d, "kt"), "*kernel_trace.csv"):
        k = kname(r["Kernel_Name"])
        ms[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        disp[k] += 1
    hbm = defaultdict(float)
    for sub, ctr, mul in (("pf", "FETCH_SIZE", 2.0), ("pw", "WRITE_SIZE", 1.0)):
        for r in rows(os.path.join(d, sub), "*counter_collection.csv"):
            if r["Counter_Name"] == ctr:
                hbm[kname(r["Kernel_Name"])] += mul * float(r["Counter_Value"]) * 1024
    tot = sum(ms.values()) / calls
    stages = []
    for k in sorted(ms, key=lambda k: -ms[k]):
        t = ms[k] / calls
        b = hbm.get(k, 0.0) / calls
        stages.append({"stage": k, "dispatches_per_call": round(disp[k] / calls, 1), "ms": round(t, 3),
                       "share": round(t / tot, 4) if tot else 0, "hbm_GB": round(b / 1e9, 3),
                       "hbm_GBps": round(b / 1e9 / (t / 1e3), 1) if t else None})
    doc = {"input_bytes_per_call": nbytes, "calls": calls, "kernel_ms_per_call": round(tot, 3),
           "hbm_GB_per_call": round(sum(s["hbm_GB"] for s in stages), 3),
           "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch (MI355X_MICROARCH.md HBM), summed / calls",
           "stages": stages}
    out = json.dumps(doc, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(out)
    for s in stages[:24]:
        print(f"{s['stage']:34s} {s['dispatches_per_call']:6.1f} x  {s['ms']:7.3f} ms  {s['share']:6.1%}  "
              f"{s['hbm_GB']:7.3f} GB  {s['hbm_GBps']} GB/s")
    print(f"total {tot:.3f} ms of kernels per call, {doc['hbm_GB_per_call']} GB")


if __name__ == "__main__":
    main()
