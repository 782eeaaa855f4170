#!/usr/bin/env python3
"""Wall time of one batched encode of a subset of the Calgary files (median of 7 after warmup):
python tools/cal_subset_time.py [--streams S] file ... ; prints ms and MB/s."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("files", nargs="+")
a = ap.parse_args()
datas = [open(os.path.join(REPO, "tests", "golden", "calgary", f), "rb").read() for f in a.files]
ctx = bmh.Context(0)
arr = np.frombuffer(b"".join(datas), np.uint8)
offs = np.cumsum([0] + [len(b) for b in datas]).astype(np.uint64)
d_in = ctx.alloc(arr.size)
d_in.upload(arr)
cap = sum(int(bmh.lib().bmh_record_bound(len(b))) for b in datas)
d_out = ctx.alloc(cap)
ts = []
for i in range(9):
    ctx.sync()
    t0 = time.perf_counter()
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    ctx.sync()
    ts.append(time.perf_counter() - t0)
ms = float(np.median(ts[2:])) * 1e3
print(f"{' '.join(a.files)[:60]:60s} {ms:8.3f} ms {arr.size / ms / 1e3:8.1f} MB/s")
