#!/usr/bin/env python3
"""Calgary batch time on a context before and after the headline legs ran on it (diagnoses
bench.py's Calgary leg being slower than tools/cal_subset_time.py):
python tools/cal_after.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

CAL = ["bib", "book1", "book2", "geo", "news", "obj1", "obj2", "paper1", "paper2", "pic", "progc", "progl",
       "progp", "trans"]
datas = [open(os.path.join(REPO, "tests", "golden", "calgary", f), "rb").read() for f in CAL]
ctx = bmh.Context(0)


def cal(tag):
    arr = np.frombuffer(b"".join(datas), np.uint8)
    offs = np.cumsum([0] + [len(b) for b in datas]).astype(np.uint64)
    d_in = ctx.alloc(arr.size)
    d_in.upload(arr)
    cap = sum(int(bmh.lib().bmh_record_bound(len(b))) for b in datas)
    d_out = ctx.alloc(cap)
    ts = []
    for _ in range(9):
        t0 = time.perf_counter()
        ctx.encode_blocks_dev(d_in, offs, d_out, cap)
        ts.append(time.perf_counter() - t0)
    d_in.free()
    d_out.free()
    print(f"{tag:28s} calgary {np.median(ts[2:]) * 1e3:7.3f} ms  min {min(ts[2:]) * 1e3:7.3f}", flush=True)


if "--fresh-first" in sys.argv:
    cal("fresh")
n = 1 << 30
d = ctx.alloc(n)
ctx.synth_splitmix64(d, n)
offs = np.arange(0, n + 1, 4 << 20, dtype=np.uint64)
cap = int(bmh.lib().bmh_record_bound(4 << 20)) * (n >> 22)
o = ctx.alloc(cap)
for _ in range(3):
    ctx.encode_blocks_dev(d, offs, o, cap)
o.free()
if "--fresh-first" in sys.argv:
    cal("after 1 GiB device encode")
h = ctx.alloc_host(n)
h.a[:] = d.download()
d.free()
hout = ctx.alloc_host(int(bmh.lib().bmh_compress_bound(n, 4 << 20)))
for _ in range(2):
    ctx.compress_into(h.a, 4 << 20, hout.a)
cal("after pinned compress_host")
h.free()
hout.free()
cal("after freeing pinned")
