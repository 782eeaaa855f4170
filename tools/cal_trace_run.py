#!/usr/bin/env python3
"""Encode Calgary files (default: pic) a few times for a rocprofv3 kernel trace; the last call is
the one analysed by tools/round_trace.py. usage: python tools/cal_trace_run.py [--opts k=v,..] [file ...]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

args = sys.argv[1:]
opts = args[1] if args[:1] == ["--opts"] else ""
names = (args[2:] if opts else args) or ["pic"]
datas = [open(os.path.join(REPO, "tests", "golden", "calgary", f), "rb").read() for f in names]
ctx = bmh.Context(0)
ctx.set_options(opts)
arr = np.frombuffer(b"".join(datas), np.uint8)
offs = np.cumsum([0] + [len(b) for b in datas]).astype(np.uint64)
d_in = ctx.alloc(arr.size)
d_in.upload(arr)
cap = sum(int(bmh.lib().bmh_record_bound(len(b))) for b in datas)
d_out = ctx.alloc(cap)
import time  # noqa: E402
for _ in range(3):
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)  # returns after the device finished
    time.sleep(0.05)  # > 1 ms of GPU idle between calls: tools/round_trace.py splits calls there
print("ok", names, arr.size)
