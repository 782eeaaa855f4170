#!/usr/bin/env python3
"""Kernel / host-wall breakdown of the Calgary encode (BASELINE configs 1-2) on one GPU:
python tools/calgary_prof.py [--mode whole|256k] [--steps 5] [--opts name=value,...]. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

CAL = ["bib", "book1", "book2", "geo", "news", "obj1", "obj2", "paper1", "paper2", "pic", "progc", "progl",
       "progp", "trans"]
ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="whole", choices=["whole", "256k", "each"])
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--opts", default="", help="bmh_ctx_set_option list name=value,...")
a = ap.parse_args()
datas = [open(os.path.join(REPO, "tests", "golden", "calgary", f), "rb").read() for f in CAL]
ctx = bmh.Context(0)
ctx.set_options(a.opts)


def run(blocks, steps):
    arr = np.frombuffer(b"".join(blocks), np.uint8)
    offs = np.cumsum([0] + [len(b) for b in blocks]).astype(np.uint64)
    d_in = ctx.alloc(arr.size)
    d_in.upload(arr)
    cap = sum(int(bmh.lib().bmh_record_bound(len(b))) for b in blocks)
    d_out = ctx.alloc(cap)
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    dt = (time.perf_counter() - t0) / steps
    ctx.reset_stats()
    ctx.set_timing(True)
    for _ in range(steps):
        ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    st = ctx.kernel_stats()
    ctx.set_timing(False)
    d_in.free()
    d_out.free()
    return dt, {k: (v[0] / steps, round(v[1] / steps, 3)) for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])}


if a.mode == "each":
    out = {}
    for f, d in zip(CAL, datas):
        dt, st = run([d], a.steps)
        out[f] = {"ms": round(dt * 1e3, 3), "top": dict(list(st.items())[:6])}
    print(json.dumps(out))
else:
    blocks = datas if a.mode == "whole" else [d[i:i + (1 << 18)] for d in datas for i in range(0, len(d), 1 << 18)]
    dt, st = run(blocks, a.steps)
    print(json.dumps({"mode": a.mode, "ms": round(dt * 1e3, 3), "kernels": st}))
