#!/usr/bin/env python3
"""Per-step wall times of the bench workload (1 GiB random, 4 MiB blocks) over many steps,
to expose warm-up / power-state effects. usage: python tools/step_times.py [steps] [options]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ctx = bmh.Context(0)
ctx.set_options(sys.argv[2] if len(sys.argv) > 2 else "")
bs, nblk = 4 << 20, 256
offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
d_in = ctx.alloc(bs * nblk)
for i in range(nblk):
    ctx.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, i * bs)
cap = nblk * int(bmh.lib().bmh_record_bound(bs))
d_out = ctx.alloc(cap)
ts = []
for s in range(steps):
    t0 = time.perf_counter()
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    ts.append((time.perf_counter() - t0) * 1e3)
print(" ".join(f"{t:.1f}" for t in ts))
