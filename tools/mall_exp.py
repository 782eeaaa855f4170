#!/usr/bin/env python3
"""Experiment: per-byte kernel time of the encode stages vs batch size (4 MiB random blocks).
Small batches keep the 8-byte rotation records (32 MiB per block) inside the 256 MiB
Infinity Cache between the global pass and the dense finish; large ones do not.
usage: python tools/mall_exp.py [nblocks ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
os.environ["BMH_STREAMS"] = "1"
import bmh  # noqa: E402

bs = 4 << 20
sizes = [int(x) for x in sys.argv[1:]] or [2, 4, 6, 8, 16, 64, 256]
ctx = bmh.Context(0)
for nb in sizes:
    d = ctx.alloc(bs * nb)
    for i in range(nb):
        ctx.synth_splitmix64(d.ptr.value + i * bs, bs, 0, i * bs)
    offs = np.arange(nb + 1, dtype=np.uint64) * np.uint64(bs)
    cap = nb * int(bmh.lib().bmh_record_bound(bs))
    out = ctx.alloc(cap)
    reps = max(1, 64 // nb)
    for _ in range(2):
        ctx.encode_blocks_dev(d, offs, out, cap)
    ctx.reset_stats()
    ctx.set_timing(True)
    for _ in range(reps):
        ctx.encode_blocks_dev(d, offs, out, cap)
    st = ctx.kernel_stats()
    ctx.set_timing(False)
    gib = nb * bs * reps / 2**30
    row = {k: round(v[1] / gib, 3) for k, v in st.items() if not k.startswith("wall")}
    top = dict(sorted(row.items(), key=lambda kv: -kv[1])[:8])
    print(f"nb={nb:4d} ms/GiB: {top}", flush=True)
    del d, out
