#!/usr/bin/env python3
"""Per-context spread probe for PMC runs: the headline workload (1 GiB
splitmix64, 4 MiB blocks) on several contexts created one after another in ONE process, each
with fresh buffers behind a pad allocation of a different size, one pipeline (one stream, so a
kernel's duration is its own), a 0.3 s idle gap between contexts so a trace splits them.
usage: python tools/ctx_pmc.py [contexts] [steps]"""
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

nctx = int(sys.argv[1]) if len(sys.argv) > 1 else 6
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
bs, nblk = 4 << 20, 256
offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
for k in range(nctx):
    ctx = bmh.Context(0)
    ctx.set_option("pipelines", 1)
    pad = ctx.alloc((k * 37 + 1) << 20)  # shifts the following allocations
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
    print(f"ctx {k}: in 0x{d_in.ptr.value:x} out 0x{d_out.ptr.value:x} median {statistics.median(ts[1:]):.2f} ms "
          f"steps {' '.join(f'{t:.2f}' for t in ts)}", flush=True)
    d_in.free()
    d_out.free()
    pad.free()
    ctx.close()
    time.sleep(0.3)
