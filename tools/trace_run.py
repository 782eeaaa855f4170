#!/usr/bin/env python3
"""Encode calls of the headline workload (splitmix64 bytes in HBM) for a rocprofv3 kernel trace,
separated by idle gaps so tools/stream_trace.py can split them.
usage: python tools/trace_run.py [total_MiB] [block_MiB] [calls] [options]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

total = (int(sys.argv[1]) if len(sys.argv) > 1 else 128) << 20
bs = (int(sys.argv[2]) if len(sys.argv) > 2 else 4) << 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ctx = bmh.Context(0)
ctx.set_options(sys.argv[4] if len(sys.argv) > 4 else "")
nblk = total // bs
offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
d_in = ctx.alloc(total)
for i in range(nblk):
    ctx.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, i * bs)
cap = nblk * int(bmh.lib().bmh_record_bound(bs))
d_out = ctx.alloc(cap)
ts = []
for _ in range(calls):
    time.sleep(0.05)
    t0 = time.perf_counter()
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    ts.append((time.perf_counter() - t0) * 1e3)
print("host ms per call:", " ".join(f"{t:.3f}" for t in ts))
