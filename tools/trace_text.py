#!/usr/bin/env python3
"""Encode calls of a Zipf text batch for a rocprofv3 kernel trace, separated by
idle gaps so tools/call_timeline.py can split them.
usage: python tools/trace_text.py [MB] [block_MiB] [calls] [options]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402
from bmh import synth  # noqa: E402

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 100
bs = (int(sys.argv[2]) if len(sys.argv) > 2 else 1) << 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n = mb * 1000 * 1000
ctx = bmh.Context(0)
ctx.set_options(sys.argv[4] if len(sys.argv) > 4 else "")
nb = (n + bs - 1) // bs
offs = np.minimum(np.arange(nb + 1, dtype=np.uint64) * np.uint64(bs), np.uint64(n))
d_in = ctx.alloc(n)
d_in.upload(synth.zipf_text(n))
cap = sum(int(bmh.lib().bmh_record_bound(int(offs[i + 1] - offs[i]))) for i in range(nb))
d_out = ctx.alloc(cap)
ts = []
for _ in range(calls):
    time.sleep(0.05)
    t0 = time.perf_counter()
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    ts.append((time.perf_counter() - t0) * 1e3)
print("host ms per call:", " ".join(f"{t:.3f}" for t in ts))
