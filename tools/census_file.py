#!/usr/bin/env python3
"""Per-round BWT list census (BMH_DBG_LISTS=1) and kernel breakdown of one file encoded as a
single block: BMH_DBG_LISTS=1 python tools/census_file.py PATH"""
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
os.environ.setdefault("BMH_STREAMS", "1")
import bmh  # noqa: E402

data = np.fromfile(sys.argv[1], np.uint8)
ctx = bmh.Context(0)
offs = np.array([0, data.size], np.uint64)
d_in = ctx.alloc(data.size)
d_in.upload(data)
cap = int(bmh.lib().bmh_record_bound(data.size))
d_out = ctx.alloc(cap)
ctx.encode_blocks_dev(d_in, offs, d_out, cap)
print("---- second run (context settled)", file=sys.stderr, flush=True)
ctx.reset_stats()
ctx.set_timing(True)
ctx.encode_blocks_dev(d_in, offs, d_out, cap)
st = ctx.kernel_stats()
print(json.dumps({k: [v[0], round(v[1], 3)] for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])}))
