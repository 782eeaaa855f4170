#!/usr/bin/env python3
"""Per-round BWT list census on Zipf text (diagnostics): the check_lists option makes the library
check and print each finish round's segment lists to stderr. usage: python tools/list_census.py MB block_MiB"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402
from bmh import synth  # noqa: E402

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 100
bs = (int(sys.argv[2]) if len(sys.argv) > 2 else 1) << 20
n = mb * 1000 * 1000
z = synth.zipf_text(n)
ctx = bmh.Context(0)
ctx.set_option("pipelines", 1)
ctx.set_option("check_lists", 1)
nb = (n + bs - 1) // bs
offs = np.minimum(np.arange(nb + 1, dtype=np.uint64) * np.uint64(bs), np.uint64(n))
d_in = ctx.alloc(n)
d_in.upload(z)
cap = sum(int(bmh.lib().bmh_record_bound(int(offs[i + 1] - offs[i]))) for i in range(nb))
d_out = ctx.alloc(cap)
ctx.encode_blocks_dev(d_in, offs, d_out, cap)
