#!/usr/bin/env python3
"""Per-kernel times of the GPU decode on the bench workload (1 GiB random, 4 MiB blocks)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

bs, nb = 4 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = bmh.Context(0)
offs = np.arange(nb + 1, dtype=np.uint64) * np.uint64(bs)
d_in = ctx.alloc(bs * nb)
ctx.synth_splitmix64(d_in, bs * nb, 0, 0)
cap = nb * int(bmh.lib().bmh_record_bound(bs))
d_rec = ctx.alloc(cap)
ro = ctx.encode_blocks_dev(d_in, offs, d_rec, cap)
d_dec = ctx.alloc(bs * nb)
ctx.decode_blocks_dev(d_rec, ro, d_dec, bs * nb)
ctx.reset_stats()
ctx.set_timing(True)
ctx.decode_blocks_dev(d_rec, ro, d_dec, bs * nb)
st = ctx.kernel_stats()
for k, (n, ms) in sorted(st.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:24s} {n:4d} {ms:9.3f} ms")
