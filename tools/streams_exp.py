#!/usr/bin/env python3
"""Experiment: the 1 GiB / 4 MiB-block workload split over S contexts (streams) on one GPU,
driven by S host threads, vs one context. usage: python tools/streams_exp.py [S] [steps]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
bs, nblk = 4 << 20, 256
per = nblk // S
ctxs = [bmh.Context(0) for _ in range(S)]
ins, outs, caps = [], [], []
offs = np.arange(per + 1, dtype=np.uint64) * np.uint64(bs)
for s, c in enumerate(ctxs):
    d = c.alloc(bs * per)
    for i in range(per):
        c.synth_splitmix64(d.ptr.value + i * bs, bs, 0, (s * per + i) * bs)
    cap = per * int(bmh.lib().bmh_record_bound(bs))
    ins.append(d)
    outs.append(c.alloc(cap))
    caps.append(cap)


def run(s, n):
    for _ in range(n):
        ctxs[s].encode_blocks_dev(ins[s], offs, outs[s], caps[s])


for it in range(2):
    ths = [threading.Thread(target=run, args=(s, 2 if it == 0 else steps)) for s in range(S)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
print(f"S={S}: {dt / steps * 1e3:.2f} ms/step, {nblk * bs * steps / dt / 1e6:.0f} MB/s")
