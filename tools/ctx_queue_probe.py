import os, statistics, sys, time
import numpy as np
import torch
sys.path.insert(0, "bwt-mtf-huffman-compressor_amd")
import bmh
bs, nblk = 4 << 20, 256
offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
ctx0 = bmh.Context(0)
d_in = ctx0.alloc(bs * nblk)
for i in range(nblk):
    ctx0.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, i * bs)
cap = nblk * int(bmh.lib().bmh_record_bound(bs))
d_out = ctx0.alloc(cap)
keep = []
for k in range(int(sys.argv[1])):
    ctx = bmh.Context(0)
    ts = []
    for s in range(10):
        t0 = time.perf_counter()
        ctx.encode_blocks_dev(d_in, offs, d_out, cap)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"ctx {k} extra_streams {len(keep)} median {statistics.median(ts[2:]):.2f}", flush=True)
    ctx.close()
    keep.append(torch.cuda.Stream())
