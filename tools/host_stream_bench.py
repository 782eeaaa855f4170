#!/usr/bin/env python3
"""Host-buffer (PCIe-inclusive) encode throughput through bmh_compress_host: the streaming
pipeline (pinned staging slots, H2D / D2H on side streams) on one GPU.
usage: python tools/host_stream_bench.py [--data random|zipf] [--mib 1024] [--block-mib 16] [--steps 3]
Prints one JSON line; the round trip is checked with the GPU decoder (bmh_decompress_dev)."""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402
from bmh import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--data", default="zipf", choices=["random", "zipf"])
ap.add_argument("--mib", type=int, default=1024)
ap.add_argument("--block-mib", type=int, default=16)
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
n = a.mib << 20
bs = a.block_mib << 20
t0 = time.perf_counter()
if a.data == "zipf":
    src = synth.zipf_text(min(n, 256 << 20))
    data = np.resize(src, n)  # the 256 MiB Zipf prefix repeated (blocks are encoded independently)
else:
    ctx0 = bmh.Context(0)
    d = ctx0.alloc(n)
    ctx0.synth_splitmix64(d, n, 0, 0)
    data = d.download(n)
    d.free()
gen_s = time.perf_counter() - t0
ctx = bmh.Context(0)
L = bmh.lib()
cap = int(L.bmh_compress_bound(n, bs))
out = np.empty(cap, dtype=np.uint8)
olen = C.c_uint64()


def run():
    st = L.bmh_compress_host(ctx.h, data.ctypes.data_as(C.c_void_p), n, bs, out.ctypes.data_as(C.c_void_p), cap,
                             C.byref(olen))
    if st != 0:
        raise RuntimeError(L.bmh_last_error().decode())


run()  # warm-up (staging buffers, workspaces)
ts = []
for _ in range(a.steps):
    t1 = time.perf_counter()
    run()
    ts.append(time.perf_counter() - t1)
dt = min(ts)
rec = out[: olen.value]
back = np.empty(n, dtype=np.uint8)
nout = C.c_uint64()
st = L.bmh_decompress_dev(ctx.h, rec.ctypes.data_as(C.c_void_p), rec.size, back.ctypes.data_as(C.c_void_p), n,
                          C.byref(nout))
ok = st == 0 and nout.value == n and np.array_equal(back, data)
print(json.dumps({"data": a.data, "MiB": a.mib, "block_MiB": a.block_mib, "ms": round(dt * 1e3, 2),
                  "MBps_pcie_inclusive": round(n / dt / 1e6, 1), "ms_all": [round(x * 1e3, 2) for x in ts],
                  "ratio": round(olen.value / n, 6), "roundtrip_bit_exact": bool(ok),
                  "stream_batch": os.environ.get("BMH_STREAM_BATCH", "268435456"),
                  "sha256_16": hashlib.sha256(rec.tobytes()).hexdigest()[:16], "gen_s": round(gen_s, 1)}))
