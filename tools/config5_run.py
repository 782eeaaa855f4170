#!/usr/bin/env python3
"""BASELINE config 5 at full size on one GPU: 8 GiB of Zipf text in 16 MiB blocks
(512 blocks), streamed from host memory by bmh_compress_host (H2D / encode / D2H overlapped) and,
when asked, by bmh_compress_host_multi over several contexts (the multi-GPU deal; on a 1-GPU box
the contexts share device 0). The text is the true App. D stream, generated in HBM by
bmh_synth_zipf_dev and copied to pageable host memory; every record is checked against the
reference's 512-block manifest (zipf_16m, tests/golden/make_golden.py) and the whole container
is round-tripped by the GPU decoder (bmh_decompress_dev).
Per-rank rehearsal of config 5 at N = 8: --gib 1 is one rank's share (64 x 16
MiB blocks); --pinned puts input and output in page-locked memory (DMA-only copies); --steps
times several calls; --opts copy_threads=2 gives the staging copies the 2 threads a site that 8
contexts sharing a 16-CPU quota get (bmh_copy_threads).
usage: python tools/config5_run.py [--gib 8] [--contexts 1] [--pinned] [--steps 1] [--opts name=value,...]"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=int, default=8)
ap.add_argument("--contexts", type=int, default=1)
ap.add_argument("--opts", default="", help="bmh_ctx_set_option list name=value,...")
ap.add_argument("--pinned", action="store_true", help="page-locked input and output buffers")
ap.add_argument("--steps", type=int, default=1)
a = ap.parse_args()
n = a.gib << 30
bs = 16 << 20
L = bmh.lib()
ctxs = [bmh.Context(0) for _ in range(a.contexts)]
for c in ctxs:
    c.set_options(a.opts)
t0 = time.perf_counter()
hold = []
if a.pinned:
    hold.append(ctxs[0].alloc_host(n))
    data = hold[-1].a
else:
    data = np.empty(n, dtype=np.uint8)
piece = 1 << 30
d = ctxs[0].alloc(piece)
for off in range(0, n, piece):
    m = min(piece, n - off)
    ctxs[0].synth_zipf(d, m, off)
    bmh._check(L.bmh_memcpy_d2h(ctxs[0].h, bmh._ptr(data[off:off + m]), d.ptr, m), "d2h")
d.free()
gen_s = time.perf_counter() - t0
cap = int(L.bmh_compress_bound(n, bs))
if a.pinned:
    hold.append(ctxs[0].alloc_host(cap))
    out = hold[-1].a
else:
    out = np.empty(cap, dtype=np.uint8)
olen = C.c_uint64()


def run():
    if a.contexts == 1:
        st = L.bmh_compress_host(ctxs[0].h, data.ctypes.data_as(C.c_void_p), n, bs, out.ctypes.data_as(C.c_void_p),
                                 cap, C.byref(olen))
    else:
        arr = (C.c_void_p * a.contexts)(*[c.h for c in ctxs])
        st = L.bmh_compress_host_multi(arr, a.contexts, data.ctypes.data_as(C.c_void_p), n, bs,
                                       out.ctypes.data_as(C.c_void_p), cap, C.byref(olen))
    if st != 0:
        raise RuntimeError(L.bmh_last_error().decode())


run()  # warm-up
each = []
for _ in range(a.steps):
    t1 = time.perf_counter()
    run()
    each.append(time.perf_counter() - t1)
dt = sorted(each)[len(each) // 2]  # median
rec = out[: olen.value]
recs = bmh.container_records(rec)
man = json.load(open(os.path.join(REPO, "tests", "golden", "manifests", "zipf_16m.json")))
nchk = min(len(recs), len(man["blocks"]))
ref_eq = sum(hashlib.sha256(recs[i]).hexdigest() == man["blocks"][i]["sha256"] for i in range(nchk))
back = np.empty(n, dtype=np.uint8)
nout = C.c_uint64()
t2 = time.perf_counter()
st = L.bmh_decompress_dev(ctxs[0].h, rec.ctypes.data_as(C.c_void_p), rec.size, back.ctypes.data_as(C.c_void_p), n,
                          C.byref(nout))
dec_s = time.perf_counter() - t2
ok = st == 0 and nout.value == n and np.array_equal(back, data)
print(json.dumps({"config": "5: Zipf text, 16 MiB blocks, host buffers in and out", "GiB": a.gib,
                  "blocks": len(recs), "contexts": a.contexts, "ms": round(dt * 1e3, 1),
                  "MBps_pcie_inclusive": round(n / dt / 1e6, 1), "ratio": round(olen.value / n, 6),
                  "records_equal_reference_manifest": f"{ref_eq}/{nchk}", "roundtrip_bit_exact": bool(ok),
                  "decode_s": round(dec_s, 2), "gen_s": round(gen_s, 1), "pinned": a.pinned, "opts": a.opts,
                  "steps_ms": [round(x * 1e3, 1) for x in each], "host_cpus": int(L.bmh_host_cpus())}))
