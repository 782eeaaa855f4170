#!/usr/bin/env python3
"""Repeat the Calgary whole-file batch through each stage and count mismatches against the
oracle (a nondeterminism hunt: one process, many repetitions, workspace scrambled between
them by small unrelated encodes).  usage: python tools/stress_calgary.py [reps]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"), os.path.join(REPO, "tests")]
import bmh  # noqa: E402
from oracle_ffi import Oracle, golden_calgary  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only_bwt = len(sys.argv) > 2 and sys.argv[2] == "bwt"
orc = Oracle()
names, datas, recs = zip(*golden_calgary())
arrs = [np.frombuffer(d, np.uint8) for d in datas]
offs = np.zeros(len(arrs) + 1, np.uint64)
offs[1:] = np.cumsum([a.size for a in arrs])
cat = np.concatenate(arrs)
ref = [orc.bwt(d) for d in datas]
refL = np.concatenate([np.frombuffer(L, np.uint8) for _, L in ref])
refM = np.concatenate([np.frombuffer(orc.mtf(L), np.uint8) for _, L in ref])
ctx = bmh.Context(0)
rng = np.random.default_rng(1)
bad = {"encode": {}, "bwt": {}, "mtf": {}}
for r in range(reps):
    # scramble the workspaces with an unrelated small batch
    ctx.encode_blocks([rng.integers(0, 256, int(rng.integers(1, 200000)), dtype=np.uint8).tobytes()
                       for _ in range(int(rng.integers(1, 6)))])
    if not only_bwt:
        out = ctx.encode_blocks(datas)
        for n, o, rr in zip(names, out, recs):
            if o != rr:
                bad["encode"][n] = bad["encode"].get(n, 0) + 1
    d_in, d_L, d_M = ctx.alloc(cat.size), ctx.alloc(cat.size), ctx.alloc(cat.size)
    d_in.upload(cat)
    prim = ctx.bwt_dev(d_in, offs, d_L)
    L = d_L.download()
    for i, n in enumerate(names):
        a, b = int(offs[i]), int(offs[i + 1])
        if int(prim[i]) != ref[i][0] or not np.array_equal(L[a:b], refL[a:b]):
            bad["bwt"][n] = bad["bwt"].get(n, 0) + 1
    if not only_bwt:
        d_L.upload(refL)
        ctx.mtf_dev(d_L, offs, d_M)
        M = d_M.download()
        for i, n in enumerate(names):
            a, b = int(offs[i]), int(offs[i + 1])
            if not np.array_equal(M[a:b], refM[a:b]):
                bad["mtf"][n] = bad["mtf"].get(n, 0) + 1
    for d in (d_in, d_L, d_M):
        d.free()
    if r % 20 == 19:
        print(f"rep {r}: {bad}", flush=True)
ctx.close()
print("FAIL" if any(bad.values()) else "OK", bad)
