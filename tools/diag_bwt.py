#!/usr/bin/env python3
"""BWT diagnostics (experiments): GPU BWT of one Calgary file vs the oracle; prints the rows whose
last-column byte differs, each with its rotation's LCP to the neighbouring rows in the true order.
usage: [BMH_LIB=...] python tools/diag_bwt.py [name]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import bmh  # noqa: E402
from oracle_ffi import Oracle  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bib"
data = open(os.path.join(REPO, "tests", "golden", "calgary", name), "rb").read()
a = np.frombuffer(data, np.uint8)
n = a.size
ctx = bmh.Context(0)
prim, L = bmh.bwt(data, ctx)
oprim, oL = Oracle().bwt(data)
Lg = np.frombuffer(L, np.uint8)
Lo = np.frombuffer(oL, np.uint8)
bad = np.nonzero(Lg != Lo)[0]
print(f"{name}: n={n} primary gpu {prim} oracle {oprim}; {bad.size} rows differ")
if bad.size:
    # cyclic suffix array by prefix doubling (numpy)
    rank = a.astype(np.int64)
    k = 1
    idx = np.arange(n)
    while True:
        key2 = rank[(idx + k) % n]
        order = np.lexsort((key2, rank))
        r1, r2 = rank[order], key2[order]
        newr = np.empty(n, np.int64)
        newr[order] = np.concatenate([[0], np.cumsum((r1[1:] != r1[:-1]) | (r2[1:] != r2[:-1]))])
        rank = newr
        if rank.max() == n - 1 or k >= n:
            break
        k *= 2
    sa = order

    def lcp(p, q):
        m = 0
        while m < n and a[(p + m) % n] == a[(q + m) % n]:
            m += 1
        return m

    print("first bad rows:", bad[:20].tolist(), "last:", bad[-5:].tolist())
    runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
    print(f"{len(runs)} runs of bad rows; sizes:", [len(r) for r in runs[:20]])
    for r in runs[:8]:
        i = int(r[0])
        lo, hi = max(0, i - 1), min(n - 1, int(r[-1]) + 1)
        l_in = [lcp(int(sa[j]), int(sa[j + 1])) for j in range(lo, hi)]
        print(f"  rows {int(r[0])}..{int(r[-1])}: LCP(bytes) of neighbours {l_in[:12]}; text {bytes(a[int(sa[i]):int(sa[i]) + 24])!r}")
