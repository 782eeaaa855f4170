#!/usr/bin/env python3
"""oracle/alloc_trace/band_trace.py — TEST INFRASTRUCTURE ONLY.

The reference's Huffman tie-break compares BTree* heap addresses (main.cpp:232 priority_queue of
pair<long, BTree*>, nodes from `new BTree` at :240,:252). This module restates the heap calls a
standalone `ref_COMPRESS in out` run makes before its last BTree node, as a function of the block
size n and the leaf count L, replays them through glibc_heap.Heap, and returns the address rank
of every node id (leaves 0..L-1 in first-occurrence order, internal nodes L.. in creation order).

The heap calls, in order (each cites the reference line that makes it):
  libstdc++ start-up             M 72704 (the exception-handling emergency pool)
  read_bytes io_utilities.h:40-41 ifstream: M 472 (FILE), M 8192 (buffer); istreambuf_iterator
                                  growth of `bytes`: M 1, then M 2c / F c while c < n; close:
                                  F buffer, F FILE
             io_utilities.h:50,54 `data = bytes` M n; the returned tuple M n; F bytes, F data
  bwt        main.cpp:77-91       by-value copy M n; shift_order M 8n; stable_sort buffer
                                  M 8*ceil(n/2), F; encoded M n; make_pair copy M n; F encoded,
                                  F shift_order, F copy
  compress   main.cpp:308         bwt_data = bwt_result.second M n
  move_to_front main.cpp:93-112   by-value copy M n; alphabet M 256; encoded_data M n; F
                                  alphabet, F copy
  huffman    main.cpp:229-257     frequencies M 2048; already_in_queue M 32; per new leaf i:
                                  M 24 (node i), then the queue's push grows its vector of
                                  16-byte pairs when full (M 16c', F old); then L-1 times M 24
                                  (internal nodes; pops never shrink the vector).

`--validate` runs oracle/_ref/ref_COMPRESS_mtrace (oracle/Makefile `mtrace`, this container
only) on every band case, checks that the traced calls up to the last BTree node are exactly
these, that the emulator returns the traced address for every call, and that a Huffman build
with the resulting ranks reproduces the reference's record byte for byte.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from glibc_heap import Heap  # noqa: E402


def heap_calls(n: int, L: int):
    """('M', size, name) / ('F', name) of a standalone COMPRESS run up to its last BTree node."""
    yield ("M", 72704, "eh_pool")
    yield ("M", 472, "FILE")
    yield ("M", 8192, "filebuf")
    c = 1
    yield ("M", 1, "bytes1")
    while c < n:
        yield ("M", 2 * c, f"bytes{2 * c}")
        yield ("F", f"bytes{c}")
        c *= 2
    yield ("F", "filebuf")
    yield ("F", "FILE")
    yield ("M", n, "data")
    yield ("M", n, "ret")
    yield ("F", f"bytes{c}")
    yield ("F", "data")
    yield ("M", n, "bwt_arg")
    yield ("M", 8 * n, "shift_order")
    yield ("M", 8 * ((n + 1) // 2), "stable_buf")
    yield ("F", "stable_buf")
    yield ("M", n, "encoded")
    yield ("M", n, "pair")
    yield ("F", "encoded")
    yield ("F", "shift_order")
    yield ("F", "bwt_arg")
    yield ("M", n, "bwt_data")
    yield ("M", n, "mtf_arg")
    yield ("M", 256, "alphabet")
    yield ("M", n, "mtf_data")
    yield ("F", "alphabet")
    yield ("F", "mtf_arg")
    yield ("M", 2048, "frequencies")
    yield ("M", 32, "in_queue")
    cap = 0
    for i in range(L):
        yield ("M", 24, ("node", i))
        if i == cap:  # push into a full vector of pairs
            nc = max(1, 2 * cap)
            yield ("M", 16 * nc, f"pq{nc}")
            if cap:
                yield ("F", f"pq{cap}")
            cap = nc
    for i in range(L, 2 * L - 1):
        yield ("M", 24, ("node", i))


def replay(n: int, L: int, heap: Heap | None = None):
    """Emulated addresses: {name: address} for every block allocated, and the node addresses."""
    h = heap or Heap()
    live, addr, nodes = {}, [], [0] * (2 * L - 1)
    for call in heap_calls(n, L):
        if call[0] == "M":
            a = h.malloc(call[1])
            live[call[2]] = a
            addr.append((call[2], call[1], a))
            if isinstance(call[2], tuple):
                nodes[call[2][1]] = a
        else:
            h.free_(live.pop(call[1]))
    return nodes, addr


def node_ranks(n: int, L: int) -> list[int]:
    """rank[s] = position of node s in ascending heap-address order."""
    nodes, _ = replay(n, L)
    order = sorted(range(2 * L - 1), key=lambda s: nodes[s])
    rank = [0] * (2 * L - 1)
    for k, s in enumerate(order):
        rank[s] = k
    return rank


def model_ranks(L: int) -> list[int]:
    """SURVEY App. B.3's address-rank model (oracle.c addr_ranks), for comparison."""
    if L <= 128:
        order = [1] + list(range(3, 128)) + [0, 2] + list(range(128, 512))
    else:
        order = [1] + list(range(3, 65)) + list(range(129, 193)) + list(range(65, 128)) + [0, 2, 128] + \
            list(range(193, 512))
    rank, k = [0] * (2 * L - 1), 0
    for s in order:
        if s < 2 * L - 1:
            rank[s] = k
            k += 1
    return rank


# ---- a Huffman build with explicit ranks (main.cpp:245-254; pops: smallest freq, then the
# larger address), codes (traverse :132-147), preorder tree bits (dfs :174-187), record
# (write_bytes io_utilities.h:7-27). Used only to check the ranks against reference records.
def record_with_ranks(block: bytes, rank_fn) -> bytes:
    import numpy as np

    sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
    from oracle_ffi import Oracle

    orc = Oracle()
    primary, L_col = orc.bwt(block)
    mtf = np.frombuffer(orc.mtf(L_col), np.uint8)
    freq = np.bincount(mtf, minlength=256)
    seen, leaves = set(), []
    for v in mtf.tolist():
        if v not in seen:
            seen.add(v)
            leaves.append(v)
    L = len(leaves)
    rank = rank_fn(len(block), L)
    f = [int(freq[v]) for v in leaves]
    kids = []
    alive = list(range(L))
    while len(alive) > 1:
        pick = []
        for _ in range(2):
            best = min(alive, key=lambda s: (f[s], -rank[s]))
            alive.remove(best)
            pick.append(best)
        f.append(f[pick[0]] + f[pick[1]])
        kids.append(pick)
        alive.append(len(f) - 1)
    root = alive[0]
    codes, bits = {}, []

    def walk(s, code):
        if s < L:
            codes[leaves[s]] = code
            bits.append("0" + format(leaves[s], "08b"))
            return
        bits.append("1")
        walk(kids[s - L][0], code + "0")
        walk(kids[s - L][1], code + "1")

    walk(root, "")

    def pack(b: str) -> bytes:
        b += "0" * (-len(b) % 8)
        return bytes(int(b[i:i + 8], 2) for i in range(0, len(b), 8)) or b"\x00"

    tree = pack("".join(bits))
    payload = pack("".join(codes[v] for v in mtf.tolist()))
    hdr = primary.to_bytes(8, "little") + len(block).to_bytes(8, "little") + len(tree).to_bytes(8, "little")
    return hdr + tree + payload


def _traced_calls(path: str):
    """The traced binary's calls up to its last BTree node, as (op, size) with frees by index."""
    out, idx = [], {}
    for line in open(path):
        f = line.split()
        if f[0] == "M":
            idx[int(f[2], 16)] = len(out)
            out.append(("M", int(f[1]), int(f[2], 16)))
        elif f[0] == "F":
            a = int(f[1], 16)
            out.append(("F", idx.pop(a, None), a))
    return out


def validate(cases=None, verbose=False) -> int:
    import json
    import subprocess
    import tempfile

    repo = os.path.abspath(os.path.join(HERE, "..", ".."))
    sys.path.insert(0, os.path.join(repo, "tests", "golden"))
    sys.path.insert(0, os.path.join(repo, "bwt-mtf-huffman-compressor_amd"))
    from make_bands import source

    binp = os.path.join(repo, "oracle", "_ref", "ref_COMPRESS_mtrace")
    man = json.load(open(os.path.join(repo, "tests", "golden", "manifests", "bands.json")))
    bad = 0
    exact_model = exact_emul = 0
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for case in man["cases"]:
            kind, n = case["kind"], case["n"]
            if cases and (kind, n) not in cases:
                continue
            data = source(kind, n)
            with open(os.path.join(tmp, "in"), "wb") as f:
                f.write(data)
            with open(os.path.join(tmp, "trace"), "w") as tr:
                subprocess.run([binp, "in", "out.bzap"], cwd=tmp, stdout=subprocess.DEVNULL, stderr=tr, check=True)
            ref = open(os.path.join(tmp, "out.bzap"), "rb").read()
            import hashlib
            assert hashlib.sha256(ref).hexdigest() == case["sha256"], (kind, n)
            traced = _traced_calls(os.path.join(tmp, "trace"))
            # leaf count from the record's tree: L = (tree bits + 1) / 10 for a full binary tree
            rec_model = record_with_ranks(data, lambda nn, LL: model_ranks(LL))
            L = None
            rec_emul = record_with_ranks(data, lambda nn, LL: node_ranks(nn, LL))
            # the template vs the trace, call by call, up to the last node
            _, emu = replay(n, _leaf_count(data))
            msizes = [c[1] for c in traced if c[0] == "M"][:len(emu)]
            ok_calls = msizes == [e[1] for e in emu]
            base = traced[0][2] - emu[0][2]
            taddrs = [c[2] - base for c in traced if c[0] == "M"][:len(emu)]
            ok_addr = taddrs == [e[2] if e[2] < (1 << 40) else t for e, t in zip(emu, taddrs)]
            em, ee = rec_model == ref, rec_emul == ref
            exact_model += em
            exact_emul += ee
            rows.append((kind, n, ok_calls, ok_addr, em, ee))
            if not (ok_calls and ok_addr and ee):
                bad += 1
            if verbose or not (ok_calls and ok_addr and ee):
                print(f"{kind:6s} n={n:6d} calls={'ok' if ok_calls else 'DIFF'} addrs={'ok' if ok_addr else 'DIFF'} "
                      f"model_exact={em} emulated_exact={ee}")
    print(f"{len(rows)} cases: model byte-exact {exact_model}, emulated-heap byte-exact {exact_emul}, bad {bad}")
    return bad


def _leaf_count(block: bytes) -> int:
    sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
    from oracle_ffi import Oracle
    import numpy as np

    orc = Oracle()
    _, L_col = orc.bwt(block)
    return int(np.count_nonzero(np.bincount(np.frombuffer(orc.mtf(L_col), np.uint8), minlength=256)))


if __name__ == "__main__":
    if "--validate" in sys.argv:
        sys.exit(1 if validate(verbose="-v" in sys.argv) else 0)
    n, L = int(sys.argv[1]), int(sys.argv[2])
    print(node_ranks(n, L))
