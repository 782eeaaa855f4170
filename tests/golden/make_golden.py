#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REAL reference (dev container only).

Runs oracle/_ref/ref_COMPRESS (compiled from /root/reference/main.cpp by oracle/Makefile,
one process per block, like SURVEY §6) and records its outputs:

  calgary/<file>            Calgary corpus inputs (the reference's own test data,
                            cmake-build-release/calgarycorpus/*)
  calgary_records/<file>.bzap  whole-file records written by ref_COMPRESS
  calgary_stdout.txt        ref_COMPRESS stdout per file (main.cpp:321, 402-413)
  small/<name>, small/<name>.bzap  small known-answer inputs and records
  manifests/*.json          per-block {n, primary, record_len, sha256} for the block configs:
                            calgary_256k, random_1g_4m (App. C), zipf_16m, zipf100m_1m

Usage: python tests/golden/make_golden.py [--skip-random] [--jobs 8]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
from bmh import synth  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "ref_COMPRESS")
CORPUS_SRC = "/root/reference/cmake-build-release/calgarycorpus"
CALGARY = ["bib", "book1", "book2", "geo", "news", "obj1", "obj2", "paper1", "paper2",
           "pic", "progc", "progl", "progp", "trans"]  # main.cpp:418-419 order


def run_ref(data: bytes, tmpdir: str, tag: str) -> tuple[bytes, str]:
    src = os.path.join(tmpdir, tag)
    dst = src + ".bzap"
    with open(src, "wb") as f:
        f.write(data)
    out = subprocess.run([REF, src, dst], capture_output=True, check=True, text=True).stdout
    with open(dst, "rb") as f:
        rec = f.read()
    os.remove(src)
    os.remove(dst)
    return rec, out


def entry(rec: bytes) -> dict:
    return {"n": int.from_bytes(rec[8:16], "little"),
            "primary": int.from_bytes(rec[0:8], "little"),
            "tree_len": int.from_bytes(rec[16:24], "little"),
            "record_len": len(rec),
            "sha256": hashlib.sha256(rec).hexdigest()}


def blocks_manifest(name: str, gen, nblocks: int, jobs: int, tmpdir: str, note: str) -> None:
    """gen(b) -> block b's bytes. It is called in block order from this thread (so a sequential
    generator works); at most 2 * jobs blocks are held in memory at a time."""
    t0 = time.time()

    def one(b, data):
        rec, _ = run_ref(data, tmpdir, f"{name}_{b}")
        return rec

    ents = [None] * nblocks
    agg = hashlib.sha256()
    with cf.ThreadPoolExecutor(jobs) as ex:
        pending = {}
        nxt = 0  # next block to fold into the aggregate (records are hashed in block order)
        for b in range(nblocks):
            pending[b] = ex.submit(one, b, gen(b))
            while len(pending) >= 2 * jobs or (b == nblocks - 1 and pending):
                rec = pending.pop(nxt).result()
                ents[nxt] = entry(rec)
                agg.update(rec)
                nxt += 1
                if nxt % 32 == 0:
                    print(f"  {name}: {nxt}/{nblocks} blocks, {time.time() - t0:.0f} s", flush=True)
    man = {"config": name, "note": note, "blocks": ents,
           "total_record_bytes": sum(e["record_len"] for e in ents), "aggregate_sha256": agg.hexdigest(),
           "generated_by": "oracle/_ref/ref_COMPRESS (reference main.cpp, g++ -O3)",
           "ref_wall_s": round(time.time() - t0, 2), "ref_procs": jobs}
    os.makedirs(os.path.join(HERE, "manifests"), exist_ok=True)
    with open(os.path.join(HERE, "manifests", name + ".json"), "w") as f:
        json.dump(man, f, indent=1)
    print(f"{name}: {nblocks} blocks, {man['total_record_bytes']} B, "
          f"{man['aggregate_sha256'][:16]}, {man['ref_wall_s']} s", flush=True)


SMALL = {
    "a": b"a",
    "aaaaaaaa": b"aaaaaaaa",
    "abababab": b"abababab",
    "banana": b"banana",
    "zeros1000": bytes(1000),
    "ab_x3": b"ab" * 3 + b"c",
    "hello": b"hello world, hello bwt!\n" * 5,
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--skip-random", action="store_true")
    ap.add_argument("--zipf-blocks", type=int, default=512)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit("build oracle/_ref first: make -C oracle")
    tmp = tempfile.mkdtemp(prefix="bmh_golden_")
    only = set(a.only.split(",")) if a.only else None
    try:
        if not only or "calgary" in only:
            os.makedirs(os.path.join(HERE, "calgary"), exist_ok=True)
            os.makedirs(os.path.join(HERE, "calgary_records"), exist_ok=True)
            lines = []
            for fn in CALGARY:
                with open(os.path.join(CORPUS_SRC, fn), "rb") as f:
                    data = f.read()
                with open(os.path.join(HERE, "calgary", fn), "wb") as f:
                    f.write(data)
                rec, out = run_ref(data, tmp, fn)
                with open(os.path.join(HERE, "calgary_records", fn + ".bzap"), "wb") as f:
                    f.write(rec)
                # the reference prints the OUTPUT path it was given; keep the part after it
                lines.append({"file": fn, "stdout_tail": out.split(" $$ initial_data_size:")[1]})
            with open(os.path.join(HERE, "calgary_stdout.json"), "w") as f:
                json.dump(lines, f, indent=1)
            print("calgary whole-file records written", flush=True)
        if not only or "small" in only:
            os.makedirs(os.path.join(HERE, "small"), exist_ok=True)
            for name, data in SMALL.items():
                rec, _ = run_ref(data, tmp, name)
                with open(os.path.join(HERE, "small", name), "wb") as f:
                    f.write(data)
                with open(os.path.join(HERE, "small", name + ".bzap"), "wb") as f:
                    f.write(rec)
            print("small records written", flush=True)
        if not only or "calgary_256k" in only:
            blocks = []
            for fn in CALGARY:
                with open(os.path.join(CORPUS_SRC, fn), "rb") as f:
                    d = f.read()
                for i in range(0, len(d), 262144):
                    blocks.append(d[i:i + 262144])
            blocks_manifest("calgary_256k", lambda b: blocks[b], len(blocks), a.jobs, tmp,
                            "Calgary corpus, file order (main.cpp:418), each file cut into 256 KiB blocks")
        if not only or "zipf_16m" in only:
            # config 5: the whole 8 GiB App. D stream, 512 x 16 MiB blocks, generated block by
            # block by the oracle's sequential C generator (checked against the App. D sha256 of
            # the first 16 MiB and against bmh.synth.zipf_text in tests/test_oracle.py)
            sys.path.insert(0, os.path.dirname(HERE))
            from oracle_ffi import Oracle, ZipfStream
            zs = ZipfStream(Oracle())
            blocks_manifest("zipf_16m", lambda b: zs.read(16 << 20).tobytes(), a.zipf_blocks, a.jobs, tmp,
                            f"config 5: the App. D Zipf text stream cut into 16 MiB blocks, blocks "
                            f"0..{a.zipf_blocks - 1} ({a.zipf_blocks * 16 >> 10} GiB)")
        if not only or "zipf100m_1m" in only:
            z = synth.zipf_text(100_000_000).tobytes()
            nb = (len(z) + (1 << 20) - 1) >> 20
            blocks_manifest("zipf100m_1m", lambda b: z[b << 20:(b + 1) << 20], nb, a.jobs, tmp,
                            "enwik8 substitute: first 100,000,000 B of the App. D Zipf stream, 1 MiB blocks")
        if (not only or "random_1g_4m" in only) and not a.skip_random:
            blocks_manifest("random_1g_4m", lambda b: synth.splitmix64_bytes(0, b << 22, 1 << 22).tobytes(),
                            256, a.jobs, tmp, "splitmix64(seed 0) 1 GiB, 4 MiB blocks b0000..b0255")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
