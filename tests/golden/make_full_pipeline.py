#!/usr/bin/env python3
"""Fixtures of the reference's FULL_PIPELINE mode (main.cpp:416-438; dev container only).

Runs oracle/_ref/ref_FULL_PIPELINE (compiled from /root/reference/main.cpp) in a scratch
directory holding calgarycorpus/ (the 14 Calgary files, tests/golden/calgary) and keeps its
outputs: full_pipeline/<file>.bzap (the records it writes; the Huffman tie-break carries heap
history from file to file, so 13 of 14 differ in tree bytes from standalone COMPRESS records,
SURVEY §0.5) and full_pipeline/stdout.txt.

Usage: python tests/golden/make_full_pipeline.py
"""
import os
import shutil
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "ref_FULL_PIPELINE")
CALGARY = ["bib", "book1", "book2", "geo", "news", "obj1", "obj2", "paper1", "paper2",
           "pic", "progc", "progl", "progp", "trans"]


def main() -> None:
    out = os.path.join(HERE, "full_pipeline")
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(os.path.join(HERE, "calgary"), os.path.join(tmp, "calgarycorpus"))
        r = subprocess.run([REF], cwd=tmp, check=True, capture_output=True, text=True)
        for f in CALGARY:
            shutil.copy(os.path.join(tmp, "calgarycorpus", f + ".bzap"), os.path.join(out, f + ".bzap"))
    with open(os.path.join(out, "stdout.txt"), "w") as f:
        f.write(r.stdout)
    print(r.stdout)


if __name__ == "__main__":
    main()
