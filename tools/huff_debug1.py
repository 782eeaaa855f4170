#!/usr/bin/env python3
"""Debug aid: one block (default zipf 39 800) through the encode, for a BMH_DEBUG_HUFF build."""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "bwt-mtf-huffman-compressor_amd"))
import bmh  # noqa: E402
from bmh import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 39800
ctx = bmh.Context(0)
print(len(ctx.encode_blocks([synth.zipf_text(n).tobytes()])[0]))
