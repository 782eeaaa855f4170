#!/bin/bash
# GPU decode of 1 GiB random (4 MiB blocks): per-kernel times and wall for several LF group sizes,
# then the same on Zipf text (run on the GPU box).
set -e
mkdir -p gpurun_out
for g in 4294967296; do
  echo "BMH_LF_GROUP=$g"
  BMH_LF_GROUP=$g timeout -k 10 120 python3 tools/decode_prof.py | head -8
done
