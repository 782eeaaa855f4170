#!/bin/bash
# Timelines of the PCIe-inclusive leg (bench.py's pcie_inclusive: bmh_compress_host, page-locked
# in / out, 1 GiB random at 4 MiB blocks) under rocprofv3 --kernel-trace --memory-copy-trace, at
# the default 256 MiB batches and at 64 MiB; summarised by tools/pcie_timeline.py.
set -e
export TMPDIR=/tmp
o=gpurun_out/pcie; mkdir -p $o
args="--steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --calgary-steps 0 --pcie-steps 2"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $o/b256 -o run --output-format csv -- python3 bench.py $args > $o/b256.json 2> $o/b256.err
python3 tools/pcie_timeline.py $o/b256 40 > $o/timeline_256m.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $o/b64 -o run --output-format csv -- python3 bench.py $args --opt stream_batch=$((64 << 20)) > $o/b64.json 2> $o/b64.err
python3 tools/pcie_timeline.py $o/b64 50 > $o/timeline_64m.txt
timeout -k 10 200 python3 bench.py $args > $o/plain256.json 2> $o/plain256.err
timeout -k 10 200 python3 bench.py $args --opt stream_batch=$((64 << 20)) > $o/plain64.json 2> $o/plain64.err
echo pcie trace done
