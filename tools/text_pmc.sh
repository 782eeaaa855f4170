#!/bin/bash
# Config 3: per-stage HBM GB/s of the Zipf 100 MB text at 1 MiB blocks, one stream:
# stats pass + FETCH_SIZE pass + WRITE_SIZE pass over tools/text_bench.py, then tools/stage_gbs.py.
set -e
export TMPDIR=/tmp BMH_STREAMS=1
o=gpurun_out/textpmc
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/stats -o run --output-format csv -- python3 tools/text_bench.py 100 1 > $o/stats.json 2> $o/stats.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $o/pmc/p1 -o run --output-format csv -- python3 tools/text_bench.py 100 1 > $o/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $o/pmc/p2 -o run --output-format csv -- python3 tools/text_bench.py 100 1 > $o/p2.log 2>&1
python3 tools/stage_gbs.py $o/stats $o/pmc 100000000 $o/text100_stage_gbs.json
