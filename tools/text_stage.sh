#!/bin/bash
# Config 3 (Zipf 100 MB, 1 MiB blocks, one stream) per-stage HBM table: a kernel-trace pass and
# one PMC pass per counter over tools/text_bench.py (5 encode calls), then tools/text_stage_gbs.py
o=gpurun_out/${TAG:-tstage}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- python3 tools/text_bench.py 100 1 pipelines=1 > $o/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $o/pf -o run --output-format csv -- python3 tools/text_bench.py 100 1 pipelines=1 > $o/pf.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $o/pw -o run --output-format csv -- python3 tools/text_bench.py 100 1 pipelines=1 > $o/pw.log 2>&1 || exit 1
python3 tools/text_stage_gbs.py $o 100000000 5 $o/stage_gbs.json
