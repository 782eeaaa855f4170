#!/bin/bash
# kernel timeline of one 128 MiB random encode call (default options: dense probe, one pipeline)
o=gpurun_out/${TAG:-tl128}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t0 -o run --output-format csv -- python3 tools/trace_run.py 128 4 3 > $o/t0.log 2>&1 || exit 1
python3 tools/call_timeline.py $o/t0 > $o/tl0.txt; cat $o/tl0.txt
