#!/bin/bash
# Kernel traces of the Calgary whole-file batch (3 calls, the last analysed by
# tools/round_trace.py / tools/stream_trace.py): default pipelines, then one stream.
set -e
export TMPDIR=/tmp
o=gpurun_out/cal2; mkdir -p $o
files="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t -o run --output-format csv -- python3 tools/cal_trace_run.py $files > $o/log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t1 -o run --output-format csv -- python3 tools/cal_trace_run.py --opts pipelines=1 $files > $o/log1 2>&1
echo ok
