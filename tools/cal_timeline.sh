#!/bin/bash
# Calgary whole-file batch: kernel timeline of one call (default pipelines)
o=gpurun_out/${TAG:-caltl}; mkdir -p $o
export TMPDIR=/tmp
files="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t -o run --output-format csv -- python3 tools/cal_trace_run.py $files > $o/log 2>&1 || exit 1
python3 tools/call_timeline.py $o/t 3 > $o/tl.txt; head -1 $o/tl.txt; wc -l $o/tl.txt
