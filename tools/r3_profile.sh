#!/bin/bash
# Round-3 profiling pass on the GPU box (run from the repo root there):
#   tools/profile_round.sh (bench.py default line, rocprofv3 --kernel-trace --stats, PMC traffic)
#   + a kernel trace of the Calgary whole-file batch (tools/cal_trace_run.py, last call analysed
#   by tools/round_trace.py) -> gpurun_out/prof/
set -e
export TMPDIR=/tmp
o=gpurun_out/prof
mkdir -p $o
bash tools/profile_round.sh
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/caltrace -o run --output-format csv -- \
    python3 tools/cal_trace_run.py bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans > $o/caltrace.log 2>&1
python3 tools/round_trace.py $o/caltrace > $o/calgary_rounds.txt
echo r3 profile done
