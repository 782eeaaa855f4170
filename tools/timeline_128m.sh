#!/bin/bash
# kernel timeline of one random encode call (default options): bash tools/timeline_128m.sh [MiB]
mib=${1:-128}
o=gpurun_out/${TAG:-tl$mib}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $o/t0 -o run --output-format csv -- python3 tools/trace_run.py $mib 4 3 > $o/t0.log 2>&1 || exit 1
python3 tools/call_timeline.py $o/t0 5 > $o/tl0.txt; head -1 $o/tl0.txt
python3 - $o/tl0.txt <<'P'
import collections, sys
L = open(sys.argv[1]).read().splitlines()[1:]
q = collections.defaultdict(list)
for l in L:
    p = l.split()
    q[p[2] + p[3]].append((float(p[0]), float(p[1]), p[-1]))
for k, v in sorted(q.items()):
    print(k, len(v), "busy", round(sum(d for _, d, _ in v), 1), "first", v[0][0], "end", round(max(s + d for s, d, _ in v), 1))
P
