#!/bin/bash
# Per-process step-time mode of the headline workload: several fresh processes, median step each
# (2 run streams by default; pipelines=1 for the serial reference). Run on the GPU box.
set -e
mkdir -p gpurun_out/mode
for i in 1 2 3 4 5 6; do
    timeout -k 10 60 python3 tools/step_times.py 20 > gpurun_out/mode/s2_$i.txt
done
for i in 1 2; do
    timeout -k 10 60 python3 tools/step_times.py 20 pipelines=1 > gpurun_out/mode/s1_$i.txt
done
python3 - <<'P'
import glob, statistics
for f in sorted(glob.glob("gpurun_out/mode/*.txt")):
    v = [float(x) for x in open(f).read().split()][3:]
    print(f.split("/")[-1], "median %.2f min %.2f max %.2f" % (statistics.median(v), min(v), max(v)))
P
