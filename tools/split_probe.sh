#!/bin/bash
# Step time of the headline workload against the two runs' split (BMH_SPLIT = percent of the
# batch in run 0), 4 fresh processes per setting (run-to-run spread is per process).
set -e
mkdir -p gpurun_out/split
for sp in ${SPLITS:-50 40 60 30 70}; do
    for i in $(seq ${REPS:-4}); do
        BMH_SPLIT=$sp timeout -k 10 60 python3 tools/step_times.py 16 > gpurun_out/split/p${sp}_$i.txt
    done
done
export SPLITS="${SPLITS:-50 40 60 30 70}"
python3 - <<'P'
import glob, statistics
for sp in [int(x) for x in __import__("os").environ.get("SPLITS", "50 40 60 30 70").split()]:
    meds = []
    for f in sorted(glob.glob(f"gpurun_out/split/p{sp}_*.txt")):
        v = [float(x) for x in open(f).read().split()][3:]
        meds.append(statistics.median(v))
    print(sp, " ".join("%.2f" % m for m in meds), "mean %.2f" % statistics.mean(meds))
P
