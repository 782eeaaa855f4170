#!/bin/bash
# Round-5 evidence pass: headline line + rocprofv3 stats + PMC traffic (tools/profile_round.sh),
# the strong-scaling rehearsal, the config-3 per-stage HBM table, the text configs.
export TMPDIR=/tmp
o=gpurun_out/${TAG:-evid}; mkdir -p $o
bash tools/profile_round.sh || exit 1
echo "profile ok"; tail -c 600 gpurun_out/prof/bench.json; echo
timeout -k 10 600 python3 tools/strong_rehearsal.py $o/strong_rehearsal.json --reps 2 > $o/rehearsal.log 2>&1 || exit 1
tail -4 $o/rehearsal.log
TAG=${TAG:-evid}_text bash tools/text_stage.sh > $o/text_stage.txt 2>&1 || exit 1
tail -3 $o/text_stage.txt
for cfg in "100 1" "128 16" "128 4"; do
  timeout -k 10 150 python3 tools/text_bench.py $cfg > $o/t_${cfg// /_}.json || exit 1
  python3 -c "import json; d=json.load(open('$o/t_${cfg// /_}.json')); print('$cfg', d['ms'], d['MBps'], d.get('parity'))"
done
