#!/bin/bash
# On the GPU box: Zipf text configs over pipeline counts (BMH_OPT_PIPELINES), fresh process each:
# bash tools/text_pipes.sh TAG ROUNDS "MB BLOCK_MiB" "p1 p2 ..."
tag=$1; rounds=$2; cfg=$3; pipes=$4
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
  for p in $pipes; do
    timeout -k 10 150 python3 tools/text_bench.py $cfg pipelines=$p > $o/t_${cfg// /_}_p${p}_$r.json || exit 1
    python3 -c "import json; d=json.load(open('$o/t_${cfg// /_}_p${p}_$r.json')); print('$cfg pipelines=$p', d['ms'], d.get('parity'))"
  done
done
