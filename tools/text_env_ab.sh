#!/bin/bash
# A/B of a library option on the Zipf text configs (tools/text_bench.py):
# tools/text_env_ab.sh NAME "valA valB" "<MB> <block_MiB>" [rounds]
var=$1; vals=$2; args=$3; rounds=${4:-2}
for r in $(seq $rounds); do
  for v in $vals; do
    timeout -k 10 200 python3 tools/text_bench.py $args $var=$v 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$var=$v', '$args', d['ms'], d['MBps'], d.get('parity'))" || exit 1
  done
done
