#!/bin/bash
# A/B of the Calgary leg over a library option: tools/cal_ab.sh NAME "valA valB" [rounds]
# (bench.py Calgary leg only, alternating fresh processes) -> one line per run
var=$1; vals=$2; rounds=${3:-2}
for r in $(seq $rounds); do
  for v in $vals; do
    timeout -k 10 120 python3 bench.py --opt $var=$v --steps 1 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 30 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d['calgary']; print('$var=$v', c['whole_files']['ms'], c['blocks_256k']['ms'], c['whole_files']['records_byte_identical_to_reference'], c['blocks_256k']['records_byte_identical_to_reference'])" || exit 1
  done
done
