#!/bin/bash
# Headline step at several pipeline counts, fresh process each: bash tools/pipes_ab.sh ROUNDS P1 P2 ...
rounds=$1; shift
for r in $(seq $rounds); do
  for p in "$@"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --pipelines $p 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('pipelines $p', d['ms_per_step'], d['value'], d['parity'][:7])" || exit 1
  done
done
