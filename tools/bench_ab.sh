#!/bin/bash
# A/B of the headline bench line over library builds: tools/bench_ab.sh "libA libB" [rounds]
# (BMH_LIB per fresh process, alternating; device-resident leg only)
libs=$1; rounds=${2:-2}
for r in $(seq $rounds); do
  for l in $libs; do
    BMH_LIB=$l timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$l', d['value'], d['ms_per_step'], d['parity'])" || exit 1
  done
done
