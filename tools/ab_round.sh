#!/bin/bash
# On the GPU box: the GPU suite, then the headline bench alternating over bench.py option sets in
# fresh processes (rounds x sets), then optionally the strong-scaling rehearsal.
#   bash tools/ab_round.sh TAG ROUNDS "--opt mtf_chunk=4096" "" ...   (STRONG=1: + rehearsal)
tag=$1; rounds=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq $rounds); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 2 --calgary-steps 3 $cfg \
      > $o/b${r}_$i.json 2> $o/b${r}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$o/b${r}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(f\"[{sys.argv[1]:28s}] {d['value']:9.1f} MB/s {d['ms_per_step']:7.3f} ms pcie {d['pcie_inclusive']['ms_per_step']:6.2f} cal {d['calgary']['whole_files']['ms']:.2f}/{d['calgary']['blocks_256k']['ms']:.2f} {d['parity'][:7]}\", {a: k[a] for a in list(k)[:6]})" "$cfg"
  done
done
if [ -n "$STRONG" ]; then
  timeout -k 10 500 python3 -u tools/strong_rehearsal.py $o/strong_rehearsal.json > $o/rehearsal.log 2>&1 || exit $?
  tail -4 $o/rehearsal.log
fi
