#!/bin/bash
# On the GPU box: headline workload (splitmix64, 4 MiB blocks) at several batch sizes x pipeline
# counts, fresh process each: bash tools/pipe_sweep.sh TAG "128 256 512 1024" "0 1 2 4" [rounds]
tag=$1; sizes=$2; pipes=$3; rounds=${4:-1}
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
for mb in $sizes; do
  for p in $pipes; do
    timeout -k 10 120 python3 bench.py --total-bytes $((mb<<20)) --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --pipelines $p > $o/b${mb}_$p.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$o/b${mb}_$p.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('MiB $mb pipes $p', d['ms_per_step'], d['parity'][:6], 'ksum', round(sum(k.values()),3), {a:k[a] for a in list(k)[:5]})"
  done
done
done
