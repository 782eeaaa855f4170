#!/bin/bash
# 128 MiB (the N = 8 strong-scaling share) steps alternating over library builds, fresh process each
o=gpurun_out/${TAG:-ab128}; mkdir -p $o
rounds=$1; shift
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    BMH_LIB=$lib timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes 134217728 > $o/${n}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$o/${n}_$r.json').read().strip().splitlines()[-1]); print('$l'.ljust(28), d['ms_per_step'], d['parity'][:6])"
  done
done
