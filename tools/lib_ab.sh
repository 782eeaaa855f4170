#!/bin/bash
# On the GPU box: headline bench (device-resident leg + kernel pass) alternating over library
# builds, fresh process each: bash tools/lib_ab.sh TAG ROUNDS lib1 lib2 ...  (lib "." = in-tree)
tag=$1; rounds=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    BMH_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 \
      > $o/${n}_$r.json 2> $o/${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/${n}_$r.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$l'.ljust(28), d['value'], d['ms_per_step'], d['parity'][:7], {a: k[a] for a in list(k)[:5]})"
  done
done
