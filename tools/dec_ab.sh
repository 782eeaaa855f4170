#!/bin/bash
# On the GPU box: the bench's GPU decode leg alternating over library builds, fresh process each:
# bash tools/dec_ab.sh TAG ROUNDS lib1 lib2 ...
tag=$1; rounds=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    BMH_LIB=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 --calgary-steps 0 --decode-steps 5 \
      > $o/${n}_$r.json 2> $o/${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/${n}_$r.json').read().strip().splitlines()[-1]); x=d['decode']; print('$l'.ljust(28), x['value'], x['ms_per_step'], x.get('roundtrip_bit_exact'))"
  done
done
