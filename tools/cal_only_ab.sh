#!/bin/bash
# On the GPU box: Calgary (whole files, 256 KiB blocks) alternating over library builds, fresh
# process each: bash tools/cal_only_ab.sh TAG ROUNDS lib1 lib2 ...
tag=$1; rounds=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    BMH_LIB=$lib timeout -k 10 100 python3 tools/calgary_prof.py --mode whole --steps 10 > $o/${n}_cw_$r.json || exit 1
    BMH_LIB=$lib timeout -k 10 100 python3 tools/calgary_prof.py --mode 256k --steps 10 > $o/${n}_ck_$r.json || exit 1
    python3 -c "import json; a=json.load(open('$o/${n}_cw_$r.json')); b=json.load(open('$o/${n}_ck_$r.json')); print('$l'.ljust(28), 'whole', a['ms'], '256k', b['ms'])"
  done
done
