#!/bin/bash
# On the GPU box: text configs 3 / 5 and Calgary (whole files, 256 KiB blocks) alternating over
# library builds, fresh process each: bash tools/text_cal_ab.sh TAG ROUNDS lib1 lib2 ...
tag=$1; rounds=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    BMH_LIB=$lib timeout -k 10 150 python3 tools/text_bench.py 100 1 > $o/${n}_t100_$r.json || exit 1
    BMH_LIB=$lib timeout -k 10 150 python3 tools/text_bench.py 128 16 > $o/${n}_t128_$r.json || exit 1
    BMH_LIB=$lib timeout -k 10 100 python3 tools/calgary_prof.py --mode whole --steps 10 > $o/${n}_cw_$r.json || exit 1
    BMH_LIB=$lib timeout -k 10 100 python3 tools/calgary_prof.py --mode 256k --steps 10 > $o/${n}_ck_$r.json || exit 1
    python3 - $o $n $r $l <<'P'
import json, sys
o, n, r, l = sys.argv[1:]
t = [json.load(open(f"{o}/{n}_{c}_{r}.json")) for c in ("t100", "t128", "cw", "ck")]
print(l.ljust(26), "text100", t[0]["ms"], "text128", t[1]["ms"], "cal whole", t[2]["ms"], "cal 256k", t[3]["ms"], t[0].get("parity"))
P
  done
done
