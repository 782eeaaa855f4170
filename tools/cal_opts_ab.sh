#!/bin/bash
# Calgary (whole files and 256 KiB blocks) alternating over option sets, fresh process each:
# bash tools/cal_opts_ab.sh ROUNDS "" "mtf_chunk=128" ...   ("" = the library's defaults)
o=gpurun_out/${TAG:-calopts}; mkdir -p $o
rounds=$1; shift
for r in $(seq $rounds); do
  for op in "$@"; do
    n=$(echo "x$op" | tr '=,' '__')
    for m in whole 256k; do
      timeout -k 10 120 python3 tools/calgary_prof.py --mode $m --steps 10 --opts "$op" > $o/${n}_${m}_$r.json 2>/dev/null || exit 1
    done
    python3 -c "import json; a=json.load(open('$o/${n}_whole_$r.json')); b=json.load(open('$o/${n}_256k_$r.json')); print('[$op]'.ljust(22), a['ms'], b['ms'])"
  done
done
