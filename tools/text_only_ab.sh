#!/bin/bash
# Text configs alternating over library builds (no test suite): bash tools/text_only_ab.sh ROUNDS lib...
rounds=$1; shift
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    line="$l"
    for cfg in "100 1" "128 16" "128 4"; do
      out=$(BMH_LIB=$lib timeout -k 10 150 python3 tools/text_bench.py $cfg) || exit 1
      line="$line | $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernels_ms']; print(d['ms'], d.get('parity'), 'tiny', k.get('bwt_finish_tiny', [0, 0])[1])")"
    done
    echo "$line"
  done
done
