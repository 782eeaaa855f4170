#!/bin/bash
# A/B of the Calgary leg over library builds, fresh process each (run on the GPU box):
# tools/cal_lib_ab.sh ROUNDS lib1 lib2 ...   (lib "." = in-tree) -> one line per run: whole-file ms,
# 256 KiB ms, records equal the reference's
rounds=$1; shift
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    BMH_LIB=$lib timeout -k 10 120 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 30 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d['calgary']; print('$l'.ljust(26), c['whole_files']['ms'], c['blocks_256k']['ms'], c['whole_files']['records_byte_identical_to_reference'], c['blocks_256k']['records_byte_identical_to_reference'])" || exit 1
  done
done
