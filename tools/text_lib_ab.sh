#!/bin/bash
# GPU suite, then text configs and random 1 GiB / 128 MiB alternating over library builds
o=gpurun_out/${TAG:-textab}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    for cfg in "100 1" "128 16" "128 4"; do
      BMH_LIB=$lib timeout -k 10 150 python3 tools/text_bench.py $cfg > $o/${n}_t${cfg// /_}_$r.json || exit 1
    done
    BMH_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/${n}_b_$r.json 2>/dev/null || exit 1
    python3 - $o $n $r $l <<'P'
import json, sys
o, n, r, l = sys.argv[1:]
t = [json.load(open(f"{o}/{n}_t{c}_{r}.json")) for c in ("100_1", "128_16", "128_4")]
b = json.loads(open(f"{o}/{n}_b_{r}.json").read().strip().splitlines()[-1])
print(l.ljust(26), "text", [x["ms"] for x in t], t[0].get("parity"), "| 1GiB", b["ms_per_step"], b["parity"][:7])
P
  done
done
