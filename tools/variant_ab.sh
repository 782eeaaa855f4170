#!/bin/bash
# GPU suite under every library build, then text configs and Calgary (whole files) alternating
# over the builds, fresh process each: bash tools/variant_ab.sh ROUNDS . variants/x/libbmh.so ...
o=gpurun_out/${TAG:-varab}; mkdir -p $o
export TMPDIR=/tmp
rounds=$1; shift
# TESTED="lib ..." skips the suite for builds an earlier call already ran it on
for l in "$@"; do
  lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
  n=$(echo $l | tr '/.' '__')
  case " $TESTED " in *" $l "*) continue;; esac
  BMH_LIB=$lib timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/${n}_tests.log 2>&1
  rc=$?; echo "$l: $(tail -1 $o/${n}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    if [ -n "$CAL_ONLY" ]; then  # CAL_ONLY=1: Calgary only
      for m in whole 256k; do
        BMH_LIB=$lib timeout -k 10 120 python3 tools/calgary_prof.py --mode $m --steps 10 > $o/${n}_${m}_$r.json 2>/dev/null || exit 1
      done
      python3 -c "import json; print('$l'.ljust(26), 'calgary whole/256k', [json.load(open('$o/${n}_'+m+'_$r.json'))['ms'] for m in ('whole', '256k')])"
      continue
    fi
    for cfg in "100 1" "128 16" "128 4"; do
      BMH_LIB=$lib timeout -k 10 150 python3 tools/text_bench.py $cfg > $o/${n}_t${cfg// /_}_$r.json || exit 1
    done
    BMH_LIB=$lib timeout -k 10 120 python3 tools/calgary_prof.py --mode whole --steps 10 > $o/${n}_cal_$r.json 2>/dev/null || exit 1
    BMH_LIB=$lib timeout -k 10 120 python3 tools/calgary_prof.py --mode 256k --steps 10 > $o/${n}_c256_$r.json 2>/dev/null || exit 1
    if [ -n "$BENCH" ]; then  # BENCH=1: the 1 GiB headline step too
      BMH_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 2>/dev/null | tail -1 > $o/${n}_b_$r.json || exit 1
      python3 -c "import json; print('   1GiB', json.load(open('$o/${n}_b_$r.json'))['ms_per_step'])"
    fi
    python3 - $o $n $r $l <<'P'
import json, sys
o, n, r, l = sys.argv[1:]
t = [json.load(open(f"{o}/{n}_t{c}_{r}.json")) for c in ("100_1", "128_16", "128_4")]
c = [json.load(open(f"{o}/{n}_{m}_{r}.json"))["ms"] for m in ("cal", "c256")]
print(l.ljust(26), "text", [x["ms"] for x in t], t[0].get("parity"), "| calgary whole/256k", c)
P
  done
done
