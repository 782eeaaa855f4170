#!/bin/bash
# GPU suite, text configs, 1 GiB and 128 MiB random steps (two rounds)
o=gpurun_out/${TAG:-r5m2}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "100 1" "128 16" "128 4"; do
    timeout -k 10 150 python3 tools/text_bench.py $cfg > $o/t_${cfg// /_}_$r.json || exit 1
  done
  for tb in 1073741824 134217728; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes $tb > $o/b_${tb}_$r.json 2>/dev/null || exit 1
  done
  python3 - $o $r <<'P'
import json, sys
o, r = sys.argv[1:]
t = [json.load(open(f"{o}/t_{c}_{r}.json")) for c in ("100_1", "128_16", "128_4")]
b = [json.loads(open(f"{o}/b_{tb}_{r}.json").read().strip().splitlines()[-1]) for tb in (1073741824, 134217728)]
print("text", [x["ms"] for x in t], t[0].get("parity"), "| 1GiB", b[0]["ms_per_step"], b[0]["parity"][:7], "| 128MiB", b[1]["ms_per_step"],
      {k: v for k, v in b[0]["kernels_ms_per_step"].items() if k.startswith("mtf")})
P
done
