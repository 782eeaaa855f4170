#!/bin/bash
# Text path A/B: the in-tree library against variants/<name>/libbmh.so (tools/build_variant.sh):
# tools/text_ab.sh TAG name -> gpurun_out/TAG_{lib,name}_{text100,text128}.json + census files
tag=$1; v=$2
run() {  # $1 = label, env BMH_LIB set by the caller
  timeout -k 10 200 python3 tools/text_bench.py 100 1 > gpurun_out/${tag}_$1_text100.json 2> /dev/null || return 1
  timeout -k 10 200 python3 tools/text_bench.py 128 16 > gpurun_out/${tag}_$1_text128.json 2> /dev/null || return 1
  timeout -k 10 200 python3 tools/list_census.py 100 1 > /dev/null 2> gpurun_out/${tag}_$1_census100.txt || return 1
  timeout -k 10 200 python3 tools/list_census.py 128 16 > /dev/null 2> gpurun_out/${tag}_$1_census128.txt || return 1
}
run lib || exit 1
BMH_LIB=variants/$v/libbmh.so run $v || exit 1
python3 - "$tag" "$v" <<'P'
import json, sys
t, v = sys.argv[1:]
for lab in ("lib", v):
    for f in ("text100", "text128"):
        d = json.loads(open(f"gpurun_out/{t}_{lab}_{f}.json").read().strip().splitlines()[-1])
        ks = sorted(d["kernels_ms"].items(), key=lambda kv: -kv[1][1])[:8]
        print(lab, f, d.get("ms"), d.get("MBps"), {k: v for k, v in d.items() if k not in ("kernels_ms", "ms", "MBps")})
        print("   ", [(k, round(x[1], 2)) for k, x in ks])
P
