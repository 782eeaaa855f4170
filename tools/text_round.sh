#!/bin/bash
# Text path (configs 3 and 5) on the GPU box: throughput + kernel breakdown, and the per-round list
# census. tools/text_round.sh TAG -> gpurun_out/TAG_text100.json, TAG_text128.json, TAG_census100.txt
tag=${1:-t}
timeout -k 10 200 python3 tools/text_bench.py 100 1 > gpurun_out/${tag}_text100.json 2> gpurun_out/${tag}_text100.err || exit 1
timeout -k 10 200 python3 tools/text_bench.py 128 16 > gpurun_out/${tag}_text128.json 2> gpurun_out/${tag}_text128.err || exit 1
timeout -k 10 200 python3 tools/list_census.py 100 1 > /dev/null 2> gpurun_out/${tag}_census100.txt || exit 1
timeout -k 10 200 python3 tools/list_census.py 128 16 > /dev/null 2> gpurun_out/${tag}_census128.txt || exit 1
python3 - "$tag" <<'P'
import json, sys
t = sys.argv[1]
for f in ("text100", "text128"):
    d = json.loads(open(f"gpurun_out/{t}_{f}.json").read().strip().splitlines()[-1])
    print(f, d.get("ms"), d.get("MBps"), {k: v for k, v in d.items() if k not in ("kernels_ms", "ms", "MBps")})
    print(sorted(d["kernels_ms"].items(), key=lambda kv: -kv[1][1])[:14])
P
