#!/bin/bash
# On the GPU box: the headline bench under several bench.py option sets, one short run each:
#   bash tools/env_bench.sh "--pipelines 2" "--opt mtf_chunk=2048" ...
# -> gpurun_out/envb/<i>.json and a one-line summary per setting.
set -e
export TMPDIR=/tmp
o=gpurun_out/envb
mkdir -p $o
i=0
for cfg in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python3 bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 \
        > $o/$i.json 2> $o/$i.err
    python3 -c "import json,sys; d=json.loads(open('$o/$i.json').read().strip().splitlines()[-1]); print(f\"{sys.argv[1]:40s} {d['value']:9.1f} MB/s {d['ms_per_step']:7.3f} ms  {d['parity']}\")" "$cfg"
done
