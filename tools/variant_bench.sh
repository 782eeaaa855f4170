#!/bin/bash
# On the GPU box: headline bench for the in-tree library and each variants/<name>/libbmh.so,
# one short run each (no CPU baseline, no decode): gpurun_out/variants/<name>.json
#   bash tools/variant_bench.sh [name ...]
set -e
export TMPDIR=/tmp
o=gpurun_out/variants
mkdir -p $o
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/base.json 2> $o/base.err
names=${@:-$(ls variants)}
for n in $names; do
    BMH_LIB=variants/$n/libbmh.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
        --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/$n.json 2> $o/$n.err
done
python3 - <<'EOF'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/variants/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    top = ", ".join(f"{n} {v}" for n, v in list(k.items())[:6])
    print(f"{os.path.basename(f)[:-5]:12s} {d['value']:9.1f} MB/s {d['ms_per_step']:7.3f} ms  parity: {d['parity']}  | {top}")
EOF
