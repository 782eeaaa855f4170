#!/bin/bash
# GPU suite + headline bench (run on the GPU box): gpurun_out/<tag>_tests.log, <tag>_bench.json
tag=${1:-r}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 3 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
python3 - "$tag" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}_bench.json").read().strip().splitlines()[-1])
print("bench", d["value"], d["ms_per_step"], d["parity"], "calgary", d["calgary"]["whole_files"]["MBps"], d["calgary"]["blocks_256k"]["MBps"])
print(list(d["kernels_ms_per_step"].items())[:10])
P
