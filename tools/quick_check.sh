#!/bin/bash
# GPU parity suite, then the text / Calgary / headline timings (run on the GPU box).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/qc_tests.log 2>&1
tail -2 gpurun_out/qc_tests.log
timeout -k 10 100 python3 tools/text_bench.py 100 1 > gpurun_out/qc_text100.json
timeout -k 10 100 python3 tools/text_bench.py 128 16 > gpurun_out/qc_text128.json
timeout -k 10 100 python3 tools/calgary_prof.py --mode whole > gpurun_out/qc_cal.json
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --pcie-steps 0 --decode-steps 0 --calgary-steps 0 > gpurun_out/qc_bench.json
python3 - <<'P'
import json
for f in ["qc_text100", "qc_text128"]:
    d = json.load(open(f"gpurun_out/{f}.json")); print(f, d["ms"], "ms", d["MBps"], "MB/s", d.get("parity"), {k: v for k, v in list(d["kernels_ms"].items())[:8]})
d = json.load(open("gpurun_out/qc_cal.json")); print("calgary", d["ms"], "ms")
d = json.loads(open("gpurun_out/qc_bench.json").read().strip().splitlines()[-1]); print("bench", d["value"], d["ms_per_step"], d["parity"])
P
