#!/bin/bash
# One profiling pass of the headline bench on the GPU box (run from the repo root there):
#   1. bench.py (default config, incl. CPU baseline)            -> gpurun_out/prof/bench.json
#   2. rocprofv3 --kernel-trace --stats over bench.py            -> gpurun_out/prof/stats/
#   3. PMC FETCH_SIZE / WRITE_SIZE passes + per-kernel traffic  -> gpurun_out/prof/pmc_traffic.json
set -e
export TMPDIR=/tmp
o=gpurun_out/prof
mkdir -p $o
timeout -k 10 400 python3 bench.py > $o/bench.json 2> $o/bench.err
# one stream, like bench.py's per-kernel pass, so the per-kernel durations agree with its roofline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- \
    python3 bench.py --pipelines 1 --steps 5 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/stats_bench.json 2> $o/stats.err
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" timeout -k 10 600 bash tools/pmc_run.sh $o/pmc --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --pipelines 1
python3 tools/pmc_traffic.py $o/pmc $((1 << 30)) $o/pmc_traffic.json
echo profile done
