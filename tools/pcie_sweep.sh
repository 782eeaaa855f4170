#!/bin/bash
# On the GPU box: the PCIe-inclusive leg of bench.py (pinned host -> records in pinned host) under
# several stream_batch option sizes: one line per setting.
set -e
export TMPDIR=/tmp
for b in "$@"; do
    timeout -k 10 200 python3 bench.py --opt stream_batch=$b --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 \
        --calgary-steps 0 --pcie-steps 5 > gpurun_out/pcie_$b.json 2> gpurun_out/pcie_$b.err
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/pcie_$b.json').read().strip().splitlines()[-1]); p=d['pcie_inclusive']; print(f\"batch {int(sys.argv[1])>>20:5d} MiB  {p['value']:9.1f} MB/s  {p['ms_per_step']:8.3f} ms  records equal: {p['records_equal_device_encode']}  device {d['value']:.0f} MB/s  steps {p['rank0_step_ms']}\")" $b
done
