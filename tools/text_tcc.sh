#!/bin/bash
# Config 3 (Zipf 100 MB, 1 MiB blocks, one stream): L2 hits / misses and memory-side read requests
# of the list-round kernels, one rocprofv3 --pmc pass each, then a per-kernel
# table (tools/text_tcc_sum.py). Run on the GPU box.
o=gpurun_out/${TAG:-ttcc}; mkdir -p $o
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $o/p1 -o run --output-format csv -- python3 tools/text_bench.py 100 1 pipelines=1 > $o/p1.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $o/p2 -o run --output-format csv -- python3 tools/text_bench.py 100 1 pipelines=1 > $o/p2.log 2>&1 || exit 1
python3 tools/text_tcc_sum.py $o > $o/summary.txt; cat $o/summary.txt
