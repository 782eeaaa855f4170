#!/bin/bash
# On the GPU box: per-context spread (tools/ctx_pmc.py) without a profiler, then with address-
# translation and L2/fabric request counters (one rocprofv3 --pmc pass per counter group).
o=gpurun_out/${1:-ctxpmc}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ctx_pmc.py 6 6 > $o/plain.txt 2>&1 || exit 1
cat $o/plain.txt
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $o/p$i -o run --output-format csv -- python3 tools/ctx_pmc.py 6 4 > $o/p$i.log 2>&1 || exit 1
done
python3 tools/ctx_pmc_sum.py $o/p1 $o/p2
