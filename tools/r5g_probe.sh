#!/bin/bash
# On the GPU box: the counters rocprofv3 offers for address translation / memory requests, and the
# per-context step-time spread of the headline workload (tools/ctx_probe.py, 8 contexts).
o=gpurun_out/r5g; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $o/counters.txt 2>&1 || true
grep -iE "UTCL|TLB|TRANSLATION|EA0_RDREQ|EA0_WRREQ|TCC_EA" $o/counters.txt | head -60 > $o/counters_tlb.txt || true
wc -l $o/counters.txt $o/counters_tlb.txt
timeout -k 10 300 python3 tools/ctx_probe.py 8 12 > $o/ctx.txt 2>&1 || exit 1
cat $o/ctx.txt
