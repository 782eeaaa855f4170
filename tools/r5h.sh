#!/bin/bash
# GPU suite, then the text configs and the headline (packed records A/B vs the previous library)
o=gpurun_out/r5h; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "100 1" "128 16" "128 4"; do
    timeout -k 10 100 python3 tools/text_bench.py $cfg > $o/t_${cfg// /_}_$r.json || exit 1
    python3 -c "import json; d=json.load(open('$o/t_${cfg// /_}_$r.json')); print('$cfg', d['ms'], d['MBps'], d.get('parity'), list(d['kernels_ms'].items())[2:8])"
  done
done
timeout -k 10 300 python3 tools/ctx_probe.py 6 12 > $o/ctx.txt 2>&1 || exit 1
cat $o/ctx.txt
timeout -k 10 60 rocprofv3 -L > $o/counters.txt 2>&1 || true
grep -iE "UTCL|TLB|TRANSLATION|EA0_RDREQ|EA0_WRREQ" $o/counters.txt | head -60 > $o/counters_tlb.txt || true
wc -l $o/counters.txt $o/counters_tlb.txt
