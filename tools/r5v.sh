#!/bin/bash
# GPU suite, a 128 MiB call timeline, then 128 MiB / 1 GiB steps
o=gpurun_out/${TAG:-r5v}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t0 -o run --output-format csv -- python3 tools/trace_run.py 128 4 3 > $o/t0.log 2>&1 || exit 1
python3 tools/call_timeline.py $o/t0 > $o/tl0.txt; head -14 $o/tl0.txt
for r in 1 2; do
  for tb in 134217728 1073741824; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes $tb \
      > $o/b_${tb}_$r.json 2> $o/b_${tb}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/b_${tb}_$r.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print($tb>>20, d['ms_per_step'], d['parity'][:7], {a: k[a] for a in list(k)[:8]})"
  done
done
