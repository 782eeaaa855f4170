#!/bin/bash
# GPU suite, then the headline and the 128 MiB strong-scaling share twice each, then Calgary
o=gpurun_out/${TAG:-r5r}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for tb in 1073741824 134217728; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes $tb \
      > $o/b_${tb}_$r.json 2> $o/b_${tb}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$o/b_${tb}_$r.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print($tb>>20, d['ms_per_step'], d['parity'][:7], {a: k[a] for a in list(k)[:12]})"
  done
done
timeout -k 10 120 python3 tools/calgary_prof.py --mode whole --steps 5 > $o/cal_whole.json 2> $o/cal_whole.err || exit 1
timeout -k 10 120 python3 tools/calgary_prof.py --mode 256k --steps 5 > $o/cal_256k.json 2> $o/cal_256k.err || exit 1
python3 -c "
import json
for f in ['$o/cal_whole.json','$o/cal_256k.json']:
    d=json.load(open(f)); k=d['kernels']; print(f, d['ms'], {a:k[a] for a in list(k) if a.startswith(('mtf','huff'))})"
