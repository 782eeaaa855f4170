#!/bin/bash
# dense-finish phase ticks on text (config 3 and 16 MiB blocks) and random data, then the GPU
# suite and the text configs on the in-tree library
o=gpurun_out/${TAG:-dphase}; mkdir -p $o
export TMPDIR=/tmp
for cfg in "100 1" "128 16"; do
  BMH_LIB=variants/denseprof/libbmh.so timeout -k 10 150 python3 tools/text_bench.py $cfg pipelines=1 > $o/dp_${cfg// /_}.json 2> $o/dp_${cfg// /_}.err || exit 1
  echo "text $cfg: $(grep -h 'phases' $o/dp_${cfg// /_}.err | tail -1)"
done
BMH_LIB=variants/denseprof/libbmh.so timeout -k 10 150 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --pipelines 1 > $o/dp_rand.json 2> $o/dp_rand.err || exit 1
echo "random: $(grep -h 'phases' $o/dp_rand.err | tail -1)"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "100 1" "128 16" "128 4"; do
  timeout -k 10 150 python3 tools/text_bench.py $cfg > $o/t_${cfg// /_}.json || exit 1
  python3 -c "import json; d=json.load(open('$o/t_${cfg// /_}.json')); print('$cfg', d['ms'], d['MBps'], d.get('parity'), [(k,v) for k,v in d['kernels_ms'].items() if k.startswith('mtf')])"
done
