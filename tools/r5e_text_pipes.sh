#!/bin/bash
# On the GPU box: Zipf text configs under pipeline counts (fresh process each)
o=gpurun_out/r5e; mkdir -p $o
for p in 0 1 2 3 4; do
  timeout -k 10 100 python3 tools/text_bench.py 100 1 pipelines=$p > $o/t100_$p.json || exit 1
  python3 -c "import json; d=json.load(open('$o/t100_$p.json')); print('zipf100/1M pipes $p', d['ms'], d['MBps'], d.get('parity'))"
done
for p in 0 1 2; do
  timeout -k 10 100 python3 tools/text_bench.py 128 16 pipelines=$p > $o/t128_$p.json || exit 1
  python3 -c "import json; d=json.load(open('$o/t128_$p.json')); print('zipf128/16M pipes $p', d['ms'], d['MBps'])"
  timeout -k 10 100 python3 tools/text_bench.py 128 4 pipelines=$p > $o/t128b_$p.json || exit 1
  python3 -c "import json; d=json.load(open('$o/t128b_$p.json')); print('zipf128/4M pipes $p', d['ms'], d['MBps'])"
done
for p in 0 1; do
  timeout -k 10 200 python3 tools/config5_run.py --gib 2 --opts pipelines=$p > $o/c5_$p.json 2> $o/c5_$p.err || exit 1
  tail -c 400 $o/c5_$p.json; echo
done
