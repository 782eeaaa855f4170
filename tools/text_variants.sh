#!/bin/bash
# On the GPU box: tools/text_bench.py (Zipf text) for the in-tree library and each named
# variant: bash tools/text_variants.sh "<MB> <block_MiB>" name ...
set -e
export TMPDIR=/tmp
o=gpurun_out/textv
mkdir -p $o
args=$1; shift
for n in base "$@"; do
    lib=""
    [ "$n" != base ] && lib="BMH_LIB=variants/$n/libbmh.so"
    env $lib timeout -k 10 200 python3 tools/text_bench.py $args > $o/$n.json 2> $o/$n.err
    python3 -c "import json,sys; d=json.load(open('$o/$n.json')); print(f\"{sys.argv[1]:8s} {d['MBps']:8.1f} MB/s {d['ms']:8.2f} ms parity {d.get('parity')} \", list(d['kernels_ms'].items())[:8])" $n
done
