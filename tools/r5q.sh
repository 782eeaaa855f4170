#!/bin/bash
# GPU suite on the in-tree library, then 1 GiB and 128 MiB steps alternating over library builds
o=gpurun_out/r5q; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in "$@"; do
    lib=$l; [ "$l" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
    n=$(echo $l | tr '/.' '__')
    for tb in 1073741824 134217728; do
      BMH_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes $tb \
        > $o/${n}_${tb}_$r.json 2> $o/${n}_${tb}_$r.err || exit 1
      python3 -c "import json; d=json.loads(open('$o/${n}_${tb}_$r.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$l'.ljust(28), $tb>>20, d['ms_per_step'], d['parity'][:7], {a: k[a] for a in list(k)[:12]})"
    done
  done
done
BMH_LIB=variants/huffprof/libbmh.so timeout -k 10 100 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 --total-bytes 134217728 > $o/huffprof.json 2> $o/huffprof.err || exit 1
grep -h 'huff_build phases' $o/huffprof.err | tail -3
timeout -k 10 120 python3 tools/calgary_prof.py --mode whole --steps 5 > $o/cal_whole.json 2> $o/cal_whole.err || exit 1
timeout -k 10 120 python3 tools/calgary_prof.py --mode 256k --steps 5 > $o/cal_256k.json 2> $o/cal_256k.err || exit 1
tail -c 300 $o/cal_whole.json; echo; tail -c 300 $o/cal_256k.json; echo
