#!/bin/bash
# Dense-finish phase timing A/B (-DBMH_PROF_DENSE variants built by tools/build_variant.sh):
# tools/dense_phases.sh name... -> one line of mean s_memtime ticks per phase per variant
for v in "$@"; do
  BMH_LIB=variants/$v/libbmh.so timeout -k 10 120 python3 bench.py --pipelines 1 --steps 2 --warmup 1 --no-cpu-baseline \
      --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > gpurun_out/dph_$v.json 2> gpurun_out/dph_$v.err || exit 1
  echo "$v $(grep -h 'phases' gpurun_out/dph_$v.err | tail -1)"
done
