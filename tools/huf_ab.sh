#!/bin/bash
# k_huff_build phase timing A/B on Calgary whole files: TAG=r4p tools/huf_ab.sh <variant>... where
# each variants/<v>/libbmh.so was built with tools/build_variant.sh <v> huffman.hip -DBMH_PROF_HUFF
tag=${TAG:-r4e}
for v in "$@"; do
  BMH_LIB=variants/$v/libbmh.so timeout -k 10 120 python tools/calgary_prof.py --mode whole --steps 3 > gpurun_out/${tag}_$v.json 2> gpurun_out/${tag}_$v.err || exit 1
  echo "$v $(grep -h 'huff_build phases' gpurun_out/${tag}_$v.err | tail -2 | tr '\n' ' ')"
done
