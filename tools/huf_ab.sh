for v in "$@"; do
  BMH_LIB=variants/$v/libbmh.so timeout -k 10 120 python tools/calgary_prof.py --mode whole --steps 3 > gpurun_out/r4e_$v.json 2> gpurun_out/r4e_$v.err || exit 1
  echo "$v $(grep -h 'huff_build phases' gpurun_out/r4e_$v.err | tail -2 | tr '\n' ' ')"
done
