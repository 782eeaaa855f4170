for v in pbase pg9 psc9; do
BMH_LIB=variants/$v/libbmh.so timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > gpurun_out/$v.json 2> gpurun_out/$v.err
grep phases gpurun_out/$v.err | tail -2
done
