export TMPDIR=/tmp
BMH_LIB=variants/v2/libbmh.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "bwt or manifest or calgary or fuzz or large" > gpurun_out/v2_tests.log 2>&1; tail -2 gpurun_out/v2_tests.log
for v in pv1 pv2; do
BMH_LIB=variants/$v/libbmh.so timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > gpurun_out/$v.json 2> gpurun_out/$v.err
echo $v; grep phases gpurun_out/$v.err | tail -1
done
bash tools/variant_bench.sh v2
bash tools/run_pmc.sh v2
