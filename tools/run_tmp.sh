export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_runs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/runs_tests.log 2>&1; rc=$?; tail -25 gpurun_out/runs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "calgary or fresh or manifest or fuzz" > gpurun_out/runs_tests2.log 2>&1; rc=$?; tail -3 gpurun_out/runs_tests2.log; [ $rc -eq 0 ] || exit $rc
ALL="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
for s in 2 3; do
  BMH_STREAMS=$s timeout -k 10 60 python3 tools/cal_subset_time.py $ALL || exit 1
done
timeout -k 10 60 python3 tools/cal_subset_time.py pic || exit 1
