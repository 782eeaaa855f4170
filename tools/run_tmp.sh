export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "calgary or runs or manifest or fuzz or multi or host" > gpurun_out/aux_tests.log 2>&1; rc=$?; tail -2 gpurun_out/aux_tests.log; [ $rc -eq 0 ] || exit $rc
ALL="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
for r in 1 2 3; do timeout -k 10 60 python3 tools/cal_subset_time.py $ALL || exit 1; done
