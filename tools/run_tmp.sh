export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "calgary or runs or manifest or fuzz or mtf or huff" > gpurun_out/mv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mv_tests.log; [ $rc -eq 0 ] || exit $rc
ALL="bib book1 book2 geo news obj1 obj2 paper1 paper2 pic progc progl progp trans"
for r in 1 2 3; do timeout -k 10 60 python3 tools/cal_subset_time.py $ALL || exit 1; done
timeout -k 10 100 python3 tools/calgary_prof.py --mode whole > gpurun_out/cal_whole3.json || exit 1
