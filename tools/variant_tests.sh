#!/bin/bash
# On the GPU box: the GPU test suite against each named variant library (experiments):
#   bash tools/variant_tests.sh name ...   -> gpurun_out/vt_<name>.log
# Stops at the first run that ends other than pass / test failure (fault, abort, time limit).
mkdir -p gpurun_out
for v in "$@"; do
    BMH_LIB=variants/$v/libbmh.so timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 300 \
        --timeout-method thread > gpurun_out/vt_$v.log 2>&1
    rc=$?
    echo "$v: rc=$rc $(tail -1 gpurun_out/vt_$v.log)"
    grep FAILED gpurun_out/vt_$v.log | head -5
    case $rc in 0 | 1) ;; *) exit $rc ;; esac
done
