#!/bin/bash
# GPU suite, then the headline alternating over library builds (kernel pass shows pack_write)
o=gpurun_out/${TAG:-r5pk}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_ab.sh ${TAG:-r5pk} 2 "$@"
