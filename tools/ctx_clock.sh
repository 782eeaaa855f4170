#!/bin/bash
# On the GPU box: the shader clock of the big kernels per context, 8 contexts
# of one process (tools/ctx_pmc.py), GRBM_GUI_ACTIVE / 8 XCDs / kernel duration; contexts whose
# kernels run slower at the same clock are not clock-bound.
o=gpurun_out/${1:-ctxclk}; mkdir -p $o
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d $o/p1 -o run --output-format csv -- python3 tools/ctx_pmc.py 8 5 > $o/p1.log 2>&1 || exit 1
python3 tools/ctx_pmc_sum.py $o/p1 | tee $o/summary.txt
