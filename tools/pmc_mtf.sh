#!/bin/bash
# SQ counters of the headline kernels (in-tree lib; run on the GPU box): the two tools/run_pmc.sh
# passes plus an LDS pass (LDS-issue stalls, LDS array busy cycles) and the shader clock
# (GRBM_GUI_ACTIVE over the kernel's duration), one rocprofv3 --pmc run each.
export TMPDIR=/tmp
o=${1:-gpurun_out/pmc_mtf}
mkdir -p $o
timeout -s KILL 60 rocprofv3 -L > $o/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $o/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $o/p$i.log; exit 1; }
done
python3 tools/pmc_mtf_sum.py $o > $o/summary.json; head -c 3000 $o/summary.json
