#!/bin/bash
# SQ counters of k_pack_write (run on the GPU box): tools/pmc_pack.sh OUTDIR [lib]  — four
# rocprofv3 --pmc passes over one headline bench step, each its own run; summary via pmc_mtf_sum.py.
export TMPDIR=/tmp
o=${1:-gpurun_out/pmc_pack}; lib=${2:-.}; [ "$lib" = "." ] && lib=bwt-mtf-huffman-compressor_amd/lib/libbmh.so
mkdir -p $o
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  BMH_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $o/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > $o/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $o/p$i.log; exit 1; }
done
python3 tools/pmc_mtf_sum.py $o k_pack_write > $o/summary.json; cat $o/summary.json
