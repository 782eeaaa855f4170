#!/bin/bash
# PMC passes over one bench step (run ON the GPU box; each pass its own rocprofv3 run, counters
# only with --kernel-trace, per MI355X_MICROARCH.md §HBM / rocprofv3 slot limits).
# usage: tools/pmc_run.sh OUTDIR [bench args...]
set -e
out=${1:-gpurun_out/pmc}; shift || true
args=${@:---steps 1 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p "$out"
i=0
GROUPS_DEFAULT=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS_ATOMIC"
  "GRBM_GUI_ACTIVE")
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -r -a GROUPS_SEL <<< "$PMC_GROUPS"; else GROUPS_SEL=("${GROUPS_DEFAULT[@]}"); fi
for grp in "${GROUPS_SEL[@]}"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$out/p$i" -o run --output-format csv -- python3 bench.py $args > "$out/p$i.log" 2>&1
done
echo done
