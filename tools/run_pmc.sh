# SQ counters of the headline kernels for the in-tree lib and variants/<name> (run on the GPU box):
# instruction mix, then where the wave cycles go (two passes: the SQ block takes 8 counters)
export TMPDIR=/tmp
for v in ${@:-base}; do
  lib=""; [ "$v" = base ] || lib=variants/$v/libbmh.so
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES"; do
    i=$((i+1))
    BMH_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$v/p$i -o run --output-format csv -- python3 bench.py --pipelines 1 --steps 1 --warmup 1 --no-cpu-baseline --decode-steps 0 --pcie-steps 0 --calgary-steps 0 > gpurun_out/pmc_$v.log 2>&1 || exit 1
  done
  echo "== $v"; python3 tools/pmc_sq.py gpurun_out/pmc_$v | head -4
done
