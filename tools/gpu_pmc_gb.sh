# SQ stall counters of gemm_bench variants (separate --pmc passes per counter set)
#   V="h3r h3r_noglds_nobar" S=conv2 bash tools/gpu_pmc_gb.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${S:-conv2}
for v in ${V:-h3r}; do
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM"; do
    i=$((i+1))
    VARIANT=$v timeout -k 10 180 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/pmc_gb_${v}_$i -o run -- tools/gemm_bench 1000 2 $S > gpurun_out/pmc_gb_${v}_$i.log 2>&1 || exit $?
  done
done
