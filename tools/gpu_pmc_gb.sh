# SQ stall counters of one gemm_bench variant (separate --pmc passes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-h3c}
S=${S:-conv2}
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  VARIANT=$V timeout -k 10 180 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/pmc_gb_$i -o run -- tools/gemm_bench 1000 2 $S > gpurun_out/pmc_gb_$i.log 2>&1 || exit $?
done
